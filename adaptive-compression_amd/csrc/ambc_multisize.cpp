// ambc_multisize.cpp -- the reference's multi-size walk on the device.
//
// AdaptiveCompressor._adaptive_compress with several CHUNK_SIZE_CANDIDATES
// (adaptive_compressor.py:363-394 + _pick_best_chunk_and_method :537-590):
// at position pos every candidate size s = min(cand, remain) is encoded as one
// chunk by the reference's per-size method loop (ids ascending, strict "<" on
// len + 18), the sizes compare by their fp64 ratio (len + 18) / s, strictly,
// in list order, and the walk moves on by the winning size; a position where no
// size beats raw stores the whole remainder as one raw package (:586-588).
//
// The walk is serial -- each decision sets the next position -- so it runs as
// many walks at once: K walks start at positions spread over the input (all on
// the grid of g = gcd(candidates), where every walk position lies), and all of
// them advance in lock step.  One step evaluates every (position, size) the
// active walks need in ONE batch per size: the chunks are read in place from the
// uploaded input through a chunk-offset table (k_encode / k_dict / k_deflate,
// one workgroup per chunk), decision only (ENC_EVAL: no payload bytes).  With
// LZ4 (id 9) among the methods one parse per position serves every size: the
// largest LZ4-eligible size M is encoded with all its methods and reports the
// LZ4 block of each smaller candidate prefix (k_encode's lz4sub -- the greedy
// parse of a prefix is the chunk's own up to its last match start); the smaller
// sizes run only their other methods, and id 9 joins them last in id order on
// the host.  A walk stops when its next position has already been decided (it
// joined the path of another walk: from there on both are the same walk) or at
// the end.  Every decided position's successor is decided, so the walk from 0
// -- the reference's walk -- is then read off the decisions.  The chosen chunks
// are encoded once more (grouped by size, all methods, bytes this time) into
// slots -- the walk's decision must come out again, or the call fails -- and
// moved into the body at their offsets (k_compact with per-package lengths).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <thread>

#include <unistd.h>

#include "ambc_hostctx.h"

namespace ambc {
namespace {

// (WalkPool, the per-round host threads: ambc_sync.h)

bool eligible(const ambc_params* p, uint32_t s, uint32_t id) {
    return ((p->method_mask >> id) & 1) && p->pref_min[id] <= s && s <= p->pref_max[id];
}

bool any_eligible(const ambc_params* p, uint32_t s, uint32_t skip = 0) {
    for (uint32_t id = 1; id < 16; id++)
        if (id != skip && eligible(p, s, id)) return true;
    return false;
}

// the sizes the GPU encoders take (k_encode <= 65536, k_deflate <= 65536, k_dict <= 8192)
int check_size(const ambc_params* p, uint32_t s) {
    if (s > AMBC_MAX_CHUNK)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with eligible methods: the GPU encoders take chunks up to 65536 bytes");
    if (eligible(p, s, AMBC_M_DEFLATE) && (p->flags & AMBC_FLAG_ZLIB9) && z9_cmax(s) == 0)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with DEFLATE eligible: the GPU zlib-9 encoder takes chunks up to 65536 bytes");
    if (eligible(p, s, AMBC_M_DICT) && s > 8192)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with Dictionary eligible: the GPU Dictionary encoder takes chunks up to 8192 bytes");
    return AMBC_OK;
}

// The encoders over the s-byte chunks at pos[0..cnt) (one workgroup each) on
// stream st with the methods of p: per chunk the winner of the reference's
// method loop for that size, plen / ids copied back into hplen / hids (and, with
// subs, the LZ4 prefix blocks into hlz) -- valid after the stream synchronizes.
// The launch sequence is compress_on's (k_encode, k_dict against its winner,
// k_deflate against both, then -- bytes wanted -- the deferred emits).  eval:
// decisions only; pos must then be b.hpos (pinned, uploaded asynchronously).
int launch_batch(Batch& b, hipStream_t st, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint32_t s,
                 const uint64_t* pos, uint32_t cnt, const double* ent, bool eval, const uint32_t* subc = nullptr,
                 uint32_t nsub = 0) {
    const uint32_t C = (s + 15) & ~15u;
    const uint32_t stride = slot_stride_for(C);
    HIPCHK(b.coff.ensure((size_t)cnt * 8));
    HIPCHK(b.clen.ensure((size_t)cnt * 4));
    HIPCHK(b.slots.ensure((size_t)cnt * stride));
    HIPCHK(b.plen.ensure((size_t)cnt * 4 + 4));
    HIPCHK(b.ids.ensure((size_t)cnt + 16));
    HIPCHK(b.sizes.ensure((size_t)cnt * 8 + 8));
    HIPCHK(hipMemcpyAsync(b.coff.p, pos, (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(b.clen.p), (int)s, cnt, st));
    EncArgs ea{};
    ea.in = d_in;
    ea.n_total = n;
    ea.chunk_size = C;
    ea.n_chunks = cnt;
    ea.slots = b.slots.as<uint8_t>();
    ea.slot_stride = stride;
    ea.method_mask = p->method_mask;
    ea.plen = b.plen.as<uint32_t>();
    ea.ids = b.ids.as<uint8_t>();
    ea.sizes = b.sizes.as<uint64_t>();
    ea.coff = b.coff.as<uint64_t>();
    ea.clen = b.clen.as<uint32_t>();
    if (eval) ea.flags |= ENC_EVAL;
    for (int i = 0; i < 16; i++) { ea.pref_min[i] = p->pref_min[i]; ea.pref_max[i] = p->pref_max[i]; }
    // chunks on the 16-byte grid of the library's padded input copy: read in place
    bool aligned = ((uintptr_t)d_in & 15) == 0 && !getenv("AMBC_ENC_LDS");
    for (uint32_t q = 0; q < cnt && aligned; q++) aligned = (pos[q] & 15) == 0;
    if (aligned) ea.flags |= ENC_IN_ALIGNED;
    if (ent) {   // numpy's p*log2(p) terms for an s-byte chunk (Huffman should_use near 7.0), on the device
        if (s == C) ea.ent_full = ent;
        else ea.ent_tail = ent;
    }
    if (nsub) {
        HIPCHK(b.lz4sub.ensure((size_t)cnt * LZ4_SUB_MAX * 4));
        ea.lz4sub = b.lz4sub.as<uint32_t>();
        ea.n_subc = nsub;
        for (uint32_t j = 0; j < nsub; j++) ea.sub_c[j] = subc[j];
    }
    const bool dict = eligible(p, s, AMBC_M_DICT);
    const bool deflate = eligible(p, s, AMBC_M_DEFLATE);
    uint32_t gd_cmax = 1024;
    while (gd_cmax < C) gd_cmax <<= 1;
    if ((deflate || dict) && !eval) {       // RLE / Huffman payloads wait for ids 2 / 5
        HIPCHK(b.pending.ensure((size_t)cnt));
        ea.pending = b.pending.as<uint8_t>();
    }
    if (deflate) {
        HIPCHK(b.bestpre.ensure((size_t)cnt * 4));
        HIPCHK(b.gdseq.ensure((size_t)cnt * gd_seq_bytes(gd_cmax)));
        ea.bestpre = b.bestpre.as<uint32_t>();
        ea.gdseq = b.gdseq.as<uint8_t>();
        if (p->flags & AMBC_FLAG_ZLIB9) {
            HIPCHK(b.z9rec.ensure((size_t)cnt * z9_rec_words(z9_cmax(C)) * 4));
            ea.z9rec = b.z9rec.as<uint32_t>();
            if (z9_cmax(C) > 8192) {
                HIPCHK(b.z9scr.ensure(z9_scratch_bytes(z9_cmax(C), cnt)));
                ea.z9scr = b.z9scr.as<uint8_t>();
            }
        }
    }
    HIPCHK(launch_encode(ea, st));
    if (dict) HIPCHK(launch_dict(ea, std::min<uint32_t>(C, p->pref_max[AMBC_M_DICT]), st));
    if (deflate) HIPCHK((p->flags & AMBC_FLAG_ZLIB9) ? launch_zlib9(ea, st) : launch_deflate(ea, st));
    if (ea.pending) {
        EncArgs ep = ea;
        ep.flags |= ENC_EMIT_PENDING;
        ep.bestpre = nullptr;
        HIPCHK(launch_encode(ep, st));
    }
    HIPCHK(hipMemcpyAsync(b.hplen, b.plen.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(b.hids, b.ids.p, cnt, hipMemcpyDeviceToHost, st));
    if (nsub) HIPCHK(hipMemcpyAsync(b.hlz, b.lz4sub.p, (size_t)cnt * LZ4_SUB_MAX * 4, hipMemcpyDeviceToHost, st));
    return AMBC_OK;
}

struct Decision {
    uint32_t s;      // chunk size taken at this position (the remainder when raw)
    uint32_t plen;
    uint8_t id;      // 255: the rest of the input as one raw package
    uint8_t host;    // the package comes from a host-scored method (ambc_host_codecs)
};

// Per walk position (pos = idx * g) and candidate index i: the evaluation of
// size S_i = min(cands[i], n - pos).  Part "O": the winner of the size's methods
// other than LZ4 -- or, at the position's LZ4 size M, of all of them; part "L":
// LZ4's block for S_i < M, from M's launch.  One record per position (its state
// and its nc candidates contiguous: two or three cache lines for the reference's
// eight candidates, where a field-per-array layout touched a dozen), in pages of
// 256 positions allocated when a walk first reaches them.
struct PosTable {
    static constexpr uint32_t PB = 8;
    struct Cand {
        uint32_t plen = 0, lz = 0xFFFFFFFFu, hlen = 0;
        uint8_t id = 255, hid = 0;                  // (hid / hlen: the host codecs' winner, 0: none)
        uint16_t pad = 0;
    };
    struct Rec {
        uint32_t have = 0, req = 0;                 // bit i: part O of candidate i known / asked for
        uint32_t hhave = 0, hreq = 0;               //   ... the host part of candidate i
        uint8_t mhave = 0, mreq = 0, decided = 0;   // M's launch known / asked for; decision taken
        uint8_t pad = 0;
        Decision dec{0, 0, 0, 0};
        uint32_t epoch = 0;                         // the call this record belongs to (0: none)
        Cand* c() { return reinterpret_cast<Cand*>(this + 1); }
    };
    static_assert(sizeof(Rec) % alignof(Cand) == 0, "candidates follow the record");
    uint64_t g = 1;
    int gsh = -1;                // log2(g) when g is a power of two (the reference's list: 1024)
    uint32_t nc = 0;
    size_t rsz = 0;              // bytes per position record
    uint32_t epoch = 0;
    std::vector<std::vector<uint8_t>>* pages = nullptr;   // the context's pool (Dev::ms_pages)
    std::unique_ptr<std::atomic<uint8_t>[]> pready;       // page i allocated (touch() from several threads)
    std::mutex pmu;
    static constexpr uint32_t BUSY = 0xFFFFFFFFu;         // a record being reset by one thread
    void init(uint64_t n, uint64_t g_, uint32_t nc_, Dev& d) {
        g = g_;
        gsh = (g & (g - 1)) == 0 ? __builtin_ctzll(g) : -1;
        nc = nc_;
        rsz = sizeof(Rec) + (size_t)nc * sizeof(Cand);
        pages = &d.ms_pages;
        if (d.ms_rsz != rsz) {   // another record layout: the pool starts over
            d.ms_pages.clear();
            d.ms_rsz = rsz;
        }
        const size_t np = (size_t)((n / g >> PB) + 1);
        if (d.ms_pages.size() < np) d.ms_pages.resize(np);
        if (++d.ms_epoch == 0) {   // (wrapped: no record may carry a reused epoch)
            d.ms_pages.clear();
            d.ms_pages.resize(np);
            d.ms_epoch = 1;
        }
        epoch = d.ms_epoch;
        pready.reset(new std::atomic<uint8_t>[d.ms_pages.size()]);
        for (size_t i = 0; i < d.ms_pages.size(); i++) pready[i].store(d.ms_pages[i].empty() ? 0 : 1);
    }
    std::vector<uint8_t>& page(size_t i) {
        if (!pready[i].load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> g(pmu);
            if (!pready[i].load(std::memory_order_relaxed)) {
                (*pages)[i].resize(rsz << PB);   // (zeros: epoch 0)
                pready[i].store(1, std::memory_order_release);
            }
        }
        return (*pages)[i];
    }
    // at() from several threads at once: the reset claimed by one of them
    Rec& touch(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        Rec* r = reinterpret_cast<Rec*>(page((size_t)(x >> PB)).data() + rsz * (uint32_t)(x & ((1u << PB) - 1)));
        uint32_t e = __atomic_load_n(&r->epoch, __ATOMIC_ACQUIRE);
        while (e != epoch) {
            if (e != BUSY && __atomic_compare_exchange_n(&r->epoch, &e, BUSY, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                Rec fresh;
                fresh.epoch = BUSY;
                std::memcpy(static_cast<void*>(r), &fresh, sizeof(Rec));
                for (uint32_t i = 0; i < nc; i++) new (r->c() + i) Cand();
                __atomic_store_n(&r->epoch, epoch, __ATOMIC_RELEASE);
                break;
            }
            while ((e = __atomic_load_n(&r->epoch, __ATOMIC_ACQUIRE)) == BUSY) std::this_thread::yield();
        }
        return *r;
    }
    // the record of position pos if this call touched it already, else null (no
    // writes: safe beside other readers)
    Rec* peek(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        if (!pready[(size_t)(x >> PB)].load(std::memory_order_acquire)) return nullptr;
        const std::vector<uint8_t>& pg = (*pages)[(size_t)(x >> PB)];
        Rec* r = reinterpret_cast<Rec*>(const_cast<uint8_t*>(pg.data()) + rsz * (uint32_t)(x & ((1u << PB) - 1)));
        return r->epoch == epoch ? r : nullptr;
    }
    // the record of position pos: its page created on first use in the context,
    // the record reset on first use in this call
    Rec& at(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        const uint32_t slot = (uint32_t)(x & ((1u << PB) - 1));
        Rec* r = reinterpret_cast<Rec*>(page((size_t)(x >> PB)).data() + rsz * slot);
        if (r->epoch != epoch) {
            new (r) Rec();
            r->epoch = epoch;
            for (uint32_t i = 0; i < nc; i++) new (r->c() + i) Cand();
        }
        return *r;
    }
};

}  // namespace
}  // namespace ambc

using namespace ambc;

extern "C" int ambc_compress_multisize(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                                       const uint32_t* cands, uint32_t n_cands, const uint32_t* ent_sizes,
                                       const double* const* ent_tabs, uint32_t n_ent, uint8_t* out,
                                       uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    return ambc_compress_multisize_ex(ctx, in, n, p, cands, n_cands, ent_sizes, ent_tabs, n_ent, nullptr, out, out_cap,
                                      out_len, st);
}

extern "C" int ambc_compress_multisize_ex(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                                          const uint32_t* cands_in, uint32_t n_cands_in, const uint32_t* ent_sizes,
                                          const double* const* ent_tabs, uint32_t n_ent, const ambc_host_codecs* hc,
                                          uint8_t* out, uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    if (hc && (!hc->eval || !hc->emit)) hc = nullptr;
    if (!ctx || ctx->devs.empty() || !p || !out_len || (n && !in) || !cands_in || !n_cands_in)
        return fail(AMBC_E_INVAL, "bad arguments");
    for (uint32_t i = 0; i < n_cands_in; i++)
        if (cands_in[i] == 0 || cands_in[i] > (1u << 17)) return fail(AMBC_E_INVAL, "candidate sizes must be in [1, 131072]");
    const uint32_t allowed = (1u << AMBC_M_RLE) | (1u << AMBC_M_DICT) | (1u << AMBC_M_HUFFMAN) |
                             (1u << AMBC_M_DELTA) | (1u << AMBC_M_DEFLATE) | (1u << AMBC_M_LZ4);
    if (p->method_mask & ~allowed)
        return fail(AMBC_E_INVAL, "method_mask holds ids without a GPU encoder (allowed: 1, 2, 3, 4, 5, 9)");
    // a repeated candidate is the same package with the same ratio: never strictly better
    std::vector<uint32_t> cands;
    for (uint32_t i = 0; i < n_cands_in; i++)
        if (std::find(cands.begin(), cands.end(), cands_in[i]) == cands.end()) cands.push_back(cands_in[i]);
    const uint32_t nc = (uint32_t)cands.size();
    if (nc > 32) return fail(AMBC_E_INVAL, "at most 32 distinct candidate sizes");
    const uint64_t t0 = now_ns();
    Dev& d = ctx->devs[0];
    d.ms_body = 0;                 // a body left by an earlier call is gone from here on
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    // the entropy tables, uploaded once per call (a per-batch upload from the
    // caller's pageable arrays held the host until the stream's hardware queue
    // drained: the round's batches then ran one after another)
    std::map<uint32_t, const double*> ent;
    {
        size_t tot = 0;
        for (uint32_t i = 0; i < n_ent; i++)
            if (ent_tabs && ent_tabs[i]) tot += ((size_t)ent_sizes[i] + 1) * 8;
        if (tot) {
            HIPCHK(d.ms_ent.ensure(tot));
            std::vector<uint8_t> stage(tot);
            size_t o = 0;
            for (uint32_t i = 0; i < n_ent; i++) {
                if (!ent_tabs || !ent_tabs[i]) continue;
                const size_t b = ((size_t)ent_sizes[i] + 1) * 8;
                std::memcpy(stage.data() + o, ent_tabs[i], b);
                ent[ent_sizes[i]] = reinterpret_cast<const double*>(d.ms_ent.as<uint8_t>() + o);
                o += b;
            }
            HIPCHK(hipMemcpy(d.ms_ent.p, stage.data(), tot, hipMemcpyHostToDevice));
        }
    }
    auto ent_of = [&](uint32_t sz) -> const double* {
        auto it = ent.find(sz);
        return it == ent.end() ? nullptr : it->second;
    };
    // the input, uploaded once (64 bytes of slack for the encoders' padded loads)
    HIPCHK(d.in.ensure(n + 64));
    // (a large upload runs on a thread of its own while the first round is planned;
    // the first launch waits for it)
    std::thread upload;
    int upload_rc = AMBC_OK;
    struct Joiner {
        std::thread& t;
        ~Joiner() { if (t.joinable()) t.join(); }
    } upload_join{upload};
    auto await_upload = [&]() -> int {
        if (upload.joinable()) upload.join();
        return upload_rc;
    };
    if (n >= kStageMin) {
        upload = std::thread([&] { upload_rc = copy_staged(d, d.in.p, in, n, true, 0, 8); });
    } else if (n) {
        HIPCHK(hipMemcpyAsync(d.in.p, in, n, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemsetAsync(d.in.as<uint8_t>() + n, 0, 64, s));
    const uint8_t* d_in = d.in.as<uint8_t>();

    // ---- LZ4 shared across sizes: M (the largest LZ4-eligible size at a position)
    // reports the smaller LZ4-eligible candidates' prefixes (sorted list subc) ----
    std::vector<uint32_t> subc(cands);
    std::sort(subc.begin(), subc.end());
    const bool lzshare = ((p->method_mask >> AMBC_M_LZ4) & 1) && subc.size() <= LZ4_SUB_MAX &&
                         !getenv("AMBC_MS_NOSHARE");
    ambc_params po = *p;                       // the other methods (sizes below M)
    if (lzshare) po.method_mask &= ~(1u << AMBC_M_LZ4);
    const uint32_t nsub = (uint32_t)subc.size();

    // ---- the walks ----
    uint64_t g = 0;
    for (uint32_t c : cands) g = std::gcd(g, (uint64_t)c);
    PosTable T;
    T.init(n, g, nc, d);
    // last: the size it took the step before; cq / cs: the guess chain asked for so
    // far (positions pos + k * cs below cq are requested already)
    struct Walk { uint64_t pos; uint32_t last; uint64_t cq = 0; uint32_t cs = 0; };
    std::vector<Walk> active;
    // walks: one per 256 KiB, at most 1024 (256 MiB of mixed data, reference
    // candidates, second call: best of 512-2048 walks x 2-4 positions ahead,
    // profiles/r3_multisize_sweep.log; AMBC_MS_WALKS / AMBC_MS_SPAN / AMBC_MS_SPEC
    // override them for such sweeps)
    static const uint64_t KMAX_ = getenv("AMBC_MS_WALKS") ? strtoull(getenv("AMBC_MS_WALKS"), nullptr, 10) : 1024;
    static const uint64_t SPAN_ = getenv("AMBC_MS_SPAN") ? strtoull(getenv("AMBC_MS_SPAN"), nullptr, 10) : 256 << 10;
    uint32_t max_cand = 0;
    for (uint32_t c : cands)
        if (hc || any_eligible(p, c)) max_cand = std::max(max_cand, c);
    {
        // walk starts on the lattice of the largest eligible size: where that size
        // wins everywhere (homogeneous data) every walk runs on the same lattice
        // and joins the next one at once; elsewhere the mixed choices shift their
        // phases until they meet
        const uint64_t K = std::max<uint64_t>(1, std::min<uint64_t>(KMAX_, n / std::max<uint64_t>(SPAN_, 1)));
        const uint64_t lat = max_cand ? max_cand : g;
        std::vector<uint64_t> starts;
        for (uint64_t k = 0; k < K; k++) starts.push_back((k * n / K) / lat * lat);
        starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
        if (n)
            for (uint64_t b0 : starts) active.push_back(Walk{b0, max_cand ? max_cand : cands[0]});
    }
    // slot 0 of each group (the round's largest size: its encode is the round's
    // latency) on a high-priority stream, the smaller sizes fill in around it
    for (int i = 0; i < 16; i++) {
        if (d.mss[i]) continue;
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&d.mss[i], hipStreamNonBlocking, (i % 8) == 0 ? hi : lo));
    }
    HIPCHK(hipStreamSynchronize(s));                   // (the input upload)

    // the sizes at pos: S[i] = min(cands[i], remain); canonical = the first index
    // of its size; M = the largest LZ4-eligible one (0: none / no sharing)
    struct Sizes { uint32_t S[32]; uint32_t canon; uint32_t M; };
    const uint32_t maxc = *std::max_element(cands.begin(), cands.end());
    Sizes inner;                                       // every position with remain >= maxc
    bool have_inner = false;
    uint32_t jsub[32];                                 // subc index of cands[i]
    for (uint32_t i = 0; i < nc; i++)
        jsub[i] = (uint32_t)(std::lower_bound(subc.begin(), subc.end(), cands[i]) - subc.begin());
    auto sizes_fill = [&](uint64_t pos, Sizes& z) {
        const uint64_t remain = n - pos;
        z.canon = 0;
        z.M = 0;
        for (uint32_t i = 0; i < nc; i++) {
            z.S[i] = (uint32_t)std::min<uint64_t>(cands[i], remain);
            bool dup = false;
            for (uint32_t j = 0; j < i && !dup; j++) dup = z.S[j] == z.S[i];
            if (!dup) z.canon |= 1u << i;
            if (lzshare && eligible(p, z.S[i], AMBC_M_LZ4)) z.M = std::max(z.M, z.S[i]);
        }
    };
    if (n >= maxc) {
        sizes_fill(0, inner);
        have_inner = true;
    }
    // the sizes at pos: inner's by reference, a position near the end's in a scratch
    // record (valid until the next call)
    Sizes edge;
    auto sizes_in = [&](uint64_t pos, Sizes& scratch) -> const Sizes& {   // (thread-safe with its own scratch)
        if (have_inner && n - pos >= maxc) return inner;
        sizes_fill(pos, scratch);
        return scratch;
    };
    auto sizes_at = [&](uint64_t pos) -> const Sizes& { return sizes_in(pos, edge); };
    // part O of candidate i at a position: needed (not raw by construction)?
    auto needs_o = [&](const Sizes& z, uint32_t i) {
        return z.S[i] == z.M ? false : any_eligible(lzshare ? &po : p, z.S[i]);
    };
    auto needs_m = [&](const Sizes& z) { return z.M != 0; };
    auto ready_z = [&](const Sizes& z, const PosTable::Rec& r) -> bool {
        if (needs_m(z) && !r.mhave) return false;
        for (uint32_t i = 0; i < nc; i++)
            if (((z.canon >> i) & 1) && needs_o(z, i) && !((r.have >> i) & 1)) return false;
        if (hc && (r.hhave & z.canon) != z.canon) return false;
        return true;
    };
    // the reference's decision at pos (adaptive_compressor.py:546-590), all parts known
    auto decide_z = [&](uint64_t pos, const Sizes& z, PosTable::Rec& rec) -> Decision {
        const PosTable::Cand* cd = rec.c();
        const uint64_t remain = n - pos;
        double best_ratio = 1.0;
        uint32_t best_s = 0, best_plen = 0;
        uint8_t best_id = 255, best_host = 0;
        for (uint32_t i = 0; i < nc; i++) {
            // (the same clamped size again: same package, same ratio -- never strictly better)
            if (!((z.canon >> i) & 1)) continue;
            const uint32_t sz = z.S[i];
            if (!hc && !any_eligible(p, sz)) continue;
            const PosTable::Cand& e = cd[i];
            uint32_t plen = e.plen;
            uint8_t id = e.id;
            uint8_t host = 0;
            if (sz != z.M && !needs_o(z, i)) id = 255;            // no other method: raw so far
            if (lzshare && sz < z.M && eligible(p, sz, AMBC_M_LZ4)) {
                // id 9 comes last in id order: it wins only strictly below the others
                const uint32_t lb = e.lz;
                const uint32_t other = id == 255 ? sz : plen + HDR;
                if (lb != 0xFFFFFFFFu && (uint64_t)lb + 41 < other) { plen = lb + 23; id = 9; }
            }
            if (hc && e.hid && e.hlen + HDR < sz) {
                // the host codecs' winner joins in id order: smaller len, or a tie with a higher id
                const uint32_t hl = e.hlen;
                const uint8_t hi = e.hid;
                if (id == 255 || hl < plen || (hl == plen && hi < id)) { plen = hl; id = hi; host = 1; }
            }
            if (id == 255) continue;
            const double ratio = (double)(plen + HDR) / (double)sz;
            if (ratio < best_ratio) {
                best_ratio = ratio;
                best_s = sz;
                best_plen = plen;
                best_id = id;
                best_host = host;
            }
        }
        if (best_id == 255)
            return Decision{(uint32_t)std::min<uint64_t>(remain, 0xFFFFFFFFull), (uint32_t)remain, 255, 0};
        return Decision{best_s, best_plen, best_id, best_host};
    };
    // host-codec requests of one round: (position, size), and where they go
    std::vector<uint64_t> hpos;
    std::vector<uint32_t> hsize;
    // requests of one round: (size, kind) -> positions; kind 1 = M's launch.  A
    // handful of buckets, found by a short scan -- for inner positions (every size
    // the candidate's own) by a per-candidate cache
    using ReqKey = std::pair<uint32_t, int>;
    std::vector<std::pair<ReqKey, std::vector<uint64_t>>> req;
    int req_in[33];                                    // bucket of inner candidate i (32: M), -1: none yet
    auto req_clear = [&]() {
        req.clear();
        for (int& x : req_in) x = -1;
    };
    req_clear();
    auto req_bucket = [&](ReqKey key) -> std::vector<uint64_t>& {
        for (auto& b : req)
            if (b.first == key) return b.second;
        req.emplace_back(key, std::vector<uint64_t>());
        return req.back().second;
    };
    auto req_push = [&](bool in, int ci, ReqKey key, uint64_t pos) {
        if (!in) { req_bucket(key).push_back(pos); return; }
        if (req_in[ci] < 0) {
            req_bucket(key);
            for (size_t b = 0; b < req.size(); b++)
                if (req[b].first == key) req_in[ci] = (int)b;
        }
        req[(size_t)req_in[ci]].second.push_back(pos);
    };
    auto request = [&](uint64_t pos) {
        const Sizes& z = sizes_at(pos);
        const bool in = &z == &inner;
        PosTable::Rec& r = T.at(pos);
        if (needs_m(z) && !r.mhave && !r.mreq) {
            r.mreq = 1;
            req_push(in, 32, {z.M, 1}, pos);
        }
        for (uint32_t i = 0; i < nc; i++) {
            if (!((z.canon >> i) & 1)) continue;
            if (hc && !(((r.hhave | r.hreq) >> i) & 1)) {
                r.hreq |= 1u << i;
                hpos.push_back(pos);
                hsize.push_back(z.S[i]);
            }
            if (!needs_o(z, i)) continue;
            if (((r.have | r.req) >> i) & 1) continue;
            r.req |= 1u << i;
            req_push(in, (int)i, {z.S[i], 0}, pos);
        }
    };
    // the host codecs' answers for the round's pairs into the table
    std::vector<uint8_t> hid_out;
    std::vector<uint32_t> hlen_out;
    uint64_t t_host = 0;
    auto host_round = [&]() -> int {
        if (!hc || hpos.empty()) return AMBC_OK;
        const uint64_t th = now_ns();
        hid_out.assign(hpos.size(), 0);
        hlen_out.assign(hpos.size(), 0);
        if (hc->eval(hc->user, hpos.data(), hsize.data(), (uint32_t)hpos.size(), hid_out.data(), hlen_out.data()))
            return fail(AMBC_E_CODEC, "host codec evaluation failed");
        for (size_t q = 0; q < hpos.size(); q++) {
            const Sizes& z = sizes_at(hpos[q]);
            PosTable::Rec& r = T.at(hpos[q]);
            for (uint32_t i = 0; i < nc; i++)
                if (((z.canon >> i) & 1) && z.S[i] == hsize[q]) {
                    r.c()[i].hid = hid_out[q];
                    r.c()[i].hlen = hlen_out[q];
                    r.hhave |= 1u << i;
                }
        }
        hpos.clear();
        hsize.clear();
        t_host += now_ns() - th;
        return AMBC_OK;
    };
    // a batch's results into the table
    // (a batch's positions are distinct and were touched when requested: its
    // records fill in parallel, read through peek)
    WalkPool& pool = WalkPool::get();
    auto fill_range = [&](const Batch& bb, uint32_t sz, int kind, const std::vector<uint64_t>& poss, size_t q0,
                          size_t q1) {
        Sizes scr;
        for (size_t q = q0; q < q1; q++) {
            const uint64_t pos = poss[q];
            const Sizes& z = sizes_in(pos, scr);
            PosTable::Rec& r = *T.peek(pos);
            PosTable::Cand* cd = r.c();
            for (uint32_t i = 0; i < nc; i++) {
                if (!((z.canon >> i) & 1)) continue;
                if (z.S[i] == sz && (kind == 1 || z.S[i] != z.M)) {
                    cd[i].plen = bb.hplen[q];
                    cd[i].id = bb.hids[q];
                    r.have |= 1u << i;
                }
                if (kind == 1 && z.S[i] < z.M) cd[i].lz = bb.hlz[q * LZ4_SUB_MAX + jsub[i]];   // (S[i] = cands[i])
            }
            if (kind == 1) r.mhave = 1;
        }
    };
    auto fill = [&](const Batch& bb, uint32_t sz, int kind, const std::vector<uint64_t>& poss) {
        const size_t m = poss.size();
        if (m < 2048 || pool.size() == 1) { fill_range(bb, sz, kind, poss, 0, m); return; }
        pool.run([&](unsigned t, unsigned Tn) { fill_range(bb, sz, kind, poss, m * t / Tn, m * (t + 1) / Tn); });
    };

    uint32_t steps = 0;
    uint64_t evaluated = 0;
    uint64_t kernel_ns = 0;
    // Rounds: every walk decides as far as the known sizes reach; then ONE batch
    // per size evaluates each walk's next position and SPEC positions further
    // along the path it would take if it kept its last step size (a guess: a
    // right one saves a round, whose latency -- the slowest 64 KiB encode -- is
    // the walk's cost; a wrong one costs idle device time only).  AMBC_MS_GROUPS=2
    // runs the walks as two interleaved groups (the host decides and launches one
    // group while the device encodes the other's): measured slower -- 256 MiB
    // {1,3,4,9}: 55.8 -> 81.5 ms of walk at 1024 walks / 3 ahead, the groups'
    // batches contend on the device -- so one group is the default.
    // (speculation is cheap where one LZ4 parse serves every size: 6 ahead; where
    // every size runs its own encoders -- DEFLATE, zlib-9, Dictionary -- 1 ahead:
    // 256 MiB {1,3,4,9}: 4 / 5 / 6 / 8 ahead 72.4 / 64.1 / 58.4 / 94.9 ms (8 with
    // 2048 walks), {1,2,3,4,5}: 1 / 2 ahead 86.0 / 90.6 ms, like_reference() on 64
    // MiB: 0 / 1 / 2 ahead 0.229 / 0.255 / 0.224 GB/s; profiles/r3_multisize_sweep.log)
    // (round 4, with breadth speculation for the last walks: {1,2,3,4,5} 0 / 1 / 2
    // ahead 4.61-4.77 / 4.48-4.53 / 3.93-3.97 GB/s; like_reference() -- no breadth --
    // 0.31 / 0.34 / 0.28, profiles/r4_spec_ab)
    static const int SPEC_ENV = getenv("AMBC_MS_SPEC") ? atoi(getenv("AMBC_MS_SPEC")) : -1;
    const bool z9walk = (p->flags & AMBC_FLAG_ZLIB9) && ((p->method_mask >> AMBC_M_DEFLATE) & 1);
    const int SPEC = SPEC_ENV >= 0 ? SPEC_ENV : (lzshare ? 6 : z9walk ? 1 : 0);
    static const int GROUPS = getenv("AMBC_MS_GROUPS") ? std::max(1, std::min(2, atoi(getenv("AMBC_MS_GROUPS")))) : 1;
    uint64_t t_dec = 0, t_req = 0, t_launch = 0, t_wait = 0, t_fill = 0;   // (AMBC_TRACE breakdown)
    using Job = std::pair<std::pair<uint32_t, int>, std::vector<uint64_t>>;
    struct Group {
        std::vector<Walk> active;
        std::vector<Job> flight;     // batches on slots slot0.. (at most 8)
        int slot0 = 0;
        uint32_t rounds = 0;
    };
    Group grp[2];
    for (int g = 0; g < GROUPS; g++) grp[g].slot0 = 8 * g;
    for (size_t i = 0; i < active.size(); i++) grp[i % GROUPS].active.push_back(active[i]);
    auto launch_job = [&](const Job& jb, int slot) -> int {
        Batch& bb = d.msb[slot];
        const uint32_t cnt = (uint32_t)jb.second.size();
        HIPCHK(bb.host_ensure(cnt));
        std::memcpy(bb.hpos, jb.second.data(), (size_t)cnt * 8);
        const bool mk = jb.first.second == 1;
        return launch_batch(bb, d.mss[slot], d_in, n, mk || !lzshare ? p : &po, jb.first.first, bb.hpos, cnt,
                            ent_of(jb.first.first), true, mk ? subc.data() : nullptr, mk ? nsub : 0);
    };
    auto finish_job = [&](const Job& jb, int slot) -> int {
        uint64_t tl = now_ns();
        HIPCHK(hipStreamSynchronize(d.mss[slot]));
        t_wait += now_ns() - tl;
        tl = now_ns();
        fill(d.msb[slot], jb.first.first, jb.first.second, jb.second);
        evaluated += jb.second.size();
        t_fill += now_ns() - tl;
        return AMBC_OK;
    };
    // the group's batches in flight: wait and take their results
    auto complete = [&](Group& G) -> int {
        const uint64_t tk = now_ns();
        for (size_t j = 0; j < G.flight.size(); j++)
            if (int rc = finish_job(G.flight[j], G.slot0 + (int)j)) return rc;
        G.flight.clear();
        kernel_ns += now_ns() - tk;
        return AMBC_OK;
    };
    // decide as far as known, then ask for the next positions and launch
    auto advance = [&](Group& G) -> int {
        uint64_t tq = now_ns();
        // phase 1, in parallel and read-only: every walk's steps as far as its
        // positions are known; phase 2, in walk order: the steps into the table, a
        // walk stopping where an earlier one decided already (it joined that path:
        // the same decisions from there on) -- the sequential loop's outcome
        const size_t na = G.active.size();
        struct Trail { std::vector<std::pair<uint64_t, Decision>> steps; Walk end; bool open; };
        std::vector<Trail> trails(na);
        auto walk_range = [&](size_t a0, size_t a1) {
            Sizes scr;
            for (size_t a = a0; a < a1; a++) {
                Trail& tr = trails[a];
                tr.steps.clear();
                Walk w = G.active[a];
                tr.open = false;
                for (;;) {
                    PosTable::Rec* r = T.peek(w.pos);
                    if (r && r->decided) break;            // joined a decided path
                    const Sizes& z = sizes_in(w.pos, scr);
                    if (!r || !ready_z(z, *r)) { tr.open = true; break; }
                    const Decision dd = decide_z(w.pos, z, *r);
                    tr.steps.emplace_back(w.pos, dd);
                    if (dd.id == 255) break;               // the rest is raw: done
                    w.last = dd.s;
                    w.pos += dd.s;
                    if (w.pos >= n) break;
                }
                tr.end = w;
            }
        };
        if (na < 64 || pool.size() == 1) walk_range(0, na);
        else pool.run([&](unsigned t, unsigned Tn) { walk_range(na * t / Tn, na * (t + 1) / Tn); });
        std::vector<Walk> still;
        for (size_t a = 0; a < na; a++) {
            Trail& tr = trails[a];
            bool joined = false;
            for (const auto& st : tr.steps) {
                PosTable::Rec& r = T.at(st.first);
                if (r.decided) { joined = true; break; }
                r.decided = 1;
                r.dec = st.second;
            }
            if (joined || !tr.open) continue;
            PosTable::Rec* r = T.peek(tr.end.pos);
            if (r && r->decided) continue;                  // (decided by an earlier walk this round)
            still.push_back(tr.end);
        }
        // (two walks at one position: keep one)
        std::sort(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos < y.pos; });
        still.erase(std::unique(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos == y.pos; }),
                    still.end());
        G.active.swap(still);
        t_dec += now_ns() - tq;
        tq = now_ns();
        if (G.active.empty()) return AMBC_OK;
        req_clear();
        hpos.clear();
        hsize.clear();
        static const bool rechain = getenv("AMBC_MS_RECHAIN") != nullptr;
        // each walk's guess chain; many walks: on the pool, the records claimed by
        // atomic bit sets, the positions into per-thread buckets merged afterwards
        auto chain_of = [&](Walk& w, auto&& ask, auto&& rec_of) {
            uint64_t q = w.pos;
            int k = 0;
            // still on last round's chain: its requested prefix is skipped (with SPEC
            // 6 a walk re-asked for six positions a round, most of them known)
            if (!rechain && w.cs == w.last && w.cq > w.pos && (w.cq - w.pos) % w.last == 0) {
                k = (int)std::min<uint64_t>((w.cq - w.pos) / w.last, (uint64_t)SPEC + 1);
                q = w.pos + (uint64_t)k * w.last;
                // the walk's own position is always asked for again (its record
                // knows what is requested already): a speculative request there
                // may have been forgotten (a size check_size refuses), and the walk
                // would otherwise wait for it forever
                ask(w.pos);
            }
            for (; k <= SPEC && q < n; k++, q += w.last) {
                if (k && rec_of(q).decided) break;
                ask(q);
            }
            w.cs = w.last;
            w.cq = q;
        };
        const size_t nw = G.active.size();
        if (nw < 64 || pool.size() == 1) {
            for (Walk& w : G.active) chain_of(w, request, [&](uint64_t q) -> PosTable::Rec& { return T.at(q); });
        } else {
            struct TL {
                std::vector<std::pair<ReqKey, std::vector<uint64_t>>> b;
                int in_idx[33];
                std::vector<uint64_t> hp;
                std::vector<uint32_t> hs;
            };
            std::vector<TL> tl(pool.size());
            pool.run([&](unsigned t, unsigned Tn) {
                TL& L = tl[t];
                for (int& x : L.in_idx) x = -1;
                Sizes scr;
                auto push = [&](bool in, int ci, ReqKey key, uint64_t pos) {
                    int bi = in ? L.in_idx[ci] : -1;
                    if (bi < 0) {
                        for (size_t b = 0; b < L.b.size() && bi < 0; b++)
                            if (L.b[b].first == key) bi = (int)b;
                        if (bi < 0) { L.b.emplace_back(key, std::vector<uint64_t>()); bi = (int)L.b.size() - 1; }
                        if (in) L.in_idx[ci] = bi;
                    }
                    L.b[(size_t)bi].second.push_back(pos);
                };
                auto ask = [&](uint64_t pos) {
                    const Sizes& z = sizes_in(pos, scr);
                    const bool in = &z == &inner;
                    PosTable::Rec& r = T.touch(pos);
                    if (needs_m(z) && !r.mhave && !__atomic_exchange_n(&r.mreq, (uint8_t)1, __ATOMIC_ACQ_REL))
                        push(in, 32, {z.M, 1}, pos);
                    uint32_t want = 0, hwant = 0;
                    for (uint32_t i = 0; i < nc; i++) {
                        if (!((z.canon >> i) & 1)) continue;
                        if (hc && !((r.hhave >> i) & 1)) hwant |= 1u << i;
                        if (needs_o(z, i) && !((r.have >> i) & 1)) want |= 1u << i;
                    }
                    if (hwant) {
                        const uint32_t got = hwant & ~__atomic_fetch_or(&r.hreq, hwant, __ATOMIC_ACQ_REL);
                        for (uint32_t i = 0; i < nc; i++)
                            if ((got >> i) & 1) { L.hp.push_back(pos); L.hs.push_back(z.S[i]); }
                    }
                    if (want) {
                        const uint32_t got = want & ~__atomic_fetch_or(&r.req, want, __ATOMIC_ACQ_REL);
                        for (uint32_t i = 0; i < nc; i++)
                            if ((got >> i) & 1) push(in, (int)i, {z.S[i], 0}, pos);
                    }
                };
                for (size_t a = nw * t / Tn; a < nw * (t + 1) / Tn; a++)
                    chain_of(G.active[a], ask, [&](uint64_t q) -> PosTable::Rec& { return T.touch(q); });
            });
            for (TL& L : tl) {
                for (auto& b : L.b) {
                    std::vector<uint64_t>& dst = req_bucket(b.first);
                    dst.insert(dst.end(), b.second.begin(), b.second.end());
                }
                hpos.insert(hpos.end(), L.hp.begin(), L.hp.end());
                hsize.insert(hsize.end(), L.hs.begin(), L.hs.end());
            }
            for (int& x : req_in) x = -1;   // (bucket indices moved: the inner cache starts over)
        }
        // few walks left (the device idles behind one chunk's latency): each walk
        // also asks for every position its next step can reach, and a guess chain
        // from each, within BREADTH positions a round -- the next round then decides
        // at least two steps whatever size wins (AMBC_MS_BREADTH=0: off).  Budget: what
        // one round's latency hides, ~2048 chunks of 64 KiB ({1,2,3,4,5} 3.55-3.60 ->
        // 3.79-3.80 GB/s, {1,3,4,9} unchanged); none with zlib-9, whose 64 KiB parse
        // holds a CU per chunk (like_reference() 0.33 -> 0.20 GB/s with it,
        // profiles/r4_breadth_ab)
        static const int64_t BREADTH_ENV = getenv("AMBC_MS_BREADTH") ? atoll(getenv("AMBC_MS_BREADTH")) : -1;
        const uint64_t BREADTH = BREADTH_ENV >= 0 ? (uint64_t)BREADTH_ENV
                                                  : (z9walk ? 0 : 2048);
        if (BREADTH && !G.active.empty() && G.active.size() * nc <= BREADTH) {
            const uint64_t per = BREADTH / G.active.size();
            for (const Walk& w : G.active) {
                const Sizes z = sizes_at(w.pos);           // (a copy: request() reuses the scratch)
                const uint32_t nsz = (uint32_t)__builtin_popcount(z.canon);
                const uint64_t depth = std::min<uint64_t>((uint64_t)SPEC + 1, std::max<uint64_t>(1, per / nsz));
                for (uint32_t i = 0; i < nc; i++) {
                    if (!((z.canon >> i) & 1) || z.S[i] == w.last) continue;   // (the main chain)
                    uint64_t q = w.pos + z.S[i];
                    for (uint64_t k = 0; k < depth && q < n; k++, q += z.S[i]) {
                        if (T.at(q).decided) break;
                        request(q);
                    }
                }
            }
        }
        std::vector<Job> jobs;
        for (auto& r : req) {
            const ambc_params* pk = r.first.second == 1 || !lzshare ? p : &po;
            if (int rc = check_size(pk, r.first.first)) {
                // only an error if a walk itself needs this size (not a speculative position)
                for (uint64_t q : r.second)
                    if (std::binary_search(G.active.begin(), G.active.end(), Walk{q, 0},
                                           [](const Walk& x, const Walk& y) { return x.pos < y.pos; }))
                        return rc;
                // speculative only: never decided from -- forget the requests
                for (uint64_t q : r.second) {
                    const Sizes& z = sizes_at(q);
                    PosTable::Rec& rec = T.at(q);
                    if (r.first.second == 1) rec.mreq = 0;
                    for (uint32_t i = 0; i < nc; i++)
                        if (z.S[i] == r.first.first) rec.req &= ~(1u << i);
                }
                continue;
            }
            jobs.emplace_back(r.first, std::move(r.second));
        }
        // the largest size first (slot 0, the high-priority stream)
        static const bool noprio = getenv("AMBC_MS_NOPRIO") != nullptr;
        if (!noprio)
            std::stable_sort(jobs.begin(), jobs.end(), [](const Job& a, const Job& b) {
                return a.first.first != b.first.first ? a.first.first > b.first.first : a.first.second > b.first.second;
            });
        t_req += now_ns() - tq;
        if (!jobs.empty()) G.rounds++;
        // up to 8 batches at once, each on its own stream and batch buffers (the
        // 64 KiB class runs at 20 workgroups per CU in place: the small ones fill
        // in); more than 8: the earlier ones are finished here, the last 8 fly
        const uint64_t tk = now_ns();
        if (!jobs.empty())
            if (int rc = await_upload()) return rc;
        for (size_t j0 = 0; j0 < jobs.size(); j0 += 8) {
            const size_t j1 = std::min(jobs.size(), j0 + 8);
            const uint64_t tl = now_ns();
            // the largest size first (its own high-priority stream), then the rest
            // smallest first: streams share hardware queues, and a 1 KiB batch
            // queued behind an 8 KiB Dictionary chain ended the round
            static const bool desc = getenv("AMBC_MS_LAUNCH_DESC") != nullptr;
            for (size_t x = 0; x < j1 - j0; x++) {
                const size_t j = desc || x == 0 ? j0 + x : j1 - x;
                if (int rc = launch_job(jobs[j], G.slot0 + (int)(j - j0))) return rc;
            }
            t_launch += now_ns() - tl;
            if (j0 == 0)                           // the host codecs while the device works
                if (int rc = host_round()) return rc;
            if (j1 < jobs.size()) {
                for (size_t j = j0; j < j1; j++)
                    if (int rc = finish_job(jobs[j], G.slot0 + (int)(j - j0))) return rc;
            } else {
                for (size_t j = j0; j < j1; j++) G.flight.push_back(std::move(jobs[j]));
            }
        }
        if (jobs.empty())
            if (int rc = host_round()) return rc;
        kernel_ns += now_ns() - tk;
        return AMBC_OK;
    };
    // ---- the reference's walk from 0, read off the decisions as they come, and its
    // packages encoded once more (bytes) beside the walk's later rounds ----
    struct Pkg { uint64_t pos; uint32_t s, plen; uint8_t id, host; uint64_t off; };
    std::vector<Pkg> path;
    uint64_t body = 0, path_pos = 0;
    bool path_end = false;
    // the body buffer at its largest: every package is smaller than its chunk but
    // the raw remainder, each adds a header
    const uint64_t body_cap = n + (uint64_t)HDR * (n / *std::min_element(cands.begin(), cands.end()) + 2) + END_CHUNK;
    HIPCHK(d.ms_out.ensure(body_cap + 64));
    uint8_t* d_body = d.ms_out.as<uint8_t>();
    auto extend_path = [&]() -> int {
        while (!path_end) {
            if (path_pos >= n) { path_end = true; break; }
            PosTable::Rec* r = T.peek(path_pos);
            if (!r || !r->decided) break;
            const Decision dd = r->dec;
            if (dd.id == 255 && n - path_pos > 0xFFFFFFFFull)
                return fail(AMBC_E_RANGE, "raw remainder exceeds a u32 chunk field");
            path.push_back(Pkg{path_pos, dd.s, dd.plen, dd.id, dd.host, body});
            body += HDR + (uint64_t)dd.plen;
            if (dd.id == 255) { path_end = true; break; }
            path_pos += dd.s;
        }
        return AMBC_OK;
    };
    // The final encode, after the walk: grouped by (size, winning id), each group
    // encoded with its winner alone -- the method encoders are deterministic, so the
    // winner's bytes are those of the full loop, and the losers' encoders (a 64 KiB
    // DEFLATE parse behind an RLE winner) do not run again; every package's plen / id
    // is checked against the walk's decision when its slot is done.  The groups go
    // onto all 15 batch slots as they free up (polled), not 8 at a time.  (Encoding
    // the path's packages beside the walk's later rounds was measured slower: the
    // walk's latency-bound rounds lose more than the final encode saves.)
    constexpr int FSN = 15;
    auto fslot = [](int k) { return k < 7 ? 9 + k : k - 7; };   // slots 9..15, then 0..7
    struct FinalJob { std::vector<size_t> idx; bool busy = false; };
    FinalJob fj[FSN];
    static const bool allm = getenv("AMBC_MS_FINAL_ALL") != nullptr;
    // verify slot k's group: blocking, or only if its stream is done (false: busy)
    auto final_finish = [&](int k, bool wait) -> int {
        if (!fj[k].busy) return AMBC_OK;
        if (wait) {
            HIPCHK(hipStreamSynchronize(d.mss[fslot(k)]));
        } else {
            const hipError_t q = hipStreamQuery(d.mss[fslot(k)]);
            if (q == hipErrorNotReady) return AMBC_OK;
            HIPCHK(q);
        }
        const Batch& bb = d.msb[fslot(k)];
        for (size_t q = 0; q < fj[k].idx.size(); q++) {
            const Pkg& pk = path[fj[k].idx[q]];
            if (bb.hplen[q] != pk.plen || bb.hids[q] != pk.id)
                return fail(AMBC_E_DEVICE, "multi-size walk: re-encode differs");
        }
        fj[k].busy = false;
        return AMBC_OK;
    };
    using FGroup = std::pair<std::pair<uint32_t, uint8_t>, std::vector<size_t>>;
    std::vector<FGroup> fpend;                       // groups waiting for a free slot
    auto final_group = [&](size_t i0, size_t i1) {
        std::map<std::pair<uint32_t, uint8_t>, std::vector<size_t>> groups;
        for (size_t i = i0; i < i1; i++)
            if (path[i].id != 255 && !path[i].host) groups[{path[i].s, allm ? (uint8_t)0 : path[i].id}].push_back(i);
        for (auto& gr : groups) fpend.emplace_back(gr.first, std::move(gr.second));
    };
    auto final_launch = [&](int k, FGroup& gr) -> int {
        const uint32_t sz = gr.first.first;
        ambc_params pw = *p;
        if (gr.first.second) pw.method_mask = 1u << gr.first.second;
        Batch& bb = d.msb[fslot(k)];
        hipStream_t xs = d.mss[fslot(k)];
        const uint32_t cnt = (uint32_t)gr.second.size();
        HIPCHK(bb.host_ensure(cnt));
        for (uint32_t q = 0; q < cnt; q++) {
            bb.hpos[q] = path[gr.second[q]].pos;
            bb.hoff[q] = path[gr.second[q]].off;
        }
        if (int rc = launch_batch(bb, xs, d_in, n, &pw, sz, bb.hpos, cnt, ent_of(sz), false)) return rc;
        HIPCHK(bb.off.ensure((size_t)cnt * 8));
        HIPCHK(hipMemcpyAsync(bb.off.p, bb.hoff, (size_t)cnt * 8, hipMemcpyHostToDevice, xs));
        CompactArgs ca{};
        ca.slots = bb.slots.as<uint8_t>();
        ca.slot_stride = slot_stride_for((sz + 15) & ~15u);
        ca.plen = bb.plen.as<uint32_t>();
        ca.ids = bb.ids.as<uint8_t>();
        ca.off = bb.off.as<uint64_t>();
        ca.n_chunks = cnt;
        ca.clen = bb.clen.as<uint32_t>();
        ca.n_total = n;
        ca.chunk_size = (sz + 15) & ~15u;
        ca.out = d_body;
        HIPCHK(launch_compact(ca, xs));
        fj[k].idx = std::move(gr.second);
        fj[k].busy = true;
        return AMBC_OK;
    };
    // the groups onto slots as they free up, then every slot done and checked
    auto final_run = [&]() -> int {
        size_t gi = 0;
        while (gi < fpend.size()) {
            bool launched = false;
            for (int k = 0; k < FSN && gi < fpend.size(); k++) {
                if (int rc = final_finish(k, false)) return rc;
                if (fj[k].busy) continue;
                if (int rc = final_launch(k, fpend[gi++])) return rc;
                launched = true;
            }
            if (!launched) std::this_thread::yield();
        }
        fpend.clear();
        for (int k = 0; k < FSN; k++)
            if (int rc = final_finish(k, true)) return rc;
        return AMBC_OK;
    };
    for (int g = 0; g < GROUPS; g++)
        if (int rc = advance(grp[g])) return rc;
    for (;;) {
        bool any = false;
        for (int g = 0; g < GROUPS; g++) {
            Group& G = grp[g];
            if (G.active.empty() && G.flight.empty()) continue;
            any = true;
            if (int rc = complete(G)) return rc;
            if (int rc = advance(G)) return rc;
        }
        if (!any) break;
    }
    for (int g = 0; g < GROUPS; g++) steps = std::max(steps, grp[g].rounds);

    const uint64_t t_walk = now_ns() - t0;
    TRACE("multisize walk ms: decide %.2f requests %.2f launch %.2f wait %.2f fill %.2f host %.2f (total %.2f)",
          t_dec / 1e6, t_req / 1e6, t_launch / 1e6, t_wait / 1e6, t_fill / 1e6, t_host / 1e6, t_walk / 1e6);
    if (int rc = await_upload()) return rc;
    if (int rc = extend_path()) return rc;
    if (!path_end) return fail(AMBC_E_DEVICE, "multi-size walk: undecided position on the path");
    body += END_CHUNK;
    d.ms_body = 0;
    if (out && out_cap < body) return fail(AMBC_E_CAPACITY, "output capacity below the body size");
    const uint64_t te = now_ns();
    // (largest chunks first: their encodes are the longest)
    final_group(0, path.size());
    std::stable_sort(fpend.begin(), fpend.end(), [](const FGroup& x, const FGroup& y) { return x.first.first > y.first.first; });
    if (int rc = final_run()) return rc;
    {   // host-scored packages: header + the caller's payload bytes
        std::vector<uint8_t> hb;
        for (const Pkg& pk : path) {
            if (!pk.host) continue;
            hb.assign((size_t)HDR + pk.plen, 0);
            const uint8_t h[6] = {0xFF, 0xFF, 0, 0, pk.id, 0};
            std::memcpy(hb.data(), h, 6);
            const uint32_t f[3] = {pk.s, pk.s, pk.plen};
            std::memcpy(hb.data() + 6, f, 12);
            if (hc->emit(hc->user, pk.pos, pk.s, pk.id, hb.data() + HDR, pk.plen))
                return fail(AMBC_E_CODEC, "host codec emit failed");
            HIPCHK(hipMemcpy(d_body + pk.off, hb.data(), hb.size(), hipMemcpyHostToDevice));
        }
    }
    if (!path.empty() && path.back().id == 255) {   // the raw remainder package
        const Pkg& pk = path.back();
        uint8_t h[HDR] = {0xFF, 0xFF, 0, 0, 255, 0};
        for (int b = 0; b < 4; b++) {
            h[6 + b] = (uint8_t)(pk.s >> (8 * b));
            h[10 + b] = (uint8_t)(pk.s >> (8 * b));
            h[14 + b] = (uint8_t)(pk.s >> (8 * b));
        }
        HIPCHK(hipMemcpyAsync(d_body + pk.off, h, HDR, hipMemcpyHostToDevice, s));
        HIPCHK(launch_copy(d_body + pk.off + HDR, d_in + pk.pos, pk.s, s));
    }
    HIPCHK(launch_end_chunk(d_body + body - END_CHUNK, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint64_t tc = now_ns();
    kernel_ns += tc - te;
    if (!out) {
        d.ms_body = body;                       // (ambc_fetch_body)
    } else if (body >= kStageMin) {
        int rc = copy_staged(d, out, d_body, body, false);
        if (rc) return rc;
    } else {
        HIPCHK(hipMemcpy(out, d_body, body, hipMemcpyDeviceToHost));
    }
    *out_len = body;
    d.ms_steps = steps;
    d.ms_evaluated = evaluated;
    d.ms_walk_ns = t_walk;
    d.ms_emit_ns = now_ns() - te;
    TRACE("multisize n=%llu steps=%u evaluated=%llu path=%zu emit %.2f ms (copy back %.2f)", (unsigned long long)n,
          steps, (unsigned long long)evaluated, path.size(), (now_ns() - te) / 1e6, (now_ns() - tc) / 1e6);
    if (st) {
        std::memset(st, 0, sizeof *st);
        for (const Pkg& pk : path) {
            st->total_chunks++;
            if (pk.id == 255) { st->raw_chunks++; continue; }
            st->compressed_chunks++;
            st->method_usage[pk.id]++;
            st->payload_bytes += pk.plen;
            st->bytes_saved += pk.s - (pk.plen + HDR);
        }
        st->overhead_bytes = (uint64_t)HDR * st->compressed_chunks + END_CHUNK;
        st->kernel_ns = kernel_ns;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

extern "C" int ambc_fetch_body(ambc_ctx* ctx, uint8_t* out, uint64_t cap) {
    if (!ctx || ctx->devs.empty() || !out) return fail(AMBC_E_INVAL, "bad arguments");
    Dev& d = ctx->devs[0];
    if (!d.ms_body) return fail(AMBC_E_INVAL, "no body kept on the device");
    if (cap < d.ms_body) return fail(AMBC_E_CAPACITY, "output capacity below the body size");
    HIPCHK(hipSetDevice(d.id));
    const uint64_t body = d.ms_body;
    d.ms_body = 0;
    if (body >= kStageMin) return copy_staged(d, out, d.ms_out.p, body, false);
    HIPCHK(hipMemcpy(out, d.ms_out.p, body, hipMemcpyDeviceToHost));
    return AMBC_OK;
}

extern "C" int ambc_last_multisize_info(ambc_ctx* ctx, uint32_t* steps, uint64_t* evaluated,
                                        uint64_t* walk_ns, uint64_t* emit_ns) {
    if (!ctx || ctx->devs.empty()) return fail(AMBC_E_INVAL, "bad context");
    if (steps) *steps = ctx->devs[0].ms_steps;
    if (evaluated) *evaluated = ctx->devs[0].ms_evaluated;
    if (walk_ns) *walk_ns = ctx->devs[0].ms_walk_ns;
    if (emit_ns) *emit_ns = ctx->devs[0].ms_emit_ns;
    return AMBC_OK;
}
