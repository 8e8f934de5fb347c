// ambc_multisize.cpp -- the reference's multi-size walk on the device.
//
// AdaptiveCompressor._adaptive_compress with several CHUNK_SIZE_CANDIDATES
// (adaptive_compressor.py:363-394 + _pick_best_chunk_and_method :537-590).  The
// walk's decisions are ambc_walkcore.h's (many lock-step walks, one batch per
// candidate size and round); this file is its device backend -- each batch is
// the encoders over the chunks read in place from the uploaded input through a
// chunk-offset table (k_encode / k_dict / k_deflate / zlib-9, one workgroup per
// chunk), decision only (ENC_EVAL: no payload bytes), up to 8 batches in flight
// on their own streams -- and the final encode: the chosen chunks are encoded
// once more (grouped by size and winner, bytes this time) into slots -- the
// walk's decision must come out again, or the call fails -- and moved into the
// body at their offsets (k_compact with per-package lengths).
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
#include "ambc_walkcore.h"

namespace ambc {
namespace {

// (WalkPool, the per-round host threads: ambc_sync.h)

inline bool eligible(const ambc_params* p, uint32_t s, uint32_t id) { return ms_eligible(p, s, id); }

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
    HIPCHK(b.slots.ensure((size_t)cnt * stride));
    HIPCHK(b.plen.ensure((size_t)cnt * 4 + 4));
    HIPCHK(b.ids.ensure((size_t)cnt + 16));
    HIPCHK(b.sizes.ensure((size_t)cnt * 8 + 8));
    // the chunk table is read in place from the pinned positions (each workgroup
    // reads its own once) and every chunk is s bytes: no copy, no fill per batch
    // (each was a blit of ~50 us on the batch's stream, before its kernels)
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
    ea.coff = pos;
    ea.clen = nullptr;
    ea.clen_all = s;
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
    // the results straight into the pinned host arrays: one small kernel instead of
    // two or three copies
    HIPCHK(launch_results_to_host(b.plen.as<uint32_t>(), b.ids.as<uint8_t>(), nsub ? b.lz4sub.as<uint32_t>() : nullptr,
                                  cnt, nsub ? LZ4_SUB_MAX : 0u, b.hplen, b.hids, b.hlz, st));
    return AMBC_OK;
}

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
    // (a large upload runs in ordered pieces beside the walk: its first rounds take
    // the walks whose chunks have arrived, the others as the pieces come in; the
    // final encode waits for all of it)
    // AMBC_MS_UPLOAD (A/B): "staged" -- pinned staging buffers on 8 threads beside
    // the walk; "first" -- the walk after the whole upload.  Default, measured on
    // 256 MiB (profiles/r5_upload_ab): staged where every size runs its own encoders,
    // first with LZ4 among the methods, whose walk asks six positions ahead and loses
    // more to the forgotten requests than the overlap gains ({1,3,4,9} 6.17-6.22 vs
    // 5.26-5.88).  (Round 5's third mode pinned the caller's pages for DMA; the
    // library no longer maps caller memory into the GPU)
    static const char* upenv = getenv("AMBC_MS_UPLOAD");
    const char* upmode = upenv ? upenv : ((p->method_mask >> AMBC_M_LZ4) & 1) ? "first" : "staged";
    std::unique_ptr<OrderedUpload> up;
    if (n >= kStageMin) {
        up.reset(new OrderedUpload());
        if (int rc = start_ordered_upload(d, d.in.as<uint8_t>(), in, n, stage_threads(n, 8), *up)) return rc;
    } else if (n) {
        HIPCHK(hipMemcpyAsync(d.in.p, in, n, hipMemcpyHostToDevice, s));
    }
    auto await_upload = [&]() -> int {
        if (up && !up->wait_prefix(n)) return fail(AMBC_E_DEVICE, "input upload failed");
        if (up) up->join();
        return AMBC_OK;
    };
    HIPCHK(hipMemsetAsync(d.in.as<uint8_t>() + n, 0, 64, s));
    const uint8_t* d_in = d.in.as<uint8_t>();

    // slot 0 of each group (the round's largest size: its encode is the round's
    // latency) on a high-priority stream, the smaller sizes fill in around it
    for (int i = 0; i < 16; i++) {
        if (d.mss[i]) continue;
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&d.mss[i], hipStreamNonBlocking, (i % 8) == 0 ? hi : lo));
    }
    HIPCHK(hipStreamSynchronize(s));                   // (the input upload)

    // ---- the walk (ambc_walkcore.h) over decision-only device batches ----
    struct Backend {
        Dev& d;
        const uint8_t* d_in;
        uint64_t n;
        std::function<const double*(uint32_t)> ent_of;
        OrderedUpload* up;
        int launch(int slot, const ambc_params* pk, uint32_t sz, const uint64_t* pos, uint32_t cnt,
                   const uint32_t* subc, uint32_t nsub) {
            Batch& bb = d.msb[slot];
            HIPCHK(bb.host_ensure(cnt));
            std::memcpy(bb.hpos, pos, (size_t)cnt * 8);
            return launch_batch(bb, d.mss[slot], d_in, n, pk, sz, bb.hpos, cnt, ent_of(sz), true, subc, nsub);
        }
        bool ready(int slot) { return hipStreamQuery(d.mss[slot]) != hipErrorNotReady; }
        int finish(int slot, const uint32_t** plen, const uint8_t** ids, const uint32_t** lz) {
            HIPCHK(hipStreamSynchronize(d.mss[slot]));
            *plen = d.msb[slot].hplen;
            *ids = d.msb[slot].hids;
            *lz = d.msb[slot].hlz;
            return AMBC_OK;
        }
        bool whole;   // AMBC_MS_UPLOAD_FIRST: the walk starts after the whole upload (A/B, tests)
        uint64_t avail() {
            if (up && whole) (void)up->wait_prefix(n);
            return up ? up->avail() : n;
        }
        int wait_avail(uint64_t want) {
            if (up && !up->wait_prefix(std::min(want, n))) return fail(AMBC_E_DEVICE, "input upload failed");
            return AMBC_OK;
        }
        int check_size(const ambc_params* pk, uint32_t sz) { return ::ambc::check_size(pk, sz); }
    } be{d, d_in, n, ent_of, up.get(), getenv("AMBC_MS_UPLOAD_FIRST") != nullptr || !strcmp(upmode, "first")};
    static const WalkConfig cfg = WalkConfig::from_env();
    WalkOutcome wo;
    if (int rc = walk_decide(be, d.ms_mem, WalkPool::get(), cfg, n, p, cands, hc, wo)) return rc;
    uint64_t kernel_ns = wo.wait_ns;
    const uint32_t steps = wo.steps;
    const uint64_t evaluated = wo.evaluated;
    const uint64_t t_walk = now_ns() - t0;
    TRACE("multisize walk ms: decide %.2f requests %.2f launch %.2f wait %.2f fill %.2f host %.2f (total %.2f)",
          wo.t_dec / 1e6, wo.t_req / 1e6, wo.t_launch / 1e6, wo.t_wait / 1e6, wo.t_fill / 1e6, wo.t_host / 1e6,
          t_walk / 1e6);
    if (int rc = await_upload()) return rc;
    std::vector<WalkPkg>& path = wo.path;
    using Pkg = WalkPkg;
    uint64_t body = wo.body;
    // the body buffer at its largest: every package is smaller than its chunk but
    // the raw remainder, each adds a header
    const uint64_t body_cap = n + (uint64_t)HDR * (n / *std::min_element(cands.begin(), cands.end()) + 2) + END_CHUNK;
    HIPCHK(d.ms_out.ensure(body_cap + 64));
    uint8_t* d_body = d.ms_out.as<uint8_t>();
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
        ca.clen = nullptr;
        ca.clen_all = sz;
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
