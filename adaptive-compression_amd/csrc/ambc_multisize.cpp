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
// one workgroup per chunk).  A walk stops when its next position has already
// been decided (it joined the path of another walk: from there on both are the
// same walk) or at the end.  Every decided position's successor is decided, so
// the walk from 0 -- the reference's walk -- is then read off the decisions.
// The chosen chunks are encoded once more (grouped by size) into slots and
// moved into the body at their offsets (k_compact with per-package lengths).
#include <algorithm>
#include <cstring>
#include <map>
#include <numeric>
#include <set>
#include <unordered_map>

#include "ambc_hostctx.h"

namespace ambc {
namespace {

struct Eval {
    uint32_t plen;   // payload of the size's winner
    uint8_t id;      // 255: no method beats raw at this size
};

bool eligible(const ambc_params* p, uint32_t s, uint32_t id) {
    return ((p->method_mask >> id) & 1) && p->pref_min[id] <= s && s <= p->pref_max[id];
}

bool any_eligible(const ambc_params* p, uint32_t s) {
    for (uint32_t id = 1; id < 16; id++)
        if (eligible(p, s, id)) return true;
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

// The encoders over the s-byte chunks at pos[] (one workgroup each) on stream
// st: per chunk the winner of the reference's method loop for that size, its
// payload left in the batch's slot k, plen / ids copied back into hp / hi (valid
// after the stream synchronizes).  The launch sequence is compress_on's
// (k_encode, k_dict against its winner, k_deflate against both, then the
// deferred emits).
int launch_batch(Batch& b, hipStream_t st, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint32_t s,
                 const std::vector<uint64_t>& pos, const double* ent) {
    const uint32_t cnt = (uint32_t)pos.size();
    HIPCHK(b.host_ensure(cnt));
    const uint32_t C = (s + 15) & ~15u;
    const uint32_t stride = slot_stride_for(C);
    HIPCHK(b.coff.ensure((size_t)cnt * 8));
    HIPCHK(b.clen.ensure((size_t)cnt * 4));
    HIPCHK(b.slots.ensure((size_t)cnt * stride));
    HIPCHK(b.plen.ensure((size_t)cnt * 4 + 4));
    HIPCHK(b.ids.ensure((size_t)cnt + 16));
    HIPCHK(b.sizes.ensure((size_t)cnt * 8 + 8));
    HIPCHK(hipMemcpyAsync(b.coff.p, pos.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
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
    for (int i = 0; i < 16; i++) { ea.pref_min[i] = p->pref_min[i]; ea.pref_max[i] = p->pref_max[i]; }
    // chunks on the 16-byte grid of the library's padded input copy: read in place
    bool aligned = ((uintptr_t)d_in & 15) == 0 && !getenv("AMBC_ENC_LDS");
    for (uint64_t q : pos) aligned = aligned && (q & 15) == 0;
    if (aligned) ea.flags |= ENC_IN_ALIGNED;
    if (ent) {   // numpy's p*log2(p) terms for an s-byte chunk (Huffman should_use near 7.0)
        HIPCHK(b.ent.ensure((size_t)(s + 1) * 8));
        HIPCHK(hipMemcpyAsync(b.ent.p, ent, (size_t)(s + 1) * 8, hipMemcpyHostToDevice, st));
        if (s == C) ea.ent_full = b.ent.as<double>();
        else ea.ent_tail = b.ent.as<double>();
    }
    const bool dict = eligible(p, s, AMBC_M_DICT);
    const bool deflate = eligible(p, s, AMBC_M_DEFLATE);
    uint32_t gd_cmax = 1024;
    while (gd_cmax < C) gd_cmax <<= 1;
    if (deflate) {
        HIPCHK(b.bestpre.ensure((size_t)cnt * 4));
        HIPCHK(b.gdseq.ensure((size_t)cnt * gd_seq_bytes(gd_cmax)));
        HIPCHK(b.pending.ensure((size_t)cnt));
        ea.bestpre = b.bestpre.as<uint32_t>();
        ea.gdseq = b.gdseq.as<uint8_t>();
        ea.pending = b.pending.as<uint8_t>();
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
    if (deflate) {
        HIPCHK((p->flags & AMBC_FLAG_ZLIB9) ? launch_zlib9(ea, st) : launch_deflate(ea, st));
        EncArgs ep = ea;
        ep.flags |= ENC_EMIT_PENDING;
        ep.bestpre = nullptr;
        HIPCHK(launch_encode(ep, st));
    }
    HIPCHK(hipMemcpyAsync(b.hplen, b.plen.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(b.hids, b.ids.p, cnt, hipMemcpyDeviceToHost, st));
    return AMBC_OK;
}

struct Decision {
    uint32_t s;      // chunk size taken at this position (the remainder when raw)
    uint32_t plen;
    uint8_t id;      // 255: the rest of the input as one raw package
};

inline uint64_t key(uint64_t pos, uint32_t s) { return pos << 18 | s; }

}  // namespace
}  // namespace ambc

using namespace ambc;

extern "C" int ambc_compress_multisize(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                                       const uint32_t* cands, uint32_t n_cands, const uint32_t* ent_sizes,
                                       const double* const* ent_tabs, uint32_t n_ent, uint8_t* out,
                                       uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    if (!ctx || ctx->devs.empty() || !p || !out_len || (n && !in) || !cands || !n_cands)
        return fail(AMBC_E_INVAL, "bad arguments");
    for (uint32_t i = 0; i < n_cands; i++)
        if (cands[i] == 0 || cands[i] > (1u << 17)) return fail(AMBC_E_INVAL, "candidate sizes must be in [1, 131072]");
    const uint32_t allowed = (1u << AMBC_M_RLE) | (1u << AMBC_M_DICT) | (1u << AMBC_M_HUFFMAN) |
                             (1u << AMBC_M_DELTA) | (1u << AMBC_M_DEFLATE) | (1u << AMBC_M_LZ4);
    if (p->method_mask & ~allowed)
        return fail(AMBC_E_INVAL, "method_mask holds ids without a GPU encoder (allowed: 1, 2, 3, 4, 5, 9)");
    const uint64_t t0 = now_ns();
    Dev& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    std::map<uint32_t, const double*> ent;
    for (uint32_t i = 0; i < n_ent; i++)
        if (ent_tabs && ent_tabs[i]) ent[ent_sizes[i]] = ent_tabs[i];
    auto ent_of = [&](uint32_t sz) -> const double* {
        auto it = ent.find(sz);
        return it == ent.end() ? nullptr : it->second;
    };
    // the input, uploaded once (64 bytes of slack for the encoders' padded loads)
    HIPCHK(d.in.ensure(n + 64));
    if (n) HIPCHK(hipMemcpyAsync(d.in.p, in, n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d.in.as<uint8_t>() + n, 0, 64, s));
    const uint8_t* d_in = d.in.as<uint8_t>();

    // ---- the walks ----
    uint64_t g = 0;
    for (uint32_t i = 0; i < n_cands; i++) g = std::gcd(g, (uint64_t)cands[i]);
    std::unordered_map<uint64_t, Eval> cache;          // (pos, s) -> the size's winner
    std::unordered_map<uint64_t, Decision> dec;        // pos -> the reference's decision there
    struct Walk { uint64_t pos; uint32_t last; };      // last: the size it took the step before
    std::vector<Walk> active;
    // walks: one per 512 KiB, at most 512; speculation: 2 positions ahead (256
    // MiB of mixed data, reference candidates: best of 1-8 ahead x 256-2048
    // walks; AMBC_MS_WALKS / AMBC_MS_SPEC override them for such sweeps)
    static const uint64_t KMAX_ = getenv("AMBC_MS_WALKS") ? strtoull(getenv("AMBC_MS_WALKS"), nullptr, 10) : 512;
    static const uint64_t SPAN_ = getenv("AMBC_MS_SPAN") ? strtoull(getenv("AMBC_MS_SPAN"), nullptr, 10) : 512 << 10;
    uint32_t max_cand = 0;
    for (uint32_t i = 0; i < n_cands; i++)
        if (any_eligible(p, cands[i])) max_cand = std::max(max_cand, cands[i]);
    {
        // walk starts on the lattice of the largest eligible size: where that size
        // wins everywhere (homogeneous data) every walk runs on the same lattice
        // and joins the next one at once; elsewhere the mixed choices shift their
        // phases until they meet
        const uint64_t K = std::max<uint64_t>(1, std::min<uint64_t>(KMAX_, n / std::max<uint64_t>(SPAN_, 1)));
        const uint64_t lat = max_cand ? max_cand : g;
        std::set<uint64_t> starts;
        for (uint64_t k = 0; k < K; k++) starts.insert((k * n / K) / lat * lat);
        if (n)
            for (uint64_t b0 : starts) active.push_back(Walk{b0, max_cand ? max_cand : cands[0]});
    }
    for (auto& x : d.mss)
        if (!x) HIPCHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    HIPCHK(hipStreamSynchronize(s));                   // (the input upload)
    uint32_t steps = 0;
    uint64_t evaluated = 0;
    uint64_t kernel_ns = 0;
    // the (position, size) pairs a decision at pos needs; false when all are known
    auto needs = [&](uint64_t pos, std::map<uint32_t, std::vector<uint64_t>>* req) -> bool {
        bool any = false;
        const uint64_t remain = n - pos;
        for (uint32_t i = 0; i < n_cands; i++) {
            const uint32_t sz = (uint32_t)std::min<uint64_t>(cands[i], remain);
            if (!any_eligible(p, sz)) continue;
            const uint64_t kk = key(pos, sz);
            if (cache.count(kk)) continue;
            any = true;
            if (req) {
                cache[kk] = Eval{0, 0xFE};     // requested (filled by the batch)
                (*req)[sz].push_back(pos);
            }
        }
        return any;
    };
    // the reference's decision at pos (adaptive_compressor.py:546-590), all sizes known
    auto decide = [&](uint64_t pos) -> Decision {
        const uint64_t remain = n - pos;
        double best_ratio = 1.0;
        uint32_t best_s = 0, best_plen = 0;
        uint8_t best_id = 255;
        std::vector<uint32_t> seen;
        for (uint32_t i = 0; i < n_cands; i++) {
            const uint32_t sz = (uint32_t)std::min<uint64_t>(cands[i], remain);
            // the same clamped size again: same package, same ratio (never strictly better)
            if (std::find(seen.begin(), seen.end(), sz) != seen.end()) continue;
            seen.push_back(sz);
            if (!any_eligible(p, sz)) continue;
            const Eval& e = cache[key(pos, sz)];
            if (e.id == 255) continue;
            const double ratio = (double)(e.plen + HDR) / (double)sz;
            if (ratio < best_ratio) {
                best_ratio = ratio;
                best_s = sz;
                best_plen = e.plen;
                best_id = e.id;
            }
        }
        if (best_id == 255) return Decision{(uint32_t)std::min<uint64_t>(remain, 0xFFFFFFFFull), (uint32_t)remain, 255};
        return Decision{best_s, best_plen, best_id};
    };
    // Rounds: every walk decides as far as the known sizes reach; then ONE batch
    // per size evaluates each walk's next position and SPEC positions further
    // along the path it would take if it kept its last step size (a guess: a
    // right one saves a round, whose latency -- the slowest 64 KiB encode -- is
    // the walk's cost; a wrong one costs idle device time only)
    static const int SPEC = getenv("AMBC_MS_SPEC") ? atoi(getenv("AMBC_MS_SPEC")) : 2;
    uint64_t t_dec = 0, t_req = 0, t_launch = 0, t_wait = 0, t_fill = 0;   // (AMBC_TRACE breakdown)
    while (!active.empty()) {
        uint64_t tq = now_ns();
        std::vector<Walk> still;
        for (Walk w : active) {
            for (;;) {
                if (dec.count(w.pos)) break;               // joined a decided path
                if (needs(w.pos, nullptr)) { still.push_back(w); break; }
                const Decision dd = decide(w.pos);
                if (dd.id == 255 && n - w.pos > 0xFFFFFFFFull)
                    return fail(AMBC_E_RANGE, "raw remainder exceeds a u32 chunk field");
                dec[w.pos] = dd;
                if (dd.id == 255) break;                   // the rest is raw: done
                w.last = dd.s;
                w.pos += dd.s;
                if (w.pos >= n) break;
            }
        }
        // (two walks at one position: keep one)
        std::sort(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos < y.pos; });
        still.erase(std::unique(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos == y.pos; }),
                    still.end());
        active.swap(still);
        t_dec += now_ns() - tq;
        tq = now_ns();
        if (active.empty()) break;
        steps++;
        std::map<uint32_t, std::vector<uint64_t>> req;
        for (const Walk& w : active) {
            uint64_t q = w.pos;
            for (int k = 0; k <= SPEC && q < n; k++, q += w.last) {
                if (k && dec.count(q)) break;
                (void)needs(q, &req);
            }
        }
        for (auto& r : req) {
            int rc = check_size(p, r.first);
            if (rc) {
                // only an error if a walk itself needs this size (not a speculative position)
                for (uint64_t q : r.second)
                    if (std::binary_search(active.begin(), active.end(), Walk{q, 0},
                                           [](const Walk& x, const Walk& y) { return x.pos < y.pos; }))
                        return rc;
            }
        }
        const uint64_t tk = now_ns();
        t_req += tk - tq;
        std::vector<std::pair<uint32_t, std::vector<uint64_t>>> jobs;
        for (auto& r : req) {
            if (check_size(p, r.first)) {       // speculative only: never decided from
                for (uint64_t q : r.second) cache.erase(key(q, r.first));
                continue;
            }
            jobs.emplace_back(r.first, std::move(r.second));
        }
        // up to 8 size classes at once, each on its own stream and batch buffers
        // (the 64 KiB class runs at 2 workgroups per CU: the small ones fill in)
        for (size_t j0 = 0; j0 < jobs.size(); j0 += 8) {
            const size_t j1 = std::min(jobs.size(), j0 + 8);
            uint64_t tl = now_ns();
            for (size_t j = j0; j < j1; j++) {
                int rc = launch_batch(d.msb[j - j0], d.mss[j - j0], d_in, n, p, jobs[j].first, jobs[j].second,
                                      ent_of(jobs[j].first));
                if (rc) return rc;
            }
            t_launch += now_ns() - tl;
            for (size_t j = j0; j < j1; j++) {
                tl = now_ns();
                HIPCHK(hipStreamSynchronize(d.mss[j - j0]));
                t_wait += now_ns() - tl;
                tl = now_ns();
                const Batch& bb = d.msb[j - j0];
                for (size_t q = 0; q < jobs[j].second.size(); q++)
                    cache[key(jobs[j].second[q], jobs[j].first)] = Eval{bb.hplen[q], bb.hids[q]};
                evaluated += jobs[j].second.size();
                t_fill += now_ns() - tl;
            }
        }
        kernel_ns += now_ns() - tk;
    }

    const uint64_t t_walk = now_ns() - t0;
    TRACE("multisize walk ms: decide %.2f requests %.2f launch %.2f wait %.2f fill %.2f (total %.2f)", t_dec / 1e6,
          t_req / 1e6, t_launch / 1e6, t_wait / 1e6, t_fill / 1e6, t_walk / 1e6);
    // ---- the reference's walk from 0, read off the decisions ----
    struct Pkg { uint64_t pos; uint32_t s, plen; uint8_t id; uint64_t off; };
    std::vector<Pkg> path;
    uint64_t body = 0;
    for (uint64_t pos = 0; pos < n;) {
        auto it = dec.find(pos);
        if (it == dec.end()) return fail(AMBC_E_DEVICE, "multi-size walk: undecided position on the path");
        const Decision& dd = it->second;
        path.push_back(Pkg{pos, dd.s, dd.plen, dd.id, body});
        body += HDR + (uint64_t)dd.plen;
        if (dd.id == 255) break;
        pos += dd.s;
    }
    body += END_CHUNK;
    if (out_cap < body) return fail(AMBC_E_CAPACITY, "output capacity below the body size");

    // ---- the chosen chunks, encoded again per size, into the body ----
    HIPCHK(d.out.ensure(body + 64));
    uint8_t* d_body = d.out.as<uint8_t>();
    const uint64_t te = now_ns();
    std::map<uint32_t, std::vector<size_t>> groups;
    for (size_t i = 0; i < path.size(); i++)
        if (path[i].id != 255) groups[path[i].s].push_back(i);
    std::vector<std::pair<uint32_t, std::vector<size_t>>> gl(groups.begin(), groups.end());
    for (size_t j0 = 0; j0 < gl.size(); j0 += 8) {
        const size_t j1 = std::min(gl.size(), j0 + 8);
        std::vector<std::vector<uint64_t>> offs(j1 - j0);
        for (size_t j = j0; j < j1; j++) {
            const uint32_t sz = gl[j].first;
            Batch& bb = d.msb[j - j0];
            hipStream_t xs = d.mss[j - j0];
            std::vector<uint64_t> pos;
            for (size_t i : gl[j].second) {
                pos.push_back(path[i].pos);
                offs[j - j0].push_back(path[i].off);
            }
            int rc = launch_batch(bb, xs, d_in, n, p, sz, pos, ent_of(sz));
            if (rc) return rc;
            HIPCHK(bb.off.ensure(pos.size() * 8));
            HIPCHK(hipMemcpyAsync(bb.off.p, offs[j - j0].data(), pos.size() * 8, hipMemcpyHostToDevice, xs));
            CompactArgs ca{};
            ca.slots = bb.slots.as<uint8_t>();
            ca.slot_stride = slot_stride_for((sz + 15) & ~15u);
            ca.plen = bb.plen.as<uint32_t>();
            ca.ids = bb.ids.as<uint8_t>();
            ca.off = bb.off.as<uint64_t>();
            ca.n_chunks = (uint32_t)pos.size();
            ca.clen = bb.clen.as<uint32_t>();
            ca.n_total = n;
            ca.chunk_size = (sz + 15) & ~15u;
            ca.out = d_body;
            HIPCHK(launch_compact(ca, xs));
        }
        for (size_t j = j0; j < j1; j++) {
            HIPCHK(hipStreamSynchronize(d.mss[j - j0]));
            const Batch& bb = d.msb[j - j0];
            for (size_t q = 0; q < gl[j].second.size(); q++) {
                const Pkg& pk = path[gl[j].second[q]];
                if (bb.hplen[q] != pk.plen || bb.hids[q] != pk.id)
                    return fail(AMBC_E_DEVICE, "multi-size walk: re-encode differs");
            }
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
    HIPCHK(hipMemcpyAsync(out, d_body, body, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    kernel_ns += now_ns() - te;
    *out_len = body;
    d.ms_steps = steps;
    d.ms_evaluated = evaluated;
    d.ms_walk_ns = t_walk;
    d.ms_emit_ns = now_ns() - te;
    TRACE("multisize n=%llu steps=%u evaluated=%llu path=%zu", (unsigned long long)n, steps,
          (unsigned long long)evaluated, path.size());
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

extern "C" int ambc_last_multisize_info(ambc_ctx* ctx, uint32_t* steps, uint64_t* evaluated,
                                        uint64_t* walk_ns, uint64_t* emit_ns) {
    if (!ctx || ctx->devs.empty()) return fail(AMBC_E_INVAL, "bad context");
    if (steps) *steps = ctx->devs[0].ms_steps;
    if (evaluated) *evaluated = ctx->devs[0].ms_evaluated;
    if (walk_ns) *walk_ns = ctx->devs[0].ms_walk_ns;
    if (emit_ns) *emit_ns = ctx->devs[0].ms_emit_ns;
    return AMBC_OK;
}
