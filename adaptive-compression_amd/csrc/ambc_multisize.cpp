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

// the sizes the GPU encoders take (k_encode <= 65536, k_deflate <= 16384, k_dict <= 8192)
int check_size(const ambc_params* p, uint32_t s) {
    if (s > AMBC_MAX_CHUNK)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with eligible methods: the GPU encoders take chunks up to 65536 bytes");
    if (eligible(p, s, AMBC_M_DEFLATE) && s > 16384)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with DEFLATE eligible: the GPU DEFLATE encoder takes chunks up to 16384 bytes");
    if (eligible(p, s, AMBC_M_DICT) && s > 8192)
        return fail(AMBC_E_INVAL, "a candidate chunk of " + std::to_string(s) +
                                      " bytes with Dictionary eligible: the GPU Dictionary encoder takes chunks up to 8192 bytes");
    return AMBC_OK;
}

// The encoders over the s-byte chunks at pos[] (one workgroup each): per chunk
// the winner of the reference's method loop for that size, its payload left in
// the batch's slot k.  The launch sequence is compress_on's (k_encode, k_dict
// against its winner, k_deflate against both, then the deferred emits).
int run_batch(Dev& d, Batch& b, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint32_t s,
              const std::vector<uint64_t>& pos, const double* ent, std::vector<uint32_t>& plen,
              std::vector<uint8_t>& ids) {
    hipStream_t st = d.stream;
    const uint32_t cnt = (uint32_t)pos.size();
    const uint32_t C = (s + 15) & ~15u;
    const uint32_t stride = slot_stride_for(C);
    HIPCHK(b.coff.ensure((size_t)cnt * 8));
    HIPCHK(b.clen.ensure((size_t)cnt * 4));
    HIPCHK(b.slots.ensure((size_t)cnt * stride));
    HIPCHK(b.plen.ensure((size_t)cnt * 4 + 4));
    HIPCHK(b.ids.ensure((size_t)cnt + 16));
    HIPCHK(b.sizes.ensure((size_t)cnt * 8 + 8));
    std::vector<uint32_t> cl(cnt, s);
    HIPCHK(hipMemcpyAsync(b.coff.p, pos.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(b.clen.p, cl.data(), (size_t)cnt * 4, hipMemcpyHostToDevice, st));
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
        HIPCHK(b.gdseq.ensure((size_t)cnt * 2 * gd_cmax));
        HIPCHK(b.pending.ensure((size_t)cnt));
        ea.bestpre = b.bestpre.as<uint32_t>();
        ea.gdseq = b.gdseq.as<uint8_t>();
        ea.pending = b.pending.as<uint8_t>();
    }
    HIPCHK(launch_encode(ea, st));
    if (dict) HIPCHK(launch_dict(ea, std::min<uint32_t>(C, p->pref_max[AMBC_M_DICT]), st));
    if (deflate) {
        HIPCHK(launch_deflate(ea, st));
        EncArgs ep = ea;
        ep.flags |= ENC_EMIT_PENDING;
        ep.bestpre = nullptr;
        HIPCHK(launch_encode(ep, st));
    }
    plen.resize(cnt);
    ids.resize(cnt);
    HIPCHK(hipMemcpyAsync(plen.data(), b.plen.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(ids.data(), b.ids.p, cnt, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
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
    std::vector<uint64_t> active;
    {
        const uint64_t K = std::max<uint64_t>(1, std::min<uint64_t>(2048, n / (128 << 10)));
        std::set<uint64_t> starts;
        for (uint64_t k = 0; k < K; k++) starts.insert((k * n / K) / g * g);
        active.assign(starts.begin(), starts.end());
        if (n == 0) active.clear();
    }
    Batch& B = d.msb;
    uint32_t steps = 0;
    uint64_t evaluated = 0;
    uint64_t kernel_ns = 0;
    while (!active.empty()) {
        steps++;
        // (a position another walk decided meanwhile needs nothing more)
        active.erase(std::remove_if(active.begin(), active.end(), [&](uint64_t q) { return dec.count(q) > 0; }),
                     active.end());
        if (active.empty()) break;
        // every (position, size) an active walk needs that is not known yet, per size
        std::map<uint32_t, std::vector<uint64_t>> req;
        for (uint64_t pos : active) {
            const uint64_t remain = n - pos;
            for (uint32_t i = 0; i < n_cands; i++) {
                const uint32_t sz = (uint32_t)std::min<uint64_t>(cands[i], remain);
                if (!any_eligible(p, sz)) continue;
                const uint64_t kk = key(pos, sz);
                if (cache.count(kk)) continue;
                int rc = check_size(p, sz);
                if (rc) return rc;
                cache[kk] = Eval{0, 0xFE};     // requested (filled below)
                req[sz].push_back(pos);
            }
        }
        const uint64_t tk = now_ns();
        for (auto& r : req) {
            std::vector<uint32_t> pl;
            std::vector<uint8_t> id;
            int rc = run_batch(d, B, d_in, n, p, r.first, r.second, ent_of(r.first), pl, id);
            if (rc) return rc;
            for (size_t j = 0; j < r.second.size(); j++) cache[key(r.second[j], r.first)] = Eval{pl[j], id[j]};
            evaluated += r.second.size();
        }
        kernel_ns += now_ns() - tk;
        // the decisions (adaptive_compressor.py:546-590) and the next positions
        std::set<uint64_t> next;
        for (uint64_t pos : active) {
            const uint64_t remain = n - pos;
            double best_ratio = 1.0;
            uint32_t best_s = 0, best_plen = 0;
            uint8_t best_id = 255;
            uint32_t seen[64];
            uint32_t nseen = 0;
            for (uint32_t i = 0; i < n_cands; i++) {
                const uint32_t sz = (uint32_t)std::min<uint64_t>(cands[i], remain);
                if (std::find(seen, seen + nseen, sz) != seen + nseen) {
                    // the same clamped size again: same package, same ratio (never strictly better)
                    continue;
                }
                if (nseen < 64) seen[nseen++] = sz;
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
            if (best_id == 255) {            // (remain, 255): the rest, raw
                if (remain > 0xFFFFFFFFull) return fail(AMBC_E_RANGE, "raw remainder exceeds a u32 chunk field");
                dec[pos] = Decision{(uint32_t)remain, (uint32_t)remain, 255};
                continue;
            }
            dec[pos] = Decision{best_s, best_plen, best_id};
            const uint64_t nx = pos + best_s;
            if (nx < n && !dec.count(nx)) next.insert(nx);
        }
        active.assign(next.begin(), next.end());
    }

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
    for (auto& gr : groups) {
        const uint32_t sz = gr.first;
        std::vector<uint64_t> pos;
        for (size_t i : gr.second) pos.push_back(path[i].pos);
        std::vector<uint32_t> pl;
        std::vector<uint8_t> id;
        int rc = run_batch(d, B, d_in, n, p, sz, pos, ent_of(sz), pl, id);
        if (rc) return rc;
        std::vector<uint64_t> offs;
        for (size_t j = 0; j < gr.second.size(); j++) {
            const Pkg& pk = path[gr.second[j]];
            if (pl[j] != pk.plen || id[j] != pk.id) return fail(AMBC_E_DEVICE, "multi-size walk: re-encode differs");
            offs.push_back(pk.off);
        }
        HIPCHK(B.off.ensure(offs.size() * 8));
        HIPCHK(hipMemcpyAsync(B.off.p, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, s));
        CompactArgs ca{};
        ca.slots = B.slots.as<uint8_t>();
        ca.slot_stride = slot_stride_for((sz + 15) & ~15u);
        ca.plen = B.plen.as<uint32_t>();
        ca.ids = B.ids.as<uint8_t>();
        ca.off = B.off.as<uint64_t>();
        ca.n_chunks = (uint32_t)offs.size();
        ca.clen = B.clen.as<uint32_t>();
        ca.n_total = n;
        ca.chunk_size = (sz + 15) & ~15u;
        ca.out = d_body;
        HIPCHK(launch_compact(ca, s));
        HIPCHK(hipStreamSynchronize(s));   // the next group reuses the batch buffers
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

extern "C" int ambc_last_multisize_info(ambc_ctx* ctx, uint32_t* steps, uint64_t* evaluated) {
    if (!ctx || ctx->devs.empty()) return fail(AMBC_E_INVAL, "bad context");
    if (steps) *steps = ctx->devs[0].ms_steps;
    if (evaluated) *evaluated = ctx->devs[0].ms_evaluated;
    return AMBC_OK;
}
