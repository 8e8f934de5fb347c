// ambc_zlib9.hip -- the reference's own id-5 bytes on gfx950: zlib.compress(data, 9).
//
// DeflateCompression.compress is zlib.compress(data, level=9)
// (advanced_compression.py:76-81): zlib 1.2.11's deflate_slow (lazy matching,
// good 32 / lazy 258 / nice 258 / chain 4096, 15-bit rolling hash of 3 bytes,
// TOO_FAR 4096, a block per 16383 symbols) and _tr_flush_block (stored /
// static / dynamic by zlib's size rules, heap-built Huffman trees with zlib's
// tie order, length limiting, code-length RLE).  oracle/zlib9_model.c restates
// the same algorithm on the CPU; tests compare both with the system zlib.
// Chunks up to 4096 bytes (the walkers' tables live in LDS).
//
// Two launches per chunk range (after k_encode / k_dict, like k_deflate):
//
// k_z9_parse<CMAX>: one workgroup of NW waves per chunk.
//   1. the chunk in LDS (zeros past n: zlib's WIN_INIT padding is what its
//      match scan reads beyond the input);
//   2. positions 1..n-3 (zlib inserts every position with 3 bytes of
//      lookahead; position 0 is its NIL) counting-sorted by a 10-bit hash OF
//      THE 15-bit zlib hash, stably: a bucket's entries below p, read downward,
//      are p's hash chain (most recent first) plus other-hash entries that the
//      search skips by recomputing their 15-bit hash;
//   3. the lazy parse by walkers (8-lane groups).  zlib's longest_match at p
//      is the first chain entry reaching the longest length (capped at
//      min(258, n - p)), over the first 4096 entries -- or 1024 when the
//      previous match was >= 32 long (the walker knows which).  After
//      a match the parser state is fresh, so the step from one fresh position
//      to the next (literals, then the match that ends the segment) is a pure
//      function of the position: walkers start from spread positions, record
//      seg[q] for every fresh q they reach and stop on one another walker
//      recorded; walker 0 starts at 0, so the path from 0 is complete;
//   4. thread 0 follows the path and writes the segments (literal count,
//      match length, distance) and zlib's block starts (a block ends with its
//      16383rd symbol, except the final literal) to the chunk's record area.
//
// k_z9_code<CMAX>: one wave per chunk (11 KB LDS).  Per block: symbol
// frequencies by a position-major pass (match starts in a bitmask, coverage by
// a running max of match ends); zlib's build_tree for the literal/length and
// distance trees at once on lanes 0 and 1 (the heap holds packed
// freq | depth | node keys, so a step compares without indirection), the
// code-length RLE scan, the bit-length tree, _tr_flush_block's choice; then the
// block's bits (header on lane 0, symbols position-major with prefix sums and
// LDS atomics).  A one-block chunk knows its exact length before emitting and
// stops there when id 5 loses.  Selection is k_deflate's: id 5 wins iff
// len + 18 < T.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

#include "ambc_z9.h"

namespace ambc {
namespace {


#ifndef AMBC_Z9_NW4096
#define AMBC_Z9_NW4096 8
#endif
// lanes per walker (the candidates one search step compares): fewer lanes give
// more walkers per wave instruction where chains are short
#ifndef AMBC_Z9_G
#define AMBC_Z9_G 8
#endif
// Compact LDS (round 6): 1024 sort buckets (10 bits of the 15-bit hash) and the
// segments' match distances inside the segment words -- 51 -> 40 KB at 4 KiB,
// four workgroups per CU instead of three: {1,3,4,5z} 21.66 -> 23.92 GB/s
// same-box (profiles/r6_z9_compact_ab/)
constexpr uint32_t ZBITS = 10u;
constexpr uint32_t ZB4 = 1u << ZBITS;   // the small parse's sort buckets
__device__ __forceinline__ uint32_t zb(uint32_t h15) { return z_bucket_b<ZBITS>(h15); }
// segment words: bit 31 set; a run of c literals (c < 2^22), or a match of L
// (3..258) at distance d (< 2^13) after c lazy literals (c < 256: each lazy step
// finds a strictly longer match)
__device__ __forceinline__ uint32_t seg_lits(uint32_t c) { return 0x80000000u | c; }
__device__ __forceinline__ uint32_t seg_match(uint32_t L, uint32_t d, uint32_t c) { return 0x80000000u | L << 22 | d << 9 | c; }
__device__ __forceinline__ uint32_t seg_L(uint32_t t) { return (t >> 22) & 0x1FFu; }
__device__ __forceinline__ uint32_t seg_c(uint32_t t) { return seg_L(t) ? (t & 0x1FFu) : (t & 0x3FFFFFu); }
__device__ __forceinline__ uint32_t seg_d(uint32_t t) { return (t >> 9) & 0x1FFFu; }

template <int CMAX> struct Z9Cfg {
    static constexpr int NW = CMAX <= 1024 ? 2 : (CMAX <= 2048 ? 4 : (CMAX <= 4096 ? AMBC_Z9_NW4096 : 16));
    static constexpr int G = AMBC_Z9_G;
};

template <int CMAX>
struct Z9Smem {
    static constexpr int NW = Z9Cfg<CMAX>::NW;
    alignas(16) uint8_t ch[CMAX + 320];      // the chunk, zeros past n
    alignas(16) uint16_t lst[CMAX];          // positions by bucket, ascending inside one
    alignas(16) uint16_t slot[CMAX];         // position -> its index in lst
    alignas(16) uint32_t bend32[ZB4 / 2];    // bucket ends (u16 pairs)
    // the sort's per-range cursors [NR][ZB4] u16; then the parse: seg[q] = 0
    // (not reached) or 1 << 31 | L << 16 | c for a clean position q: c
    // literals, then a match of L (0: none); the next clean position is q + c + L
    alignas(16) uint32_t seg[CMAX];
    uint16_t entry[CMAX / 64], rbase[CMAX / 64];   // the path: entry lane / match rank per window
    uint16_t wrs[CMAX / 32];                 // the walk: the byte run holding position 32 w starts here
    uint32_t mask[CMAX / 32];                // the path's match starts
    uint32_t cov[CMAX / 32];                 // positions the path's matches cover
    uint32_t nmatch;
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

template <int CMAX>
__device__ __forceinline__ uint32_t z_gram(const Z9Smem<CMAX>& S, uint32_t i) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    return __builtin_amdgcn_alignbyte(c32[(i >> 2) + 1], c32[i >> 2], i & 3) & 0xFFFFFFu;
}

// Stable counting sort of positions [1, m) into lst[] by zb(z_h15) --
// ambc_dict.hip's build_buckets with the zlib hash and each position's slot.
template <int CMAX>
__device__ void z9_sort(Z9Smem<CMAX>& S, uint32_t m, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NW = Z9Smem<CMAX>::NW, T = 64u * NW;
    constexpr uint32_t NR = (uint32_t)CMAX / 1024, GR = 16;
    static_assert(NR >= 1 && NR <= NW && NR * ZB4 * 2 <= (uint32_t)CMAX * 4, "cursor arrays live in seg[]");
    uint16_t* cnt = reinterpret_cast<uint16_t*>(S.seg);
    const uint32_t tid = wave * 64u + lane;
    for (uint32_t b = tid; b < NR * ZB4 / 2; b += T) S.seg[b] = 0;
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t loc[GR];
    if (wave < NR) {
        uint16_t* c = cnt + wave * ZB4;
#pragma unroll
        for (uint32_t g = 0; g < GR; g++) {
            const uint32_t i = (wave * GR + g) * 64 + lane;
            const bool v = i >= 1 && i < m;
            const uint32_t h = v ? zb(z_h15(z_gram(S, i))) : 0u;
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int b = 0; b < (int)ZBITS; b++) {
                const uint64_t mb = __ballot(v && ((h >> b) & 1u));
                peers &= ((h >> b) & 1u) ? mb : ~mb;
            }
            const uint32_t base = v ? (uint32_t)c[h] : 0u;
            loc[g] = v ? (base + (uint32_t)__popcll(peers & below)) | h << 16 : ~0u;
            if (v && (peers >> lane) == 1ull) c[h] = (uint16_t)(base + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    for (uint32_t h = tid; h < ZB4; h += T) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t r = 0; r < NR; r++) {
            const uint32_t x = cnt[r * ZB4 + h];
            cnt[r * ZB4 + h] = (uint16_t)run;
            run += x;
        }
        S.bend()[h] = (uint16_t)run;
    }
    __syncthreads();
    if (wave == 0) {
        constexpr int WPL = (int)ZB4 / 128;   // u16 pairs per lane
        uint32_t c[WPL], t = 0;
#pragma unroll
        for (int j = 0; j < WPL; j++) {
            c[j] = S.bend32[lane * WPL + j];
            t += (c[j] & 0xFFFFu) + (c[j] >> 16);
        }
        uint32_t run = wave_incl_sum(t) - t;
#pragma unroll
        for (int j = 0; j < WPL; j++) {
            const uint32_t r0 = run + (c[j] & 0xFFFFu), r1 = r0 + (c[j] >> 16);
            S.bend32[lane * WPL + j] = r0 | r1 << 16;
            run = r1;
        }
    }
    __syncthreads();
    if (wave < NR) {
#pragma unroll
        for (uint32_t g = 0; g < GR; g++) {
            if (loc[g] != ~0u) {
                const uint32_t h = loc[g] >> 16;
                const uint32_t idx = S.bstart(h) + cnt[wave * ZB4 + h] + (loc[g] & 0xFFFFu);
                const uint32_t pos = (wave * GR + g) * 64 + lane;
                S.lst[idx] = (uint16_t)pos;
                S.slot[pos] = (uint16_t)idx;
            }
        }
    }
    __syncthreads();
}


// Positions where zlib finds no match at all: no earlier position with the same
// 15-bit hash (hash_head is NIL), position 0 (zlib's NIL) and the last two
// (fewer than MIN_MATCH bytes of lookahead).  From a clean position on such a
// run is all literals, each position clean again, so a walker takes it in one
// step (seg[q] = c literals, no match).  Bit s of S.mask (free until the path).
// A bucket whose entries below s are more than 4 is taken as "maybe a match".
template <int CMAX>
__device__ __forceinline__ void z9_literal_mask(Z9Smem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NW = Z9Smem<CMAX>::NW;
    for (uint32_t b = wave * 64u; b < (uint32_t)CMAX; b += 64u * NW) {
        const uint32_t s = b + lane;
        bool lit = true;
        if (s >= 1 && s + 3 <= n) {
            const uint32_t h = z_h15(z_gram(S, s));
            const uint32_t lo = S.bstart(zb(h)), j = S.slot[s];
            if (j > lo + 4) {
                lit = false;
            } else {
                for (uint32_t t = lo; t < j; t++)
                    if (z_h15(z_gram(S, S.lst[t])) == h) { lit = false; break; }
            }
        }
        const uint64_t m = __ballot(lit);
        // byte runs: bit p of S.cov (free until the path) = a run starts at p (and
        // every p >= n, which bounds the walks' forward scans)
        const bool rb = s == 0 || s >= n || S.ch[s] != S.ch[s - 1];
        const uint64_t rm = __ballot(rb);
        if (lane == 0) {
            S.mask[b >> 5] = (uint32_t)m; S.mask[(b >> 5) + 1] = (uint32_t)(m >> 32);
            S.cov[b >> 5] = (uint32_t)rm; S.cov[(b >> 5) + 1] = (uint32_t)(rm >> 32);
        }
    }
    __syncthreads();
    // per 32-position word: the start of the run holding its first position (the
    // last run start before it, by an exclusive max-scan over the words)
    if (wave == 0) {
        constexpr uint32_t NWD = (uint32_t)CMAX / 32, K = (NWD + 63) / 64;
        int last = -1;
        int lb[K];
#pragma unroll
        for (uint32_t t = 0; t < K; t++) {
            const uint32_t w = lane * K + t;
            const uint32_t x = w < NWD ? S.cov[w] : 0u;
            lb[t] = x ? (int)(w * 32 + 31 - __builtin_clz(x)) : -1;
            last = max(last, lb[t]);
        }
        int run = wave_excl_max(last, -1);
#pragma unroll
        for (uint32_t t = 0; t < K; t++) {
            const uint32_t w = lane * K + t;
            if (w < NWD) S.wrs[w] = (uint16_t)((S.cov[w] & 1u) ? w * 32 : (uint32_t)max(run, 0));
            run = max(run, lb[t]);
        }
    }
}

// The lazy parse's walkers (deflate_slow).  A position is CLEAN when the
// parser stands there with no pending match (prev_length < 3): right after a
// match, or with a pending literal and no match at the previous position.
// Everything zlib emits from a clean position on depends on the position only,
// so walkers start anywhere, record seg[q] for every clean q they leave (one
// literal, or the lazy chain's literals and the match that ends it) and stop
// on one another walker recorded.  Per 8-lane group: q = the current clean
// position, s = the position being looked at, P / Pd = the pending match at
// s - 1 (prev_length / distance), c = literals since q.  One longest_match per
// iteration for every active group.
template <int CMAX>
__device__ __forceinline__ void z9_walkers(Z9Smem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane) {
    constexpr uint32_t G = (uint32_t)Z9Cfg<CMAX>::G;
    constexpr uint32_t NWK = (uint32_t)Z9Cfg<CMAX>::NW * (64u / G);
    typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
    lds_vu32* vs = (lds_vu32*)S.seg;
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    const uint32_t g = lane / G, r = lane % G;
    const uint32_t wid = wave * (64u / G) + g;
    // (measured and not kept: starts at n * sqrt(w / NWK), for chains that grow
    // along the chunk -- ASCII 17.3 -> 23.7 ms per 256 MiB: the walkers' overrun
    // until they meet another walker's path, not the chain lengths, sets the time)
    uint32_t q = (uint32_t)(((uint64_t)n * wid) / NWK);
    uint32_t s = q, P = 2, Pd = 0, c = 0;
    bool clean = true, done = false;
#pragma unroll 1
    for (;;) {
        if (clean && !done && (q >= n || vs[q] != 0u)) done = true;
        if (__all(done)) break;
        // a run of literal positions from a clean q: one step
        bool skip = false;
#ifndef AMBC_Z9_NOSKIP
        if (clean && !done && ((S.mask[q >> 5] >> (q & 31)) & 1u)) {
            uint32_t e = q;
            for (;;) {
                const uint32_t sh = e & 31u;
                const uint32_t w = ~(S.mask[e >> 5] >> sh);   // bit t: e + t takes a match (t < 32 - sh)
                const uint32_t t = w ? (uint32_t)__builtin_ctz(w) : 32u;
                if (t < 32u - sh) { e += t; break; }
                e += 32u - sh;
                if (e >= n) break;
            }
            e = min(e, n);
            if (r == 0) vs[q] = seg_lits(e - q);
            q = e;
            s = q;
            skip = true;
        }
#endif
        const bool act = !done && !skip && s >= 1 && s + 3 <= n && P < 258;   // position 0 is zlib's NIL
        // ---- longest_match(s) over the first lim chain entries (zlib's
        // max_chain 4096, a quarter when the pending match is >= good_match);
        // key = min(len, nice) << 16 | candidate (the longest, then the most
        // recent) ----
        uint32_t k0 = 0;
        const uint32_t lim = P >= Z_GOOD ? Z_CHAIN / 4 : Z_CHAIN;
        {
            uint32_t tg[4] = {0, 0, 0, 0}, h = 0, lo = 0, j = 0, nice = 0;
            const uint32_t ss = s & 3u;
            if (act) {
                const uint32_t a = s >> 2;
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = c32[a + t];
#pragma unroll
                for (int t = 0; t < 4; t++) tg[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], ss);
                h = z_h15(tg[0] & 0xFFFFFFu);
                lo = S.bstart(zb(h));
                j = S.slot[s];
                nice = min(Z_MAXM, n - s);
            }
            uint32_t cnt = 0;
#ifndef AMBC_Z9_NORUN
            // Inside a byte run [rs, re) with s + 3 <= re, every earlier position of
            // the run is a chain entry (same 3 bytes, one bucket, contiguous in lst
            // just below s) and matches exactly re - s bytes (then s sees the run's
            // end and the candidate the run): the most recent, s - 1, stands for them
            // all; the chain goes on below the run (zlib counts those entries).
            if (act && s >= 2 && (tg[0] & 0xFFFFFFu) == (tg[0] & 0xFFu) * 0x010101u && S.ch[s - 1] == (tg[0] & 0xFFu)) {
                const uint32_t w = s >> 5, b = s & 31u;
                const uint32_t xb = S.cov[w] & (b == 31u ? ~0u : ((2u << b) - 1u));
                const uint32_t rs = max(1u, xb ? w * 32 + 31 - (uint32_t)__builtin_clz(xb) : (uint32_t)S.wrs[w]);
                uint32_t wf = w, xf = S.cov[w] & (b == 31u ? 0u : ~((2u << b) - 1u)), re = s + Z_MAXM + 3;
#pragma unroll 1
                for (int t = 0; t < 10; t++) {
                    if (xf) { re = wf * 32 + (uint32_t)__builtin_ctz(xf); break; }
                    if (++wf >= (uint32_t)CMAX / 32) { re = CMAX; break; }
                    xf = S.cov[wf];
                }
                const uint32_t B = s - rs;
                if (re >= s + 3 && B >= 8 && B <= j - lo) {
                    const uint32_t key = min(min(re - s, Z_MAXM), nice) << 16 | (s - 1);
                    k0 = key;
                    cnt = B;
                    j -= B;
                }
            }
#endif
            bool gd = !act || j <= lo || cnt >= lim || (k0 >> 16) >= nice;
            int ji = (int)j;
            // the chain limit can only bind where the bucket below s holds more
            // entries than are left to count (runs, long repeats): elsewhere the
            // counting is skipped for the whole wave
            const bool cnt_live = __any(act && cnt + (j - lo) > lim);
#pragma unroll 1
            while (__any(!gd)) {
                const int idx = ji - 1 - (int)r;
                const bool v = !gd & (idx >= (int)lo);
                // every lane loads (an index in range; a lane past the chain is masked by v)
                const uint32_t c = (uint32_t)S.lst[max(idx, 0)];
                const uint32_t a = c >> 2, sh = c & 3u;
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = c32[a + t];
                uint32_t x[4];
#pragma unroll
                for (int t = 0; t < 4; t++) x[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                const bool same = v & (z_h15(x[0] & 0xFFFFFFu) == h);
                uint32_t sm = 0;
                bool klim = true;
                if (cnt_live) {
                    sm = grp_bits<G>(__ballot(same), g);
                    klim = cnt + (uint32_t)__popc(sm & ((1u << r) - 1u)) + 1u <= lim;
                }
                // (a chunk of at most MAX_DIST bytes has every candidate in the window)
                constexpr bool WIN_ALL = (uint32_t)CMAX <= Z_MAXD;
                const bool inwin = WIN_ALL || s - c <= Z_MAXD;
                const bool ok = same & inwin & klim;
                uint32_t fm = ~0u;
#pragma unroll
                for (int t = 0; t < 4; t++) fm = min(fm, ffbl_raw(x[t] ^ tg[t]) | (uint32_t)t << 5);
                uint32_t len = fm == ~0u ? 16u : fm >> 3;
                // zlib's scan_end test: a candidate whose byte at the current best
                // length differs cannot be longer -- no full compare for it
                const uint32_t best = k0 >> 16;
                const bool can = best < 16 || S.ch[c + best] == S.ch[s + best];
#ifdef AMBC_Z9_SOLOEXT
                bool ext = ok && fm == ~0u && can;
#pragma unroll 1
                while (__any(ext)) {
                    if (ext) {
                        const uint32_t ac = (c + len) >> 2, as = (s + len) >> 2;
                        uint32_t wc[5], ws[5];
#pragma unroll
                        for (int t = 0; t < 5; t++) { wc[t] = c32[ac + t]; ws[t] = c32[as + t]; }
                        uint32_t f = ~0u;
#pragma unroll
                        for (int t = 0; t < 4; t++)
                            f = min(f, ffbl_raw(__builtin_amdgcn_alignbyte(wc[t + 1], wc[t], sh) ^
                                                __builtin_amdgcn_alignbyte(ws[t + 1], ws[t], ss)) |
                                           (uint32_t)t << 5);
                        if (f != ~0u) { len += f >> 3; ext = false; }
                        else { len += 16; if (len >= Z_MAXM) ext = false; }
                    }
                }
#else
                // the first 16 bytes equal: the group extends its candidates together,
                // the most recent first, 128 bytes a step (lane r compares bytes
                // [16 r, 16 r + 16) past the known length); once one reaches nice the
                // older ones cannot win (longest_match stops there)
                uint32_t em = grp_bits<G>(__ballot(ok && fm == ~0u && can), g);
#pragma unroll 1
                while (__any(em != 0u)) {
                    const bool gact = em != 0u;
                    const uint32_t rr = gact ? (uint32_t)__builtin_ctz(em) : 0u;
                    const uint32_t src = g * G + rr;
                    const uint32_t cc = (uint32_t)__shfl((int)c, (int)src);
                    const uint32_t ll = (uint32_t)__shfl((int)len, (int)src);
                    const uint32_t off = ll + 16u * r;
                    uint32_t f = ~0u;
                    if (gact && off < Z_MAXM) {
                        const uint32_t ac = (cc + off) >> 2, as = (s + off) >> 2, csh = cc & 3u;
                        uint32_t wc[5], ws[5];
#pragma unroll
                        for (int t = 0; t < 5; t++) { wc[t] = c32[ac + t]; ws[t] = c32[as + t]; }
#pragma unroll
                        for (int t = 0; t < 4; t++)
                            f = min(f, ffbl_raw(__builtin_amdgcn_alignbyte(wc[t + 1], wc[t], csh) ^
                                                __builtin_amdgcn_alignbyte(ws[t + 1], ws[t], ss)) |
                                           (uint32_t)t << 5);
                    } else if (gact) {
                        f = 0;          // past the longest match zlib takes: the length is capped there
                    }
                    const uint32_t mm = grp_bits<G>(__ballot(gact && f != ~0u), g);
                    const uint32_t r0 = mm ? (uint32_t)__builtin_ctz(mm) : 0u;
                    const uint32_t f0 = (uint32_t)__shfl((int)f, (int)(g * G + r0));
                    const uint32_t L2 = mm ? ll + 16u * r0 + (f0 >> 3) : ll + 16u * G;
                    if (gact && r == rr) len = L2;
                    if (gact && (mm || L2 >= Z_MAXM)) {
                        em &= em - 1u;                                       // this candidate is done
                        if (min(L2, Z_MAXM) >= nice) em = 0;                 // reached nice
                    }
                }
#endif
                const uint32_t Lp = min(min(len, Z_MAXM), nice);
                const uint32_t key = ok && can ? (Lp << 16 | c) : 0u;
                k0 = max(k0, grp_max<G>(key));
                cnt += (uint32_t)__popc(sm);
                const uint32_t far = WIN_ALL ? 0u : grp_bits<G>(__ballot(v && !inwin), g);
                ji -= (int)G;
                gd = gd | (ji <= (int)lo) | (far != 0) | (cnt >= lim) | ((k0 >> 16) >= nice);
            }
        }
        if (!done && !skip) {
            uint32_t ML = 2, MD = 0;
            if (act) {
                const uint32_t key = k0;
                const uint32_t L = key >> 16, d = s - (key & 0xFFFFu);
                if (L >= 3 && !(L == 3 && d > Z_TOOFAR)) { ML = L; MD = d; }
            }
            if (clean) {
                if (ML < 3) {
                    // a literal; the next position is clean again
                    if (r == 0) vs[q] = seg_lits(1u);
                    q++;
                    s = q;
                } else {
                    P = ML;
                    Pd = MD;
                    c = 0;
                    s = q + 1;
                    clean = false;
                }
            } else if (ML <= P) {
                // the pending match at s - 1 is emitted: its end is clean
                if (r == 0) {
                    vs[q] = seg_match(P, Pd, c);
                }
                q = s - 1 + P;
                s = q;
                P = 2;
                clean = true;
            } else {
                // a longer match at s: s - 1 goes out as a literal (lazy evaluation)
                c++;
                P = ML;
                Pd = MD;
                s++;
            }
        }
    }
}

// A chunk id 5 cannot win, decided before the parse (round 6).  When no 3-byte
// string occurs twice in the chunk, zlib's longest_match finds nothing anywhere
// and deflate emits n literals in one block (n <= 8192 < 16383 symbols); that
// block is at least min(dynamic, static, stored) long: dynamic >= 3 + 14 (HLIT,
// HDIST, HCLEN) + 12 (four code-length codes) + n H0 (any prefix code of the
// literals: Gibbs' inequality) + 1 (end of block) bits, static exactly 3 + 8 / 9
// bits a literal + 7, stored n + 5 bytes; zlib adds 2 + 4 bytes.  If even that
// bound loses (len + 18 >= T), so does id 5.  Random chunks (a third of the mixed
// input) are decided here, without the sort, the walkers, k_z9_heap and
// k_z9_code.  The repeat test is a hash set of the 3-byte strings in the sort's
// arrays (lst .. seg, free until the sort): a string met twice, or a probe run
// past 64 slots, means "maybe a match" (no decision).
template <int CMAX>
__device__ bool z9_cannot_win(Z9Smem<CMAX>& S, uint32_t n, uint32_t T, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NW = Z9Smem<CMAX>::NW, TT = 64u * NW, TB = 2u * (uint32_t)CMAX;
    static_assert(offsetof(Z9Smem<CMAX>, slot) == offsetof(Z9Smem<CMAX>, lst) + 2 * CMAX &&
                  offsetof(Z9Smem<CMAX>, bend32) == offsetof(Z9Smem<CMAX>, slot) + 2 * CMAX &&
                  offsetof(Z9Smem<CMAX>, seg) == offsetof(Z9Smem<CMAX>, bend32) + 2 * ZB4 &&
                  4 * TB <= 4 * CMAX + 2 * ZB4 + 4 * CMAX, "the hash set spans lst .. seg");
    const uint32_t tid = wave * 64u + lane;
    uint32_t* hist = S.seg + CMAX - 256;          // (the set's last slots hold no string yet)
    for (uint32_t i = tid; i < 256; i += TT) hist[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += TT) atomicAdd(&hist[S.ch[i]], 1u);
    __syncthreads();
    if (wave == 0) {
        double ent = 0.0;
        uint32_t stat = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t sy = lane + 64u * j, c = hist[sy];
            if (c) ent += (double)c * log2((double)n / (double)c);
            stat += c * (sy < 144 ? 8u : 9u);
        }
        ent = wave_sum<double>(ent);
        stat = wave_sum_u32(stat);
        const uint64_t dyn = 30 + (uint64_t)floor(ent * (1.0 - 1e-12));
        const uint64_t sta = 3 + (uint64_t)stat + 7;
        const uint64_t body = min((min(dyn, sta) + 7) / 8, (uint64_t)n + 5);
        if (lane == 0) S.nmatch = body + 6 + 18 >= T ? 1u : 0u;
    }
    __syncthreads();
    if (!S.nmatch) return false;
    uint32_t* tab = reinterpret_cast<uint32_t*>(S.lst);
    for (uint32_t i = tid; i < TB; i += TT) tab[i] = 0;
    __syncthreads();
    bool rep = false;
    for (uint32_t i = tid; i + 3 <= n; i += TT) {
        const uint32_t g = z_gram(S, i) + 1u;
        uint32_t h = (g * 2654435761u) >> (32 - __builtin_ctz(TB));
        for (int pr = 0; pr < 64; pr++) {
            const uint32_t old = atomicCAS(&tab[h], 0u, g);
            if (old == 0u) break;
            if (old == g || pr == 63) { rep = true; break; }
            h = (h + 1u) & (TB - 1u);
        }
    }
    if (lane == 0) S.nmatch = 0;
    __syncthreads();
    if (__any(rep) && lane == 0) S.nmatch = 1;   // (wave-level any, then one LDS flag)
    __syncthreads();
    return S.nmatch == 0;
}

#ifdef AMBC_STAMPS
// diagnostic build only: wave 0's phase cycles per parsed chunk in
// A.stamps[(2 M + k) * 8 + phase] (k_dict's slots; phase 7 = 1 marks a parse)
#define PSTAMP_DECL uint64_t _pt = __builtin_amdgcn_s_memtime(); uint64_t _pa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PSTAMP(ph)                                                 \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _pa[ph] += _t - _pt;                                       \
        _pt = _t;                                                  \
    } while (0)
#define PSTAMP_FLUSH                                                                  \
    if (threadIdx.x == 0 && A.stamps) {                                               \
        _pa[7] = 1;                                                                   \
        for (int _p = 0; _p < 8; _p++) A.stamps[(2ull * A.n_chunks + k) * 8 + _p] = _pa[_p]; \
    }
#else
#define PSTAMP_DECL
#define PSTAMP(ph) do {} while (0)
#define PSTAMP_FLUSH
#endif

template <int CMAX>
__global__ __launch_bounds__(64 * Z9Cfg<CMAX>::NW) void k_z9_parse(EncArgs A) {
    constexpr int NW = Z9Cfg<CMAX>::NW;
    __shared__ Z9Smem<CMAX> S;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
    PSTAMP_DECL
    const uint8_t* src = A.in + pos0;
    {
        const uint32_t TT = 64u * NW;
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            const uint32_t nv = n >> 4;
            for (uint32_t q = threadIdx.x; q < nv; q += TT)
                reinterpret_cast<uint4*>(S.ch)[q] = reinterpret_cast<const uint4*>(src)[q];
            for (uint32_t i = (nv << 4) + threadIdx.x; i < n; i += TT) S.ch[i] = src[i];
        } else {
            for (uint32_t i = threadIdx.x; i < n; i += TT) S.ch[i] = src[i];
        }
        for (uint32_t i = n + threadIdx.x; i < (uint32_t)CMAX + 320; i += TT) S.ch[i] = 0;
    }
    __syncthreads();
    PSTAMP(0);
    {
        uint32_t* R0 = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
        if (z9_cannot_win(S, n, T, wave, lane)) {
            if (threadIdx.x == 0) R0[1] = Z9_LOSES;
            return;
        }
        if (threadIdx.x == 0) R0[1] = 0;
    }
    z9_sort(S, n - 2, wave, lane);
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX; i += 64u * NW) S.seg[i] = 0;
    z9_literal_mask(S, n, wave, lane);
    __syncthreads();
    PSTAMP(1);
    z9_walkers(S, n, wave, lane);
    PSTAMP(2);
    __syncthreads();
    PSTAMP(3);
    // ---- the path from 0.  Per 64-position window, pointer doubling over the
    // lanes gives every clean position's exit from the window (the first path
    // position past it) and the matches on the way; thread 0 chains the windows
    // (one step per visited window); then every window's path is walked on the
    // scalar unit from its entry, and its matches are written at their ranks ----
    constexpr uint32_t NWIN = (uint32_t)CMAX / 64;
    const uint32_t nwin = (n + 63) / 64;
    const uint64_t below = (1ull << lane) - 1ull;
    uint16_t* xit = S.lst;    // the sort's lists are dead: exit position per position
    uint16_t* xm = S.slot;    // and matches to the exit
    for (uint32_t w = wave; w < nwin; w += NW) {
        const uint32_t p = w * 64 + lane;
        const uint32_t t = p < n ? S.seg[p] : 0u;
        uint32_t J = t ? lane + seg_c(t) + seg_L(t) : lane + 1;
        uint32_t M = seg_L(t) ? 1u : 0u;
#pragma unroll
        for (int it = 0; it < 6; it++) {
            const int src = (int)(min(J, 63u) << 2);
            const uint32_t Jj = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)J);
            const uint32_t Mj = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)M);
            M = J < 64 ? M + Mj : M;
            J = J < 64 ? Jj : J;
        }
        xit[p] = (uint16_t)(w * 64 + J);
        xm[p] = (uint16_t)M;
    }
    for (uint32_t i = threadIdx.x; i < NWIN; i += 64u * NW) S.entry[i] = 0xFFFFu;
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 32; i += 64u * NW) { S.mask[i] = 0; S.cov[i] = 0; }
    uint32_t* lf = S.bend32;   // the walkers are done: symbol counts (286 + 30 u32)
    for (uint32_t i = threadIdx.x; i < 316; i += 64u * NW) lf[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t cur = 0, mr = 0;
        while (cur < n) {
            S.entry[cur >> 6] = (uint16_t)(cur & 63u);
            S.rbase[cur >> 6] = (uint16_t)mr;
            mr += xm[cur];
            cur = xit[cur];
        }
        S.nmatch = mr;
    }
    __syncthreads();
    PSTAMP(4);
    uint32_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
    for (uint32_t w = wave; w < nwin; w += NW) {
        const uint32_t e = S.entry[w];
        if (e == 0xFFFFu) continue;
        const uint32_t p = w * 64 + lane;
        const uint32_t t = p < n ? S.seg[p] : 0u;
        const uint32_t c = seg_c(t), L = seg_L(t);
        const uint32_t J1 = lane + max(1u, c + L);   // (t != 0 on the path; never stall)
        uint64_t on = 0;
        for (uint32_t q = e; q < 64;) {
            on |= 1ull << q;
            q = readlane(J1, q);
        }
        const bool mt = ((on >> lane) & 1u) && L != 0;
        const uint64_t mm = __ballot(mt);
        if (mt) {
            const uint32_t ms = p + c, d = seg_d(t);
            atomicOr(&S.mask[ms >> 5], 1u << (ms & 31));
            R[Z9Rec<CMAX>::MATCH + S.rbase[w] + (uint32_t)__popcll(mm & below)] = L | d << 16;
            for (uint32_t b = ms, e2 = ms + L; b < e2;) {
                const uint32_t wd = b >> 5, hi = min(e2, (wd + 1) * 32);
                const uint32_t bits = (hi - b == 32 ? ~0u : ((1u << (hi - b)) - 1u)) << (b & 31);
                atomicOr(&S.cov[wd], bits);
                b = hi;
            }
            atomicAdd(&lf[257 + z_lcode(L)], 1u);
            atomicAdd(&lf[286 + z_dcode(d)], 1u);
        }
    }
    __syncthreads();
    // the literals: every position no match covers
    for (uint32_t i = threadIdx.x; i < n; i += 64u * NW)
        if (!((S.cov[i >> 5] >> (i & 31)) & 1u)) atomicAdd(&lf[S.ch[i]], 1u);
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 32; i += 64u * NW) R[Z9Rec<CMAX>::MASK + i] = S.mask[i];
    if (threadIdx.x == 0) R[0] = S.nmatch;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 158; i += 64u * NW) R[Z9Rec<CMAX>::FREQ + i] = lf[2 * i] | lf[2 * i + 1] << 16;
    PSTAMP(5);
    PSTAMP_FLUSH
}

template <int CMAX>
struct Z9CSmem {
    static constexpr int WORDS = (CMAX + 5 * (int)Z_NBLK + 64) / 4 + 4;
    // the body's bits only exist once the trees are built: they share the literal
    // tree's heap and the pointer-jumping scratch (round 6: 15.2 -> 11.0 KB at 4
    // KiB, 14 waves per CU instead of 10; {1,3,4,5z} 25.0 -> 25.9 GB/s same-box,
    // profiles/r6_z9_code_union_ab/)
    union {
        alignas(16) uint32_t bits[WORDS];    // the deflate body, LSB first
        struct {
            uint32_t heapL[LT_N + 1];
            uint16_t pjd[LT_N + 3], pja[LT_N + 3];   // z9_build_w's pointer-jumping scratch
        } tr;
    };
    uint32_t mstart[CMAX / 32 + 2];          // match starts (bitmask by position)
    uint32_t ecl[288], ecd[32];              // emission codes: code | len << 16
    uint32_t heapD[DT_N + 1];
    uint16_t lfreq[LT_N + 1], ldad[LT_N + 1], lcode[288];
    uint16_t dfreq[DT_N + 1], ddad[DT_N + 1], dcode[32];
    uint16_t bfreq[BT_N + 1], bdad[BT_N + 1], bcode[20];
    uint16_t blcL[16], blcD[16], blcB[16];
    uint32_t blc32[16], cnt32[20];
    uint8_t llen[LT_N + 1], dlen[DT_N + 1], blen[BT_N + 1];
    uint32_t misc[16];
};

#ifdef AMBC_STAMPS
// diagnostic build only: k_z9_code's phase cycles per chunk in A.stamps[(M + k) * 8 + phase]
#define ZSTAMP_DECL uint64_t _st_t = __builtin_amdgcn_s_memtime(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define ZSTAMP(ph)                                                 \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _acc[ph] += _t - _st_t;                                    \
        _st_t = _t;                                                \
    } while (0)
#define ZSTAMP_FLUSH                                               \
    if (lane == 0 && A.stamps)                                     \
        for (int _p = 0; _p < 8; _p++) A.stamps[((uint64_t)A.n_chunks + k) * 8 + _p] = _acc[_p];
#else
#define ZSTAMP_DECL
#define ZSTAMP(ph) do {} while (0)
#define ZSTAMP_FLUSH
#endif

template <int CMAX>
__global__ __launch_bounds__(64) void k_z9_code(EncArgs A) {
    __shared__ Z9CSmem<CMAX> S;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
    ZSTAMP_DECL
    const uint8_t* src = A.in + pos0;
    const uint32_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
    if (R[1] == Z9_LOSES) return;                    // (k_z9_parse: id 5 cannot win)
    const uint32_t* rec = R + Z9Rec<CMAX>::MATCH;   // the path's matches, L | dist << 16
    constexpr uint32_t nblk = Z_NBLK;
    static_assert(CMAX < (int)Z_BLKSYM, "one block per chunk");
    const uint64_t below = (1ull << lane) - 1ull;
    l32* W = (l32*)S.bits;
    const Z9Tree LT{(l16*)S.lfreq, (l16*)S.ldad, (l8*)S.llen, (l16*)S.lcode, (l32*)S.tr.heapL, (l16*)S.blcL};
    const Z9Tree DT{(l16*)S.dfreq, (l16*)S.ddad, (l8*)S.dlen, (l16*)S.dcode, (l32*)S.heapD, (l16*)S.blcD};
    const Z9Tree BT{(l16*)S.bfreq, (l16*)S.bdad, (l8*)S.blen, (l16*)S.bcode, (l32*)S.heapD, (l16*)S.blcB};

    // ---- the parse's match starts ----
    for (uint32_t i = lane; i < (uint32_t)CMAX / 32 + 2; i += 64)
        S.mstart[i] = i < (uint32_t)CMAX / 32 ? R[Z9Rec<CMAX>::MASK + i] : 0u;
    wave_sync();

    // the block's symbols over [bs, be), position-major, written from bit bp
    // (returns the bits written)
    auto pass = [&](uint32_t bs, uint32_t be, uint32_t rank0, uint32_t bp) -> uint32_t {
        uint32_t rank = rank0, out = 0;
        int carry = (int)bs;
        // a round's global loads (its matches, its bytes) are issued one round
        // ahead, so their latency hides behind the previous round's work
        auto fetch = [&](uint32_t q0, uint32_t rk, uint64_t& bmo, uint32_t& xo, uint32_t& co) {
            const uint32_t pos = q0 + lane;
            const bool in = pos >= bs && pos < be;
            const bool m = in && ((S.mstart[pos >> 5] >> (pos & 31)) & 1u);
            bmo = __ballot(m);
            xo = m ? rec[rk + (uint32_t)__popcll(bmo & below)] : 0u;
            co = in ? (uint32_t)src[pos] : 0u;
        };
        uint64_t bmn = 0;
        uint32_t xn = 0, cn = 0;
        fetch(bs & ~63u, rank, bmn, xn, cn);
#pragma unroll 1
        for (uint32_t p0 = bs & ~63u; p0 < be; p0 += 64) {
            const uint64_t bm = bmn;
            const uint32_t x = xn, cb = cn;
            const uint32_t rank2 = rank + (uint32_t)__popcll(bm);
            if (p0 + 64 < be) fetch(p0 + 64, rank2, bmn, xn, cn);
            const uint32_t pos = p0 + lane;
            const bool in = pos >= bs && pos < be;
            const bool ms = (bm >> lane) & 1u;
            const uint32_t L = ms ? x & 0xFFFFu : 0u, d = x >> 16;
            const int e = ms ? (int)(pos + L) : 0;
            const int E = max(carry, wave_incl_max_i32(e));
            carry = max(carry, wave_max_i32(e));
            rank = rank2;
            const bool lit = in && !ms && E <= (int)pos;
            const uint32_t c = lit ? cb : 0u;
            const uint32_t lc = ms ? z_lcode(L) : 0u, dc = ms ? z_dcode(d) : 0u;
            {
                uint32_t cost = 0, e1 = 0, e2 = 0, v1 = 0, v2 = 0;
                if (lit) {
                    e1 = S.ecl[c] >> 16;
                    v1 = S.ecl[c] & 0xFFFFu;
                } else if (ms) {
                    const uint32_t a = S.ecl[257 + lc], b = S.ecd[dc];
                    const uint32_t la = a >> 16, lb = b >> 16;
                    // the extra bits are the low bits of L - 3 / d - 1 (code bases
                    // are multiples of their extra range)
                    const uint32_t xl = z_xlb(lc), xd = z_xdb(dc);
                    e1 = la + xl;
                    v1 = (a & 0xFFFFu) | ((L - 3) & ((1u << xl) - 1u)) << la;
                    e2 = lb + xd;
                    v2 = (b & 0xFFFFu) | ((d - 1) & ((1u << xd) - 1u)) << lb;
                }
                cost = e1 + e2;
                const uint32_t incl = wave_incl_sum(cost);
                const uint32_t b = bp + out + incl - cost;
                z_put_atomic(S.bits, b, v1, e1);
                z_put_atomic(S.bits, b + e1, v2, e2);
                out += readlane(incl, 63);
            }
        }
        return out;
    };

    uint32_t bp = 0;
    for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t bs = 0, be = n;
        const uint32_t last = b + 1 == nblk ? 1u : 0u;
        // match starts before bs
        uint32_t rank0 = 0;
        for (uint32_t i = lane; i < (bs >> 5); i += 64) rank0 += (uint32_t)__popc(S.mstart[i]);
        if (lane == 0 && (bs & 31)) rank0 += (uint32_t)__popc(S.mstart[bs >> 5] & ((1u << (bs & 31)) - 1u));
        rank0 = wave_sum_u32(rank0);
        // the block's symbol counts (k_z9_parse) + the end of block
        const uint16_t* F = reinterpret_cast<const uint16_t*>(R + Z9Rec<CMAX>::FREQ);
        if (lane < 20) S.cnt32[lane] = 0;
        for (uint32_t i = lane; i < 286; i += 64) S.lfreq[i] = (uint16_t)(F[i] + (i == 256 ? 1u : 0u));
        if (lane < 30) S.dfreq[lane] = F[286 + lane];
        wave_sync();
        ZSTAMP(0);
        // ---- the trees: build_tree x 2, scan_tree x 2, build_bl_tree ----
        l16* PJD = (l16*)S.tr.pjd;
        l16* PJA = (l16*)S.tr.pja;
        l32* BLC = (l32*)S.blc32;
        l32* MISC = (l32*)(S.misc + 12);
        uint32_t optL = 0, statL = 0, optD = 0, statD = 0, optB = 0, statB = 0;
        const int lmax = z9_build_w<5, true>(LT, PJD, PJA, BLC, MISC, 286, 15, 0, optL, statL, lane,
                                               R + Z9Rec<CMAX>::MERGE);
        const int dmax = z9_build_w<1, true>(DT, PJD, PJA, BLC, MISC, 30, 15, 1, optD, statD, lane,
                                              R + Z9Rec<CMAX>::MERGE + 285);
        VHeap<5> LL;
        VHeap<1> DL;
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const uint32_t x = 64u * j + lane;
            LL.h[j] = (int)x <= lmax ? (uint32_t)S.llen[x] : 0u;
        }
        DL.h[0] = (int)lane <= dmax ? (uint32_t)S.dlen[lane] : 0u;
        (void)z9_rle_par(LL, lmax, false, (l32*)S.cnt32, 0u, S.bits, 0u, lane);
        (void)z9_rle_par(DL, dmax, false, (l32*)S.cnt32, 0u, S.bits, 0u, lane);
        wave_sync();
        if (lane < 19) S.bfreq[lane] = (uint16_t)S.cnt32[lane];
        wave_sync();
        (void)z9_build_w<1, false>(BT, PJD, PJA, BLC, MISC, 19, 7, 2, optB, statB, lane);
        ZSTAMP(2);
        int maxbl;
        for (maxbl = 18; maxbl >= 3; maxbl--) if (S.blen[z_blord[maxbl]] != 0) break;
        const uint32_t opt = optL + optD + optB + 3u * (uint32_t)(maxbl + 1) + 5 + 5 + 4;
        const uint32_t stl = statL + statD;
        uint32_t opt_lenb = (opt + 3 + 7) >> 3;
        const uint32_t static_lenb = (stl + 3 + 7) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        ZSTAMP(3);
        const uint32_t kind = be - bs + 4 <= opt_lenb ? 0u : (static_lenb == opt_lenb ? 1u : 2u);
        S.misc[8] = kind == 2 ? opt : stl;   // the block's bits after its 3 header bits
        if (nblk == 1) {
            // the exact length before any bit is written
            const uint32_t bits = kind == 0 ? ((3 + 7) & ~7u) + 32 + 8 * n : 3 + S.misc[8];
            const uint32_t total = 2 + (bits + 7) / 8 + 4;
            if (total + 18 >= T) { ZSTAMP_FLUSH; return; }
            if (A.flags & ENC_EVAL) {   // the multi-size walk's decision: no bits
                if (lane == 0) {
                    A.ids[k] = 5;
                    A.plen[k] = total;
                    A.sizes[k] = 18ull + total;
                }
                ZSTAMP_FLUSH;
                return;
            }
        }
        // the trees are done: their scratch becomes the body's bits
        for (uint32_t i = lane; i < (uint32_t)Z9CSmem<CMAX>::WORDS; i += 64) S.bits[i] = 0;
        wave_sync();
        if (kind == 0) {
            // stored: the 3 header bits, byte alignment, LEN / NLEN, the bytes
            const uint32_t stored_len = be - bs;
            uint32_t o = 0;
            if (lane == 0) z_put(W, bp, last, 3);
            bp = (bp + 3 + 7) & ~7u;
            uint8_t* by = reinterpret_cast<uint8_t*>(S.bits);
            o = bp >> 3;
            wave_sync();
            if (lane < 4) {
                const uint32_t v = lane < 2 ? stored_len : ~stored_len;
                by[o + lane] = (uint8_t)(v >> (8 * (lane & 1)));
            }
            for (uint32_t i = lane; i < stored_len; i += 64) by[o + 4 + i] = src[bs + i];
            bp += 8 * (4 + stored_len);
            wave_sync();
            continue;
        }
        // code tables for emission
        if (kind == 1) {
            for (uint32_t i = lane; i < 288; i += 64) {
                uint32_t c, l;
                if (i < 144) { c = 0x30 + i; l = 8; }
                else if (i < 256) { c = 0x190 + (i - 144); l = 9; }
                else if (i < 280) { c = i - 256; l = 7; }
                else { c = 0xC0 + (i - 280); l = 8; }
                S.ecl[i] = (__builtin_bitreverse32(c) >> (32 - l)) | l << 16;
            }
            if (lane < 30) S.ecd[lane] = (__builtin_bitreverse32(lane) >> 27) | 5u << 16;
        } else {
            for (uint32_t i = lane; i < 286; i += 64) S.ecl[i] = S.lcode[i] | (uint32_t)S.llen[i] << 16;
            if (lane < 30) S.ecd[lane] = S.dcode[lane] | (uint32_t)S.dlen[lane] << 16;
        }
        {
            // the block header on the scalar unit (the stream is word-aligned here)
            SBits sb{0ull, bp & 31u, bp >> 5};
            sb.acc = sb.n ? (uint64_t)(S.bits[sb.w] & ((1u << sb.n) - 1u)) : 0ull;
            sb_put(sb, W, kind << 1 | last, 3, lane);
            if (kind == 2) {
                sb_put(sb, W, (uint32_t)lmax + 1 - 257, 5, lane);
                sb_put(sb, W, (uint32_t)dmax, 5, lane);
                sb_put(sb, W, (uint32_t)maxbl + 1 - 4, 4, lane);
                for (int r = 0; r <= maxbl; r++) sb_put(sb, W, S.blen[z_blord[r]], 3, lane);
                const uint32_t bcl = lane < 19 ? (uint32_t)S.bcode[lane] | (uint32_t)S.blen[lane] << 16 : 0u;
                if (sb.n && lane == 0) W[sb.w] = (uint32_t)sb.acc;
                wave_sync();
                uint32_t p = sb.w * 32 + sb.n;
                p += z9_rle_par(LL, lmax, true, (l32*)S.cnt32, bcl, S.bits, p, lane);
                p += z9_rle_par(DL, dmax, true, (l32*)S.cnt32, bcl, S.bits, p, lane);
                sb.w = p >> 5;
                sb.n = p & 31u;
                sb.acc = 0;   // (the partial word is in LDS already)
            } else if (sb.n && lane == 0) {
                W[sb.w] = (uint32_t)sb.acc;
            }
            S.misc[9] = sb.w * 32 + sb.n;
        }
        wave_sync();
        ZSTAMP(4);
        bp = S.misc[9];
        bp += pass(bs, be, rank0, bp);
        wave_sync();
        if (lane == 0) z_put(W, bp, S.ecl[256] & 0xFFFFu, S.ecl[256] >> 16);
        bp += S.ecl[256] >> 16;
        wave_sync();
    }
    ZSTAMP(5);
    const uint32_t body = (bp + 7) >> 3;
    const uint32_t total = 2 + body + 4;
    if (total + 18 >= T) { ZSTAMP_FLUSH; return; }
    // ---- Adler-32 of the chunk ----
    const uint32_t adler = adler32_wave(src, n, lane);
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;
    const uint8_t* bb = reinterpret_cast<const uint8_t*>(S.bits);
    for (uint32_t i = lane; i < total; i += 64) {
        uint8_t o;
        if (i == 0) o = 0x78;
        else if (i == 1) o = 0xDA;
        else if (i < 2 + body) o = bb[i - 2];
        else o = (uint8_t)(adler >> (8 * (3 - (i - 2 - body))));
        slot[i] = o;
    }
    if (lane == 0) {
        A.ids[k] = 5;
        A.plen[k] = total;
        A.sizes[k] = 18ull + total;
    }
    ZSTAMP(6);
    ZSTAMP_FLUSH;
}

template <int CMAX>
hipError_t launch_z9_parse_t(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_z9_parse<CMAX>, dim3(a.n_chunks), dim3(64 * Z9Cfg<CMAX>::NW), 0, s, a);
    return hipGetLastError();
}
template <int CMAX>
hipError_t launch_z9_tail_t(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_z9_heap<CMAX>, dim3((a.n_chunks + ZH_L - 1) / ZH_L), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_z9_code<CMAX>, dim3(a.n_chunks), dim3(64), 0, s, a);
    return hipGetLastError();
}
template <int CMAX>
hipError_t launch_z9_t(const EncArgs& a, hipStream_t s) {
    const hipError_t e = launch_z9_parse_t<CMAX>(a, s);
    return e != hipSuccess ? e : launch_z9_tail_t<CMAX>(a, s);
}

}  // namespace

uint32_t z9_cmax(uint32_t chunk) {
    return chunk <= 1024 ? 1024u : chunk <= 2048 ? 2048u : chunk <= 4096 ? 4096u : chunk <= 8192 ? 8192u
         : chunk <= 16384 ? 16384u : chunk <= 32768 ? 32768u : chunk <= 65536 ? 65536u : 0u;
}

size_t z9_rec_words(uint32_t cmax) {
    switch (cmax) {
        case 1024: return Z9Rec<1024>::STRIDE;
        case 2048: return Z9Rec<2048>::STRIDE;
        case 4096: return Z9Rec<4096>::STRIDE;
        case 8192: return Z9Rec<8192>::STRIDE;
        default: return z9_rec_words_big(cmax);
    }
}

hipError_t launch_zlib9_parse(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    switch (z9_cmax(a.chunk_size)) {
        case 1024: return launch_z9_parse_t<1024>(a, s);
        case 2048: return launch_z9_parse_t<2048>(a, s);
        case 4096: return launch_z9_parse_t<4096>(a, s);
        case 8192: return launch_z9_parse_t<8192>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_zlib9_tail(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    switch (z9_cmax(a.chunk_size)) {
        case 1024: return launch_z9_tail_t<1024>(a, s);
        case 2048: return launch_z9_tail_t<2048>(a, s);
        case 4096: return launch_z9_tail_t<4096>(a, s);
        case 8192: return launch_z9_tail_t<8192>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_zlib9(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    switch (z9_cmax(a.chunk_size)) {
        case 1024: return launch_z9_t<1024>(a, s);
        case 2048: return launch_z9_t<2048>(a, s);
        case 4096: return launch_z9_t<4096>(a, s);
        case 8192: return launch_z9_t<8192>(a, s);
        default: return launch_zlib9_big(a, s);
    }
}

}  // namespace ambc
