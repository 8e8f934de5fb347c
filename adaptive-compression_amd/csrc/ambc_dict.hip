// ambc_dict.hip -- the Dictionary (id 2) encoder for gfx950.
//
// DictionaryCompression.compress (compression_methods.py:195-233) is a greedy
// LZ77 parse: at every position p the longest match of up to 32 bytes
// (lookahead, capped at n - p) against any start i in [max(0, p - 4096), p) --
// the EARLIEST i among the longest (strict '>' in _find_longest_match,
// :279-313) -- is emitted as (1, dist lo, dist hi, len) when len > 2, else the
// literal (0, byte).  should_use (:315-343) is "distinct 3-grams over the first
// min(n - 3, 1000) positions / min(1000, n) < 0.8" for n >= 100.  Both are
// reproduced byte for byte (oracle/ambc_oracle.c orc_dict_*).
//
// A match of length > 2 starts with the same 3 bytes, so the candidates of p
// are exactly the earlier positions of its 3-gram -- and the match at p does
// not depend on how the parse reached p.  One workgroup of NW waves per chunk:
//   1. the chunk in LDS; should_use's quick reject (distinct 13-bit hashes);
//   2. the 3-gram positions counting-sorted by an 11-bit hash into lst[],
//      STABLY (ascending inside a bucket): per 1024-position range and wave,
//      ballot ranks + range cursors, then per-bucket range offsets;
//      should_use exactly over the buckets (a repeat = an earlier entry of
//      the bucket with the same 3 bytes);
//   3. the parse by 64 / DG walkers per wave (DG-lane groups) from NW * 64 / DG
//      starts: a walker's match search takes the bucket's ascending run DG
//      candidates at a time (12 bytes compared first, 32 only when a
//      candidate matched 12), a group max over (len << 16 | ~i) keeps the
//      longest, earliest one; it records tok[p] and stops on a position another
//      walker visited (parses meet within a few tokens);
//   4. the path from 0 through tok[]: pointer doubling per 64-position window,
//      window tables composed per wave block, one serial pass over the blocks,
//      then every wave writes its block's tokens at their prefix offsets.
//
// Selection keeps the reference's order (ids ascending, strict '<'): k_encode
// has already picked the best of ids 1/3/4/9 (exact length of the winner;
// everything it skipped is provably no shorter), so id 2 wins iff
// len + 18 < T, or len + 18 == T against ids 3/4/9; T = winner len + 18 (raw:
// n).  Walker 0 stops the parse as soon as its length plus a lower bound of the
// rest (4 bytes per 32 still to cover) can no longer win, and the path's token
// bytes are known before any is written, so the slot keeps k_encode's payload
// unless id 2 wins.  Runs between
// k_encode and k_deflate, which then sees id 2's length as the bar to beat.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

// 1024 buckets up to 4 KiB (round 6): their cursor arrays for all eight waves'
// ranges fit tok[] (2048 buckets: four waves rank, four wait) -- {1,2,3,4} 98.1 ->
// 99.0 GB/s same-box (profiles/r6_dict_nb10_ab/); 8 KiB keeps 2048 (all its waves
// rank already; 1024 there: the {1,2,3,4,5} walk 5.6 -> 5.4 GB/s,
// profiles/r6_dict_nb_walk_ab/)
#ifndef AMBC_DICT_NB10
#define AMBC_DICT_NB10 1
#endif
// 3-gram hash buckets per chunk size: 1024 up to 4 KiB (1: 8 KiB keeps 2048,
// whose eight ranges already fill tok[] and every wave; 2: 1024 everywhere)
template <int CMAX> struct DictHash {
    static constexpr uint32_t BITS = AMBC_DICT_NB10 == 0 ? 11u : AMBC_DICT_NB10 == 2 ? 10u : (CMAX >= 8192 ? 11u : 10u);
    static constexpr uint32_t NB = 1u << BITS;
};
constexpr uint32_t DWIN = 4096;     // compression_methods.py:187 window_size
constexpr uint32_t DLOOK = 32;      // :187 lookahead_size

#ifndef AMBC_DICT_DG
#define AMBC_DICT_DG 8
#endif
constexpr uint32_t DG = AMBC_DICT_DG;   // lanes per walker (8 or 16)
#ifndef AMBC_DICT_2STAGE
#define AMBC_DICT_2STAGE 1
#endif
// the winner's tokens staged in LDS and stored 16 bytes at a time (round 6):
// {1,2,3,4} 98.9 -> 103.1 GB/s same-box (profiles/r6_dict_stage_ab/)
#ifndef AMBC_DICT_STAGE
#define AMBC_DICT_STAGE 1
#endif
#ifndef AMBC_DICT_NW4K
#define AMBC_DICT_NW4K 8
#endif
// NW waves per chunk, 64 / DG walkers of DG lanes each
template <int CMAX> struct DictCfg {
    static constexpr int NW = CMAX <= 1024 ? 2 : (CMAX <= 2048 ? 4 : (CMAX <= 4096 ? AMBC_DICT_NW4K : 8));
};


template <int CMAX>
struct DictSmem {
    static constexpr int NW = DictCfg<CMAX>::NW;
    alignas(16) uint8_t ch[CMAX + 64];   // the chunk, zero padded
    union {
        // 3-gram positions by bucket, ascending inside one
        alignas(16) uint16_t lst[CMAX];
        uint32_t bits[256];                 // before the sort: should_use's hash bitmap
        struct {
            // after the parse, per wave's block of 64-position windows and entry
            // offset e < 32 into its first window: the next block's entry | bytes << 8
            uint32_t etab[NW][32];
            uint32_t be[NW], bo[NW];        // each block's entry and token bytes before it
        } path;
    };
    // counts (u16 pairs, 32-bit atomics) -> bucket starts (the scatter's cursors)
    // -> bucket ends: after the scatter bucket h is lst[h ? bend[h-1] : 0, bend[h])
    alignas(16) uint32_t bend32[DictHash<CMAX>::NB / 2];
    // the sort: per range and bucket a cursor (u16);
    // the parse: tok[p] = 0 (not visited) or 1 << 31 | len << 16 | dist (a
    // literal: len 1) for every position a walker has visited
    alignas(16) uint32_t tok[CMAX];
    uint32_t flag;    // abort broadcast
    uint32_t cnt;     // should_use's repeats, then the path's step count
    uint32_t olen;    // the path's token bytes
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

// v_ffbl_b32 as the hardware defines it: the lowest set bit, ~0 for 0
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

template <int CMAX>
__device__ __forceinline__ uint32_t h3(uint32_t v) { return ((v & 0xFFFFFFu) * 2654435761u) >> (32 - DictHash<CMAX>::BITS); }

// the 3-gram at position i (bytes i..i+2, little-endian)
template <int CMAX>
__device__ __forceinline__ uint32_t gram_at(const DictSmem<CMAX>& S, uint32_t i) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    const uint32_t lo = c32[i >> 2], hi = c32[(i >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, i & 3) & 0xFFFFFFu;
}

// Stable counting sort of positions [0, m) by h3 into lst[] (bucket ends in
// bend[]).  The chunk splits into CMAX / 1024 ranges of 16 64-position groups,
// one wave each, with its own cursor per bucket (in tok[], free until the
// parse): a group ranks its lanes among its equal-hash lanes (eleven ballots)
// and advances the range's cursors -- 16 dependent steps per range, ranges in
// parallel.  Per bucket the ranges' counts turn into offsets, one wave scans
// the totals into bucket ends, and the ranges scatter without further order.
template <int CMAX>
__device__ void build_buckets(DictSmem<CMAX>& S, uint32_t m, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NW = DictSmem<CMAX>::NW, T = 64u * NW;
    constexpr uint32_t DBITS = DictHash<CMAX>::BITS, DNB = DictHash<CMAX>::NB;
    constexpr uint32_t NR = DBITS == 10 ? ((uint32_t)CMAX / 512 < NW ? (uint32_t)CMAX / 512 : NW) : (uint32_t)CMAX / 1024;
    constexpr uint32_t GR = (uint32_t)CMAX / (64 * NR);
    static_assert(NR >= 1 && NR <= NW && NR * DNB * 2 <= (uint32_t)CMAX * 4, "cursor arrays live in tok[]");
    uint16_t* cnt = reinterpret_cast<uint16_t*>(S.tok);   // [NR][DNB]
    const uint32_t tid = wave * 64u + lane;
    for (uint32_t b = tid; b < NR * DNB / 2; b += T) S.tok[b] = 0;
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t loc[GR];   // my index inside my bucket's part of the range | h << 16, ~0: none
    if (wave < NR) {
        uint16_t* c = cnt + wave * DNB;
#pragma unroll
        for (uint32_t g = 0; g < GR; g++) {
            const uint32_t i = (wave * GR + g) * 64 + lane;
            const bool v = i < m;
            const uint32_t h = v ? h3<CMAX>(gram_at(S, i)) : 0u;
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int b = 0; b < (int)DBITS; b++) {
                const uint64_t mb = __ballot(v && ((h >> b) & 1u));
                peers &= ((h >> b) & 1u) ? mb : ~mb;
            }
            const uint32_t base = v ? (uint32_t)c[h] : 0u;
            loc[g] = v ? (base + (uint32_t)__popcll(peers & below)) | h << 16 : ~0u;
            if (v && (peers >> lane) == 1ull) c[h] = (uint16_t)(base + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    // per bucket: the ranges' counts -> their offsets inside the bucket; the total
    for (uint32_t h = tid; h < DNB; h += T) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t r = 0; r < NR; r++) {
            const uint32_t x = cnt[r * DNB + h];
            cnt[r * DNB + h] = (uint16_t)run;
            run += x;
        }
        S.bend()[h] = (uint16_t)run;
    }
    __syncthreads();
    if (wave == 0) {
        // inclusive scan in place (32 buckets per lane): bucket ends
        constexpr int WPL = (int)DNB / 128;   // u16 pairs per lane
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
                S.lst[S.bstart(h) + cnt[wave * DNB + h] + (loc[g] & 0xFFFFu)] = (uint16_t)((wave * GR + g) * 64 + lane);
            }
        }
    }
    __syncthreads();
}

// minimum token bytes to cover r more bytes: 4 per 32, the rest one match or literals
__device__ __forceinline__ uint32_t lb_cost(uint32_t r) {
    const uint32_t q = r & 31u;
    return 4u * (r >> 5) + (q ? min(4u, 2u * q) : 0u);
}

#ifdef AMBC_STAMPS
// diagnostic build only: wave 0's phase cycles per parsed chunk (s_memtime) in
// A.stamps[(2 M + k) * 8 + phase]; phase 7 = 1 marks a chunk that was parsed
#define DSTAMP_DECL uint64_t _st_t = __builtin_amdgcn_s_memtime(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define DSTAMP(ph)                                                 \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _acc[ph] += _t - _st_t;                                    \
        _st_t = _t;                                                \
    } while (0)
#define DSTAMP_FLUSH                                                                  \
    if (threadIdx.x == 0 && A.stamps) {                                               \
        _acc[7] = 1;                                                                  \
        for (int _p = 0; _p < 8; _p++) A.stamps[(2ull * A.n_chunks + k) * 8 + _p] = _acc[_p]; \
    }
#else
#define DSTAMP_DECL
#define DSTAMP(ph) do {} while (0)
#define DSTAMP_FLUSH
#endif

// should_use (compression_methods.py:315-343), all waves.  First the distinct
// 13-bit hashes of the first lim 3-grams (<= the distinct 3-grams): when they
// already reach 0.8 ss it is False without the exact count (random data).
template <int CMAX>
__device__ bool dict_su_maybe(DictSmem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane) {
    constexpr uint32_t T = 64u * DictSmem<CMAX>::NW;
    const uint32_t tid = wave * 64u + lane;
    const uint32_t ss = min(1000u, n), lim = min(n - 3, ss);
    for (uint32_t w = tid; w < 256; w += T) S.bits[w] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < lim; i += T) {
        const uint32_t h = (gram_at(S, i) * 2654435761u) >> 19;
        atomicOr(&S.bits[h >> 5], 1u << (h & 31));
    }
    __syncthreads();
    uint32_t dh = 0;
    for (uint32_t w = lane; w < 256; w += 64) dh += __popc(S.bits[w]);
    dh = wave_sum_u32(dh);
    __syncthreads();   // the bitmap's words are the sort's next
    return 5 * dh < 4 * ss;
}

// the exact count over the buckets (ascending positions: a position repeats iff
// an earlier entry of its bucket holds the same 3 bytes); S.cnt = 0 beforehand
template <int CMAX>
__device__ bool dict_su_exact(DictSmem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane) {
    constexpr uint32_t T = 64u * DictSmem<CMAX>::NW;
    const uint32_t tid = wave * 64u + lane;
    const uint32_t ss = min(1000u, n), lim = min(n - 3, ss);
    uint32_t rep = 0;
    for (uint32_t i = tid; i < lim; i += T) {
        const uint32_t g = gram_at(S, i);
        for (uint32_t j = S.bstart(h3<CMAX>(g));; j++) {
            const uint32_t q = S.lst[j];
            if (q >= i) break;
            if (gram_at(S, q) == g) { rep++; break; }
        }
    }
    rep = wave_sum_u32(rep);
    if (lane == 0 && rep) atomicAdd(&S.cnt, rep);
    __syncthreads();
    return 5 * (lim - S.cnt) < 4 * ss;   // u / ss < 0.8 exactly (the quotient is never within an ulp of 0.8)
}

// max over the DG lanes of a group (every lane gets it): quad butterflies,
// then the half-row mirror (8 lanes) and the row mirror (16 lanes)
__device__ __forceinline__ uint32_t grp_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, true));  // row_half_mirror
    if (DG == 16) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, true));  // row_mirror
    return x;
}

// lanes of my group set in a ballot
__device__ __forceinline__ uint32_t grp_bits(uint64_t m, uint32_t g) {
    return (uint32_t)(m >> (DG * g)) & ((1u << DG) - 1u);
}


// The greedy parse's walkers (compression_methods.py:208-233).  The longest
// match at p (:279-313) -- the earliest i among the longest, found over the
// bucket's candidates 16 at a time as the max of len << 16 | (0xFFFF - i) --
// does not depend on how p was reached, so 4 NW walkers parse from as many
// starts at once, each a 16-lane group; a walker records tok[] for the
// positions it visits and stops on reaching one another walker visited (the
// rest of the path is the same).  Every visited position's successor is
// visited, so the path from 0 is complete in tok[].  Control flow is uniform
// over the wave; per-walker state is group-uniform in VGPRs.
template <int CMAX>
__device__ __forceinline__ void dict_walkers(DictSmem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane,
                                             bool force, int lim2) {
    constexpr uint32_t NWK = (uint32_t)DictCfg<CMAX>::NW * (64u / DG);
    typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
    lds_vu32* vt = (lds_vu32*)S.tok;
    lds_vu32* vflag = (lds_vu32*)&S.flag;
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    const uint32_t g = lane / DG, r = lane % DG;
    const uint32_t wid = wave * (64u / DG) + g;
    const bool w0 = wid == 0;     // walker 0: tracks the token bytes for the early stop
    uint32_t p = (uint32_t)(((uint64_t)n * wid) / NWK);
    uint32_t o = 0;
    bool done = false;
#pragma unroll 1
    for (;;) {
        // the lookahead bytes p .. p+31 as dwords (the group's lanes read the
        // same words), issued together with the visited check
        uint32_t tg[8];
        {
            const uint32_t a = p < n ? p >> 2 : 0u, sh = p & 3;
            uint32_t w[9];
#pragma unroll
            for (int q = 0; q < 9; q++) w[q] = c32[a + q];
            const uint32_t seen = p < n ? vt[p] : 1u;
            done = done || seen != 0 || *vflag != 0;
#pragma unroll
            for (int q = 0; q < 8; q++) tg[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
        }
        if (w0 && !done && !force && (int)(o + lb_cost(n - p)) > lim2) {
            if (r == 0) *vflag = 1u;   // id 2 cannot win: every walker stops
            done = true;
        }
        if (__all(done)) break;
        const uint32_t look = done ? 0u : min(DLOOK, n - p);
        const uint32_t h = h3<CMAX>(tg[0]);
        uint32_t j = S.bstart(h);
        const uint32_t e = look >= 3 ? (uint32_t)S.bend()[h] : j;
        if (CMAX > (int)DWIN) {
            // window start (:294): the first bucket entry >= p - 4096, by a
            // 16-ary search over the ascending run [j, e)
            const uint32_t ws = p > DWIN ? p - DWIN : 0u;
            uint32_t lo = j, hi = ws ? e : j;
#pragma unroll 1
            while (__any(hi > lo)) {
                const uint32_t len = hi - lo;
                const uint32_t st = (len + DG - 1) / DG;
                const uint32_t idx = lo + r * st;
                const uint32_t c = __popc(grp_bits(__ballot(hi > lo && idx < hi && S.lst[idx] < ws), g));
                if (hi > lo) {
                    if (c == 0) hi = lo;
                    else {
                        const uint32_t nlo = lo + (c - 1) * st + 1;
                        hi = min(lo + c * st, hi);
                        lo = nlo;
                    }
                }
            }
            j = ws ? lo : j;
        }
        uint32_t key = 0;
        bool gd = j >= e;
#pragma unroll 1
        while (__any(!gd)) {
            const uint32_t idx = j + r;
            const uint32_t i = (!gd && idx < e) ? S.lst[idx] : 0xFFFFu;
            const bool v = i < p;
            // the candidate's 32 bytes (nine dwords issued together), compared
            // as dwords: 32 q + the first differing bit of dword q, ffbl(0) = ~0
            const uint32_t a = v ? i >> 2 : 0u, sh = i & 3;
#if AMBC_DICT_2STAGE
            // the first 12 bytes; the other 20 only when a candidate matches all 12
            uint32_t w[9], f[8];
#pragma unroll
            for (int q = 0; q < 4; q++) w[q] = c32[a + q];
#pragma unroll
            for (int q = 0; q < 3; q++)
                f[q] = ffbl_raw((uint32_t)__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) ^ tg[q]) | (uint32_t)q << 5;
            uint32_t fm = min(min(f[0], f[1]), f[2]);
            if (__any(v && fm == ~0u)) {
#pragma unroll
                for (int q = 4; q < 9; q++) w[q] = c32[a + q];
#pragma unroll
                for (int q = 3; q < 8; q++)
                    f[q] = ffbl_raw((uint32_t)__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) ^ tg[q]) | (uint32_t)q << 5;
                fm = min(fm, min(min(min(f[3], f[4]), min(f[5], f[6])), f[7]));
            }
#else
            uint32_t w[9];
#pragma unroll
            for (int q = 0; q < 9; q++) w[q] = c32[a + q];
            uint32_t f[8];
#pragma unroll
            for (int q = 0; q < 8; q++)
                f[q] = ffbl_raw((uint32_t)__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) ^ tg[q]) | (uint32_t)q << 5;
            const uint32_t fm = min(min(min(f[0], f[1]), min(f[2], f[3])), min(min(f[4], f[5]), min(f[6], f[7])));
#endif
            const uint32_t L = v ? min(fm >> 3, look) : 0u;
            key = max(key, grp_max(v ? (L << 16 | (0xFFFFu - i)) : 0u));
            // ascending candidates: stop at the cap (the earliest reaching it
            // wins) or once the run reached p or the bucket's end
            const uint32_t vg = grp_bits(__ballot(v), g);
            gd = gd || vg != (1u << DG) - 1u || (key >> 16) >= look;
            j += DG;
        }
        if (!done) {
            const uint32_t L = key >> 16;
            if (r == 0) vt[p] = L > 2 ? 0x80000000u | L << 16 | (p - (0xFFFFu - (key & 0xFFFFu))) : 0x80010000u;
            o += L > 2 ? 4u : 2u;
            p += L > 2 ? L : 1u;
        }
    }
}


template <int CMAX>
__global__ __launch_bounds__(64 * DictCfg<CMAX>::NW) void k_dict(EncArgs A) {
    constexpr int NW = DictCfg<CMAX>::NW;
    __shared__ DictSmem<CMAX> S;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    const bool force = A.flags & ENC_FORCE;
    const bool analyze = A.flags & ENC_ANALYZE;
    const bool elig = ((A.method_mask >> 2) & 1u) && n >= A.pref_min[2] && n <= A.pref_max[2] &&
                      n <= (uint32_t)CMAX;
    if (A.flags & ENC_EMIT_PENDING) return;
    if (!elig && !analyze) return;
    if (n == 0) return;
    // selection bar from k_encode's winner (adaptive_compressor.py:559-579)
    int lim2 = 0;
    if (!force) {
        const uint32_t w = A.ids[k];
        const uint32_t T = w == 255 ? n : A.plen[k] + HDR;
        lim2 = (int)T - (int)HDR - ((w == 255 || w == 1) ? 1 : 0);
    }
    const bool want = elig && (force || lim2 >= (int)(2 + lb_cost(n - 1)));
    if (!want && !analyze) return;
    DSTAMP_DECL
    const uint8_t* src = A.in + pos0;
    const uint32_t ns = min(n, (uint32_t)CMAX);
    {
        const uint32_t T = 64u * NW;
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            const uint32_t nv = ns >> 4;
            for (uint32_t q = threadIdx.x; q < nv; q += T)
                reinterpret_cast<uint4*>(S.ch)[q] = reinterpret_cast<const uint4*>(src)[q];
            for (uint32_t i = (nv << 4) + threadIdx.x; i < ns; i += T) S.ch[i] = src[i];
        } else {
            for (uint32_t i = threadIdx.x; i < ns; i += T) S.ch[i] = src[i];
        }
        for (uint32_t i = ns + threadIdx.x; i < (uint32_t)CMAX + 64; i += T) S.ch[i] = 0;
    }
    if (threadIdx.x == 0) {
        S.flag = 0;
        S.cnt = 0;
    }
    __syncthreads();
    DSTAMP(0);

    // ---- should_use (compression_methods.py:315-343) and the buckets ----
    const uint32_t m = n >= 3 ? n - 2 : 0;
    const bool need_su = !force && n >= 100;
    const bool maybe = need_su && dict_su_maybe(S, n, wave, lane);
    DSTAMP(1);
    if (!(force || maybe)) return;   // su False: nothing to record, no parse
    // (analyze mode also sees chunks beyond CMAX: should_use reads only the
    // first 1003 bytes, and the sort stays inside the loaded ns)
    build_buckets(S, min(m, ns - 2), wave, lane);
    DSTAMP(2);
    const bool su = need_su && dict_su_exact(S, n, wave, lane);
    if (analyze && A.su && threadIdx.x == 0) A.su[k] |= su ? 4 : 0;
    DSTAMP(1);
    if (!want || (!force && !su)) return;
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX; i += 64u * NW) S.tok[i] = 0;
    __syncthreads();
    DSTAMP(3);

    // ---- the greedy parse (compression_methods.py:208-233) ----
    dict_walkers(S, n, wave, lane, force, lim2);
    DSTAMP(4);
    __syncthreads();
    DSTAMP(5);
    if (S.flag) return;

    // ---- walker 0's path from 0.  Each wave takes a block of consecutive
    // 64-position windows; per window, pointer doubling over lanes gives every
    // position's chain to the first position past the window (entries are the
    // window's first 32 positions) and its token bytes; composed over the block
    // they form a 32-entry table, and one short serial pass over the blocks
    // yields every block's entry and output offset -- the token bytes decide the
    // selection before anything is written ----
    constexpr uint32_t WPB = ((uint32_t)CMAX / 64 + NW - 1) / NW;   // windows per block, at most
    const uint32_t nwin = (n + 63) / 64;
    const uint32_t wpb = (nwin + NW - 1) / NW;
    const uint32_t wb0 = wave * wpb;
    const uint64_t below = (1ull << lane) - 1ull;
    {
        uint32_t E = lane & 31u, BB = 0;
#pragma unroll
        for (uint32_t i = 0; i < WPB; i++) {
            const uint32_t wi = wb0 + i;
            if (i >= wpb || wi >= nwin) break;
            const uint32_t pos = wi * 64 + lane;
            const uint32_t t = pos < n ? S.tok[pos] : 0u;
            const uint32_t L = (t >> 16) & 0xFFu;
            uint32_t J = pos < n ? lane + max(L, 1u) : 64u;
            uint32_t B = pos < n && t ? (L > 2 ? 4u : 2u) : 0u;
#pragma unroll
            for (int r = 0; r < 6; r++) {
                const int src = (int)(min(J, 63u) << 2);
                const uint32_t Bj = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)B);
                const uint32_t Jj = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)J);
                B = J < 64 ? B + Bj : B;
                J = J < 64 ? Jj : J;
            }
            // J - 64 < 32: the entry into the next window
            const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(E << 2), (int)((J - 64) | B << 8));
            BB += x >> 8;
            E = x & 31u;
        }
        if (lane < 32) S.path.etab[wave][lane] = E | BB << 8;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t e = 0, o = 0;
        for (uint32_t w = 0; w < (uint32_t)NW; w++) {
            S.path.be[w] = e;
            S.path.bo[w] = o;
            if (w * wpb < nwin) {
                const uint32_t x = S.path.etab[w][e];
                e = x & 31u;
                o += x >> 8;
            }
        }
        S.olen = o;
        if (!force && (int)o > lim2) S.flag = 1u;   // id 2 loses
    }
    __syncthreads();
    if (S.flag) return;
    // ---- id 2 wins (or is forced): every wave walks its block's path from its
    // entry (chain walk in registers) and writes the tokens into the slot at
    // their prefix offsets ----
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;
    uint16_t* s16 = reinterpret_cast<uint16_t*>(slot);
    const uint32_t o = S.olen;
    // the tokens staged in LDS (lst[] past the path tables, dead after the walk)
    // and copied out with 16-byte stores, instead of 2-byte stores scattered over
    // the slot; a forced encode (plugins, up to 2n bytes) writes directly
    constexpr uint32_t SOFF = 2048;
    static_assert(sizeof(S.path) <= SOFF, "the path tables stay below the staging area");
    const bool stg = AMBC_DICT_STAGE && !force && o + SOFF <= 2u * (uint32_t)CMAX &&
                     (reinterpret_cast<uintptr_t>(slot) & 15) == 0;
    typedef __attribute__((address_space(3))) uint16_t lds_u16;
    lds_u16* L16 = (lds_u16*)(reinterpret_cast<uint8_t*>(S.lst) + SOFF);
    if (!(A.flags & ENC_EVAL)) {   // (the multi-size walk's decision-only batches: no bytes)
        uint32_t e = S.path.be[wave], ob = S.path.bo[wave];
#pragma unroll 1
        for (uint32_t i = 0; i < wpb; i++) {
            const uint32_t wi = wb0 + i;
            if (wi >= nwin) break;
            const uint32_t p0 = wi * 64;
            const uint32_t t = p0 + lane < n ? S.tok[p0 + lane] : 0u;
            uint64_t on = 0;
            uint32_t q = e;
            while (q < 64 && p0 + q < n) {
                const uint32_t tq = __builtin_amdgcn_readlane(t, q);
                on |= 1ull << q;
                q += max(1u, (tq >> 16) & 0xFFu);
            }
            const bool me = (on >> lane) & 1u;
            const uint32_t L = (t >> 16) & 0xFFu;
            const bool mt = me && L > 2;
            const uint64_t mm = __ballot(mt);
            const uint32_t off = ob + 2u * (uint32_t)(__popcll(on & below) + __popcll(mm & below));
            if (mt) {
                const uint32_t d = t & 0xFFFFu;
                const uint16_t w0 = (uint16_t)(1u | (d & 0xFFu) << 8), w1 = (uint16_t)((d >> 8) | L << 8);
                if (stg) { L16[off >> 1] = w0; L16[(off >> 1) + 1] = w1; }
                else { s16[off >> 1] = w0; s16[(off >> 1) + 1] = w1; }
            } else if (me) {
                const uint16_t w0 = (uint16_t)(S.ch[p0 + lane] << 8);
                if (stg) L16[off >> 1] = w0;
                else s16[off >> 1] = w0;
            }
            ob += 2u * (uint32_t)(__popcll(on) + __popcll(mm));
            e = q - 64;
        }
        if (stg) {
            __syncthreads();
            const uint4* src4 = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(S.lst) + SOFF);
            uint4* dst4 = reinterpret_cast<uint4*>(slot);
            for (uint32_t q = threadIdx.x; q < (o + 15) / 16; q += 64u * NW) dst4[q] = src4[q];
        }
    }
    if (threadIdx.x == 0) {
        A.ids[k] = 2;
        A.plen[k] = o;
        A.sizes[k] = (uint64_t)HDR + o;
        if (A.pending) A.pending[k] = 0;
        if (A.bestpre) A.bestpre[k] = (A.bestpre[k] & 0xC0000000u) | (o + HDR);
    }
    DSTAMP(6);
    DSTAMP_FLUSH
}

template <int CMAX>
hipError_t launch_dict_t(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_dict<CMAX>, dim3(a.n_chunks), dim3(64 * DictCfg<CMAX>::NW), 0, s, a);
    return hipGetLastError();
}

}  // namespace

// cmax: the largest chunk id 2 may take (min(chunk_size, pref_max[2]), <= 8192)
hipError_t launch_dict(const EncArgs& a, uint32_t cmax, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    if (cmax <= 1024) return launch_dict_t<1024>(a, s);
    if (cmax <= 2048) return launch_dict_t<2048>(a, s);
    if (cmax <= 4096) return launch_dict_t<4096>(a, s);
    return launch_dict_t<8192>(a, s);
}

}  // namespace ambc
