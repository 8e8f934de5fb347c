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
// are exactly the earlier positions of its 3-gram.  One 64-lane wavefront per
// chunk:
//   1. the chunk in LDS; the 3-gram positions counting-sorted by an 11-bit
//      hash into lst[] -- STABLY (positions ascending inside a bucket: ranks
//      among equal-hash lanes of a 64-position group from LDS bucket masks +
//      four ballots), bst[] = bucket starts;
//   2. should_use: the same sort over the first lim positions; a position is
//      a repeat iff an earlier entry of its bucket holds the same 3 bytes;
//   3. the greedy parse, serial over tokens: for p, the bucket's entries in
//      the window are a contiguous ascending run (the window start advances
//      monotonically per bucket, wp[], for chunks beyond the 4096-byte
//      window); 64 candidates per step compare 32
//      bytes as dwords (v_alignbyte), and a wave max over (len << 16 | ~i)
//      keeps the longest, earliest one.  Oldest-first order lets a step stop
//      as soon as a candidate reaches the lookahead cap (runs, repeats).
//
// Selection keeps the reference's order (ids ascending, strict '<'): k_encode
// has already picked the best of ids 1/3/4/9 (exact length of the winner;
// everything it skipped is provably no shorter), so id 2 wins iff
// len + 18 < T, or len + 18 == T against ids 3/4/9; T = winner len + 18 (raw:
// n).  The parse stops as soon as its length plus a lower bound of the rest
// (4 bytes per 32 still to cover) can no longer win, and stages its tokens in
// LDS, so the slot keeps k_encode's payload unless id 2 wins.  Runs between
// k_encode and k_deflate, which then sees id 2's length as the bar to beat.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

constexpr uint32_t DNB = 2048;      // 3-gram hash buckets (11 bits)
constexpr uint32_t DWIN = 4096;     // compression_methods.py:187 window_size
constexpr uint32_t DLOOK = 32;      // :187 lookahead_size

template <int CMAX>
struct DictSmem {
    alignas(16) uint8_t ch[CMAX + 64];   // the chunk, zero padded
    alignas(16) uint16_t lst[CMAX];      // 3-gram positions by bucket, ascending inside one
    // counts (u16 pairs, 32-bit atomics) -> bucket starts (the scatter's cursors)
    // -> bucket ends: after the scatter bucket h is lst[h ? bend[h-1] : 0, bend[h])
    alignas(16) uint32_t bend32[DNB / 2];
    union {
        unsigned long long bk[128];      // sort: lane masks per 7-bit bucket
        // the parse: tok[p] = 0 (not visited) or 1 << 31 | len << 16 | dist
        // (a literal: len 1) for every position a walker has visited
        uint32_t tok[CMAX];
    };
    uint32_t flag;                       // should_use / abort broadcast
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

// v_ffbl_b32 as the hardware defines it: the lowest set bit, ~0 for 0
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t h3(uint32_t v) { return ((v & 0xFFFFFFu) * 2654435761u) >> 21; }

// the 3-gram at position i (bytes i..i+2, little-endian)
template <int CMAX>
__device__ __forceinline__ uint32_t gram_at(const DictSmem<CMAX>& S, uint32_t i) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    const uint32_t lo = c32[i >> 2], hi = c32[(i >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, i & 3) & 0xFFFFFFu;
}

// stable counting sort of positions [0, m) by h3 into lst[] (bucket ends in bend[])
template <int CMAX>
__device__ void build_buckets(DictSmem<CMAX>& S, uint32_t m, uint32_t lane) {
    for (uint32_t b = lane; b < DNB / 2; b += 64) S.bend32[b] = 0;
    unsigned long long* bk = S.bk;
    for (uint32_t b = lane; b < 128; b += 64) bk[b] = 0;
    wave_sync();
    // counts < 2^16: two buckets per dword
    for (uint32_t i = lane; i < m; i += 64) {
        const uint32_t h = h3(gram_at(S, i));
        atomicAdd(&S.bend32[h >> 1], 1u << (16 * (h & 1)));
    }
    wave_sync();
    // exclusive scan in place (32 buckets per lane): bucket starts = cursors
    {
        uint32_t c[16], t = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            c[j] = S.bend32[lane * 16 + j];
            t += (c[j] & 0xFFFFu) + (c[j] >> 16);
        }
        uint32_t run = wave_incl_sum(t) - t;
        wave_sync();
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t r0 = run, r1 = run + (c[j] & 0xFFFFu);
            S.bend32[lane * 16 + j] = r0 | r1 << 16;
            run = r1 + (c[j] >> 16);
        }
    }
    wave_sync();
    uint16_t* cur = S.bend();
    // scatter, 64 ascending positions per step; equal-hash lanes keep lane order;
    // each cursor ends at its bucket's end
#pragma unroll 1
    for (uint32_t g = 0; g < m; g += 64) {
        const uint32_t i = g + lane;
        const bool v = i < m;
        const uint32_t h = v ? h3(gram_at(S, i)) : 0u;
        if (v) atomicOr(&bk[h & 127u], 1ull << lane);
        wave_sync();
        uint64_t peers = v ? bk[h & 127u] : 0ull;
#pragma unroll
        for (int b = 7; b < 11; b++) {
            const uint64_t mb = __ballot(v && ((h >> b) & 1u));
            peers &= ((h >> b) & 1u) ? mb : ~mb;
        }
        const uint32_t base = v ? cur[h] : 0u;
        wave_sync();
        if (v) {
            bk[h & 127u] = 0ull;
            S.lst[base + __popcll(peers & ((1ull << lane) - 1ull))] = (uint16_t)i;
            if ((peers >> lane) == 1ull) cur[h] = (uint16_t)(base + (uint32_t)__popcll(peers));
        }
        wave_sync();
    }
}

// minimum token bytes to cover r more bytes: 4 per 32, the rest one match or literals
__device__ __forceinline__ uint32_t lb_cost(uint32_t r) {
    const uint32_t q = r & 31u;
    return 4u * (r >> 5) + (q ? min(4u, 2u * q) : 0u);
}

// should_use (compression_methods.py:315-343) by one wave
template <int CMAX>
__device__ bool dict_should_use(DictSmem<CMAX>& S, uint32_t n, uint32_t lane) {
    const uint32_t ss = min(1000u, n);
    const uint32_t lim = min(n - 3, ss);
    // distinct 13-bit hashes <= distinct 3-grams: when they already reach
    // 0.8 ss, should_use is False without the exact count (random data)
    uint32_t* bits = reinterpret_cast<uint32_t*>(S.bk);    // 8192 bits
    for (uint32_t w = lane; w < 256; w += 64) bits[w] = 0;
    wave_sync();
    for (uint32_t i = lane; i < lim; i += 64) {
        const uint32_t h = (gram_at(S, i) * 2654435761u) >> 19;
        atomicOr(&bits[h >> 5], 1u << (h & 31));
    }
    wave_sync();
    uint32_t dh = 0;
    for (uint32_t w = lane; w < 256; w += 64) dh += __popc(bits[w]);
    dh = wave_sum_u32(dh);
    wave_sync();
    if (5 * dh >= 4 * ss) return false;
    build_buckets(S, lim, lane);
    uint32_t rep = 0;
    for (uint32_t i = lane; i < lim; i += 64) {
        const uint32_t g = gram_at(S, i);
        const uint32_t h = h3(g);
        for (uint32_t j = S.bstart(h);; j++) {
            const uint32_t q = S.lst[j];
            if (q >= i) break;
            if (gram_at(S, q) == g) { rep++; break; }
        }
    }
    const uint32_t u = lim - wave_sum_u32(rep);
    wave_sync();
    return 5 * u < 4 * ss;   // u / ss < 0.8 exactly (the quotient is never within an ulp of 0.8)
}

// max over the 16 lanes of a DPP row (every lane gets it): quad butterflies,
// then rotations by 4 and 8 inside the row
__device__ __forceinline__ uint32_t row16_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, true));  // row_ror:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, true));  // row_ror:8
    return x;
}

// lanes of my 16-lane group set in a ballot
__device__ __forceinline__ uint32_t grp16(uint64_t m, uint32_t g) { return (uint32_t)(m >> (16 * g)) & 0xFFFFu; }

constexpr uint32_t DG = 16;   // lanes per walker: 4 walkers per wave

// NW waves per chunk, 4 walkers of 16 lanes each
template <int CMAX> struct DictCfg { static constexpr int NW = CMAX <= 1024 ? 2 : (CMAX <= 2048 ? 4 : 8); };

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
        {
            const uint32_t seen = p < n ? vt[p] : 1u;
            done = done || seen != 0 || *vflag != 0;
        }
        if (w0 && !done && !force && (int)(o + lb_cost(n - p)) > lim2) {
            if (r == 0) *vflag = 1u;   // id 2 cannot win: every walker stops
            done = true;
        }
        if (__all(done)) break;
        const uint32_t look = done ? 0u : min(DLOOK, n - p);
        // the lookahead bytes p .. p+31 as dwords (the group's lanes read the same words)
        uint32_t tg[8];
        {
            const uint32_t a = done ? 0u : p >> 2, sh = p & 3;
            uint32_t w[9];
#pragma unroll
            for (int q = 0; q < 9; q++) w[q] = c32[a + q];
#pragma unroll
            for (int q = 0; q < 8; q++) tg[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
        }
        const uint32_t h = h3(tg[0]);
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
                const uint32_t c = __popc(grp16(__ballot(hi > lo && idx < hi && S.lst[idx] < ws), g));
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
            uint32_t w[9];
#pragma unroll
            for (int q = 0; q < 9; q++) w[q] = c32[a + q];
            uint32_t f[8];
#pragma unroll
            for (int q = 0; q < 8; q++)
                f[q] = ffbl_raw((uint32_t)__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) ^ tg[q]) | (uint32_t)q << 5;
            const uint32_t fm = min(min(min(f[0], f[1]), min(f[2], f[3])), min(min(f[4], f[5]), min(f[6], f[7])));
            const uint32_t L = v ? min(fm >> 3, look) : 0u;
            key = max(key, row16_max(v ? (L << 16 | (0xFFFFu - i)) : 0u));
            // ascending candidates: stop at the cap (the earliest reaching it
            // wins) or once the run reached p or the bucket's end
            const uint32_t vg = grp16(__ballot(v), g);
            gd = gd || vg != 0xFFFFu || (key >> 16) >= look;
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
    const uint32_t n = A.coff ? A.clen[k] : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
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
    __syncthreads();

    const uint32_t m = n >= 3 ? n - 2 : 0;
    if (wave == 0) {
        const bool su = !force && n >= 100 && dict_should_use(S, n, lane);
        if (analyze && A.su && lane == 0) A.su[k] |= su ? 4 : 0;
        const bool go = want && (force || su);
        if (go) build_buckets(S, m, lane);
        if (lane == 0) S.flag = go ? 0u : 1u;
    }
    __syncthreads();
    if (S.flag) return;
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX; i += 64u * NW) S.tok[i] = 0;
    __syncthreads();

    // ---- the greedy parse (compression_methods.py:208-233) ----
    dict_walkers(S, n, wave, lane, force, lim2);
    __syncthreads();
    if (wave != 0 || S.flag) return;

    // ---- walker 0's path, 64 positions per step: chain walk over tok[] in
    // registers, then every token of the step written at its prefix offset ----
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;
    // tokens: a forced encode writes the slot; otherwise they stage in the
    // slot's upper half (C bytes >= any winning payload) and move down only if
    // id 2 wins, so k_encode's payload stays intact
    uint8_t* stage = force ? slot : slot + A.chunk_size + 64;
    uint16_t* stg16 = reinterpret_cast<uint16_t*>(stage);
    uint32_t p = 0, o = 0;
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll 1
    while (p < n) {
        const uint32_t t = p + lane < n ? S.tok[p + lane] : 0u;
        uint64_t on = 0;
        uint32_t q = p;
        while (q < n && q < p + 64) {
            const uint32_t tq = __builtin_amdgcn_readlane(t, q - p);
            on |= 1ull << (q - p);
            q += max(1u, (tq >> 16) & 0xFFu);
        }
        const bool me = (on >> lane) & 1u;
        const uint32_t L = (t >> 16) & 0xFFu;
        const bool mt = me && L > 2;
        const uint64_t mm = __ballot(mt);
        const uint32_t tot = 2u * (uint32_t)(__popcll(on) + __popcll(mm));
        if (!force && (int)(o + tot) > lim2) return;   // id 2 loses
        const uint32_t off = o + 2u * (uint32_t)(__popcll(on & below) + __popcll(mm & below));
        if (mt) {
            const uint32_t d = t & 0xFFFFu;
            stg16[off >> 1] = (uint16_t)(1u | (d & 0xFFu) << 8);
            stg16[(off >> 1) + 1] = (uint16_t)((d >> 8) | L << 8);
        } else if (me) {
            stg16[off >> 1] = (uint16_t)(S.ch[p + lane] << 8);
        }
        o += tot;
        p = q;
    }
    if (!force) {
        // id 2 wins: its tokens replace k_encode's payload
        __threadfence();
        wave_sync();
        const uint32_t nw = (o + 3) >> 2;
        const uint32_t* src32 = reinterpret_cast<const uint32_t*>(stage);
        for (uint32_t q = lane; q < nw; q += 64) reinterpret_cast<uint32_t*>(slot)[q] = src32[q];
    }
    if (lane == 0) {
        A.ids[k] = 2;
        A.plen[k] = o;
        A.sizes[k] = (uint64_t)HDR + o;
        if (A.pending) A.pending[k] = 0;
        if (A.bestpre) A.bestpre[k] = (A.bestpre[k] & 0xC0000000u) | (o + HDR);
    }
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
