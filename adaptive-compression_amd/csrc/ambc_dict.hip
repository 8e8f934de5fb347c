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
    alignas(16) unsigned long long bk[128];   // sort: lane masks per 7-bit bucket
    // window start per bucket: only chunks longer than the 4096-byte window need it
    alignas(16) uint16_t wp[CMAX > (int)DWIN ? DNB : 8];
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

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

template <int CMAX>
__global__ __launch_bounds__(64) void k_dict(EncArgs A) {
    __shared__ DictSmem<CMAX> S;
    const uint32_t lane = threadIdx.x;
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
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            const uint32_t nv = ns >> 4;
            for (uint32_t q = lane; q < nv; q += 64)
                reinterpret_cast<uint4*>(S.ch)[q] = reinterpret_cast<const uint4*>(src)[q];
            for (uint32_t i = (nv << 4) + lane; i < ns; i += 64) S.ch[i] = src[i];
        } else {
            for (uint32_t i = lane; i < ns; i += 64) S.ch[i] = src[i];
        }
        for (uint32_t i = ns + lane; i < (uint32_t)CMAX + 64; i += 64) S.ch[i] = 0;
    }
    wave_sync();

    // ---- should_use (compression_methods.py:315-343) ----
    bool su = false;
    if (!force && n >= 100) {
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
        if (5 * dh >= 4 * ss) goto su_done;
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
        su = 5 * u < 4 * ss;   // u / ss < 0.8 exactly (the quotient is never within an ulp of 0.8)
        wave_sync();
    }
su_done:
    if (analyze && A.su && lane == 0) A.su[k] |= su ? 4 : 0;
    if (!want || (!force && !su)) return;

    // ---- the greedy parse (compression_methods.py:208-233, :279-313) ----
    const uint32_t m = n >= 3 ? n - 2 : 0;
    build_buckets(S, m, lane);
    if (CMAX > (int)DWIN && n > DWIN + 1)
        for (uint32_t b = lane; b < DNB; b += 64) S.wp[b] = (uint16_t)S.bstart(b);
    wave_sync();
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;
    // tokens: a forced encode writes the slot; otherwise they stage in the
    // slot's upper half (C bytes >= any winning payload) and move down only if
    // id 2 wins, so k_encode's payload stays intact
    uint8_t* stage = force ? slot : slot + A.chunk_size + 64;
    uint16_t* stg16 = reinterpret_cast<uint16_t*>(stage);
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    uint32_t p = 0, o = 0;
    bool lost = false;
#pragma unroll 1
    while (p < n) {
        p = __builtin_amdgcn_readfirstlane(p);
        o = __builtin_amdgcn_readfirstlane(o);
        const uint32_t r = n - p;
        if (!force && (int)(o + lb_cost(r)) > lim2) { lost = true; break; }
        const uint32_t look = min(DLOOK, r);
        uint32_t key = 0;
        if (look >= 3) {
            const uint32_t h = __builtin_amdgcn_readfirstlane(h3(gram_at(S, p)));
            uint32_t j = __builtin_amdgcn_readfirstlane(CMAX > (int)DWIN && n > DWIN + 1 ? S.wp[h] : S.bstart(h));
            const uint32_t e = __builtin_amdgcn_readfirstlane(S.bend()[h]);
            if (CMAX > (int)DWIN && p > DWIN) {
                // window start: skip the bucket's entries below p - 4096 (ascending run)
                const uint32_t ws = p - DWIN;
                uint32_t j0 = j;
                for (;;) {
                    const uint32_t idx = j0 + lane;
                    const uint64_t below = __ballot(idx < e && S.lst[idx] < ws);
                    const uint32_t c = (uint32_t)__popcll(below);
                    j0 += c;
                    if (c < 64) break;
                }
                j = __builtin_amdgcn_readfirstlane(j0);
                wave_sync();
                if (lane == 0) S.wp[h] = (uint16_t)j;
            }
            // the lookahead bytes p .. p+31 as dwords
            uint32_t tg[8];
            {
                const uint32_t a = p >> 2, sh = p & 3;
                uint32_t lo = c32[a];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const uint32_t hi = c32[a + q + 1];
                    tg[q] = __builtin_amdgcn_alignbyte(hi, lo, sh);
                    lo = hi;
                }
            }
#pragma unroll 1
            for (; j < e; j += 64) {
                const uint32_t idx = j + lane;
                const uint32_t i = idx < e ? S.lst[idx] : 0xFFFFu;
                const bool v = i < p;
                if (!__any(v)) break;                // ascending: nothing earlier than p follows
                uint32_t L = 0;
                bool act = v;
                const uint32_t a = v ? i >> 2 : 0u, sh = i & 3;
                uint32_t lo = c32[a];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    if (4u * q >= look || !__any(act)) break;
                    const uint32_t hi = c32[a + q + 1];
                    const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, sh) ^ tg[q];
                    if (act) {
                        if (x) { L = 4u * q + ((uint32_t)__builtin_ctz(x) >> 3); act = false; }
                        else L = 4u * q + 4u;
                    }
                    lo = hi;
                }
                L = min(L, look);
                const int kv = v ? (int)(L << 16 | (0xFFFFu - i)) : 0;
                key = max(key, (uint32_t)wave_max_i32(kv));
                if ((key >> 16) >= look) break;      // cap reached by the earliest candidate so far
                if (!__all(v)) break;                // the run reached p
            }
        }
        key = __builtin_amdgcn_readfirstlane(key);
        const uint32_t L = key >> 16;
        if (L > 2) {
            const uint32_t d = p - (0xFFFFu - (key & 0xFFFFu));
            if (lane == 0) {
                stg16[o >> 1] = (uint16_t)(1u | (d & 0xFFu) << 8);
                stg16[(o >> 1) + 1] = (uint16_t)((d >> 8) | L << 8);
            }
            o += 4;
            p += L;
        } else {
            if (lane == 0) stg16[o >> 1] = (uint16_t)(S.ch[p] << 8);
            o += 2;
            p += 1;
        }
    }
    if (!force && (lost || (int)o > lim2)) return;
    wave_sync();
    if (!force) {
        // id 2 wins: its tokens replace k_encode's payload (lane 0's stores made
        // visible to the whole wave first)
        __threadfence();
        const uint32_t nw = (o + 3) >> 2;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(stage);
        for (uint32_t q = lane; q < nw; q += 64) reinterpret_cast<uint32_t*>(slot)[q] = src[q];
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
    hipLaunchKernelGGL(k_dict<CMAX>, dim3(a.n_chunks), dim3(64), 0, s, a);
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
