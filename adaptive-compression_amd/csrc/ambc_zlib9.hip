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
//      lookahead; position 0 is its NIL) counting-sorted by an 11-bit hash OF
//      THE 15-bit zlib hash, stably: a bucket's entries below p, read downward,
//      are p's hash chain (most recent first) plus other-hash entries that the
//      search skips by recomputing their 15-bit hash;
//   3. the lazy parse by walkers (8-lane groups).  zlib's longest_match at p
//      is the first chain entry reaching the longest length (capped at
//      min(258, n - p)), over the first 4096 entries -- or 1024 when the
//      previous match was >= 32 long: both answers come out of one scan.  After
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

namespace ambc {
namespace {

constexpr uint32_t ZNB = 2048;               // sort buckets (11 bits of the 15-bit hash)
constexpr uint32_t Z_MAXM = 258;             // MAX_MATCH
constexpr uint32_t Z_MAXD = 32768 - 262;     // MAX_DIST: w_size - MIN_LOOKAHEAD
constexpr uint32_t Z_CHAIN = 4096;           // max_chain at level 9
constexpr uint32_t Z_GOOD = 32;              // good_length: chain >> 2 beyond it
constexpr uint32_t Z_TOOFAR = 4096;
constexpr uint32_t Z_BLKSYM = 16383;         // lit_bufsize - 1 symbols per block
constexpr uint32_t Z_NBLK = 8;               // record-area block starts (n <= 65536: <= 5 blocks)

__constant__ uint16_t z_lbase[29] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  10,  12,  14,  16,  20, 24,
                                     28, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 255};
__constant__ uint8_t z_xl[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t z_dbase[30] = {0,    1,    2,    3,    4,    6,    8,     12,    16,    24,
                                     32,   48,   64,   96,   128,  192,  256,   384,   512,   768,
                                     1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 24576};
__constant__ uint8_t z_xd[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t z_blord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// length code (0..28) of a match length 3..258 (zlib's _length_code)
__device__ __forceinline__ uint32_t z_lcode(uint32_t L) {
    if (L == 258) return 28;
    const uint32_t y = L - 3;
    if (y < 8) return y;
    const uint32_t b = 31 - __builtin_clz(y);
    return 4 * (b - 1) + ((y >> (b - 2)) & 3);
}
// distance code (0..29) of a distance 1..32768 (zlib's d_code)
__device__ __forceinline__ uint32_t z_dcode(uint32_t D) {
    const uint32_t x = D - 1;
    if (x < 4) return x;
    const uint32_t b = 31 - __builtin_clz(x);
    return 2 * b + ((x >> (b - 1)) & 1);
}

// zlib's hash of the 3 bytes at p (UPDATE_HASH three times, hash_shift 5, 15 bits)
__device__ __forceinline__ uint32_t z_h15(uint32_t g) {
    return (((g & 0xFFu) << 10) ^ (((g >> 8) & 0xFFu) << 5) ^ ((g >> 16) & 0xFFu)) & 0x7FFFu;
}
__device__ __forceinline__ uint32_t z_bucket(uint32_t h15) { return (h15 * 2654435761u) >> 21; }

__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// the chunk gate and selection bar of k_deflate (ambc_deflate.hip): false = id 5
// is not tried for chunk k
__device__ __forceinline__ bool z9_gate(const EncArgs& A, uint32_t k, uint32_t n, uint32_t& T) {
    if (!((A.method_mask >> 5) & 1) || n < A.pref_min[5] || n > A.pref_max[5] || n < 64) return false;
    const uint32_t w0 = A.ids[k];
    const uint32_t bp0 = A.bestpre[k];
    if (bp0 >> 31) return false;   // calculate_entropy == 8.0: should_use is False
    const uint32_t bestpre = bp0 & 0x3FFFFFFFu;
    T = w0 == 9 ? min(bestpre, A.plen[k] + 18 + 1) : bestpre;
    return T > 18 + 6;
}

// per chunk: [0] = records | blocks << 32, [1 .. Z_NBLK] block starts, then
// records c | L << 16 | dist << 32 (c literals, then a match of L, or L = 0 at the end)
template <int CMAX> struct Z9Rec {
    static constexpr uint32_t STRIDE = 1 + Z_NBLK + CMAX / 3 + 3;   // u64 words
};

template <int CMAX> struct Z9Cfg {
    static constexpr int NW = CMAX <= 1024 ? 2 : (CMAX <= 2048 ? 4 : 8);
};

template <int CMAX>
struct Z9Smem {
    static constexpr int NW = Z9Cfg<CMAX>::NW;
    alignas(16) uint8_t ch[CMAX + 320];      // the chunk, zeros past n
    alignas(16) uint16_t lst[CMAX];          // positions by bucket, ascending inside one
    alignas(16) uint16_t slot[CMAX];         // position -> its index in lst
    alignas(16) uint32_t bend32[ZNB / 2];    // bucket ends (u16 pairs)
    // the sort's per-range cursors [NR][ZNB] u16; then the parse: seg[q] = 0
    // (not reached) or 1 << 31 | L << 16 | c for a fresh position q
    alignas(16) uint32_t seg[CMAX];
    alignas(16) uint16_t sd[CMAX];           // the segment's match distance
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

template <int CMAX>
__device__ __forceinline__ uint32_t z_gram(const Z9Smem<CMAX>& S, uint32_t i) {
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    return __builtin_amdgcn_alignbyte(c32[(i >> 2) + 1], c32[i >> 2], i & 3) & 0xFFFFFFu;
}

// Stable counting sort of positions [1, m) into lst[] by z_bucket(z_h15) --
// ambc_dict.hip's build_buckets with the zlib hash and each position's slot.
template <int CMAX>
__device__ void z9_sort(Z9Smem<CMAX>& S, uint32_t m, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NW = Z9Smem<CMAX>::NW, T = 64u * NW;
    constexpr uint32_t NR = (uint32_t)CMAX / 1024, GR = 16;
    static_assert(NR >= 1 && NR <= NW && NR * ZNB * 2 <= (uint32_t)CMAX * 4, "cursor arrays live in seg[]");
    uint16_t* cnt = reinterpret_cast<uint16_t*>(S.seg);
    const uint32_t tid = wave * 64u + lane;
    for (uint32_t b = tid; b < NR * ZNB / 2; b += T) S.seg[b] = 0;
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t loc[GR];
    if (wave < NR) {
        uint16_t* c = cnt + wave * ZNB;
#pragma unroll
        for (uint32_t g = 0; g < GR; g++) {
            const uint32_t i = (wave * GR + g) * 64 + lane;
            const bool v = i >= 1 && i < m;
            const uint32_t h = v ? z_bucket(z_h15(z_gram(S, i))) : 0u;
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int b = 0; b < 11; b++) {
                const uint64_t mb = __ballot(v && ((h >> b) & 1u));
                peers &= ((h >> b) & 1u) ? mb : ~mb;
            }
            const uint32_t base = v ? (uint32_t)c[h] : 0u;
            loc[g] = v ? (base + (uint32_t)__popcll(peers & below)) | h << 16 : ~0u;
            if (v && (peers >> lane) == 1ull) c[h] = (uint16_t)(base + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    for (uint32_t h = tid; h < ZNB; h += T) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t r = 0; r < NR; r++) {
            const uint32_t x = cnt[r * ZNB + h];
            cnt[r * ZNB + h] = (uint16_t)run;
            run += x;
        }
        S.bend()[h] = (uint16_t)run;
    }
    __syncthreads();
    if (wave == 0) {
        uint32_t c[16], t = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            c[j] = S.bend32[lane * 16 + j];
            t += (c[j] & 0xFFFFu) + (c[j] >> 16);
        }
        uint32_t run = wave_incl_sum(t) - t;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t r0 = run + (c[j] & 0xFFFFu), r1 = r0 + (c[j] >> 16);
            S.bend32[lane * 16 + j] = r0 | r1 << 16;
            run = r1;
        }
    }
    __syncthreads();
    if (wave < NR) {
#pragma unroll
        for (uint32_t g = 0; g < GR; g++) {
            if (loc[g] != ~0u) {
                const uint32_t h = loc[g] >> 16;
                const uint32_t idx = S.bstart(h) + cnt[wave * ZNB + h] + (loc[g] & 0xFFFFu);
                const uint32_t pos = (wave * GR + g) * 64 + lane;
                S.lst[idx] = (uint16_t)pos;
                S.slot[pos] = (uint16_t)idx;
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t grp_max8(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, true));  // row_half_mirror
    return x;
}
__device__ __forceinline__ uint32_t grp8(uint64_t m, uint32_t g) { return (uint32_t)(m >> (8 * g)) & 0xFFu; }

// The lazy parse's walkers (deflate_slow).  Per 8-lane group: q = the fresh
// position its current segment started at, s = the position being looked at,
// P / Pd = the previous position's match (prev_length / distance), avail =
// match_available.  One longest_match per iteration for every active group.
template <int CMAX>
__device__ __forceinline__ void z9_walkers(Z9Smem<CMAX>& S, uint32_t n, uint32_t wave, uint32_t lane) {
    constexpr uint32_t NWK = (uint32_t)Z9Cfg<CMAX>::NW * 8u;
    typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
    lds_vu32* vs = (lds_vu32*)S.seg;
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.ch);
    const uint32_t g = lane >> 3, r = lane & 7;
    const uint32_t wid = wave * 8u + g;
    uint32_t q = (uint32_t)(((uint64_t)n * wid) / NWK);
    uint32_t s = q, P = 2, Pd = 0;
    bool fresh = true, done = false;
#pragma unroll 1
    for (;;) {
        if (fresh && !done && (q >= n || vs[q] != 0u)) done = true;
        if (__all(done)) break;
        const bool act = !done && s >= 1 && s + 3 <= n && P < 258;   // position 0 is zlib's NIL
        // ---- longest_match(s): k0 over the first 4096 chain entries, k1 over
        // the first 1024; key = min(len, nice) << 16 | candidate (the longest,
        // then the most recent) ----
        uint32_t k0 = 0, k1 = 0;
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
                lo = S.bstart(z_bucket(h));
                j = S.slot[s];
                nice = min(Z_MAXM, n - s);
            }
            bool gd = !act || j <= lo;
            uint32_t cnt = 0;
#pragma unroll 1
            while (__any(!gd)) {
                const int idx = (int)j - 1 - (int)r;
                const bool v = !gd && idx >= (int)lo;
                const uint32_t c = v ? (uint32_t)S.lst[idx] : 0u;
                const uint32_t a = c >> 2, sh = c & 3u;
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = c32[a + t];
                uint32_t x[4];
#pragma unroll
                for (int t = 0; t < 4; t++) x[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                const bool same = v && z_h15(x[0] & 0xFFFFFFu) == h;
                const uint32_t sm = grp8(__ballot(same), g);
                const uint32_t kidx = cnt + (uint32_t)__popc(sm & ((1u << r) - 1u)) + 1u;
                const bool inwin = s - c <= Z_MAXD;
                const bool ok = same && inwin && kidx <= Z_CHAIN;
                uint32_t fm = ~0u;
#pragma unroll
                for (int t = 0; t < 4; t++) fm = min(fm, ffbl_raw(x[t] ^ tg[t]) | (uint32_t)t << 5);
                uint32_t len = fm == ~0u ? 16u : fm >> 3;
                bool ext = ok && fm == ~0u;
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
                const uint32_t Lp = min(min(len, Z_MAXM), nice);
                const uint32_t key = ok ? (Lp << 16 | c) : 0u;
                k0 = max(k0, grp_max8(key));
                k1 = max(k1, grp_max8(ok && kidx <= Z_CHAIN / 4 ? key : 0u));
                cnt += (uint32_t)__popc(sm);
                const uint32_t far = grp8(__ballot(v && !inwin), g);
                j = j > lo + 8 ? j - 8 : lo;
                gd = gd || j <= lo || far != 0 || cnt >= Z_CHAIN || (k0 >> 16) >= nice;
            }
        }
        if (!done) {
            if (s >= n) {
                // the input ends: the segment's literals run to n
                if (r == 0) vs[q] = 0x80000000u | (n - q);
                done = true;
            } else {
                uint32_t ML = 2, MD = 0;
                if (act) {
                    const uint32_t key = P >= Z_GOOD ? k1 : k0;
                    const uint32_t L = key >> 16, d = s - (key & 0xFFFFu);
                    if (L >= 3 && !(L == 3 && d > Z_TOOFAR)) { ML = L; MD = d; }
                }
                if (P >= 3 && ML <= P) {
                    // the previous position's match: the segment ends with it
                    const uint32_t ms = s - 1;
                    if (r == 0) {
                        S.sd[q] = (uint16_t)Pd;
                        vs[q] = 0x80000000u | P << 16 | (ms - q);
                    }
                    q = ms + P;
                    s = q;
                    P = 2;
                    fresh = true;
                } else {
                    P = ML;
                    Pd = MD;
                    s++;
                    fresh = false;
                }
            }
        }
    }
}

template <int CMAX>
__global__ __launch_bounds__(64 * Z9Cfg<CMAX>::NW) void k_z9_parse(EncArgs A) {
    constexpr int NW = Z9Cfg<CMAX>::NW;
    __shared__ Z9Smem<CMAX> S;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? A.clen[k] : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
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
    z9_sort(S, n - 2, wave, lane);
    for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX; i += 64u * NW) S.seg[i] = 0;
    __syncthreads();
    z9_walkers(S, n, wave, lane);
    __syncthreads();
    // the path from 0, its segments and zlib's block starts
    if (threadIdx.x == 0) {
        uint64_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
        uint64_t* rec = R + 1 + Z_NBLK;
        uint32_t q = 0, i = 0, sym = 0, nb = Z_BLKSYM, nblk = 1;
        R[1] = 0;
        while (q < n) {
            const uint32_t x = S.seg[q];
            if (!(x >> 31)) { i = 0; nblk = 0; break; }   // (cannot happen: the path is complete)
            const uint32_t c = x & 0xFFFFu, L = (x >> 16) & 0x1FFu;
            const uint32_t d = L ? S.sd[q] : 0u;
            rec[i++] = (uint64_t)(c | L << 16) | (uint64_t)d << 32;
            // a block ends with its 16383rd symbol -- not with the final literal,
            // tallied after deflate_slow's loop without the flush check
            const uint32_t cl = L ? c : c - 1;
            while (sym + cl >= nb && nblk < Z_NBLK) {
                R[1 + nblk++] = q + (nb - sym);
                nb += Z_BLKSYM;
            }
            sym += c;
            if (L) {
                sym++;
                if (sym == nb && nblk < Z_NBLK) {
                    R[1 + nblk++] = q + c + L;
                    nb += Z_BLKSYM;
                }
            }
            q += c + L;
        }
        R[0] = (uint64_t)i | (uint64_t)nblk << 32;
    }
}

// ---------------------------------------------------------------------------
// k_z9_code: trees, _tr_flush_block's choice and the bits

typedef __attribute__((address_space(3))) uint16_t l16;
typedef __attribute__((address_space(3))) uint8_t l8;
typedef __attribute__((address_space(3))) uint32_t l32;

constexpr int LT_N = 2 * 286 + 1, DT_N = 2 * 30 + 1, BT_N = 2 * 19 + 1;

// one tree's arrays: nodes (leaves, then internal), the heap (packed keys
// freq << 16 | depth << 10 | node: zlib's smaller() is the key order), bl_count
struct Z9Tree {
    l16* freq;
    l16* dad;
    l8* len;
    l16* code;
    l32* heap;
    l16* blc;
};

__device__ __forceinline__ uint32_t z_xbits(int kind, int n) {
    if (kind == 0) return n >= 257 ? z_xl[n - 257] : 0u;
    if (kind == 1) return z_xd[n];
    return n == 16 ? 2u : n == 17 ? 3u : n == 18 ? 7u : 0u;
}
__device__ __forceinline__ uint32_t z_slen(int kind, int n) {
    if (kind == 0) return n < 144 ? 8u : n < 256 ? 9u : n < 280 ? 7u : 8u;
    return 5u;
}

__device__ __forceinline__ void z9_down(l32* heap, int heap_len, int k) {
    const uint32_t v = heap[k];
    int j = k << 1;
    while (j <= heap_len) {
        uint32_t hj = heap[j];
        if (j < heap_len) {
            const uint32_t hj1 = heap[j + 1];
            if ((hj1 >> 10) <= (hj >> 10)) { j++; hj = hj1; }
        }
        if ((v >> 10) <= (hj >> 10)) break;
        heap[k] = hj;
        k = j;
        j <<= 1;
    }
    heap[k] = v;
}

// zlib's build_tree + gen_bitlen + gen_codes (oracle/zlib9_model.c build()), on
// the calling lane.  kind 0: literal/length (static lengths 8/9/7/8), 1:
// distance (static 5), 2: bit lengths (no static tree).  Returns max_code.
__device__ int z9_build(Z9Tree t, int elems, int maxlen, int kind, uint32_t& opt, uint32_t& stat) {
    const int HSZ = 2 * elems + 1;
    int heap_len = 0, heap_max = HSZ, max_code = -1;
    for (int n = 0; n < elems; n++) {
        const uint32_t f = t.freq[n];
        if (f) { t.heap[++heap_len] = f << 16 | (uint32_t)n; max_code = n; }
        else t.len[n] = 0;
    }
    while (heap_len < 2) {
        const int node = max_code < 2 ? ++max_code : 0;
        t.heap[++heap_len] = 1u << 16 | (uint32_t)node;
        t.freq[node] = 1;
        opt--;
        if (kind < 2) stat -= z_slen(kind, node);
    }
    for (int n = heap_len / 2; n >= 1; n--) z9_down(t.heap, heap_len, n);
    int node = elems;
    do {
        const uint32_t hn = t.heap[1];
        t.heap[1] = t.heap[heap_len--];
        z9_down(t.heap, heap_len, 1);
        const uint32_t hm = t.heap[1];
        t.heap[--heap_max] = hn;
        t.heap[--heap_max] = hm;
        const uint32_t f = (hn >> 16) + (hm >> 16);
        const uint32_t dep = max((hn >> 10) & 63u, (hm >> 10) & 63u) + 1u;
        t.freq[node] = (uint16_t)f;
        t.dad[hn & 1023u] = (uint16_t)node;
        t.dad[hm & 1023u] = (uint16_t)node;
        t.heap[1] = f << 16 | dep << 10 | (uint32_t)node;
        node++;
        z9_down(t.heap, heap_len, 1);
    } while (heap_len >= 2);
    t.heap[--heap_max] = t.heap[1];
    for (int b = 0; b <= 15; b++) t.blc[b] = 0;
    t.len[t.heap[heap_max] & 1023u] = 0;
    int overflow = 0;
    for (int h = heap_max + 1; h < HSZ; h++) {
        const int n = (int)(t.heap[h] & 1023u);
        int b = t.len[t.dad[n]] + 1;
        if (b > maxlen) { b = maxlen; overflow++; }
        t.len[n] = (uint8_t)b;
        if (n > max_code) continue;
        t.blc[b]++;
        const uint32_t xb = z_xbits(kind, n), f = t.freq[n];
        opt += f * ((uint32_t)b + xb);
        if (kind < 2) stat += f * (z_slen(kind, n) + xb);
    }
    if (overflow) {
        do {
            int b = maxlen - 1;
            while (t.blc[b] == 0) b--;
            t.blc[b]--;
            t.blc[b + 1] += 2;
            t.blc[maxlen]--;
            overflow -= 2;
        } while (overflow > 0);
        int h = HSZ;
        for (int b = maxlen; b != 0; b--) {
            int k = t.blc[b];
            while (k) {
                const int m = (int)(t.heap[--h] & 1023u);
                if (m > max_code) continue;
                if (t.len[m] != b) {
                    opt += (uint32_t)((b - (int)t.len[m]) * (int)t.freq[m]);
                    t.len[m] = (uint8_t)b;
                }
                k--;
            }
        }
    }
    // gen_codes
    uint32_t next[16], code = 0;
    next[0] = 0;
    for (int b = 1; b <= 15; b++) { code = (code + t.blc[b - 1]) << 1; next[b] = code; }
    for (int n = 0; n <= max_code; n++) {
        const int l = t.len[n];
        if (l) {
            uint32_t c = 0;
            switch (l) {   // next[] indexed by a divergent value stays in registers
#define Z_NX(B) case B: c = next[B]++; break;
                Z_NX(1) Z_NX(2) Z_NX(3) Z_NX(4) Z_NX(5) Z_NX(6) Z_NX(7) Z_NX(8)
                Z_NX(9) Z_NX(10) Z_NX(11) Z_NX(12) Z_NX(13) Z_NX(14) Z_NX(15)
#undef Z_NX
                default: break;
            }
            t.code[n] = (uint16_t)(__builtin_bitreverse32(c) >> (32 - l));
        }
    }
    return max_code;
}

__device__ __forceinline__ void z_put(l32* w, uint32_t b, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t i = b >> 5, o = b & 31;
    w[i] |= v << o;
    if (o + nb > 32) w[i + 1] |= v >> (32 - o);
}
__device__ __forceinline__ void z_put_atomic(uint32_t* w, uint32_t b, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t i = b >> 5, o = b & 31;
    atomicOr(&w[i], v << o);
    if (o + nb > 32) atomicOr(&w[i + 1], v >> (32 - o));
}


// scan_tree (send = false: counts into cnt[0..19)) / send_tree (send = true:
// the bits at bp with the bit-length codes bcode / blen) over len[0..max_code]
__device__ void z9_rle(const l8* len, int max_code, bool send, l16* cnt, const l16* bcode, const l8* blen,
                       l32* w, uint32_t& bp) {
    int prevlen = -1, nextlen = len[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = n + 1 <= max_code ? (int)len[n + 1] : 0xFFFF;   // zlib's guard entry
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            if (!send) cnt[curlen] += (uint16_t)count;
            else {
                const uint32_t c = bcode[curlen], l = blen[curlen];
                do { z_put(w, bp, c, l); bp += l; } while (--count);
            }
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                if (!send) cnt[curlen]++;
                else { z_put(w, bp, bcode[curlen], blen[curlen]); bp += blen[curlen]; count--; }
            }
            if (!send) cnt[16]++;
            else {
                z_put(w, bp, bcode[16], blen[16]); bp += blen[16];
                z_put(w, bp, (uint32_t)count - 3, 2); bp += 2;
            }
        } else if (count <= 10) {
            if (!send) cnt[17]++;
            else {
                z_put(w, bp, bcode[17], blen[17]); bp += blen[17];
                z_put(w, bp, (uint32_t)count - 3, 3); bp += 3;
            }
        } else {
            if (!send) cnt[18]++;
            else {
                z_put(w, bp, bcode[18], blen[18]); bp += blen[18];
                z_put(w, bp, (uint32_t)count - 11, 7); bp += 7;
            }
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

template <int CMAX>
struct Z9CSmem {
    static constexpr int WORDS = (CMAX + 5 * (int)Z_NBLK + 64) / 4 + 4;
    alignas(16) uint32_t bits[WORDS];        // the deflate body, LSB first
    uint32_t mstart[CMAX / 32 + 2];          // match starts (bitmask by position)
    uint32_t lf32[288], df32[32];            // block frequencies (counted with atomics)
    uint32_t ecl[288], ecd[32];              // emission codes: code | len << 16
    uint32_t heapL[LT_N + 1], heapD[DT_N + 1];
    uint16_t lfreq[LT_N + 1], ldad[LT_N + 1], lcode[288];
    uint16_t dfreq[DT_N + 1], ddad[DT_N + 1], dcode[32];
    uint16_t bfreq[BT_N + 1], bdad[BT_N + 1], bcode[20];
    uint16_t blcL[16], blcD[16], blcB[16];
    uint16_t cnt19[2][20];
    uint8_t llen[LT_N + 1], dlen[DT_N + 1], blen[BT_N + 1];
    uint32_t misc[16];
};

template <int CMAX>
__global__ __launch_bounds__(64) void k_z9_code(EncArgs A) {
    __shared__ Z9CSmem<CMAX> S;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? A.clen[k] : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
    const uint8_t* src = A.in + pos0;
    const uint64_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
    const uint64_t hdr = R[0];
    const uint32_t nrec = (uint32_t)hdr, nblk = (uint32_t)(hdr >> 32);
    const uint64_t* rec = R + 1 + Z_NBLK;
    const uint64_t below = (1ull << lane) - 1ull;
    l32* W = (l32*)S.bits;
    const Z9Tree LT{(l16*)S.lfreq, (l16*)S.ldad, (l8*)S.llen, (l16*)S.lcode, (l32*)S.heapL, (l16*)S.blcL};
    const Z9Tree DT{(l16*)S.dfreq, (l16*)S.ddad, (l8*)S.dlen, (l16*)S.dcode, (l32*)S.heapD, (l16*)S.blcD};
    const Z9Tree BT{(l16*)S.bfreq, (l16*)S.bdad, (l8*)S.blen, (l16*)S.bcode, (l32*)S.heapD, (l16*)S.blcB};

    // ---- match starts from the segments ----
    for (uint32_t i = lane; i < (uint32_t)CMAX / 32 + 2; i += 64) S.mstart[i] = 0;
    for (uint32_t i = lane; i < (uint32_t)Z9CSmem<CMAX>::WORDS; i += 64) S.bits[i] = 0;
    wave_sync();
    {
        uint32_t carry = 0;
        for (uint32_t e0 = 0; e0 < nrec; e0 += 64) {
            const uint32_t e = e0 + lane;
            const uint64_t x = e < nrec ? rec[e] : 0ull;
            const uint32_t c = (uint32_t)x & 0xFFFFu, L = (uint32_t)(x >> 16) & 0x1FFu;
            const uint32_t span = c + L, incl = wave_incl_sum(span);
            const uint32_t p = carry + incl - span + c;
            if (e < nrec && L) atomicOr(&S.mstart[p >> 5], 1u << (p & 31));
            carry += readlane(incl, 63);
        }
    }
    wave_sync();

    // one position-major pass over [bs, be): emit = false counts the block's
    // symbols, emit = true writes them at bit bp (returns the bits written)
    auto pass = [&](uint32_t bs, uint32_t be, uint32_t rank0, bool emit, uint32_t bp) -> uint32_t {
        uint32_t rank = rank0, out = 0;
        int carry = (int)bs;
#pragma unroll 1
        for (uint32_t p0 = bs & ~63u; p0 < be; p0 += 64) {
            const uint32_t pos = p0 + lane;
            const bool in = pos >= bs && pos < be;
            const bool ms = in && ((S.mstart[pos >> 5] >> (pos & 31)) & 1u);
            const uint64_t bm = __ballot(ms);
            uint32_t L = 0, d = 0;
            if (ms) {
                const uint64_t x = rec[rank + (uint32_t)__popcll(bm & below)];
                L = (uint32_t)(x >> 16) & 0x1FFu;
                d = (uint32_t)(x >> 32);
            }
            const int e = ms ? (int)(pos + L) : 0;
            const int E = max(carry, wave_incl_max_i32(e));
            carry = max(carry, wave_max_i32(e));
            rank += (uint32_t)__popcll(bm);
            const bool lit = in && !ms && E <= (int)pos;
            const uint32_t c = lit ? src[pos] : 0u;
            const uint32_t lc = ms ? z_lcode(L) : 0u, dc = ms ? z_dcode(d) : 0u;
            if (!emit) {
                if (lit) atomicAdd(&S.lf32[c], 1u);
                if (ms) {
                    atomicAdd(&S.lf32[257 + lc], 1u);
                    atomicAdd(&S.df32[dc], 1u);
                }
            } else {
                uint32_t cost = 0, e1 = 0, e2 = 0, v1 = 0, v2 = 0;
                if (lit) {
                    e1 = S.ecl[c] >> 16;
                    v1 = S.ecl[c] & 0xFFFFu;
                } else if (ms) {
                    const uint32_t a = S.ecl[257 + lc], b = S.ecd[dc];
                    const uint32_t la = a >> 16, lb = b >> 16;
                    e1 = la + z_xl[lc];
                    v1 = (a & 0xFFFFu) | (L - 3 - z_lbase[lc]) << la;
                    e2 = lb + z_xd[dc];
                    v2 = (b & 0xFFFFu) | (d - 1 - z_dbase[dc]) << lb;
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
        const uint32_t bs = (uint32_t)R[1 + b];
        const uint32_t be = b + 1 < nblk ? (uint32_t)R[2 + b] : n;
        const uint32_t last = b + 1 == nblk ? 1u : 0u;
        // match starts before bs
        uint32_t rank0 = 0;
        for (uint32_t i = lane; i < (bs >> 5); i += 64) rank0 += (uint32_t)__popc(S.mstart[i]);
        if (lane == 0 && (bs & 31)) rank0 += (uint32_t)__popc(S.mstart[bs >> 5] & ((1u << (bs & 31)) - 1u));
        rank0 = wave_sum_u32(rank0);
        for (uint32_t i = lane; i < 288; i += 64) S.lf32[i] = 0;
        if (lane < 32) S.df32[lane] = 0;
        if (lane < 40) S.cnt19[lane / 20][lane % 20] = 0;
        wave_sync();
        pass(bs, be, rank0, false, 0);
        wave_sync();
        for (uint32_t i = lane; i < 286; i += 64) S.lfreq[i] = (uint16_t)(S.lf32[i] + (i == 256 ? 1u : 0u));
        if (lane < 30) S.dfreq[lane] = (uint16_t)S.df32[lane];
        if (lane < 19) S.bfreq[lane] = 0;
        wave_sync();
        // ---- the trees (build_tree x 2 at once, scan_tree x 2, build_bl_tree) ----
        if (lane < 2) {
            uint32_t opt = 0, stat = 0;
            const int mc = z9_build(lane ? DT : LT, lane ? 30 : 286, 15, (int)lane, opt, stat);
            uint32_t dummy = 0;
            z9_rle(lane ? (const l8*)S.dlen : (const l8*)S.llen, mc, false, (l16*)S.cnt19[lane],
                   (const l16*)S.bcode, (const l8*)S.blen, W, dummy);
            S.misc[lane] = (uint32_t)mc;
            S.misc[2 + lane] = opt;
            S.misc[4 + lane] = stat;
        }
        wave_sync();
        if (lane == 0) {
            for (int i = 0; i < 19; i++) S.bfreq[i] = (uint16_t)(S.cnt19[0][i] + S.cnt19[1][i]);
            uint32_t opt = 0, stat = 0;
            (void)z9_build(BT, 19, 7, 2, opt, stat);
            int maxbl;
            for (maxbl = 18; maxbl >= 3; maxbl--) if (S.blen[z_blord[maxbl]] != 0) break;
            opt += S.misc[2] + S.misc[3] + 3u * (uint32_t)(maxbl + 1) + 5 + 5 + 4;
            const uint32_t stl = S.misc[4] + S.misc[5];
            uint32_t opt_lenb = (opt + 3 + 7) >> 3;
            const uint32_t static_lenb = (stl + 3 + 7) >> 3;
            if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
            const uint32_t stored_len = be - bs;
            const uint32_t kind = stored_len + 4 <= opt_lenb ? 0u : (static_lenb == opt_lenb ? 1u : 2u);
            S.misc[6] = kind;
            S.misc[7] = (uint32_t)maxbl;
            S.misc[8] = kind == 2 ? opt : stl;   // the block's bits after its 3 header bits
        }
        wave_sync();
        const uint32_t kind = S.misc[6];
        if (nblk == 1) {
            // the exact length before any bit is written
            const uint32_t bits = kind == 0 ? ((3 + 7) & ~7u) + 32 + 8 * n : 3 + S.misc[8];
            const uint32_t total = 2 + (bits + 7) / 8 + 4;
            if (total + 18 >= T) return;
        }
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
        if (lane == 0) {
            z_put(W, bp, kind << 1 | last, 3);
            uint32_t p = bp + 3;
            if (kind == 2) {
                const int lmax = (int)S.misc[0], dmax = (int)S.misc[1], maxbl = (int)S.misc[7];
                z_put(W, p, (uint32_t)lmax + 1 - 257, 5); p += 5;
                z_put(W, p, (uint32_t)dmax, 5); p += 5;
                z_put(W, p, (uint32_t)maxbl + 1 - 4, 4); p += 4;
                for (int r = 0; r <= maxbl; r++) { z_put(W, p, S.blen[z_blord[r]], 3); p += 3; }
                z9_rle((const l8*)S.llen, lmax, true, (l16*)S.cnt19[0], (const l16*)S.bcode, (const l8*)S.blen, W, p);
                z9_rle((const l8*)S.dlen, dmax, true, (l16*)S.cnt19[0], (const l16*)S.bcode, (const l8*)S.blen, W, p);
            }
            S.misc[9] = p;
        }
        wave_sync();
        bp = S.misc[9];
        bp += pass(bs, be, rank0, true, bp);
        wave_sync();
        if (lane == 0) z_put(W, bp, S.ecl[256] & 0xFFFFu, S.ecl[256] >> 16);
        bp += S.ecl[256] >> 16;
        wave_sync();
    }
    const uint32_t body = (bp + 7) >> 3;
    const uint32_t total = 2 + body + 4;
    if (total + 18 >= T) return;
    // ---- Adler-32 of the chunk ----
    uint32_t adler;
    {
        uint64_t asum = 0, bsum = 0;
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t c = src[i];
            asum += c;
            bsum += (uint64_t)(n - i) * c;
        }
        asum = wave_sum<uint64_t>(asum);
        bsum = wave_sum<uint64_t>(bsum);
        adler = (uint32_t)(((n + bsum) % 65521) << 16 | ((1 + asum) % 65521));
    }
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
}

template <int CMAX>
hipError_t launch_z9_t(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_z9_parse<CMAX>, dim3(a.n_chunks), dim3(64 * Z9Cfg<CMAX>::NW), 0, s, a);
    hipLaunchKernelGGL(k_z9_code<CMAX>, dim3(a.n_chunks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace

uint32_t z9_cmax(uint32_t chunk) {
    return chunk <= 1024 ? 1024u : chunk <= 2048 ? 2048u : chunk <= 4096 ? 4096u : 0u;
}

size_t z9_rec_words(uint32_t cmax) {
    switch (cmax) {
        case 1024: return Z9Rec<1024>::STRIDE;
        case 2048: return Z9Rec<2048>::STRIDE;
        case 4096: return Z9Rec<4096>::STRIDE;
        default: return 0;
    }
}

hipError_t launch_zlib9(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    switch (z9_cmax(a.chunk_size)) {
        case 1024: return launch_z9_t<1024>(a, s);
        case 2048: return launch_z9_t<2048>(a, s);
        case 4096: return launch_z9_t<4096>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ambc
