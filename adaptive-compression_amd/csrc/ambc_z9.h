// ambc_z9.h -- device pieces shared by the zlib-9 encoders (ambc_zlib9.hip: chunks
// <= 8192 with the walkers' tables in LDS; ambc_zlib9_big.hip: 16 / 32 / 64 KiB with
// them in device scratch): zlib 1.2.11's constants and codes, the chunk gate, the
// per-chunk record layout, build_tree / gen_bitlen / gen_codes for a wave, the
// code-length RLE and the bit writers.
#pragma once
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
constexpr uint32_t Z_NBLK = 1;               // chunks <= 4096 bytes: < 16383 symbols, one block

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
// the same hash to BITS bits (the small-chunk parse's bucket count)
template <uint32_t BITS>
__device__ __forceinline__ uint32_t z_bucket_b(uint32_t h15) { return (h15 * 2654435761u) >> (32 - BITS); }

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

// per chunk (u32 words): [0] = matches, [1] = blocks; per block (BLK, 4 words):
// first position, end position, matches before it, flags (Z9B_NOSTORE); the
// match-start bitmask (CMAX / 32 words); the matches in order, L | dist << 16;
// per block its symbol counts (FREQ) and zlib's heap merges (MERGE).  zlib ends a
// block with its 16383rd symbol: chunks <= 16382 bytes hold one block, 64 KiB
// at most five.
constexpr uint32_t Z9B_NOSTORE = 1;   // flushed after the window slid, begun before 32768: no stored block
// record word 1 of a chunk <= 8192 (one block): k_z9_parse found that id 5 cannot
// win (no 3-byte string occurs twice, and the all-literal block's lower bound
// loses); k_z9_heap / k_z9_code skip the chunk
constexpr uint32_t Z9_LOSES = 0xFFFFFFFFu;
template <int CMAX> struct Z9Rec {
    static constexpr uint32_t NBLK = (uint32_t)CMAX / 16383u + 1u;
    static constexpr uint32_t BLK = 2, MASK = BLK + 4 * NBLK, MATCH = MASK + CMAX / 32;
    static constexpr uint32_t FREQ = MATCH + CMAX / 3 + 4;   // 286 + 30 u16 symbol counts (EOB not counted)
    static constexpr uint32_t MERGE = FREQ + 158 * NBLK;      // zlib's heap merges: lit 285 + dist 29, n | m << 16
    static constexpr uint32_t STRIDE = MERGE + 316 * NBLK;
};

__device__ __forceinline__ uint32_t grp_max8(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, true));  // row_half_mirror
    return x;
}
__device__ __forceinline__ uint32_t grp8(uint64_t m, uint32_t g) { return (uint32_t)(m >> (8 * g)) & 0xFFu; }
// the same for lane groups of G = 1, 2, 4 or 8 lanes
template <int G>
__device__ __forceinline__ uint32_t grp_max(uint32_t x) {
    if constexpr (G >= 2) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, true));
    if constexpr (G >= 4) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, true));
    if constexpr (G >= 8) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, true));
    return x;
}
template <int G>
__device__ __forceinline__ uint32_t grp_bits(uint64_t m, uint32_t g) {
    return (uint32_t)(m >> (G * g)) & ((1u << G) - 1u);
}

// ---------------------------------------------------------------------------
// k_z9_heap: zlib's build_tree heap for the literal/length and distance trees,
// one chunk per LANE (64 chunks per wave), the heaps in LDS interleaved by lane
// ([index][lane]: conflict-free).  The heap walk is inherently serial per tree;
// across chunks it is plain SIMT.  Output: the merge sequence (the two nodes
// each step pops) -- everything gen_bitlen needs (k_z9_code rebuilds the
// parent links and the heap_max order from it).
constexpr uint32_t ZH_N = 290;
// chunks (lanes) per wave: the heaps of 64 chunks fill 74 KB of LDS, two waves
// per CU; fewer lanes per wave keep about as many heaps resident in more waves,
// which hide each other's dependent LDS reads ({1,3,4,5z} same-box: 64 -> 16 ->
// 8 lanes 23.9 -> 24.4 -> 24.9 GB/s, profiles/r6_z9_heap_lanes_ab/)
#ifndef AMBC_ZH_L
#define AMBC_ZH_L 8
#endif
constexpr uint32_t ZH_L = AMBC_ZH_L;
__device__ __forceinline__ void zh_down(uint32_t* H, uint32_t lane, uint32_t heap_len, uint32_t k) {
    const uint32_t v = H[k * ZH_L + lane], kv = v >> 10;
    uint32_t j = k << 1;
    while (j <= heap_len) {
        uint32_t hj = H[j * ZH_L + lane];
        if (j < heap_len) {
            const uint32_t hj1 = H[(j + 1) * ZH_L + lane];
            if ((hj1 >> 10) <= (hj >> 10)) { j++; hj = hj1; }
        }
        if (kv <= (hj >> 10)) break;
        H[k * ZH_L + lane] = hj;
        k = j;
        j <<= 1;
    }
    H[k * ZH_L + lane] = v;
}

template <int CMAX>
__global__ __launch_bounds__(64) void k_z9_heap(EncArgs A) {
    __shared__ uint32_t H[ZH_N * ZH_L];
    constexpr uint32_t NB = Z9Rec<CMAX>::NBLK;   // one lane per (chunk, block)
    const uint32_t lane = threadIdx.x;
    if (lane >= ZH_L) return;
    const uint32_t item = blockIdx.x * ZH_L + lane;
    const uint32_t k = item / NB, blk = item % NB;
    if (k >= A.n_chunks) return;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
    uint32_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
    if (R[1] == Z9_LOSES) return;
    if (NB > 1 && blk >= R[1]) return;
    const uint16_t* F = reinterpret_cast<const uint16_t*>(R + Z9Rec<CMAX>::FREQ + 158 * blk);
    uint32_t* MG = R + Z9Rec<CMAX>::MERGE + 316 * blk;
#pragma unroll 1
    for (int tree = 0; tree < 2; tree++) {
        const uint32_t elems = tree ? 30u : 286u, fb = tree ? 286u : 0u, mb = tree ? 285u : 0u;
        uint32_t heap_len = 0;
        int max_code = -1;
#pragma unroll 8
        for (uint32_t s = 0; s < elems; s++) {
            const uint32_t f = (uint32_t)F[fb + s] + (tree == 0 && s == 256 ? 1u : 0u);   // + the end of block
            if (f) {
                H[(++heap_len) * ZH_L + lane] = f << 16 | s;
                max_code = (int)s;
            }
        }
        while (heap_len < 2) {   // at least two codes
            const int node = max_code < 2 ? ++max_code : 0;
            H[(++heap_len) * ZH_L + lane] = 1u << 16 | (uint32_t)node;
        }
        for (uint32_t q = heap_len / 2; q >= 1; q--) zh_down(H, lane, heap_len, q);
        uint32_t node = elems, i = 0;
        do {
            const uint32_t hn = H[ZH_L + lane];
            H[ZH_L + lane] = H[heap_len * ZH_L + lane];
            heap_len--;
            zh_down(H, lane, heap_len, 1);
            const uint32_t hm = H[ZH_L + lane];
            MG[mb + i++] = (hn & 1023u) | (hm & 1023u) << 16;
            const uint32_t f = (hn >> 16) + (hm >> 16);
            const uint32_t dep = max((hn >> 10) & 63u, (hm >> 10) & 63u) + 1u;
            H[ZH_L + lane] = f << 16 | dep << 10 | node;
            node++;
            zh_down(H, lane, heap_len, 1);
        } while (heap_len >= 2);
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

// extra bits of length code lc / distance code dc (zlib's extra_lbits / extra_dbits)
__device__ __forceinline__ uint32_t z_xlb(uint32_t lc) { return lc < 8 || lc == 28 ? 0u : (lc >> 2) - 1; }
__device__ __forceinline__ uint32_t z_xdb(uint32_t dc) { return dc < 4 ? 0u : (dc >> 1) - 1; }
__device__ __forceinline__ uint32_t z_xbits(int kind, int n) {
    if (kind == 0) return n >= 257 ? z_xlb((uint32_t)n - 257) : 0u;
    if (kind == 1) return z_xdb((uint32_t)n);
    return n == 16 ? 2u : n == 17 ? 3u : n == 18 ? 7u : 0u;
}
__device__ __forceinline__ uint32_t z_slen(int kind, int n) {
    if (kind == 0) return n < 144 ? 8u : n < 256 ? 9u : n < 280 ? 7u : 8u;
    return 5u;
}

// zlib's heap held in R VGPRs (entry i at lane i & 63 of register i >> 6):
// the heap walk runs on the scalar unit (v_readlane, branch-free selects, a
// compare-and-select write), without an LDS round trip per level
template <int R>
struct VHeap {
    uint32_t h[R];
};
template <int R>
__device__ __forceinline__ uint32_t vh_get(const VHeap<R>& H, uint32_t i) {
    const uint32_t l = i & 63u, r = i >> 6;
    uint32_t x = readlane(H.h[0], l);
#pragma unroll
    for (int q = 1; q < R; q++) {
        const uint32_t y = readlane(H.h[q], l);
        x = r >= (uint32_t)q ? y : x;
    }
    return x;
}
template <int R>
__device__ __forceinline__ void vh_set(VHeap<R>& H, uint32_t i, uint32_t v) {
    const uint32_t l = i & 63u, r = i >> 6;
    const bool me = __lane_id() == l;
#pragma unroll
    for (int q = 0; q < R; q++) H.h[q] = me && r == (uint32_t)q ? v : H.h[q];
}
// pqdownheap: smaller() is the order of the packed keys' freq | depth bits
template <int R>
__device__ __forceinline__ void vh_down(VHeap<R>& H, uint32_t heap_len, uint32_t k) {
    const uint32_t v = vh_get(H, k), kv = v >> 10;
    uint32_t j = k << 1;
    while (j <= heap_len) {
        uint32_t hj = vh_get(H, j);
        if (j < heap_len) {
            const uint32_t hj1 = vh_get(H, j + 1);
            if ((hj1 >> 10) <= (hj >> 10)) { j++; hj = hj1; }
        }
        if (kv <= (hj >> 10)) break;
        vh_set(H, k, hj);
        k = j;
        j <<= 1;
    }
    vh_set(H, k, v);
}

// zlib's build_tree + gen_bitlen + gen_codes with the whole wave (uniform
// control flow; oracle/zlib9_model.c build() is the serial statement).  The
// heap runs as above; gen_bitlen's depths come from pointer jumping over the
// parent links (len = min(depth, maxlen), overflow = nodes deeper than maxlen,
// exactly gen_bitlen's clamped recursion), its rare overflow repair runs on
// lane 0; gen_codes ranks equal lengths by ballots.  pjd / pja: scratch of
// 2 * elems + 1 entries; blc32: 16 u32.  Returns max_code.
template <int R, bool MERGED>
__device__ __forceinline__ int z9_build_w(Z9Tree t, l16* pjd, l16* pja, l32* blc32, l32* misc, int elems, int maxlen, int kind,
                          uint32_t& opt, uint32_t& stat, uint32_t lane, const uint32_t* MG = nullptr) {
    const uint32_t HSZ = 2u * (uint32_t)elems + 1u;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t cnt = 0;
    int max_code = -1;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t n = 64u * j + lane;
        const uint32_t f = n < (uint32_t)elems ? (uint32_t)t.freq[n] : 0u;
        const uint64_t m = __ballot(f != 0);
        if (f) t.heap[1 + cnt + (uint32_t)__popcll(m & below)] = f << 16 | n;
        else if (n < (uint32_t)elems) t.len[n] = 0;
        if (m) max_code = 64 * j + 63 - __clzll((long long)m);
        cnt += (uint32_t)__popcll(m);
    }
    if (lane < 16) blc32[lane] = 0;
    wave_sync();
    uint32_t node, root;
    if (MERGED) {
        // k_z9_heap's merge sequence: the heap_max order and the parent links
        uint32_t heap_len = cnt;
        while (heap_len < 2) {   // at least two codes (k_z9_heap forced the same nodes)
            const int nd = max_code < 2 ? ++max_code : 0;
            heap_len++;
            if (lane == 0) t.freq[nd] = 1;
            opt--;
            if (kind < 2) stat -= z_slen(kind, nd);
        }
        const uint32_t nm = heap_len - 1;
        for (uint32_t i = lane; i < nm; i += 64) {
            const uint32_t x = MG[i], a = x & 1023u, b = x >> 16;
            t.heap[HSZ - 1 - 2 * i] = a;
            t.heap[HSZ - 2 - 2 * i] = b;
            t.dad[a] = (uint16_t)(elems + i);
            t.dad[b] = (uint16_t)(elems + i);
        }
        node = (uint32_t)elems + nm;
        root = node - 1;
        if (lane == 0) t.heap[HSZ - 1 - 2 * nm] = root;
        wave_sync();
    } else {
        VHeap<R> H;
    #pragma unroll
        for (int j = 0; j < R; j++) H.h[j] = 64u * j + lane <= cnt ? (uint32_t)t.heap[64 * j + lane] : 0u;
        uint32_t heap_len = cnt;
        while (heap_len < 2) {   // at least two codes
            const int nd = max_code < 2 ? ++max_code : 0;
            vh_set(H, ++heap_len, 1u << 16 | (uint32_t)nd);
            if (lane == 0) t.freq[nd] = 1;
            opt--;
            if (kind < 2) stat -= z_slen(kind, nd);
        }
        for (uint32_t k = heap_len / 2; k >= 1; k--) vh_down(H, heap_len, k);
        node = (uint32_t)elems;
        uint32_t heap_max = HSZ;
        do {
            const uint32_t hn = vh_get(H, 1);
            vh_set(H, 1, vh_get(H, heap_len));
            heap_len--;
            vh_down(H, heap_len, 1);
            const uint32_t hm = vh_get(H, 1);
            heap_max -= 2;
            if (lane == 0) {
                t.heap[heap_max + 1] = hn & 1023u;
                t.heap[heap_max] = hm & 1023u;
                t.dad[hn & 1023u] = (uint16_t)node;
                t.dad[hm & 1023u] = (uint16_t)node;
            }
            const uint32_t f = (hn >> 16) + (hm >> 16);
            const uint32_t dep = max((hn >> 10) & 63u, (hm >> 10) & 63u) + 1u;
            vh_set(H, 1, f << 16 | dep << 10 | node);
            node++;
            vh_down(H, heap_len, 1);
        } while (heap_len >= 2);
        root = vh_get(H, 1) & 1023u;
        heap_max--;
        if (lane == 0) t.heap[heap_max] = root;
        wave_sync();
    }
    // ---- depths: pointer jumping over dad[] (nodes 0 .. node-1) ----
    const uint32_t nn = node;
    uint32_t d[9], a[9];
    bool leaf_in[5];
#pragma unroll
    for (int j = 0; j < 9; j++) {
        const uint32_t x = 64u * j + lane;
        bool in = false;
        if (x < (uint32_t)elems) {
            in = (int)x <= max_code && t.freq[x] != 0;
            if (j < 5) leaf_in[j] = in;
        } else {
            in = x < nn;
        }
        const bool nr = in && x != root;
        d[j] = nr ? 1u : 0u;
        a[j] = nr ? (uint32_t)t.dad[x] : x;
        if (x < HSZ) { pjd[x] = (uint16_t)d[j]; pja[x] = (uint16_t)a[j]; }
    }
    wave_sync();
#pragma unroll 1
    for (int it = 0; it < 10; it++) {
        uint32_t nd[9], na[9];
#pragma unroll
        for (int j = 0; j < 9; j++) {
            const uint32_t x = 64u * j + lane;
            nd[j] = x < nn ? d[j] + pjd[a[j]] : d[j];
            na[j] = x < nn ? (uint32_t)pja[a[j]] : a[j];
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < 9; j++) {
            const uint32_t x = 64u * j + lane;
            d[j] = nd[j];
            a[j] = na[j];
            if (x < nn) { pjd[x] = (uint16_t)d[j]; pja[x] = (uint16_t)a[j]; }
        }
        wave_sync();
    }
    // ---- lengths, bl_count, opt_len / static_len, overflow ----
    uint32_t ovf = 0, po = 0, ps = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
        const uint32_t x = 64u * j + lane;
        const bool in = x < (uint32_t)elems ? (j < 5 && leaf_in[j]) : x < nn;
        if (in && x != root && d[j] > (uint32_t)maxlen) ovf++;
        if (j < 5 && x < (uint32_t)elems && leaf_in[j]) {
            const uint32_t b = min(d[j], (uint32_t)maxlen);
            t.len[x] = (uint8_t)b;
            atomicAdd((uint32_t*)&blc32[b], 1u);
            const uint32_t f = t.freq[x], xb = z_xbits(kind, (int)x);
            po += f * (b + xb);
            if (kind < 2) ps += f * (z_slen(kind, (int)x) + xb);
        }
    }
    ovf = wave_sum_u32(ovf);
    opt += wave_sum_u32(po);
    stat += wave_sum_u32(ps);
    wave_sync();
    if (lane < 16) t.blc[lane] = (uint16_t)blc32[lane];
    wave_sync();
    if (ovf) {
        // gen_bitlen's repair, serially on lane 0 (zlib's order over the heap's
        // removed nodes, from the least frequent)
        if (lane == 0) {
            int overflow = (int)ovf;
            uint32_t od = 0;
            do {
                int b = maxlen - 1;
                while (t.blc[b] == 0) b--;
                t.blc[b]--;
                t.blc[b + 1] += 2;
                t.blc[maxlen]--;
                overflow -= 2;
            } while (overflow > 0);
            int h = (int)HSZ;
            for (int b = maxlen; b != 0; b--) {
                int k = t.blc[b];
                while (k) {
                    const int m = (int)(t.heap[--h] & 1023u);
                    if (m > max_code) continue;
                    if (t.len[m] != b) {
                        od += (uint32_t)((b - (int)t.len[m]) * (int)t.freq[m]);
                        t.len[m] = (uint8_t)b;
                    }
                    k--;
                }
            }
            misc[0] = od;
        }
        wave_sync();
        opt += misc[0];
    }
    // ---- gen_codes: next_code per length, ranks among equal lengths ----
    uint32_t nxt[16];
    {
        uint32_t code = 0;
        nxt[0] = 0;
#pragma unroll
        for (int b = 1; b <= 15; b++) { code = (code + t.blc[b - 1]) << 1; nxt[b] = code; }
    }
    uint32_t ln[5], cd[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t x = 64u * j + lane;
        ln[j] = (int)x <= max_code ? (uint32_t)t.len[x] : 0u;
        cd[j] = 0;
    }
#pragma unroll
    for (int b = 1; b <= 15; b++) {
        uint32_t run = nxt[b];
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const uint64_t m = __ballot(ln[j] == (uint32_t)b);
            if (ln[j] == (uint32_t)b) cd[j] = run + (uint32_t)__popcll(m & below);
            run += (uint32_t)__popcll(m);
        }
    }
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t x = 64u * j + lane;
        if (ln[j]) t.code[x] = (uint16_t)(__builtin_bitreverse32(cd[j]) >> (32 - ln[j]));
    }
    wave_sync();
    return max_code;
}

// the bit stream on the scalar unit: a 64-bit accumulator, whole words stored
// by lane 0 (no read-modify-write); the stream starts word-aligned
struct SBits {
    uint64_t acc;
    uint32_t n, w;
};
__device__ __forceinline__ void sb_put(SBits& b, l32* words, uint32_t v, uint32_t nb, uint32_t lane,
                                       uint32_t wm = ~0u) {
    b.acc |= (uint64_t)v << b.n;
    b.n += nb;
    if (b.n >= 32) {
        if (lane == 0) words[b.w & wm] = (uint32_t)b.acc;
        b.w++;
        b.acc >>= 32;
        b.n -= 32;
    }
}

// bit b of the stream is bit b & 31 of word (b >> 5) & wm (wm: a ring of words)
__device__ __forceinline__ void z_put(l32* w, uint32_t b, uint32_t v, uint32_t nb, uint32_t wm = ~0u) {
    if (!nb) return;
    const uint32_t i = b >> 5, o = b & 31;
    w[i & wm] |= v << o;
    if (o + nb > 32) w[(i + 1) & wm] |= v >> (32 - o);
}
__device__ __forceinline__ void z_put_atomic(uint32_t* w, uint32_t b, uint32_t v, uint32_t nb, uint32_t wm = ~0u) {
    if (!nb) return;
    const uint32_t i = b >> 5, o = b & 31;
    atomicOr(&w[i & wm], v << o);
    if (o + nb > 32) atomicOr(&w[(i + 1) & wm], v >> (32 - o));
}

// scan_tree / send_tree (the code-length RLE) one lane per maximal run of
// equal lengths.  zlib's loop cuts a run of value v and length r into chunks:
// v != 0: the first chunk takes min(r, 7) (below 4: v raw each; else v once and
// 16 for the rest), later chunks 6 each as 16 (a tail below 3 goes raw); v == 0:
// chunks of 138 as 18, the tail as 17 (3..10), 18 (11+) or raw (< 3).  A run
// start resets the chunk limits exactly as zlib's transition does (the previous
// value differs).  send = false: the symbol counts into cnt (u32); send = true:
// the bits from bit bp (codes bcl: lane i = code | len << 16 of symbol i).
// Returns the bits of the send.
template <int R>
__device__ __forceinline__ uint32_t z9_rle_par(const VHeap<R>& L, int max_code, bool send, l32* cnt, uint32_t bcl,
                                               uint32_t* words, uint32_t bp, uint32_t lane, uint32_t wm = ~0u) {
    const uint32_t N = (uint32_t)(max_code + 1);
    uint64_t st[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
        const uint32_t e = 64u * j + lane;
        uint32_t prev = AMBC_DPP(0xFFFFu, L.h[j], 0x138, 0xF, 0xF, false);   // wave_shr:1
        if (lane == 0) prev = j ? readlane(L.h[j > 0 ? j - 1 : 0], 63) : 0xFFFFu;
        st[j] = __ballot(e < N && L.h[j] != prev);
    }
    const uint32_t c16 = readlane(bcl, 16), c17 = readlane(bcl, 17), c18 = readlane(bcl, 18);
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < R; j++) {
        const uint32_t e = 64u * j + lane;
        const bool run = (st[j] >> lane) & 1u;
        const uint32_t v = L.h[j];
        uint32_t end = N;
        {
            const uint64_t above = lane < 63 ? st[j] >> (lane + 1) : 0ull;
            if (above) end = e + 1 + (uint32_t)__builtin_ctzll(above);
            else {
#pragma unroll
                for (int q = R - 1; q > j; q--)
                    if (st[q]) end = 64u * q + (uint32_t)__builtin_ctzll(st[q]);
            }
        }
        const uint32_t r = run ? end - e : 0u;
        // the run's chunks: rawA raw v, a16 (16 with extra x16a), k full chunks
        // (16 x 3 / 18 x 127), the tail (raw rawC, or one 16 / 17 / 18 with extra xt)
        uint32_t rawA = 0, a16 = 0, x16a = 0, kf = 0, rawC = 0, tsym = 0, xt = 0;
        if (run) {
            if (v != 0) {
                const uint32_t c1 = min(r, 7u);
                if (c1 < 4) rawA = c1;
                else { rawA = 1; a16 = 1; x16a = c1 - 4; }
                const uint32_t r1 = r - c1;
                kf = r1 / 6;
                const uint32_t rem = r1 % 6;
                if (rem >= 3) { tsym = 16; xt = rem - 3; }
                else rawC = rem;
            } else {
                kf = r / 138;
                const uint32_t rem = r % 138;
                if (rem < 3) rawC = rem;
                else if (rem <= 10) { tsym = 17; xt = rem - 3; }
                else { tsym = 18; xt = rem - 11; }
            }
        }
        const uint32_t ksym = v != 0 ? 16u : 18u;
        if (!send) {
            if (run) {
                if (rawA + rawC) atomicAdd((uint32_t*)&cnt[v], rawA + rawC);
                if (a16) atomicAdd((uint32_t*)&cnt[16], 1u);
                if (kf) atomicAdd((uint32_t*)&cnt[ksym], kf);
                if (tsym) atomicAdd((uint32_t*)&cnt[tsym], 1u);
            }
        } else {
            const uint32_t cv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(v, 18u) << 2), (int)bcl);   // v's code
            const uint32_t lv = cv >> 16, l16 = c16 >> 16;
            const uint32_t ck = v != 0 ? c16 : c18, lk = (ck >> 16) + (v != 0 ? 2u : 7u);
            const uint32_t ct = tsym == 16 ? c16 : tsym == 17 ? c17 : c18;
            const uint32_t lt = tsym ? (ct >> 16) + (tsym == 16 ? 2u : tsym == 17 ? 3u : 7u) : 0u;
            const uint32_t bits = run ? (rawA + rawC) * lv + a16 * (l16 + 2) + kf * lk + lt : 0u;
            const uint32_t incl = wave_incl_sum(bits);
            uint32_t b = bp + carry + incl - bits;
            carry += readlane(incl, 63);
            if (run) {
                for (uint32_t i = 0; i < rawA; i++) { z_put_atomic(words, b, cv & 0xFFFFu, lv, wm); b += lv; }
                if (a16) { z_put_atomic(words, b, (c16 & 0xFFFFu) | x16a << l16, l16 + 2, wm); b += l16 + 2; }
                const uint32_t kv = (ck & 0xFFFFu) | (v != 0 ? 3u : 127u) << (ck >> 16);
                for (uint32_t i = 0; i < kf; i++) { z_put_atomic(words, b, kv, lk, wm); b += lk; }
                for (uint32_t i = 0; i < rawC; i++) { z_put_atomic(words, b, cv & 0xFFFFu, lv, wm); b += lv; }
                if (tsym) z_put_atomic(words, b, (ct & 0xFFFFu) | xt << (ct >> 16), lt, wm);
            }
        }
    }
    return carry;
}

}  // namespace
}  // namespace ambc
