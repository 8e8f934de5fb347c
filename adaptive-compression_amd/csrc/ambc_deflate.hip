// ambc_deflate.hip -- "ambc-deflate v1": the DEFLATE (id 5) encoder for gfx950.
//
// The reference's DeflateCompression.compress is zlib.compress(data, level=9)
// (advanced_compression.py:71-81).  Any valid zlib stream decodes there
// (zlib.decompress, :83-96), and zlib bytes are only round-trip tested by the
// reference, so the GPU uses its own definition, restated bit for bit in
// oracle/ambc_oracle.c (orc_gd_*):
//   parse : h(i) = (u32le(d+i) * 2654435761) >> 21 for i <= n-4; cand(i) = last
//           j < i with h(j) == h(i); a match at p iff u32le(d+cand) ==
//           u32le(d+p) and p - cand <= 32768; greedy, full length capped at 258
//           and n - p;
//   codes : one final block, the smallest of dynamic / fixed / stored (ties in
//           that order); Huffman lengths by the two-queue construction over
//           (freq, symbol)-sorted leaves, limited to 15 (7 for the code-length
//           code) by the bl_count fix-up, assigned shortest-first from the most
//           frequent symbol; code lengths run-length coded with 16/17/18;
//   frame : 78 DA, the block (LSB-first bit order, RFC 1951), Adler-32 (BE).
//
// k_deflate runs after k_encode (which picked the best of RLE/Huffman/Delta/
// LZ4 and recorded in bestpre[] the best (len+18) before LZ4), one 64-lane
// wavefront per chunk.  Selection keeps the reference's id order: id 5 wins iff
// len5+18 < bestpre and it does not lose to an LZ4 winner (ties go to id 5).
// A stored block can never win (n + 11 + 18 >= n), and the dynamic block is
// only built when its entropy lower bound could still win.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

__constant__ uint16_t c_lbase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                     33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                     1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                   6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

#ifdef AMBC_STAMPS
// diagnostic build only: per-chunk phase cycles in A.stamps[(M + k) * 8 + phase]
#define GSTAMP_DECL uint64_t _st_t = __builtin_amdgcn_s_memtime(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define GSTAMP(ph)                                                 \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _acc[ph] += _t - _st_t;                                    \
        _st_t = _t;                                                \
    } while (0)
#define GSTAMP_FLUSH                                               \
    if (lane == 0 && A.stamps)                                     \
        for (int _p = 0; _p < 8; _p++) A.stamps[((uint64_t)A.n_chunks + k) * 8 + _p] = _acc[_p];
#else
#define GSTAMP_DECL
#define GSTAMP(ph) do {} while (0)
#define GSTAMP_FLUSH
#endif

#define GRET             \
    do {                 \
        GSTAMP_FLUSH;    \
        return;          \
    } while (0)

constexpr uint32_t GD_LCAP = 32;  // per-lane precomputed match length; longer ones extend in the walk

// length symbol index (0..28) of a match length 3..258
__device__ __forceinline__ uint32_t gd_lcode(uint32_t L) {
    if (L == 258) return 28;
    const uint32_t y = L - 3;
    if (y < 8) return y;
    const uint32_t b = 31 - __builtin_clz(y);
    return 4 * (b - 1) + ((y >> (b - 2)) & 3);
}

// distance symbol (0..29) of a distance 1..32768
__device__ __forceinline__ uint32_t gd_dcode(uint32_t D) {
    const uint32_t x = D - 1;
    if (x < 4) return x;
    const uint32_t b = 31 - __builtin_clz(x);
    return 2 * b + ((x >> (b - 1)) & 1);
}

// unaligned 4-byte little-endian read from LDS (two aligned reads)
__device__ __forceinline__ uint32_t ld32(const uint8_t* base, uint32_t i) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base);
    const uint32_t a = i >> 2;
    return __builtin_amdgcn_alignbyte(w[a + 1], w[a], i & 3);
}

// v_writelane stand-in: lane `idx` (uniform) takes `val`
__device__ __forceinline__ uint32_t wlane(uint32_t old, uint32_t idx, uint32_t val, uint32_t lane) {
    return lane == idx ? val : old;
}

// OR nb (<= 32) bits of v into an LSB-first bit stream of u32 words at bit b
__device__ __forceinline__ void put_bits_atomic(uint32_t* words, uint32_t b, uint32_t v, uint32_t nb) {
#ifdef GD_NOATOMIC
    return;
#endif
    if (!nb) return;
    const uint32_t w = b >> 5, o = b & 31;
    atomicOr(&words[w], v << o);
    if (o + nb > 32) atomicOr(&words[w + 1], v >> (32 - o));
}

// put_bits_atomic into a ring of rm + 1 words (a power of two)
__device__ __forceinline__ void put_bits_ring(uint32_t* ring, uint32_t b, uint32_t v, uint32_t nb, uint32_t rm) {
    if (!nb) return;
    const uint32_t w = b >> 5, o = b & 31;
    atomicOr(&ring[w & rm], v << o);
    if (o + nb > 32) atomicOr(&ring[(w + 1) & rm], v >> (32 - o));
}

__device__ __forceinline__ void put_bits_plain(uint32_t* words, uint32_t b, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t w = b >> 5, o = b & 31;
    words[w] |= v << o;
    if (o + nb > 32) words[w + 1] |= v >> (32 - o);
}

template <int CMAX, bool NOCHUNK = false>
struct GdSmem {
    // parse: last[] (4 KB) + 64 bucket masks (512 B); trees: 5 KB; emit: bit staging.
    // Chunks of 16 KiB and more stage their bits over the chunk itself (the
    // emission then reads literals from the input) and keep the match-start
    // masks in device scratch: 74 / 41 KB at 64 / 32 KiB, 2 / 3 workgroups per
    // CU (1 / 1 with LDS staging)
    static constexpr bool BIG = CMAX >= 16384;
    static constexpr int REGION = (CMAX > 5120 && !BIG ? CMAX : 5120) + 64;
    static constexpr int ROUNDS = (CMAX + 63) / 64;
    // zero padded (EV: decision only, chunks >= 16 KiB read in place from the input)
    alignas(16) uint8_t chunk[NOCHUNK ? 16 : CMAX + 64];
    // parse: last[] (u16 x 2048) | trees: sorted/weights/parents | emit: bit staging
    alignas(16) uint32_t region[REGION / 4];
    uint64_t sel[BIG ? 1 : ROUNDS];        // match-start positions, per 64-position round
                                           // (BIG: in the chunk's device scratch, gd_seq_bytes)
    uint32_t lf[288], df[32], cf[20];      // symbol frequencies
    uint8_t ll[288], dl[32], cl[20];       // code lengths
    uint16_t lc[288], dc[32], cc[20];      // bit-reversed canonical codes
    uint8_t rs[320], re[320];              // code-length RLE: symbols, extra values
    uint32_t blc[24];
    uint32_t misc[8];
};

// Huffman code lengths of freq[0..nsym) limited to maxbits (see the file
// header), on one wave.  scratch: >= 5120 bytes of LDS.
template <int NSYM>
__device__ __forceinline__ void gd_lengths(const uint32_t* freq, int maxbits, uint8_t* len, uint32_t* scratch,
                                           uint32_t* blc, uint32_t lane) {
    constexpr int nsym = NSYM;
    uint16_t* sorted = reinterpret_cast<uint16_t*>(scratch);       // 320 x u16
    uint32_t* w = scratch + 160;                                   // 640 x u32
    uint16_t* parent = reinterpret_cast<uint16_t*>(scratch + 800); // 640 x u16
    constexpr int J = (NSYM + 63) / 64;  // symbols lane + 64 j
    uint32_t f[J];
    uint32_t used = 0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        f[j] = s < nsym ? freq[s] : 0u;
        used += f[j] != 0;
        if (s < nsym) len[s] = 0;
    }
    const uint32_t k = wave_sum_u32(used);
    if (k == 0) return;
    if (k == 1) {
#pragma unroll
        for (int j = 0; j < J; j++)
            if (f[j]) len[lane + 64 * j] = 1;
        return;
    }
    // used symbols compacted as (freq << 9 | symbol) keys, then ranked
    uint32_t* keys = scratch + 960;  // 320 x u32 (after parent[])
    {
        const uint64_t lt = (1ull << lane) - 1;
        uint32_t base = 0;
#pragma unroll
        for (int j = 0; j < J; j++) {
            const uint64_t m = __ballot(f[j] != 0);
            if (f[j]) keys[base + (uint32_t)__popcll(m & lt)] = f[j] << 9 | (uint32_t)(lane + 64 * j);
            base += (uint32_t)__popcll(m);
        }
    }
    wave_sync();
    if (k <= 64) {
        // ranks against the k keys held one per lane (v_readlane, no LDS)
        const uint32_t kreg = lane < k ? keys[lane] : 0u;
        uint32_t r[J];
#pragma unroll
        for (int j = 0; j < J; j++) r[j] = 0;
        for (uint32_t t = 0; t < k; t++) {
            const uint32_t kt = readlane(kreg, t);
#pragma unroll
            for (int j = 0; j < J; j++) r[j] += kt < (f[j] << 9 | (uint32_t)(lane + 64 * j));
        }
#pragma unroll
        for (int j = 0; j < J; j++)
            if (f[j]) { sorted[r[j]] = (uint16_t)(lane + 64 * j); w[r[j]] = f[j]; }
    } else {
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (f[j]) {
                const uint32_t key = f[j] << 9 | (uint32_t)(lane + 64 * j);
                uint32_t r = 0;
#pragma unroll 4
                for (uint32_t t = 0; t < k; t++) r += keys[t] < key;
                sorted[r] = (uint16_t)(lane + 64 * j);
                w[r] = f[j];
            }
        }
    }
    wave_sync();
    for (int i = lane; i < 24; i += 64) blc[i] = 0;
    bool deep = true;  // a leaf deeper than maxbits: the bl_count fix-up runs
    if (k <= 64) {
        // two-queue construction in registers: leaf i and internal node t live
        // in lane i / lane t; the fronts are read with v_readlane, new nodes
        // written with lane selects (no LDS round trips on the serial chain)
        const uint32_t INF = 0xFFFFFFFFu;
        const uint32_t wl = lane < k ? w[lane] : INF;
        uint32_t wi = INF, pl = 0, pi = 0, di = 0;
        uint32_t a = 0, b = 0, nb = 0;
        for (uint32_t m = 0; m + 1 < k; m++) {
            uint32_t sum = 0;
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const uint32_t va = a < k ? readlane(wl, a) : INF;
                const uint32_t vb = b < nb ? readlane(wi, b) : INF;
                if (a < k && (b >= nb || va <= vb)) {
                    pl = wlane(pl, a, nb, lane);
                    sum += va;
                    a++;
                } else {
                    pi = wlane(pi, b, nb, lane);
                    sum += vb;
                    b++;
                }
            }
            wi = wlane(wi, nb, sum, lane);
            nb++;
        }
        // depths of the internal nodes from the root (node nb - 1) down
        di = wlane(di, nb - 1, 0u, lane);
        for (int t = (int)nb - 2; t >= 0; t--) {
            const uint32_t d = readlane(di, readlane(pi, (uint32_t)t)) + 1;
            di = wlane(di, (uint32_t)t, d, lane);
        }
        const uint32_t dleaf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)di) + 1;
        deep = wave_max_i32(lane < k ? (int)dleaf : 0) > maxbits;
        if (!deep) {
            // no length limit to enforce: bl_count by ballots, cumulative counts in
            // registers, leaf (rank) i takes the smallest d with cum[d] > k - 1 - i
            uint32_t cum[16];
            uint32_t c = 0;
#pragma unroll
            for (int d = 1; d < 16; d++) {
                if (d <= maxbits) c += (uint32_t)__popcll(__ballot(lane < k && dleaf == (uint32_t)d));
                cum[d] = c;
            }
            const uint32_t e = k - 1 - lane;
            uint32_t d = 1;
#pragma unroll
            for (int t = 1; t < 16; t++) d += (t <= maxbits && cum[t] <= e) ? 1u : 0u;
            if (lane < k) len[sorted[lane]] = (uint8_t)d;
            wave_sync();
            return;
        }
        wave_sync();
        if (lane < k) atomicAdd(&blc[dleaf > 23 ? 23 : dleaf], 1u);
    } else {
        // two-queue construction (serial, LDS): leaves 0..k-1, internal k..2k-2
        if (lane == 0) {
            uint32_t a = 0, b = k, nb = k;
            for (uint32_t m = 0; m + 1 < k; m++) {
                uint32_t pick[2];
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const bool leaf = a < k && (b >= nb || w[a] <= w[b]);
                    pick[t] = leaf ? a++ : b++;
                }
                w[nb] = w[pick[0]] + w[pick[1]];
                parent[pick[0]] = (uint16_t)nb;
                parent[pick[1]] = (uint16_t)nb;
                nb++;
            }
            // depths of the internal nodes, root first (stored in w[], reused)
            w[nb - 1] = 0;
            for (int i = (int)nb - 2; i >= (int)k; i--) w[i] = w[parent[i]] + 1;
        }
        wave_sync();
        for (uint32_t i = lane; i < k; i += 64) {
            const uint32_t d = w[parent[i]] + 1;
            atomicAdd(&blc[d > 23 ? 23 : d], 1u);
        }
    }
    wave_sync();
    if (deep && lane == 0) {
        for (int d = maxbits + 1; d < 24; d++) { blc[maxbits] += blc[d]; blc[d] = 0; }
        uint64_t total = 0;
        for (int d = 1; d <= maxbits; d++) total += (uint64_t)blc[d] << (maxbits - d);
        while (total > (1ull << maxbits)) {
            blc[maxbits]--;
            for (int d = maxbits - 1; d > 0; d--)
                if (blc[d]) { blc[d]--; blc[d + 1] += 2; break; }
            total--;
        }
    }
    wave_sync();
    // shortest lengths to the most frequent: rank i from the top gets the
    // smallest d with blc[1] + .. + blc[d] > i
    for (uint32_t i = lane; i < k; i += 64) {
        const uint32_t e = k - 1 - i;
        uint32_t cum = 0, d = 1;
        for (; d <= (uint32_t)maxbits; d++) {
            cum += blc[d];
            if (cum > e) break;
        }
        len[sorted[i]] = (uint8_t)d;
    }
    wave_sync();
}

// canonical codes of len[0..nsym) (RFC 1951 3.2.2), bit-reversed
template <int NSYM>
__device__ __forceinline__ void gd_codes(const uint8_t* len, uint16_t* rcode, uint32_t* blc, uint32_t lane) {
    // canonical assignment with ballots only: for each length b (ascending) the
    // first code follows from the previous length's first code and count, and a
    // symbol's code adds the number of same-length symbols below it
    (void)blc;
    constexpr int nsym = NSYM;
    constexpr int J = (NSYM + 63) / 64;
    uint32_t l[J], code[J];
    uint32_t lmax = 0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        l[j] = s < nsym ? len[s] : 0u;
        code[j] = 0;
        lmax = max(lmax, l[j]);
    }
    lmax = (uint32_t)wave_max_i32((int)lmax);
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t first = 0, prevcnt = 0;
    for (uint32_t b = 1; b <= lmax; b++) {
        first = (first + prevcnt) << 1;
        uint32_t seen = 0;
#pragma unroll
        for (int j = 0; j < J; j++) {
            const uint64_t m = __ballot(l[j] == b);
            if (l[j] == b) code[j] = first + seen + (uint32_t)__popcll(m & lt);
            seen += (uint32_t)__popcll(m);
        }
        prevcnt = seen;
    }
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        if (s < nsym) rcode[s] = l[j] ? (uint16_t)(__builtin_bitreverse32(code[j]) >> (32 - l[j])) : 0;
    }
    wave_sync();
}

// one run of rr equal code lengths v -> code-length symbols at rs/re[o..];
// returns the new count (the rule of the file header / orc_gd: gd_rle)
__device__ __forceinline__ uint32_t rle_flush(uint8_t* rs, uint8_t* re, uint32_t o, uint32_t v, uint32_t rr,
                                              uint32_t lane) {
    const bool w = lane == 0;
    if (v == 0) {
        while (rr >= 11) {
            const uint32_t t = min(rr, 138u);
            if (w) { rs[o] = 18; re[o] = (uint8_t)(t - 11); }
            o++;
            rr -= t;
        }
        if (rr >= 3) {
            if (w) { rs[o] = 17; re[o] = (uint8_t)(rr - 3); }
            o++;
            rr = 0;
        }
        for (; rr > 0; rr--, o++)
            if (w) { rs[o] = 0; re[o] = 0; }
    } else {
        if (w) { rs[o] = (uint8_t)v; re[o] = 0; }
        o++;
        rr--;
        while (rr >= 3) {
            const uint32_t t = min(rr, 6u);
            if (w) { rs[o] = 16; re[o] = (uint8_t)(t - 3); }
            o++;
            rr -= t;
        }
        for (; rr > 0; rr--, o++)
            if (w) { rs[o] = (uint8_t)v; re[o] = 0; }
    }
    return o;
}

// EV (ENC_EVAL, chunks >= 16 KiB, padded input): the decision only -- the chunk is
// read in place instead of staged (the 64 / 32 KiB LDS copy held the CU to 2 / 3
// workgroups through the multi-size walk's rounds) and nothing is emitted
// IP (padded input): read in place as well.  Up to 8 KiB the bits are still staged
// in the LDS region (13 -> 9 KB of LDS at 4 KiB); from 16 KiB (GB) they go straight
// into the chunk's slot by global atomics, the zlib header and the block header
// built in the LDS region first: 10 KB of LDS instead of 74 KB at 64 KiB, where the
// staged copy held a CU to 2 workgroups (half its SIMDs idle) for the multi-size
// walk's final encode
template <int CMAX, bool EV = false, bool IP = EV>
__global__ __launch_bounds__(64) void k_deflate(EncArgs A) {
    constexpr bool NOCHUNK = IP;
    constexpr bool GB = IP && !EV && CMAX >= 16384;
    __shared__ GdSmem<CMAX, NOCHUNK> S;
    constexpr int ROUNDS = GdSmem<CMAX, NOCHUNK>::ROUNDS;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    GSTAMP_DECL
    // prefs gate (adaptive_compressor.py:565-567) and should_use's n >= 64
    if (!((A.method_mask >> 5) & 1) || n < A.pref_min[5] || n > A.pref_max[5] || n < 64) GRET;
    const uint32_t w0 = A.ids[k];
    const uint32_t bp0 = A.bestpre[k];
    if (bp0 >> 31) GRET;  // calculate_entropy == 8.0: should_use is False (k_encode's histogram)
    const bool single = (bp0 >> 30) & 1;   // one byte value throughout
    const uint32_t bestpre = bp0 & 0x3FFFFFFFu;
    // id 5 wins iff len + 18 < T (ties against an LZ4 winner go to id 5)
    const uint32_t T = w0 == 9 ? min(bestpre, A.plen[k] + 18 + 1) : bestpre;
    if (T <= 18 + 6) GRET;
    const uint8_t* src = A.in + pos0;
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;

    // ---- stage the chunk in LDS ----
    const uint8_t* const ch = NOCHUNK ? src : S.chunk;
    if constexpr (!NOCHUNK) {
        const uint32_t nv = n >> 4;
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            for (uint32_t q = lane; q < nv; q += 64)
                reinterpret_cast<uint4*>(S.chunk)[q] = reinterpret_cast<const uint4*>(src)[q];
            for (uint32_t i = (nv << 4) + lane; i < n; i += 64) S.chunk[i] = src[i];
        } else {
            for (uint32_t i = lane; i < n; i += 64) S.chunk[i] = src[i];
        }
        for (uint32_t i = n + lane; i < (uint32_t)CMAX + 64; i += 64) S.chunk[i] = 0;
    }
    wave_sync();
    GSTAMP(0);
    // ---- parse ----
    // the parse's matches, in order, as (position | length << 16 | distance << 32)
    // in the chunk's window of the device scratch A.gdseq (2 CMAX bytes: at most
    // n/4 matches)
    uint8_t* const scr = A.gdseq + (uint64_t)k * gd_seq_bytes(CMAX);
    uint64_t* seq = reinterpret_cast<uint64_t*>(scr);
    uint64_t* const selp = GdSmem<CMAX, NOCHUNK>::BIG ? reinterpret_cast<uint64_t*>(scr + 2 * CMAX) : S.sel;
    uint32_t mcov = 0;  // bytes the matches cover
    unsigned long long* bk = reinterpret_cast<unsigned long long*>(S.region + 1024);  // after last[]
    uint32_t ns = 0;
    uint32_t extra = 0;  // extra bits of the length / distance codes
    for (uint32_t i = lane; i < 288; i += 64) S.lf[i] = 0;
    if (lane < 32) S.df[lane] = 0;
    if (single) {
        // one byte value: the greedy parse is a literal at 0, then distance-1
        // matches of min(258, n - p) at p = 1 + 258 j while p + 4 <= n
        const uint32_t M = n >= 5 ? (n - 5) / 258 + 1 : 0;
        // (258 > 64: at most one match start per round)
        for (uint32_t r = lane; r < (n + 63) / 64; r += 64) {
            const uint32_t p0 = 64 * r, j = p0 <= 1 ? 0u : (p0 - 1 + 257) / 258, pj = 1 + 258 * j;
            selp[r] = j < M && pj < p0 + 64 ? 1ull << (pj - p0) : 0ull;
        }
        for (uint32_t j = lane; j < M; j += 64) {
            const uint32_t pj = 1 + 258 * j;
            const uint32_t Lj = min(258u, n - pj);
            seq[j] = pj | (uint64_t)Lj << 16 | 1ull << 32;
            mcov += Lj;
        }
        ns = M;
        mcov = wave_sum_u32(mcov);
    } else {
    uint16_t* last = reinterpret_cast<uint16_t*>(S.region);
    for (uint32_t i = lane; i < 2048; i += 64) last[i] = 0xFFFF;
    bk[lane] = 0;
    wave_sync();
    const int hl = (int)n - 4;  // last hashable position
    uint32_t p = 0;
    int fcarry = 0;  // max match end so far (frequency count)
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(ch);
    // The probe runs a round ahead, its loads kept as raw aligned words until used
    // (their waits fall in the next round): at the top of round r, round r's
    // positions enter the table (last[] then holds everything before round r + 1,
    // as the serial order needs), then round r + 1's hashes, candidates and the
    // candidates' bytes, and round r + 2's own bytes (clamped to n: past n the word
    // is zero, as the padded LDS chunk has it and the in-place input may end 64
    // bytes after n).  The loads are unconditional, so the load counter stays exact.
    auto raw_at = [&](uint32_t pos, uint32_t& lo, uint32_t& hi) { lo = c32[pos >> 2]; hi = c32[(pos >> 2) + 1]; };
    // round rr's candidates (base rb, positions i = rb + lane with their words vv)
    auto probe = [&](int rb, uint32_t vv, uint32_t& hh, uint64_t& pp) -> int {
        const int ii = rb + (int)lane;
        const bool aa = ii <= hl;
        hh = (vv * 2654435761u) >> 21;
        const uint32_t c16 = last[hh];
        // lanes with my 11-bit hash: one shared hash (runs) is the active mask; else
        // an order-free LDS OR per 8-bit bucket, then 3 ballots for the top bits
        const uint64_t actm = rb + 63 <= hl ? ~0ull : __ballot(aa);
        const uint32_t h0 = __builtin_amdgcn_readfirstlane(hh);
        if (__ballot(hh != h0) == 0ull) {
            pp = actm;
        } else {
            atomicOr(&bk[hh & 63], aa ? 1ull << lane : 0ull);
            wave_sync();
            pp = bk[hh & 63] & actm;
#pragma unroll
            for (int b = 6; b < 11; b++) {
                const uint64_t m = __ballot((hh >> b) & 1u);
                const uint64_t flip = 0ull - (uint64_t)((hh >> b) & 1u);
                pp &= ~(m ^ flip);
            }
            wave_sync();
            bk[hh & 63] = 0;
        }
        const uint64_t lower = pp & ((1ull << lane) - 1ull);
        return lower ? rb + 63 - (int)__clzll((long long)lower) : (c16 == 0xFFFFu ? -1 : (int)c16);
    };
    uint32_t nlo, nhi, clo, chi, v_cur, h_cur;
    uint64_t peers_cur;
    int cand_cur;
    {
        uint32_t lo, hi;
        raw_at(min(lane, n), lo, hi);
        v_cur = lane < n ? __builtin_amdgcn_alignbyte(hi, lo, lane & 3u) : 0u;
        cand_cur = probe(0, v_cur, h_cur, peers_cur);
        raw_at((uint32_t)max(cand_cur, 0), clo, chi);
        raw_at(min(lane + 64u, n), nlo, nhi);
    }
#pragma unroll 1
    for (int r = 0; r < ROUNDS; r++) {
        const int base = r * 64;
        if (base >= (int)n) break;
        // control state is wave-uniform: keep it in SGPRs
        p = __builtin_amdgcn_readfirstlane(p);
        fcarry = (int)__builtin_amdgcn_readfirstlane((uint32_t)fcarry);
        ns = __builtin_amdgcn_readfirstlane(ns);
        const int i = base + (int)lane;
        const bool act = i <= hl;
        const uint32_t v = v_cur;
        const int cand = cand_cur;
        // (the candidate bytes are consumed before their registers take the next round's)
        const uint32_t cv = __builtin_amdgcn_alignbyte(chi, clo, (uint32_t)max(cand, 0) & 3u);
        // round r's positions into the table: each hash's highest position
        if (act && (peers_cur >> lane) == 1ull) last[h_cur] = (uint16_t)i;
        wave_sync();
        if (base + 64 < (int)n) {
            const uint32_t vn = i + 64 < (int)n ? __builtin_amdgcn_alignbyte(nhi, nlo, lane & 3u) : 0u;
            const int cn = probe(base + 64, vn, h_cur, peers_cur);
            uint32_t ca = (uint32_t)max(cn, 0), na = min((uint32_t)i + 128u, n);
            asm volatile("" : "+v"(ca), "+v"(na) : "v"(cv), "v"(vn));   // (issued after cv, vn are formed)
            raw_at(ca, clo, chi);
            raw_at(na, nlo, nhi);
            v_cur = vn;
            cand_cur = cn;
        }
        const bool valid = act && cand >= 0 && i - cand <= 32768 && cv == v;
        const uint64_t vm = __ballot(valid);
        wave_sync();
        uint32_t L = 0;
        uint64_t selm = 0;
        const uint32_t ns0 = ns;
        const uint32_t pr = p - (uint32_t)base;   // p >= base
        if (pr < 64 && (vm & (~0ull << pr)) == 0ull) {
            p = (uint32_t)base + 64;               // no match starts here: literals
        } else if (pr < 64) {
            // per-lane match length: 16 bytes per step (five aligned dwords per side
            // in flight), capped at GD_LCAP; the walk extends longer ones
            const bool run_l = valid && (uint32_t)i >= p;
            bool run = run_l;
            const uint32_t lim = run ? min(258u, n - (uint32_t)i) : 0u;
            const uint32_t cap = min(lim, GD_LCAP);
            if (run) L = 4;
            const uint32_t si = (uint32_t)i & 3u, sc = (uint32_t)cand & 3u;
#pragma unroll 1
            while (__ballot(run && L < cap)) {
                if (run && L < cap) {
                    const uint32_t ai = ((uint32_t)i + L) >> 2, ac = ((uint32_t)cand + L) >> 2;
                    uint32_t wi[5], wc[5];
#pragma unroll
                    for (int t = 0; t < 5; t++) { wi[t] = c32[ai + t]; wc[t] = c32[ac + t]; }
                    uint32_t add = 16;
#pragma unroll
                    for (int t = 3; t >= 0; t--) {
                        const uint32_t x = __builtin_amdgcn_alignbyte(wi[t + 1], wi[t], si) ^
                                           __builtin_amdgcn_alignbyte(wc[t + 1], wc[t], sc);
                        if (x) add = 4 * t + ((uint32_t)__builtin_ctz(x) >> 3);
                    }
                    L += add;
                    if (add < 16) run = false;
                }
            }
            L = min(L, lim);
            // greedy walk: every lane links to the next match start the parse takes
            // after its match (64 = none in this round, 65 = extend past GD_LCAP);
            // two bpermutes extend the link four deep, one v_readlane per four matches
            const bool longl = run_l && L >= GD_LCAP && L < lim;
            const uint32_t E = lane + L;
            uint32_t nx1;
            {
                const uint64_t mm = E < 64 ? (vm & (~0ull << E)) : 0ull;
                nx1 = longl ? 65u : (mm ? (uint32_t)__builtin_ctzll(mm) : 64u);
            }
            uint32_t nx2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(nx1, 63u) << 2), (int)nx1);
            if (nx1 >= 64) nx2 = nx1;
            const uint32_t pk1 = nx1 | nx2 << 7;
            uint32_t pk2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(nx2, 63u) << 2), (int)pk1);
            if (nx2 >= 64) pk2 = nx2 | nx2 << 7;
            const uint32_t pack = pk1 | pk2 << 14;
            uint32_t cur = (uint32_t)__builtin_ctzll(vm & (~0ull << pr));
            uint32_t endrel = 64;
            while (cur < 64) {
                selm |= 1ull << cur;
                const uint32_t pk = readlane(pack, cur);
                uint32_t x = pk & 127u, f = 1;
                while (x < 64) {
                    selm |= 1ull << x;
                    cur = x;
                    if (f == 4) break;
                    x = (pk >> (7 * f)) & 127u;
                    f++;
                }
                if (x < 64) continue;
                if (x == 64) { endrel = readlane(E, cur); break; }
                // x == 65: cur's match reaches GD_LCAP: the whole wave extends it
                const uint32_t pj = (uint32_t)base + cur;
                const uint32_t lj = min(258u, n - pj);
                uint32_t Lp = readlane(L, cur);
                const uint32_t c = readlane((uint32_t)cand, cur);
                for (;;) {
                    const uint32_t off = Lp + 4 * lane;
                    const uint32_t xx = off < lj ? (ld32(ch, c + off) ^ ld32(ch, pj + off)) : 1u;
                    const uint64_t mm = __ballot(xx != 0);
                    if (mm) {
                        const uint32_t fl = (uint32_t)__builtin_ctzll(mm);
                        const uint32_t xf = readlane(xx, fl);
                        Lp += 4 * fl + ((uint32_t)__builtin_ctz(xf) >> 3);
                        break;
                    }
                    Lp += 256;
                }
                Lp = __builtin_amdgcn_readfirstlane(min(Lp, lj));
                L = wlane(L, cur, Lp, lane);
                endrel = cur + Lp;
                const uint64_t mn = endrel < 64 ? (vm & (~0ull << endrel)) : 0ull;
                cur = mn ? (uint32_t)__builtin_ctzll(mn) : 64u;
            }
            p = (uint32_t)base + max(endrel, 64u);
        }
        // the selected matches record themselves, in position order, and the
        // round's symbol frequencies are counted (literals: positions no match covers)
        if (selm || fcarry < base + 64) {
            const bool st = (selm >> lane) & 1;
            int e = 0;
            if (st) {
                const uint32_t si = ns0 + (uint32_t)__popcll(selm & ((1ull << lane) - 1));
                const uint32_t D = (uint32_t)(i - cand);
                seq[si] = (uint64_t)i | (uint64_t)L << 16 | (uint64_t)D << 32;
                e = i + (int)L;
                const uint32_t lcd = gd_lcode(L), dcd = gd_dcode(D);
                atomicAdd(&S.lf[257 + lcd], 1u);
                atomicAdd(&S.df[dcd], 1u);
                extra += c_lext[lcd] + c_dext[dcd];
            }
            const int E = max(fcarry, wave_incl_max_i32(e));
            fcarry = max(fcarry, wave_max_i32(e));
            if (i < (int)n && E <= i) atomicAdd(&S.lf[v & 0xFFu], 1u);   // (the position's byte: v's first)
            mcov += wave_sum_u32(st ? L : 0u);
        }
        ns = ns0 + (uint32_t)__popcll(selm);
        if (lane == 0) selp[r] = selm;
    }
    }
    const uint32_t nrounds = (n + 63) / 64;
    __threadfence_block();  // the match records (global) are read back by other lanes
    wave_sync();

    GSTAMP(1);
    // ---- symbol frequencies (the general parse counted them as it went) ----
    if (single) {
        // a literal at 0 and after the last match, then the matches of seq[]
        if (lane == 0) S.lf[ch[0]] += n - mcov;
        wave_sync();
        for (uint32_t j = lane; j < ns; j += 64) {
            const uint32_t Lj = (uint32_t)(seq[j] >> 16) & 0xFFFF;
            const uint32_t lcd = gd_lcode(Lj);
            atomicAdd(&S.lf[257 + lcd], 1u);
            atomicAdd(&S.df[0], 1u);
            extra += c_lext[lcd];
        }
    }
    extra = wave_sum_u32(extra);
    if (lane == 0) S.lf[256] = 1;
    wave_sync();

    GSTAMP(2);
    // ---- fixed size and the dynamic lower bound ----
    uint64_t fixb = 0;
    double ent = 0.0;
    uint32_t F = 0;
    for (uint32_t s = lane; s < 286; s += 64) F += S.lf[s];
    F = wave_sum_u32(F);
    for (uint32_t s = lane; s < 286; s += 64) {
        const uint32_t f = S.lf[s];
        fixb += (uint64_t)f * (s < 144 ? 8u : s < 256 ? 9u : s < 280 ? 7u : 8u);
        if (f) ent += (double)f * log2((double)F / (double)f);
    }
    if (lane < 30) fixb += (uint64_t)S.df[lane] * 5u;
    fixb = wave_sum<uint64_t>(fixb) + 3 + extra;
    ent = wave_sum<double>(ent);
    const uint32_t fix_bytes = (uint32_t)((fixb + 7) / 8);
    // Huffman >= entropy per symbol; 17 header bits + at least 4 code-length codes
    const double lb_bits = ent * (1.0 - 1e-9) - 1.0 + 17 + 12 + extra;
    const uint32_t lb_bytes = lb_bits > 0 ? (uint32_t)(lb_bits / 8.0) : 0u;
    const uint32_t nblk = (n + 65534) / 65535;
    const uint32_t sto_bytes = n + 5 * nblk;
    const bool dyn_possible = lb_bytes + 6 + 18 < T;
    if (!dyn_possible && fix_bytes + 6 + 18 >= T) GRET;  // cannot win

    GSTAMP(3);
    // ---- dynamic code ----
    uint32_t dyn_bytes = 0xFFFFFFFFu;
    uint32_t hlit = 257, hdist = 1, hclen = 4, nr = 0;
    if (dyn_possible) {
        // at least two distance codes carry a length (zlib's convention)
        if (lane == 0) {
            int used = 0;
            for (int i = 0; i < 30; i++) used += S.df[i] != 0;
            S.misc[0] = S.misc[1] = 0;
            for (int i = 0; i < 2 && used < 2; i++)
                if (!S.df[i]) { S.df[i] = 1; S.misc[i] = 1; used++; }
        }
        wave_sync();
        GSTAMP(4);
        gd_lengths<286>(S.lf, 15, S.ll, S.region, S.blc, lane);
        gd_lengths<30>(S.df, 15, S.dl, S.region, S.blc, lane);
        GSTAMP(6);
        if (lane == 0) {  // the forced distance frequencies do not count as symbols
            for (int i = 0; i < 2; i++) if (S.misc[i] == 1) S.df[i] = 0;
        }
        wave_sync();
        // HLIT / HDIST
        {
            int hi = 0;
            for (uint32_t s = lane; s < 286; s += 64) if (S.ll[s]) hi = max(hi, (int)s + 1);
            hlit = (uint32_t)max(257, wave_max_i32(hi));
            int hd = 0;
            if (lane < 30 && S.dl[lane]) hd = (int)lane + 1;
            hdist = (uint32_t)max(1, wave_max_i32(hd));
        }
        // code-length RLE: the HLIT + HDIST lengths held 5 per lane (entry
        // e = 64 j + lane), walked on the scalar unit with v_readlane
        {
            const uint32_t cnt = hlit + hdist;
            uint32_t val[5];
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t e = 64 * j + lane;
                val[j] = e < hlit ? S.ll[e] : (e < cnt ? S.dl[e - hlit] : 0u);
            }
            // run starts by ballot (entry e differs from e - 1), then one
            // scalar step per run
            uint64_t bnd[5];
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t e = 64 * j + lane;
                uint32_t prev = __shfl_up(val[j], 1);
                if (lane == 0) prev = j ? readlane(val[j > 0 ? j - 1 : 0], 63) : 0xFFu;
                bnd[j] = __ballot(e < cnt && val[j] != prev);
            }
            uint32_t o = 0, cur = readlane(val[0], 0), start = 0;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                uint64_t m = bnd[j];
                while (m) {
                    const uint32_t l = (uint32_t)__builtin_ctzll(m);
                    m &= m - 1;
                    const uint32_t e = 64 * j + l;
                    if (e) o = rle_flush(S.rs, S.re, o, cur, e - start, lane);
                    cur = readlane(val[j], l);
                    start = e;
                }
            }
            o = rle_flush(S.rs, S.re, o, cur, cnt - start, lane);
            if (lane == 0) S.misc[2] = o;
            if (lane < 20) S.cf[lane] = 0;
            wave_sync();
            for (uint32_t i = lane; i < o; i += 64) atomicAdd(&S.cf[S.rs[i]], 1u);
        }
        wave_sync();
        GSTAMP(7);
        nr = S.misc[2];
        gd_lengths<19>(S.cf, 7, S.cl, S.region, S.blc, lane);
        {
            int hc = 4;
            if (lane < 19 && S.cl[c_clord[lane]]) hc = (int)lane + 1;
            hclen = (uint32_t)max(4, wave_max_i32(hc));
        }
        uint64_t dynb = 0;
        for (uint32_t i = lane; i < nr; i += 64) {
            const uint32_t sy = S.rs[i];
            dynb += S.cl[sy] + (sy == 16 ? 2u : sy == 17 ? 3u : sy == 18 ? 7u : 0u);
        }
        for (uint32_t s = lane; s < 286; s += 64) dynb += (uint64_t)S.lf[s] * S.ll[s];
        if (lane < 30) dynb += (uint64_t)S.df[lane] * S.dl[lane];
        dynb = wave_sum<uint64_t>(dynb) + 17 + 3ull * hclen + extra;
        dyn_bytes = (uint32_t)((dynb + 7) / 8);
    }
    GSTAMP(4);
    const int kind = (dyn_bytes <= fix_bytes && dyn_bytes <= sto_bytes) ? 2 : (fix_bytes <= sto_bytes ? 1 : 0);
    const uint32_t body = kind == 2 ? dyn_bytes : kind == 1 ? fix_bytes : sto_bytes;
    const uint32_t total = 2 + body + 4;
    if (kind == 0 || total + 18 >= T) GRET;  // a stored block never beats raw
    if constexpr (EV) {
        if (lane == 0) {
            A.ids[k] = 5;
            A.plen[k] = total;
            A.sizes[k] = 18ull + total;
        }
        return;
    } else {

    // ---- Adler-32 of the chunk (before a BIG chunk's bits overwrite it) ----
    const uint32_t adler = adler32_wave(ch, n, lane);
    // literal bytes during the emission: LDS, or the input (L2) for BIG chunks
    constexpr bool BIG = GdSmem<CMAX, NOCHUNK>::BIG;
    auto chb = [&](uint32_t q) -> uint32_t { return BIG || NOCHUNK ? (uint32_t)src[q] : (uint32_t)S.chunk[q]; };

    // ---- emission (this chunk's winner) ----
    if (kind == 1) {  // fixed tables
        for (uint32_t s = lane; s < 288; s += 64) S.ll[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        if (lane < 30) S.dl[lane] = 5;
        wave_sync();
        gd_codes<288>(S.ll, S.lc, S.blc, lane);
        gd_codes<30>(S.dl, S.dc, S.blc, lane);
    } else {
        gd_codes<286>(S.ll, S.lc, S.blc, lane);
        gd_codes<30>(S.dl, S.dc, S.blc, lane);
        gd_codes<19>(S.cl, S.cc, S.blc, lane);
    }
    // GB: the stream goes through a 4 KB ring in the LDS region (the header from
    // bit 16, behind 78 DA), its finished words stored to the slot after every
    // 64-position round: LDS atomics instead of global ones (same-address ORs
    // serialised in L2: a 64 KiB chunk's emission cost more than its parse)
    constexpr uint32_t RW = 1024, RM = RW - 1;
    static_assert(!GB || GdSmem<CMAX, NOCHUNK>::REGION >= 4 * (int)RW, "the ring fits the region");
    uint32_t* bits = GB ? S.region : BIG ? reinterpret_cast<uint32_t*>(S.chunk) : S.region;
    const uint32_t nwords = GB ? RW : (body + 8) / 4 + 1;
    for (uint32_t i = lane; i < nwords; i += 64) bits[i] = 0;
    wave_sync();
    const uint32_t b0 = GB ? 16u : 0u;
    uint32_t bp = 0;
    if (lane == 0) {
        if constexpr (GB) put_bits_plain(bits, 0, 0xDA78u, 16);
        put_bits_plain(bits, b0, 1u | ((uint32_t)kind << 1), 3);
        bp = b0 + 3;
        if (kind == 2) {
            put_bits_plain(bits, bp, hlit - 257, 5); bp += 5;
            put_bits_plain(bits, bp, hdist - 1, 5); bp += 5;
            put_bits_plain(bits, bp, hclen - 4, 4); bp += 4;
            for (uint32_t i = 0; i < hclen; i++) { put_bits_plain(bits, bp, S.cl[c_clord[i]], 3); bp += 3; }
            for (uint32_t i = 0; i < nr; i++) {
                const uint32_t sy = S.rs[i];
                put_bits_plain(bits, bp, S.cc[sy], S.cl[sy]); bp += S.cl[sy];
                const uint32_t eb = sy == 16 ? 2u : sy == 17 ? 3u : sy == 18 ? 7u : 0u;
                put_bits_plain(bits, bp, S.re[i], eb); bp += eb;
            }
        }
    }
    bp = readlane(bp, 0);
    wave_sync();
    uint32_t* const gw = reinterpret_cast<uint32_t*>(slot);
    uint32_t flushed = 0;   // GB: words [0, flushed) are in the slot
    auto flush = [&](uint32_t upto) {
        wave_sync();
        for (uint32_t w = flushed + lane; w < upto; w += 64) {
            gw[w] = S.region[w & RM];
            S.region[w & RM] = 0;
        }
        wave_sync();
        flushed = upto;
    };
    auto put = [&](uint32_t b, uint32_t v, uint32_t nb) {
        if constexpr (GB) put_bits_ring(S.region, b, v, nb, RM);
        else put_bits_atomic(bits, b, v, nb);
    };
    // (GB: position-major only, so that a round's bits are bounded by the ring)
    if (!GB && n - mcov <= 8 * (ns + 1)) {
        // match-major: lane e emits the literal run before match e and the
        // match (element ns: the literals after the last match); 64 matches per
        // step instead of 64 positions
        uint32_t pe_carry = 0;
#pragma unroll 1
        for (uint32_t b0 = 0; b0 <= ns; b0 += 64) {
            const uint32_t e = b0 + lane;
            const bool has = e <= ns, mt = e < ns;
            const uint64_t sq = mt ? seq[e] : 0ull;
            const uint32_t pos = mt ? (uint32_t)(sq & 0xFFFF) : n;
            const uint32_t Lx = (uint32_t)(sq >> 16) & 0xFFFF, Dx = (uint32_t)(sq >> 32);
            const uint32_t myend = mt ? pos + Lx : n;
            uint32_t pe = __shfl_up(myend, 1);
            if (lane == 0) pe = pe_carry;
            uint32_t cost = 0, lcd = 0, dcd = 0;
            if (has)
                for (uint32_t q = pe; q < pos; q++) cost += S.ll[chb(q)];
            if (mt) {
                lcd = gd_lcode(Lx);
                dcd = gd_dcode(Dx);
                cost += S.ll[257 + lcd] + c_lext[lcd] + S.dl[dcd] + c_dext[dcd];
            }
            const uint32_t incl = wave_incl_sum(cost);
            uint32_t b = bp + incl - cost;
            if (has) {
                for (uint32_t q = pe; q < pos; q++) {
                    const uint32_t c = chb(q);
                    put_bits_atomic(bits, b, S.lc[c], S.ll[c]);
                    b += S.ll[c];
                }
            }
            if (mt) {
                const uint32_t l1 = S.ll[257 + lcd], l2 = S.dl[dcd];
                put_bits_atomic(bits, b, S.lc[257 + lcd] | (Lx - c_lbase[lcd]) << l1, l1 + c_lext[lcd]);
                b += l1 + c_lext[lcd];
                put_bits_atomic(bits, b, S.dc[dcd] | (Dx - c_dbase[dcd]) << l2, l2 + c_dext[dcd]);
            }
            bp += readlane(incl, 63);
            pe_carry = readlane(myend, 63);
        }
    } else {
        // position-major (literal-heavy chunks)
        int carry = 0;
        uint32_t sb = 0;   // matches before this round
        const uint64_t lt = (1ull << lane) - 1;
        // each position's byte is read a round ahead (wave-uniform rp: the round it
        // belongs to; a round skipped inside a match reads its own)
        uint32_t rp = 0, cp = chb(min(lane, n - 1));
#pragma unroll 1
        for (uint32_t r = 0; r < nrounds; r++) {
            const uint32_t i = r * 64 + lane;
            const uint64_t sv = selp[r];
            const uint64_t sm = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sv) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sv >> 32)) << 32;
            if (!sm && carry >= (int)(r * 64 + 64)) continue;  // inside one match
            const bool st = (sm >> lane) & 1;
            int e = 0;
            uint32_t Lx = 0, Dx = 0, lcd = 0, dcd = 0, cost = 0;
            if (st) {
                const uint32_t si = sb + (uint32_t)__popcll(sm & lt);
                const uint64_t sq = seq[si];
                Lx = (uint32_t)(sq >> 16) & 0xFFFF;
                Dx = (uint32_t)(sq >> 32);
                e = (int)(i + Lx);
                lcd = gd_lcode(Lx);
                dcd = gd_dcode(Dx);
                cost = S.ll[257 + lcd] + c_lext[lcd] + S.dl[dcd] + c_dext[dcd];
            }
            const int E = max(carry, wave_incl_max_i32(e));
            carry = max(carry, wave_max_i32(e));
            const bool lit = i < n && E <= (int)i;
            uint32_t cb = rp == r ? cp : chb(min(i, n - 1));
            {
                uint32_t na = min(i + 64u, n - 1);
                asm volatile("" : "+v"(na) : "v"(cb));   // (cb formed: cp's register is free)
                cp = chb(na);
                rp = r + 1;
            }
            const uint32_t c = lit ? cb : 0u;
            if (lit) cost = S.ll[c];
            const uint32_t incl = wave_incl_sum(cost);
            uint32_t b = bp + incl - cost;
            if (lit) {
                put(b, S.lc[c], S.ll[c]);
            } else if (st) {
                const uint32_t l1 = S.ll[257 + lcd], l2 = S.dl[dcd];
                put(b, S.lc[257 + lcd] | (Lx - c_lbase[lcd]) << l1, l1 + c_lext[lcd]);
                b += l1 + c_lext[lcd];
                put(b, S.dc[dcd] | (Dx - c_dbase[dcd]) << l2, l2 + c_dext[dcd]);
            }
            bp += readlane(incl, 63);
            sb += (uint32_t)__popcll(sm);
            if constexpr (GB) flush(bp >> 5);
        }
    }
    wave_sync();
    if constexpr (GB) {
        // end of block and Adler-32 (big-endian bytes after the body) into the ring,
        // then its last words to the slot
        if (lane == 0) put_bits_ring(S.region, bp, S.lc[256], S.ll[256], RM);
        if (lane < 4) {
            const uint32_t q = 2 + body + lane;
            atomicOr(&S.region[(q >> 2) & RM], ((adler >> (8 * (3 - lane))) & 0xFFu) << (8 * (q & 3)));
        }
        flush((total + 3) / 4);
    } else {
    if (lane == 0) put_bits_plain(bits, bp, S.lc[256], S.ll[256]);
    wave_sync();
    // ---- the zlib stream into the slot ----
    const uint8_t* bb = reinterpret_cast<const uint8_t*>(bits);
    for (uint32_t i = lane; i < total; i += 64) {
        uint8_t o;
        if (i == 0) o = 0x78;
        else if (i == 1) o = 0xDA;
        else if (i < 2 + body) o = bb[i - 2];
        else o = (uint8_t)(adler >> (8 * (3 - (i - 2 - body))));
        slot[i] = o;
    }
    }
    if (lane == 0) {
        A.ids[k] = 5;
        A.plen[k] = total;
        A.sizes[k] = 18ull + total;
    }
    GSTAMP(5);
    GSTAMP_FLUSH;
    }
}

template <int CMAX>
hipError_t launch_deflate_t(const EncArgs& a, hipStream_t s) {
    if constexpr (CMAX >= 4096 && CMAX <= 8192) {
        if ((a.flags & ENC_IN_ALIGNED) && !getenv("AMBC_DEFLATE_LDS")) {
            hipLaunchKernelGGL((k_deflate<CMAX, false, true>), dim3(a.n_chunks), dim3(64), 0, s, a);
            return hipGetLastError();
        }
    }
    if constexpr (CMAX >= 16384) {
        if ((a.flags & ENC_EVAL) && (a.flags & ENC_IN_ALIGNED) && !getenv("AMBC_DEFLATE_EV_LDS")) {
            hipLaunchKernelGGL((k_deflate<CMAX, true>), dim3(a.n_chunks), dim3(64), 0, s, a);
            return hipGetLastError();
        }
        static const bool gb_lds = getenv("AMBC_DEFLATE_GB_LDS") != nullptr;
        if (!(a.flags & ENC_EVAL) && (a.flags & ENC_IN_ALIGNED) && !gb_lds) {
            hipLaunchKernelGGL((k_deflate<CMAX, false, true>), dim3(a.n_chunks), dim3(64), 0, s, a);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_deflate<CMAX, false>), dim3(a.n_chunks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_deflate(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    const uint32_t C = a.chunk_size;
    if (C <= 1024) return launch_deflate_t<1024>(a, s);
    if (C <= 2048) return launch_deflate_t<2048>(a, s);
    if (C <= 4096) return launch_deflate_t<4096>(a, s);
    if (C <= 8192) return launch_deflate_t<8192>(a, s);
    if (C <= 16384) return launch_deflate_t<16384>(a, s);
    // the reference's prefs allow id 5 up to 65536 (adaptive_compressor.py:119):
    // 73 KB / 145 KB of LDS, 2 / 1 workgroups per CU
    if (C <= 32768) return launch_deflate_t<32768>(a, s);
    return launch_deflate_t<65536>(a, s);
}

}  // namespace ambc
