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

// OR nb (<= 32) bits of v into an LSB-first bit stream of u32 words at bit b
__device__ __forceinline__ void put_bits_atomic(uint32_t* words, uint32_t b, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t w = b >> 5, o = b & 31;
    atomicOr(&words[w], v << o);
    if (o + nb > 32) atomicOr(&words[w + 1], v >> (32 - o));
}

__device__ __forceinline__ void put_bits_plain(uint32_t* words, uint32_t b, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t w = b >> 5, o = b & 31;
    words[w] |= v << o;
    if (o + nb > 32) words[w + 1] |= v >> (32 - o);
}

template <int CMAX>
struct GdSmem {
    static constexpr int REGION = (CMAX > 4608 ? CMAX : 4608) + 64;
    static constexpr int MAXSEQ = CMAX / 4 + 2;
    static constexpr int ROUNDS = (CMAX + 63) / 64;
    alignas(16) uint8_t chunk[CMAX + 64];  // zero padded
    // parse: last[] (u16 x 2048) | trees: sorted/weights/parents | emit: bit staging
    alignas(16) uint32_t region[REGION / 4];
    uint16_t slen[MAXSEQ], sdist[MAXSEQ];  // the parse's matches, in order
    uint64_t sel[ROUNDS];                  // match-start positions, per 64-position round
    uint16_t sbase[ROUNDS + 1];            // first match index of every round
    uint32_t lf[288], df[32], cf[20];      // symbol frequencies
    uint8_t ll[288], dl[32], cl[20];       // code lengths
    uint16_t lc[288], dc[32], cc[20];      // bit-reversed canonical codes
    uint8_t rs[320], re[320];              // code-length RLE: symbols, extra values
    uint32_t blc[24];
    uint32_t misc[8];
};

// Huffman code lengths of freq[0..nsym) limited to maxbits (see the file
// header), on one wave.  scratch: >= 4608 bytes of LDS.
__device__ void gd_lengths(const uint32_t* freq, int nsym, int maxbits, uint8_t* len, uint32_t* scratch,
                           uint32_t* blc, uint32_t lane) {
    uint16_t* sorted = reinterpret_cast<uint16_t*>(scratch);       // 320 x u16
    uint32_t* w = scratch + 160;                                   // 640 x u32
    uint16_t* parent = reinterpret_cast<uint16_t*>(scratch + 800); // 640 x u16
    constexpr int J = 5;  // symbols lane + 64 j, nsym <= 320
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
    // rank of every used symbol among (freq, symbol)
#pragma unroll
    for (int j = 0; j < J; j++) {
        const uint32_t s = lane + 64 * j;
        if (f[j]) {
            uint32_t r = 0;
            for (int t = 0; t < nsym; t++) {
                const uint32_t ft = freq[t];
                r += ft && (ft < f[j] || (ft == f[j] && (uint32_t)t < s));
            }
            sorted[r] = (uint16_t)s;
            w[r] = f[j];
        }
    }
    wave_sync();
    // two-queue construction (serial): leaves 0..k-1, internal k..2k-2
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
    for (int i = lane; i < 24; i += 64) blc[i] = 0;
    wave_sync();
    for (uint32_t i = lane; i < k; i += 64) {
        const uint32_t d = w[parent[i]] + 1;
        atomicAdd(&blc[d > 23 ? 23 : d], 1u);
    }
    wave_sync();
    if (lane == 0) {
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
__device__ void gd_codes(const uint8_t* len, int nsym, uint16_t* rcode, uint32_t* blc, uint32_t lane) {
    constexpr int J = 5;
    for (int i = lane; i < 24; i += 64) blc[i] = 0;
    wave_sync();
    uint32_t l[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        l[j] = s < nsym ? len[s] : 0u;
        if (l[j]) atomicAdd(&blc[l[j]], 1u);
    }
    wave_sync();
    if (lane == 0) {  // next_code per length in blc[16 + ..] -- kept in registers below
        uint32_t c = 0, prev = 0;
        for (int b = 1; b < 16; b++) {
            c = (c + prev) << 1;
            prev = blc[b];
            blc[b] = c;  // first code of length b
        }
    }
    wave_sync();
    uint32_t seen[16];
#pragma unroll
    for (int b = 0; b < 16; b++) seen[b] = 0;
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        uint32_t code = 0;
#pragma unroll
        for (int b = 1; b < 16; b++) {
            const uint64_t m = __ballot(l[j] == (uint32_t)b);
            if (l[j] == (uint32_t)b) code = blc[b] + seen[b] + (uint32_t)__popcll(m & lt);
            seen[b] += (uint32_t)__popcll(m);
        }
        if (s < nsym) rcode[s] = l[j] ? (uint16_t)(__builtin_bitreverse32(code) >> (32 - l[j])) : 0;
    }
    wave_sync();
}

template <int CMAX>
__global__ __launch_bounds__(64) void k_deflate(EncArgs A) {
    __shared__ GdSmem<CMAX> S;
    constexpr int ROUNDS = GdSmem<CMAX>::ROUNDS;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = (uint64_t)k * A.chunk_size;
    const uint32_t n = (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    // prefs gate (adaptive_compressor.py:565-567) and should_use's n >= 64
    if (!((A.method_mask >> 5) & 1) || n < A.pref_min[5] || n > A.pref_max[5] || n < 64) return;
    const uint32_t w0 = A.ids[k];
    const uint32_t bestpre = A.bestpre[k];
    // id 5 wins iff len + 18 < T (ties against an LZ4 winner go to id 5)
    const uint32_t T = w0 == 9 ? min(bestpre, A.plen[k] + 18 + 1) : bestpre;
    if (T <= 18 + 6) return;
    const uint8_t* src = A.in + pos0;
    uint8_t* slot = A.slots + (uint64_t)k * A.slot_stride;

    // ---- stage, byte histogram (should_use: entropy < 8.0 <=> not exactly uniform) ----
    {
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
    uint32_t* hist = S.region;
    for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
    wave_sync();
    uint64_t asum = 0, bsum = 0;  // Adler-32 partial sums
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t c = S.chunk[i];
        atomicAdd(&hist[c], 1u);
        asum += c;
        bsum += (uint64_t)(n - i) * c;
    }
    wave_sync();
    {
        const uint32_t h0 = hist[0];
        bool diff = false;
        for (uint32_t i = lane; i < 256; i += 64) diff |= hist[i] != h0;
        if (!__any(diff)) return;  // calculate_entropy == 8.0: should_use is False
    }
    asum = wave_sum<uint64_t>(asum);
    bsum = wave_sum<uint64_t>(bsum);
    const uint32_t adler = (uint32_t)(((n + bsum) % 65521) << 16 | ((1 + asum) % 65521));
    wave_sync();

    // ---- parse ----
    uint16_t* last = reinterpret_cast<uint16_t*>(S.region);
    for (uint32_t i = lane; i < 2048; i += 64) last[i] = 0xFFFF;
    wave_sync();
    const int hl = (int)n - 4;  // last hashable position
    uint32_t p = 0, ns = 0;
#pragma unroll 1
    for (int r = 0; r < ROUNDS; r++) {
        const int base = r * 64;
        if (base >= (int)n) break;
        const int i = base + (int)lane;
        const bool act = i <= hl;
        const uint32_t v = act ? ld32(S.chunk, (uint32_t)i) : 0u;
        const uint32_t h = (v * 2654435761u) >> 21;
        uint64_t peers = __ballot(act);
#pragma unroll
        for (int b = 0; b < 11; b++) {
            const uint64_t m = __ballot((h >> b) & 1u);
            peers &= ((h >> b) & 1u) ? m : ~m;
        }
        const uint64_t lower = lane ? (peers & ((1ull << lane) - 1)) : 0ull;
        int cand;
        if (lower) {
            cand = base + 63 - (int)__clzll((long long)lower);
        } else {
            const uint16_t c = act ? last[h] : (uint16_t)0xFFFF;
            cand = c == 0xFFFF ? -1 : (int)c;
        }
        const bool valid = act && cand >= 0 && i - cand <= 32768 && ld32(S.chunk, (uint32_t)cand) == v;
        wave_sync();
        if (act && (peers >> lane) == 1ull) last[h] = (uint16_t)i;
        uint32_t L = 0;
        if (valid) {
            const uint32_t lim = min(258u, n - (uint32_t)i);
            L = 4;
            while (L < GD_LCAP && L < lim) {
                const uint32_t x = ld32(S.chunk, (uint32_t)cand + L) ^ ld32(S.chunk, (uint32_t)i + L);
                if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
                L += 4;
            }
            L = min(L, lim);
        }
        const uint64_t vm = __ballot(valid);
        uint64_t selm = 0;
        const uint32_t ns0 = ns;
        if (p < (uint32_t)base + 64) {
            // scalar greedy walk over this round's positions
            while (p < (uint32_t)base + 64 && p < n) {
                const uint64_t m = vm >> (p - (uint32_t)base);
                if (!m) { p = (uint32_t)base + 64; break; }
                p += (uint32_t)__builtin_ctzll(m);
                const uint32_t l = p - (uint32_t)base;
                uint32_t Lp = readlane(L, l);
                const uint32_t c = readlane((uint32_t)cand, l);
                const uint32_t lim = min(258u, n - p);
                if (Lp >= GD_LCAP && Lp < lim) {
                    // extend with the whole wave: 64 dwords per step
                    for (;;) {
                        const uint32_t off = Lp + 4 * lane;
                        const uint32_t x = off < lim ? (ld32(S.chunk, c + off) ^ ld32(S.chunk, p + off)) : 1u;
                        const uint64_t mm = __ballot(x != 0);
                        if (mm) {
                            const uint32_t f = (uint32_t)__builtin_ctzll(mm);
                            const uint32_t xf = readlane(x, f);
                            Lp += 4 * f + ((uint32_t)__builtin_ctz(xf) >> 3);
                            break;
                        }
                        Lp += 256;
                    }
                    Lp = min(Lp, lim);
                }
                if (lane == 0) { S.slen[ns] = (uint16_t)Lp; S.sdist[ns] = (uint16_t)(p - c); }
                selm |= 1ull << l;
                ns++;
                p += Lp;
            }
        }
        if (lane == 0) { S.sel[r] = selm; S.sbase[r] = (uint16_t)ns0; }
    }
    const uint32_t nrounds = (n + 63) / 64;
    wave_sync();

    // ---- symbol frequencies ----
    for (uint32_t i = lane; i < 288; i += 64) S.lf[i] = 0;
    if (lane < 32) S.df[lane] = 0;
    wave_sync();
    uint32_t extra = 0;
    {
        int carry = 0;  // max match end so far
        const uint64_t lt = (1ull << lane) - 1;
#pragma unroll 1
        for (uint32_t r = 0; r < nrounds; r++) {
            const uint32_t i = r * 64 + lane;
            const uint64_t sm = S.sel[r];
            const bool st = (sm >> lane) & 1;
            int e = 0;
            if (st) {
                const uint32_t si = S.sbase[r] + (uint32_t)__popcll(sm & lt);
                const uint32_t Lx = S.slen[si], Dx = S.sdist[si];
                e = (int)(i + Lx);
                const uint32_t lcd = gd_lcode(Lx), dcd = gd_dcode(Dx);
                atomicAdd(&S.lf[257 + lcd], 1u);
                atomicAdd(&S.df[dcd], 1u);
                extra += c_lext[lcd] + c_dext[dcd];
            }
            const int E = max(carry, wave_incl_max_i32(e));
            carry = max(carry, wave_max_i32(e));
            if (i < n && E <= (int)i) atomicAdd(&S.lf[S.chunk[i]], 1u);
        }
    }
    extra = wave_sum_u32(extra);
    if (lane == 0) S.lf[256] = 1;
    wave_sync();

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
    if (!dyn_possible && fix_bytes + 6 + 18 >= T) return;  // cannot win

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
        gd_lengths(S.lf, 286, 15, S.ll, S.region, S.blc, lane);
        gd_lengths(S.df, 30, 15, S.dl, S.region, S.blc, lane);
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
        // code-length RLE (serial, lane 0)
        if (lane == 0) {
            const uint32_t cnt = hlit + hdist;
            auto L = [&](uint32_t q) { return q < hlit ? S.ll[q] : S.dl[q - hlit]; };
            uint32_t q = 0, o = 0;
            while (q < cnt) {
                const uint32_t v = L(q);
                uint32_t rr = 1;
                while (q + rr < cnt && L(q + rr) == v) rr++;
                q += rr;
                if (v == 0) {
                    while (rr >= 11) { const uint32_t t = min(rr, 138u); S.rs[o] = 18; S.re[o++] = (uint8_t)(t - 11); rr -= t; }
                    if (rr >= 3) { S.rs[o] = 17; S.re[o++] = (uint8_t)(rr - 3); rr = 0; }
                    while (rr > 0) { S.rs[o] = 0; S.re[o++] = 0; rr--; }
                } else {
                    S.rs[o] = (uint8_t)v; S.re[o++] = 0; rr--;
                    while (rr >= 3) { const uint32_t t = min(rr, 6u); S.rs[o] = 16; S.re[o++] = (uint8_t)(t - 3); rr -= t; }
                    while (rr > 0) { S.rs[o] = (uint8_t)v; S.re[o++] = 0; rr--; }
                }
            }
            S.misc[2] = o;
            for (int i = 0; i < 19; i++) S.cf[i] = 0;
            for (uint32_t i = 0; i < o; i++) S.cf[S.rs[i]]++;
        }
        wave_sync();
        nr = S.misc[2];
        gd_lengths(S.cf, 19, 7, S.cl, S.region, S.blc, lane);
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
    const int kind = (dyn_bytes <= fix_bytes && dyn_bytes <= sto_bytes) ? 2 : (fix_bytes <= sto_bytes ? 1 : 0);
    const uint32_t body = kind == 2 ? dyn_bytes : kind == 1 ? fix_bytes : sto_bytes;
    const uint32_t total = 2 + body + 4;
    if (kind == 0 || total + 18 >= T) return;  // a stored block never beats raw

    // ---- emission (this chunk's winner) ----
    if (kind == 1) {  // fixed tables
        for (uint32_t s = lane; s < 288; s += 64) S.ll[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        if (lane < 30) S.dl[lane] = 5;
        wave_sync();
        gd_codes(S.ll, 288, S.lc, S.blc, lane);
        gd_codes(S.dl, 30, S.dc, S.blc, lane);
    } else {
        gd_codes(S.ll, 286, S.lc, S.blc, lane);
        gd_codes(S.dl, 30, S.dc, S.blc, lane);
        gd_codes(S.cl, 19, S.cc, S.blc, lane);
    }
    uint32_t* bits = S.region;
    const uint32_t nwords = (body + 8) / 4 + 1;
    for (uint32_t i = lane; i < nwords; i += 64) bits[i] = 0;
    wave_sync();
    uint32_t bp = 0;
    if (lane == 0) {
        put_bits_plain(bits, 0, 1u | ((uint32_t)kind << 1), 3);
        bp = 3;
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
    {
        int carry = 0;
        const uint64_t lt = (1ull << lane) - 1;
#pragma unroll 1
        for (uint32_t r = 0; r < nrounds; r++) {
            const uint32_t i = r * 64 + lane;
            const uint64_t sm = S.sel[r];
            const bool st = (sm >> lane) & 1;
            int e = 0;
            uint32_t Lx = 0, Dx = 0, lcd = 0, dcd = 0, cost = 0;
            if (st) {
                const uint32_t si = S.sbase[r] + (uint32_t)__popcll(sm & lt);
                Lx = S.slen[si];
                Dx = S.sdist[si];
                e = (int)(i + Lx);
                lcd = gd_lcode(Lx);
                dcd = gd_dcode(Dx);
                cost = S.ll[257 + lcd] + c_lext[lcd] + S.dl[dcd] + c_dext[dcd];
            }
            const int E = max(carry, wave_incl_max_i32(e));
            carry = max(carry, wave_max_i32(e));
            const bool lit = i < n && E <= (int)i;
            const uint32_t c = lit ? S.chunk[i] : 0u;
            if (lit) cost = S.ll[c];
            const uint32_t incl = wave_incl_sum(cost);
            uint32_t b = bp + incl - cost;
            if (lit) {
                put_bits_atomic(bits, b, S.lc[c], S.ll[c]);
            } else if (st) {
                put_bits_atomic(bits, b, S.lc[257 + lcd], S.ll[257 + lcd]); b += S.ll[257 + lcd];
                put_bits_atomic(bits, b, Lx - c_lbase[lcd], c_lext[lcd]); b += c_lext[lcd];
                put_bits_atomic(bits, b, S.dc[dcd], S.dl[dcd]); b += S.dl[dcd];
                put_bits_atomic(bits, b, Dx - c_dbase[dcd], c_dext[dcd]);
            }
            bp += readlane(incl, 63);
        }
    }
    wave_sync();
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
    if (lane == 0) {
        A.ids[k] = 5;
        A.plen[k] = total;
        A.sizes[k] = 18ull + total;
    }
}

template <int CMAX>
hipError_t launch_deflate_t(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_deflate<CMAX>, dim3(a.n_chunks), dim3(64), 0, s, a);
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
    return launch_deflate_t<16384>(a, s);
}

}  // namespace ambc
