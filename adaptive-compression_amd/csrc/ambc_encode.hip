// ambc_encode.hip -- per-chunk method selection + encoders for gfx950.
//
// One 64-lane workgroup (one wavefront) owns one chunk.  The chunk is staged
// in LDS with 16-byte loads, and the wave then runs, in the reference's method
// order (ids ascending, strict "<" -- adaptive_compressor.py:559-584):
//
//   pass A  byte histogram (run-merged LDS atomics), RLE pair count (runs split
//           at 255, compression_methods.py:95-109) and the RLE should_use
//           sample count (:168-180) -- one sweep, 64 contiguous bytes per lane
//   RLE     exact payload size 2*pairs
//   Huffman should_use entropy (fp64; numpy-exact terms for near-ties,
//           :562-574), tree by repeated wave-min merges of (weight, first
//           symbol) keys (:482-494), exact payload size 1+5k+4+ceil(bits/8)
//   LZ4     "ambc-lz4 greedy v2": per 64-position window, candidates from an
//           LDS hash table of the earlier windows (ds_max keeps each hash's
//           last position; the first window resolves its own repeats by
//           ballots), then a wave-cooperative greedy walk that emits straight
//           into the chunk's scratch slot and gives up as soon as it cannot
//           beat the best so far
//   emit    the winner's payload into the slot (raw / RLE / Huffman bits)
//
// Work is integer/byte work bound by LDS and issue, not by HBM: every input
// byte is read from HBM once (16 B per lane per load), the payload is written
// once to its slot, and k_compact then moves it to its final byte offset.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {

template <int CMAX, bool GL = false>
struct EncSmem {
    // work = union, by lifetime.  Selection: hist | Huffman tree (parent / pbit,
    // whose space the first occurrences first / order reuse once the codes are
    // known) | clen | code.  LZ4: the hash table (u32 per bucket) over all of it.
    // Emit: RLE pair starts, or the Huffman bit stage over everything below clen
    // (the table is written before the stage is filled).  4 KB per workgroup: 32
    // workgroups (8 waves per SIMD) fit a CU.
    //   0    .. 1023  hist u32[256]                        | stage
    //   1024 .. 2047  parent u16[512]  | first u32[256]     | stage
    //   2048 .. 2559  pbit u8[512]     | order u8[256]      | stage
    //   2816 .. 3071  clen u8[256]
    //   3072 .. 4095  code u32[256]
    static constexpr int WORK = 4096;   // every chunk size
    static constexpr int STAGE = 2816;  // Huffman bit stage (a larger payload goes in windows)
    // zero padded up to CMAX; reads past CMAX (the LZ4 loads of lanes beyond n,
    // match lengths capped below n) land in work[], which follows: in bounds,
    // and never part of a result
    alignas(16) uint8_t chunk[GL ? 16 : CMAX];   // GL: the chunk is read in place from the input
    alignas(16) uint32_t work[WORK / 4];
    __device__ __forceinline__ uint8_t* wb() { return reinterpret_cast<uint8_t*>(work); }
    __device__ __forceinline__ uint32_t* hist() { return work; }
    __device__ __forceinline__ uint16_t* parent() { return reinterpret_cast<uint16_t*>(wb() + 1024); }
    __device__ __forceinline__ uint8_t* pbit() { return wb() + 2048; }
    __device__ __forceinline__ uint32_t* first() { return reinterpret_cast<uint32_t*>(wb() + 1024); }
    __device__ __forceinline__ uint8_t* order() { return wb() + 2048; }
    __device__ __forceinline__ uint8_t* clen() { return wb() + 2816; }
    __device__ __forceinline__ uint32_t* code() { return reinterpret_cast<uint32_t*>(wb() + 3072); }
    __device__ __forceinline__ uint32_t* last() { return work; }
    __device__ __forceinline__ uint32_t* stage() { return work; }
};
static_assert((1u << LZ4_HASH_BITS) * 4 <= 4096, "LZ4 table must fit the work area");

// Visit the bytes of a lane's block [b0, b0+BS) 16 at a time (one ds_read_b128
// per step; the 16-byte body is unrolled, the sub-block loop is not, which
// keeps the kernel small enough for the instruction cache).
// f(p, c, nx): position, byte, following byte (zero padding past the data).
// lim: 16-byte pieces starting at or past lim read as zeros -- a chunk read in
// place (GL) may end its input there (the input has 64 readable bytes after its
// end, not a whole lane block's); LDS-staged chunks are zero padded already.
template <int BS, typename F>
__device__ __forceinline__ void for_block_bytes(const uint8_t* chunk, uint32_t b0, uint32_t lim, F&& f) {
#pragma unroll 1
    for (int q = 0; q < BS / 16; q++) {
        const uint32_t base = b0 + 16 * q;
        const bool in = base < lim;
        const uint4 v = in ? *reinterpret_cast<const uint4*>(chunk + base) : make_uint4(0, 0, 0, 0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const uint32_t nxt = in ? chunk[base + 16] : 0u;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint32_t c = (w[t >> 2] >> (8 * (t & 3))) & 0xFFu;
            const uint32_t nx = t < 15 ? ((w[(t + 1) >> 2] >> (8 * ((t + 1) & 3))) & 0xFFu) : nxt;
            f(base + t, c, nx);
        }
    }
}

// unaligned 4-byte little-endian read from LDS via two aligned dword reads
__device__ __forceinline__ uint32_t lds_rd32(const uint8_t* base, uint32_t i) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base);
    const uint32_t a = i >> 2;
    return __builtin_amdgcn_alignbyte(w[a + 1], w[a], i & 3);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// XXH32 of the 10-byte LZ4 frame descriptor (FLG, BD, content size)
__device__ uint32_t xxh32_desc(uint32_t n) {
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U,
                   P5 = 374761393U;
    uint32_t h = P5 + 10u;
    h = rotl32(h + (0x68u | 0x40u << 8 | (n & 0xFFFFu) << 16) * P3, 17) * P4;
    h = rotl32(h + (n >> 16) * P3, 17) * P4;
    h = rotl32(h + 0u * P5, 11) * P1;
    h = rotl32(h + 0u * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint32_t ext_len(uint32_t v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// byte t of an LZ4 length extension for value v (>= 15) of xl bytes
__device__ __forceinline__ uint32_t ext_byte(uint32_t v, uint32_t xl, uint32_t t) {
    return t + 1 < xl ? 255u : (v - 15) % 255u;
}

// frame header byte q (0..18) of a one-block LZ4F frame; bs = block size field
__device__ __forceinline__ uint8_t lz4_hdr_byte(uint32_t q, uint32_t n, uint32_t bs) {
    if (q < 4) return (uint8_t)(0x184D2204u >> (8 * q));
    if (q == 4) return 0x68;   // FLG: v01, block independence, content size
    if (q == 5) return 0x40;   // BD: 64 KiB max block
    if (q < 14) return q < 10 ? (uint8_t)(n >> (8 * (q - 6))) : 0;
    if (q == 14) return (uint8_t)((xxh32_desc(n) >> 8) & 0xFF);
    return (uint8_t)(bs >> (8 * (q - 15)));
}

// len bytes from LDS (src: 4-byte aligned) to global memory at any alignment: the
// destination's aligned 16-byte groups one per lane and step (five LDS dwords
// shifted into place), the bytes before and after them one per lane
__device__ __forceinline__ void lds_store_bytes(uint8_t* dst, const uint8_t* src, uint32_t len, uint32_t lane) {
    const uint64_t da = reinterpret_cast<uintptr_t>(dst);
    const uint64_t g0 = (da + 15) >> 4, g1 = (da + len) >> 4;
    const uint32_t ng = g1 > g0 ? (uint32_t)(g1 - g0) : 0u;
    const uint32_t head = ng ? (uint32_t)((g0 << 4) - da) : len;
    const uint32_t tail0 = ng ? head + 16 * ng : len;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    const uint32_t sh = head & 3u;
    for (uint32_t j = lane; j < ng; j += 64) {
        const uint32_t q = (head >> 2) + 4 * j;
        const uint32_t a0 = s32[q], a1 = s32[q + 1], a2 = s32[q + 2], a3 = s32[q + 3];
        const uint32_t a4 = sh ? s32[q + 4] : 0u;
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(a1, a0, sh);
        v.y = __builtin_amdgcn_alignbyte(a2, a1, sh);
        v.z = __builtin_amdgcn_alignbyte(a3, a2, sh);
        v.w = __builtin_amdgcn_alignbyte(a4, a3, sh);
        reinterpret_cast<uint4*>(g0 << 4)[j] = v;
    }
    for (uint32_t q = lane; q < head; q += 64) dst[q] = src[q];
    for (uint32_t q = tail0 + lane; q < len; q += 64) dst[q] = src[q];
}

#ifdef AMBC_STAMPS
// diagnostic build only: per-chunk phase cycle sums via s_memtime, written once
// per chunk to A.stamps[k*8 + phase] (no atomics, so phases are not perturbed)
#define STAMP_DECL uint64_t _st_t = __builtin_amdgcn_s_memtime(); uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(ph)                                                  \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _acc[ph] += _t - _st_t;                                    \
        _st_t = _t;                                                \
    } while (0)
#define STAMP_FLUSH                                                \
    if (lane == 0 && A.stamps)                                     \
        for (int _p = 0; _p < 8; _p++) A.stamps[(uint64_t)k * 8 + _p] = _acc[_p];
#else
#define STAMP_DECL
#define STAMP(ph) do {} while (0)
#define STAMP_FLUSH
#endif

__device__ __forceinline__ uint32_t hdr_byte(uint32_t q, uint32_t type, uint32_t n, uint32_t clen) {
    if (q < 4) return q < 2 ? 0xFFu : 0u;       // marker ff ff 00 00
    if (q == 4) return type;
    if (q == 5) return 0;                        // k_value
    if (q < 10) return (n >> (8 * (q - 6))) & 0xFF;      // used_bytes
    if (q < 14) return (n >> (8 * (q - 10))) & 0xFF;     // original_length
    return (clen >> (8 * (q - 14))) & 0xFF;              // compressed_length
}

// GL (chunks of 4 KiB and more, no forced / analysed encode, 16-byte aligned
// chunk starts): the chunk is read in place from the input through the caches
// instead of a CMAX-byte LDS copy -- only LZ4 (and id 5's gates) take such
// chunks, and a 64 KiB chunk in LDS held the CU to 2 workgroups, one wave
// each, through 1024 latency-bound LZ4 rounds; in place, the work area alone
// (4 KB) lets 20 workgroups share the CU.  Reads past n stay inside the input's
// 64 bytes of slack or the next chunk and never reach a result.
// MODE (compile time, so that the headline's kernel carries none of the rest):
// ENC_MODE_PLAIN compress / plugins; ENC_MODE_WALK the multi-size walk's
// decision-only batches (ENC_EVAL, lz4sub).  (Direct emission to final offsets
// was measured in round 3 and removed: profiles/r3_direct_emission_ab.json.)
enum : int { ENC_MODE_PLAIN = 0, ENC_MODE_WALK = 1 };
// Register allocation for 8 waves per SIMD (64 VGPRs, a few spilled bytes): with
// the chunk read in place the LDS no longer caps k_encode at 5 waves, and the
// VALU-issue-bound LZ4 rounds gain from the extra waves -- same-box A/B, 4 GiB
// (profiles/r3_wpe_ab.json): 4 KiB 3.08 -> 2.86 ms per launch, 8 KiB 3.70 -> 3.48;
// 6 waves (71 VGPRs) was slower at 8 KiB.  AMBC_WPE=0 builds the compiler's own
// allocation (94 VGPRs, 5 waves).
#ifndef AMBC_WPE
#define AMBC_WPE 8
#endif
#if AMBC_WPE
#define AMBC_ENC_ATTR __attribute__((amdgpu_waves_per_eu(AMBC_WPE, AMBC_WPE)))
#else
#define AMBC_ENC_ATTR
#endif
template <int CMAX, bool GL = false, int MODE = ENC_MODE_PLAIN>
__global__ __launch_bounds__(64) AMBC_ENC_ATTR void k_encode(EncArgs A) {
    constexpr int BS = CMAX >= 4096 ? 64 : CMAX / 64;  // bytes per lane per round
    constexpr int ROUNDS = CMAX / (64 * BS);
    __shared__ EncSmem<CMAX, GL> S;

    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    const uint8_t* src = A.in + pos0;
    uint8_t* const slot0 = A.slots + (uint64_t)k * A.slot_stride;   // the chunk's scratch slot
    uint8_t* slot = slot0;              // where the payload goes
    // second pass after k_deflate: only the deferred chunks id 5 did not take
    if ((A.flags & ENC_EMIT_PENDING) && (!A.pending[k] || A.ids[k] == 5 || A.ids[k] == 2)) return;
    STAMP_DECL

    // ---- stage the chunk in LDS (16 B per lane per load, coalesced) ----
    const uint8_t* ch = GL ? src : S.chunk;
    // (for_block_bytes: in place, nothing is read from 16-byte pieces past n)
#define GLLIM (GL ? n : 0xFFFFFFFFu)
    if constexpr (GL) {
        for (uint32_t i = lane; i < 256; i += 64) S.hist()[i] = 0;
    } else {
        const uint32_t nv = n >> 4;
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            for (uint32_t v = lane; v < nv; v += 64)
                reinterpret_cast<uint4*>(S.chunk)[v] = reinterpret_cast<const uint4*>(src)[v];
            for (uint32_t i = (nv << 4) + lane; i < n; i += 64) S.chunk[i] = src[i];
        } else {
            for (uint32_t i = lane; i < n; i += 64) S.chunk[i] = src[i];
        }
        for (uint32_t i = n + lane; i < (uint32_t)CMAX; i += 64) S.chunk[i] = 0;
        for (uint32_t i = lane; i < 256; i += 64) S.hist()[i] = 0;
    }
    wave_sync();

    // ---- pass A: histogram, RLE pairs, RLE / Delta should_use samples ----
    // Word-parallel: per dword, the bytes that differ from their predecessor (a
    // run starts there) as bit 8j+7 of chg.  RLE pairs = run starts + the
    // 255-byte splits of the run carried into the lane (a run that starts inside
    // a lane is shorter than 255 there); the should_use samples at step 4 are
    // byte 0 against byte 1 of each dword; the histogram adds whole runs.
    const uint32_t mm = A.method_mask;
    const bool force = A.flags & ENC_FORCE;
    const bool analyze = A.flags & ENC_ANALYZE;
    auto eligible = [&](int id) {
        return ((mm >> id) & 1u) && (force || (A.pref_min[id] <= n && n <= A.pref_max[id]));
    };
    // pass A feeds RLE, Huffman, Delta, the should_use report and k_deflate's
    // gates; chunks only LZ4 may take (above Huffman's 8192 by the prefs) skip it
    const bool need_a = force || analyze || A.bestpre || eligible(1) || eligible(3) || eligible(4);
    // within it: RLE's pair count, and the RLE / Delta should_use samples (chunks
    // above 4096 -- C4's 8192 -- keep only Huffman's histogram)
    const bool need_p = force || analyze || eligible(1);
    const bool need_s = need_p || eligible(4);
    const uint32_t ss = n < 1000 ? n : 1000;
    const uint32_t step = max(1u, n / ss);
    const bool fast_samples = step == 4;
    uint32_t pairs = 0, samp = 0, dsamp = 0;
    int rs_carry = -1;
    uint32_t pw_carry = 0;      // the previous round's last dword (lane 63's block end)
#pragma unroll 1
    for (int r = 0; r < (need_a ? ROUNDS : 0); r++) {
        const uint32_t b0 = (uint32_t)(r * 64 + lane) * BS;
        // (GL: a lane block starting at or past n is masked by nv below -- its load
        // is clamped to the last 16-aligned BS bytes the 64-byte input padding covers)
        // The block's 16-byte loads issue together and unconditionally, ahead of the
        // LDS atomics (which the compiler will not move loads across): the chunk's
        // first read from HBM waits one latency, not one per piece, and no other
        // load precedes it -- the run byte is the block's first, the previous
        // word the previous lane's last (lane 0: the previous round's lane 63)
        const uint32_t ab = GL ? min(b0, (n + 64u - (uint32_t)BS) & ~15u) : b0;
        uint4 pv[BS / 16];
#pragma unroll
        for (int q = 0; q < BS / 16; q++)   // (a masked block's bytes are never counted)
            pv[q] = *reinterpret_cast<const uint4*>(ch + ab + 16 * q);
        const uint32_t lastw = pv[BS / 16 - 1].w;
        // previous byte; position 0 always starts a run (the reference's prev = None)
        uint32_t pw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + 63u) & 63u) << 2), (int)lastw);
        if (lane == 0) pw = r ? pw_carry : ~((pv[0].x & 0xFFu) << 24);
        pw_carry = readlane(lastw, 63);
        int lb = -1, fc = -1;
        uint32_t starts = 0, cur = pv[0].x & 0xFFu, rc = 0;
#pragma unroll
        for (int q = 0; q < BS / 16; q++) {
            const uint4 v4 = pv[q];
            const uint32_t wv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const uint32_t w = wv[e];
                const uint32_t p = b0 + 16 * q + 4 * e;
                const uint32_t x = w ^ __builtin_amdgcn_alignbyte(w, pw, 3);
                const uint32_t nv = p < n ? min(n - p, 4u) : 0u;       // valid bytes
                const uint32_t vmask = nv >= 4 ? 0xFFFFFFFFu : (1u << (8 * nv)) - 1u;
                const uint32_t chg = (x | ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu)) & 0x80808080u & vmask;
                if (need_p) {
                    starts += __builtin_popcount(chg);
                    if (chg) {
                        lb = (int)(p + ((31 - __builtin_clz(chg)) >> 3));
                        if (fc < 0) fc = (int)(p + ((uint32_t)__builtin_ctz(chg) >> 3));
                    }
                }
                if (need_s && fast_samples && p + 1 < n) {      // sample p: byte 0 against byte 1
                    const uint32_t a0 = w & 0xFFu, a1 = (w >> 8) & 0xFFu;
                    samp += (chg & 0x8000u) == 0;
                    dsamp += (a0 > a1 ? a0 - a1 : a1 - a0) < 32u;
                }
                if (chg == 0) {
                    rc += nv;                         // the current run goes on
                } else {
                    // a run ends in this dword: flush the run carried in and count
                    // the dword's bytes one by one (branch-free); the last byte's
                    // run carries on with nothing counted yet
                    atomicAdd(&S.hist()[cur], rc);
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        atomicAdd(&S.hist()[(w >> (8 * j)) & 0xFFu], (uint32_t)j < nv ? 1u : 0u);
                    cur = w >> 24;
                    rc = 0;
                }
                pw = w;
            }
        }
        if (rc) atomicAdd(&S.hist()[cur], rc);
        if (need_p) {
            const int rs = wave_excl_max(lb, rs_carry);  // run start of position b0-1
            rs_carry = max(rs_carry, wave_max_i32(lb));
            // 255-byte splits of the carried-in run inside [b0, first run start)
            const int end = fc >= 0 ? fc : (int)min(b0 + BS, n);
            if (b0 && end > (int)b0) starts += (uint32_t)((end - 1 - rs) / 255 - ((int)b0 - 1 - rs) / 255);
            pairs += starts;
        }
        if (need_s && !fast_samples) {
            // other steps: positions p = step * i in the lane's block
#pragma unroll 1
            for (uint32_t p = (b0 + step - 1) / step * step; p < b0 + BS && p + 1 < n; p += step) {
                const uint32_t c = ch[p], nx = ch[p + 1];
                samp += c == nx;
                dsamp += (c > nx ? c - nx : nx - c) < 32u;
            }
        }
    }
    pairs = wave_sum_u32(pairs);
    samp = wave_sum_u32(samp);
    dsamp = wave_sum_u32(dsamp);
    wave_sync();
    STAMP(0);

    // best (len + 18); (len+18)/n < 1.0  <=>  len + 18 < n (adaptive_compressor.py:573-577)
    uint32_t best = force ? 0xFFFFFFFFu : n;
    uint32_t win = 255, wlen = n;

    // ---- RLE (id 1) ----
    const bool rle_su = n >= 4 && ((double)samp / (double)(ss - 1)) > 0.3;
    const bool delta_su = n >= 4 && ((double)dsamp / (double)(ss - 1)) > 0.5;
    if (eligible(1) && (force || rle_su)) {
        const uint32_t l = 2 * pairs;
        if (l + HDR < best) { best = l + HDR; win = 1; wlen = l; }
    }

    // ---- Huffman (id 3) ----
    auto compute_first = [&]() {
        // first occurrence per symbol (Counter insertion order) and the ranked order
        uint32_t* first = S.first();
        for (uint32_t i = lane; i < 256; i += 64) first[i] = 0xFFFFFFFFu;
        wave_sync();
#pragma unroll 1
        for (int r = 0; r < ROUNDS; r++) {
            const uint32_t b0 = (uint32_t)(r * 64 + lane) * BS;
            uint32_t prev = b0 ? (b0 - 1 < GLLIM ? (uint32_t)ch[b0 - 1] : 0u) : 0x100u;
            // (the read first: once a lower block has posted a symbol, later
            // occurrences skip the atomic -- most bytes of a text chunk)
            for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t c, uint32_t) {
                if (p < n && c != prev && first[c] > p) atomicMin(&first[c], p);
                prev = c;
            });
        }
        wave_sync();
        // the present symbols as (first position << 8 | symbol), compacted in
        // symbol order over first[], then each ranked by the positions before it
        uint32_t f[4];
#pragma unroll
        for (int j = 0; j < 4; j++) f[j] = first[lane + 64 * j];
        wave_sync();
        uint32_t K = 0;
        const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool pr = f[j] != 0xFFFFFFFFu;
            const uint64_t m = __ballot(pr);
            if (pr) first[K + (uint32_t)__popcll(m & lt)] = f[j] << 8 | (lane + 64 * j);
            K += (uint32_t)__popcll(m);
        }
        wave_sync();
        for (uint32_t q = lane; q < K; q += 64) {
            const uint32_t key = first[q];
            uint32_t rk = 0;
#pragma unroll 4
            for (uint32_t t = 0; t < K; t++) rk += first[t] < key;
            S.order()[rk] = (uint8_t)key;
        }
        wave_sync();
    };

    uint32_t kdist = 0;
    // Huffman payload bits by the merges of the heapq order (:482-494): merge the
    // two smallest (weight, first symbol) keys -- slot s holds the active node
    // whose first symbol is s -- and every merge adds its weight once per level
    // below it, so the encoded length is the sum of the merged weights.  The tree
    // is recorded on the way (parent / pbit of each merged node) for the emission.
    // (measured: re-running the merges at emission instead -- {1,3,4} ASCII 0.81 ->
    // 0.97 ms, mixed 0.92 -> 1.22 ms per 256 MiB; the headline's set unchanged,
    // profiles/r5_huff_ab)
    bool tree_ok = false;    // parent / pbit hold this chunk's tree (the LZ4 table overlays them)
    auto huff_merge = [&]() -> uint32_t {
        uint32_t key[4], nid[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t sy = lane + 64 * j, c = S.hist()[sy];
            key[j] = c ? (c << 8 | sy) : 0xFFFFFFFFu;
            nid[j] = sy;
        }
        uint32_t nb = 0;
#pragma unroll 1
        for (uint32_t m = 0; m + 1 < kdist; m++) {
            const uint32_t lm = min(min(key[0], key[1]), min(key[2], key[3]));
            const uint32_t k1 = wave_min_u32(lm);
            uint32_t lm2 = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < 4; j++) if (key[j] != k1) lm2 = min(lm2, key[j]);
            const uint32_t k2 = wave_min_u32(lm2);
            const uint32_t s1 = k1 & 255u, s2 = k2 & 255u;
            const uint32_t wsum = (k1 >> 8) + (k2 >> 8);
            nb += wsum;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (lane + 64 * j == s1) {
                    S.parent()[nid[j]] = (uint16_t)(256 + m); S.pbit()[nid[j]] = 0;
                    key[j] = wsum << 8 | s1; nid[j] = 256 + m;
                } else if (lane + 64 * j == s2) {
                    S.parent()[nid[j]] = (uint16_t)(256 + m); S.pbit()[nid[j]] = 1;
                    key[j] = 0xFFFFFFFFu;
                }
            }
        }
        wave_sync();
        tree_ok = true;
        return nb;
    };
    // code lengths / codes into clen[] / code[] from the recorded tree (kdist >= 2):
    // every symbol walks to the root; the edge next to the root is the code's MSB
    auto huff_codes = [&]() {
        const uint32_t root = 256 + kdist - 2;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t sy = lane + 64 * j;
            if (S.hist()[sy]) {
                uint32_t nd = sy, len = 0, cd = 0;
                while (nd != root) {
                    if (len < 32) cd |= (uint32_t)S.pbit()[nd] << len;
                    len++;
                    nd = S.parent()[nd];
                }
                S.clen()[sy] = (uint8_t)min(len, 255u);
                S.code()[sy] = cd;
            }
        }
        wave_sync();
    };

    bool huff_su = false;
    bool huff_defer = false;
    uint32_t huff_lb = 0;
    if ((eligible(3) || analyze) && (n >= 100 || force)) {
        double part = 0.0;
        uint32_t kc = 0;
        // numpy's per-count terms p log2 p, tabulated on the host for full chunks
        // and the tail (an fp64 log2 per symbol cost ~6 % of a mixed chunk's issue)
        const double* etab = n == A.chunk_size ? A.ent_full : A.ent_tail;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t c = S.hist()[lane + 64 * j];
            if (c) {
                kc++;
                if (etab) {
                    part += etab[c];
                } else {
                    const double p = (double)c / (double)n;
                    part += p * log2(p);
                }
            }
        }
        kdist = wave_sum_u32(kc);
        double tot = wave_sum(part);
        double H = -__shfl(tot, 0);
        if (fabs(H - 7.0) <= 1e-9) {
            // near the threshold: reproduce numpy's sequential sum in first-occurrence order
            compute_first();
            const double* tab = n == A.chunk_size ? A.ent_full : A.ent_tail;
            double e = 0.0;
            if (lane == 0) {
                for (uint32_t q = 0; q < kdist; q++) {
                    const uint32_t c = S.hist()[S.order()[q]];
                    double t;
                    if (tab) t = tab[c];
                    else { const double p = (double)c / (double)n; t = p * log2(p); }
                    e = e - t;
                }
            }
            H = __shfl(e, 0);
        }
        huff_su = n >= 100 && H < 7.0;
        if (eligible(3) && (force || huff_su) && kdist >= 2 && kdist <= 255) {
            if (!force && !analyze && !A.bestpre && eligible(9) && n >= 1024) {
                // LZ4 goes first; Huffman's exact size only if its entropy bound
                // (average code length >= H) could still beat or tie LZ4's
                huff_defer = true;
                huff_lb = 1 + 5 * kdist + 4 + (uint32_t)floor((double)n * H * (1.0 - 1e-9) / 8.0);
            } else {
                // (code lengths stay <= 23 for n <= 65536: a Fibonacci-weighted tree)
                const uint32_t nb = huff_merge();
                const uint32_t l = 1 + 5 * kdist + 4 + (nb + 7) / 8;
                if (l + HDR < best) { best = l + HDR; win = 3; wlen = l; }
            }
        }
    }

    STAMP(1);
    // ---- LZ4 (id 9): frame = 15 B header + 4 B block size + block + 4 B end mark ----
    // "ambc-lz4 greedy v2": cand(i) = last j with the same 10-bit hash among the
    // earlier 64-position windows (j < 64*floor(i/64); in the first window any
    // j < i), valid iff the 4 bytes match; greedy from the first valid
    // position; matches start at i <= n-12 and end by n-5 (LZ4 block end rules).
    if (A.bestpre) {
        // for k_deflate: the best (len + 18) before LZ4, and bit 31 = DEFLATE's
        // should_use is False (calculate_entropy == 8.0: an exactly uniform histogram)
        // bit 30 = a single byte value (k_deflate builds that parse directly)
        const uint32_t h0 = S.hist()[0];
        bool diff = false;
        uint32_t nz = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            diff |= S.hist()[lane + 64 * j] != h0;
            nz += S.hist()[lane + 64 * j] != 0;
        }
        const bool uniform = !__any(diff);
        const bool single = wave_sum_u32(nz) == 1;
        if (lane == 0) A.bestpre[k] = best | (uniform ? 0x80000000u : 0u) | (single ? 0x40000000u : 0u);
    }
    const uint32_t best_pre = best;   // before LZ4 (a deferred Huffman compares against it)
    const bool eval = MODE == ENC_MODE_WALK && (A.flags & ENC_EVAL);
    // prefix sizes to report (ENC_EVAL + lz4sub): sub_c[sj..sj_end) -- ascending,
    // below n, within id 9's prefs; they end in order as the parse passes b - 12
    uint32_t sj = 0, sj_end = 0;
    if (MODE == ENC_MODE_WALK && A.lz4sub && ((mm >> 9) & 1u)) {
        while (sj < A.n_subc && A.sub_c[sj] < max(A.pref_min[9], 13u)) sj++;
        sj_end = sj;
        while (sj_end < A.n_subc && A.sub_c[sj_end] < n && A.sub_c[sj_end] <= A.pref_max[9]) sj_end++;
    }
    // LZ4's frame is at least 23 + 10 + ext(n - 10) bytes: a literal at 0 (no
    // candidate), one match up to n - 5, the last five bytes literal; with the
    // 18-B header it cannot win unless best > 51 + ext(n - 10) (zero runs: RLE 52)
    const bool lz4_main = eligible(9) && (force || (n >= 1024 && best > 51 + ext_len(n - 10)));
    if (lz4_main || sj < sj_end) {
        // the walk's hash table overlays hist[] and the tree: keep the counts in registers
        tree_ok = false;
        uint32_t hsave[4];
#pragma unroll
        for (int j = 0; j < 4; j++) hsave[j] = S.hist()[lane + 64 * j];
        wave_sync();
        uint32_t* last = S.last();          // 1 + last position per hash, 0 = none
        for (uint32_t i = lane; i < (1u << LZ4_HASH_BITS); i += 64) last[i] = 0;
        wave_sync();
        // LZ4 wins iff block < budget; forced (single-method) encodes fall back to a
        // stored block once the compressed block would reach n (LZ4F rule)
        // (the walk's control values are wave-uniform; said so explicitly, the loop
        // compiles to scalar branches instead of exec-mask bookkeeping per round)
        const uint32_t budget = __builtin_amdgcn_readfirstlane(force ? n : best - 41);
        const int mlim = __builtin_amdgcn_readfirstlane((int)n - 12);   // last match start; <0: none
        uint8_t* blk = slot + 19;
        uint32_t emitted = 0, anchor = 0, nextp = 0;
        bool alive = __builtin_amdgcn_readfirstlane((int)lz4_main) != 0;   // its own LZ4 can still win
        sj = __builtin_amdgcn_readfirstlane(sj);
        sj_end = __builtin_amdgcn_readfirstlane(sj_end);
        constexpr uint32_t LCAP = 16;       // per-lane precomputed match length cap
        // prefix sub_c[sj] is done: its block = emitted + add (this round's sequences
        // that start by b - 12) + the final literals from endp
        auto sub_done = [&](uint32_t add, uint32_t endp) {
            const uint32_t b = A.sub_c[sj];
            const uint32_t fl = b - endp;
            if (lane == 0) A.lz4sub[(uint64_t)k * LZ4_SUB_MAX + sj] = emitted + add + 1 + ext_len(fl) + fl;
            sj++;
        };
        // The probe runs a round ahead, its loads kept as raw aligned words until
        // used, so their waits fall in the next round: round r + 1's candidates
        // (the table then holds windows <= r, as the serial order needs) and their
        // bytes, and round r + 2's own bytes (position i's word from dwords i/4
        // and i/4 + 1, shift i & 3 = lane & 3).  The loads are unconditional, their
        // addresses clamped into the padded input (a last round's results go
        // unused), so the in-order load counter stays exact across the loop.
        // Same-box A/B (profiles/r5_lz4_prefetch_ab): headline 371 -> 406 GB/s.
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(ch);
        const uint32_t sh = lane & 3u;
        uint32_t nlo = 0, nhi = 0;
        auto raw_at = [&](uint32_t pos, uint32_t& lo, uint32_t& hi) { lo = w32[pos >> 2]; hi = w32[(pos >> 2) + 1]; };
        uint32_t v_cur = 0, clo = 0, chi = 0;
        int c_cur = -1;
        if (mlim >= 0) {
            v_cur = lds_rd32(ch, min(lane, n));
            const uint32_t h = (v_cur * 2654435761u) >> (32 - LZ4_HASH_BITS);
            // first window: the highest lower lane with my hash (peers by one ballot per bit)
            uint64_t peers = ~0ull;
#pragma unroll
            for (int b = 0; b < (int)LZ4_HASH_BITS; b++) {
                const uint64_t m = __ballot((h >> b) & 1u);
                peers &= ((h >> b) & 1u) ? m : ~m;
            }
            const uint64_t lower = peers & ((1ull << lane) - 1ull);
            c_cur = lower ? 63 - (int)__clzll((long long)lower) : -1;
            atomicMax(&last[h], lane + 1u);   // the window's highest position per hash
            raw_at((uint32_t)max(c_cur, 0), clo, chi);
            raw_at(min(lane + 64u, n), nlo, nhi);
        }
#pragma unroll 1
        for (int base = 0; base <= mlim && (alive || sj < sj_end); base += 64) {
            // control state is wave-uniform: keep it in SGPRs
            nextp = __builtin_amdgcn_readfirstlane(nextp);
            anchor = __builtin_amdgcn_readfirstlane(anchor);
            emitted = __builtin_amdgcn_readfirstlane(emitted);
            const int i = base + (int)lane;
            const bool act = i <= mlim;
            const uint32_t v = v_cur;
            const int cand = c_cur;
            // (this round's candidate bytes are consumed before their registers take
            // the next round's: no copy, and no wait, at the loop's back edge)
            const uint32_t cv = __builtin_amdgcn_alignbyte(chi, clo, (uint32_t)max(cand, 0) & 3u);
            {
                // next round's probe: the last earlier window's position with its hash
                const uint32_t vn = __builtin_amdgcn_alignbyte(nhi, nlo, sh);
                const uint32_t hn = (vn * 2654435761u) >> (32 - LZ4_HASH_BITS);
                c_cur = (int)last[hn] - 1;
                atomicMax(&last[hn], (uint32_t)i + 65u);
                v_cur = vn;
                uint32_t ca = (uint32_t)max(c_cur, 0), na = min((uint32_t)i + 128u, n);
                asm volatile("" : "+v"(ca), "+v"(na) : "v"(cv));   // (issued after cv is formed)
                raw_at(ca, clo, chi);
                raw_at(na, nlo, nhi);
            }
            const bool valid = act && cand >= 0 && cv == v;
            const uint64_t vm = __ballot(valid);
            wave_sync();
            STAMP(2);
            if (base + 63 < (int)nextp) continue;   // round lies inside the previous match
            uint32_t p = __builtin_amdgcn_readfirstlane((int)nextp > base ? nextp - (uint32_t)base : 0u);
            if ((vm & (~0ull << p)) == 0ull) {     // no match starts here: all literals
                while (sj < sj_end && (uint32_t)base + 64 > A.sub_c[sj] - 12) sub_done(0, anchor);
                continue;
            }
            // per-lane match length in one step: bytes 4..15 behind the known four
            // (four aligned dwords per side, issued together), so L <= LCAP = 16;
            // the walk extends the selected longer ones with the whole wave
            const bool run_l = valid && (uint32_t)i >= nextp;
            const uint32_t lim = run_l ? n - 5 - (uint32_t)i : 0u;
            uint32_t L = 0;
            if (run_l) {   // only possible match starts read their 12 bytes (fewer LDS bank conflicts)
                const uint32_t* c32 = reinterpret_cast<const uint32_t*>(ch);
                const uint32_t cs = (uint32_t)cand;
                const uint32_t si = (uint32_t)i & 3u, sc = cs & 3u;
                const uint32_t ai = ((uint32_t)i + 4) >> 2, ac = (cs + 4) >> 2;
                uint32_t wi[4], wc[4];
#pragma unroll
                for (int t = 0; t < 4; t++) { wi[t] = c32[ai + t]; wc[t] = c32[ac + t]; }
                uint32_t add = 12;
#pragma unroll
                for (int t = 2; t >= 0; t--) {
                    const uint32_t x = __builtin_amdgcn_alignbyte(wi[t + 1], wi[t], si) ^
                                       __builtin_amdgcn_alignbyte(wc[t + 1], wc[t], sc);
                    if (x) add = 4 * t + ((uint32_t)__builtin_ctz(x) >> 3);
                }
                L = 4 + add;
            }
            L = min(L, lim);
            STAMP(3);
            // (1) greedy walk over this round's positions.  Every lane first links
            // itself to the next match start the greedy parse would take after it
            // (first valid position >= its match end; 64 = leaves the round, 65 =
            // its match needs extending beyond LCAP).  Three doubling steps (three
            // bpermutes each) turn the links into chains of up to eight starts per
            // lane: the mask of the chain's starts and the link after its last one.
            // The scalar walk then takes eight matches per step (one OR and three
            // v_readlane), which keeps the scalar unit -- the ASCII chunks' busiest
            // port -- out of the per-match work.
            const bool longl = run_l && L >= LCAP && L < lim;
            const uint32_t E = lane + L;    // match end relative to base (lanes with L)
            uint32_t hop;
            {
                const uint64_t mm = E < 64 ? (vm & (~0ull << E)) : 0ull;
                hop = longl ? 65u : (mm ? (uint32_t)__builtin_ctzll(mm) : 64u);
            }
            uint32_t chlo = lane < 32 ? 1u << lane : 0u, chhi = lane < 32 ? 0u : 1u << (lane - 32);
#pragma unroll
            for (int lv = 0; lv < 3; lv++) {
                const int idx = (int)(min(hop, 63u) << 2);
                const uint32_t tlo = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)chlo);
                const uint32_t thi = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)chhi);
                const uint32_t th = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)hop);
                const bool in = hop < 64;
                chlo |= in ? tlo : 0u;
                chhi |= in ? thi : 0u;
                hop = in ? th : hop;
            }
            uint64_t sel = 0;
            {
                const uint64_t m0 = vm & (~0ull << p);
                uint32_t cur = m0 ? (uint32_t)__builtin_ctzll(m0) : 64u;
                while (cur < 64) {
                    sel |= (uint64_t)readlane(chlo, cur) | (uint64_t)readlane(chhi, cur) << 32;
                    const uint32_t x = readlane(hop, cur);
                    if (x < 64) { cur = x; continue; }   // eight more starts taken
                    cur = 63u - (uint32_t)__builtin_clzll(sel);   // the chain's last start
                    if (x == 64) {                 // cur's match is the round's last
                        p = readlane(E, cur);
                        break;
                    }
                    // x == 65: cur's match reaches LCAP: extend cooperatively, 256 B per step
                    const uint32_t j = (uint32_t)base + cur;
                    const uint32_t lj = n - 5 - j;
                    uint32_t Lj = readlane(L, cur);
                    const uint32_t c = readlane((uint32_t)cand, cur);
                    while (Lj < lj) {
                        const uint32_t q = Lj + 4 * lane;
                        uint32_t fd = 0;
                        bool eq = false;
                        if (q < lj) {
                            const uint32_t xx = lds_rd32(ch, j + q) ^ lds_rd32(ch, c + q);
                            eq = xx == 0;
                            fd = xx ? (uint32_t)__builtin_ctz(xx) >> 3 : 4;
                        }
                        const uint64_t ne = __ballot(!eq);
                        if (ne) {
                            const uint32_t lk = (uint32_t)__builtin_ctzll(ne);
                            Lj += 4 * lk + readlane(fd, lk);
                            break;
                        }
                        Lj += 256;
                    }
                    Lj = __builtin_amdgcn_readfirstlane(min(Lj, lj));
                    L = lane == cur ? Lj : L;
                    p = cur + Lj;
                    const uint64_t mn = p < 64 ? (vm & (~0ull << p)) : 0ull;
                    cur = mn ? (uint32_t)__builtin_ctzll(mn) : 64u;
                }
            }
            const uint32_t np = (uint32_t)base + p;
            STAMP(4);
            if (sel) {
                // (2) every selected lane emits its own sequence; literal start = the
                // previous selected match's end (exclusive max-scan), output offset =
                // exclusive prefix sum of the sequence sizes
                const bool me = (sel >> lane) & 1ull;
                const int pe = wave_excl_max(me ? i + (int)L : -1, (int)anchor);
                const uint32_t lit = me ? (uint32_t)(i - pe) : 0u;
                const uint32_t ml = me ? L - 4 : 0u;
                // length extension bytes only when some sequence needs them
                const bool ext = __ballot(lit >= 15 || ml >= 15) != 0ull;
                const uint32_t xl = ext ? ext_len(lit) : 0u, xm = ext ? ext_len(ml) : 0u;
                const uint32_t sz = me ? 3 + xl + lit + xm : 0u;
                const uint32_t incl = wave_incl_sum(sz);
                const uint32_t tot = readlane(incl, 63);
                // prefixes whose last match start b - 12 this round passes: the
                // round's sequences up to the last one starting by b - 12 (t), whose
                // match is capped at b - 5; none: the block ends with the anchor
                while (sj < sj_end && max(np, (uint32_t)base + 64) > A.sub_c[sj] - 12) {
                    const uint32_t b = A.sub_c[sj];
                    const uint32_t r = b - 12 - (uint32_t)base;      // lanes 0..r start by b - 12
                    const uint64_t sb = sel & (r >= 63 ? ~0ull : (2ull << r) - 1ull);
                    if (!sb) {
                        sub_done(0, anchor);
                    } else {
                        const uint32_t t = 63u - (uint32_t)__builtin_clzll(sb);
                        const uint32_t it = (uint32_t)base + t;
                        const uint32_t lb = min(readlane(L, t), b - 5 - it);
                        const uint32_t szb = 3 + readlane(xl, t) + readlane(lit, t) + ext_len(lb - 4);
                        sub_done(readlane(incl, t) - readlane(sz, t) + szb, it + lb);
                    }
                }
                // the sequential walk gives up at the first sequence that makes
                // block + 1 >= budget; the round total decides the same way
                if (alive && emitted + tot + 1 >= budget) alive = false;
                if (!alive && sj >= sj_end) break;
                const bool st_on = alive && !eval;           // (decision only: sizes, no bytes)
                // 32-bit offsets from the (uniform) block pointer: saddr stores
                const uint32_t q0 = emitted + incl - sz;     // token
                const uint32_t ql = q0 + 1 + xl;             // first literal
                if (me && st_on) {
                    blk[q0] = (uint8_t)((lit >= 15 ? 15 : lit) << 4 | (ml >= 15 ? 15 : ml));
                    const uint32_t offv = (uint32_t)(i - cand);
                    blk[ql + lit] = (uint8_t)offv;
                    blk[ql + lit + 1] = (uint8_t)(offv >> 8);
                }
                if (ext && me && st_on) {
                    for (uint32_t t = 0; t < xl; t++) blk[q0 + 1 + t] = (uint8_t)ext_byte(lit, xl, t);
                    for (uint32_t t = 0; t < xm; t++) blk[ql + lit + 2 + t] = (uint8_t)ext_byte(ml, xm, t);
                }
                // literals, one byte per lane: a lane inside this round that no
                // selected match covers and that some selected match follows is a
                // literal of the next selected lane's sequence, at offset i - pe
                // of its literals (its pe is that sequence's literal start); the
                // first sequence's literals from before this round by the whole wave
                if (st_on) {
                    const uint64_t rest = sel >> lane;
                    const uint32_t nx = rest ? lane + (uint32_t)__builtin_ctzll(rest) : lane;
                    const uint32_t qn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(nx << 2), (int)ql);
                    if (!me && rest && i >= pe) blk[qn + (uint32_t)(i - pe)] = (uint8_t)v;
                    if (anchor < (uint32_t)base) {
                        const uint32_t dst = readlane(ql, (uint32_t)__builtin_ctzll(sel));
                        const uint32_t len = (uint32_t)base - anchor;
                        for (uint32_t t = lane; t < len; t += 64) blk[dst + t] = ch[anchor + t];
                    }
                }
                emitted = __builtin_amdgcn_readfirstlane(emitted + tot);
                anchor = __builtin_amdgcn_readfirstlane(np);
            }
            nextp = __builtin_amdgcn_readfirstlane(np);
            STAMP(7);
        }
        // (by construction every prefix ends inside the loop; a leftover reads as lost)
        for (; sj < sj_end; sj++)
            if (lane == 0) A.lz4sub[(uint64_t)k * LZ4_SUB_MAX + sj] = 0xFFFFFFFFu;
        uint32_t fin = 0, flit = 0, fxl = 0;
        if (alive) {
            flit = n - anchor;
            fxl = ext_len(flit);
            fin = 1 + fxl + flit;
            if (emitted + fin >= budget) alive = false;
        }
        if (alive) {
            // final literals, frame header, block size, end mark
            const uint32_t blen = emitted + fin;
            uint8_t* o = blk + emitted;
            for (uint32_t t = lane; t < (eval ? 0u : fin + 4); t += 64) {
                uint32_t b;
                if (t == 0) b = (flit >= 15 ? 15 : flit) << 4;
                else if (t < 1 + fxl) b = ext_byte(flit, fxl, t - 1);
                else if (t < fin) b = ch[anchor + t - 1 - fxl];
                else b = 0;   // end mark
                o[t] = (uint8_t)b;
            }
            if (lane < 19 && !eval) slot[lane] = lz4_hdr_byte(lane, n, blen);
            win = 9;
            wlen = blen + 23;
            best = blen + 41;
        } else if (force) {
            // stored block: 15 B header, size | 0x80000000, raw bytes, end mark
            for (uint32_t t = lane; t < n + 4; t += 64) blk[t] = t < n ? ch[t] : 0;
            if (lane < 19) slot[lane] = lz4_hdr_byte(lane, n, n | 0x80000000u);
            win = 9;
            wlen = n + 23;
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < 4; j++) S.hist()[lane + 64 * j] = hsave[j];
        wave_sync();
    }

    if (huff_defer && huff_lb + HDR < best_pre && (win != 9 || huff_lb <= wlen)) {
        // Huffman comes before LZ4 in id order: it wins a tie with LZ4
        const uint32_t nb = huff_merge();
        const uint32_t l = 1 + 5 * kdist + 4 + (nb + 7) / 8;
        if (l + HDR < best_pre && (win != 9 || l <= wlen)) { best = l + HDR; win = 3; wlen = l; }
    }
    STAMP(5);
    // forced Delta (DeltaCompression.compress, compression_methods.py:585-608)
    if (force && ((mm >> 4) & 1u)) { win = 4; wlen = n; }

    // ---- emit the winner's payload into the slot ----
    // With DEFLATE enabled an RLE/Huffman payload waits for k_deflate's verdict:
    // id 5 wins most such chunks, and the few it does not are emitted by a second
    // launch (ENC_EMIT_PENDING) that repeats this chunk's selection
    const bool defer = A.pending && !(A.flags & ENC_EMIT_PENDING) && (win == 1 || win == 3);
    if (A.pending && !(A.flags & ENC_EMIT_PENDING) && lane == 0) A.pending[k] = defer ? 1 : 0;
    if (defer || eval) {
    } else if (win == 4) {
        for (uint32_t i = lane; i < n; i += 64)
            slot[i] = i ? (uint8_t)(ch[i] - ch[i - 1]) : ch[0];
    } else if (win == 255) {
        // in place: k_compact copies the chunk from the input (saves writing and
        // re-reading a third of a mixed input's bytes through the slots)
        const uint32_t nv = (A.flags & ENC_RAW_IN_PLACE) ? 0u : (n + 15) >> 4;
        for (uint32_t v = lane; v < nv; v += 64)
            reinterpret_cast<uint4*>(slot)[v] = reinterpret_cast<const uint4*>(ch)[v];
    } else if (win == 1 && S.hist()[ch[0]] == n) {
        // one byte value: (c, 255) pairs and the remainder (compression_methods.py:95-109)
        const uint32_t c = ch[0];
        for (uint32_t j = lane; j < pairs; j += 64) {
            slot[2 * j] = (uint8_t)c;
            slot[2 * j + 1] = (uint8_t)(j + 1 < pairs ? 255u : n - 255u * (pairs - 1));
        }
    } else if (win == 1) {
        // pair starts -> region (u16) in windows of CAPP entries (a forced RLE on
        // incompressible data has up to n pairs), then (byte, count) pairs
        uint16_t* ps = reinterpret_cast<uint16_t*>(S.work);
        constexpr uint32_t CAPP = EncSmem<CMAX, GL>::WORK / 2;
#pragma unroll 1
        for (uint32_t wb = 0; wb < pairs; wb += CAPP - 1) {
            uint32_t base_idx = 0;
            int rs_c = -1;
#pragma unroll 1
            for (int r = 0; r < ROUNDS; r++) {
                const uint32_t b0 = (uint32_t)(r * 64 + lane) * BS;
                const uint32_t prevb = b0 ? (b0 - 1 < GLLIM ? (uint32_t)ch[b0 - 1] : 0u) : 0x100u;
                int lb = -1;
                uint32_t cnt = 0;
                {
                    uint32_t prev = prevb;
                    for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t c, uint32_t) {
                        if (p < n && c != prev) lb = (int)p;
                        prev = c;
                    });
                }
                const int rs = wave_excl_max(lb, rs_c);
                rs_c = max(rs_c, wave_max_i32(lb));
                const uint32_t off0 = b0 == 0 ? 254u : (uint32_t)((int)(b0 - 1) - rs) % 255u;
                uint32_t off = off0, prev = prevb;
                for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t c, uint32_t) {
                    off = c != prev ? 0u : (off == 254u ? 0u : off + 1u);
                    if (p < n && off == 0) cnt++;
                    prev = c;
                });
                const uint32_t incl = wave_incl_sum(cnt);
                uint32_t idx = base_idx + incl - cnt;
                off = off0; prev = prevb;
                for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t c, uint32_t) {
                    off = c != prev ? 0u : (off == 254u ? 0u : off + 1u);
                    if (p < n && off == 0) {
                        if (idx >= wb && idx < wb + CAPP) ps[idx - wb] = (uint16_t)p;
                        idx++;
                    }
                    prev = c;
                });
                base_idx += readlane(incl, 63);
            }
            wave_sync();
            const uint32_t we = min(pairs, wb + CAPP - 1);
            for (uint32_t j = wb + lane; j < we; j += 64) {
                const uint32_t st = ps[j - wb];
                const uint32_t en = j + 1 < pairs ? ps[j + 1 - wb] : n;
                slot[2 * j] = ch[st];
                slot[2 * j + 1] = (uint8_t)(en - st);
            }
            wave_sync();
        }
    } else if (win == 3) {
        // the table: [k][sym, count u32le] x k (first-occurrence order), [nbits
        // u32le], then the bits MSB-first (compression_methods.py:354-405)
        if (!tree_ok) (void)huff_merge();   // (the LZ4 table overwrote the sizing pass's tree)
        huff_codes();
        compute_first();
        const uint32_t kk = kdist;
        if (lane == 0) slot[0] = (uint8_t)kk;
        for (uint32_t q = lane; q < kk; q += 64) {
            const uint32_t sy = S.order()[q], c = S.hist()[sy];
            uint8_t* e = slot + 1 + 5 * q;
            e[0] = (uint8_t)sy; e[1] = (uint8_t)c; e[2] = (uint8_t)(c >> 8);
            e[3] = (uint8_t)(c >> 16); e[4] = (uint8_t)(c >> 24);
        }
        const uint32_t hb = 1 + 5 * kk;
        const uint32_t nbytes = wlen - hb - 4;
        uint8_t* const pay = slot + hb + 4;
        wave_sync();   // hist / first / order are done with: the stage overlays them
        // The bits go through an LDS stage of CAPB bytes, a window of the payload
        // at a time (one window for every Huffman winner of a 4 KiB chunk; forced
        // high-entropy encodes take several): each lane packs its block's codes
        // into 32-bit words, byte-swapped so that the stage holds the payload's
        // bytes in order, ORs them in (LDS atomics: the words at the lanes' edges
        // are shared), and the window is stored with aligned 16-byte stores.
        constexpr uint32_t CAPB = EncSmem<CMAX, GL>::STAGE;
        uint32_t* bits = S.stage();
        uint32_t nbits = 0;
#pragma unroll 1
        for (uint32_t w0 = 0; w0 < nbytes; w0 += CAPB) {
            const uint32_t wl = min(CAPB, nbytes - w0);
            const uint32_t B0 = 8 * w0, B1 = 8 * (w0 + wl);    // the window's stream bits
            for (uint32_t w = lane; w < (wl + 3) / 4; w += 64) bits[w] = 0;
            wave_sync();
            uint32_t bitbase = 0;
#pragma unroll 1
            for (int r = 0; r < ROUNDS; r++) {
                const uint32_t b0 = (uint32_t)(r * 64 + lane) * BS;
                uint32_t my = 0;
                for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t c, uint32_t) {
                    if (p < n) my += S.clen()[c];
                });
                const uint32_t incl = wave_incl_sum(my);
                const uint32_t tot = readlane(incl, 63);
                uint32_t bp = bitbase + incl - my;
                if (my && bp < B1 && bp + my > B0) {
                    // words are whole inside one window (the windows are word multiples):
                    // a code across a window edge puts each of its words where it belongs
                    // and the words outside this window are dropped
                    const uint32_t nw = (wl + 3) / 4;
                    int cw = ((int)bp - (int)B0) >> 5;
                    uint32_t acc = 0;
                    auto flush = [&](int w, uint32_t v) {
                        if (v && (uint32_t)w < nw) atomicOr(&bits[w], __builtin_bswap32(v));
                    };
                    for_block_bytes<BS>(ch, b0, GLLIM, [&](uint32_t p, uint32_t sy, uint32_t) {
                        if (p < n) {
                            const uint32_t L = S.clen()[sy], cd = S.code()[sy];
                            const int rel = (int)bp - (int)B0;
                            const uint32_t o = (uint32_t)rel & 31u;
                            const int w = rel >> 5;
                            if (w != cw) { flush(cw, acc); cw = w; acc = 0; }
                            if (o + L <= 32) {
                                acc |= cd << (32 - o - L);
                            } else {
                                flush(cw, acc | cd >> (o + L - 32));
                                cw = w + 1;
                                acc = cd << (64 - o - L);
                            }
                            bp += L;
                        }
                    });
                    flush(cw, acc);
                }
                bitbase += tot;
            }
            nbits = bitbase;
            wave_sync();
            lds_store_bytes(pay + w0, reinterpret_cast<const uint8_t*>(bits), wl, lane);
            wave_sync();
        }
        if (lane < 4) slot[hb + lane] = (uint8_t)(nbits >> (8 * lane));
    }

    STAMP(6);
    STAMP_FLUSH
    if (lane == 0) {
        A.plen[k] = wlen;
        A.ids[k] = (uint8_t)win;
        A.sizes[k] = (uint64_t)HDR + wlen;
        if (A.su) A.su[k] = (uint8_t)((rle_su ? 2 : 0) | (huff_su ? 8 : 0) | (delta_su ? 16 : 0));
    }
}

// ---------------------------------------------------------------------------
// k_compact: header + payload of each package to its byte offset in the body.
// One wave per package.  The package's interior is written in 16-byte aligned
// groups of the body, one group per lane and step: each group's 16 source bytes
// lie at one fixed offset (mod 16) of the 16-byte aligned slot, so two aligned
// 16-byte loads and four v_alignbyte make it (1 KB per store instruction; the
// dword version before issued two loads and a store per 4 bytes, 0.39 ms for a
// 1 GiB segment's 262144 packages alone).  The header and the edge groups shared
// with the neighbouring packages go byte by byte.
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t pick_dword(const uint4& a, const uint4& b, uint32_t i) {
    // dword i (0..7) of the 32-byte window a:b (i wave-uniform per package)
    switch (i) {
        case 0: return a.x;
        case 1: return a.y;
        case 2: return a.z;
        case 3: return a.w;
        case 4: return b.x;
        case 5: return b.y;
        case 6: return b.z;
        default: return b.w;
    }
}

__device__ __forceinline__ void compact_package(const CompactArgs& A, uint32_t k, uint32_t lane) {
    const uint64_t o = A.off[k] + (A.base ? *A.base : 0ull);
    const uint32_t pl = A.plen[k];
    const uint32_t P = HDR + pl;
    const uint32_t type = A.ids[k];
    const uint64_t p0 = (uint64_t)k * A.chunk_size;
    const uint32_t n = A.clen ? A.clen[k] : A.clen_all ? A.clen_all : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - p0);
    const uint8_t* __restrict__ sl = type == 255 && A.in ? A.in + p0 : A.slots + (uint64_t)k * A.slot_stride;
    uint8_t* const dst = A.out + o;                       // the package's first byte
    const uint64_t da = reinterpret_cast<uintptr_t>(dst);
    // interior groups: body-aligned 16-byte groups wholly inside the payload
    const uint64_t g0 = (da + HDR + 15) >> 4, g1 = (da + P) >> 4;   // [g0, g1)
    const uint32_t ng = g1 > g0 ? (uint32_t)(g1 - g0) : 0u;
    const uint32_t head = ng ? (uint32_t)((g0 << 4) - da) : P;     // bytes before the interior
    const uint32_t tail0 = ng ? head + 16 * ng : P;                 // first byte after it
    if (ng) {
        // payload offset of group g0's first byte, and its place in the aligned source
        const uint32_t t0 = head - HDR;
        const uint32_t rr = (uint32_t)((reinterpret_cast<uintptr_t>(sl) + t0) & 15u);
        const uint32_t ds = rr >> 2, bs = (rr & 3u) * 8u;
        const uint4* src4 = reinterpret_cast<const uint4*>(sl + t0 - rr);
        uint4* dst4 = reinterpret_cast<uint4*>(g0 << 4);
        for (uint32_t j = lane; j < ng; j += 64) {
            // (a source on the 16-byte grid needs no second block: never read it --
            // for a raw package compacted from the caller's input it may lie past
            // the input's last byte, in unmapped memory)
            const uint4 a = src4[j], b = rr ? src4[j + 1] : make_uint4(0u, 0u, 0u, 0u);
            uint32_t w[5];
#pragma unroll
            for (int i = 0; i < 5; i++) w[i] = pick_dword(a, b, ds + i);
            uint4 v;
            v.x = (uint32_t)((((uint64_t)w[1] << 32) | w[0]) >> bs);
            v.y = (uint32_t)((((uint64_t)w[2] << 32) | w[1]) >> bs);
            v.z = (uint32_t)((((uint64_t)w[3] << 32) | w[2]) >> bs);
            v.w = (uint32_t)((((uint64_t)w[4] << 32) | w[3]) >> bs);
            dst4[j] = v;
        }
    }
    // the header and the edges, byte by byte
    for (uint32_t q = lane; q < head; q += 64) dst[q] = q < HDR ? hdr_byte(q, type, n, pl) : sl[q - HDR];
    for (uint32_t q = tail0 + lane; q < P; q += 64) dst[q] = q < HDR ? hdr_byte(q, type, n, pl) : sl[q - HDR];
}

// a fixed grid of resident workgroups that stride over the packages: launched
// beside the encoder, it gets its slots once instead of once per package group
__global__ __launch_bounds__(256) void k_compact(CompactArgs A) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6); k < A.n_chunks; k += gridDim.x * 4)
        compact_package(A, k, lane);
}

__global__ void k_seg_base(uint64_t* base, const uint64_t* off_last, const uint64_t* size_last) {
    if (threadIdx.x == 0) base[1] = base[0] + off_last[0] + size_last[0];
}

// the end chunk at the body offset the device holds (a pipelined call's last
// segment end), and that offset into acc_slot: one copy back for both
__global__ void k_end_chunk_at(uint8_t* out, const uint64_t* off, uint64_t* acc_slot) {
    const uint32_t t = threadIdx.x;
    const uint64_t o = *off;
    if (out && t < END_CHUNK) out[o + t] = t < 2 ? 0xFF : 0;
    if (t == 0) acc_slot[0] = o;
}

__global__ void k_end_chunk(uint8_t* dst) {
    const uint32_t t = threadIdx.x;
    if (t < END_CHUNK) dst[t] = t < 2 ? 0xFF : 0;
}

// per-method usage + byte sums (the reference's chunk_stats, :471-480)
// acc: [0..255] usage, 256 compressed, 257 raw, 258 payload bytes, 259 bytes saved
__global__ __launch_bounds__(256) void k_stats(const uint8_t* ids, const uint32_t* plen,
                                               uint32_t n_chunks, uint64_t n_total, uint32_t C,
                                               uint64_t* acc) {
    __shared__ uint32_t h[256];
    __shared__ unsigned long long sums[3];
    h[threadIdx.x] = 0;
    if (threadIdx.x < 3) sums[threadIdx.x] = 0;
    __syncthreads();
    uint64_t pay = 0, saved = 0, comp = 0;
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n_chunks; k += gridDim.x * 256) {
        const uint32_t id = ids[k];
        atomicAdd(&h[id], 1u);
        if (id != 255) {
            const uint64_t p0 = (uint64_t)k * C;
            const uint64_t n = min((uint64_t)C, n_total - p0);
            comp++;
            pay += plen[k];
            saved += n - (plen[k] + HDR);
        }
    }
    comp = wave_sum(comp); pay = wave_sum(pay); saved = wave_sum(saved);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&sums[0], (unsigned long long)comp);
        atomicAdd(&sums[1], (unsigned long long)pay);
        atomicAdd(&sums[2], (unsigned long long)saved);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd((unsigned long long*)&acc[threadIdx.x], (unsigned long long)h[threadIdx.x]);
    if (threadIdx.x == 0) {
        atomicAdd((unsigned long long*)&acc[256], sums[0]);
        atomicAdd((unsigned long long*)&acc[258], sums[1]);
        atomicAdd((unsigned long long*)&acc[259], sums[2]);
    }
}

// bulk copy to an arbitrary byte offset (reference-mode raw remainder)
// a walk batch's results into its pinned host arrays (device stores to host memory)
__global__ __launch_bounds__(256) void k_results_to_host(const uint32_t* plen, const uint8_t* ids, const uint32_t* lz,
                                                         uint32_t cnt, uint32_t nlz, uint32_t* hplen, uint8_t* hids,
                                                         uint32_t* hlz) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cnt) {
        hplen[i] = plen[i];
        hids[i] = ids[i];
    }
    if (lz)
        for (uint32_t j = i; j < cnt * nlz; j += gridDim.x * blockDim.x) hlz[j] = lz[j];
}

__global__ __launch_bounds__(256) void k_copy(uint8_t* dst, const uint8_t* src, uint64_t len) {
    const uint64_t mis = (4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3;
    const uint64_t head = mis < len ? mis : len;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (tid < head) dst[tid] = src[tid];
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
    const uint8_t* s = src + head;
    const uint64_t nw = (len - head) >> 2;
    for (uint64_t w = tid; w < nw; w += stride) {
        const uint64_t p = w << 2;
        d32[w] = (uint32_t)s[p] | (uint32_t)s[p + 1] << 8 | (uint32_t)s[p + 2] << 16 |
                 (uint32_t)s[p + 3] << 24;
    }
    for (uint64_t i = head + (nw << 2) + tid; i < len; i += stride) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// "ambc-mixed v1" synthetic generator on the device (one block per segment)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__constant__ char c_vocab[16][8] = {"alpha", "beta", "gamma", "delta", "the",   "quick",
                                    "brown", "fox",  "jumps", "over",  "lazy",  "dog",
                                    "data",  "chunk", "marker", "stream"};
__constant__ uint8_t c_vlen[16] = {5, 4, 5, 5, 3, 5, 5, 3, 5, 4, 4, 3, 4, 5, 6, 6};

// seg: [pos, len, idx] triples.  ASCII segments: words are laid out by a
// block-wide scan over 256-word batches.
// bytes [lo, hi) of the stream land at out[0, hi - lo): a rank generates its
// own shard of a stream that spans several GPUs
__global__ __launch_bounds__(256) void k_synth(uint8_t* out, const uint64_t* seg, uint64_t seed, uint64_t lo,
                                               uint64_t hi) {
    const uint64_t pos = seg[3 * blockIdx.x], L = seg[3 * blockIdx.x + 1], id = seg[3 * blockIdx.x + 2];
    const uint64_t base = mix64(seed ^ (id * 0xD1B54A32D192ED03ULL));
    const uint32_t typ = (uint32_t)(id % 3);
    const uint64_t a = lo > pos ? lo - pos : 0;           // segment bytes [a, b) are in range
    const uint64_t b = hi - pos < L ? hi - pos : L;
    uint8_t* o = out + pos - lo;                          // o[i] for i in [a, b) only
    const uint32_t t = threadIdx.x;
    if (typ == 0) {
        for (uint64_t i = a + t; i < b; i += 256) o[i] = 0;
    } else if (typ == 1) {
        for (uint64_t j = a / 8 + t; j * 8 < b; j += 256) {
            const uint64_t w = mix64(base + (j + 1) * 0x9E3779B97F4A7C15ULL);
            for (int k = 0; k < 8; k++) {
                const uint64_t i = j * 8 + k;
                if (i >= a && i < b) o[i] = (uint8_t)(w >> (8 * k));
            }
        }
    } else {
        __shared__ uint32_t scan[256];
        uint64_t q = 0;  // bytes laid out so far (uniform)
        for (uint64_t jb = 0; q < b; jb += 256) {
            const uint64_t j = jb + t;
            const uint32_t w = (uint32_t)(mix64(base + (j + 1) * 0x9E3779B97F4A7C15ULL) >> 60);
            const uint32_t wl = c_vlen[w] + 1;
            scan[t] = wl;
            __syncthreads();
            for (int off = 1; off < 256; off <<= 1) {
                uint32_t v = t >= (uint32_t)off ? scan[t - off] : 0;
                __syncthreads();
                scan[t] += v;
                __syncthreads();
            }
            const uint64_t st = q + scan[t] - wl;
            if (st + wl > a) {
                for (uint32_t k = 0; k < wl; k++) {
                    const uint64_t p = st + k;
                    if (p >= a && p < b) o[p] = k + 1 < wl ? (uint8_t)c_vocab[w][k] : (uint8_t)' ';
                }
            }
            q += scan[255];
            __syncthreads();
        }
    }
}

// *neq |= (a[i] != b[i]) over n bytes (vector loads when both are 16-B aligned)
__global__ __launch_bounds__(256) void k_equal(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* neq) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nt = (uint64_t)gridDim.x * 256;
    uint32_t diff = 0;
    if ((((uintptr_t)a | (uintptr_t)b) & 15) == 0) {
        const uint4* a4 = reinterpret_cast<const uint4*>(a);
        const uint4* b4 = reinterpret_cast<const uint4*>(b);
        const uint64_t n16 = n / 16;
        for (uint64_t i = tid; i < n16; i += nt) {
            const uint4 x = a4[i], y = b4[i];
            diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
        }
        for (uint64_t i = n16 * 16 + tid; i < n; i += nt) diff |= a[i] ^ b[i];
    } else {
        for (uint64_t i = tid; i < n; i += nt) diff |= a[i] ^ b[i];
    }
    if (__any(diff != 0) && threadIdx.x % 64 == 0) atomicOr(neq, 1u);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int CMAX>
static hipError_t launch_encode_t(const EncArgs& a, hipStream_t s) {
    // 4 KiB and more: the chunk in place (see k_encode) unless a forced / analysed
    // encode may take the other methods' LDS-bound paths.  Same-box A/Bs of the
    // 4 GiB bench (profiles/r3_gl_ab.json, r3_wpe_ab.json): 8 KiB 217.3 -> 274.4
    // GB/s in place (12 KB of LDS held the CU to 13 workgroups); 4 KiB in place
    // pays only with the 8-wave register allocation (333 -> 300 at 5 waves, 340 at 8)
    static const uint32_t gl_min = getenv("AMBC_ENC_GL_MIN") ? (uint32_t)atoi(getenv("AMBC_ENC_GL_MIN")) : 4096u;
    if constexpr (CMAX >= 1024) {
        if (CMAX >= gl_min && (a.flags & ENC_IN_ALIGNED) && !(a.flags & (ENC_FORCE | ENC_ANALYZE))) {
            if (a.flags & ENC_EVAL)
                hipLaunchKernelGGL((k_encode<CMAX, true, ENC_MODE_WALK>), dim3(a.n_chunks), dim3(64), 0, s, a);
            else
                hipLaunchKernelGGL((k_encode<CMAX, true>), dim3(a.n_chunks), dim3(64), 0, s, a);
            return hipGetLastError();
        }
    }
    if (a.flags & ENC_EVAL)
        hipLaunchKernelGGL((k_encode<CMAX, false, ENC_MODE_WALK>), dim3(a.n_chunks), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((k_encode<CMAX, false>), dim3(a.n_chunks), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_encode(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    const uint32_t C = a.chunk_size;
    if (C <= 1024) return launch_encode_t<1024>(a, s);
    if (C <= 2048) return launch_encode_t<2048>(a, s);
    if (C <= 4096) return launch_encode_t<4096>(a, s);
    if (C <= 8192) return launch_encode_t<8192>(a, s);
    if (C <= 16384) return launch_encode_t<16384>(a, s);
    if (C <= 32768) return launch_encode_t<32768>(a, s);
    return launch_encode_t<65536>(a, s);
}

hipError_t launch_seg_base(uint64_t* base, const uint64_t* off_last, const uint64_t* size_last, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_base, dim3(1), dim3(64), 0, s, base, off_last, size_last);
    return hipGetLastError();
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    // beside the encoder: a resident grid; alone (the last segment): every package group
    const uint32_t blocks = a.resident ? std::min<uint32_t>((a.n_chunks + 3) / 4, a.resident)
                                       : (a.n_chunks + 3) / 4;
    hipLaunchKernelGGL(k_compact, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_end_chunk_at(uint8_t* out, const uint64_t* off, uint64_t* acc_slot, hipStream_t s) {
    hipLaunchKernelGGL(k_end_chunk_at, dim3(1), dim3(64), 0, s, out, off, acc_slot);
    return hipGetLastError();
}

hipError_t launch_end_chunk(uint8_t* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_end_chunk, dim3(1), dim3(64), 0, s, dst);
    return hipGetLastError();
}

hipError_t launch_stats(const uint8_t* ids, const uint32_t* plen, uint32_t n_chunks,
                        uint64_t n_total, uint32_t C, uint64_t* acc, hipStream_t s) {
    if (n_chunks == 0) return hipSuccess;
    uint32_t blocks = (n_chunks + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_stats, dim3(blocks), dim3(256), 0, s, ids, plen, n_chunks, n_total, C, acc);
    return hipGetLastError();
}

hipError_t launch_results_to_host(const uint32_t* plen, const uint8_t* ids, const uint32_t* lz, uint32_t cnt, uint32_t nlz,
                                  uint32_t* hplen, uint8_t* hids, uint32_t* hlz, hipStream_t s) {
    if (cnt == 0) return hipSuccess;
    hipLaunchKernelGGL(k_results_to_host, dim3((cnt + 255) / 256), dim3(256), 0, s, plen, ids, lz, cnt, nlz, hplen, hids,
                       hlz);
    return hipGetLastError();
}

hipError_t launch_copy(uint8_t* dst, const uint8_t* src, uint64_t len, hipStream_t s) {
    if (len == 0) return hipSuccess;
    uint64_t blocks = (len / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_copy, dim3((uint32_t)blocks), dim3(256), 0, s, dst, src, len);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* out, uint64_t lo, uint64_t hi, const uint64_t* seg, uint32_t nseg,
                        uint64_t seed, hipStream_t s) {
    if (nseg == 0 || hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3(nseg), dim3(256), 0, s, out, seg, seed, lo, hi);
    return hipGetLastError();
}

hipError_t launch_equal(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* neq, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n / 16 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_equal, dim3((uint32_t)blocks), dim3(256), 0, s, a, b, n, neq);
    return hipGetLastError();
}

}  // namespace ambc
