// ambc_anylen.hip -- the single-call plugins (CompressionMethod.compress /
// should_use, compression_methods.py:7-713, advanced_compression.py:266-307)
// at ANY input length, where the batched engine's kernels take one chunk of at
// most 65536 bytes.  The reference's loop never passes more (its prefs cap RLE
// and Delta at 4096, Huffman at 8192, LZ4 at 65536); a direct plugin call may.
//
// The input is cut into 4 KiB blocks, one 256-thread workgroup each (16
// consecutive bytes per thread); what crosses blocks goes through one-workgroup
// scans over the per-block values (k_any_scan):
//   RLE   (:78-113)   a pair starts at every run start and every 255th byte of
//                     a run; the run start carried into a block is a prefix max
//                     over the blocks' last run starts.  Pair starts are counted,
//                     scanned, then written (byte, and position for the count =
//                     distance to the next pair start);
//   Delta (:586-607)  one byte each;
//   Huffman (:358-405) byte histogram and first occurrences (global atomics),
//                     the heap tree on one wave (keys weight << 8 | the first
//                     byte of the node's list -- heapq's list order, :482-494),
//                     the table in Counter order, code bits at their prefix
//                     offsets (per-thread 64-bit accumulators, whole words
//                     stored, the two edge words OR-ed), then the big-endian
//                     stream's bytes;
//   should_use samples (RLE :166-180, Delta :652-667): every step-th pair.
// LZ4 beyond 64 KiB is assembled on the host side of the C-ABI from k_encode's
// 64 KiB frames (ambc_host.cpp, k_lz4_assemble below): one frame of
// independent 64 KiB blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc.h"
#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

constexpr uint32_t AB = 4096;   // bytes per block
constexpr uint32_t AT = 256;    // threads per block
constexpr uint32_t AP = AB / AT;   // bytes per thread

// exclusive scan of v[0, nb) in place, v[nb] = the total; MAX: prefix max
// (identity -1), else prefix sum (identity 0).  One workgroup of 1024 threads,
// each over a contiguous run of ceil(nb / 1024) values.
template <bool MAX>
__global__ __launch_bounds__(1024) void k_any_scan(int64_t* v, uint32_t nb) {
    __shared__ int64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t a = min(nb, t * per), b = min(nb, a + per);
    const int64_t id = MAX ? -1 : 0;
    int64_t acc = id;
    for (uint32_t i = a; i < b; i++) acc = MAX ? max(acc, v[i]) : acc + v[i];
    part[t] = acc;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const int64_t x = t >= off ? part[t - off] : id;
        __syncthreads();
        part[t] = MAX ? max(part[t], x) : part[t] + x;
        __syncthreads();
    }
    int64_t run = t ? part[t - 1] : id;
    for (uint32_t i = a; i < b; i++) {
        const int64_t x = v[i];
        v[i] = run;
        run = MAX ? max(run, x) : run + x;
    }
    if (t == 1023) v[nb] = part[1023];
}

// block-wide exclusive scan of one value per thread (AT threads)
template <bool MAX>
__device__ __forceinline__ int64_t block_excl(int64_t x, int64_t* sh) {
    const uint32_t t = threadIdx.x;
    const int64_t id = MAX ? -1 : 0;
    sh[t] = x;
    __syncthreads();
    for (uint32_t off = 1; off < AT; off <<= 1) {
        const int64_t y = t >= off ? sh[t - off] : id;
        __syncthreads();
        sh[t] = MAX ? max(sh[t], y) : sh[t] + y;
        __syncthreads();
    }
    const int64_t r = t ? sh[t - 1] : id;
    __syncthreads();
    return r;
}

// ---- RLE ----
__device__ __forceinline__ bool run_start(const uint8_t* d, uint64_t i) { return i == 0 || d[i] != d[i - 1]; }

// the last run start of every block (-1: none)
__global__ __launch_bounds__(AT) void k_rle_last(const uint8_t* __restrict__ d, uint64_t n, int64_t* __restrict__ last) {
    __shared__ int64_t sh[AT];
    const uint64_t b0 = (uint64_t)blockIdx.x * AB, p0 = b0 + threadIdx.x * AP;
    int64_t l = -1;
    for (uint32_t j = 0; j < AP; j++) {
        const uint64_t i = p0 + j;
        if (i < n && run_start(d, i)) l = (int64_t)i;
    }
    sh[threadIdx.x] = l;
    __syncthreads();
    for (uint32_t s = AT / 2; s; s >>= 1) {
        if (threadIdx.x < s) sh[threadIdx.x] = max(sh[threadIdx.x], sh[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) last[blockIdx.x] = sh[0];
}

// pair starts per block (EMIT = false) or their bytes and positions (EMIT):
// carry[b] = the last run start before block b, base[b] = pairs before block b
template <bool EMIT>
__global__ __launch_bounds__(AT) void k_rle_pairs(const uint8_t* __restrict__ d, uint64_t n,
                                                  const int64_t* __restrict__ carry, int64_t* __restrict__ cnt,
                                                  uint32_t* __restrict__ pos, uint8_t* __restrict__ out) {
    __shared__ int64_t sh[AT];
    const uint64_t b0 = (uint64_t)blockIdx.x * AB, p0 = b0 + threadIdx.x * AP;
    int64_t l = -1;
    for (uint32_t j = 0; j < AP; j++) {
        const uint64_t i = p0 + j;
        if (i < n && run_start(d, i)) l = (int64_t)i;
    }
    int64_t rs = max(block_excl<true>(l, sh), carry[blockIdx.x]);
    uint32_t c = 0;
    for (uint32_t j = 0; j < AP; j++) {
        const uint64_t i = p0 + j;
        if (i >= n) break;
        if (run_start(d, i)) rs = (int64_t)i;
        c += ((i - (uint64_t)rs) % 255u) == 0;
    }
    if (!EMIT) {
        const int64_t tot = block_excl<false>(c, sh) + c;   // (the last thread's inclusive value)
        if (threadIdx.x == AT - 1) cnt[blockIdx.x] = tot;
        return;
    }
    uint64_t r = (uint64_t)cnt[blockIdx.x] + (uint64_t)block_excl<false>(c, sh);
    rs = max(block_excl<true>(l, sh), carry[blockIdx.x]);
    for (uint32_t j = 0; j < AP; j++) {
        const uint64_t i = p0 + j;
        if (i >= n) break;
        if (run_start(d, i)) rs = (int64_t)i;
        if (((i - (uint64_t)rs) % 255u) == 0) {
            pos[r] = (uint32_t)i;
            out[2 * r] = d[i];
            r++;
        }
    }
}

// every pair's count: the distance to the next pair start (the last: to n)
__global__ void k_rle_counts(const uint32_t* __restrict__ pos, uint64_t np, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= np) return;
    const uint64_t e = j + 1 < np ? pos[j + 1] : n;
    out[2 * j + 1] = (uint8_t)(e - pos[j]);
}

// ---- Delta ----
__global__ void k_delta_any(const uint8_t* __restrict__ d, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i ? (uint8_t)(d[i] - d[i - 1]) : d[0];
}

// ---- Huffman ----
// histogram and first occurrences (first[]: 0xFFFFFFFF before)
__global__ __launch_bounds__(AT) void k_huff_hist(const uint8_t* __restrict__ d, uint64_t n, uint32_t* __restrict__ hist,
                                                  uint32_t* __restrict__ first) {
    __shared__ uint32_t h[256], f[256];
    h[threadIdx.x] = 0;
    f[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * AB;
    for (uint32_t j = threadIdx.x; j < AB; j += AT) {
        const uint64_t i = b0 + j;
        if (i < n) {
            const uint32_t c = d[i];
            atomicAdd(&h[c], 1u);
            atomicMin(&f[c], (uint32_t)i);
        }
    }
    __syncthreads();
    if (h[threadIdx.x]) {
        atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
        atomicMin(&first[threadIdx.x], f[threadIdx.x]);
    }
}

// the two smallest of (a0 <= a1) and (b0 <= b1)
__device__ __forceinline__ void two_min(uint64_t& a0, uint64_t& a1, uint64_t b0, uint64_t b1) {
    const uint64_t lo = min(a0, b0), hi = max(a0, b0);
    a1 = min(hi, min(a1, b1));
    a0 = lo;
}

// One wave: the table (Counter order), the heap tree, codes[s] = code | len << 58,
// info[0] = 0 ok / AMBC_E_CODEC (1 or 256 symbols) / AMBC_E_RANGE (nbits >= 2^32),
// info[1] = header bytes, info[2..3] = nbits.  hdr: 1 + 5K + 4 bytes.
__global__ __launch_bounds__(64) void k_huff_tree(const uint32_t* __restrict__ hist, const uint32_t* __restrict__ first,
                                                  uint64_t* __restrict__ codes, uint8_t* __restrict__ hdr,
                                                  int32_t* __restrict__ info) {
    __shared__ uint64_t key[512];
    __shared__ uint16_t par[512];
    __shared__ uint8_t bit[512];
    __shared__ uint32_t rank[256];
    const uint32_t lane = threadIdx.x;
    uint32_t K = 0;
    for (uint32_t s = lane; s < 256; s += 64) K += hist[s] != 0;
    K = wave_sum_u32(K);
    if (K < 2 || K > 255) {   // one symbol: IndexError (:508-520 on code ""); 256: append(256) raises
        if (lane == 0) info[0] = AMBC_E_CODEC;
        return;
    }
    // Counter order: the symbols by first occurrence
    for (uint32_t s = lane; s < 256; s += 64) {
        uint32_t r = 0;
        if (hist[s]) {
            const uint32_t fs = first[s];
            for (uint32_t t = 0; t < 256; t++) r += hist[t] && first[t] < fs;
        }
        rank[s] = r;
    }
    __syncthreads();
    if (lane == 0) hdr[0] = (uint8_t)K;
    for (uint32_t s = lane; s < 256; s += 64) {
        if (!hist[s]) continue;
        uint8_t* e = hdr + 1 + 5 * rank[s];
        e[0] = (uint8_t)s;
        for (int b = 0; b < 4; b++) e[1 + b] = (uint8_t)(hist[s] >> (8 * b));
    }
    for (uint32_t x = lane; x < 512; x += 64) key[x] = x < 256 && hist[x] ? ((uint64_t)hist[x] << 8 | x) : ~0ull;
    __syncthreads();
    // K - 1 merges: the two smallest keys (lo -> '0', hi -> '1'); the new node's
    // key is the weight sum with lo's first byte (:487-494)
    for (uint32_t it = 0; it + 1 < K; it++) {
        uint64_t m0 = ~0ull, m1 = ~0ull;
        for (uint32_t x = lane; x < 256 + it; x += 64) {
            const uint64_t v = key[x];
            two_min(m0, m1, v, ~0ull);
        }
        for (int o = 32; o; o >>= 1) {
            const uint64_t b0 = __shfl_xor(m0, o), b1 = __shfl_xor(m1, o);
            two_min(m0, m1, b0, b1);
        }
        uint32_t ilo = 0xFFFFFFFFu, ihi = 0xFFFFFFFFu;
        for (uint32_t x = lane; x < 256 + it; x += 64) {
            if (key[x] == m0) ilo = x;
            if (key[x] == m1) ihi = x;
        }
        ilo = wave_min_u32(ilo);
        ihi = wave_min_u32(ihi);
        __syncthreads();
        if (lane == 0) {
            const uint32_t nn = 256 + it;
            key[nn] = (((m0 >> 8) + (m1 >> 8)) << 8) | (m0 & 0xFFu);
            key[ilo] = ~0ull;
            key[ihi] = ~0ull;
            par[ilo] = (uint16_t)nn;
            bit[ilo] = 0;
            par[ihi] = (uint16_t)nn;
            bit[ihi] = 1;
        }
        __syncthreads();
    }
    const uint32_t root = 256 + K - 2;
    uint64_t nb = 0;
    for (uint32_t s = lane; s < 256; s += 64) {
        uint64_t c = 0;
        uint32_t L = 0;
        if (hist[s]) {
            for (uint32_t x = s; x != root; x = par[x]) {
                c |= (uint64_t)bit[x] << L;
                L++;
            }
            nb += (uint64_t)hist[s] * L;
        }
        codes[s] = c | (uint64_t)L << 58;
    }
    for (int o = 32; o; o >>= 1) nb += __shfl_xor(nb, o);
    if (lane == 0) {
        const uint32_t h = 1 + 5 * K;
        info[0] = nb >> 32 ? AMBC_E_RANGE : 0;     // num_bits.to_bytes(4) raises (:397)
        info[1] = (int32_t)(h + 4);
        info[2] = (int32_t)(uint32_t)nb;
        info[3] = (int32_t)(uint32_t)(nb >> 32);
        for (int b = 0; b < 4; b++) hdr[h + b] = (uint8_t)(nb >> (8 * b));
    }
}

// code bits per block (the scan's input)
__global__ __launch_bounds__(AT) void k_huff_blen(const uint8_t* __restrict__ d, uint64_t n, const uint64_t* __restrict__ codes,
                                                  int64_t* __restrict__ bb) {
    __shared__ int64_t sh[AT];
    const uint64_t p0 = (uint64_t)blockIdx.x * AB + threadIdx.x * AP;
    int64_t s = 0;
    for (uint32_t j = 0; j < AP; j++)
        if (p0 + j < n) s += (int64_t)(codes[d[p0 + j]] >> 58);
    const int64_t ex = block_excl<false>(s, sh);
    if (threadIdx.x == AT - 1) bb[blockIdx.x] = ex + s;
}

__device__ __forceinline__ void put_word(uint32_t* be, uint64_t j, uint32_t w, bool edge) {
    if (edge) atomicOr(&be[j], w);
    else be[j] = w;
}

// every byte's code at its bit offset in the big-endian word stream be[] (zeroed)
__global__ __launch_bounds__(AT) void k_huff_bits(const uint8_t* __restrict__ d, uint64_t n, const uint64_t* __restrict__ codes,
                                                  const int64_t* __restrict__ bb, uint32_t* __restrict__ be) {
    __shared__ int64_t sh[AT];
    const uint64_t p0 = (uint64_t)blockIdx.x * AB + threadIdx.x * AP;
    int64_t s = 0;
    for (uint32_t j = 0; j < AP; j++)
        if (p0 + j < n) s += (int64_t)(codes[d[p0 + j]] >> 58);
    const uint64_t o = (uint64_t)bb[blockIdx.x] + (uint64_t)block_excl<false>(s, sh);
    if (s == 0) return;
    uint64_t acc = 0, wj = o >> 5;
    uint32_t nb = (uint32_t)(o & 31);     // pending bits (the word's earlier bits: zeros)
    bool first = true;
    for (uint32_t j = 0; j < AP; j++) {
        if (p0 + j >= n) break;
        const uint64_t cw = codes[d[p0 + j]];
        uint32_t L = (uint32_t)(cw >> 58);
        const uint64_t c = cw & ((1ull << 58) - 1);
        while (L) {
            const uint32_t t = min(L, 32u);
            const uint64_t part = (c >> (L - t)) & ((1ull << t) - 1);
            acc = (acc << t) | part;
            nb += t;
            L -= t;
            if (nb >= 32) {
                put_word(be, wj, (uint32_t)(acc >> (nb - 32)), first);
                first = false;
                wj++;
                nb -= 32;
                acc &= nb ? ((1ull << nb) - 1) : 0ull;
            }
        }
    }
    if (nb) put_word(be, wj, (uint32_t)(acc << (32 - nb)), true);
}

// the big-endian stream's first nbytes bytes
__global__ void k_huff_pack(const uint32_t* __restrict__ be, uint64_t nbytes, uint8_t* __restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nbytes) out[j] = (uint8_t)(be[j >> 2] >> (24 - 8 * (j & 3)));
}

// ---- should_use samples: i = 0, step, 2 step, ... < n - 1 ----
__global__ void k_su_samples(const uint8_t* __restrict__ d, uint64_t n, uint64_t step, uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = t * step;
    bool rep = false, small = false;
    if (i + 1 < n) {
        const int a = d[i], b = d[i + 1];
        rep = a == b;
        small = (a > b ? a - b : b - a) < 32;
    }
    const uint32_t r = wave_sum_u32(rep ? 1u : 0u), s = wave_sum_u32(small ? 1u : 0u);
    if ((threadIdx.x & 63u) == 0) {
        if (r) atomicAdd(&out[0], r);
        if (s) atomicAdd(&out[1], s);
    }
}

// ---- LZ4: one frame of independent 64 KiB blocks from k_encode's one-block
// frames (slot k: 15-byte header, block size field, block, end mark) ----
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ uint32_t xxh32_desc64(uint64_t n) {
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
    uint8_t b[10] = {0x68, 0x40};
    for (int q = 0; q < 8; q++) b[2 + q] = (uint8_t)(n >> (8 * q));
    uint32_t h = P5 + 10u;
    for (int q = 0; q < 8; q += 4) {
        const uint32_t w = b[q] | (uint32_t)b[q + 1] << 8 | (uint32_t)b[q + 2] << 16 | (uint32_t)b[q + 3] << 24;
        h = rotl(h + w * P3, 17) * P4;
    }
    for (int q = 8; q < 10; q++) h = rotl(h + b[q] * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(256) void k_lz4_assemble(const uint8_t* __restrict__ slots, uint64_t stride,
                                                      const uint32_t* __restrict__ plen, const uint64_t* __restrict__ off,
                                                      uint32_t m, uint64_t n, uint8_t* __restrict__ out) {
    const uint32_t k = blockIdx.x;
    if (k == m) {   // the frame header and the end mark
        if (threadIdx.x < 15) {
            const uint32_t q = threadIdx.x;
            uint8_t v;
            if (q < 4) v = (uint8_t)(0x184D2204u >> (8 * q));
            else if (q == 4) v = 0x68;
            else if (q == 5) v = 0x40;
            else if (q < 14) v = (uint8_t)(n >> (8 * (q - 6)));
            else v = (uint8_t)((xxh32_desc64(n) >> 8) & 0xFF);
            out[q] = v;
        } else if (threadIdx.x < 19) {
            out[off[m] + threadIdx.x - 15] = 0;
        }
        return;
    }
    const uint8_t* s = slots + (uint64_t)k * stride + 15;
    const uint64_t len = plen[k] - 19;      // block size field + block
    uint8_t* o = out + off[k];
    for (uint64_t i = threadIdx.x; i < len; i += 256) o[i] = s[i];
}

}  // namespace

uint32_t any_blocks(uint64_t n) { return (uint32_t)((n + AB - 1) / AB); }

hipError_t launch_delta_any(const uint8_t* d, uint64_t n, uint8_t* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_delta_any, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, out);
    return hipGetLastError();
}

// RLE: scratch last/carry (nb + 1 int64), cnt (nb + 1 int64), pos (n u32);
// *np_dev = pairs (cnt[nb] after the count pass)
hipError_t launch_rle_any_count(const uint8_t* d, uint64_t n, int64_t* carry, int64_t* cnt, hipStream_t s) {
    const uint32_t nb = any_blocks(n);
    hipLaunchKernelGGL(k_rle_last, dim3(nb), dim3(AT), 0, s, d, n, carry);
    hipLaunchKernelGGL(k_any_scan<true>, dim3(1), dim3(1024), 0, s, carry, nb);
    hipLaunchKernelGGL(k_rle_pairs<false>, dim3(nb), dim3(AT), 0, s, d, n, carry, cnt, nullptr, nullptr);
    hipLaunchKernelGGL(k_any_scan<false>, dim3(1), dim3(1024), 0, s, cnt, nb);
    return hipGetLastError();
}

hipError_t launch_rle_any_emit(const uint8_t* d, uint64_t n, const int64_t* carry, int64_t* cnt, uint32_t* pos,
                               uint64_t np, uint8_t* out, hipStream_t s) {
    const uint32_t nb = any_blocks(n);
    hipLaunchKernelGGL(k_rle_pairs<true>, dim3(nb), dim3(AT), 0, s, d, n, carry, cnt, pos, out);
    hipLaunchKernelGGL(k_rle_counts, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, pos, np, n, out);
    return hipGetLastError();
}

hipError_t launch_huff_any_hist(const uint8_t* d, uint64_t n, uint32_t* hist, uint32_t* first, hipStream_t s) {
    hipLaunchKernelGGL(k_huff_hist, dim3(any_blocks(n)), dim3(AT), 0, s, d, n, hist, first);
    return hipGetLastError();
}

hipError_t launch_huff_any_tree(const uint32_t* hist, const uint32_t* first, uint64_t* codes, uint8_t* hdr, int32_t* info,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_huff_tree, dim3(1), dim3(64), 0, s, hist, first, codes, hdr, info);
    return hipGetLastError();
}

// bits of the stream into be[] (zeroed, ceil(nbits / 32) + 1 words), then its
// bytes to out; bb: nb + 1 int64 scratch
hipError_t launch_huff_any_bits(const uint8_t* d, uint64_t n, const uint64_t* codes, int64_t* bb, uint32_t* be,
                                uint64_t nbytes, uint8_t* out, hipStream_t s) {
    const uint32_t nb = any_blocks(n);
    hipLaunchKernelGGL(k_huff_blen, dim3(nb), dim3(AT), 0, s, d, n, codes, bb);
    hipLaunchKernelGGL(k_any_scan<false>, dim3(1), dim3(1024), 0, s, bb, nb);
    hipLaunchKernelGGL(k_huff_bits, dim3(nb), dim3(AT), 0, s, d, n, codes, bb, be);
    if (nbytes) hipLaunchKernelGGL(k_huff_pack, dim3((unsigned)((nbytes + 255) / 256)), dim3(256), 0, s, be, nbytes, out);
    return hipGetLastError();
}

hipError_t launch_su_samples(const uint8_t* d, uint64_t n, uint64_t step, uint32_t* out2, hipStream_t s) {
    const uint64_t ns = n > 1 ? (n - 2) / step + 1 : 0;
    if (ns) hipLaunchKernelGGL(k_su_samples, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, d, n, step, out2);
    return hipGetLastError();
}

hipError_t launch_lz4_assemble(const uint8_t* slots, uint64_t stride, const uint32_t* plen, const uint64_t* off,
                               uint32_t m, uint64_t n, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_lz4_assemble, dim3(m + 1), dim3(256), 0, s, slots, stride, plen, off, m, n, out);
    return hipGetLastError();
}

}  // namespace ambc
