// Exclusive scan of package sizes -> byte offsets of each package in the body.
//
// Three launches over tiles of 4096 sizes (256 threads x 16 consecutive):
// per-tile sums, one workgroup scanning the tile sums, then every tile
// rescanned from its base.  A package is at most 18 + 3C + 1344 bytes (C <=
// 65536), so a tile's sum fits 32 bits and the in-tile scans are DPP wave scans
// of u32; only the tile bases are 64-bit.  (hipCUB's decoupled look-back scan
// measured the same beside the encoder: its blocks spin on predecessors queued
// behind the encoder's workgroups as these launches wait for slots.)
#include <hip/hip_runtime.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

constexpr uint32_t ST = 256, SPT = 16, TILE = ST * SPT;

// exclusive prefix of x over the workgroup (u32) and its total
__device__ __forceinline__ uint32_t tile_excl(uint32_t x, uint32_t* ws, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_sum(x);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (uint32_t w = 0; w < ST / 64; w++) {
        before += w < wave ? ws[w] : 0u;
        total += ws[w];
    }
    return before + incl - x;
}

__device__ __forceinline__ void load16(const uint64_t* sizes, uint32_t count, uint32_t i0, uint32_t v[SPT]) {
#pragma unroll
    for (uint32_t q = 0; q < SPT; q++) v[q] = i0 + q < count ? (uint32_t)sizes[i0 + q] : 0u;
}

__global__ __launch_bounds__(ST) void k_scan_reduce(const uint64_t* sizes, uint32_t count, uint64_t* tsum) {
    __shared__ uint32_t ws[ST / 64];
    uint32_t v[SPT], s = 0;
    load16(sizes, count, blockIdx.x * TILE + threadIdx.x * SPT, v);
#pragma unroll
    for (uint32_t q = 0; q < SPT; q++) s += v[q];
    uint32_t total;
    (void)tile_excl(s, ws, total);
    if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(64) void k_scan_bases(uint64_t* tsum, uint32_t ntiles) {
    uint64_t carry = 0;
    for (uint32_t b = 0; b < ntiles; b += 64) {
        const uint32_t i = b + threadIdx.x;
        const uint64_t x = i < ntiles ? tsum[i] : 0ull;
        // (tile sums < 2^32: a u32 scan of the wave, then the 64-bit carry)
        const uint32_t incl = wave_incl_sum((uint32_t)x);
        if (i < ntiles) tsum[i] = carry + incl - (uint32_t)x;
        carry += readlane(incl, 63);
    }
}

__global__ __launch_bounds__(ST) void k_scan_tiles(const uint64_t* sizes, uint64_t* off, uint32_t count,
                                                   const uint64_t* tbase) {
    __shared__ uint32_t ws[ST / 64];
    const uint32_t i0 = blockIdx.x * TILE + threadIdx.x * SPT;
    uint32_t v[SPT], s = 0;
    load16(sizes, count, i0, v);
#pragma unroll
    for (uint32_t q = 0; q < SPT; q++) s += v[q];
    uint32_t total;
    uint64_t o = tbase[blockIdx.x] + tile_excl(s, ws, total);
#pragma unroll
    for (uint32_t q = 0; q < SPT; q++) {
        if (i0 + q < count) off[i0 + q] = o;
        o += v[q];
    }
}

}  // namespace

hipError_t scan_sizes(const uint64_t* sizes, uint64_t* off, uint32_t count, void* tmp,
                      size_t* tmp_bytes, hipStream_t s) {
    const uint32_t ntiles = (count + TILE - 1) / TILE;
    if (!tmp) {                       // size query
        *tmp_bytes = (size_t)(ntiles + 2) * sizeof(uint64_t);
        return hipSuccess;
    }
    if (!count) return hipSuccess;
    uint64_t* tsum = static_cast<uint64_t*>(tmp);
    hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(ST), 0, s, sizes, count, tsum);
    hipLaunchKernelGGL(k_scan_bases, dim3(1), dim3(64), 0, s, tsum, ntiles);
    hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(ST), 0, s, sizes, off, count, tsum);
    return hipGetLastError();
}

}  // namespace ambc
