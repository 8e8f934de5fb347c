// Wavefront (64-lane) primitives for gfx950.  Everything here assumes the
// whole wave is active (EXEC all ones) -- callers keep control flow
// wave-uniform around these helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ambc {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        uint64_t t = __shfl_xor(v, o);
        v = t < v ? t : v;
    }
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// inclusive prefix sum over lanes
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o);
        if (l >= (uint32_t)o) v += t;
    }
    return v;
}

// exclusive prefix max over lanes (lane 0 gets `init`)
__device__ __forceinline__ int wave_excl_max(int v, int init) {
    const uint32_t l = lane_id();
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(x, o);
        if (l >= (uint32_t)o) x = max(x, t);
    }
    int ex = __shfl_up(x, 1);
    return l == 0 ? init : max(ex, init);
}

__device__ __forceinline__ uint32_t bcast0(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace ambc
