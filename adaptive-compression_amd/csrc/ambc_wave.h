// Wavefront (64-lane) primitives for gfx950.  Everything here assumes the
// whole wave is active (EXEC all ones) -- callers keep control flow
// wave-uniform around these helpers.
//
// Scans and reductions use DPP row shifts + row_bcast15/31 (VALU, a few cycles
// each) instead of ds_bpermute shuffles (an LDS round trip each), and read the
// result back with v_readlane.  Define AMBC_SHFL_PRIMITIVES to fall back to
// the __shfl versions (debugging aid).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ambc {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// only wavefront-scope ordering is needed inside a one-wave workgroup: LDS
// instructions of a wave execute in order, so this is a compiler barrier and
// never waits on outstanding global stores (unlike __syncthreads()).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

#define AMBC_DPP(old, v, ctrl, rm, bm, bc) \
    ((uint32_t)__builtin_amdgcn_update_dpp((int)(old), (int)(v), ctrl, rm, bm, bc))

#ifndef AMBC_SHFL_PRIMITIVES

// inclusive prefix sum over lanes
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += AMBC_DPP(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += AMBC_DPP(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += AMBC_DPP(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += AMBC_DPP(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += AMBC_DPP(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1,3
    v += AMBC_DPP(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2,3
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) { return readlane(wave_incl_sum(v), 63); }

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    const uint32_t M = 0xFFFFFFFFu;
    v = min(v, AMBC_DPP(M, v, 0x111, 0xF, 0xF, false));
    v = min(v, AMBC_DPP(M, v, 0x112, 0xF, 0xF, false));
    v = min(v, AMBC_DPP(M, v, 0x114, 0xF, 0xF, false));
    v = min(v, AMBC_DPP(M, v, 0x118, 0xF, 0xF, false));
    v = min(v, AMBC_DPP(M, v, 0x142, 0xA, 0xF, false));
    v = min(v, AMBC_DPP(M, v, 0x143, 0xC, 0xF, false));
    return readlane(v, 63);
}

// inclusive prefix max of signed values (identity INT_MIN)
__device__ __forceinline__ int wave_incl_max_i32(int v) {
    const int M = (int)0x80000000;
    v = max(v, (int)AMBC_DPP(M, v, 0x111, 0xF, 0xF, false));
    v = max(v, (int)AMBC_DPP(M, v, 0x112, 0xF, 0xF, false));
    v = max(v, (int)AMBC_DPP(M, v, 0x114, 0xF, 0xF, false));
    v = max(v, (int)AMBC_DPP(M, v, 0x118, 0xF, 0xF, false));
    v = max(v, (int)AMBC_DPP(M, v, 0x142, 0xA, 0xF, false));
    v = max(v, (int)AMBC_DPP(M, v, 0x143, 0xC, 0xF, false));
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) { return (int)readlane((uint32_t)wave_incl_max_i32(v), 63); }

// exclusive prefix max over lanes (lane 0 gets `init`)
__device__ __forceinline__ int wave_excl_max(int v, int init) {
    const int incl = wave_incl_max_i32(v);
    const int ex = (int)AMBC_DPP(0x80000000u, incl, 0x138, 0xF, 0xF, false);  // wave_shr:1
    return lane_id() == 0 ? init : max(ex, init);
}

#else  // __shfl fallbacks

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o);
        if (l >= (uint32_t)o) v += t;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
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

#endif

// generic (64-bit / fp64) reductions stay on shuffles: off the hot loops
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
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

__device__ __forceinline__ uint32_t bcast0(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Values loaded from memory are not known to be wave-uniform even when every
// lane loaded the same address; these make that explicit so that the code
// depending on them stays on the scalar unit.
// (the builtin returns int: go through uint32_t so that nothing sign-extends)
__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return (uint64_t)uniform_u32((uint32_t)v) | (uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32;
}
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    return reinterpret_cast<T*>(uniform_u64(reinterpret_cast<uint64_t>(p)));
}

// zlib's Adler-32 of n bytes at src, by one whole wave: whole 16-byte pieces of a
// 16-byte aligned source as vector loads four in flight per lane, each dword's
// byte sum (v_sad_u8) and index-weighted sum (v_dot4) folded in at once; the rest
// (and any unaligned source) a byte per lane; nothing is read at or past src + n.
// (A byte per lane per iteration waits on one load at a time: 64 serial load
// latencies for a 4 KiB chunk.)
__device__ __forceinline__ uint32_t adler32_wave(const uint8_t* src, uint32_t n, uint32_t lane) {
    uint64_t asum = 0, bsum = 0;
    const uint32_t nq = (reinterpret_cast<uintptr_t>(src) & 15) == 0 ? n / 16 : 0;
#pragma unroll 1
    for (uint32_t q0 = 0; q0 < nq; q0 += 256) {
        uint4 w[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t q = q0 + (uint32_t)t * 64 + lane;
            w[t] = q < nq ? reinterpret_cast<const uint4*>(src)[q] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t i0 = 16 * (q0 + (uint32_t)t * 64 + lane);
            const uint32_t ww[4] = {w[t].x, w[t].y, w[t].z, w[t].w};
#pragma unroll
            for (int d = 0; d < 4; d++) {
                // bytes c_j at i0 + 4d + j: sum c_j (n - i0 - 4d - j) = (n - i0 - 4d) sum c_j - sum j c_j
                const uint32_t s0 = __builtin_amdgcn_sad_u8(ww[d], 0u, 0u);
                const uint32_t s1 = __builtin_amdgcn_udot4(ww[d], 0x03020100u, 0u, false);
                asum += s0;
                bsum += (uint64_t)((n - i0 - 4u * (uint32_t)d) * s0 - s1);   // (zero for pieces past nq)
            }
        }
    }
    for (uint32_t i = 16 * nq + lane; i < n; i += 64) {
        const uint32_t c = src[i];
        asum += c;
        bsum += (uint64_t)(n - i) * c;
    }
    asum = wave_sum<uint64_t>(asum);
    bsum = wave_sum<uint64_t>(bsum);
    return (uint32_t)(((n + bsum) % 65521) << 16 | ((1 + asum) % 65521));
}

}  // namespace ambc
