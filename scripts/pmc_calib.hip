// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the
// encode kernels use (MI355X_MICROARCH.md: only 16-B-per-lane streaming reads
// are calibrated -- they count half; every other width must be calibrated on a
// known byte count).  Each kernel touches exactly NB bytes of a buffer larger
// than the MALL once, in one of the patterns below; run it under
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib     (and again with WRITE_SIZE)
// and divide the counter (KiB) by NB / 1024.
//
//   rd16   global_load_dwordx4, lane-consecutive (pass A, k_compact)
//   rd4    global_load_dword, lane-consecutive
//   rd1    global_load_ubyte, lane-consecutive (emission, raw copies)
//   rdu    every byte position reads the two aligned dwords around it
//          (k_encode's LZ4 probe: 64 consecutive positions per wave)
//   rdblk  every lane owns 64 contiguous bytes, read as four 16-B loads
//          (k_encode's pass A at chunks >= 4 KiB: BS = 64)
//   rdpa   rdblk plus the dword before the block and its first byte (pass A's
//          previous word and run byte)
//   wr16 / wr4 / wr1   the same widths as stores
//
//   hipcc --offload-arch=gfx950 -O3 -o pmc_calib scripts/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void rd16(const uint4* __restrict__ p, size_t n16, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void rd4(const uint32_t* __restrict__ p, size_t n4, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void rd1(const uint8_t* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// position i reads dwords i/4 and i/4 + 1 (the last position of the buffer
// reads one dword past i/4 only while it is inside)
__global__ void rdu(const uint32_t* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const size_t n4 = n / 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t w = i >> 2;
        const uint32_t lo = p[w], hi = w + 1 < n4 ? p[w + 1] : 0u;
        acc ^= __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(i & 3) * 8u);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <bool PA>
__global__ void rdblk(const uint8_t* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t b = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * 64; b < n; b += (size_t)gridDim.x * blockDim.x * 64) {
        if (PA) {
            acc ^= b ? reinterpret_cast<const uint32_t*>(p)[(b >> 2) - 1] : 0u;
            acc += p[b];
        }
#pragma unroll 1
        for (int q = 0; q < 4; q++) {
            const uint4 v = *reinterpret_cast<const uint4*>(p + b + 16 * q);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void wr16(uint4* __restrict__ p, size_t n16, uint32_t s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i ^ s, (uint32_t)i + s, (uint32_t)i * s, s);
}

__global__ void wr4(uint32_t* __restrict__ p, size_t n4, uint32_t s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i ^ s;
}

__global__ void wr1(uint8_t* __restrict__ p, size_t n, uint32_t s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint8_t)(i ^ s);
}

int main(int argc, char** argv) {
    const size_t NB = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t)1 << 30);
    const int reps = 3, blocks = 8192, threads = 256;
    uint8_t* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, NB + 64));
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    CHECK(hipMemset(buf, 0x5a, NB + 64));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto run = [&](const char* name, auto&& launch) {
        for (int r = 0; r < reps; r++) {
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            printf("{\"kernel\": \"%s\", \"rep\": %d, \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n",
                   name, r, NB, ms, NB / (ms * 1e6));
        }
    };
    run("rd16", [&] { rd16<<<blocks, threads>>>((const uint4*)buf, NB / 16, out); });
    run("rd4", [&] { rd4<<<blocks, threads>>>((const uint32_t*)buf, NB / 4, out); });
    run("rd1", [&] { rd1<<<blocks, threads>>>(buf, NB, out); });
    run("rdu", [&] { rdu<<<blocks, threads>>>((const uint32_t*)buf, NB, out); });
    run("rdblk", [&] { rdblk<false><<<blocks, threads>>>(buf, NB, out); });
    run("rdpa", [&] { rdblk<true><<<blocks, threads>>>(buf, NB, out); });
    run("wr16", [&] { wr16<<<blocks, threads>>>((uint4*)buf, NB / 16, 7u); });
    run("wr4", [&] { wr4<<<blocks, threads>>>((uint32_t*)buf, NB / 4, 7u); });
    run("wr1", [&] { wr1<<<blocks, threads>>>(buf, NB, 7u); });
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
