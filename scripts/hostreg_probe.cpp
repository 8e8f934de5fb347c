// Probe: cost of hipHostRegister on pageable buffers (fresh calloc'd, pre-faulted)
// and DMA rates from / to registered vs staged memory.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static void touch(uint8_t* p, size_t n, int T) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back([=] { for (size_t i = n * t / T; i < n * (t + 1) / T; i += 4096) p[i] = 1; });
    for (auto& x : th) x.join();
}
int main() {
    const size_t N = 4ull << 30;
    void* dev = nullptr;
    CK(hipMalloc(&dev, N));
    for (int mode = 0; mode < 3; mode++) {
        uint8_t* h = (uint8_t*)calloc(N, 1);
        if (mode >= 1) madvise((void*)(((uintptr_t)h + (2 << 20) - 1) & ~(uintptr_t)((2 << 20) - 1)), N - (4 << 20), MADV_HUGEPAGE);
        double t0 = now();
        if (mode == 2) touch(h, N, 16);
        double t1 = now();
        CK(hipHostRegister(h, N, hipHostRegisterDefault));
        double t2 = now();
        CK(hipMemcpy(h, dev, N, hipMemcpyDeviceToHost));
        double t3 = now();
        CK(hipMemcpy(dev, h, N, hipMemcpyHostToDevice));
        double t4 = now();
        CK(hipHostUnregister(h));
        double t5 = now();
        printf("mode %d (0 fresh, 1 fresh+THP, 2 THP+prefault16): prefault %.1f ms register %.1f ms D2H %.1f ms (%.1f GB/s) H2D %.1f ms (%.1f GB/s) unregister %.1f ms\n",
               mode, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, N / (t3 - t2) / 1e9, (t4 - t3) * 1e3, N / (t4 - t3) / 1e9, (t5 - t4) * 1e3);
        free(h);
    }
    // concurrent H2D (2 GiB) + D2H (4 GiB) from registered buffers on two streams
    uint8_t* a = (uint8_t*)malloc(N); uint8_t* b = (uint8_t*)malloc(N / 2);
    touch(a, N, 16); touch(b, N / 2, 16);
    CK(hipHostRegister(a, N, 0)); CK(hipHostRegister(b, N / 2, 0));
    void* dev2; CK(hipMalloc(&dev2, N / 2));
    hipStream_t s1, s2; CK(hipStreamCreate(&s1)); CK(hipStreamCreate(&s2));
    double t0 = now();
    CK(hipMemcpyAsync(a, dev, N, hipMemcpyDeviceToHost, s1));
    CK(hipMemcpyAsync(dev2, b, N / 2, hipMemcpyHostToDevice, s2));
    CK(hipStreamSynchronize(s1)); double t1 = now(); CK(hipStreamSynchronize(s2)); double t2 = now();
    printf("concurrent: D2H 4 GiB %.1f ms, H2D 2 GiB done at %.1f ms\n", (t1 - t0) * 1e3, (t2 - t0) * 1e3);
    return 0;
}
