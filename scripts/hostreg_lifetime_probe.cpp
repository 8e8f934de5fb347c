// Diagnostic (round 6): does a caller range stay locked at the ROCr level after
// hipHostUnregister returns?  Queries only -- no buffer is freed while a DMA or a
// registration could still touch it, no fault is provoked.
//
// Scenarios, each on its own fresh mmap'd range (as Python's large bytes are):
//   up   : pieces registered, H2D DMA per piece + event record on one stream
//          (start_registered_upload's pattern), sync, unregister
//   down : pieces registered, D2H DMA per piece as the stream's LAST command
//          (OutDMA's pattern), sync, unregister
//   page : pageable 1 MiB / 8 MiB hipMemcpy both ways (the runtime's own path)
// After each step the probe prints hsa_amd_pointer_info's type for every piece
// (0 unknown, 1 hsa, 2 locked ...).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static int ptype(const void* p) {
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof info);
    info.size = sizeof info;
    if (hsa_amd_pointer_info(const_cast<void*>(p), &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return -1;
    return (int)info.type;
}

static void show(const char* tag, const std::vector<uint8_t*>& pcs) {
    printf("  %-34s", tag);
    for (auto* p : pcs) printf(" %d", ptype(p));
    int hp = -1;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, pcs.back()) == hipSuccess) hp = (int)a.type;
    (void)hipGetLastError();
    printf("   (hipPointerGetAttributes type %d)\n", hp);
}

static uint8_t* fresh(size_t n) {
    void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) { printf("mmap failed\n"); exit(1); }
    for (size_t i = 0; i < n; i += 4096) static_cast<uint8_t*>(p)[i] = 1;
    return static_cast<uint8_t*>(p);
}

static void scenario(const char* name, bool to_dev, bool event_after, size_t n, size_t piece) {
    printf("%s: %zu MiB in %zu MiB pieces, %s, %s\n", name, n >> 20, piece >> 20, to_dev ? "H2D" : "D2H",
           event_after ? "event record after each DMA" : "DMA is the stream's last command");
    uint8_t* h = fresh(n);
    void* d = nullptr;
    CK(hipMalloc(&d, n));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<uint8_t*> pcs;
    for (size_t o = 0; o < n; o += piece) pcs.push_back(h + o);
    show("before register", pcs);
    for (size_t k = 0; k < pcs.size(); k++) {
        const size_t len = std::min(piece, n - k * piece);
        CK(hipHostRegister(pcs[k], len, hipHostRegisterDefault));
    }
    show("registered", pcs);
    for (size_t k = 0; k < pcs.size(); k++) {
        const size_t len = std::min(piece, n - k * piece);
        uint8_t* dk = static_cast<uint8_t*>(d) + k * piece;
        if (to_dev) CK(hipMemcpyAsync(dk, pcs[k], len, hipMemcpyHostToDevice, s));
        else CK(hipMemcpyAsync(pcs[k], dk, len, hipMemcpyDeviceToHost, s));
        if (event_after) CK(hipEventRecord(ev, s));
    }
    CK(hipStreamSynchronize(s));
    show("DMAs done (synced)", pcs);
    for (auto* p : pcs) CK(hipHostUnregister(p));
    show("unregistered", pcs);
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    show("200 ms later", pcs);
    CK(hipMemsetAsync(d, 0, 64, s));
    CK(hipStreamSynchronize(s));
    show("a device memset on the stream", pcs);
    CK(hipStreamDestroy(s));
    show("stream destroyed", pcs);
    CK(hipDeviceSynchronize());
    show("device synchronized", pcs);
    CK(hipEventDestroy(ev));
    CK(hipFree(d));
    munmap(h, n);
    show("after munmap", pcs);
}

static void pageable(size_t n) {
    printf("page: pageable %zu KiB hipMemcpy both ways (malloc'd)\n", n >> 10);
    uint8_t* h = static_cast<uint8_t*>(malloc(n));
    memset(h, 3, n);
    void* d = nullptr;
    CK(hipMalloc(&d, n));
    std::vector<uint8_t*> pcs{h};
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    show("after H2D", pcs);
    CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    show("after D2H", pcs);
    CK(hipFree(d));
    free(h);
}

int main() {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    scenario("up", true, true, 96ull << 20, 64ull << 20);
    scenario("down", false, false, 96ull << 20, 32ull << 20);
    scenario("down-ev", false, true, 96ull << 20, 32ull << 20);
    pageable(1 << 20);
    pageable(8 << 20);
    printf("done\n");
    return 0;
}
