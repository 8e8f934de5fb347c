// ambc_host.cpp -- the C-ABI of libambc_hip.so (include/ambc.h).
//
// Host orchestration only: device workspaces, streams, H2D/D2H, the serial
// chunk-header walk of _adaptive_decompress (adaptive_compressor.py:399-445,
// which cannot be parallelised without the lengths it reads) and the launch
// sequences.  Every byte of codec work runs in the HIP kernels; there is no
// CPU codec path here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>
#include <zlib.h>

#include "../../include/ambc.h"
#include "ambc_hostctx.h"
#include "ambc_internal.h"

using namespace ambc;

namespace ambc {
thread_local std::string g_err;
}  // namespace ambc


// a chunk's scratch slot: winners are < n bytes; forced single-method encodes
// (ambc_encode_method) can reach 2n (RLE) or ~1.13n + 1284 (Huffman), plus the
// Huffman bit staging area behind the payload.  A Huffman winner of more than
// 2812 bytes stages its bits behind the payload too (k_encode's LDS staging
// holds 2816 B), hence 2C.
constexpr uint32_t NSEG = 4;   // pipelined compress segments (<= 8 = Dev::pev)

uint32_t ambc::slot_stride_for(uint32_t C, bool forced) {
    const uint32_t need = forced ? 3 * C + 1344 : 2 * C + 64;
    return (need + 15) & ~15u;
}

extern "C" {

int ambc_abi_version(void) { return AMBC_ABI_VERSION; }
const char* ambc_last_error(void) { return g_err.c_str(); }

int ambc_device_count(int* count) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) { *count = 0; return fail(AMBC_E_DEVICE, hipGetErrorString(e)); }
    *count = c;
    return AMBC_OK;
}

int ambc_init(const int* device_ids, int n_devices, ambc_ctx** out) {
    if (!out) return fail(AMBC_E_INVAL, "out is NULL");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        return fail(AMBC_E_DEVICE, "no HIP device available (libambc_hip has no CPU fallback)");
    std::unique_ptr<ambc_ctx> ctx(new ambc_ctx());
    int nd = n_devices > 0 ? n_devices : 1;
    if (device_ids && nd > 1) {
        // in-process RCCL ranks (ambc_shard.cpp make_transports): every connection
        // at ncclCommInitAll rather than inside a rank thread's first collective
        // (RCCL 2.27 connects lazily and waits for its peers there).  Set here, once,
        // when a multi-device ctx is made -- before any of the library's threads
        // exist -- and only if the caller has not chosen (setenv's overwrite = 0).
        std::set<int> distinct(device_ids, device_ids + nd);
        if ((int)distinct.size() > 1) setenv("NCCL_RUNTIME_CONNECT", "0", 0);
    }
    for (int i = 0; i < nd; i++) {
        Dev d;
        d.id = device_ids ? device_ids[i] : i;
        if (d.id < 0 || d.id >= count) return fail(AMBC_E_INVAL, "device id out of range");
        HIPCHK(hipSetDevice(d.id));
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, d.id));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(AMBC_E_DEVICE, std::string("libambc_hip is built for gfx950, device is ") +
                                           prop.gcnArchName);
        HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        for (auto& ev : d.ev) HIPCHK(hipEventCreate(&ev));
        for (auto& x : d.xs) HIPCHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        for (auto& ev : d.xev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        // the scan + compaction stream; AMBC_CS_PRIO=1: high priority (measured, §4)
        if (getenv("AMBC_CS_PRIO") && atoi(getenv("AMBC_CS_PRIO")) > 0) {
            int lo = 0, hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(hipStreamCreateWithPriority(&d.cs, hipStreamNonBlocking, hi));
        } else {
            HIPCHK(hipStreamCreateWithFlags(&d.cs, hipStreamNonBlocking));
        }
        for (auto& ev : d.pev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIPCHK(hipStreamCreateWithFlags(&d.zs, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&d.zev, hipEventDisableTiming));
        ctx->devs.push_back(d);
    }
    *out = ctx.release();
    return AMBC_OK;
}

void ambc_destroy(ambc_ctx* ctx) {
    if (!ctx) return;
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    for (ncclComm_t c : ctx->dev_comms) if (c) (void)ncclCommDestroy(c);
    for (auto& d : ctx->devs) {
        (void)hipSetDevice(d.id);
        (void)hipStreamSynchronize(d.stream);
        for (Buf* b : {&d.in, &d.out, &d.slots, &d.plen, &d.ids, &d.sizes, &d.off, &d.scan_tmp,
                       &d.acc, &d.ent_full, &d.ent_tail, &d.body, &d.jobs, &d.produced, &d.dout,
                       &d.scratch, &d.seg, &d.list, &d.bestpre, &d.gdseq, &d.pending, &d.z9rec, &d.z9scr, &d.segbase, &d.coll,
                       &d.inffix, &d.ms_out, &d.ms_ent})
            b->release();
        if (d.hacc) { (void)hipHostFree(d.hacc); d.hacc = nullptr; }
        for (auto& b : d.msb) b.release();
        d.dw.release();
        for (auto& x : d.mss) if (x) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); }
        for (void* b : d.stage) (void)hipHostFree(b);
        for (auto& ev : d.stage_ev) (void)hipEventDestroy(ev);
        for (auto& x : d.stage_st) (void)hipStreamDestroy(x);
        for (void* b : d.stage1) (void)hipHostFree(b);
        for (auto& ev : d.stage1_ev) (void)hipEventDestroy(ev);
        for (auto& x : d.stage1_st) (void)hipStreamDestroy(x);
        for (auto& ev : d.ev) (void)hipEventDestroy(ev);
        for (auto& ev : d.xev) (void)hipEventDestroy(ev);
        for (auto& x : d.xs) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); }
        for (auto& ev : d.pev) (void)hipEventDestroy(ev);
        (void)hipStreamSynchronize(d.cs);
        (void)hipStreamDestroy(d.cs);
        if (d.zs) { (void)hipStreamSynchronize(d.zs); (void)hipStreamDestroy(d.zs); }
        if (d.zev) (void)hipEventDestroy(d.zev);
        (void)hipStreamDestroy(d.stream);
    }
    delete ctx;
}

uint64_t ambc_compress_bound(uint64_t n, uint32_t chunk) {
    if (chunk == 0) return 0;
    return n + (uint64_t)HDR * ((n + chunk - 1) / chunk) + END_CHUNK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// compress (device resident)
// ---------------------------------------------------------------------------
// the largest chunk id 2 can be eligible for (k_dict's template bucket)
static uint32_t dict_cmax(const ambc_params* p) { return std::min(p->chunk_size, p->pref_max[AMBC_M_DICT]); }

int ambc::check_params(const ambc_params* p) {
    if (!p) return fail(AMBC_E_INVAL, "params is NULL");
    const uint32_t C = p->chunk_size;
    if (C < 16 || C > AMBC_MAX_CHUNK || (C & 15))
        return fail(AMBC_E_INVAL, "chunk_size must be a multiple of 16 in [16, 65536]");
    if (p->mode > 1) return fail(AMBC_E_INVAL, "mode must be AMBC_MODE_NATIVE or AMBC_MODE_REFERENCE");
    const uint32_t allowed = (1u << AMBC_M_RLE) | (1u << AMBC_M_DICT) | (1u << AMBC_M_HUFFMAN) |
                             (1u << AMBC_M_DELTA) | (1u << AMBC_M_DEFLATE) | (1u << AMBC_M_LZ4);
    if (p->method_mask & ~allowed)
        return fail(AMBC_E_INVAL, "method_mask holds ids without a GPU encoder (allowed: 1, 2, 3, 4, 5, 9)");
    if (((p->method_mask >> AMBC_M_DEFLATE) & 1) && (p->flags & AMBC_FLAG_ZLIB9) && z9_cmax(C) == 0)
        return fail(AMBC_E_INVAL, "the GPU zlib-9 encoder (AMBC_FLAG_ZLIB9) supports chunk_size <= 65536");
    if (((p->method_mask >> AMBC_M_DICT) & 1) && p->pref_min[AMBC_M_DICT] <= dict_cmax(p) &&
        dict_cmax(p) > 8192)
        return fail(AMBC_E_INVAL, "the GPU Dictionary encoder takes chunks <= 8192 bytes "
                                  "(chunk_size or pref_max[2] <= 8192)");
    return AMBC_OK;
}

// The raw remainder of reference mode (adaptive_compressor.py:586-588: the
// first position with no winner stores the rest of the file as ONE raw chunk).
// In a sharded call the remainder can span ranks: the rank holding its first
// chunk writes the 18-B header with the WHOLE remainder's length and its own
// bytes of it; every later rank contributes its shard's bytes verbatim.
struct Remainder {
    bool hdr = false;        // this rank writes the remainder's chunk header
    uint64_t rem_total = 0;  // used / orig / comp_len of that header
    uint64_t copy_off = 0;   // local input bytes [copy_off, copy_off + copy_len) follow
    uint64_t copy_len = 0;
};

// the raw remainder, end chunk, kernel times and stats of one compress call,
// after the R packages are in the body and acc[] is on the host
static int finish_compress(Dev& d, const ambc_params* p, uint32_t R, const Remainder& rm, uint8_t* d_out,
                           uint64_t body_len, const std::vector<uint64_t>& acc, const uint8_t* d_in,
                           bool end, uint64_t* out_len, ambc_stats* st, uint64_t t0, bool end_written = false) {
    hipStream_t s = d.stream;
    if (rm.hdr) {
        const uint64_t rem = rm.rem_total;
        uint8_t h[HDR] = {0xFF, 0xFF, 0, 0, 255, 0};
        for (int b = 0; b < 4; b++) {
            h[6 + b] = (uint8_t)(rem >> (8 * b));
            h[10 + b] = (uint8_t)(rem >> (8 * b));
            h[14 + b] = (uint8_t)(rem >> (8 * b));
        }
        HIPCHK(hipMemcpy(d_out + body_len, h, HDR, hipMemcpyHostToDevice));
        body_len += HDR;
    }
    if (rm.copy_len) {
        HIPCHK(launch_copy(d_out + body_len, d_in + rm.copy_off, rm.copy_len, s));
        body_len += rm.copy_len;
    }
    if (end) {
        if (!end_written) HIPCHK(launch_end_chunk(d_out + body_len, s));
        body_len += END_CHUNK;
    }
    HIPCHK(hipEventRecord(d.ev[4], s));
    HIPCHK(hipStreamSynchronize(s));
    TRACE("tail done");
    float ms_enc = 0, ms_scan = 0, ms_cmp = 0, ms_all = 0;
    HIPCHK(hipEventElapsedTime(&ms_enc, d.ev[0], d.ev[1]));
    HIPCHK(hipEventElapsedTime(&ms_scan, d.ev[1], d.ev[2]));
    HIPCHK(hipEventElapsedTime(&ms_cmp, d.ev[2], d.ev[3]));
    HIPCHK(hipEventElapsedTime(&ms_all, d.ev[0], d.ev[4]));
    d.t_encode = (uint64_t)(ms_enc * 1e6);
    d.t_scan = (uint64_t)(ms_scan * 1e6);
    d.t_compact = (uint64_t)(ms_cmp * 1e6);
    *out_len = body_len;
    if (st) {
        std::memset(st, 0, sizeof *st);
        for (int i = 0; i < 256; i++) st->method_usage[i] = acc[i];
        st->method_usage[255] = 0;   // the reference counts compressed chunks only
        st->compressed_chunks = acc[256];
        st->total_chunks = R + (rm.hdr ? 1 : 0);
        st->raw_chunks = st->total_chunks - st->compressed_chunks;
        st->payload_bytes = acc[258];
        st->bytes_saved = acc[259];
        st->overhead_bytes = (uint64_t)HDR * st->compressed_chunks + (end ? END_CHUNK : 0);
        st->kernel_ns = (uint64_t)(ms_all * 1e6);
        st->total_ns = now_ns() - t0;
    }
    (void)p;
    return AMBC_OK;
}

// workgroups of the compaction grid that runs beside the next segment's encoder
// (AMBC_COMPACT_RESIDENT overrides, for measurements).  With the 16-byte group
// compaction a larger grid finishes sooner beside the encoder: same-box A/B of the
// headline, 1024 -> 256 / 512 / 2048 / 4096 / 8192 / 16384 / 65536 workgroups:
// 365.3 -> 346.8 / 358.0 / 369.0 / 371.1 / 371.0 / 371.0 / 369.5 GB/s
// (profiles/r4_compact_grid_ab)
static uint32_t compact_resident() {
    static const uint32_t r = [] {
        const char* e = getenv("AMBC_COMPACT_RESIDENT");
        return e && atoi(e) > 0 ? (uint32_t)atoi(e) : 8192u;
    }();
    return r;
}

// compress_on's body.  `armed` is set once the pre-flight checks passed (every
// rank of a sharded call fails those alike) and `joined` once the call entered
// reference mode's remainder exchange: compress_on joins that exchange on behalf
// of any later failure, so that no peer waits in it for a rank that left.
// the sharded tests' failure injection (ambc_test_inject_failure; -1: none)
static std::atomic<int> g_fail_rank{-1};

static int compress_on_body(Dev& d, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint8_t* d_out,
                            uint64_t out_cap, uint64_t* out_len, ambc_stats* st, const ShardInfo* si,
                            bool& armed, bool& joined) {
    int rc = check_params(p);
    if (rc) return rc;
    const uint32_t C = p->chunk_size;
    const uint64_t M64 = (n + C - 1) / C;
    if (M64 > 0x7FFFFFFFull) return fail(AMBC_E_INVAL, "too many chunks for one device call");
    const uint32_t M = (uint32_t)M64;
    const bool end = !(p->flags & AMBC_FLAG_NO_END_CHUNK);
    const uint64_t bound = ambc_compress_bound(n, C) - (end ? 0 : END_CHUNK);
    if (out_cap < bound) return fail(AMBC_E_CAPACITY, "device output capacity < ambc_compress_bound");
    armed = true;
    if (si && g_fail_rank.load(std::memory_order_relaxed) == si->rank)   // (ambc_test_inject_failure)
        return fail(AMBC_E_DEVICE, "injected failure (ambc_test_inject_failure)");
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    const uint64_t t0 = now_ns();
    const uint32_t stride = slot_stride_for(C);
    HIPCHK(d.slots.ensure((size_t)std::max<uint32_t>(M, 1) * stride));
    HIPCHK(d.plen.ensure((size_t)(M + 1) * 4));
    HIPCHK(d.ids.ensure((size_t)M + 16));
    HIPCHK(d.sizes.ensure((size_t)(M + 1) * 8));
    HIPCHK(d.off.ensure((size_t)(M + 1) * 8));
    HIPCHK(d.acc.ensure(264 * 8));
    // exact entropy tables (optional)
    const double* ef = nullptr;
    const double* et = nullptr;
    if (p->ent_full) {
        HIPCHK(d.ent_full.ensure((size_t)(C + 1) * 8));
        HIPCHK(hipMemcpyAsync(d.ent_full.p, p->ent_full, (size_t)(C + 1) * 8, hipMemcpyHostToDevice, s));
        ef = d.ent_full.as<double>();
    }
    const uint32_t tail = (uint32_t)(n % C);
    if (p->ent_tail && tail) {
        HIPCHK(d.ent_tail.ensure((size_t)(tail + 1) * 8));
        HIPCHK(hipMemcpyAsync(d.ent_tail.p, p->ent_tail, (size_t)(tail + 1) * 8, hipMemcpyHostToDevice, s));
        et = d.ent_tail.as<double>();
    }
    EncArgs ea{};
    ea.in = d_in;
    ea.n_total = n;
    ea.chunk_size = C;
    ea.n_chunks = M;
    ea.slots = d.slots.as<uint8_t>();
    ea.slot_stride = stride;
    ea.method_mask = p->method_mask;
    ea.plen = d.plen.as<uint32_t>();
    ea.ids = d.ids.as<uint8_t>();
    ea.sizes = d.sizes.as<uint64_t>();
    ea.ent_full = ef;
    ea.ent_tail = et;
    for (int i = 0; i < 16; i++) { ea.pref_min[i] = p->pref_min[i]; ea.pref_max[i] = p->pref_max[i]; }
    // raw packages go from the input straight to the body (aligned inputs: k_compact's dword loads)
    const bool raw_in_place = ((uintptr_t)d_in & 3) == 0 && !getenv("AMBC_RAW_VIA_SLOT");
    if (raw_in_place) ea.flags |= ENC_RAW_IN_PLACE;
    // chunks read in place (k_encode, >= 16 KiB): 16-byte aligned chunk starts and
    // 64 readable bytes after the input (the library's own input buffers have them)
    const bool padded = (p->flags & AMBC_FLAG_INPUT_PADDED) ||
                        (d.in.p && d_in >= d.in.as<uint8_t>() && d_in + n + 64 <= d.in.as<uint8_t>() + d.in.cap);
    if (((uintptr_t)d_in & 15) == 0 && (C & 15) == 0 && padded && !getenv("AMBC_ENC_LDS")) ea.flags |= ENC_IN_ALIGNED;

    TRACE("compress_on n=%llu M=%u C=%u", (unsigned long long)n, M, C);
    std::vector<unsigned long long> stamps;
    if (getenv("AMBC_STAMPS")) {   // k_encode: M x 8 records, k_deflate: the next M x 8
        HIPCHK(d.seg.ensure((size_t)std::max<uint32_t>(M, 1) * 192));   // + k_dict: the third M x 8
        HIPCHK(hipMemsetAsync(d.seg.p, 0, (size_t)M * 192, s));
        ea.stamps = d.seg.as<unsigned long long>();
    }
    const bool deflate = (p->method_mask >> AMBC_M_DEFLATE) & 1;
    const bool z9 = deflate && (p->flags & AMBC_FLAG_ZLIB9);   // id 5 = zlib-9's bytes
    uint32_t gd_cmax = 1024;                  // launch_deflate's template bucket
    while (gd_cmax < C) gd_cmax <<= 1;
    const bool dict = (p->method_mask >> AMBC_M_DICT) & 1;
    if (deflate || dict) {
        // RLE / Huffman payloads wait for the later encoders' verdict (id 2, id 5);
        // a second k_encode launch emits the ones they did not replace
        HIPCHK(d.pending.ensure((size_t)std::max<uint32_t>(M, 1)));
        ea.pending = d.pending.as<uint8_t>();
    }
    if (deflate) {
        HIPCHK(d.bestpre.ensure((size_t)std::max<uint32_t>(M, 1) * 4));
        ea.bestpre = d.bestpre.as<uint32_t>();
        HIPCHK(d.gdseq.ensure((size_t)std::max<uint32_t>(M, 1) * gd_seq_bytes(gd_cmax)));
        ea.gdseq = d.gdseq.as<uint8_t>();
        if (z9) {
            HIPCHK(d.z9rec.ensure((size_t)std::max<uint32_t>(M, 1) * z9_rec_words(z9_cmax(C)) * 4));
            ea.z9rec = d.z9rec.as<uint32_t>();
            if (z9_cmax(C) > 8192) {   // the big parse's scratch: per resident workgroup, reused by segments
                HIPCHK(d.z9scr.ensure(z9_scratch_bytes(z9_cmax(C), std::max<uint32_t>(M, 1))));
                ea.z9scr = d.z9scr.as<uint8_t>();
            }
        }
    }
    // the kernels of one chunk range [k0, k1): every per-chunk array offset to k0
    auto seg_args = [&](uint32_t k0, uint32_t k1) {
        EncArgs e = ea;
        e.in += (uint64_t)k0 * C;
        e.n_total = std::min<uint64_t>(n - (uint64_t)k0 * C, (uint64_t)(k1 - k0) * C);
        e.n_chunks = k1 - k0;
        e.slots += (uint64_t)k0 * stride;
        e.plen += k0;
        e.ids += k0;
        e.sizes += k0;
        if (e.bestpre) e.bestpre += k0;
        if (e.pending) e.pending += k0;
        if (e.gdseq) e.gdseq += (uint64_t)k0 * gd_seq_bytes(gd_cmax);
        if (e.z9rec) e.z9rec += (uint64_t)k0 * z9_rec_words(z9_cmax(C));
        e.kbase = k0;
        return e;
    };
    // zlib-9 over pipelined segments (chunks up to 8 KiB, every scratch array per
    // chunk): a segment's trees, emission and pending payloads go to d.zs behind
    // its parse, so they run beside the next segment's encode and parse (the
    // parse is issue-bound at 4 workgroups per CU, the tree / emission kernels
    // latency-bound at low occupancy); its compaction waits for them
    static const bool z9_one_stream = getenv("AMBC_Z9_ONESTREAM") != nullptr;
    bool z9split = false;
    auto encode_range = [&](const EncArgs& e) -> int {
        HIPCHK(launch_encode(e, s));
        if (dict) HIPCHK(launch_dict(e, dict_cmax(p), s));   // id 2 against k_encode's winner
        // id 5 after 1/2/3/4, against LZ4 (ties -> 5)
        hipStream_t ts = s;
        if (deflate && z9 && z9split) {
            HIPCHK(launch_zlib9_parse(e, s));
            HIPCHK(hipEventRecord(d.zev, s));
            HIPCHK(hipStreamWaitEvent(d.zs, d.zev, 0));
            ts = d.zs;
            HIPCHK(launch_zlib9_tail(e, ts));
        } else if (deflate) {
            HIPCHK(z9 ? launch_zlib9(e, s) : launch_deflate(e, s));
        }
        if (deflate || dict) {
            EncArgs ep = e;                 // RLE/Huffman payloads ids 2 / 5 did not replace
            ep.flags |= ENC_EMIT_PENDING;
            ep.bestpre = nullptr;
            ep.stamps = nullptr;
            HIPCHK(launch_encode(ep, ts));
        }
        return AMBC_OK;
    };
    // Native mode over many chunks runs as NSEG pipelined segments: segment
    // i+1 encodes on the main stream while segment i is scanned and compacted
    // on d.cs (memory-bound work under the LDS-bound encoder).  Measured: one
    // encode stream beats launches alternating over two, 4 segments beat 5, 6
    // or 8 (the last segment's compaction stays exposed, ~0.4 ms), and equal
    // segments beat a short last one (3:3:3:1, 3:3:3:2, 4:4:4:1: +3 % step).  Reference mode
    // needs every verdict before the scan (remainder-raw rule): one range.
    static const uint32_t nseg = getenv("AMBC_NSEG") ? std::max(1, std::min(8, atoi(getenv("AMBC_NSEG")))) : NSEG;
    const uint32_t S = (p->mode != AMBC_MODE_REFERENCE && M >= 16384 && !ea.stamps) ? nseg : 1;
    d.n_launch = S;
    z9split = z9 && S > 1 && z9_cmax(C) <= 8192 && !z9_one_stream;
    HIPCHK(hipEventRecord(d.ev[0], s));
    if (S > 1) {
        size_t tmpb = 0;
        HIPCHK(scan_sizes(nullptr, nullptr, M / S + 1, nullptr, &tmpb, d.cs));
        HIPCHK(d.scan_tmp.ensure(tmpb));
        HIPCHK(d.segbase.ensure((S + 1) * 8));
        HIPCHK(hipMemsetAsync(d.segbase.p, 0, 8, d.cs));
        HIPCHK(hipMemsetAsync(d.acc.p, 0, 260 * 8, s));
        uint64_t* sb = d.segbase.as<uint64_t>();
        for (uint32_t i = 0; i < S; i++) {
            const uint32_t k0 = (uint32_t)((uint64_t)M * i / S), k1 = (uint32_t)((uint64_t)M * (i + 1) / S);
            rc = encode_range(seg_args(k0, k1));
            if (rc) return rc;
            HIPCHK(hipEventRecord(d.pev[i], z9split ? d.zs : s));
            if (z9split && i + 1 == S) HIPCHK(hipStreamWaitEvent(s, d.pev[i], 0));   // the statistics read every id
            if (i + 1 == S) HIPCHK(hipEventRecord(d.ev[1], s));
            HIPCHK(hipStreamWaitEvent(d.cs, d.pev[i], 0));
            size_t tb = tmpb;
            HIPCHK(scan_sizes(d.sizes.as<uint64_t>() + k0, d.off.as<uint64_t>() + k0, k1 - k0, d.scan_tmp.p,
                              &tb, d.cs));
            HIPCHK(launch_seg_base(sb + i, d.off.as<uint64_t>() + k1 - 1, d.sizes.as<uint64_t>() + k1 - 1, d.cs));
            if (i + 1 == S) HIPCHK(hipEventRecord(d.ev[2], d.cs));
            CompactArgs ca{};
            ca.slots = d.slots.as<uint8_t>() + (uint64_t)k0 * stride;
            ca.slot_stride = stride;
            ca.plen = d.plen.as<uint32_t>() + k0;
            ca.ids = d.ids.as<uint8_t>() + k0;
            ca.off = d.off.as<uint64_t>() + k0;
            ca.base = sb + i;
            ca.n_chunks = k1 - k0;
            ca.n_total = std::min<uint64_t>(n - (uint64_t)k0 * C, (uint64_t)(k1 - k0) * C);
            ca.chunk_size = C;
            ca.out = d_out;
            ca.in = raw_in_place ? d_in + (uint64_t)k0 * C : nullptr;
            // beside the next segment's encoder the compaction runs as a resident
            // grid (per-package-group workgroups would wait behind the encoder's
            // queued workgroups for every dispatch); the last one runs alone
            ca.resident = i + 1 < S ? compact_resident() : 0;
            HIPCHK(launch_compact(ca, d.cs));
        }
        // the statistics once, over every chunk, behind the last encode and beside the
        // last compaction.  Per-segment k_stats launches (round 3, on a stream of
        // their own) waited milliseconds for CU slots beside the next encode, and with
        // 4 hardware queues per process that stream shared one with d.cs: each held
        // the next segment's scan and compaction back (profiles/r4_stats_once_ab)
        HIPCHK(launch_stats(d.ids.as<uint8_t>(), d.plen.as<uint32_t>(), M, n, C, d.acc.as<uint64_t>(), s));
        // the end chunk and the body length behind the last compaction, then one
        // pinned copy back and one synchronisation (were two pageable copies, a
        // synchronisation, the end chunk's launch and another)
        HIPCHK(launch_end_chunk_at(end ? d_out : nullptr, sb + S, d.acc.as<uint64_t>() + 260, d.cs));
        HIPCHK(hipEventRecord(d.ev[3], d.cs));
        HIPCHK(hipStreamWaitEvent(s, d.ev[3], 0));
        if (!d.hacc) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&d.hacc), 264 * 8, hipHostMallocDefault));
        HIPCHK(hipMemcpyAsync(d.hacc, d.acc.p, 261 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<uint64_t> acc(d.hacc, d.hacc + 260);
        return finish_compress(d, p, M, Remainder(), d_out, d.hacc[260], acc, d_in, end, out_len, st, t0, true);
    }
    rc = encode_range(ea);
    if (rc) return rc;
    HIPCHK(hipEventRecord(d.ev[1], s));
    if (ea.stamps) {
        stamps.resize((size_t)M * 8);
        HIPCHK(hipMemcpyAsync(stamps.data(), d.seg.p, (size_t)M * 64, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        double sum[8] = {0};
        for (size_t q = 0; q < stamps.size(); q++) sum[q & 7] += (double)stamps[q];
        fprintf(stderr, "[ambc stamps] M=%u cycles/chunk: passA %.0f huff %.0f lz4hash %.0f lz4len %.0f "
                "lz4walk %.0f lz4tail+emit %.0f final %.0f lz4emit %.0f\n", M, sum[0] / M, sum[1] / M,
                sum[2] / M, sum[3] / M, sum[4] / M, sum[5] / M, sum[6] / M, sum[7] / M);
        if ((p->method_mask >> AMBC_M_DICT) & 1) {
            std::vector<unsigned long long> g((size_t)M * 8);
            HIPCHK(hipMemcpyAsync(g.data(), d.seg.as<unsigned long long>() + (size_t)M * 16, (size_t)M * 64,
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            double gs[8] = {0};
            for (size_t q = 0; q < g.size(); q++) gs[q & 7] += (double)g[q];
            const double c = std::max(gs[7], 1.0);
            fprintf(stderr, "[ambc stamps] dict parsed=%.0f wave-0 cycles/chunk: load %.0f should_use %.0f "
                    "buckets %.0f clear %.0f walk %.0f wait %.0f path+out %.0f\n", gs[7], gs[0] / c, gs[1] / c,
                    gs[2] / c, gs[3] / c, gs[4] / c, gs[5] / c, gs[6] / c);
        }
        if (z9 && !((p->method_mask >> AMBC_M_DICT) & 1)) {
            std::vector<unsigned long long> g((size_t)M * 8);
            HIPCHK(hipMemcpyAsync(g.data(), d.seg.as<unsigned long long>() + (size_t)M * 16, (size_t)M * 64,
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            double gs[8] = {0};
            for (size_t q = 0; q < g.size(); q++) gs[q & 7] += (double)g[q];
            const double c = std::max(gs[7], 1.0);
            fprintf(stderr, "[ambc stamps] z9 parsed=%.0f wave-0 cycles/chunk: load %.0f sort %.0f walk %.0f "
                    "wait %.0f path %.0f out %.0f\n", gs[7], gs[0] / c, gs[1] / c, gs[2] / c, gs[3] / c,
                    gs[4] / c, gs[5] / c);
            {   // big kernel, wave 0's walkers: iterations | chain steps << 16 | extension steps << 32 | searches << 48
                double it = 0, stp = 0, ex = 0, sr = 0;
                for (uint32_t q = 0; q < M; q++)
                    if (g[(size_t)q * 8 + 7]) {
                        const uint64_t w = g[(size_t)q * 8 + 6];
                        it += (double)(w & 0xFFFF); stp += (double)((w >> 16) & 0xFFFF);
                        ex += (double)((w >> 32) & 0xFFFF); sr += (double)(w >> 48);
                    }
                fprintf(stderr, "[ambc stamps] z9 wave-0 walker loop per chunk: iterations %.0f chain steps %.0f "
                        "extension steps %.0f searches %.0f\n", it / c, stp / c, ex / c, sr / c);
            }
            // the spread over chunks: percentiles of a parsed chunk's cycles, and the
            // share of all cycles in the slowest 10 %
            std::vector<double> tot;
            for (uint32_t q = 0; q < M; q++)
                if (g[(size_t)q * 8 + 7]) {
                    double t = 0;
                    for (int ph = 0; ph < 6; ph++) t += (double)g[(size_t)q * 8 + ph];
                    tot.push_back(t);
                }
            if (!tot.empty()) {
                std::sort(tot.begin(), tot.end());
                auto pct = [&](double f) { return tot[std::min(tot.size() - 1, (size_t)(f * tot.size()))]; };
                double all = 0, top = 0;
                for (size_t q = 0; q < tot.size(); q++) { all += tot[q]; if (q >= tot.size() * 9 / 10) top += tot[q]; }
                fprintf(stderr, "[ambc stamps] z9 chunk cycles p10 %.0f p50 %.0f p90 %.0f p99 %.0f max %.0f; "
                        "slowest 10%% hold %.1f%%\n", pct(0.1), pct(0.5), pct(0.9), pct(0.99), tot.back(),
                        100.0 * top / all);
            }
        }
        if (deflate) {
            std::vector<unsigned long long> g((size_t)M * 8);
            HIPCHK(hipMemcpyAsync(g.data(), d.seg.as<unsigned long long>() + (size_t)M * 8, (size_t)M * 64,
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            double gs[8] = {0};
            for (size_t q = 0; q < g.size(); q++) gs[q & 7] += (double)g[q];
            fprintf(stderr, "[ambc stamps] deflate cycles/chunk: stage %.0f parse %.0f freq %.0f "
                    "bound %.0f trees(rest) %.0f emit %.0f lengths %.0f rle %.0f\n", gs[0] / M, gs[1] / M,
                    gs[2] / M, gs[3] / M, gs[4] / M, gs[5] / M, gs[6] / M, gs[7] / M);
        }
    }

    // reference mode: the first chunk with no winner swallows the remainder
    uint32_t R = M;
    Remainder rm;
    if (p->mode == AMBC_MODE_REFERENCE && (M || si)) {
        std::vector<uint8_t> ids(M);
        if (M) HIPCHK(hipMemcpyAsync(ids.data(), d.ids.p, M, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (uint32_t k = 0; k < M; k++) if (ids[k] == 255) { R = k; break; }
        uint64_t g = R < M ? R : UINT64_MAX;          // first no-winner chunk (global index)
        uint64_t n_total = n, k0 = 0;
        if (si) {
            k0 = si->k0;
            n_total = si->n_total;
            if (g != UINT64_MAX) g += k0;
            joined = true;
            int rc2 = shard_allreduce_min(si->t, &g, AMBC_OK);  // AllReduce(MIN) across the ranks
            if (rc2) return rc2;
        }
        if (g != UINT64_MAX) {
            const uint64_t rem_total = n_total - g * C;
            if (rem_total > 0xFFFFFFFFull)
                return fail(AMBC_E_RANGE, "raw remainder does not fit the u32 chunk fields (struct.error)");
            if (g >= k0 + M) {
                R = M;                                  // a later rank holds the remainder's start
            } else if (g >= k0) {
                R = (uint32_t)(g - k0);                 // it starts in this shard
                rm.hdr = true;
                rm.rem_total = rem_total;
                rm.copy_off = (uint64_t)R * C;
                rm.copy_len = n - rm.copy_off;
            } else {
                R = 0;                                  // an earlier rank started it: all raw bytes
                rm.copy_len = n;
            }
        }
    }
    HIPCHK(hipMemsetAsync(d.sizes.as<uint64_t>() + R, 0, 8, s));
    size_t tmpb = 0;
    HIPCHK(scan_sizes(nullptr, nullptr, R + 1, nullptr, &tmpb, s));
    HIPCHK(d.scan_tmp.ensure(tmpb));
    TRACE("scan tmp=%zu", tmpb);
    HIPCHK(scan_sizes(d.sizes.as<uint64_t>(), d.off.as<uint64_t>(), R + 1, d.scan_tmp.p, &tmpb, s));
    HIPCHK(hipEventRecord(d.ev[2], s));
    if (trace_on()) { HIPCHK(hipStreamSynchronize(s)); TRACE("scan done"); }
    CompactArgs ca{};
    ca.slots = d.slots.as<uint8_t>();
    ca.slot_stride = stride;
    ca.plen = d.plen.as<uint32_t>();
    ca.ids = d.ids.as<uint8_t>();
    ca.off = d.off.as<uint64_t>();
    ca.n_chunks = R;
    ca.n_total = n;
    ca.chunk_size = C;
    ca.out = d_out;
    ca.in = raw_in_place ? d_in : nullptr;
    HIPCHK(launch_compact(ca, s));
    HIPCHK(hipEventRecord(d.ev[3], s));
    if (trace_on()) { HIPCHK(hipStreamSynchronize(s)); TRACE("compact done"); }
    HIPCHK(hipMemsetAsync(d.acc.p, 0, 260 * 8, s));
    HIPCHK(launch_stats(d.ids.as<uint8_t>(), d.plen.as<uint32_t>(), R, n, C, d.acc.as<uint64_t>(), s));
    uint64_t body_len = 0;
    HIPCHK(hipMemcpyAsync(&body_len, d.off.as<uint64_t>() + R, 8, hipMemcpyDeviceToHost, s));
    std::vector<uint64_t> acc(260);
    HIPCHK(hipMemcpyAsync(acc.data(), d.acc.p, 260 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    TRACE("stats done body_len=%llu", (unsigned long long)body_len);
    return finish_compress(d, p, R, rm, d_out, body_len, acc, d_in, end, out_len, st, t0);
}

int ambc::compress_on(Dev& d, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint8_t* d_out,
                      uint64_t out_cap, uint64_t* out_len, ambc_stats* st, const ShardInfo* si) {
    bool armed = false, joined = false;
    const int rc = compress_on_body(d, d_in, n, p, d_out, out_cap, out_len, st, si, armed, joined);
    if (rc && armed && !joined && si && p->mode == AMBC_MODE_REFERENCE) {
        // every failure after the pre-flight (buffers, launches, an asynchronous
        // kernel fault seen at a sync) joins the remainder exchange the peers wait in
        uint64_t g = UINT64_MAX;
        (void)shard_allreduce_min(si->t, &g, rc);
    }
    return rc;
}

extern "C" int ambc_compress_device(ambc_ctx* ctx, int dev, const void* d_in, uint64_t n,
                                    const ambc_params* p, void* d_out, uint64_t out_cap,
                                    uint64_t* out_len, ambc_stats* st, void* stream) {
    (void)stream;
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    if (!out_len) return fail(AMBC_E_INVAL, "out_len is NULL");
    return compress_on(ctx->devs[dev], (const uint8_t*)d_in, n, p, (uint8_t*)d_out, out_cap, out_len, st);
}

void ambc::add_stats(ambc_stats* a, const ambc_stats& b) {
    for (int i = 0; i < 256; i++) a->method_usage[i] += b.method_usage[i];
    a->total_chunks += b.total_chunks;
    a->compressed_chunks += b.compressed_chunks;
    a->raw_chunks += b.raw_chunks;
    a->bytes_saved += b.bytes_saved;
    a->payload_bytes += b.payload_bytes;
    a->overhead_bytes += b.overhead_bytes;
    a->kernel_ns = std::max(a->kernel_ns, b.kernel_ns);
}

// Host buffers in, host body out, with the copies overlapped: the input goes up
// in chunk-aligned slabs on one copy stream while the previous slab is being
// compressed and the one before that comes back on a second copy stream
// (double-buffered on the device).  Native mode only: slabs are independent
// there, so their bodies simply concatenate (the last one carries the end chunk).
// The overlap needs page-locked host buffers (ambc_host_alloc).
static constexpr uint64_t kSlabBytes = 256ull << 20;

// slab size of the host-fed pipelines (AMBC_SLAB_BYTES overrides, for tests)
uint64_t ambc::slab_bytes() {
    const char* e = getenv("AMBC_SLAB_BYTES");
    return e && strtoull(e, nullptr, 10) > 0 ? strtoull(e, nullptr, 10) : kSlabBytes;
}

static int compress_slabs(Dev& d, const uint8_t* in, uint64_t n, const ambc_params* p, uint8_t* out,
                          uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    const uint64_t t0 = now_ns();
    const uint32_t C = p->chunk_size;
    const uint64_t SLAB = std::max<uint64_t>(C, slab_bytes() / C * C);
    const uint64_t ns = (n + SLAB - 1) / SLAB;
    const uint64_t sb = ambc_compress_bound(SLAB, C) + 64;
    HIPCHK(hipSetDevice(d.id));
    HIPCHK(d.in.ensure(2 * (SLAB + 64)));
    HIPCHK(d.out.ensure(2 * sb));
    uint8_t* din[2] = {d.in.as<uint8_t>(), d.in.as<uint8_t>() + SLAB + 64};
    uint8_t* dout[2] = {d.out.as<uint8_t>(), d.out.as<uint8_t>() + sb};
    hipEvent_t* h2d_done = d.xev;
    hipEvent_t* comp_done = d.xev + 2;
    hipEvent_t* d2h_done = d.xev + 4;
    auto slab_len = [&](uint64_t k) { return std::min(SLAB, n - k * SLAB); };
    auto up = [&](uint64_t k) -> int {
        if (k >= 2) HIPCHK(hipStreamWaitEvent(d.xs[0], comp_done[k & 1], 0));  // din[k&1] free
        HIPCHK(hipMemcpyAsync(din[k & 1], in + k * SLAB, slab_len(k), hipMemcpyHostToDevice, d.xs[0]));
        HIPCHK(hipEventRecord(h2d_done[k & 1], d.xs[0]));
        return AMBC_OK;
    };
    ambc_stats tot{};
    uint64_t o = 0, kern = 0;
    int rc = up(0);
    for (uint64_t k = 0; k < ns && rc == AMBC_OK; k++) {
        if (k + 1 < ns && (rc = up(k + 1)) != AMBC_OK) break;
        HIPCHK(hipStreamWaitEvent(d.stream, h2d_done[k & 1], 0));
        if (k >= 2) HIPCHK(hipStreamWaitEvent(d.stream, d2h_done[k & 1], 0));  // dout[k&1] free
        ambc_params q = *p;
        if (k + 1 != ns) { q.flags |= AMBC_FLAG_NO_END_CHUNK; q.ent_tail = nullptr; }
        uint64_t len = 0;
        ambc_stats s1{};
        if ((rc = compress_on(d, din[k & 1], slab_len(k), &q, dout[k & 1], sb, &len, &s1)) != AMBC_OK) break;
        HIPCHK(hipEventRecord(comp_done[k & 1], d.stream));
        if (o + len > out_cap) { rc = fail(AMBC_E_CAPACITY, "output buffer too small for the body"); break; }
        HIPCHK(hipStreamWaitEvent(d.xs[1], comp_done[k & 1], 0));
        HIPCHK(hipMemcpyAsync(out + o, dout[k & 1], len, hipMemcpyDeviceToHost, d.xs[1]));
        HIPCHK(hipEventRecord(d2h_done[k & 1], d.xs[1]));
        o += len;
        kern += s1.kernel_ns;
        add_stats(&tot, s1);
    }
    HIPCHK(hipStreamSynchronize(d.xs[0]));
    HIPCHK(hipStreamSynchronize(d.xs[1]));
    if (rc != AMBC_OK) return rc;
    *out_len = o;
    if (st) {
        *st = tot;
        st->kernel_ns = kern;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

extern "C" int ambc_compress_batch(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                                   uint8_t* out, uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    if (!ctx || (!in && n) || !out || !out_len) return fail(AMBC_E_INVAL, "NULL argument");
    int rc = check_params(p);
    if (rc) return rc;
    const uint64_t t0 = now_ns();
    const uint32_t C = p->chunk_size;
    const uint64_t M = (n + C - 1) / C;
    // several devices in the ctx: contiguous chunk shards, one host thread per
    // device, sizes / stats / the reference-mode remainder over RCCL (ambc_shard.cpp)
    if (ctx->devs.size() > 1 && M >= ctx->devs.size())
        return compress_batch_multi(ctx, in, n, p, out, out_cap, out_len, st);
    Dev& d = ctx->devs[0];
    if (p->mode == AMBC_MODE_NATIVE && n > slab_bytes())
        return compress_slabs(d, in, n, p, out, out_cap, out_len, st);
    const uint64_t bound = ambc_compress_bound(n, C);
    HIPCHK(hipSetDevice(d.id));
    HIPCHK(d.in.ensure(n + 64));
    HIPCHK(d.out.ensure(bound + 64));
    uint64_t t = now_ns();
    if (n) HIPCHK(hipMemcpyAsync(d.in.p, in, n, hipMemcpyHostToDevice, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    const uint64_t h2d = now_ns() - t;
    uint64_t len = 0;
    rc = compress_on(d, d.in.as<uint8_t>(), n, p, d.out.as<uint8_t>(), d.out.cap, &len, st);
    if (rc) return rc;
    if (len > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small for the body");
    t = now_ns();
    HIPCHK(hipMemcpyAsync(out, d.out.p, len, hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    *out_len = len;
    if (st) {
        st->h2d_ns = h2d;
        st->d2h_ns = now_ns() - t;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

// ---------------------------------------------------------------------------
// per-chunk plugin entry points
// ---------------------------------------------------------------------------
static int run_encode_only(Dev& d, const uint8_t* h_in, uint64_t n, const ambc_params* p,
                           uint32_t flags, std::vector<uint8_t>& ids, std::vector<uint32_t>& plen,
                           std::vector<uint8_t>* su, std::vector<uint8_t>* slot0) {
    const uint32_t C = p->chunk_size;
    const uint32_t M = (uint32_t)((n + C - 1) / C);
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    const uint32_t stride = slot_stride_for(C, (flags & ENC_FORCE) != 0);
    HIPCHK(d.in.ensure(n + 64));
    HIPCHK(d.slots.ensure((size_t)std::max<uint32_t>(M, 1) * stride));
    HIPCHK(d.plen.ensure((size_t)(M + 1) * 4));
    HIPCHK(d.ids.ensure((size_t)M + 16));
    HIPCHK(d.sizes.ensure((size_t)(M + 1) * 8));
    HIPCHK(d.seg.ensure((size_t)M + 16));
    if (n) HIPCHK(hipMemcpyAsync(d.in.p, h_in, n, hipMemcpyHostToDevice, s));
    const double* ef = nullptr;
    const double* et = nullptr;
    if (p->ent_full) {
        HIPCHK(d.ent_full.ensure((size_t)(C + 1) * 8));
        HIPCHK(hipMemcpyAsync(d.ent_full.p, p->ent_full, (size_t)(C + 1) * 8, hipMemcpyHostToDevice, s));
        ef = d.ent_full.as<double>();
    }
    const uint32_t tail = (uint32_t)(n % C);
    if (p->ent_tail && tail) {
        HIPCHK(d.ent_tail.ensure((size_t)(tail + 1) * 8));
        HIPCHK(hipMemcpyAsync(d.ent_tail.p, p->ent_tail, (size_t)(tail + 1) * 8, hipMemcpyHostToDevice, s));
        et = d.ent_tail.as<double>();
    }
    EncArgs ea{};
    ea.in = d.in.as<uint8_t>();
    ea.n_total = n;
    ea.chunk_size = C;
    ea.n_chunks = M;
    ea.slots = d.slots.as<uint8_t>();
    ea.slot_stride = stride;
    ea.method_mask = p->method_mask;
    ea.plen = d.plen.as<uint32_t>();
    ea.ids = d.ids.as<uint8_t>();
    ea.sizes = d.sizes.as<uint64_t>();
    ea.ent_full = ef;
    ea.ent_tail = et;
    ea.su = su ? d.seg.as<uint8_t>() : nullptr;
    ea.flags = flags;
    for (int i = 0; i < 16; i++) { ea.pref_min[i] = p->pref_min[i]; ea.pref_max[i] = p->pref_max[i]; }
    HIPCHK(launch_encode(ea, s));
    // id 2: selection, and its should_use bit under ENC_ANALYZE
    if (((p->method_mask >> AMBC_M_DICT) & 1) || (flags & ENC_ANALYZE))
        HIPCHK(launch_dict(ea, std::min<uint32_t>(dict_cmax(p), 8192), s));
    ids.resize(M);
    plen.resize(M);
    if (M) {
        HIPCHK(hipMemcpyAsync(ids.data(), d.ids.p, M, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(plen.data(), d.plen.p, (size_t)M * 4, hipMemcpyDeviceToHost, s));
    }
    if (su) {
        su->resize(M);
        if (M) HIPCHK(hipMemcpyAsync(su->data(), d.seg.p, M, hipMemcpyDeviceToHost, s));
    }
    if (slot0) {
        slot0->resize(stride);
        HIPCHK(hipMemcpyAsync(slot0->data(), d.slots.p, stride, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return AMBC_OK;
}

extern "C" int ambc_encode_method(ambc_ctx* ctx, int method_id, const uint8_t* in, uint32_t n,
                                  uint8_t* out, uint32_t out_cap, uint32_t* out_len) {
    if (!ctx || ctx->devs.empty() || !out_len || (!in && n)) return fail(AMBC_E_INVAL, "NULL argument");
    if (method_id != AMBC_M_RLE && method_id != AMBC_M_DICT && method_id != AMBC_M_HUFFMAN &&
        method_id != AMBC_M_LZ4 && method_id != AMBC_M_DELTA)
        return fail(AMBC_E_INVAL, "ambc_encode_method supports ids 1, 2, 3, 4 and 9");
    if (n == 0) { *out_len = 0; return AMBC_OK; }          // every codec: empty -> b''
    if (n > AMBC_MAX_CHUNK) return fail(AMBC_E_INVAL, "single-chunk encode is limited to 65536 bytes");
    if (method_id == AMBC_M_DICT && n > 8192)
        return fail(AMBC_E_INVAL, "the GPU Dictionary encoder takes at most 8192 bytes");
    ambc_params p{};
    p.chunk_size = (n + 15) & ~15u;
    p.method_mask = 1u << method_id;
    for (int i = 0; i < 16; i++) { p.pref_min[i] = 0; p.pref_max[i] = 0xFFFFFFFFu; }
    std::vector<uint8_t> ids, slot;
    std::vector<uint32_t> plen;
    int rc = run_encode_only(ctx->devs[0], in, n, &p, ENC_FORCE, ids, plen, nullptr, &slot);
    if (rc) return rc;
    if (ids[0] != method_id) return fail(AMBC_E_CODEC, "codec raises on this input");
    if (plen[0] > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small");
    std::memcpy(out, slot.data(), plen[0]);
    *out_len = plen[0];
    return AMBC_OK;
}

extern "C" int ambc_dict_encode(ambc_ctx* ctx, const uint8_t* in, uint64_t n, int64_t window_size,
                                int64_t lookahead_size, uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
    if (!ctx || ctx->devs.empty() || !out_len || (!in && n) || (!out && out_cap)) return fail(AMBC_E_INVAL, "NULL argument");
    if (n == 0) { *out_len = 0; return AMBC_OK; }            // :202-203 empty -> b''
    if (n >= (1ull << 32) - (1ull << 24)) return fail(AMBC_E_INVAL, "ambc_dict_encode takes n < 2^32 - 2^24");
    Dev& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    struct Scratch {
        Buf in, tok, tab, gtab, gent, gbase, bent, bbase, res, out;
        ~Scratch() { for (Buf* b : {&in, &tok, &tab, &gtab, &gent, &gbase, &bent, &bbase, &res, &out}) b->release(); }
    } sc;
    const uint32_t nb = dict_any_blocks(n), ng = dict_any_groups(n);
    HIPCHK(sc.in.ensure(n + 64));
    HIPCHK(sc.tok.ensure(n * 4));
    HIPCHK(sc.tab.ensure(dict_any_table_bytes(n)));
    HIPCHK(sc.gtab.ensure(dict_any_gtable_bytes(n)));
    HIPCHK(sc.gent.ensure((size_t)ng * 4));
    HIPCHK(sc.gbase.ensure((size_t)ng * 8));
    HIPCHK(sc.bent.ensure((size_t)nb * 4));
    HIPCHK(sc.bbase.ensure((size_t)nb * 8));
    HIPCHK(sc.res.ensure(8));
    HIPCHK(hipMemsetAsync(sc.in.as<uint8_t>() + n, 0, 64, s));
    HIPCHK(hipMemcpyAsync(sc.in.p, in, n, hipMemcpyHostToDevice, s));
    DictAnyArgs a{};
    a.in = sc.in.as<uint8_t>();
    a.n = (uint32_t)n;
    const int64_t lim = 1ll << 62;
    a.window = std::max(-lim, std::min(lim, window_size));
    a.look = std::max(-lim, std::min(lim, lookahead_size));
    a.tok = sc.tok.as<uint32_t>();
    a.tab = sc.tab.as<uint64_t>();
    a.gtab = sc.gtab.as<uint64_t>();
    a.gent = sc.gent.as<uint32_t>();
    a.gbase = sc.gbase.as<uint64_t>();
    a.bent = sc.bent.as<uint32_t>();
    a.bbase = sc.bbase.as<uint64_t>();
    a.res = sc.res.as<uint64_t>();
    HIPCHK(launch_dict_any_parse(a, s));
    uint64_t res = 0;
    HIPCHK(hipMemcpyAsync(&res, a.res, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (res >> 63) return fail(AMBC_E_CODEC, "a match longer than 255 bytes (the reference's bytearray.append raises)");
    const uint64_t olen = res & ((1ull << 48) - 1);
    *out_len = olen;
    if (olen > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small");
    HIPCHK(sc.out.ensure(olen + 16));
    a.out = sc.out.as<uint8_t>();
    HIPCHK(launch_dict_any_emit(a, s));
    HIPCHK(hipMemcpyAsync(out, a.out, olen, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return AMBC_OK;
}

// one-block frames of k_encode (forced LZ4, 64 KiB chunks) -> one frame of
// independent 64 KiB blocks (the same bytes as ambc_encode_method up to 64 KiB)
static int lz4_any(Dev& d, const uint8_t* in, uint64_t n, Buf& dout, uint64_t* olen) {
    ambc_params p{};
    p.chunk_size = 65536;
    p.method_mask = 1u << AMBC_M_LZ4;
    for (int i = 0; i < 16; i++) { p.pref_min[i] = 0; p.pref_max[i] = 0xFFFFFFFFu; }
    std::vector<uint8_t> ids;
    std::vector<uint32_t> plen;
    int rc = run_encode_only(d, in, n, &p, ENC_FORCE, ids, plen, nullptr, nullptr);
    if (rc) return rc;
    const uint32_t M = (uint32_t)plen.size();
    std::vector<uint64_t> off(M + 1);
    uint64_t o = 15;                                    // the frame header
    for (uint32_t k = 0; k < M; k++) {
        if (ids[k] != AMBC_M_LZ4 || plen[k] < 23) return fail(AMBC_E_DEVICE, "LZ4 block encode failed");
        off[k] = o;
        o += plen[k] - 19;                              // size field + block
    }
    off[M] = o;
    *olen = o + 4;                                      // + the end mark
    Buf doff;
    struct Rel { Buf& b; ~Rel() { b.release(); } } rel{doff};
    HIPCHK(doff.ensure((M + 1) * 8));
    HIPCHK(dout.ensure(*olen + 16));
    hipStream_t s = d.stream;
    HIPCHK(hipMemcpyAsync(doff.p, off.data(), (M + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHK(launch_lz4_assemble(d.slots.as<uint8_t>(), slot_stride_for(65536, true), d.plen.as<uint32_t>(),   // (run_encode_only's, still on the device)
                               doff.as<uint64_t>(), M, n, dout.as<uint8_t>(), s));
    HIPCHK(hipStreamSynchronize(s));
    return AMBC_OK;
}

extern "C" int ambc_encode_any(ambc_ctx* ctx, int method_id, const uint8_t* in, uint64_t n, uint8_t* out,
                               uint64_t out_cap, uint64_t* out_len) {
    if (!ctx || ctx->devs.empty() || !out_len || (!in && n) || (!out && out_cap)) return fail(AMBC_E_INVAL, "NULL argument");
    if (method_id != AMBC_M_RLE && method_id != AMBC_M_HUFFMAN && method_id != AMBC_M_DELTA && method_id != AMBC_M_LZ4)
        return fail(AMBC_E_INVAL, "ambc_encode_any supports ids 1, 3, 4 and 9 (id 2: ambc_dict_encode)");
    if (n == 0) { *out_len = 0; return AMBC_OK; }
    if (n >= (1ull << 32) - (1ull << 24)) return fail(AMBC_E_INVAL, "ambc_encode_any takes n < 2^32 - 2^24");
    Dev& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    struct Scratch {
        Buf in, out, a, b, c, e;
        ~Scratch() { for (Buf* x : {&in, &out, &a, &b, &c, &e}) x->release(); }
    } sc;
    uint64_t olen = 0;
    if (method_id == AMBC_M_LZ4) {
        int rc = lz4_any(d, in, n, sc.out, &olen);
        if (rc) return rc;
    } else {
        HIPCHK(sc.in.ensure(n + 64));
        HIPCHK(hipMemcpyAsync(sc.in.p, in, n, hipMemcpyHostToDevice, s));
        const uint8_t* din = sc.in.as<uint8_t>();
        const uint32_t nb = any_blocks(n);
        if (method_id == AMBC_M_DELTA) {
            olen = n;
            HIPCHK(sc.out.ensure(n));
            HIPCHK(launch_delta_any(din, n, sc.out.as<uint8_t>(), s));
        } else if (method_id == AMBC_M_RLE) {
            HIPCHK(sc.a.ensure((size_t)(nb + 1) * 8));     // carry
            HIPCHK(sc.b.ensure((size_t)(nb + 1) * 8));     // pair counts -> bases
            HIPCHK(launch_rle_any_count(din, n, sc.a.as<int64_t>(), sc.b.as<int64_t>(), s));
            int64_t np = 0;
            HIPCHK(hipMemcpyAsync(&np, sc.b.as<int64_t>() + nb, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            olen = 2ull * (uint64_t)np;
            HIPCHK(sc.c.ensure((size_t)np * 4 + 4));
            HIPCHK(sc.out.ensure(olen + 16));
            HIPCHK(launch_rle_any_emit(din, n, sc.a.as<int64_t>(), sc.b.as<int64_t>(), sc.c.as<uint32_t>(), (uint64_t)np,
                                       sc.out.as<uint8_t>(), s));
        } else {   // Huffman
            HIPCHK(sc.a.ensure(256 * 4 * 2 + 256 * 8 + 16));   // hist, first, codes, info
            uint32_t* hist = sc.a.as<uint32_t>();
            uint32_t* first = hist + 256;
            uint64_t* codes = reinterpret_cast<uint64_t*>(first + 256);
            int32_t* info = reinterpret_cast<int32_t*>(codes + 256);
            HIPCHK(hipMemsetAsync(hist, 0, 1024, s));
            HIPCHK(hipMemsetAsync(first, 0xFF, 1024, s));
            HIPCHK(hipMemsetAsync(info, 0, 16, s));
            HIPCHK(sc.e.ensure(1 + 5 * 256 + 4 + 16));         // the table and nbits
            HIPCHK(launch_huff_any_hist(din, n, hist, first, s));
            HIPCHK(launch_huff_any_tree(hist, first, codes, sc.e.as<uint8_t>(), info, s));
            int32_t hi[4];
            HIPCHK(hipMemcpyAsync(hi, info, 16, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (hi[0] == AMBC_E_CODEC) return fail(AMBC_E_CODEC, "Huffman on 1 or 256 distinct bytes (the reference raises)");
            if (hi[0] == AMBC_E_RANGE) return fail(AMBC_E_RANGE, "Huffman bit count >= 2^32 (the reference's to_bytes(4) raises)");
            const uint64_t hdr = (uint32_t)hi[1];
            const uint64_t nbits = (uint64_t)(uint32_t)hi[2] | (uint64_t)(uint32_t)hi[3] << 32;
            const uint64_t nbytes = (nbits + 7) / 8;
            olen = hdr + nbytes;
            HIPCHK(sc.b.ensure((size_t)(nb + 1) * 8));
            HIPCHK(sc.c.ensure((size_t)(nbits / 32 + 2) * 4));
            HIPCHK(hipMemsetAsync(sc.c.p, 0, (size_t)(nbits / 32 + 2) * 4, s));
            HIPCHK(sc.out.ensure(olen + 16));
            HIPCHK(hipMemcpyAsync(sc.out.p, sc.e.p, hdr, hipMemcpyDeviceToDevice, s));
            HIPCHK(launch_huff_any_bits(din, n, codes, sc.b.as<int64_t>(), sc.c.as<uint32_t>(), nbytes,
                                        sc.out.as<uint8_t>() + hdr, s));
        }
    }
    *out_len = olen;
    if (olen > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small");
    HIPCHK(hipMemcpyAsync(out, sc.out.p, olen, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return AMBC_OK;
}

extern "C" int ambc_analyze_any(ambc_ctx* ctx, const uint8_t* in, uint64_t n, uint64_t step, uint32_t* stats) {
    if (!ctx || ctx->devs.empty() || !stats || (!in && n) || step == 0) return fail(AMBC_E_INVAL, "bad argument");
    if (n >= (1ull << 32) - (1ull << 24)) return fail(AMBC_E_INVAL, "ambc_analyze_any takes n < 2^32 - 2^24");
    Dev& d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    Buf din, st;
    struct Rel { Buf& a; Buf& b; ~Rel() { a.release(); b.release(); } } rel{din, st};
    HIPCHK(din.ensure(n + 64));
    HIPCHK(st.ensure(514 * 4));
    uint32_t* sv = st.as<uint32_t>();
    HIPCHK(hipMemsetAsync(sv, 0, 258 * 4, s));
    HIPCHK(hipMemsetAsync(sv + 258, 0xFF, 256 * 4, s));
    if (n) {
        HIPCHK(hipMemcpyAsync(din.p, in, n, hipMemcpyHostToDevice, s));
        HIPCHK(launch_su_samples(din.as<uint8_t>(), n, step, sv, s));
        HIPCHK(launch_huff_any_hist(din.as<uint8_t>(), n, sv + 2, sv + 258, s));
    }
    HIPCHK(hipMemcpyAsync(stats, sv, 514 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return AMBC_OK;
}

extern "C" int ambc_analyze(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                            uint8_t* ids_out, uint32_t* plen_out, uint8_t* su_out) {
    if (!ctx || ctx->devs.empty() || (!in && n)) return fail(AMBC_E_INVAL, "NULL argument");
    int rc = check_params(p);
    if (rc) return rc;
    std::vector<uint8_t> ids, su;
    std::vector<uint32_t> plen;
    rc = run_encode_only(ctx->devs[0], in, n, p, ENC_ANALYZE, ids, plen, &su, nullptr);
    if (rc) return rc;
    if (ids_out) std::memcpy(ids_out, ids.data(), ids.size());
    if (plen_out) std::memcpy(plen_out, plen.data(), plen.size() * 4);
    if (su_out) std::memcpy(su_out, su.data(), su.size());
    return AMBC_OK;
}

// ---------------------------------------------------------------------------
// decompress
// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t STAGE_DEC = 8192;    // must match ambc_decode.hip STAGE

bool registered_id(const uint64_t reg[4], uint32_t t) { return (reg[t >> 6] >> (t & 63)) & 1; }

uint32_t rd32le(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

// upper bound of an LZ4 frame's decoded content (for scratch sizing); 0 if unknown/small
uint64_t lz4_content_bound(const uint8_t* p, uint32_t plen) {
    // Upper bound on what the frame can decode to: the block walk (a compressed
    // block of sz bytes yields at most min(block max, 255*sz) bytes).  A declared
    // content size above it can never match the decoded length, so the frame is
    // invalid and needs no more room than the walk bound.
    if (plen < 7 || rd32le(p) != 0x184D2204u) return 0;
    const uint32_t flg = p[4], bd = p[5];
    const uint32_t bsid = (bd >> 4) & 7;
    if (bsid < 4) return 0;
    const uint64_t bmax = 1ull << (8 + 2 * bsid);
    uint64_t hp = 6, cs = 0;
    const bool has_cs = (flg >> 3) & 1;
    if (has_cs) {
        if (hp + 8 > plen) return 0;
        for (int b = 0; b < 8; b++) cs |= (uint64_t)p[hp + b] << (8 * b);
        hp += 8;
    }
    if (flg & 1) hp += 4;
    hp += 1;
    uint64_t bound = 0;
    while (hp + 4 <= plen) {
        const uint32_t bs = rd32le(p + hp);
        hp += 4;
        if (bs == 0) break;
        const uint32_t sz = bs & 0x7FFFFFFFu;
        bound += (bs & 0x80000000u) ? sz : std::min<uint64_t>(bmax, 255ull * sz + 16);
        hp += (uint64_t)sz + (((flg >> 4) & 1) ? 4 : 0);
    }
    return has_cs ? std::min(cs, bound) : bound;
}

struct Walk {
    std::vector<DecJob> jobs;
    std::vector<uint32_t> src_index;   // job -> package ordinal
    std::vector<uint8_t> kind;         // job -> DEC_KIND_* kernel
    std::vector<ambc_host_chunk> host;    // decoded by the caller (ids 6, 7, 8, ...)
    std::vector<ambc_host_chunk> zlib;    // id 5: inflated here on host threads
    uint64_t total = 0;
    uint64_t scratch = 0;
    bool marker_error = false;
};

// bytes the reference's decode of one package appends when its codec behaves
// (adaptive_compressor.py:426-442): unregistered ids copy the payload, raw
// pads/truncates to orig, Delta yields min(clen, orig), codecs yield orig
// (an empty payload decodes to nothing)
uint64_t expect_len(uint32_t t, uint32_t clen, uint32_t orig, const uint64_t reg[4]) {
    if (!registered_id(reg, t)) return clen;
    if (t == 255) return orig;
    if (t == 4) return clen ? std::min(clen, orig) : 0;
    return clen ? orig : 0;
}

// One package of the _adaptive_decompress walk (adaptive_compressor.py:399-445)
// whose 18-B header starts at hp: its decode job (offsets left to the caller),
// decode kernel, expected output length and device scratch reservation.
// Returns false where the walk stops at this header (type 0, payload overrun).
bool make_job(const uint8_t* body, uint64_t blen, uint64_t hp, uint32_t ord, const uint64_t reg[4],
              const std::map<uint32_t, uint64_t>& known, DecJob& j, int& kind, uint64_t& expect,
              uint64_t& sneed) {
    const uint32_t t = body[hp + 4];
    const uint32_t orig = rd32le(body + hp + 10);
    const uint32_t clen = rd32le(body + hp + 14);
    const uint64_t pos = hp + HDR;
    if (t == 0 || pos + clen > blen) return false;
    j = DecJob{};
    kind = DEC_KIND_HEAVY;
    sneed = 0;
    j.body_off = pos;
    j.clen = clen;
    j.orig = orig;
    j.scratch_off = ~0ull;
    j.scratch_cap = 0;
    if (!registered_id(reg, t)) {
        j.type = DEC_VERBATIM;
        kind = DEC_KIND_LIGHT;
    } else if (t == 5 && clen && orig <= AMBC_MAX_CHUNK) {
        // zlib payload: inflated on the GPU (host zlib if it decodes past the map;
        // the LDS map of u16 entries indexes at most 32768 output bytes, larger
        // packages keep a u32 map of orig entries in device scratch)
        j.type = 5;
        kind = orig <= 4096 ? DEC_KIND_INFLATE_4K : orig <= 8192 ? DEC_KIND_INFLATE_8K
             : orig <= 16384 ? DEC_KIND_INFLATE_16K : orig <= 32768 ? DEC_KIND_INFLATE_32K : DEC_KIND_INFLATE_G;
        if (kind == DEC_KIND_INFLATE_G) {
            j.scratch_cap = orig;
            sneed = (4ull * orig + 15) & ~15ull;
        }
    } else if (t == 5 || !device_decodes(t)) {
        j.type = DEC_SKIP;
        kind = DEC_KIND_LIGHT;
    } else {
        if (t == 255 || t == 1 || t == 4) kind = DEC_KIND_LIGHT;
        if (t == 3) {
            // AMBC_HUFF_ROUTE (A/B, tests): 0 = the serial k_decode, 8 = the 8 KiB kernel
            static const char* hr = getenv("AMBC_HUFF_ROUTE");
            kind = huff_kind(orig, clen);
            if (hr && atoi(hr) == 0) kind = DEC_KIND_HEAVY;
            else if (hr && atoi(hr) == 8 && kind == DEC_KIND_HUFF_4K) kind = DEC_KIND_HUFF_8K;
        }
        j.type = t;
        if (t == 9 && clen) {
            const uint64_t cb = lz4_content_bound(body + pos, clen);
            if (clen >= 7 && !((body[pos + 4] >> 2) & 1) && cb < 0x80000000ull) {
                // dec_lz4_par's domain (no content checksum): LDS source map of u16
                // entries for small frames, else a u32 map in device scratch
                if (clen <= 0x7FFF && cb <= 16384) {
                    kind = cb <= 4096 ? DEC_KIND_LZ4_4K : cb <= 8192 ? DEC_KIND_LZ4_8K : DEC_KIND_LZ4_16K;
                } else {
                    kind = DEC_KIND_LZ4_G;
                    j.scratch_cap = cb;
                    sneed = (4 * cb + 15) & ~15ull;
                }
            } else if (cb > STAGE_DEC) {
                j.scratch_cap = cb;
                sneed = (cb + 15) & ~15ull;
            }
        }
        if (t == 2 && clen && clen <= 0x7FFF && (uint64_t)orig + 256 <= 16640) {
            // dec_dict_par: an LDS source map of u16 entries (payload index < 0x8000)
            kind = orig + 256 <= 4352 ? DEC_KIND_DICT_4K : orig + 256 <= 8448 ? DEC_KIND_DICT_8K : DEC_KIND_DICT_16K;
        } else if (t == 2 && clen && (uint64_t)orig + 256 > STAGE_DEC) {
            j.scratch_cap = (uint64_t)orig + 256;
            sneed = (j.scratch_cap + 15) & ~15ull;
        }
    }
    expect = expect_len(t, clen, orig, reg);
    auto it = known.find(ord);
    if (it != known.end()) expect = it->second;
    j.expect = (uint32_t)std::min<uint64_t>(expect, 0xFFFFFFFFull);
    return true;
}

inline bool is_marker(const uint8_t* p) { return p[0] == 0xFF && p[1] == 0xFF && p[2] == 0 && p[3] == 0; }

// append package j at output offset out (scratch and host-codec lists in walk order)
void push_job(Walk& w, DecJob j, int kind, uint64_t expect, uint64_t sneed, uint32_t ord, uint64_t out,
              const uint8_t* body) {
    if (sneed) { j.scratch_off = w.scratch; w.scratch += sneed; }
    j.out_off = out;
    if (j.type == DEC_SKIP) {
        const uint32_t t = body[j.body_off - HDR + 4];
        ambc_host_chunk h{j.body_off, out, j.clen, j.orig, t, 0};
        if (t == 5) { if (j.clen) w.zlib.push_back(h); }
        else w.host.push_back(h);
    }
    w.jobs.push_back(j);
    w.kind.push_back((uint8_t)kind);
    w.src_index.push_back(ord);
    (void)expect;
}

// _adaptive_decompress header walk (adaptive_compressor.py:399-445)
void walk_body_serial(const uint8_t* body, uint64_t blen, uint64_t orig_size, const uint64_t reg[4],
                      const std::map<uint32_t, uint64_t>& known, Walk& w) {
    uint64_t pos = 0, out = 0;
    uint32_t ord = 0;
    while (pos < blen) {
        if (pos + HDR > blen) break;
        if (!is_marker(body + pos)) { w.marker_error = true; return; }
        DecJob j;
        int kind;
        uint64_t expect, sneed;
        if (!make_job(body, blen, pos, ord, reg, known, j, kind, expect, sneed)) break;
        push_job(w, j, kind, expect, sneed, ord, out, body);
        out += expect;
        pos = j.body_off + j.clen;
        ord++;
        if (out >= orig_size) break;
    }
    w.total = out;
}

// Follow the header chain from `start` while positions stay below `limit`:
// header positions go to `hp`; returns 1 at a marker mismatch (position in
// *exit), 0 otherwise with *exit = the first header position >= limit, or
// UINT64_MAX where the chain ends (truncated header, type 0, payload overrun --
// that last header is listed).
int follow_chain(const uint8_t* body, uint64_t blen, uint64_t start, uint64_t limit,
                 std::vector<uint64_t>& hp, uint64_t* exit) {
    uint64_t pos = start;
    while (pos < limit) {
        if (pos + HDR > blen) { *exit = UINT64_MAX; return 0; }
        if (!is_marker(body + pos)) { *exit = pos; return 1; }
        hp.push_back(pos);
        const uint32_t t = body[pos + 4];
        const uint64_t clen = rd32le(body + pos + 14);
        if (t == 0 || pos + HDR + clen > blen) { *exit = UINT64_MAX; return 0; }
        pos += HDR + clen;
    }
    *exit = pos;
    return 0;
}

// The same walk for large bodies on host threads.  Every thread follows the
// chain from the first marker in its segment that leads consistently to the
// segment's end; the true chain (from offset 0) is stitched segment by segment --
// where it enters a segment at a position of that thread's chain, the rest of
// the chain is the thread's (the walk is deterministic), else it is walked there.
// Jobs are built in parallel; offsets by one serial prefix pass.
void walk_body(const uint8_t* body, uint64_t blen, uint64_t orig_size, const uint64_t reg[4],
               const std::map<uint32_t, uint64_t>& known, Walk& w, unsigned tmax = 16) {
    const unsigned T = std::min(tmax, std::max(1u, std::thread::hardware_concurrency()));
    if (blen < (32ull << 20) || T < 2) { walk_body_serial(body, blen, orig_size, reg, known, w); return; }
    const bool tr = getenv("AMBC_WALK_TRACE") != nullptr;
    uint64_t tm[8], tn = 0;
    tm[tn++] = now_ns();
    std::vector<std::vector<uint64_t>> seg(T);
    std::vector<uint64_t> sexit(T, UINT64_MAX);
    std::vector<int> sstat(T, 0);
    std::vector<uint64_t> s0(T + 1);
    for (unsigned t = 0; t <= T; t++) s0[t] = blen * t / T;
    auto discover = [&](unsigned t) {
        if (t == 0) { sstat[0] = follow_chain(body, blen, 0, s0[1], seg[0], &sexit[0]); return; }
        uint64_t c = s0[t];
        for (int tries = 0; tries < 256 && c < s0[t + 1]; tries++) {
            const void* f = memchr(body + c, 0xFF, s0[t + 1] - c);
            if (!f) break;
            c = (uint64_t)((const uint8_t*)f - body);
            if (c + HDR <= blen && is_marker(body + c)) {
                seg[t].clear();
                uint64_t ex;
                if (follow_chain(body, blen, c, s0[t + 1], seg[t], &ex) == 0) { sexit[t] = ex; return; }
            }
            c++;
        }
        seg[t].clear();
        sstat[t] = -1;   // nothing consistent found: walked when the chain gets here
    };
    {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; t++) th.emplace_back(discover, t);
        discover(0);
        for (auto& x : th) x.join();
    }
    tm[tn++] = now_ns();
    // stitch the true chain
    std::vector<uint64_t> H(seg[0]);
    uint64_t q = sexit[0];
    int status = sstat[0];
    for (unsigned t = 1; t < T && status == 0 && q != UINT64_MAX; t++) {
        if (q >= s0[t + 1]) continue;               // one package spans this segment
        auto it = sstat[t] == 0 ? std::lower_bound(seg[t].begin(), seg[t].end(), q) : seg[t].end();
        if (it != seg[t].end() && *it == q) {
            H.insert(H.end(), it, seg[t].end());
            q = sexit[t];
        } else {
            status = follow_chain(body, blen, q, s0[t + 1], H, &q);
        }
    }
    tm[tn++] = now_ns();
    // jobs in parallel, then offsets and the out >= orig_size stop in order
    const size_t K = H.size();
    std::vector<DecJob> J(K);
    std::vector<int> kinds(K);
    std::vector<uint64_t> ex(K), sn(K);
    std::vector<uint8_t> ok(K);
    {
        auto build = [&](unsigned t) {
            for (size_t k = K * t / T; k < K * (t + 1) / T; k++)
                ok[k] = make_job(body, blen, H[k], (uint32_t)k, reg, known, J[k], kinds[k], ex[k], sn[k]);
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; t++) th.emplace_back(build, t);
        build(0);
        for (auto& x : th) x.join();
    }
    tm[tn++] = now_ns();
    // offsets: per-block sums, a prefix over the blocks, then each block finds its
    // own stop (a header that ends the walk, or out reaching orig_size) and fills
    // in its offsets; the walk stops at the first block's stop
    std::vector<uint64_t> bo(T + 1, 0), bs(T + 1, 0);
    std::vector<size_t> stop(T, SIZE_MAX);
    auto bsum = [&](unsigned t) {
        uint64_t a = 0, b = 0;
        for (size_t k = K * t / T; k < K * (t + 1) / T; k++) { a += ex[k]; b += sn[k]; }
        bo[t + 1] = a;
        bs[t + 1] = b;
    };
    auto fill = [&](unsigned t) {
        uint64_t out = bo[t], scr = bs[t];
        for (size_t k = K * t / T; k < K * (t + 1) / T; k++) {
            if (!ok[k]) { stop[t] = k; return; }        // walk ends before this header
            J[k].out_off = out;
            if (sn[k]) { J[k].scratch_off = scr; scr += sn[k]; }
            out += ex[k];
            if (out >= orig_size) { stop[t] = k + 1; return; }
        }
    };
    auto par = [&](auto&& f) {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; t++) th.emplace_back(f, t);
        f(0);
        for (auto& x : th) x.join();
    };
    par(bsum);
    for (unsigned t = 0; t < T; t++) { bo[t + 1] += bo[t]; bs[t + 1] += bs[t]; }
    par(fill);
    tm[tn++] = now_ns();
    size_t nj = K;
    bool stopped = false;
    for (unsigned t = 0; t < T; t++)
        if (stop[t] != SIZE_MAX) { nj = stop[t]; stopped = true; break; }
    if (!stopped && status == 1) { w.marker_error = true; return; }
    J.resize(nj);
    w.jobs = std::move(J);
    w.kind.resize(nj);
    w.src_index.resize(nj);
    uint64_t total = 0, scr = 0;
    for (size_t k = 0; k < nj; k++) {
        w.kind[k] = (uint8_t)kinds[k];
        w.src_index[k] = (uint32_t)k;
        total += ex[k];
        scr += sn[k];
        const DecJob& j = w.jobs[k];
        if (j.type == DEC_SKIP) {
            const uint32_t t = body[j.body_off - HDR + 4];
            ambc_host_chunk h{j.body_off, j.out_off, j.clen, j.orig, t, 0};
            if (t == 5) { if (j.clen) w.zlib.push_back(h); }
            else w.host.push_back(h);
        }
    }
    w.scratch = scr;
    w.total = total;
    tm[tn++] = now_ns();
    if (tr) {
        fprintf(stderr, "[ambc walk] T=%u K=%zu:", T, K);
        for (uint64_t i = 1; i < tn; i++) fprintf(stderr, " %.2f", (tm[i] - tm[i - 1]) / 1e6);
        fprintf(stderr, " ms (discover, stitch, jobs, offsets, finish)\n");
    }
}

}  // namespace

// DeflateCompression.decompress (advanced_compression.py:83-96): zlib.decompress
// of the payload (zlib wrapper, Adler-32 checked, bytes after the end of the
// stream ignored, an unfinished stream is an error), then pad / truncate to
// orig; any error -> orig zero bytes.
static void inflate_chunk(const uint8_t* in, uint32_t n, uint8_t* out, uint32_t orig) {
    z_stream zs{};
    bool ok = inflateInit(&zs) == Z_OK;
    uint64_t produced = 0;
    if (ok) {
        uint8_t discard[16384];
        zs.next_in = const_cast<Bytef*>(in);
        zs.avail_in = n;
        for (;;) {
            const bool spill = produced >= orig;
            zs.next_out = spill ? discard : out + produced;
            zs.avail_out = spill ? (uInt)sizeof discard : (uInt)(orig - produced);
            const uInt room = zs.avail_out;
            const int rc = inflate(&zs, Z_NO_FLUSH);
            produced += room - zs.avail_out;
            if (rc == Z_STREAM_END) break;
            if (rc == Z_OK && zs.avail_out == 0) continue;         // output full: keep going
            if (rc == Z_OK || rc == Z_BUF_ERROR) {
                if (zs.avail_in == 0) { ok = false; break; }        // truncated stream
                if (rc == Z_OK) continue;
            }
            ok = false;                                             // data / header / checksum error
            break;
        }
        inflateEnd(&zs);
    }
    if (!ok) std::memset(out, 0, orig);
    else if (produced < orig) std::memset(out + produced, 0, orig - produced);
}

static void inflate_all(const uint8_t* body, const std::vector<ambc_host_chunk>& jobs, uint8_t* out,
                        uint64_t orig_size) {
    if (jobs.empty()) return;
    const char* e = getenv("AMBC_HOST_THREADS");
    unsigned nt = e ? (unsigned)std::max(1, atoi(e)) : std::min(16u, std::thread::hardware_concurrency());
    nt = std::max(1u, std::min<unsigned>(nt, (unsigned)((jobs.size() + 63) / 64)));
    auto run = [&](unsigned w) {
        std::vector<uint8_t> tmp;
        for (size_t i = w; i < jobs.size(); i += nt) {
            const ambc_host_chunk& h = jobs[i];
            if (h.out_off >= orig_size) continue;
            // the last chunk may run past orig_size (the final truncate): decode aside
            if (h.out_off + h.orig <= orig_size) {
                inflate_chunk(body + h.body_off, h.clen, out + h.out_off, h.orig);
            } else {
                tmp.resize(h.orig);
                inflate_chunk(body + h.body_off, h.clen, tmp.data(), h.orig);
                std::memcpy(out + h.out_off, tmp.data(), orig_size - h.out_off);
            }
        }
    };
    if (nt == 1) { run(0); return; }
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; w++) th.emplace_back(run, w);
    for (auto& t : th) t.join();
}

// Large copies between pageable host memory and the device: T threads, each
// owning a contiguous range and two pinned buffers, overlap their own DMA with
// the CPU copy of the previous piece; the host side (memcpy, and the first-touch
// page faults of a freshly allocated output) runs on all T threads at once.

struct StageSet {
    std::vector<void*>* buf;
    std::vector<hipStream_t>* st;
    std::vector<hipEvent_t>* ev;
};
static StageSet stage_set(Dev& d, int set) {
    return set ? StageSet{&d.stage1, &d.stage1_st, &d.stage1_ev} : StageSet{&d.stage, &d.stage_st, &d.stage_ev};
}

static int ensure_stage(Dev& d, unsigned T, int set = 0) {
    StageSet S = stage_set(d, set);
    if (S.st->size() >= T) return AMBC_OK;
    HIPCHK(hipSetDevice(d.id));
    while (S.st->size() < T) {
        void* b[2] = {nullptr, nullptr};
        hipStream_t st;
        hipEvent_t ev[2];
        HIPCHK(hipHostMalloc(&b[0], kStagePiece, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&b[1], kStagePiece, hipHostMallocDefault));
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
        S.buf->push_back(b[0]); S.buf->push_back(b[1]);
        S.st->push_back(st);
        S.ev->push_back(ev[0]); S.ev->push_back(ev[1]);
    }
    return AMBC_OK;
}

unsigned ambc::stage_threads(uint64_t n, unsigned cap) {
    const char* e = getenv("AMBC_HOST_THREADS");
    unsigned t = e ? (unsigned)std::max(1, atoi(e)) : std::min(cap, std::thread::hardware_concurrency());
    return std::max(1u, std::min<unsigned>(t, (unsigned)(n / kStagePiece) + 1));
}

static void hugepage_advice(void* dst, uint64_t n) {
    // a fresh output (calloc'd bytes) is faulted in on first touch: ask for 2 MiB
    // pages so that 4 GiB is 2048 faults, not a million (advice only)
    static const bool off = getenv("AMBC_NO_HUGEPAGE") != nullptr;   // (measurements)
    if (off) return;
    const uintptr_t lo = ((uintptr_t)dst + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    const uintptr_t hi = ((uintptr_t)dst + n) & ~(uintptr_t)((2u << 20) - 1);
    if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_HUGEPAGE);
}

// to_dev: host src -> device dst; else device src -> host dst
int ambc::copy_staged(Dev& d, void* dst, const void* src, uint64_t n, bool to_dev, int set, unsigned cap) {
    const unsigned T = stage_threads(n, cap);
    int rc = ensure_stage(d, T, set);
    if (rc) return rc;
    StageSet S = stage_set(d, set);
    if (!to_dev) hugepage_advice(dst, n);
    std::vector<int> err(T, 0);
    auto run = [&](unsigned t) {
        if (hipSetDevice(d.id) != hipSuccess) { err[t] = 1; return; }
        const uint64_t a = n * t / T, b = n * (t + 1) / T;
        uint8_t* pb[2] = {static_cast<uint8_t*>((*S.buf)[2 * t]), static_cast<uint8_t*>((*S.buf)[2 * t + 1])};
        hipEvent_t* ev = &(*S.ev)[2 * t];
        hipStream_t st = (*S.st)[t];
        const uint8_t* s8 = static_cast<const uint8_t*>(src);
        uint8_t* d8 = static_cast<uint8_t*>(dst);
        if (to_dev) {
            // memcpy piece k into buffer k%2 (after its previous DMA finished), then DMA it
            int cur = 0;
            for (uint64_t off = a; off < b; off += kStagePiece, cur ^= 1) {
                const size_t len = (size_t)std::min<uint64_t>(kStagePiece, b - off);
                if (off >= a + 2 * kStagePiece && hipEventSynchronize(ev[cur]) != hipSuccess) { err[t] = 1; return; }
                std::memcpy(pb[cur], s8 + off, len);
                if (hipMemcpyAsync(d8 + off, pb[cur], len, hipMemcpyHostToDevice, st) != hipSuccess ||
                    hipEventRecord(ev[cur], st) != hipSuccess) { err[t] = 1; return; }
            }
            if (hipStreamSynchronize(st) != hipSuccess) err[t] = 1;
        } else {
            // DMA piece k+1 while piece k is copied out of its buffer
            int cur = 0;
            if (a < b) {
                const size_t len0 = (size_t)std::min<uint64_t>(kStagePiece, b - a);
                if (hipMemcpyAsync(pb[0], s8 + a, len0, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipEventRecord(ev[0], st) != hipSuccess) { err[t] = 1; return; }
            }
            for (uint64_t off = a; off < b; off += kStagePiece, cur ^= 1) {
                const size_t len = (size_t)std::min<uint64_t>(kStagePiece, b - off);
                const uint64_t nx = off + kStagePiece;
                if (nx < b) {
                    const size_t ln = (size_t)std::min<uint64_t>(kStagePiece, b - nx);
                    if (hipMemcpyAsync(pb[cur ^ 1], s8 + nx, ln, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipEventRecord(ev[cur ^ 1], st) != hipSuccess) { err[t] = 1; return; }
                }
                if (hipEventSynchronize(ev[cur]) != hipSuccess) { err[t] = 1; return; }
                std::memcpy(d8 + off, pb[cur], len);
            }
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; t++) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
    for (int e : err) if (e) return fail(AMBC_E_DEVICE, "staged copy failed");
    return AMBC_OK;
}

int ambc::start_ordered_upload(Dev& d, uint8_t* dst, const uint8_t* src, uint64_t n, unsigned T, OrderedUpload& u) {
    int rc = ensure_stage(d, T, 0);
    if (rc) return rc;
    const uint64_t np = (n + kStagePiece - 1) / kStagePiece;
    u.n = n;
    u.done.assign(np, 0);
    for (unsigned t = 0; t < T; t++) {
        u.th.emplace_back([&d, &u, dst, src, n, np, t, T] {
            if (hipSetDevice(d.id) != hipSuccess) { u.fail_all(); return; }
            uint8_t* pb[2] = {static_cast<uint8_t*>(d.stage[2 * t]), static_cast<uint8_t*>(d.stage[2 * t + 1])};
            hipEvent_t* ev = &d.stage_ev[2 * t];
            hipStream_t st = d.stage_st[t];
            uint64_t pend[2] = {UINT64_MAX, UINT64_MAX};   // piece in flight per buffer
            int cur = 0;
            for (uint64_t q = t; q < np; q += T, cur ^= 1) {
                if (pend[cur] != UINT64_MAX) {
                    if (hipEventSynchronize(ev[cur]) != hipSuccess) { u.fail_all(); return; }
                    u.mark(pend[cur]);
                }
                const uint64_t off = q * kStagePiece;
                const size_t len = (size_t)std::min<uint64_t>(kStagePiece, n - off);
                std::memcpy(pb[cur], src + off, len);
                if (hipMemcpyAsync(dst + off, pb[cur], len, hipMemcpyHostToDevice, st) != hipSuccess ||
                    hipEventRecord(ev[cur], st) != hipSuccess) { u.fail_all(); return; }
                pend[cur] = q;
            }
            for (int b = 0; b < 2; b++) {
                const int c = cur ^ b;
                if (pend[c] == UINT64_MAX) continue;
                if (hipEventSynchronize(ev[c]) != hipSuccess) { u.fail_all(); return; }
                u.mark(pend[c]);
            }
        });
    }
    return AMBC_OK;
}

// The copy back of a decode: the caller's output is cut into pieces of about
// PIECE bytes (ends on 2 MiB page boundaries); a helper thread faults each piece
// in ahead of the decode (2 MiB pages where the kernel grants them, 8 threads),
// and each decoded piece goes down through the library's pinned staging on a
// worker thread as soon as the kernels that wrote it are done, overlapping the
// decode and upload of later pieces.  The caller's pages are never mapped into
// the GPU (no hipHostRegister of caller memory).
struct OutCopy {
    static constexpr uint64_t PG = 4096, HP = 2u << 20, PIECE = 128u << 20;
    struct Piece { uint64_t lo, hi; };  // output offsets
    Dev& d;
    uint8_t* out;
    uint64_t n;
    const uint8_t* src;                 // device bytes
    std::vector<Piece> pcs;
    std::mutex m;
    std::condition_variable cv;
    size_t prepped = 0;                 // pieces [0, prepped) faulted in
    bool stop_prep = false;
    size_t pnext = 0;                   // first piece not yet queued
    std::thread prep;
    struct StageJob { uint64_t lo, hi; hipEvent_t after; };
    std::deque<StageJob> sq;            // decoded pieces for the staging worker
    bool sq_done = false, sq_abort = false;
    int sq_rc = AMBC_OK;
    std::thread stg;

    OutCopy(Dev& dv, uint8_t* o, uint64_t len, const uint8_t* s) : d(dv), out(o), n(len), src(s) {
        const uintptr_t ob = (uintptr_t)out;
        for (uint64_t x = 0; x < n;) {
            uint64_t y = ((ob + x + PIECE) & ~(uintptr_t)(HP - 1)) - ob;
            if (y <= x) y = x + PIECE;
            y = std::min(y, n);
            pcs.push_back(Piece{x, y});
            x = y;
        }
        hugepage_advice(out, n);
        prep = std::thread([this] { run_prep(); });
    }
    ~OutCopy() { abort(); }

    void run_stage() {
        if (hipSetDevice(d.id) != hipSuccess) { std::lock_guard<std::mutex> lk(m); sq_rc = AMBC_E_DEVICE; }
        for (;;) {
            StageJob j;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return sq_abort || sq_done || !sq.empty(); });
                if (sq_abort || sq_rc || sq.empty()) return;   // (sq_done with nothing left)
                j = sq.front();
                sq.pop_front();
            }
            int rc = AMBC_OK;
            if (j.after && hipEventSynchronize(j.after) != hipSuccess) rc = AMBC_E_DEVICE;
            else if (j.hi - j.lo >= kStageMin) rc = copy_staged(d, out + j.lo, src + j.lo, j.hi - j.lo, false, 1);
            else if (hipMemcpy(out + j.lo, src + j.lo, j.hi - j.lo, hipMemcpyDeviceToHost) != hipSuccess) rc = AMBC_E_DEVICE;
            if (rc) { std::lock_guard<std::mutex> lk(m); sq_rc = rc; return; }
        }
    }
    // wait for the worker (drain: finish every queued piece; else drop the rest)
    int join_stage(bool drain) {
        {
            std::lock_guard<std::mutex> lk(m);
            if (drain) sq_done = true; else sq_abort = true;
        }
        cv.notify_all();
        if (stg.joinable()) stg.join();
        std::lock_guard<std::mutex> lk(m);
        return sq_rc;
    }

    void run_prep() {
        static const unsigned tp_env = getenv("AMBC_PREP_THREADS") ? (unsigned)std::max(1, atoi(getenv("AMBC_PREP_THREADS"))) : 8u;
        const unsigned TP = std::max(1u, std::min(tp_env, stage_threads(n, tp_env)));
        const uintptr_t ob = (uintptr_t)out;
        for (size_t j = 0; j < pcs.size(); j++) {
            { std::lock_guard<std::mutex> lk(m); if (stop_prep) break; }
            const Piece pc = pcs[j];
            std::vector<std::thread> th;
            for (unsigned t = 0; t < TP; t++)
                th.emplace_back([pc, t, TP, ob] {
                    const uintptr_t a = ob + pc.lo + (pc.hi - pc.lo) * t / TP, b = ob + pc.lo + (pc.hi - pc.lo) * (t + 1) / TP;
                    // one byte of every page in [a, b) (a fresh output: zeros)
                    for (uintptr_t x = a; x < b; x = (x & ~(uintptr_t)(PG - 1)) + PG)
                        *reinterpret_cast<volatile uint8_t*>(x) = 0;
                });
            for (auto& x : th) x.join();
            { std::lock_guard<std::mutex> lk(m); prepped = j + 1; }
            cv.notify_all();
        }
        std::lock_guard<std::mutex> lk(m);
        prepped = pcs.size();
        cv.notify_all();
    }
    // drop what is queued, stop faulting in, join both helpers
    void abort() {
        (void)join_stage(false);
        { std::lock_guard<std::mutex> lk(m); stop_prep = true; }
        if (prep.joinable()) prep.join();
    }
    // queue the pieces entirely below output offset upto, to go after event `after`
    int copy_ready(uint64_t upto, hipEvent_t after) {
        std::unique_lock<std::mutex> lk(m);
        while (pnext < pcs.size() && pcs[pnext].hi <= upto) {
            cv.wait(lk, [&] { return prepped > pnext; });
            sq.push_back(StageJob{pcs[pnext].lo, pcs[pnext].hi, after});
            if (!stg.joinable()) stg = std::thread([this] { run_stage(); });
            cv.notify_all();
            pnext++;
        }
        return AMBC_OK;
    }
    // the rest after `after`; returns when every byte is in the output
    int finish(hipEvent_t after) {
        int rc = copy_ready(n, after);
        if (rc) { abort(); return rc; }
        rc = join_stage(true);
        abort();
        if (rc) return fail(rc, "staged copy failed");
        return AMBC_OK;
    }
};

// Large host-to-host decodes as a pipeline (SURVEY 8(d) T_api): the body goes
// up in ordered pieces while the host walks its headers; the jobs are cut into
// slabs of about kSlabOut output bytes, slab s is decoded as soon as the body
// pieces its packages read have arrived, and copied back (pinned staging on its
// own threads) while slab s+1 decodes and the upload goes on -- PCIe carries the
// body up and the output down at once.  PIPE_FALLBACK: some package decoded to
// another length than its header announced (the reference's lenient paths need
// the re-walk of the sequential path below, which redoes the whole call).
constexpr int PIPE_FALLBACK = 1;
constexpr uint64_t kSlabOut = 256ull << 20;

static int decompress_pipelined(Dev& d, const uint8_t* body, uint64_t blen, uint64_t orig_size,
                                const uint64_t reg[4], uint8_t* out, std::vector<ambc_host_chunk>& host,
                                ambc_stats* st) {
    const uint64_t t0 = now_ns();
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    HIPCHK(d.body.ensure(blen + 64));
    std::unique_ptr<OrderedUpload> upp(new OrderedUpload());
    // the body through the pinned staging buffers, in order
    int rc = start_ordered_upload(d, d.body.as<uint8_t>(), body, blen, stage_threads(blen, 8), *upp);
    if (rc) return rc;
    OrderedUpload& up = *upp;
    // the header walk meanwhile, on the host body
    std::map<uint32_t, uint64_t> known;
    Walk w;
    uint64_t t = now_ns();
    walk_body(body, blen, orig_size, reg, known, w, 12);
    const uint64_t walk_ns = now_ns() - t;
    if (w.marker_error) {
        up.release();
        return fail(AMBC_E_MARKER, "Marker mismatch in chunk header.");
    }
    const uint32_t nj = (uint32_t)w.jobs.size();
    const uint64_t cap = std::max(w.total, orig_size) + 64;
    HIPCHK(d.dout.ensure(cap));
    HIPCHK(d.jobs.ensure((size_t)std::max<uint32_t>(nj, 1) * sizeof(DecJob)));
    HIPCHK(d.produced.ensure((size_t)std::max<uint32_t>(nj, 1) * 4));
    HIPCHK(d.scratch.ensure(w.scratch + 64));
    HIPCHK(d.list.ensure((size_t)std::max<uint32_t>(nj, 1) * 4));
    // slabs of jobs (by output offset), per slab one list per decode kernel
    const char* es = getenv("AMBC_DECODE_SLAB");   // (tests: many slabs on small bodies)
    const uint64_t slab_out = es && strtoull(es, nullptr, 10) ? strtoull(es, nullptr, 10) : kSlabOut;
    std::vector<uint32_t> sj{0};
    for (uint32_t i = 1; i < nj; i++)
        if (w.jobs[i].out_off >= (uint64_t)sj.size() * slab_out) sj.push_back(i);
    sj.push_back(nj);
    const size_t S = sj.size() - 1;
    std::vector<uint32_t> lists(nj), lcnt(S * DEC_KINDS, 0), lbase(S * DEC_KINDS, 0);
    std::vector<uint64_t> bneed(S, 0), o0(S + 1, 0);
    {
        uint32_t at = 0;
        for (size_t q = 0; q < S; q++) {
            for (uint32_t i = sj[q]; i < sj[q + 1]; i++) {
                lcnt[q * DEC_KINDS + w.kind[i]]++;
                bneed[q] = std::max<uint64_t>(bneed[q], w.jobs[i].body_off + w.jobs[i].clen);
            }
            for (int k = 0; k < DEC_KINDS; k++) { lbase[q * DEC_KINDS + k] = at; at += lcnt[q * DEC_KINDS + k]; }
            std::vector<uint32_t> fill(lbase.begin() + q * DEC_KINDS, lbase.begin() + (q + 1) * DEC_KINDS);
            for (uint32_t i = sj[q]; i < sj[q + 1]; i++) lists[fill[w.kind[i]]++] = i;
            o0[q] = q == 0 ? 0 : std::min<uint64_t>(w.jobs[sj[q]].out_off, orig_size);
        }
        o0[S] = orig_size;
        if (S) bneed[S - 1] = blen;   // (the last slab waits for the whole body)
    }
    if (nj) HIPCHK(hipMemcpyAsync(d.jobs.p, w.jobs.data(), nj * sizeof(DecJob), hipMemcpyHostToDevice, s));
    if (nj) HIPCHK(hipMemcpyAsync(d.list.p, lists.data(), nj * 4, hipMemcpyHostToDevice, s));
    if (w.total < orig_size) HIPCHK(hipMemsetAsync(d.dout.as<uint8_t>() + w.total, 0, orig_size - w.total, s));
    if (!d.inffix_ok) {
        HIPCHK(d.inffix.ensure(INF_FIXED_U16 * 2));
        HIPCHK(launch_inflate_fixed_tables(d.inffix.as<uint16_t>(), s));
        d.inffix_ok = true;
    }
    DecArgs a{};
    a.body = d.body.as<uint8_t>();
    a.out = d.dout.as<uint8_t>();
    a.out_cap = cap;
    a.jobs = d.jobs.as<DecJob>();
    a.n_jobs = nj;
    a.scratch = d.scratch.as<uint8_t>();
    a.produced = d.produced.as<uint32_t>();
    a.inf_fixed = d.inffix.as<uint16_t>();
    std::vector<hipEvent_t> evb(S), eve(S);
    struct EvFree {
        std::vector<hipEvent_t>& a; std::vector<hipEvent_t>& b;
        ~EvFree() { for (auto e : a) if (e) (void)hipEventDestroy(e); for (auto e : b) if (e) (void)hipEventDestroy(e); }
    } evfree{evb, eve};
    for (size_t q = 0; q < S; q++) {
        HIPCHK(hipEventCreate(&evb[q]));
        HIPCHK(hipEventCreate(&eve[q]));
    }
    OutCopy od(d, out, orig_size, d.dout.as<uint8_t>());
    const uint64_t tk = now_ns();
    for (size_t q = 0; q < S; q++) {
        if (!up.wait_prefix(bneed[q])) { od.abort(); up.release(); return fail(AMBC_E_DEVICE, "staged body upload failed"); }
        HIPCHK(hipEventRecord(evb[q], s));
        for (int k = 0; k < DEC_KINDS; k++) {
            a.list = d.list.as<uint32_t>() + lbase[q * DEC_KINDS + k];
            a.n_list = lcnt[q * DEC_KINDS + k];
            const hipError_t e = launch_decode(k, a, s);
            if (e != hipSuccess) { od.abort(); up.release(); return fail(AMBC_E_DEVICE, hipGetErrorString(e)); }
        }
        HIPCHK(hipEventRecord(eve[q], s));
        const int rc2 = od.copy_ready(o0[q + 1], eve[q]);
        if (rc2) { od.abort(); up.release(); return rc2; }
    }
    up.release();
    const uint64_t h2d_ns = now_ns() - t0;
    std::vector<uint32_t> prod(nj);
    if (nj) HIPCHK(hipMemcpyAsync(prod.data(), d.produced.p, nj * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    rc = od.finish(S ? eve[S - 1] : nullptr);
    if (rc) return rc;
    const uint64_t d2h_busy = now_ns() - tk;
    uint64_t kern_ns = 0;
    for (size_t q = 0; q < S; q++) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, evb[q], eve[q]));
        kern_ns += (uint64_t)(ms * 1e6);
    }
    std::vector<ambc_host_chunk> hostinf;
    for (uint32_t i = 0; i < nj; i++) {
        if (prod[i] == DEC_PRODUCED_HOST) {
            const DecJob& jb = w.jobs[i];
            hostinf.push_back(ambc_host_chunk{jb.body_off, jb.out_off, jb.clen, jb.orig, 5, 0});
            continue;
        }
        if (prod[i] == 0xFFFFFFFFu) return fail(AMBC_E_DEVICE, "decode job failed");
        if (prod[i] != w.jobs[i].expect) return PIPE_FALLBACK;
    }
    const uint64_t t_inf = now_ns();
    inflate_all(body, w.zlib, out, orig_size);
    inflate_all(body, hostinf, out, orig_size);
    const uint64_t inflate_ns = now_ns() - t_inf;
    host = w.host;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->total_chunks = w.jobs.size();
        st->payload_bytes = w.total;
        st->h2d_ns = h2d_ns;            // the upload's span (overlapped with the walk and the decode)
        st->d2h_ns = d2h_busy;          // from the first decode launch to the last output byte
        st->walk_ns = walk_ns;
        st->kernel_ns = kern_ns;
        st->host_codec_ns = inflate_ns;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

// ---- the decode pipeline with the header walk on the device (ambc_walk.hip) ----
constexpr uint64_t kWalkPiece = 128ull << 20;    // body bytes of header positions per walked piece
constexpr uint32_t kWalkHostCap = 1u << 20;      // packages for host codecs the device lists hold
constexpr uint64_t kOutSlack = 1ull << 20;       // output room past orig_size (a last package's overshoot)
static_assert(sizeof(HostChunk) == sizeof(ambc_host_chunk), "HostChunk mirrors ambc_host_chunk");

static uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* e = getenv(name);
    return e && *e ? strtoull(e, nullptr, 10) : dflt;
}

static int walk_buffers(Dev& d, uint64_t piece) {
    DevWalk& w = d.dw;
    if (!w.ws) {
        // the walk's launches are short and gate the next piece's decode: ahead of
        // the decode kernels' workgroups in the dispatch queue
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&w.ws, hipStreamNonBlocking, hi));
    }
    for (auto& e : w.ev) if (!e) HIPCHK(hipEventCreate(&e));
    if (!w.hst) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&w.hst), sizeof(WalkState), hipHostMallocDefault));
    if (w.sized >= piece) return AMBC_OK;
    const uint64_t nc = piece / 4 + 2;     // a marker takes 4 bytes: candidates of a piece
    const uint64_t nn = piece / 18 + 2;    // headers are >= 18 bytes apart: chain nodes of a piece
    HIPCHK(w.state.ensure(sizeof(WalkState)));
    HIPCHK(w.tcnt.ensure((piece / 65536 + 4) * 4));
    HIPCHK(w.cand.ensure(nc * 8));
    HIPCHK(w.ja.ensure((nc + 1) * 4));
    HIPCHK(w.jb.ensure((nc + 1) * 4));
    HIPCHK(w.flg.ensure(nc));
    HIPCHK(w.mark.ensure(nc));
    HIPCHK(w.bc.ensure((nc / 1024 + 2) * 4));
    HIPCHK(w.chain.ensure(nn * 4));
    HIPCHK(w.olen.ensure(nn * 8));
    HIPCHK(w.slen.ensure(nn * 8));
    HIPCHK(w.bo.ensure((nn / 1024 + 2) * 8));
    HIPCHK(w.bs.ensure((nn / 1024 + 2) * 8));
    HIPCHK(w.kind.ensure(nn));
    HIPCHK(w.host.ensure((size_t)kWalkHostCap * sizeof(HostChunk)));
    HIPCHK(w.hinf.ensure((size_t)kWalkHostCap * sizeof(HostChunk)));
    for (int q = 0; q < 2; q++) {
        HIPCHK(w.jobs[q].ensure(nn * sizeof(DecJob)));
        HIPCHK(w.list[q].ensure(nn * 4));
        HIPCHK(w.produced[q].ensure(nn * 4));
    }
    w.sized = piece;
    return AMBC_OK;
}

// Large host-to-host decodes with the header walk on the device: the body goes
// up in order; each piece of kWalkPiece bytes of header positions is walked on
// the walk stream as soon as it (plus the 17 bytes after it) has arrived, its
// jobs are decoded on the decode stream once the payloads they read are up, and
// the decoded range goes back through the pinned staging (OutCopy) -- the walk of
// piece k + 1, the decode of piece k, the upload and the copy back all overlap.  The host sees a few counters per piece (kernel grids) and, at the
// end, the packages left to host codecs.  PIPE_FALLBACK as decompress_pipelined.
static int decompress_devwalk(Dev& d, const uint8_t* body, uint64_t blen, uint64_t orig_size,
                              const uint64_t reg[4], uint8_t* out, std::vector<ambc_host_chunk>& host,
                              ambc_stats* st) {
    const uint64_t t0 = now_ns();
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    DevWalk& w = d.dw;
    // pieces of kWalkPiece bytes, the first ones smaller (8 MiB, doubling) so that
    // the decode and the copy back start early; AMBC_WALK_PIECE: one fixed size
    const uint64_t fixed = env_u64("AMBC_WALK_PIECE", 0);
    const uint64_t piece = fixed ? std::max<uint64_t>(64, fixed) : kWalkPiece;
    uint64_t plen = fixed ? piece : std::min<uint64_t>(piece, 8ull << 20);
    int rc = walk_buffers(d, piece);
    if (rc) return rc;
    HIPCHK(d.body.ensure(blen + 64));
    const uint64_t cap = orig_size + kOutSlack;
    HIPCHK(d.dout.ensure(cap + 64));
    if (!d.inffix_ok) {
        HIPCHK(d.inffix.ensure(INF_FIXED_U16 * 2));
        HIPCHK(launch_inflate_fixed_tables(d.inffix.as<uint16_t>(), s));
        d.inffix_ok = true;
    }
    HIPCHK(hipMemsetAsync(w.state.p, 0, sizeof(WalkState), w.ws));
    std::unique_ptr<OrderedUpload> upp(new OrderedUpload());
    rc = start_ordered_upload(d, d.body.as<uint8_t>(), body, blen, stage_threads(blen, 8), *upp);
    if (rc) return rc;
    OrderedUpload& up = *upp;
    std::vector<hipEvent_t> evs;   // per piece: decode start, decode end, after the check
    struct EvFree {
        std::vector<hipEvent_t>& v;
        ~EvFree() { for (auto e : v) if (e) (void)hipEventDestroy(e); }
    } evfree{evs};
    OutCopy od(d, out, orig_size, d.dout.as<uint8_t>());   // (after evs: joins its copies before they go)
    auto abort_all = [&](int code) {
        od.abort();
        up.release();
        (void)hipStreamSynchronize(w.ws);
        (void)hipStreamSynchronize(s);
        return code;
    };
    WalkArgs wa{};
    wa.body = d.body.as<uint8_t>();
    wa.blen = blen;
    wa.orig_size = orig_size;
    std::memcpy(wa.reg, reg, sizeof wa.reg);
    wa.st = w.state.as<WalkState>();
    wa.tcnt = w.tcnt.as<uint32_t>();
    wa.cand = w.cand.as<uint64_t>();
    wa.ja = w.ja.as<uint32_t>();
    wa.jb = w.jb.as<uint32_t>();
    wa.flg = w.flg.as<uint8_t>();
    wa.mark = w.mark.as<uint8_t>();
    wa.bc = w.bc.as<uint32_t>();
    wa.chain = w.chain.as<uint32_t>();
    wa.olen = w.olen.as<uint64_t>();
    wa.slen = w.slen.as<uint64_t>();
    wa.bo = w.bo.as<uint64_t>();
    wa.bs = w.bs.as<uint64_t>();
    wa.kind = w.kind.as<uint8_t>();
    wa.host = w.host.as<HostChunk>();
    wa.host_cap = kWalkHostCap;
    wa.hinf = w.hinf.as<HostChunk>();
    wa.hinf_cap = kWalkHostCap;
    DecArgs a{};
    a.body = d.body.as<uint8_t>();
    a.out = d.dout.as<uint8_t>();
    a.out_cap = cap;
    a.inf_fixed = d.inffix.as<uint16_t>();
    const uint64_t emax = blen >= HDR ? blen - (HDR - 1) : 0;   // header positions [0, emax)
    uint64_t walk_ns = 0, njobs = 0, total = 0;
    const uint64_t tk = now_ns();
    for (uint64_t pa = 0, k = 0;; pa += plen, plen = std::min(piece, 2 * plen), k++) {
        const uint64_t e = std::min(emax, pa + plen);
        const bool last = e >= emax;
        if (!up.wait_prefix(last ? blen : e + HDR - 1)) return abort_all(fail(AMBC_E_DEVICE, "body upload failed"));
        const int q = (int)(k & 1);
        if (k >= 2) HIPCHK(hipStreamWaitEvent(w.ws, evs[3 * (k - 2) + 2], 0));   // piece k-2's buffers are free
        wa.a = pa;
        wa.e = std::max(pa, e);
        wa.last = last ? 1u : 0u;
        wa.jobs = w.jobs[q].as<DecJob>();
        wa.list = w.list[q].as<uint32_t>();
        wa.produced = w.produced[q].as<uint32_t>();
        HIPCHK(hipEventRecord(w.ev[0], w.ws));
        const hipError_t he = launch_walk_piece(wa, w.ws);
        if (he != hipSuccess) return abort_all(fail(AMBC_E_DEVICE, hipGetErrorString(he)));
        HIPCHK(hipEventRecord(w.ev[1], w.ws));
        HIPCHK(hipMemcpyAsync(w.hst, w.state.p, sizeof(WalkState), hipMemcpyDeviceToHost, w.ws));
        HIPCHK(hipStreamSynchronize(w.ws));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, w.ev[0], w.ev[1]));
        walk_ns += (uint64_t)(ms * 1e6);
        const WalkState hs = *w.hst;
        if (getenv("AMBC_WALK_TRACE"))
            fprintf(stderr, "[ambc devwalk] piece %llu [%llu, %llu) nc %u root %u nchain %u nj %u stop %u entry %lld "
                    "err %u out %llu\n", (unsigned long long)k, (unsigned long long)wa.a,
                    (unsigned long long)wa.e, hs.nc, hs.root, hs.nchain, hs.nj, hs.stop, (long long)hs.entry, hs.err,
                    (unsigned long long)hs.out);
        if (hs.err) return abort_all(fail(AMBC_E_MARKER, "Marker mismatch in chunk header."));
        if (hs.nhost > kWalkHostCap || hs.out > cap) return abort_all(PIPE_FALLBACK);
        const uint32_t nj = hs.nj;
        njobs += nj;
        total = hs.out;
        if (hs.scr) {
            // (a reallocation waits for the device: the pieces before are done with it)
            HIPCHK(w.scratch[q].ensure(hs.scr + 64));
        }
        if (!up.wait_prefix(hs.bneed)) return abort_all(fail(AMBC_E_DEVICE, "body upload failed"));
        for (int x = 0; x < 3; x++) {
            evs.push_back(nullptr);
            HIPCHK(hipEventCreate(&evs.back()));
        }
        a.jobs = wa.jobs;
        a.n_jobs = nj;
        a.scratch = w.scratch[q].as<uint8_t>();
        a.produced = w.produced[q].as<uint32_t>();
        HIPCHK(hipEventRecord(evs[3 * k], s));
        for (int kk = 0, kb = 0; kk < DEC_KINDS; kb += hs.kcount[kk++]) {
            a.list = wa.list + kb;
            a.n_list = hs.kcount[kk];
            const hipError_t e2 = launch_decode(kk, a, s);
            if (e2 != hipSuccess) return abort_all(fail(AMBC_E_DEVICE, hipGetErrorString(e2)));
        }
        HIPCHK(hipEventRecord(evs[3 * k + 1], s));
        wa.nj = nj;
        const hipError_t e3 = launch_walk_check(wa, s);
        if (e3 != hipSuccess) return abort_all(fail(AMBC_E_DEVICE, hipGetErrorString(e3)));
        HIPCHK(hipEventRecord(evs[3 * k + 2], s));
        rc = od.copy_ready(std::min(total, orig_size), evs[3 * k + 1]);
        if (rc) return abort_all(rc);
        if (hs.entry == WALK_ENDED) break;
    }
    if (total < orig_size) HIPCHK(hipMemsetAsync(d.dout.as<uint8_t>() + total, 0, orig_size - total, s));
    hipEvent_t evz = nullptr;
    HIPCHK(hipEventCreate(&evz));
    evs.push_back(evz);
    HIPCHK(hipEventRecord(evz, s));
    up.release();
    const uint64_t h2d_ns = now_ns() - t0;
    HIPCHK(hipMemcpyAsync(w.hst, w.state.p, sizeof(WalkState), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const WalkState hs = *w.hst;
    if (hs.failed) return abort_all(fail(AMBC_E_DEVICE, "decode job failed"));
    if (hs.mismatch || hs.nhinf > kWalkHostCap) return abort_all(PIPE_FALLBACK);
    rc = od.finish(evz);
    if (rc) return rc;
    const uint64_t d2h_busy = now_ns() - tk;
    uint64_t kern_ns = 0;
    for (size_t k = 0; k + 2 < evs.size(); k += 3) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, evs[k], evs[k + 1]));
        kern_ns += (uint64_t)(ms * 1e6);
    }
    // the packages left to host codecs, in body order
    std::vector<ambc_host_chunk> hl(hs.nhost), hinf(hs.nhinf), zl;
    if (hs.nhost) HIPCHK(hipMemcpy(hl.data(), w.host.p, hs.nhost * sizeof(HostChunk), hipMemcpyDeviceToHost));
    if (hs.nhinf) HIPCHK(hipMemcpy(hinf.data(), w.hinf.p, hs.nhinf * sizeof(HostChunk), hipMemcpyDeviceToHost));
    auto by_body = [](const ambc_host_chunk& x, const ambc_host_chunk& y) { return x.body_off < y.body_off; };
    std::sort(hl.begin(), hl.end(), by_body);
    std::sort(hinf.begin(), hinf.end(), by_body);
    host.clear();
    for (const auto& h : hl) (h.type == 5 ? zl : host).push_back(h);
    const uint64_t t_inf = now_ns();
    inflate_all(body, zl, out, orig_size);
    inflate_all(body, hinf, out, orig_size);
    const uint64_t inflate_ns = now_ns() - t_inf;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->total_chunks = njobs;
        st->payload_bytes = total;
        st->h2d_ns = h2d_ns;            // the upload's span (overlapped with the walk and the decode)
        st->d2h_ns = d2h_busy;          // from the first walk to the last output byte
        st->walk_ns = walk_ns;          // device time of the walk kernels (overlapped with the decode)
        st->kernel_ns = kern_ns;
        st->host_codec_ns = inflate_ns;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

int ambc::decompress_on(Dev& d, const uint8_t* body, uint64_t blen, uint64_t orig_size,
                        const uint64_t reg[4], uint8_t* out, std::vector<ambc_host_chunk>& host,
                        ambc_stats* st, uint8_t* d_out_ext) {
    if (!d_out_ext && out && blen >= env_u64("AMBC_DEVWALK_MIN", kStageMin) && !getenv("AMBC_DECODE_SEQUENTIAL")) {
        const int prc = getenv("AMBC_HOST_WALK") ? decompress_pipelined(d, body, blen, orig_size, reg, out, host, st)
                                                 : decompress_devwalk(d, body, blen, orig_size, reg, out, host, st);
        if (prc != PIPE_FALLBACK) return prc;   // (lenient package lengths: the sequential path below)
        if (getenv("AMBC_DECODE_STRICT")) return fail(AMBC_E_DEVICE, "decode pipeline fell back (AMBC_DECODE_STRICT)");
    }
    const uint64_t t0 = now_ns();
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    HIPCHK(d.body.ensure(blen + 64));
    uint64_t t = now_ns();
    // a large body goes up on its own thread (pinned staging, 16 copy threads)
    // while this thread walks the headers: the walk only reads the host body
    struct Upload {
        std::thread th;
        int rc = AMBC_OK;
        uint64_t ns = 0;
        void join() { if (th.joinable()) th.join(); }
        ~Upload() { join(); }
    } up;
    if (blen >= kStageMin) {
        up.th = std::thread([&d, &up, body, blen] {
            const uint64_t t1 = now_ns();
            up.rc = copy_staged(d, d.body.p, body, blen, true);
            up.ns = now_ns() - t1;
        });
    } else if (blen) {
        // through the library's own pinned staging (one thread for a small body)
        if (int rc = copy_staged(d, d.body.p, body, blen, true)) return rc;
    }
    uint64_t h2d = 0;
    std::map<uint32_t, uint64_t> known;
    Walk w;
    std::vector<ambc_host_chunk> hostinf;   // id-5 packages the GPU handed back
    uint64_t walk_ns = 0, kern_ns = 0;
    for (int iter = 0; iter < 64; iter++) {
        w = Walk();
        t = now_ns();
        walk_body(body, blen, orig_size, reg, known, w);
        walk_ns += now_ns() - t;
        if (iter == 0) {
            t = now_ns();
            up.join();
            if (up.rc) return fail(AMBC_E_DEVICE, "staged body upload failed");
            HIPCHK(hipStreamSynchronize(s));
            h2d = std::max(up.ns, now_ns() - t);   // the upload's own time (overlapped with the walk)
        }
        if (w.marker_error) return fail(AMBC_E_MARKER, "Marker mismatch in chunk header.");
        const uint32_t nj = (uint32_t)w.jobs.size();
        const uint64_t cap = std::max(w.total, orig_size) + 64;
        HIPCHK(d.dout.ensure(cap));
        HIPCHK(d.jobs.ensure((size_t)std::max<uint32_t>(nj, 1) * sizeof(DecJob)));
        HIPCHK(d.produced.ensure((size_t)std::max<uint32_t>(nj, 1) * 4));
        HIPCHK(d.scratch.ensure(w.scratch + 64));
        // job lists per decode kernel, concatenated
        std::vector<uint32_t> lists(nj);
        uint32_t cnt[DEC_KINDS] = {0}, base[DEC_KINDS + 1] = {0};
        for (uint32_t i = 0; i < nj; i++) cnt[w.kind[i]]++;
        for (int k = 0; k < DEC_KINDS; k++) base[k + 1] = base[k] + cnt[k];
        {
            uint32_t fill[DEC_KINDS];
            for (int k = 0; k < DEC_KINDS; k++) fill[k] = base[k];
            for (uint32_t i = 0; i < nj; i++) lists[fill[w.kind[i]]++] = i;
        }
        HIPCHK(d.list.ensure((size_t)std::max<uint32_t>(nj, 1) * 4));
        if (nj) HIPCHK(hipMemcpyAsync(d.jobs.p, w.jobs.data(), nj * sizeof(DecJob), hipMemcpyHostToDevice, s));
        if (nj) HIPCHK(hipMemcpyAsync(d.list.p, lists.data(), nj * 4, hipMemcpyHostToDevice, s));
        if (w.total < orig_size) HIPCHK(hipMemsetAsync(d.dout.as<uint8_t>() + w.total, 0, orig_size - w.total, s));
        DecArgs a{};
        a.body = d.body.as<uint8_t>();
        a.out = d.dout.as<uint8_t>();
        a.out_cap = cap;
        a.jobs = d.jobs.as<DecJob>();
        a.n_jobs = nj;
        a.scratch = d.scratch.as<uint8_t>();
        a.produced = d.produced.as<uint32_t>();
        if (!d.inffix_ok) {
            HIPCHK(d.inffix.ensure(INF_FIXED_U16 * 2));
            HIPCHK(launch_inflate_fixed_tables(d.inffix.as<uint16_t>(), s));
            d.inffix_ok = true;
        }
        a.inf_fixed = d.inffix.as<uint16_t>();
        if (getenv("AMBC_STAMPS") && nj) {
            HIPCHK(d.seg.ensure((size_t)nj * 64));
            HIPCHK(hipMemsetAsync(d.seg.p, 0, (size_t)nj * 64, s));
            a.stamps = d.seg.as<unsigned long long>();
        }
        const bool hdbg = getenv("AMBC_HUFF_DEBUG") && nj;   // k_decode_huff: per-lane segments of job 0
        if (hdbg) {
            HIPCHK(d.seg.ensure((size_t)nj * 4096));
            HIPCHK(hipMemsetAsync(d.seg.p, 0, (size_t)nj * 4096, s));
            a.stamps = d.seg.as<unsigned long long>();
        }
        HIPCHK(hipEventRecord(d.ev[0], s));
        for (int k = 0; k < DEC_KINDS; k++) {
            a.list = d.list.as<uint32_t>() + base[k];
            a.n_list = cnt[k];
            HIPCHK(launch_decode(k, a, s));
        }
        HIPCHK(hipEventRecord(d.ev[1], s));
        if (hdbg) {
            std::vector<unsigned long long> sv(512);
            HIPCHK(hipMemcpyAsync(sv.data(), d.seg.p, 4096, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            fprintf(stderr, "[ambc huff] nbits %llu rounds %llu\n", sv[7] >> 32, sv[7] & 0xFFFFFFFFull);
            for (int l = 0; l < 64; l++)
                fprintf(stderr, "[ambc huff] lane %2d s %6llu | pass1 f %10llu cnt %5llu ex %10llu | final f %10llu cnt %5llu ex %10llu\n",
                        l, sv[l * 8], sv[l * 8 + 1], sv[l * 8 + 2], sv[l * 8 + 3], sv[l * 8 + 4], sv[l * 8 + 5], sv[l * 8 + 6]);
            a.stamps = nullptr;
        } else if (a.stamps) {
            std::vector<unsigned long long> sv((size_t)nj * 8);
            HIPCHK(hipMemcpyAsync(sv.data(), d.seg.p, (size_t)nj * 64, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            double sum[8] = {0};
            uint64_t cnt = 0, tagged[16] = {0};
            for (uint32_t i = 0; i < nj; i++) {
                tagged[sv[i * 8 + 7] & 15]++;
                if (sv[i * 8 + 7] != 9) continue;
                cnt++;
                for (int q = 0; q < 7; q++) sum[q] += (double)sv[i * 8 + q];
            }
            fprintf(stderr, "[ambc stamps] jobs=%u tagged9=%llu untagged=%llu\n", nj,
                    (unsigned long long)tagged[9], (unsigned long long)tagged[0]);
            if (tagged[5]) {
                double g5[7] = {0};
                for (uint32_t i = 0; i < nj; i++)
                    if (sv[i * 8 + 7] == 5) for (int q = 0; q < 7; q++) g5[q] += (double)sv[i * 8 + q];
                const double c5 = (double)tagged[5];
                fprintf(stderr, "[ambc stamps] inflate jobs=%.0f cycles/job: tables %.0f symbols %.0f "
                        "(spec %.0f chain %.0f writes %.0f layout+rest %.0f) resolve %.0f adler+out %.0f\n", c5,
                        g5[0] / c5, (g5[1] + g5[4] + g5[5] + g5[6]) / c5, g5[4] / c5, g5[5] / c5, g5[6] / c5,
                        g5[1] / c5, g5[2] / c5, g5[3] / c5);
            }
            if (cnt)
                fprintf(stderr, "[ambc stamps] lz4 jobs=%llu cycles/job: pre %.0f spec %.0f chain %.0f "
                        "seqs %.0f writes %.0f resolve %.0f gather %.0f\n", (unsigned long long)cnt,
                        sum[0] / cnt, sum[1] / cnt, sum[2] / cnt, sum[3] / cnt, sum[4] / cnt, sum[5] / cnt,
                        sum[6] / cnt);
        }
        std::vector<uint32_t> prod(nj);
        if (nj) HIPCHK(hipMemcpyAsync(prod.data(), d.produced.p, nj * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, d.ev[0], d.ev[1]));
        kern_ns += (uint64_t)(ms * 1e6);
        bool redo = false;
        hostinf.clear();
        for (uint32_t i = 0; i < nj; i++) {
            if (prod[i] == DEC_PRODUCED_HOST) {   // inflate on host after the copy back
                const DecJob& jb = w.jobs[i];
                hostinf.push_back(ambc_host_chunk{jb.body_off, jb.out_off, jb.clen, jb.orig, 5, 0});
                continue;
            }
            if (prod[i] == 0xFFFFFFFFu) return fail(AMBC_E_DEVICE, "decode job failed");
            if (prod[i] != w.jobs[i].expect) { known[w.src_index[i]] = prod[i]; redo = true; }
        }
        if (!redo) break;
    }
    if (d_out_ext && (!w.zlib.empty() || !hostinf.empty() || !w.host.empty()))
        return fail(AMBC_E_HOSTCODEC, "body has packages decoded by host codecs: use ambc_decompress_ex");
    t = now_ns();
    if (d_out_ext) {   // device-resident output (multi-GPU decode): no copy back
        if (orig_size) HIPCHK(hipMemcpyAsync(d_out_ext, d.dout.p, orig_size, hipMemcpyDeviceToDevice, s));
    } else if (orig_size) {   // (any size through the staging, as the body upload above)
        HIPCHK(hipStreamSynchronize(s));
        int rc = copy_staged(d, out, d.dout.p, orig_size, false);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(s));
    const uint64_t d2h_ns = now_ns() - t;
    const uint64_t t_inf = now_ns();
    inflate_all(body, w.zlib, out, orig_size);
    inflate_all(body, hostinf, out, orig_size);
    const uint64_t inflate_ns = now_ns() - t_inf;
    host = w.host;
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->total_chunks = w.jobs.size();
        st->payload_bytes = w.total;   // bytes the chunks produced before the final pad/truncate
        st->h2d_ns = h2d;
        st->d2h_ns = d2h_ns;
        st->walk_ns = walk_ns;
        st->kernel_ns = kern_ns;
        st->host_codec_ns = inflate_ns;
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

void ambc::default_registered(const uint64_t* registered, uint64_t reg[4]) {
    reg[0] = reg[1] = reg[2] = reg[3] = 0;
    if (registered) std::memcpy(reg, registered, 4 * sizeof(uint64_t));
    else for (uint32_t t : {1u, 2u, 3u, 4u, 5u, 6u, 7u, 9u, 255u}) reg[t >> 6] |= 1ull << (t & 63);
}

extern "C" int ambc_decompress_ex(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len,
                                  uint64_t orig_size, const uint64_t registered[4], uint8_t* out,
                                  ambc_host_chunk* host_chunks, uint32_t host_cap, uint32_t* n_host,
                                  ambc_stats* st) {
    if (!ctx || ctx->devs.empty() || (!body && body_len) || (!out && orig_size))
        return fail(AMBC_E_INVAL, "NULL argument");
    uint64_t reg[4] = {0, 0, 0, 0};
    if (registered) std::memcpy(reg, registered, sizeof reg);
    else for (uint32_t t : {1u, 2u, 3u, 4u, 5u, 6u, 7u, 9u, 255u}) reg[t >> 6] |= 1ull << (t & 63);
    std::vector<ambc_host_chunk> host;
    int rc = decompress_on(ctx->devs[0], body, body_len, orig_size, reg, out, host, st);
    if (rc) return rc;
    if (n_host) *n_host = (uint32_t)host.size();
    if (host.size() > host_cap) {
        if (!host_chunks && !n_host) return fail(AMBC_E_HOSTCODEC, "body has packages for host codecs (bz2 / lzma / zstd)");
        if (host.size() > host_cap) return fail(AMBC_E_CAPACITY, "host_chunks capacity too small");
    }
    for (size_t i = 0; i < host.size(); i++) host_chunks[i] = host[i];
    return AMBC_OK;
}

extern "C" int ambc_decompress_batch(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len,
                                     uint64_t orig_size, uint8_t* out, ambc_stats* st) {
    uint32_t nh = 0;
    int rc = ambc_decompress_ex(ctx, body, body_len, orig_size, nullptr, out, nullptr, 0, &nh, st);
    if (rc == AMBC_E_CAPACITY && nh) return fail(AMBC_E_HOSTCODEC, "body has packages for host codecs (bz2 / lzma / zstd): use ambc_decompress_ex");
    return rc;
}

extern "C" int ambc_decompress_device(ambc_ctx* ctx, int dev, const uint8_t* body, uint64_t body_len,
                                      uint64_t orig_size, const uint64_t registered[4], void* d_out,
                                      ambc_stats* st) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || (!body && body_len) || (!d_out && orig_size))
        return fail(AMBC_E_INVAL, "bad argument");
    uint64_t reg[4] = {0, 0, 0, 0};
    if (registered) std::memcpy(reg, registered, sizeof reg);
    else for (uint32_t t : {1u, 2u, 3u, 4u, 5u, 6u, 7u, 9u, 255u}) reg[t >> 6] |= 1ull << (t & 63);
    std::vector<ambc_host_chunk> host;
    return decompress_on(ctx->devs[dev], body, body_len, orig_size, reg, nullptr, host, st,
                         static_cast<uint8_t*>(d_out));
}

// host code only (diagnostics): the threaded header walk of the decode path on
// a host body -> packages, output bytes, wall ns (threads: 0 = default)
extern "C" int ambc_test_inject_failure(int rank) { return g_fail_rank.exchange(rank); }

extern "C" int ambc_debug_walk(const uint8_t* body, uint64_t blen, uint64_t orig_size, uint32_t threads,
                               uint64_t* n_pkgs, uint64_t* total, uint64_t* ns) {
    uint64_t reg[4];
    default_registered(nullptr, reg);
    std::map<uint32_t, uint64_t> known;
    Walk w;
    const uint64_t t = now_ns();
    walk_body(body, blen, orig_size, reg, known, w, threads ? threads : 16);
    if (ns) *ns = now_ns() - t;
    if (n_pkgs) *n_pkgs = w.jobs.size();
    if (total) *total = w.total;
    return w.marker_error ? AMBC_E_MARKER : AMBC_OK;
}

// Multi-GPU decode split: the reference's header walk with the
// expected package sizes, cut at package boundaries into nparts ranges of
// about orig_size / nparts output bytes each.  Part r = body bytes
// [body_off[r], body_off[r+1]) decoding to [out_off[r], out_off[r+1]); the last
// non-empty part runs to the end of the body (end chunk included) so that its
// own walk stops where the whole-body walk stops.  Host code only.
extern "C" int ambc_split_body(const uint8_t* body, uint64_t blen, uint64_t orig_size,
                               const uint64_t registered[4], uint32_t nparts, uint64_t* body_off,
                               uint64_t* out_off) {
    if ((!body && blen) || nparts == 0 || !body_off || !out_off) return fail(AMBC_E_INVAL, "bad argument");
    uint64_t reg[4] = {0, 0, 0, 0};
    if (registered) std::memcpy(reg, registered, sizeof reg);
    else for (uint32_t t : {1u, 2u, 3u, 4u, 5u, 6u, 7u, 9u, 255u}) reg[t >> 6] |= 1ull << (t & 63);
    auto target = [&](uint32_t r) {
        return (uint64_t)(((unsigned __int128)orig_size * r) / nparts);
    };
    body_off[0] = 0;
    out_off[0] = 0;
    uint32_t next = 1;
    uint64_t pos = 0, out = 0;
    while (pos < blen) {
        if (pos + HDR > blen) break;
        if (!(body[pos] == 0xFF && body[pos + 1] == 0xFF && body[pos + 2] == 0 && body[pos + 3] == 0))
            return fail(AMBC_E_MARKER, "Marker mismatch in chunk header.");
        const uint32_t t = body[pos + 4];
        const uint32_t orig = rd32le(body + pos + 10);
        const uint32_t clen = rd32le(body + pos + 14);
        if (t == 0 || pos + HDR + clen > blen) break;
        while (next < nparts && out >= target(next)) {
            body_off[next] = pos;
            out_off[next] = out;
            next++;
        }
        out += expect_len(t, clen, orig, reg);
        pos += HDR + (uint64_t)clen;
        if (out >= orig_size) break;
    }
    for (; next < nparts; next++) { body_off[next] = blen; out_off[next] = orig_size; }
    body_off[nparts] = blen;
    out_off[nparts] = orig_size;
    return AMBC_OK;
}

// ---------------------------------------------------------------------------
// memory helpers, synth, timings
// ---------------------------------------------------------------------------
extern "C" void* ambc_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<uint64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        g_err = "hipHostMalloc failed";
        return nullptr;
    }
    return p;
}
extern "C" void ambc_host_free(void* p) { if (p) (void)hipHostFree(p); }

extern "C" void* ambc_device_alloc(ambc_ctx* ctx, int dev, uint64_t bytes) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) { g_err = "bad ctx/dev"; return nullptr; }
    if (hipSetDevice(ctx->devs[dev].id) != hipSuccess) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, std::max<uint64_t>(bytes, 1)) != hipSuccess) { g_err = "hipMalloc failed"; return nullptr; }
    return p;
}
extern "C" void ambc_device_free(ambc_ctx* ctx, int dev, void* p) {
    if (!ctx || !p || dev < 0 || dev >= (int)ctx->devs.size()) return;
    (void)hipSetDevice(ctx->devs[dev].id);
    (void)hipFree(p);
}
extern "C" int ambc_memcpy_h2d(ambc_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    HIPCHK(hipSetDevice(ctx->devs[dev].id));
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return AMBC_OK;
}
extern "C" int ambc_memcpy_d2h(ambc_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    HIPCHK(hipSetDevice(ctx->devs[dev].id));
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return AMBC_OK;
}
extern "C" int ambc_memcpy_d2d(ambc_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    HIPCHK(hipSetDevice(ctx->devs[dev].id));
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
    return AMBC_OK;
}
extern "C" int ambc_memset_device(ambc_ctx* ctx, int dev, void* dst, int value, uint64_t bytes) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    HIPCHK(hipSetDevice(ctx->devs[dev].id));
    HIPCHK(hipMemset(dst, value, bytes));
    HIPCHK(hipDeviceSynchronize());
    return AMBC_OK;
}
extern "C" int ambc_synchronize(ambc_ctx* ctx, int dev) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    HIPCHK(hipSetDevice(ctx->devs[dev].id));
    HIPCHK(hipDeviceSynchronize());
    return AMBC_OK;
}

static uint64_t mix64h(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void synth_segments(uint64_t n, uint64_t seed, std::vector<uint64_t>& seg) {
    uint64_t s = seed, pos = 0, idx = 0;
    while (pos < n) {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t L = 1024 + mix64h(s) % 130049ULL;
        if (L > n - pos) L = n - pos;
        seg.push_back(pos); seg.push_back(L); seg.push_back(idx);
        pos += L; idx++;
    }
}

extern "C" void ambc_synth_fill(uint8_t* out, uint64_t n, uint64_t seed) {
    static const char* V[16] = {"alpha", "beta", "gamma", "delta", "the",  "quick", "brown", "fox",
                                "jumps", "over", "lazy",  "dog",   "data", "chunk", "marker", "stream"};
    std::vector<uint64_t> seg;
    synth_segments(n, seed, seg);
    const size_t ns = seg.size() / 3;
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; w++) {
        th.emplace_back([&, w]() {
            for (size_t g = w; g < ns; g += nt) {
                const uint64_t p = seg[3 * g], L = seg[3 * g + 1], id = seg[3 * g + 2];
                uint8_t* o = out + p;
                const uint64_t base = mix64h(seed ^ (id * 0xD1B54A32D192ED03ULL));
                if (id % 3 == 0) std::memset(o, 0, L);
                else if (id % 3 == 1) {
                    for (uint64_t j = 0; j * 8 < L; j++) {
                        const uint64_t v = mix64h(base + (j + 1) * 0x9E3779B97F4A7C15ULL);
                        for (int b = 0; b < 8 && j * 8 + b < L; b++) o[j * 8 + b] = (uint8_t)(v >> (8 * b));
                    }
                } else {
                    uint64_t q = 0;
                    for (uint64_t j = 0; q < L; j++) {
                        const char* wd = V[mix64h(base + (j + 1) * 0x9E3779B97F4A7C15ULL) >> 60];
                        for (; *wd && q < L; wd++) o[q++] = (uint8_t)*wd;
                        if (q < L) o[q++] = ' ';
                    }
                }
            }
        });
    }
    for (auto& t : th) t.join();
}

extern "C" int ambc_synth_device_range(ambc_ctx* ctx, int dev, void* d_out, uint64_t n_total, uint64_t begin,
                                       uint64_t end, uint64_t seed) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    if (begin > end || end > n_total) return fail(AMBC_E_INVAL, "need begin <= end <= n_total");
    Dev& d = ctx->devs[dev];
    HIPCHK(hipSetDevice(d.id));
    std::vector<uint64_t> seg, mine;
    synth_segments(n_total, seed, seg);
    for (size_t g = 0; g < seg.size(); g += 3)       // the segments that meet [begin, end)
        if (seg[g] < end && seg[g] + seg[g + 1] > begin) mine.insert(mine.end(), &seg[g], &seg[g] + 3);
    const uint32_t ns = (uint32_t)(mine.size() / 3);
    HIPCHK(d.seg.ensure(mine.size() * 8 + 8));
    if (ns) HIPCHK(hipMemcpyAsync(d.seg.p, mine.data(), mine.size() * 8, hipMemcpyHostToDevice, d.stream));
    HIPCHK(launch_synth((uint8_t*)d_out, begin, end, d.seg.as<uint64_t>(), ns, seed, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    return AMBC_OK;
}

extern "C" int ambc_synth_device(ambc_ctx* ctx, int dev, void* d_out, uint64_t n, uint64_t seed) {
    return ambc_synth_device_range(ctx, dev, d_out, n, 0, n, seed);
}

extern "C" int ambc_device_equal(ambc_ctx* ctx, int dev, const void* a, const void* b, uint64_t n, int* equal) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !equal) return fail(AMBC_E_INVAL, "bad argument");
    Dev& d = ctx->devs[dev];
    HIPCHK(hipSetDevice(d.id));
    HIPCHK(d.coll.ensure(64));
    HIPCHK(hipMemsetAsync(d.coll.p, 0, 4, d.stream));
    HIPCHK(launch_equal((const uint8_t*)a, (const uint8_t*)b, n, d.coll.as<uint32_t>(), d.stream));
    uint32_t neq = 1;
    HIPCHK(hipMemcpyAsync(&neq, d.coll.p, 4, hipMemcpyDeviceToHost, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    *equal = neq == 0;
    return AMBC_OK;
}

extern "C" int ambc_last_encode_launches(ambc_ctx* ctx, int dev, uint32_t* n_launch) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !n_launch) return fail(AMBC_E_INVAL, "bad ctx/dev");
    *n_launch = ctx->devs[dev].n_launch;
    return AMBC_OK;
}

extern "C" int ambc_last_kernel_times(ambc_ctx* ctx, int dev, uint64_t* encode_ns, uint64_t* scan_ns,
                                      uint64_t* compact_ns) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(AMBC_E_INVAL, "bad ctx/dev");
    Dev& d = ctx->devs[dev];
    if (encode_ns) *encode_ns = d.t_encode;
    if (scan_ns) *scan_ns = d.t_scan;
    if (compact_ns) *compact_ns = d.t_compact;
    return AMBC_OK;
}
