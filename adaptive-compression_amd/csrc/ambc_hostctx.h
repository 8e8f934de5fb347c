// ambc_hostctx.h -- host-side state shared by ambc_host.cpp (single-device
// compress / decompress) and ambc_shard.cpp (sharded calls over RCCL).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <thread>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ambc.h"
#include "ambc_internal.h"
#include "ambc_hostutil.h"
#include "ambc_sync.h"
#include "ambc_walkcore.h"

namespace ambc {

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return ::ambc::fail(AMBC_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define NCCLCHK(expr)                                                                  \
    do {                                                                               \
        ncclResult_t _r = (expr);                                                      \
        if (_r != ncclSuccess)                                                         \
            return ::ambc::fail(AMBC_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

// device buffers of one multi-size walk batch (ambc_multisize.cpp)
struct Batch {
    Buf coff, clen, slots, plen, ids, sizes, bestpre, gdseq, pending, ent, off, z9rec, z9scr, lz4sub;
    uint32_t* hplen = nullptr;  // pinned copies of plen / ids / LZ4 prefix lengths for the host walk
    uint8_t* hids = nullptr;
    uint32_t* hlz = nullptr;
    uint64_t* hpos = nullptr;   // pinned chunk positions (the upload's source)
    uint64_t* hoff = nullptr;   // pinned body offsets (a final encode's compaction)
    size_t hcap = 0;
    void host_free() {
        if (hplen) (void)hipHostFree(hplen);
        if (hids) (void)hipHostFree(hids);
        if (hlz) (void)hipHostFree(hlz);
        if (hpos) (void)hipHostFree(hpos);
        if (hoff) (void)hipHostFree(hoff);
        hplen = nullptr; hids = nullptr; hlz = nullptr; hpos = nullptr; hoff = nullptr; hcap = 0;
    }
    hipError_t host_ensure(size_t n) {
        if (n <= hcap) return hipSuccess;
        host_free();
        n = std::max<size_t>(n, 1024);
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&hplen), n * 4);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&hids), n);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&hlz), n * 4 * LZ4_SUB_MAX);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&hpos), n * 8);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&hoff), n * 8);
        if (e == hipSuccess) hcap = n;
        return e;
    }
    void release() {
        for (Buf* b : {&coff, &clen, &slots, &plen, &ids, &sizes, &bestpre, &gdseq, &pending, &ent, &off, &z9rec, &z9scr,
                       &lz4sub})
            b->release();
        host_free();
    }
};

// buffers of the device header walk (ambc_walk.hip) in the decode pipeline:
// the walk's per-piece arrays, and the jobs / lists / produced / scratch of two
// pieces in flight (piece k decodes while piece k + 1 is walked)
struct DevWalk {
    Buf state, tcnt, cand, ja, jb, flg, mark, bc, chain, olen, slen, bo, bs, kind, host, hinf;
    Buf jobs[2], list[2], produced[2], scratch[2];
    hipStream_t ws = nullptr;      // the walk's stream
    WalkState* hst = nullptr;      // pinned copy of the state
    hipEvent_t ev[2] = {};         // around a piece's walk (timing)
    uint64_t sized = 0;            // piece bytes the buffers are sized for
    void release() {
        for (Buf* b : {&state, &tcnt, &cand, &ja, &jb, &flg, &mark, &bc, &chain, &olen, &slen, &bo, &bs, &kind,
                       &host, &hinf, &jobs[0], &jobs[1], &list[0], &list[1], &produced[0], &produced[1],
                       &scratch[0], &scratch[1]})
            b->release();
        if (ws) { (void)hipStreamSynchronize(ws); (void)hipStreamDestroy(ws); ws = nullptr; }
        if (hst) (void)hipHostFree(hst);
        hst = nullptr;
        for (auto& e : ev) if (e) { (void)hipEventDestroy(e); e = nullptr; }
        sized = 0;
    }
};

struct Dev {
    int id = 0;
    DevWalk dw;
    hipStream_t stream = nullptr;
    hipEvent_t ev[6] = {};
    hipStream_t xs[2] = {};     // copy streams of the slab pipeline: H2D, D2H
    hipEvent_t xev[6] = {};     // h2d_done[2], comp_done[2], d2h_done[2]
    Buf in, out, slots, plen, ids, sizes, off, scan_tmp, acc, ent_full, ent_tail;
    Buf body, jobs, produced, dout, scratch, seg, list, bestpre, gdseq, pending;
    Buf z9rec;                  // zlib-9 id 5: the parse's segments per chunk
    Buf z9scr;                  // zlib-9 id 5 above 8 KiB: the parse's scratch per resident workgroup
    Buf coll;                   // small device buffers of the collectives (sizes, stats, flags)
    Buf inffix;                 // fixed-Huffman inflate tables (built on the first decode)
    bool inffix_ok = false;
    Batch msb[16];              // multi-size walk batches: 8 concurrent size classes per walk group
    hipStream_t mss[16] = {};   //   and their streams (created on the first walk)
    uint32_t ms_steps = 0;      // last multi-size walk: batched evaluation rounds,
    uint64_t ms_evaluated = 0;  //   chunk encodes they ran,
    uint64_t ms_walk_ns = 0, ms_emit_ns = 0;  // and the time of the walk / of the final encode
    Buf ms_out;                 // the multi-size walk's body (its own buffer: no other call writes it)
    Buf ms_ent;                 // the multi-size walk's entropy tables (one upload per call)
    uint64_t* hacc = nullptr;   // pinned: a pipelined call's statistics and body length, copied back once
    uint64_t ms_body = 0;       // a multi-size body kept in `ms_out` for ambc_fetch_body (0: none)
    WalkMemory ms_mem;          // the multi-size walk's position records, kept across calls (ambc_walkcore.h)
    uint64_t t_encode = 0, t_scan = 0, t_compact = 0;
    uint32_t n_launch = 1;      // k_encode launches of the last compress call (pipelined segments)
    hipStream_t cs = nullptr;   // scan + compaction of pipelined segments
    hipEvent_t pev[8] = {};     // segment i encoded
    hipStream_t zs = nullptr;   // zlib-9 trees + emission of segment i beside the parse of i + 1
    hipEvent_t zev = nullptr;   // segment i parsed
    Buf segbase;                // body offset of every segment (device)
    // pinned staging for large pageable copies: 2 buffers + 2 events per copy
    // thread; set 0 uploads, set 1 downloads (the decode pipeline runs both at once)
    std::vector<void*> stage, stage1;
    std::vector<hipStream_t> stage_st, stage1_st;
    std::vector<hipEvent_t> stage_ev, stage1_ev;
};

// One shard of a sharded compress (ambc_shard.cpp): in reference mode the
// remainder-raw rule is global, so compress_on asks the transport for the first
// chunk without a winner on ANY rank (AllReduce MIN) before it compacts.
struct Transport;
struct ShardInfo {
    Transport* t;
    uint64_t k0;        // global index of this shard's first chunk
    uint64_t n_total;   // bytes of the whole logical input
    int rank;           // this shard's rank in t
};

}  // namespace ambc

struct ambc_ctx {
    std::vector<ambc::Dev> devs;
    // process-per-GPU communicator (ambc_comm_init_rank): this process is rank
    // `rank` of `nranks`, on devs[0]
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // in-process multi-device communicators (ncclCommInitAll over distinct devices),
    // created on the first sharded call
    std::vector<ncclComm_t> dev_comms;
    ambc::AbortGate comm_gate;         // a failed rank's abort against enqueues in progress (ambc_shard.cpp)
};

namespace ambc {

uint32_t slot_stride_for(uint32_t C, bool forced = false);
int check_params(const ambc_params* p);
int compress_on(Dev& d, const uint8_t* d_in, uint64_t n, const ambc_params* p, uint8_t* d_out,
                uint64_t out_cap, uint64_t* out_len, ambc_stats* st, const ShardInfo* si = nullptr);
int decompress_on(Dev& d, const uint8_t* body, uint64_t blen, uint64_t orig_size, const uint64_t reg[4],
                  uint8_t* out, std::vector<ambc_host_chunk>& host, ambc_stats* st,
                  uint8_t* d_out_ext = nullptr);
void default_registered(const uint64_t* registered, uint64_t reg[4]);
void add_stats(ambc_stats* a, const ambc_stats& b);   // sums (kernel_ns: max)
uint64_t slab_bytes();                                 // host-fed pipelines' slab size
// large pageable <-> device copies through pinned staging buffers on T threads
constexpr uint64_t kStageMin = 64ull << 20;            // below this the runtime's own path
int copy_staged(Dev& d, void* dst, const void* src, uint64_t n, bool to_dev, int set = 0, unsigned cap = 16);

constexpr size_t kStagePiece = 8u << 20;               // staged copies' piece
unsigned stage_threads(uint64_t n, unsigned cap = 16);

// An upload in pieces taken in file order (piece q by thread q % T), each
// marked done once its DMA has completed, so that a consumer can start on the
// prefix [0, x) as soon as it has arrived (wait_prefix).
struct OrderedUpload {
    std::mutex m;
    std::condition_variable cv;
    std::vector<uint8_t> done;
    uint64_t n = 0, ready = 0;     // ready: the leading pieces all done
    bool failed = false;
    std::vector<std::thread> th;
    void mark(uint64_t q) {
        std::lock_guard<std::mutex> lk(m);
        done[q] = 1;
        while (ready < done.size() && done[ready]) ready++;
        cv.notify_all();
    }
    void fail_all() {
        std::lock_guard<std::mutex> lk(m);
        failed = true;
        cv.notify_all();
    }
    // bytes [0, avail()) are on the device
    uint64_t avail() {
        std::lock_guard<std::mutex> lk(m);
        return ready >= done.size() ? n : ready * kStagePiece;
    }
    // false when the upload failed
    bool wait_prefix(uint64_t bytes) {
        const uint64_t need = std::min<uint64_t>(done.size(), (bytes + kStagePiece - 1) / kStagePiece);
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return failed || ready >= need; });
        return !failed;
    }
    void join() { for (auto& x : th) if (x.joinable()) x.join(); th.clear(); }
    void release() { join(); }
    ~OrderedUpload() { release(); }
};

// an ordered upload of n bytes from host src to device dst through the pinned
// staging buffers on T threads (the caller's pages are never registered)
int start_ordered_upload(Dev& d, uint8_t* dst, const uint8_t* src, uint64_t n, unsigned T, OrderedUpload& u);

// collective of the sharded calls (ambc_shard.cpp)
int shard_allreduce_min(Transport* t, uint64_t* v, int rc_local);
int compress_batch_multi(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p, uint8_t* out,
                         uint64_t out_cap, uint64_t* out_len, ambc_stats* st);

}  // namespace ambc
