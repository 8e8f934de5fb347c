// ambc_shard.cpp -- the multi-GPU path of libambc_hip.
//
// The reference has no parallelism at all (adaptive_compressor.py:363-394 is a
// serial loop); native-mode chunks are independent, so a node shards the input
// into contiguous chunk ranges, one per GPU, and the only exchanges are small:
//
//   1. AllGather of the per-rank body sizes          -> file-order offsets
//   2. AllReduce(SUM) of the chunk statistics          -> the stats dict
//   3. reference mode only: AllReduce(MIN) of the first chunk without a
//      winner (the remainder-raw rule, adaptive_compressor.py:586-588, is
//      global: that chunk and everything after it become ONE raw chunk)
//   4. optionally a variable-size gather of the bodies into file order on
//      rank 0 (grouped ncclSend/ncclRecv over xGMI: every peer streams over its
//      own link), when one GPU must hold the whole body.
//
// Ranks are either one process per GPU (ambc_comm_init_rank: RCCL
// ncclCommInitRank, the unique id exchanged by the caller) or the devices of
// one ctx driven by one host thread each (ncclCommInitAll over distinct
// devices).  A ctx that lists the same device twice (several shards on one
// GPU) exchanges through shared host memory and device copies instead: RCCL
// admits one rank per device.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../../include/ambc.h"
#include "ambc_hostctx.h"
#include "ambc_internal.h"
#include "ambc_sync.h"

namespace ambc {

// the collectives one sharded call needs, on W ranks
struct Transport {
    int W = 1, r = 0;
    virtual ~Transport() = default;
    // all[q*k + i] = rank q's mine[i]
    virtual int allgather_u64(const uint64_t* mine, uint32_t k, uint64_t* all) = 0;
    // element-wise over the ranks, in place
    virtual int allreduce_u64(uint64_t* v, uint32_t k, int op) = 0;
    // rank `root` receives rank q's lens[q] bytes at dst + offs[q]; the others send src
    virtual int gather(const uint8_t* src, uint8_t* dst, const uint64_t* offs, const uint64_t* lens,
                       int root) = 0;
    // a failed rank tells the others, so that none waits for it forever
    virtual void abort() {}
};

// connect_group's Send / Recv warm-up: every rank sends rank 0 one piece of
// this size, as the gather does (RCCL spreads a p2p operation of a size over the
// peer's channels and connects each on first use: an 8-byte warm-up connects one)
constexpr uint64_t kP2pPiece = 64ull << 20;

// ---------------------------------------------------------------------------
// RCCL (one rank per device)
// ---------------------------------------------------------------------------
struct RcclTransport : Transport {
    ncclComm_t comm;
    Dev& d;
    // in-process ranks: every rank's communicator lives in the ctx, and a failed
    // rank aborts all of them (ncclCommAbort releases peers blocked in a
    // collective); the ctx builds fresh ones on its next sharded call
    std::vector<ncclComm_t>* group = nullptr;
    AbortGate* gate = nullptr;
    RcclTransport(ncclComm_t c, Dev& dev, int nranks, int rank) : comm(c), d(dev) { W = nranks; r = rank; }
    // Enqueue this rank's operations on its communicator.  No lock spans the
    // enqueue (a peer's first collective may wait inside its call for this rank):
    // in-process ranks pass the group's AbortGate, so a failed peer's abort()
    // waits for the enqueue to return before it frees the communicators, and an
    // enqueue after the abort fails.  Once enqueued, an abort cancels the
    // operation in flight (ncclCommAbort's purpose) and the stream wait that
    // follows returns.
    template <typename F>
    int enqueue(F&& ops) {
        if (!group) return ops(comm);
        if (!gate->enter()) return fail(AMBC_E_COMM, "communicator aborted by a failed rank");
        const int rc = ops((*group)[r]);
        gate->leave();
        return rc;
    }

    int allgather_u64(const uint64_t* mine, uint32_t k, uint64_t* all) override {
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(d.coll.ensure((size_t)(W + 1) * k * 8));
        uint64_t* buf = d.coll.as<uint64_t>();
        HIPCHK(hipMemcpyAsync(buf, mine, (size_t)k * 8, hipMemcpyHostToDevice, d.stream));
        int rc = enqueue([&](ncclComm_t c) -> int {
            NCCLCHK(ncclAllGather(buf, buf + k, k, ncclUint64, c, d.stream));
            return AMBC_OK;
        });
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(all, buf + k, (size_t)W * k * 8, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        return AMBC_OK;
    }
    int allreduce_u64(uint64_t* v, uint32_t k, int op) override {
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(d.coll.ensure((size_t)k * 8));
        uint64_t* buf = d.coll.as<uint64_t>();
        HIPCHK(hipMemcpyAsync(buf, v, (size_t)k * 8, hipMemcpyHostToDevice, d.stream));
        const ncclRedOp_t o = op == AMBC_OP_MIN ? ncclMin : op == AMBC_OP_MAX ? ncclMax : ncclSum;
        int rc = enqueue([&](ncclComm_t c) -> int {
            NCCLCHK(ncclAllReduce(buf, buf, k, ncclUint64, o, c, d.stream));
            return AMBC_OK;
        });
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(v, buf, (size_t)k * 8, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        return AMBC_OK;
    }
    int gather(const uint8_t* src, uint8_t* dst, const uint64_t* offs, const uint64_t* lens, int root) override {
        HIPCHK(hipSetDevice(d.id));
        // pieces of kP2pPiece bytes per send/recv (both sides cut the same way):
        // the size connect_group's warm-up sent, so no piece needs a p2p channel
        // that the warm-up left unconnected (§7 of DESIGN.md)
        const uint64_t PIECE = kP2pPiece;
        int rc = enqueue([&](ncclComm_t c) -> int {
            NCCLCHK(ncclGroupStart());
            if (r == root) {
                for (int q = 0; q < W; q++) {
                    if (q == root) continue;
                    for (uint64_t o = 0; o < lens[q]; o += PIECE)
                        NCCLCHK(ncclRecv(dst + offs[q] + o, std::min(PIECE, lens[q] - o), ncclUint8, q, c, d.stream));
                }
            } else {
                for (uint64_t o = 0; o < lens[r]; o += PIECE)
                    NCCLCHK(ncclSend(src + o, std::min(PIECE, lens[r] - o), ncclUint8, root, c, d.stream));
            }
            NCCLCHK(ncclGroupEnd());
            return AMBC_OK;
        });
        if (rc) return rc;
        if (r == root && lens[r] && src != dst + offs[r])
            HIPCHK(hipMemcpyAsync(dst + offs[r], src, lens[r], hipMemcpyDeviceToDevice, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        return AMBC_OK;
    }
    void abort() override {
        if (!group) return;   // a process per GPU: the status exchanges keep the ranks in step
        gate->abort([&] {
            for (ncclComm_t& c : *group)
                if (c) { (void)ncclCommAbort(c); c = nullptr; }
        });
    }
};

// ---------------------------------------------------------------------------
// host threads of one process (a ctx that lists a device more than once)
// ---------------------------------------------------------------------------
struct LocalTransport : Transport {
    Hub& hub;
    Dev& d;
    LocalTransport(Hub& h, Dev& dev, int rank) : hub(h), d(dev) { W = h.W; r = rank; }
    int sync() { return hub.wait() ? AMBC_OK : fail(AMBC_E_COMM, "another shard failed"); }

    int allgather_u64(const uint64_t* mine, uint32_t k, uint64_t* all) override {
        hub.vals[r].assign(mine, mine + k);
        int rc = sync();
        if (rc) return rc;
        for (int q = 0; q < W; q++) std::memcpy(all + (size_t)q * k, hub.vals[q].data(), (size_t)k * 8);
        return sync();
    }
    int allreduce_u64(uint64_t* v, uint32_t k, int op) override {
        std::vector<uint64_t> all((size_t)W * k);
        int rc = allgather_u64(v, k, all.data());
        if (rc) return rc;
        for (uint32_t i = 0; i < k; i++) {
            uint64_t a = all[i];
            for (int q = 1; q < W; q++) {
                const uint64_t b = all[(size_t)q * k + i];
                a = op == AMBC_OP_MIN ? std::min(a, b) : op == AMBC_OP_MAX ? std::max(a, b) : a + b;
            }
            v[i] = a;
        }
        return AMBC_OK;
    }
    int gather(const uint8_t* src, uint8_t* dst, const uint64_t* offs, const uint64_t* lens, int root) override {
        hub.srcs[r] = src;
        int rc = sync();
        if (rc) return rc;
        if (r == root) {
            HIPCHK(hipSetDevice(d.id));
            for (int q = 0; q < W; q++)
                if (lens[q] && hub.srcs[q] != dst + offs[q])
                    HIPCHK(hipMemcpyAsync(dst + offs[q], hub.srcs[q], lens[q], hipMemcpyDefault, d.stream));
            HIPCHK(hipStreamSynchronize(d.stream));
        }
        return sync();   // the sources stay valid until the root has copied them
    }
    void abort() override { hub.fail(); }
};

// one rank (no communicator)
struct SelfTransport : Transport {
    Dev& d;
    explicit SelfTransport(Dev& dev) : d(dev) {}
    int allgather_u64(const uint64_t* mine, uint32_t k, uint64_t* all) override {
        std::memcpy(all, mine, (size_t)k * 8);
        return AMBC_OK;
    }
    int allreduce_u64(uint64_t*, uint32_t, int) override { return AMBC_OK; }
    int gather(const uint8_t* src, uint8_t* dst, const uint64_t* offs, const uint64_t* lens, int) override {
        if (lens[0] && src != dst + offs[0]) {
            HIPCHK(hipSetDevice(d.id));
            HIPCHK(hipMemcpyAsync(dst + offs[0], src, lens[0], hipMemcpyDeviceToDevice, d.stream));
            HIPCHK(hipStreamSynchronize(d.stream));
        }
        return AMBC_OK;
    }
};

// the reference-mode remainder exchange: MIN of the first no-winner chunk, and
// of an ok flag, so that a rank that failed before the exchange still joins it
// and every rank leaves together
int shard_allreduce_min(Transport* t, uint64_t* v, int rc_local) {
    uint64_t x[2] = {*v, rc_local ? 0ull : 1ull};
    int rc = t->allreduce_u64(x, 2, AMBC_OP_MIN);
    if (rc) return rc;
    if (rc_local) return rc_local;
    if (!x[1]) return fail(AMBC_E_COMM, "another rank failed before the remainder exchange");
    *v = x[0];
    return AMBC_OK;
}

// every rank's status (MIN of 64 + rc): the ranks continue together or fail
// together, so that none waits in a collective for a rank that already left
static int all_ok(Transport& t, int rc_local) {
    const std::string mine = g_err;
    uint64_t v = (uint64_t)(64 + rc_local);
    int rc = t.allreduce_u64(&v, 1, AMBC_OP_MIN);
    if (rc) return rc;
    const int code = (int)v - 64;
    if (code == AMBC_OK) return AMBC_OK;
    return fail(code, rc_local ? mine : "another rank failed (" + std::to_string(code) + ")");
}

static void shard_bounds(uint64_t n_total, uint32_t C, int W, int r, uint64_t* k0, uint64_t* k1) {
    const uint64_t M = (n_total + C - 1) / C;
    *k0 = (uint64_t)(((unsigned __int128)M * r) / W);
    *k1 = (uint64_t)(((unsigned __int128)M * (r + 1)) / W);
}

// stats of all ranks (AllReduce SUM); kernel / copy times stay this rank's
constexpr uint32_t NSTAT = 262;
static int reduce_stats(Transport& t, ambc_stats* st) {
    uint64_t v[NSTAT];
    std::memcpy(v, st->method_usage, 256 * 8);
    v[256] = st->total_chunks;
    v[257] = st->compressed_chunks;
    v[258] = st->raw_chunks;
    v[259] = st->bytes_saved;
    v[260] = st->payload_bytes;
    v[261] = st->overhead_bytes;
    int rc = t.allreduce_u64(v, NSTAT, AMBC_OP_SUM);
    if (rc) return rc;
    std::memcpy(st->method_usage, v, 256 * 8);
    st->total_chunks = v[256];
    st->compressed_chunks = v[257];
    st->raw_chunks = v[258];
    st->bytes_saved = v[259];
    st->payload_bytes = v[260];
    st->overhead_bytes = v[261];
    return AMBC_OK;
}

// Compress this rank's shard (chunks [k0, k1) of the logical input) into d_out;
// root 0 gathers the whole body into its d_out, root -1 leaves every rank's
// packages in place (info->offset says where they go in the file-order body).
static int shard_compress(Dev& d, Transport& t, const uint8_t* d_shard, uint64_t n_total, const ambc_params* p,
                          uint8_t* d_out, uint64_t out_cap, int root, ambc_shard_info* info, ambc_stats* st) {
    int rc = check_params(p);
    if (rc) return rc;
    if (root != 0 && root != -1) return fail(AMBC_E_INVAL, "root must be 0 or -1");
    const uint32_t C = p->chunk_size;
    uint64_t k0, k1;
    shard_bounds(n_total, C, t.W, t.r, &k0, &k1);
    const uint64_t b0 = std::min(k0 * C, n_total), b1 = std::min(k1 * C, n_total);
    ambc_params q = *p;
    if (t.r != t.W - 1) q.flags |= AMBC_FLAG_NO_END_CHUNK;   // the last rank ends the body
    // reference mode exchanges inside compress_on (the remainder): first agree
    // that no rank leaves before it (its own check of the output capacity)
    if (t.W > 1 && p->mode == AMBC_MODE_REFERENCE) {
        const uint64_t bound = ambc_compress_bound(b1 - b0, C) - (t.r != t.W - 1 ? END_CHUNK : 0);
        const int pre = out_cap < bound ? fail(AMBC_E_CAPACITY, "device output capacity < ambc_compress_bound")
                                        : AMBC_OK;
        if ((rc = all_ok(t, pre))) return rc;
    }
    ShardInfo si{&t, k0, n_total, t.r};
    uint64_t len = 0;
    ambc_stats lst{};
    rc = compress_on(d, d_shard, b1 - b0, &q, d_out, out_cap, &len, &lst, t.W > 1 ? &si : nullptr);
    const std::string err = g_err;
    const uint64_t t0 = now_ns();
    // 1. sizes, the root's capacity and every rank's status -> file offsets (a
    //    rank whose compress failed still joins, and all leave together)
    std::vector<uint64_t> all((size_t)3 * t.W);
    const uint64_t mine[3] = {len, out_cap, (uint64_t)(64 + rc)};
    int rc2 = t.allgather_u64(mine, 3, all.data());
    if (rc) return fail(rc, err);
    if (rc2) return rc2;
    std::vector<uint64_t> offs(t.W + 1, 0), lens(t.W);
    for (int i = 0; i < t.W; i++) {
        const int code = (int)all[3 * i + 2] - 64;
        if (code != AMBC_OK) return fail(code, "another rank failed to compress its shard (" + std::to_string(code) + ")");
        lens[i] = all[3 * i];
        offs[i + 1] = offs[i] + lens[i];
    }
    // 2. statistics
    if ((rc = reduce_stats(t, &lst))) return rc;
    // 4. optional gather onto rank 0
    if (root == 0) {
        if (offs[t.W] > all[1]) return fail(AMBC_E_CAPACITY, "root's output capacity < the whole body");   // (rank 0's cap)
        if ((rc = t.gather(d_out, d_out, offs.data(), lens.data(), 0))) return rc;
    }
    lst.total_ns += now_ns() - t0;
    if (info) {
        info->local_len = len;
        info->offset = offs[t.r];
        info->total = offs[t.W];
        info->shard_begin = b0;
        info->shard_end = b1;
    }
    if (st) *st = lst;
    return AMBC_OK;
}

constexpr int SHARD_WHOLE = 1;   // root -1 and the ranks need the whole-body fallback

// Decode across the ranks: every rank holds the host body; ambc_split_body cuts
// it at package boundaries into W ranges of about orig_size / W output bytes;
// rank q decodes its range into device memory (rank 0 straight into its slot of
// the output).  A body whose packages decode to other lengths than announced
// (the reference's lenient paths) cannot be cut in advance: the ranks agree on
// that (AllReduce MIN of a flag) and rank 0 then decodes the whole body.
static int shard_decompress(Dev& d, Transport& t, const uint8_t* body, uint64_t blen, uint64_t orig_size,
                            const uint64_t reg[4], uint8_t* d_out, uint64_t out_cap, int root,
                            ambc_shard_info* info, ambc_stats* st) {
    if (root != 0 && root != -1) return fail(AMBC_E_INVAL, "root must be 0 or -1");
    std::vector<uint64_t> bo(t.W + 1), oo(t.W + 1);
    int rc = ambc_split_body(body, blen, orig_size, reg, (uint32_t)t.W, bo.data(), oo.data());
    if (rc) return rc;      // a marker mismatch is found identically by every rank
    int last = t.W - 1;
    while (last > 0 && bo[last + 1] == bo[last]) last--;
    const uint64_t b0 = bo[t.r], b1 = bo[t.r + 1], o0 = oo[t.r], o1 = oo[t.r + 1];
    ambc_stats lst{};
    uint64_t ok = 1;
    int drc = AMBC_OK;
    std::string derr;
    if (o1 - o0 > out_cap) {
        drc = fail(AMBC_E_CAPACITY, "device output capacity < this rank's decoded range");
    } else if (root == 0 && t.r == 0 && out_cap < orig_size) {
        // the root gathers (or, lenient bodies, decodes) the whole output
        drc = fail(AMBC_E_CAPACITY, "root's capacity < orig_size");
    } else if (b1 > b0) {
        std::vector<ambc_host_chunk> host;
        drc = decompress_on(d, body + b0, b1 - b0, o1 - o0, reg, nullptr, host, &lst, d_out);
        ok = (t.r >= last || lst.payload_bytes == o1 - o0) ? 1 : 0;
    } else if (o1 > o0) {   // an empty range that must still produce bytes: only the lenient case
        ok = 0;
    }
    if (drc) derr = g_err;
    // status of all ranks: [ok, 64 + rc] (MIN picks any failure)
    uint64_t v[2] = {ok, (uint64_t)(64 + drc)};
    if ((rc = t.allreduce_u64(v, 2, AMBC_OP_MIN))) return rc;
    if ((int)v[1] - 64 != AMBC_OK) {
        const int code = (int)v[1] - 64;
        return fail(code, drc ? derr : "another rank failed to decode its range");
    }
    bool whole = false;
    if (v[0]) {
        if (root == 0) {
            std::vector<uint64_t> lens(t.W);
            for (int q = 0; q < t.W; q++) lens[q] = oo[q + 1] - oo[q];
            if ((rc = t.gather(d_out, d_out, oo.data(), lens.data(), 0))) return rc;
        }
    } else {
        if (root != 0) return SHARD_WHOLE;
        if (t.r == 0) {   // (out_cap >= orig_size: checked with the status above)
            std::vector<ambc_host_chunk> host;
            if ((rc = decompress_on(d, body, blen, orig_size, reg, nullptr, host, &lst, d_out))) return rc;
        }
        whole = true;
    }
    if (info) {
        info->local_len = whole ? (t.r == 0 ? orig_size : 0) : o1 - o0;
        info->offset = whole ? 0 : o0;
        info->total = orig_size;
        info->shard_begin = whole ? 0 : b0;
        info->shard_end = whole ? (t.r == 0 ? blen : 0) : b1;
    }
    if (st) *st = lst;
    return AMBC_OK;
}

// One thread issues, as one group over every communicator of the ctx, each
// collective kind the in-process ranks use -- AllGather and AllReduce of u64 at
// the sizes the calls exchange, and every rank's Send / Recv to rank 0 (the
// gather) -- so that every connection exists before the rank threads start:
// after this no enqueue waits for a peer.  (This is the single-process multi-GPU
// pattern of SURVEY.md §5; it stays unverified until an 8-GPU node runs it.)
static int connect_group(ambc_ctx* ctx) {
    const int G = (int)ctx->devs.size();
    constexpr uint32_t K = 262;            // (NSTAT: the largest u64 exchange)
    for (int g = 0; g < G; g++) {
        Dev& d = ctx->devs[g];
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(d.coll.ensure((size_t)(G + 1) * K * 8));
        HIPCHK(hipMemsetAsync(d.coll.p, 0, (size_t)(G + 1) * K * 8, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
    }
    for (uint32_t k : {1u, 3u, K}) {
        NCCLCHK(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            Dev& d = ctx->devs[g];
            uint64_t* buf = d.coll.as<uint64_t>();
            NCCLCHK(ncclAllGather(buf, buf + k, k, ncclUint64, ctx->dev_comms[g], d.stream));
        }
        NCCLCHK(ncclGroupEnd());
        NCCLCHK(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            Dev& d = ctx->devs[g];
            uint64_t* buf = d.coll.as<uint64_t>();
            NCCLCHK(ncclAllReduce(buf, buf, k, ncclUint64, ncclSum, ctx->dev_comms[g], d.stream));
        }
        NCCLCHK(ncclGroupEnd());
    }
    // the gather's Send / Recv pairs at its piece size and at a small size
    // (device scratch: rank 0 receives G - 1 pieces)
    std::vector<Buf> wb(G);
    for (int g = 0; g < G; g++) {
        HIPCHK(hipSetDevice(ctx->devs[g].id));
        HIPCHK(wb[g].ensure((size_t)(g == 0 ? std::max(1, G - 1) : 1) * kP2pPiece));
    }
    for (uint64_t bytes : {kP2pPiece, (uint64_t)8}) {
        NCCLCHK(ncclGroupStart());
        for (int g = 0; g < G; g++) {
            Dev& d = ctx->devs[g];
            uint8_t* buf = wb[g].as<uint8_t>();
            if (g == 0) {
                for (int q = 1; q < G; q++)
                    NCCLCHK(ncclRecv(buf + (q - 1) * kP2pPiece, bytes, ncclUint8, q, ctx->dev_comms[0], d.stream));
            } else {
                NCCLCHK(ncclSend(buf, bytes, ncclUint8, 0, ctx->dev_comms[g], d.stream));
            }
        }
        NCCLCHK(ncclGroupEnd());
    }
    for (int g = 0; g < G; g++) {
        HIPCHK(hipSetDevice(ctx->devs[g].id));
        HIPCHK(hipStreamSynchronize(ctx->devs[g].stream));
        wb[g].release();
    }
    return AMBC_OK;
}

// in-process multi-device: one transport per device
static int make_transports(ambc_ctx* ctx, std::unique_ptr<Hub>& hub, std::vector<std::unique_ptr<Transport>>& ts) {
    const int G = (int)ctx->devs.size();
    std::set<int> ids;
    for (auto& d : ctx->devs) ids.insert(d.id);
    if ((int)ids.size() == G && !getenv("AMBC_LOCAL_TRANSPORT")) {
        bool fresh = ctx->dev_comms.empty();
        for (ncclComm_t c : ctx->dev_comms) fresh = fresh || !c;   // aborted by a failed call
        if (fresh) {
            for (ncclComm_t c : ctx->dev_comms) if (c) (void)ncclCommDestroy(c);
            std::vector<int> dl;
            for (auto& d : ctx->devs) dl.push_back(d.id);
            ctx->dev_comms.assign(G, nullptr);
            // every connection at init (NCCL_RUNTIME_CONNECT=0, set by ambc_init
            // for a multi-device ctx unless the caller chose otherwise), and the
            // warm-up below connects whatever the init leaves to the first call
            NCCLCHK(ncclCommInitAll(ctx->dev_comms.data(), G, dl.data()));
            ctx->comm_gate.reset();
            if (int rc = connect_group(ctx)) {
                for (ncclComm_t& c : ctx->dev_comms) if (c) { (void)ncclCommAbort(c); c = nullptr; }
                return rc;
            }
        }
        for (int g = 0; g < G; g++) {
            RcclTransport* rt = new RcclTransport(ctx->dev_comms[g], ctx->devs[g], G, g);
            rt->group = &ctx->dev_comms;
            rt->gate = &ctx->comm_gate;
            ts.emplace_back(rt);
        }
    } else {
        hub.reset(new Hub(G));
        for (int g = 0; g < G; g++) ts.emplace_back(new LocalTransport(*hub, ctx->devs[g], g));
    }
    return AMBC_OK;
}

// runs fn(g) on one host thread per device; the first error wins
template <typename F>
static int run_ranks(std::vector<std::unique_ptr<Transport>>& ts, F fn) {
    const int G = (int)ts.size();
    std::vector<int> rcs(G, 0);
    std::vector<std::string> errs(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++)
        th.emplace_back([&, g]() {
            rcs[g] = fn(g);
            if (rcs[g]) {
                errs[g] = g_err;
                ts[g]->abort();
            }
        });
    for (auto& x : th) x.join();
    for (int g = 0; g < G; g++)   // report the root cause, not a peer's "another shard failed"
        if (rcs[g] && rcs[g] != AMBC_E_COMM) return fail(rcs[g], errs[g]);
    for (int g = 0; g < G; g++)
        if (rcs[g]) return fail(rcs[g], errs[g]);
    return AMBC_OK;
}

// Host buffers over several devices.  Native mode: the input streams through
// the devices in chunk-aligned slabs dealt round-robin (slab s on device s % G);
// every device overlaps the H2D of its next slab, the compression of this one and
// the D2H of the previous one (compress_slabs' pipeline, ambc_host.cpp), and after
// every round an AllGather of the slabs' body sizes gives each slab its file
// offset, so every body goes straight to its place in the host output.  The
// AllGather carries each rank's status: a failed rank still joins it and all
// leave together.  Reference mode (the remainder-raw rule is global): contiguous
// shards, one compress each (shard_compress), whole-shard copies.
static int compress_multi_slabs(ambc_ctx* ctx, std::vector<std::unique_ptr<Transport>>& ts, const uint8_t* in,
                                uint64_t n, const ambc_params* p, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                ambc_stats* st) {
    const uint64_t t0 = now_ns();
    const int G = (int)ts.size();
    const uint32_t C = p->chunk_size;
    const uint64_t SLAB = std::max<uint64_t>(C, slab_bytes() / C * C);
    const uint64_t ns = (n + SLAB - 1) / SLAB;
    const uint64_t rounds = (ns + G - 1) / G;
    const uint64_t sb = ambc_compress_bound(SLAB, C) + 64;
    std::vector<ambc_stats> sst(G);
    std::vector<uint64_t> kern(G, 0), total(G, 0);
    auto slab_len = [&](uint64_t s) { return s < ns ? std::min(SLAB, n - s * SLAB) : 0ull; };
    int rc = run_ranks(ts, [&](int g) -> int {
      Dev& d = ctx->devs[g];
      auto rank_body = [&]() -> int {
        Transport& t = *ts[g];
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(d.in.ensure(2 * (SLAB + 64)));
        HIPCHK(d.out.ensure(2 * sb));
        uint8_t* din[2] = {d.in.as<uint8_t>(), d.in.as<uint8_t>() + SLAB + 64};
        uint8_t* dout[2] = {d.out.as<uint8_t>(), d.out.as<uint8_t>() + sb};
        hipEvent_t* h2d_done = d.xev;
        hipEvent_t* comp_done = d.xev + 2;
        hipEvent_t* d2h_done = d.xev + 4;
        auto up = [&](uint64_t j) -> int {
            const uint64_t s = j * G + g;
            if (s >= ns) return AMBC_OK;
            if (j >= 2) HIPCHK(hipStreamWaitEvent(d.xs[0], comp_done[j & 1], 0));  // din[j&1] free
            HIPCHK(hipMemcpyAsync(din[j & 1], in + s * SLAB, slab_len(s), hipMemcpyHostToDevice, d.xs[0]));
            HIPCHK(hipEventRecord(h2d_done[j & 1], d.xs[0]));
            return AMBC_OK;
        };
        ambc_stats tot{};
        uint64_t base = 0;
        int rl = up(0);
        std::vector<uint64_t> all((size_t)2 * G);
        for (uint64_t j = 0; j < rounds; j++) {
            const uint64_t s = j * G + g;
            uint64_t len = 0;
            ambc_stats s1{};
            if (rl == AMBC_OK && j + 1 < rounds) rl = up(j + 1);
            if (rl == AMBC_OK && s < ns) {
                auto run = [&]() -> int {
                    HIPCHK(hipStreamWaitEvent(d.stream, h2d_done[j & 1], 0));
                    if (j >= 2) HIPCHK(hipStreamWaitEvent(d.stream, d2h_done[j & 1], 0));  // dout[j&1] free
                    ambc_params q = *p;
                    if (s + 1 != ns) { q.flags |= AMBC_FLAG_NO_END_CHUNK; q.ent_tail = nullptr; }
                    int r2 = compress_on(d, din[j & 1], slab_len(s), &q, dout[j & 1], sb, &len, &s1);
                    if (r2) return r2;
                    HIPCHK(hipEventRecord(comp_done[j & 1], d.stream));
                    return AMBC_OK;
                };
                rl = run();
            }
            // this round's body sizes and statuses -> the slabs' file offsets
            const std::string err = g_err;
            const uint64_t mine[2] = {len, (uint64_t)(64 + rl)};
            int rc2 = t.allgather_u64(mine, 2, all.data());
            if (rc2) return rc2;
            uint64_t off = base, round_total = 0;
            int peer = AMBC_OK;
            for (int q = 0; q < G; q++) {
                if (q < g) off += all[2 * q];
                round_total += all[2 * q];
                if ((int)all[2 * q + 1] - 64 != AMBC_OK && peer == AMBC_OK) peer = (int)all[2 * q + 1] - 64;
            }
            if (rl) return fail(rl, err);
            if (peer) return fail(peer, "another device failed its slab (" + std::to_string(peer) + ")");
            if (base + round_total > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small for the body");
            if (len) {
                HIPCHK(hipStreamWaitEvent(d.xs[1], comp_done[j & 1], 0));
                HIPCHK(hipMemcpyAsync(out + off, dout[j & 1], len, hipMemcpyDeviceToHost, d.xs[1]));
                HIPCHK(hipEventRecord(d2h_done[j & 1], d.xs[1]));
            }
            base += round_total;
            kern[g] += s1.kernel_ns;
            add_stats(&tot, s1);
        }
        HIPCHK(hipStreamSynchronize(d.xs[0]));
        HIPCHK(hipStreamSynchronize(d.xs[1]));
        int rc3 = reduce_stats(t, &tot);
        if (rc3) return rc3;
        sst[g] = tot;
        total[g] = base;
        return AMBC_OK;
      };
      const int r = rank_body();
      // every exit, failures included: no copy on the caller's buffers (the next
      // slab's H2D from `in`, an earlier round's D2H into `out`) outlives the call
      (void)hipSetDevice(d.id);
      const hipError_t e0 = hipStreamSynchronize(d.xs[0]), e1 = hipStreamSynchronize(d.xs[1]),
                       e2 = hipStreamSynchronize(d.stream);
      if (r) return r;
      for (hipError_t e : {e0, e1, e2})
          if (e != hipSuccess) return fail(AMBC_E_DEVICE, std::string("slab pipeline sync: ") + hipGetErrorString(e));
      return AMBC_OK;
    });
    if (rc) return rc;
    *out_len = total[0];
    if (st) {
        *st = sst[0];
        st->kernel_ns = *std::max_element(kern.begin(), kern.end());
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

int compress_batch_multi(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p, uint8_t* out,
                         uint64_t out_cap, uint64_t* out_len, ambc_stats* st) {
    const uint64_t t0 = now_ns();
    std::unique_ptr<Hub> hub;
    std::vector<std::unique_ptr<Transport>> ts;
    int rc = make_transports(ctx, hub, ts);
    if (rc) return rc;
    if (p->mode == AMBC_MODE_NATIVE) return compress_multi_slabs(ctx, ts, in, n, p, out, out_cap, out_len, st);
    const int G = (int)ts.size();
    std::vector<ambc_stats> sst(G);
    std::vector<ambc_shard_info> inf(G);
    std::vector<uint64_t> h2d(G, 0), d2h(G, 0);
    rc = run_ranks(ts, [&](int g) -> int {
        Dev& d = ctx->devs[g];
        uint64_t k0, k1;
        shard_bounds(n, p->chunk_size, G, g, &k0, &k1);
        const uint64_t b0 = std::min(k0 * p->chunk_size, n), b1 = std::min(k1 * p->chunk_size, n);
        const uint64_t bound = ambc_compress_bound(b1 - b0, p->chunk_size);
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(d.in.ensure(b1 - b0 + 64));
        HIPCHK(d.out.ensure(bound + 64));
        uint64_t t = now_ns();
        if (b1 > b0) HIPCHK(hipMemcpyAsync(d.in.p, in + b0, b1 - b0, hipMemcpyHostToDevice, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        h2d[g] = now_ns() - t;
        int r = shard_compress(d, *ts[g], d.in.as<uint8_t>(), n, p, d.out.as<uint8_t>(), d.out.cap, -1, &inf[g],
                               &sst[g]);
        if (r) return r;
        // every rank writes its packages at its file offset (the totals agree on every rank)
        if (inf[g].total > out_cap) return fail(AMBC_E_CAPACITY, "output buffer too small for the body");
        t = now_ns();
        if (inf[g].local_len)
            HIPCHK(hipMemcpyAsync(out + inf[g].offset, d.out.p, inf[g].local_len, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        d2h[g] = now_ns() - t;
        return AMBC_OK;
    });
    if (rc) return rc;
    *out_len = inf[0].total;
    if (st) {
        *st = sst[0];
        st->kernel_ns = 0;
        for (int g = 0; g < G; g++) {
            st->kernel_ns = std::max(st->kernel_ns, sst[g].kernel_ns);
            st->h2d_ns += h2d[g];
            st->d2h_ns += d2h[g];
        }
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

}  // namespace ambc

using namespace ambc;

static Transport* proc_transport(ambc_ctx* ctx, std::unique_ptr<Transport>& hold) {
    if (ctx->comm) hold.reset(new RcclTransport(ctx->comm, ctx->devs[0], ctx->nranks, ctx->rank));
    else hold.reset(new SelfTransport(ctx->devs[0]));
    return hold.get();
}

extern "C" {

int ambc_comm_unique_id(uint8_t* id) {
    if (!id) return fail(AMBC_E_INVAL, "id is NULL");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, AMBC_COMM_ID_BYTES);
    return AMBC_OK;
}

int ambc_comm_init_rank(ambc_ctx* ctx, int nranks, int rank, const uint8_t* id) {
    if (!ctx || ctx->devs.size() != 1 || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(AMBC_E_INVAL, "ambc_comm_init_rank needs a one-device ctx, 0 <= rank < nranks and an id");
    if (ctx->comm) return fail(AMBC_E_INVAL, "communicator already initialised");
    ncclUniqueId u;
    std::memcpy(u.internal, id, AMBC_COMM_ID_BYTES);
    HIPCHK(hipSetDevice(ctx->devs[0].id));
    ncclComm_t c = nullptr;
    NCCLCHK(ncclCommInitRank(&c, nranks, u, rank));
    ctx->comm = c;
    ctx->nranks = nranks;
    ctx->rank = rank;
    return AMBC_OK;
}

int ambc_comm_size(ambc_ctx* ctx, int* nranks, int* rank) {
    if (!ctx) return fail(AMBC_E_INVAL, "ctx is NULL");
    if (nranks) *nranks = ctx->nranks;
    if (rank) *rank = ctx->rank;
    return AMBC_OK;
}

int ambc_comm_allreduce_u64(ambc_ctx* ctx, uint64_t* v, uint32_t k, int op) {
    if (!ctx || (!v && k) || op < AMBC_OP_SUM || op > AMBC_OP_MAX) return fail(AMBC_E_INVAL, "bad argument");
    std::unique_ptr<Transport> hold;
    return proc_transport(ctx, hold)->allreduce_u64(v, k, op);
}

int ambc_comm_allgather_u64(ambc_ctx* ctx, const uint64_t* mine, uint32_t k, uint64_t* all) {
    if (!ctx || ((!mine || !all) && k)) return fail(AMBC_E_INVAL, "bad argument");
    std::unique_ptr<Transport> hold;
    return proc_transport(ctx, hold)->allgather_u64(mine, k, all);
}

int ambc_comm_barrier(ambc_ctx* ctx) {
    if (!ctx) return fail(AMBC_E_INVAL, "ctx is NULL");
    uint64_t one = 1;
    std::unique_ptr<Transport> hold;
    int rc = proc_transport(ctx, hold)->allreduce_u64(&one, 1, AMBC_OP_SUM);
    if (rc) return rc;
    HIPCHK(hipSetDevice(ctx->devs[0].id));
    HIPCHK(hipDeviceSynchronize());
    return AMBC_OK;
}

int ambc_comm_gather(ambc_ctx* ctx, const void* d_src, uint64_t len, void* d_dst, uint64_t dst_cap,
                     uint64_t* offset, uint64_t* total) {
    if (!ctx || (!d_src && len)) return fail(AMBC_E_INVAL, "bad argument");
    std::unique_ptr<Transport> hold;
    Transport* t = proc_transport(ctx, hold);
    std::vector<uint64_t> all((size_t)2 * t->W);
    const uint64_t mine[2] = {len, dst_cap};
    int rc = t->allgather_u64(mine, 2, all.data());
    if (rc) return rc;
    std::vector<uint64_t> offs(t->W + 1, 0), lens(t->W);
    for (int i = 0; i < t->W; i++) {
        lens[i] = all[2 * i];
        offs[i + 1] = offs[i] + lens[i];
    }
    if (offs[t->W] > all[1]) return fail(AMBC_E_CAPACITY, "rank 0's capacity < the gathered bytes");
    if (t->r == 0 && !d_dst) return fail(AMBC_E_INVAL, "rank 0 needs d_dst");
    if ((rc = t->gather((const uint8_t*)d_src, (uint8_t*)d_dst, offs.data(), lens.data(), 0))) return rc;
    if (offset) *offset = offs[t->r];
    if (total) *total = offs[t->W];
    return AMBC_OK;
}

int ambc_shard_range(uint64_t n_total, uint32_t chunk, int nranks, int rank, uint64_t* begin, uint64_t* end) {
    if (chunk == 0 || nranks < 1 || rank < 0 || rank >= nranks || !begin || !end)
        return fail(AMBC_E_INVAL, "bad argument");
    uint64_t k0, k1;
    shard_bounds(n_total, chunk, nranks, rank, &k0, &k1);
    *begin = std::min<uint64_t>(k0 * chunk, n_total);
    *end = std::min<uint64_t>(k1 * chunk, n_total);
    return AMBC_OK;
}

int ambc_compress_shard(ambc_ctx* ctx, const void* d_shard, uint64_t n_total, const ambc_params* p, void* d_out,
                        uint64_t out_cap, int root, ambc_shard_info* info, ambc_stats* st) {
    if (!ctx || ctx->devs.size() != 1) return fail(AMBC_E_INVAL, "ambc_compress_shard needs a one-device ctx");
    std::unique_ptr<Transport> hold;
    Transport* t = proc_transport(ctx, hold);
    return shard_compress(ctx->devs[0], *t, (const uint8_t*)d_shard, n_total, p, (uint8_t*)d_out, out_cap, root,
                          info, st);
}

int ambc_decompress_shard(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                          const uint64_t registered[4], void* d_out, uint64_t out_cap, int root,
                          ambc_shard_info* info, ambc_stats* st) {
    if (!ctx || ctx->devs.size() != 1 || (!body && body_len))
        return fail(AMBC_E_INVAL, "ambc_decompress_shard needs a one-device ctx and a body");
    uint64_t reg[4];
    default_registered(registered, reg);
    std::unique_ptr<Transport> hold;
    Transport* t = proc_transport(ctx, hold);
    int rc = shard_decompress(ctx->devs[0], *t, body, body_len, orig_size, reg, (uint8_t*)d_out, out_cap, root,
                              info, st);
    if (rc == SHARD_WHOLE)
        return fail(AMBC_E_INVAL, "the body's packages decode to other lengths than announced: "
                                  "it needs the whole-body fallback of root 0");
    return rc;
}

int ambc_decompress_multi(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                          const uint64_t registered[4], uint8_t* out, ambc_stats* st) {
    if (!ctx || ctx->devs.empty() || (!body && body_len) || (!out && orig_size))
        return fail(AMBC_E_INVAL, "NULL argument");
    const uint64_t t0 = now_ns();
    uint64_t reg[4];
    default_registered(registered, reg);
    std::unique_ptr<Hub> hub;
    std::vector<std::unique_ptr<Transport>> ts;
    int rc = make_transports(ctx, hub, ts);
    if (rc) return rc;
    const int G = (int)ts.size();
    std::vector<ambc_stats> sst(G);
    std::vector<ambc_shard_info> inf(G);
    rc = run_ranks(ts, [&](int g) -> int {
        Dev& d = ctx->devs[g];
        HIPCHK(hipSetDevice(d.id));
        // rank 0 may need the whole output (lenient fallback); the others their range
        HIPCHK(d.out.ensure(orig_size + 64));
        int r = shard_decompress(d, *ts[g], body, body_len, orig_size, reg, d.out.as<uint8_t>(), orig_size, -1,
                                 &inf[g], &sst[g]);
        if (r == SHARD_WHOLE) {
            // the ranks agreed on the whole-body fallback: rank 0 decodes it alone
            if (g != 0) { inf[g].local_len = 0; return AMBC_OK; }
            std::vector<ambc_host_chunk> host;
            if ((r = decompress_on(d, body, body_len, orig_size, reg, nullptr, host, &sst[g], d.out.as<uint8_t>())))
                return r;
            inf[g].local_len = orig_size;
            inf[g].offset = 0;
        } else if (r) {
            return r;
        }
        if (inf[g].local_len)
            HIPCHK(hipMemcpyAsync(out + inf[g].offset, d.out.p, inf[g].local_len, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        return AMBC_OK;
    });
    if (rc) return rc;
    if (st) {
        std::memset(st, 0, sizeof *st);
        for (int g = 0; g < G; g++) {
            st->total_chunks += sst[g].total_chunks;
            st->payload_bytes += sst[g].payload_bytes;
            st->kernel_ns = std::max(st->kernel_ns, sst[g].kernel_ns);
        }
        st->total_ns = now_ns() - t0;
    }
    return AMBC_OK;
}

}  // extern "C"
