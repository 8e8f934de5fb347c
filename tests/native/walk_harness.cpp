// walk_harness.cpp -- the host concurrency of libambc_hip on the CPU, for the
// sanitizer builds (tests/test_native_sanitizers.py: -fsanitize=thread, and
// -fsanitize=address,undefined).  It drives the library's own code, not copies:
//
//   * WalkPool (ambc_sync.h): tasks of every size, two threads submitting at once;
//   * Hub (ambc_sync.h): ranks exchanging values at barriers, a failing rank;
//   * AbortGate (ambc_sync.h): ranks enqueueing on "communicators" (heap objects)
//     while a failed rank aborts them -- a use after free shows under ASan / TSan;
//   * walk_decide (ambc_walkcore.h): the multi-size walk over a synthetic backend
//     (per-chunk payload lengths from a deterministic cost model of mixed data) --
//     parallel walks, the two-phase decide, guess chains with request-bit claims
//     and per-thread buckets, breadth speculation, LZ4 shared across sizes and
//     host-scored methods -- and its path compared with a serial restatement of
//     the reference's loop (adaptive_compressor.py:363-394, :537-590) over the same
//     model; plus a size the backend refuses near the end (must fail or finish,
//     never hang).
//
//     walk_harness [threads]     exit 0: every check passed
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ambc.h"
#include "../../adaptive-compression_amd/csrc/ambc_walkcore.h"

namespace ambc {
thread_local std::string g_err;   // (defined by ambc_host.cpp in the library)
}
using namespace ambc;

static int g_failures = 0;
#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            g_failures++;                                                  \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);           \
            fprintf(stderr, __VA_ARGS__);                                  \
            fputc('\n', stderr);                                           \
        }                                                                  \
    } while (0)

static uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ---------------------------------------------------------------------------
static void test_pool(unsigned T) {
    WalkPool pool(T);
    CHECK(pool.size() == T, "pool size %u != %u", pool.size(), T);
    std::vector<uint64_t> acc(1 << 16, 0);
    for (int round = 0; round < 300; round++) {
        const size_t m = 1 + (size_t)(splitmix(round) % acc.size());
        pool.run([&](unsigned t, unsigned Tn) {
            for (size_t i = m * t / Tn; i < m * (t + 1) / Tn; i++) acc[i] += (i ^ (uint64_t)round) | (1ull << 40);
        });
        // (results visible to the caller after run() returns)
        uint64_t s = 0;
        for (size_t i = 0; i < m; i++) s += acc[i] != 0;
        CHECK(s == m, "round %d: %zu of %zu slots written", round, (size_t)s, m);
        std::fill(acc.begin(), acc.begin() + m, 0);
    }
    // two submitters take turns on one pool
    std::atomic<uint64_t> total{0};
    auto submit = [&](int who) {
        for (int r = 0; r < 200; r++)
            pool.run([&](unsigned t, unsigned) { total.fetch_add(1 + t * 0 + (uint64_t)who * 0); });
    };
    std::thread a(submit, 0), b(submit, 1);
    a.join();
    b.join();
    CHECK(total.load() == 400ull * T, "submitters: %llu slices, expected %llu",
          (unsigned long long)total.load(), 400ull * T);
}

// ---------------------------------------------------------------------------
static void test_hub() {
    const int W = 4;
    Hub hub(W);
    std::vector<uint64_t> sums(W, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < W; r++)
        th.emplace_back([&, r] {
            for (int step = 0; step < 200; step++) {
                hub.vals[r].assign(3, (uint64_t)(r + 1) * (step + 1));
                if (!hub.wait()) return;
                uint64_t s = 0;
                for (int q = 0; q < W; q++) s += hub.vals[q][1];
                sums[r] += s;
                if (!hub.wait()) return;   // (everyone has read before the next write)
            }
        });
    for (auto& t : th) t.join();
    uint64_t want = 0;
    for (int step = 0; step < 200; step++) want += (uint64_t)(1 + 2 + 3 + 4) * (step + 1);
    for (int r = 0; r < W; r++) CHECK(sums[r] == want, "hub rank %d: %llu != %llu", r, (unsigned long long)sums[r], (unsigned long long)want);
    // a failing rank releases the others
    Hub h2(3);
    std::atomic<int> released{0};
    std::vector<std::thread> t2;
    for (int r = 0; r < 2; r++) t2.emplace_back([&] { if (!h2.wait()) released++; });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    h2.fail();
    for (auto& t : t2) t.join();
    CHECK(released.load() == 2, "hub fail released %d of 2 waiters", released.load());
    CHECK(!h2.wait(), "a failed hub lets nobody pass");
}

// ---------------------------------------------------------------------------
struct FakeComm {
    std::atomic<uint64_t> ops{0};
};

static void test_gate() {
    for (int trial = 0; trial < 50; trial++) {
        const int W = 4;
        AbortGate gate;
        std::vector<FakeComm*> comms(W);
        for (auto& c : comms) c = new FakeComm();
        std::atomic<int> refused{0};
        std::vector<std::thread> th;
        for (int r = 0; r < W; r++)
            th.emplace_back([&, r] {
                for (int k = 0; k < 2000; k++) {
                    if (r == 0 && k == 37 + trial) {   // rank 0 fails and aborts the group
                        gate.abort([&] {
                            for (auto& c : comms) { delete c; c = nullptr; }
                        });
                        return;
                    }
                    if (!gate.enter()) { refused++; return; }
                    comms[r]->ops.fetch_add(1);       // the "enqueue": touches the communicator
                    gate.leave();
                }
            });
        for (auto& t : th) t.join();
        for (auto& c : comms) CHECK(c == nullptr, "gate: communicator left alive");
        CHECK(!gate.enter(), "gate: enter after abort");
        for (auto& c : comms) delete c;
    }
    // an enqueuer that never returns by itself (a peer that never joins): abort()
    // still completes after its bounded wait, kills the communicators -- which is
    // what releases the stuck enqueuer -- and reports that it did not wait clean
    {
        AbortGate gate;
        FakeComm* comm = new FakeComm();
        std::atomic<bool> killed{false}, entered{false};
        std::thread stuck([&] {
            if (!gate.enter()) return;
            comm->ops.fetch_add(1);                             // (the enqueue's last use of it)
            entered = true;
            while (!killed.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));   // "inside the call"
            gate.leave();                                       // released by the abort: no further use
        });
        while (!entered.load()) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        const bool clean = gate.abort([&] { delete comm; comm = nullptr; killed = true; }, 150);
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        stuck.join();
        CHECK(!clean, "gate: a stuck enqueuer reported as clean");
        CHECK(comm == nullptr, "gate: communicator not killed after the bounded wait");
        CHECK(ms >= 140 && ms < 5000, "gate: bounded wait took %lld ms", (long long)ms);
        CHECK(!gate.enter(), "gate: enter after a bounded abort");
    }
}

// ---------------------------------------------------------------------------
// the synthetic data: classes per 256-byte cell in runs of 1..96 cells; a
// method's payload length is a cost over the chunk's class counts
struct Model {
    uint64_t n;
    std::vector<uint8_t> cls;            // per cell
    std::vector<uint64_t> pre[4];        // bytes of class c before cell i
    explicit Model(uint64_t n_, uint64_t seed) : n(n_) {
        const uint64_t cells = (n + 255) / 256;
        cls.resize(cells);
        uint64_t i = 0, s = seed;
        while (i < cells) {
            s = splitmix(s);
            const uint64_t run = 1 + (s >> 8) % 96;
            for (uint64_t j = 0; j < run && i < cells; j++) cls[i++] = (uint8_t)(s % 4);
        }
        for (auto& p : pre) p.assign(cells + 1, 0);
        for (uint64_t c = 0; c < cells; c++) {
            const uint64_t b = std::min<uint64_t>(256, n - c * 256);
            for (int k = 0; k < 4; k++) pre[k][c + 1] = pre[k][c] + (cls[c] == k ? b : 0);
        }
    }
    uint64_t count(int k, uint64_t a, uint64_t b) const {   // class-k bytes in [a, b)
        auto upto = [&](uint64_t x) {
            const uint64_t c = x / 256;
            return pre[k][c] + (c < cls.size() && cls[c] == k ? x - c * 256 : 0);
        };
        return upto(b) - upto(a);
    }
    // payload bytes of method id on [pos, pos + s)
    uint32_t cost(uint32_t id, uint64_t pos, uint32_t s) const {
        uint64_t c[4];
        for (int k = 0; k < 4; k++) c[k] = count(k, pos, pos + s);
        const uint32_t present = (c[0] > 0) + (c[1] > 0) + (c[2] > 0) + (c[3] > 0);
        switch (id) {
            case 1: return (uint32_t)(2 * (c[0] / 200 + c[1] + c[2] + c[3]) + 2);
            case 2: return (uint32_t)(c[0] / 30 + c[1] * 2 + c[2] * 3 / 5 + c[3] + 4);
            case 3: return (uint32_t)(5 + 5 * (8 + 20 * present) + (c[0] + 8 * c[1] + 43 * c[2] / 10 + 6 * c[3]) / 8);
            case 4: return s;
            case 6: return (uint32_t)(40 + c[0] / 100 + c[1] * 101 / 100 + c[2] * 3 / 10 + c[3] * 55 / 100);
            case 7: return (uint32_t)(60 + c[0] / 120 + c[1] + c[2] * 28 / 100 + c[3] / 2);
            case 9: return (uint32_t)(33 + c[0] / 250 * 4 + c[1] * 1004 / 1000 + c[2] * 45 / 100 + c[3] * 7 / 10 +
                                      (s <= 4096 ? 50 : 0));
            default: return s;
        }
    }
};

static const uint32_t kHostIds[] = {6, 7};

// the reference's per-size method loop: ids ascending, strict "<" on len + 18,
// below the chunk's length (id 0 / 255: none)
static void winner(const Model& m, const ambc_params* p, uint64_t pos, uint32_t s, bool host, uint32_t* plen,
                   uint8_t* id) {
    uint32_t best = s;
    *id = 255;
    *plen = s;
    for (uint32_t t = 1; t < 16; t++) {
        const bool dev = ms_eligible(p, s, t);
        const bool hst = host && (t == 6 || t == 7) && p->pref_min[t] <= s && s <= p->pref_max[t];
        if (!dev && !hst) continue;
        const uint32_t l = m.cost(t, pos, s);
        if (l + HDR < best) { best = l + HDR; *id = (uint8_t)t; *plen = l; }
    }
}

struct SynthBackend {
    const Model& m;
    uint32_t refuse_dict_above = 0;      // check_size: Dictionary eligible above this fails (0: never)
    struct Slot { std::vector<uint32_t> plen, lz; std::vector<uint8_t> ids; };
    Slot slots[16];
    uint64_t launches = 0;
    int launch(int slot, const ambc_params* pk, uint32_t sz, const uint64_t* pos, uint32_t cnt,
               const uint32_t* subc, uint32_t nsub) {
        Slot& S = slots[slot];
        S.plen.assign(cnt, 0);
        S.ids.assign(cnt, 255);
        S.lz.assign((size_t)cnt * LZ4_SUB_MAX, 0xFFFFFFFFu);
        for (uint32_t q = 0; q < cnt; q++) {
            if (pos[q] + sz > m.n) return fail(AMBC_E_INVAL, "batch past the input");
            winner(m, pk, pos[q], sz, false, &S.plen[q], &S.ids[q]);
            for (uint32_t j = 0; j < nsub; j++)
                if (subc[j] < sz) S.lz[(size_t)q * LZ4_SUB_MAX + j] = m.cost(9, pos[q], subc[j]) - 23;
        }
        launches++;
        return AMBC_OK;
    }
    uint64_t queries = 0;   // (a batch "still runs" on every third query: results come out of order)
    bool ready(int slot) { return (++queries + (uint64_t)slot) % 3 != 0; }
    int finish(int slot, const uint32_t** plen, const uint8_t** ids, const uint32_t** lz) {
        *plen = slots[slot].plen.data();
        *ids = slots[slot].ids.data();
        *lz = slots[slot].lz.data();
        return AMBC_OK;
    }
    // the input arrives in pieces: every call sees `step` more bytes (0: all at once)
    uint64_t step = 0, av = 0;
    uint64_t avail() {
        if (!step) return m.n;
        const uint64_t a = std::min(av, m.n);
        av += step;
        return a;
    }
    int wait_avail(uint64_t want) {
        if (want > m.n) want = m.n;
        if (av < want) av = want;
        return AMBC_OK;
    }
    int check_size(const ambc_params* pk, uint32_t s) {
        if (refuse_dict_above && ms_eligible(pk, s, AMBC_M_DICT) && s > refuse_dict_above)
            return fail(AMBC_E_INVAL, "refused size");
        return AMBC_OK;
    }
};

struct HostCtx { const Model* m; const ambc_params* p; std::atomic<uint64_t> pairs{0}; };

static int host_eval(void* user, const uint64_t* pos, const uint32_t* size, uint32_t count, uint8_t* id,
                     uint32_t* len) {
    HostCtx* h = static_cast<HostCtx*>(user);
    for (uint32_t i = 0; i < count; i++) {
        uint32_t best = size[i];
        id[i] = 0;
        len[i] = 0;
        for (uint32_t t : kHostIds) {
            if (!(h->p->pref_min[t] <= size[i] && size[i] <= h->p->pref_max[t])) continue;
            const uint32_t l = h->m->cost(t, pos[i], size[i]);
            if (l + HDR < best) { best = l + HDR; id[i] = (uint8_t)t; len[i] = l; }
        }
    }
    h->pairs += count;
    return 0;
}
static int host_emit(void*, uint64_t, uint32_t, uint8_t, uint8_t*, uint32_t) { return 1; }

// the reference's walk, serially: every candidate size clamped to the remainder
// (duplicates skipped), the per-size winner, the strict fp64 ratio minimum in
// list order; no winner -> the remainder raw
static std::vector<WalkPkg> serial_walk(const Model& m, const ambc_params* p, const std::vector<uint32_t>& cands,
                                        bool host) {
    std::vector<WalkPkg> path;
    uint64_t pos = 0, body = 0;
    while (pos < m.n) {
        const uint64_t remain = m.n - pos;
        double br = 1.0;
        uint32_t bs = 0, bl = 0;
        uint8_t bid = 255;
        std::vector<uint32_t> seen;
        for (uint32_t c : cands) {
            const uint32_t s = (uint32_t)std::min<uint64_t>(c, remain);
            if (std::find(seen.begin(), seen.end(), s) != seen.end()) continue;
            seen.push_back(s);
            uint32_t l;
            uint8_t id;
            winner(m, p, pos, s, host, &l, &id);
            if (id == 255) continue;
            const double r = (double)(l + HDR) / (double)s;
            if (r < br) { br = r; bs = s; bl = l; bid = id; }
        }
        if (bid == 255) {
            path.push_back(WalkPkg{pos, (uint32_t)remain, (uint32_t)remain, 255, 0, body});
            break;
        }
        path.push_back(WalkPkg{pos, bs, bl, bid, (uint8_t)(host && (bid == 6 || bid == 7)), body});
        body += HDR + bl;
        pos += bs;
    }
    return path;
}

static ambc_params make_params(std::initializer_list<uint32_t> ids) {
    ambc_params p;
    std::memset(&p, 0, sizeof p);
    const uint32_t lo[16] = {0, 32, 128, 32, 32, 64, 1024, 8192, 512, 1024, 1024, 1024, 0, 0, 0, 0};
    const uint32_t hi[16] = {0, 4096, 8192, 8192, 4096, 65536, 262144, 524288, 262144, 65536, 262144, 262144, 0, 0, 0, 0};
    for (int i = 0; i < 16; i++) { p.pref_min[i] = lo[i]; p.pref_max[i] = hi[i]; }
    for (uint32_t t : ids) p.method_mask |= 1u << t;
    return p;
}

static bool same_path(const std::vector<WalkPkg>& a, const std::vector<WalkPkg>& b, std::string* why) {
    if (a.size() != b.size()) { *why = "length " + std::to_string(a.size()) + " vs " + std::to_string(b.size()); }
    for (size_t i = 0; i < std::min(a.size(), b.size()); i++)
        if (a[i].pos != b[i].pos || a[i].s != b[i].s || a[i].plen != b[i].plen || a[i].id != b[i].id ||
            a[i].off != b[i].off) {
            *why = "package " + std::to_string(i) + " at " + std::to_string(a[i].pos) + ": s " + std::to_string(a[i].s) +
                   "/" + std::to_string(b[i].s) + " id " + std::to_string(a[i].id) + "/" + std::to_string(b[i].id);
            return false;
        }
    return a.size() == b.size();
}

static void test_walks(unsigned T) {
    WalkPool pool(T);
    WalkMemory mem;   // (reused across calls: the epochs must keep calls apart)
    const std::vector<std::vector<uint32_t>> cand_lists = {
        {131072, 65536, 32768, 16384, 8192, 4096, 2048, 1024}, {65536, 3072, 1024}, {6144, 2048, 1536, 1024},
        {16384, 1024, 8192, 4096}, {3000, 1000}};
    struct MS { std::initializer_list<uint32_t> ids; bool host; };
    const MS msets[] = {{{1, 3, 4, 9}, false}, {{1, 3, 4}, false}, {{9}, false}, {{1, 3, 4, 9}, true}, {{1, 2, 3, 4}, false}};
    WalkConfig cfgs[5];
    cfgs[0].walks = 1; cfgs[0].spec = 0; cfgs[0].breadth = 0;                 // the plain serial walk
    cfgs[1].walks = 1024; cfgs[1].span = 16384;                                // many walks, library defaults
    cfgs[2].walks = 512; cfgs[2].span = 8192; cfgs[2].spec = 3; cfgs[2].breadth = 4096; cfgs[2].groups = 2;
    cfgs[3].walks = 300; cfgs[3].span = 4096; cfgs[3].rechain = true; cfgs[3].noshare = true; cfgs[3].launch_desc = true;
    cfgs[4].walks = 2048; cfgs[4].span = 1024; cfgs[4].spec = 6;           // batches of thousands: parallel fills
    const uint64_t sizes[] = {3 * (1u << 20) + 777, 200000, 1025, 7};
    int runs = 0;
    uint64_t pkgs = 0, rounds = 0, evals = 0, ids_seen = 0;
    for (uint64_t n : sizes)
        for (size_t ci = 0; ci < cand_lists.size(); ci++)
            for (const MS& ms : msets) {
                const Model m(n, 0x5EED0000ull + n * 31 + ci);
                const ambc_params p = make_params(ms.ids);
                const auto want = serial_walk(m, &p, cand_lists[ci], ms.host);
                for (const WalkConfig& cfg : cfgs) {
                    SynthBackend be{m};
                    // (every other configuration: the input arriving in pieces)
                    if ((&cfg - cfgs) % 2 == 1) be.step = std::max<uint64_t>(4096, n / 7);
                    HostCtx hctx{&m, &p};
                    ambc_host_codecs hc{host_eval, host_emit, &hctx};
                    WalkOutcome wo;
                    const int rc = walk_decide(be, mem, pool, cfg, n, &p, cand_lists[ci], ms.host ? &hc : nullptr, wo);
                    std::string why;
                    CHECK(rc == AMBC_OK, "walk n=%llu cands#%zu: rc %d (%s)", (unsigned long long)n, ci, rc, g_err.c_str());
                    if (rc == AMBC_OK)
                        CHECK(same_path(wo.path, want, &why), "walk n=%llu cands#%zu walks=%llu: %s",
                              (unsigned long long)n, ci, (unsigned long long)cfg.walks, why.c_str());
                    runs++;
                    pkgs += wo.path.size();
                    rounds += wo.steps;
                    evals += wo.evaluated;
                    for (const WalkPkg& k : wo.path) ids_seen |= 1ull << (k.id & 63);
                }
            }
    // a size the backend refuses near the end (Dictionary's prefs up to 12288, its
    // encoder to 8192): the walk fails or finishes -- the serial walk's path when it
    // finishes -- and never waits forever on a forgotten request
    for (uint64_t n : {5ull * 4096 + 10000, 9ull * 4096 + 10000, 64ull * 4096 + 10000})
        for (const WalkConfig& cfg : cfgs) {
            const Model m(n, 77 + n);
            ambc_params p = make_params({1, 2, 3, 4, 9});
            p.pref_max[2] = 12288;
            SynthBackend be{m};
            be.refuse_dict_above = 8192;
            WalkOutcome wo;
            const std::vector<uint32_t> cands = {16384, 4096};
            const int rc = walk_decide(be, mem, pool, cfg, n, &p, cands, nullptr, wo);
            CHECK(rc == AMBC_OK || rc == AMBC_E_INVAL, "refused size: rc %d", rc);
            if (rc == AMBC_OK) {
                std::string why;
                CHECK(same_path(wo.path, serial_walk(m, &p, cands, false), &why), "refused size: %s", why.c_str());
            }
            runs++;
        }
    printf("walks: %d runs, %llu packages, %llu rounds, %llu chunk evaluations, ids seen %llx\n", runs,
           (unsigned long long)pkgs, (unsigned long long)rounds, (unsigned long long)evals,
           (unsigned long long)ids_seen);
}

int main(int argc, char** argv) {
    const unsigned T = argc > 1 ? (unsigned)std::max(1, atoi(argv[1])) : 4;
    test_pool(T);
    test_hub();
    test_gate();
    test_walks(T);
    printf("walk_harness threads=%u: %s (%d failures)\n", T, g_failures ? "FAILED" : "ok", g_failures);
    return g_failures ? 1 : 0;
}
