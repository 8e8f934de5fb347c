// ambc_walkcore.h -- the decision part of the reference's multi-size walk
// (AdaptiveCompressor._adaptive_compress with several CHUNK_SIZE_CANDIDATES,
// adaptive_compressor.py:363-394 + _pick_best_chunk_and_method :537-590), free of
// HIP types: ambc_multisize.cpp runs it over the device's batched encoders, and
// tests/native/walk_harness.cpp over synthetic batch results on the CPU, under
// ThreadSanitizer and AddressSanitizer (race detection).
//
// At position pos every candidate size s = min(cand, remain) is encoded as one
// chunk by the reference's per-size method loop (ids ascending, strict "<" on
// len + 18), the sizes compare by their fp64 ratio (len + 18) / s, strictly, in
// list order, and the walk moves on by the winning size; a position where no
// size beats raw stores the whole remainder as one raw package (:586-588).
//
// The walk is serial -- each decision sets the next position -- so it runs as
// many walks at once: K walks start at positions spread over the input (all on
// the grid of g = gcd(candidates), where every walk position lies), and all of
// them advance in lock step.  One step evaluates every (position, size) the
// active walks need in ONE batch per size (the backend: one workgroup per chunk
// on the device).  With LZ4 (id 9) among the methods one parse per position
// serves every size: the largest LZ4-eligible size M is encoded with all its
// methods and reports the LZ4 block of each smaller candidate prefix (k_encode's
// lz4sub); the smaller sizes run only their other methods, and id 9 joins them
// last in id order here.  A walk stops when its next position has already been
// decided (it joined the path of another walk: from there on both are the same
// walk) or at the end.  Every decided position's successor is decided, so the
// walk from 0 -- the reference's walk -- is then read off the decisions.
//
// Host concurrency (the part the sanitizer harness exists for): a WalkPool runs
// each round's fills (records of distinct positions), the walks' read-only step
// phase, and the guess-chain requests (records reset by one claiming thread via
// an epoch compare-exchange, request bits claimed by atomic or, positions into
// per-thread buckets merged afterwards).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ambc.h"
#include "ambc_consts.h"
#include "ambc_hostutil.h"
#include "ambc_sync.h"

namespace ambc {

inline bool ms_eligible(const ambc_params* p, uint32_t s, uint32_t id) {
    return ((p->method_mask >> id) & 1) && p->pref_min[id] <= s && s <= p->pref_max[id];
}

inline bool ms_any_eligible(const ambc_params* p, uint32_t s, uint32_t skip = 0) {
    for (uint32_t id = 1; id < 16; id++)
        if (id != skip && ms_eligible(p, s, id)) return true;
    return false;
}

struct Decision {
    uint32_t s;      // chunk size taken at this position (the remainder when raw)
    uint32_t plen;
    uint8_t id;      // 255: the rest of the input as one raw package
    uint8_t host;    // the package comes from a host-scored method (ambc_host_codecs)
};

// the position records of one context, kept across calls (a fresh 40 KB page per
// 256 positions cost ~25 ms of page faults and construction per 256 MiB call): a
// record belongs to the call whose epoch it carries
struct WalkMemory {
    std::vector<std::vector<uint8_t>> pages;
    size_t rsz = 0;
    uint32_t epoch = 0;
};

// Per walk position (pos = idx * g) and candidate index i: the evaluation of
// size S_i = min(cands[i], n - pos).  Part "O": the winner of the size's methods
// other than LZ4 -- or, at the position's LZ4 size M, of all of them; part "L":
// LZ4's block for S_i < M, from M's launch.  One record per position (its state
// and its nc candidates contiguous: two or three cache lines for the reference's
// eight candidates, where a field-per-array layout touched a dozen), in pages of
// 256 positions allocated when a walk first reaches them.
struct PosTable {
    static constexpr uint32_t PB = 8;
    struct Cand {
        uint32_t plen = 0, lz = 0xFFFFFFFFu, hlen = 0;
        uint8_t id = 255, hid = 0;                  // (hid / hlen: the host codecs' winner, 0: none)
        uint16_t pad = 0;
    };
    struct Rec {
        uint32_t have = 0, req = 0;                 // bit i: part O of candidate i known / asked for
        uint32_t hhave = 0, hreq = 0;               //   ... the host part of candidate i
        uint8_t mhave = 0, mreq = 0, decided = 0;   // M's launch known / asked for; decision taken
        uint8_t pad = 0;
        Decision dec{0, 0, 0, 0};
        uint32_t epoch = 0;                         // the call this record belongs to (0: none)
        Cand* c() { return reinterpret_cast<Cand*>(this + 1); }
    };
    static_assert(sizeof(Rec) % alignof(Cand) == 0, "candidates follow the record");
    uint64_t g = 1;
    int gsh = -1;                // log2(g) when g is a power of two (the reference's list: 1024)
    uint32_t nc = 0;
    size_t rsz = 0;              // bytes per position record
    uint32_t epoch = 0;
    std::vector<std::vector<uint8_t>>* pages = nullptr;   // the context's pool (WalkMemory::pages)
    std::unique_ptr<std::atomic<uint8_t>[]> pready;       // page i allocated (touch() from several threads)
    std::mutex pmu;
    static constexpr uint32_t BUSY = 0xFFFFFFFFu;         // a record being reset by one thread
    void init(uint64_t n, uint64_t g_, uint32_t nc_, WalkMemory& m) {
        g = g_;
        gsh = (g & (g - 1)) == 0 ? __builtin_ctzll(g) : -1;
        nc = nc_;
        rsz = sizeof(Rec) + (size_t)nc * sizeof(Cand);
        pages = &m.pages;
        if (m.rsz != rsz) {   // another record layout: the pool starts over
            m.pages.clear();
            m.rsz = rsz;
        }
        const size_t np = (size_t)((n / g >> PB) + 1);
        if (m.pages.size() < np) m.pages.resize(np);
        if (++m.epoch == 0) {   // (wrapped: no record may carry a reused epoch)
            m.pages.clear();
            m.pages.resize(np);
            m.epoch = 1;
        }
        epoch = m.epoch;
        pready.reset(new std::atomic<uint8_t>[m.pages.size()]);
        for (size_t i = 0; i < m.pages.size(); i++) pready[i].store(m.pages[i].empty() ? 0 : 1);
    }
    std::vector<uint8_t>& page(size_t i) {
        if (!pready[i].load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(pmu);
            if (!pready[i].load(std::memory_order_relaxed)) {
                (*pages)[i].resize(rsz << PB);   // (zeros: epoch 0)
                pready[i].store(1, std::memory_order_release);
            }
        }
        return (*pages)[i];
    }
    // at() from several threads at once: the reset claimed by one of them
    Rec& touch(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        Rec* r = reinterpret_cast<Rec*>(page((size_t)(x >> PB)).data() + rsz * (uint32_t)(x & ((1u << PB) - 1)));
        uint32_t e = __atomic_load_n(&r->epoch, __ATOMIC_ACQUIRE);
        while (e != epoch) {
            if (e != BUSY && __atomic_compare_exchange_n(&r->epoch, &e, BUSY, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                Rec fresh;
                fresh.epoch = BUSY;
                std::memcpy(static_cast<void*>(r), &fresh, sizeof(Rec));
                for (uint32_t i = 0; i < nc; i++) new (r->c() + i) Cand();
                __atomic_store_n(&r->epoch, epoch, __ATOMIC_RELEASE);
                break;
            }
            while ((e = __atomic_load_n(&r->epoch, __ATOMIC_ACQUIRE)) == BUSY) std::this_thread::yield();
        }
        return *r;
    }
    // the record of position pos if this call touched it already, else null (no
    // writes: safe beside other readers)
    Rec* peek(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        if (!pready[(size_t)(x >> PB)].load(std::memory_order_acquire)) return nullptr;
        const std::vector<uint8_t>& pg = (*pages)[(size_t)(x >> PB)];
        Rec* r = reinterpret_cast<Rec*>(const_cast<uint8_t*>(pg.data()) + rsz * (uint32_t)(x & ((1u << PB) - 1)));
        return __atomic_load_n(&r->epoch, __ATOMIC_ACQUIRE) == epoch ? r : nullptr;
    }
    // the record of position pos: its page created on first use in the context,
    // the record reset on first use in this call (one thread only)
    Rec& at(uint64_t pos) {
        const uint64_t x = gsh >= 0 ? pos >> gsh : pos / g;
        const uint32_t slot = (uint32_t)(x & ((1u << PB) - 1));
        Rec* r = reinterpret_cast<Rec*>(page((size_t)(x >> PB)).data() + rsz * slot);
        if (r->epoch != epoch) {
            new (r) Rec();
            r->epoch = epoch;
            for (uint32_t i = 0; i < nc; i++) new (r->c() + i) Cand();
        }
        return *r;
    }
};

// the walk's tuning (library defaults; AMBC_MS_* environment overrides for sweeps)
struct WalkConfig {
    // walks: one per `span` input bytes, at most `walks` (256 MiB of mixed data,
    // reference candidates, second call: best of 512-2048 walks x 2-4 positions
    // ahead, profiles/r3_multisize_sweep.log)
    uint64_t walks = 1024, span = 256 << 10;
    // positions guessed ahead per walk (-1: by method set, below) and breadth
    // speculation for the last walks (-1: by method set)
    int spec = -1;
    int64_t breadth = -1;
    int groups = 1;             // interleaved walk groups (2: measured slower)
    bool rechain = false;       // re-ask a walk's whole guess chain every round
    bool noprio = false;        // launch the round's sizes in request order
    bool launch_desc = false;   // launch them largest first (default: largest, then smallest first)
    bool noshare = false;       // no LZ4 parse shared across sizes
    // host-scored codecs (ids 6 / 7 / 8, ambc_host_codecs): the positions of a walk's
    // guess chain that also get the host codecs (0: the walk's own position only;
    // -1: by default, below), and whether breadth positions get them (default no):
    // a host evaluation costs ~100 ms of a core per position (bz2 at eight sizes,
    // LZMA at five), a device one microseconds
    int hspec = -1;
    bool hbreadth = false;
    static WalkConfig from_env() {
        WalkConfig c;
        if (const char* e = getenv("AMBC_MS_WALKS")) c.walks = strtoull(e, nullptr, 10);
        if (const char* e = getenv("AMBC_MS_SPAN")) c.span = strtoull(e, nullptr, 10);
        if (const char* e = getenv("AMBC_MS_SPEC")) c.spec = atoi(e);
        if (const char* e = getenv("AMBC_MS_BREADTH")) c.breadth = atoll(e);
        if (const char* e = getenv("AMBC_MS_GROUPS")) c.groups = std::max(1, std::min(2, atoi(e)));
        c.rechain = getenv("AMBC_MS_RECHAIN") != nullptr;
        c.noprio = getenv("AMBC_MS_NOPRIO") != nullptr;
        c.launch_desc = getenv("AMBC_MS_LAUNCH_DESC") != nullptr;
        c.noshare = getenv("AMBC_MS_NOSHARE") != nullptr;
        if (const char* e = getenv("AMBC_MS_HSPEC")) c.hspec = atoi(e);
        c.hbreadth = getenv("AMBC_MS_HBREADTH") != nullptr;
        return c;
    }
};

// one package of the reference's walk from 0, at body offset `off`
struct WalkPkg { uint64_t pos; uint32_t s, plen; uint8_t id, host; uint64_t off; };

struct WalkOutcome {
    std::vector<WalkPkg> path;   // the packages in file order
    uint64_t body = 0;           // bytes of the packages (without the end chunk)
    uint32_t steps = 0;          // evaluation rounds
    uint64_t evaluated = 0;      // chunk evaluations they ran
    uint64_t wait_ns = 0;        // time in the backend's batches (launch to results)
    uint64_t t_dec = 0, t_req = 0, t_launch = 0, t_wait = 0, t_fill = 0, t_host = 0;
};

// The walk's decisions through a backend B:
//   int launch(int slot, const ambc_params* p, uint32_t size, const uint64_t* pos, uint32_t cnt,
//              const uint32_t* subc, uint32_t nsub)
//       evaluate the size-`size` chunks at pos[0..cnt) with p's methods on batch slot
//       `slot` (0..15; <= 8 in flight; nsub > 0: also the LZ4 block of every prefix
//       subc[j] below size); pos is only read during the call
//   bool ready(int slot)  slot's batch is done (no wait)
//   int finish(int slot, const uint32_t** plen, const uint8_t** ids, const uint32_t** lz)
//       wait for slot's batch: per chunk the payload length, the winning id (255:
//       raw) and lz[q * LZ4_SUB_MAX + j] (prefix j's block, 0xFFFFFFFF: LZ4 gave up)
//   uint64_t avail()     input bytes a batch may read: [0, avail()) is uploaded (n: all);
//                        a chunk [pos, pos + s) is launched once pos + s + 64 <= avail()
//                        or avail() == n, else its request waits for a later round
//   int wait_avail(uint64_t want)   block until avail() >= min(want, n)
//   int check_size(const ambc_params* p, uint32_t s)   AMBC_OK when the encoders take
//       an s-byte chunk with p's eligible methods
// Returns AMBC_OK with the walk from 0 in `out`, or the error code (g_err set).
template <class B>
int walk_decide(B& be, WalkMemory& mem, WalkPool& pool, const WalkConfig& cfg, uint64_t n, const ambc_params* p,
                const std::vector<uint32_t>& cands, const ambc_host_codecs* hc, WalkOutcome& out) {
    const uint32_t nc = (uint32_t)cands.size();
    // ---- LZ4 shared across sizes: M (the largest LZ4-eligible size at a position)
    // reports the smaller LZ4-eligible candidates' prefixes (sorted list subc) ----
    std::vector<uint32_t> subc(cands);
    std::sort(subc.begin(), subc.end());
    const bool lzshare = ((p->method_mask >> AMBC_M_LZ4) & 1) && subc.size() <= LZ4_SUB_MAX && !cfg.noshare;
    ambc_params po = *p;                       // the other methods (sizes below M)
    if (lzshare) po.method_mask &= ~(1u << AMBC_M_LZ4);
    const uint32_t nsub = (uint32_t)subc.size();

    // ---- the walks ----
    uint64_t g = 0;
    for (uint32_t c : cands) g = std::gcd(g, (uint64_t)c);
    PosTable T;
    T.init(n, g, nc, mem);
    // last: the size it took the step before; cq / cs: the guess chain asked for so
    // far (positions pos + k * cs below cq are requested already)
    struct Walk { uint64_t pos; uint32_t last; uint64_t cq = 0; uint32_t cs = 0; };
    std::vector<Walk> active;
    uint32_t max_cand = 0;
    for (uint32_t c : cands)
        if (hc || ms_any_eligible(p, c)) max_cand = std::max(max_cand, c);
    {
        // walk starts on the lattice of the largest eligible size: where that size
        // wins everywhere (homogeneous data) every walk runs on the same lattice
        // and joins the next one at once; elsewhere the mixed choices shift their
        // phases until they meet
        const uint64_t K = std::max<uint64_t>(1, std::min<uint64_t>(cfg.walks, n / std::max<uint64_t>(cfg.span, 1)));
        const uint64_t lat = max_cand ? max_cand : g;
        std::vector<uint64_t> starts;
        for (uint64_t k = 0; k < K; k++) starts.push_back((k * n / K) / lat * lat);
        starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
        if (n)
            for (uint64_t b0 : starts) active.push_back(Walk{b0, max_cand ? max_cand : cands[0]});
    }

    // the sizes at pos: S[i] = min(cands[i], remain); canonical = the first index
    // of its size; M = the largest LZ4-eligible one (0: none / no sharing)
    struct Sizes { uint32_t S[32]; uint32_t canon; uint32_t M; };
    const uint32_t maxc = *std::max_element(cands.begin(), cands.end());
    Sizes inner;                                       // every position with remain >= maxc
    bool have_inner = false;
    uint32_t jsub[32];                                 // subc index of cands[i]
    for (uint32_t i = 0; i < nc; i++)
        jsub[i] = (uint32_t)(std::lower_bound(subc.begin(), subc.end(), cands[i]) - subc.begin());
    auto sizes_fill = [&](uint64_t pos, Sizes& z) {
        const uint64_t remain = n - pos;
        z.canon = 0;
        z.M = 0;
        for (uint32_t i = 0; i < nc; i++) {
            z.S[i] = (uint32_t)std::min<uint64_t>(cands[i], remain);
            bool dup = false;
            for (uint32_t j = 0; j < i && !dup; j++) dup = z.S[j] == z.S[i];
            if (!dup) z.canon |= 1u << i;
            if (lzshare && ms_eligible(p, z.S[i], AMBC_M_LZ4)) z.M = std::max(z.M, z.S[i]);
        }
    };
    if (n >= maxc) {
        sizes_fill(0, inner);
        have_inner = true;
    }
    // the sizes at pos: inner's by reference, a position near the end's in a scratch
    // record (valid until the next call)
    Sizes edge;
    auto sizes_in = [&](uint64_t pos, Sizes& scratch) -> const Sizes& {   // (thread-safe with its own scratch)
        if (have_inner && n - pos >= maxc) return inner;
        sizes_fill(pos, scratch);
        return scratch;
    };
    auto sizes_at = [&](uint64_t pos) -> const Sizes& { return sizes_in(pos, edge); };
    // part O of candidate i at a position: needed (not raw by construction)?
    auto needs_o = [&](const Sizes& z, uint32_t i) {
        return z.S[i] == z.M ? false : ms_any_eligible(lzshare ? &po : p, z.S[i]);
    };
    auto needs_m = [&](const Sizes& z) { return z.M != 0; };
    auto ready_z = [&](const Sizes& z, const PosTable::Rec& r) -> bool {
        if (needs_m(z) && !r.mhave) return false;
        for (uint32_t i = 0; i < nc; i++)
            if (((z.canon >> i) & 1) && needs_o(z, i) && !((r.have >> i) & 1)) return false;
        if (hc && (r.hhave & z.canon) != z.canon) return false;
        return true;
    };
    // the reference's decision at pos (adaptive_compressor.py:546-590), all parts known
    auto decide_z = [&](uint64_t pos, const Sizes& z, PosTable::Rec& rec) -> Decision {
        const PosTable::Cand* cd = rec.c();
        const uint64_t remain = n - pos;
        double best_ratio = 1.0;
        uint32_t best_s = 0, best_plen = 0;
        uint8_t best_id = 255, best_host = 0;
        for (uint32_t i = 0; i < nc; i++) {
            // (the same clamped size again: same package, same ratio -- never strictly better)
            if (!((z.canon >> i) & 1)) continue;
            const uint32_t sz = z.S[i];
            if (!hc && !ms_any_eligible(p, sz)) continue;
            const PosTable::Cand& e = cd[i];
            uint32_t plen = e.plen;
            uint8_t id = e.id;
            uint8_t host = 0;
            if (sz != z.M && !needs_o(z, i)) id = 255;            // no other method: raw so far
            if (lzshare && sz < z.M && ms_eligible(p, sz, AMBC_M_LZ4)) {
                // id 9 comes last in id order: it wins only strictly below the others
                const uint32_t lb = e.lz;
                const uint32_t other = id == 255 ? sz : plen + HDR;
                if (lb != 0xFFFFFFFFu && (uint64_t)lb + 41 < other) { plen = lb + 23; id = 9; }
            }
            if (hc && e.hid && e.hlen + HDR < sz) {
                // the host codecs' winner joins in id order: smaller len, or a tie with a higher id
                const uint32_t hl = e.hlen;
                const uint8_t hi = e.hid;
                if (id == 255 || hl < plen || (hl == plen && hi < id)) { plen = hl; id = hi; host = 1; }
            }
            if (id == 255) continue;
            const double ratio = (double)(plen + HDR) / (double)sz;
            if (ratio < best_ratio) {
                best_ratio = ratio;
                best_s = sz;
                best_plen = plen;
                best_id = id;
                best_host = host;
            }
        }
        if (best_id == 255)
            return Decision{(uint32_t)std::min<uint64_t>(remain, 0xFFFFFFFFull), (uint32_t)remain, 255, 0};
        return Decision{best_s, best_plen, best_id, best_host};
    };
    // host-codec requests of one round: (position, size), and where they go
    std::vector<uint64_t> hpos;
    std::vector<uint32_t> hsize;
    // requests of one round: (size, kind) -> positions; kind 1 = M's launch.  A
    // handful of buckets, found by a short scan -- for inner positions (every size
    // the candidate's own) by a per-candidate cache
    using ReqKey = std::pair<uint32_t, int>;
    std::vector<std::pair<ReqKey, std::vector<uint64_t>>> req;
    int req_in[33];                                    // bucket of inner candidate i (32: M), -1: none yet
    auto req_clear = [&]() {
        req.clear();
        for (int& x : req_in) x = -1;
    };
    req_clear();
    auto req_bucket = [&](ReqKey key) -> std::vector<uint64_t>& {
        for (auto& b : req)
            if (b.first == key) return b.second;
        req.emplace_back(key, std::vector<uint64_t>());
        return req.back().second;
    };
    auto req_push = [&](bool in, int ci, ReqKey key, uint64_t pos) {
        if (!in) { req_bucket(key).push_back(pos); return; }
        if (req_in[ci] < 0) {
            req_bucket(key);
            for (size_t b = 0; b < req.size(); b++)
                if (req[b].first == key) req_in[ci] = (int)b;
        }
        req[(size_t)req_in[ci]].second.push_back(pos);
    };
    auto request = [&](uint64_t pos, bool host) {
        const Sizes& z = sizes_at(pos);
        const bool in = &z == &inner;
        PosTable::Rec& r = T.at(pos);
        if (needs_m(z) && !r.mhave && !r.mreq) {
            r.mreq = 1;
            req_push(in, 32, {z.M, 1}, pos);
        }
        for (uint32_t i = 0; i < nc; i++) {
            if (!((z.canon >> i) & 1)) continue;
            if (hc && host && !(((r.hhave | r.hreq) >> i) & 1)) {
                r.hreq |= 1u << i;
                hpos.push_back(pos);
                hsize.push_back(z.S[i]);
            }
            if (!needs_o(z, i)) continue;
            if (((r.have | r.req) >> i) & 1) continue;
            r.req |= 1u << i;
            req_push(in, (int)i, {z.S[i], 0}, pos);
        }
    };
    // the host codecs' answers for the round's pairs into the table
    std::vector<uint8_t> hid_out;
    std::vector<uint32_t> hlen_out;
    auto host_round = [&]() -> int {
        if (!hc || hpos.empty()) return AMBC_OK;
        const uint64_t th = now_ns();
        hid_out.assign(hpos.size(), 0);
        hlen_out.assign(hpos.size(), 0);
        if (hc->eval(hc->user, hpos.data(), hsize.data(), (uint32_t)hpos.size(), hid_out.data(), hlen_out.data()))
            return fail(AMBC_E_CODEC, "host codec evaluation failed");
        for (size_t q = 0; q < hpos.size(); q++) {
            const Sizes& z = sizes_at(hpos[q]);
            PosTable::Rec& r = T.at(hpos[q]);
            for (uint32_t i = 0; i < nc; i++)
                if (((z.canon >> i) & 1) && z.S[i] == hsize[q]) {
                    r.c()[i].hid = hid_out[q];
                    r.c()[i].hlen = hlen_out[q];
                    r.hhave |= 1u << i;
                }
        }
        hpos.clear();
        hsize.clear();
        out.t_host += now_ns() - th;
        return AMBC_OK;
    };
    // a batch's results into the table
    // (a batch's positions are distinct and were touched when requested: its
    // records fill in parallel, read through peek)
    auto fill_range = [&](const uint32_t* hplen, const uint8_t* hids, const uint32_t* hlz, uint32_t sz, int kind,
                          const std::vector<uint64_t>& poss, size_t q0, size_t q1) {
        Sizes scr;
        for (size_t q = q0; q < q1; q++) {
            const uint64_t pos = poss[q];
            const Sizes& z = sizes_in(pos, scr);
            PosTable::Rec& r = *T.peek(pos);
            PosTable::Cand* cd = r.c();
            for (uint32_t i = 0; i < nc; i++) {
                if (!((z.canon >> i) & 1)) continue;
                if (z.S[i] == sz && (kind == 1 || z.S[i] != z.M)) {
                    cd[i].plen = hplen[q];
                    cd[i].id = hids[q];
                    r.have |= 1u << i;
                }
                if (kind == 1 && z.S[i] < z.M) cd[i].lz = hlz[q * LZ4_SUB_MAX + jsub[i]];   // (S[i] = cands[i])
            }
            if (kind == 1) r.mhave = 1;
        }
    };
    auto fill = [&](const uint32_t* hplen, const uint8_t* hids, const uint32_t* hlz, uint32_t sz, int kind,
                    const std::vector<uint64_t>& poss) {
        const size_t m = poss.size();
        if (m < 2048 || pool.size() == 1) { fill_range(hplen, hids, hlz, sz, kind, poss, 0, m); return; }
        pool.run([&](unsigned t, unsigned Tn) {
            fill_range(hplen, hids, hlz, sz, kind, poss, m * t / Tn, m * (t + 1) / Tn);
        });
    };

    // Rounds: every walk decides as far as the known sizes reach; then ONE batch
    // per size evaluates each walk's next position and SPEC positions further
    // along the path it would take if it kept its last step size (a guess: a
    // right one saves a round, whose latency -- the slowest 64 KiB encode -- is
    // the walk's cost; a wrong one costs idle device time only).  groups = 2
    // runs the walks as two interleaved groups (the host decides and launches one
    // group while the device encodes the other's): measured slower -- 256 MiB
    // {1,3,4,9}: 55.8 -> 81.5 ms of walk at 1024 walks / 3 ahead, the groups'
    // batches contend on the device -- so one group is the default.
    // (speculation is cheap where one LZ4 parse serves every size: 6 ahead; where
    // every size runs its own encoders -- DEFLATE, zlib-9, Dictionary -- 1 ahead:
    // 256 MiB {1,3,4,9}: 4 / 5 / 6 / 8 ahead 72.4 / 64.1 / 58.4 / 94.9 ms (8 with
    // 2048 walks), {1,2,3,4,5}: 1 / 2 ahead 86.0 / 90.6 ms, like_reference() on 64
    // MiB: 0 / 1 / 2 ahead 0.229 / 0.255 / 0.224 GB/s; profiles/r3_multisize_sweep.log)
    // (round 4, with breadth speculation for the last walks: {1,2,3,4,5} 0 / 1 / 2
    // ahead 4.61-4.77 / 4.48-4.53 / 3.93-3.97 GB/s; like_reference() -- no breadth --
    // 0.31 / 0.34 / 0.28, profiles/r4_spec_ab)
    const bool z9walk = (p->flags & AMBC_FLAG_ZLIB9) && ((p->method_mask >> AMBC_M_DEFLATE) & 1);
    const int SPEC = cfg.spec >= 0 ? cfg.spec : (lzshare ? 6 : z9walk ? 1 : 0);
    // host codecs on the walk's own position only (16 MiB like_reference(full_set=True):
    // guesses with host codecs 3.68 s, without 2.59 s; profiles/r6_fullwalk_hspec)
    const int HSPEC = cfg.hspec >= 0 ? cfg.hspec : hc ? 0 : SPEC;
    const int GROUPS = cfg.groups;
    using Job = std::pair<std::pair<uint32_t, int>, std::vector<uint64_t>>;
    struct Group {
        std::vector<Walk> active;
        std::vector<Job> flight;     // batches on slots slot0.. (at most 8)
        int slot0 = 0;
        uint32_t rounds = 0;
    };
    Group grp[2];
    for (int gi = 0; gi < GROUPS; gi++) grp[gi].slot0 = 8 * gi;
    for (size_t i = 0; i < active.size(); i++) grp[i % GROUPS].active.push_back(active[i]);
    auto launch_job = [&](const Job& jb, int slot) -> int {
        const bool mk = jb.first.second == 1;
        return be.launch(slot, mk || !lzshare ? p : &po, jb.first.first, jb.second.data(), (uint32_t)jb.second.size(),
                         mk ? subc.data() : nullptr, mk ? nsub : 0);
    };
    auto finish_job = [&](const Job& jb, int slot) -> int {
        uint64_t tl = now_ns();
        const uint32_t* hplen = nullptr;
        const uint8_t* hids = nullptr;
        const uint32_t* hlz = nullptr;
        if (int rc = be.finish(slot, &hplen, &hids, &hlz)) return rc;
        out.t_wait += now_ns() - tl;
        tl = now_ns();
        fill(hplen, hids, hlz, jb.first.first, jb.first.second, jb.second);
        out.evaluated += jb.second.size();
        out.t_fill += now_ns() - tl;
        return AMBC_OK;
    };
    // the group's batches in flight: their results as they come (a small size's
    // batch fills the table while the round's largest -- launched first, on the
    // high-priority slot -- still runs)
    auto complete = [&](Group& G) -> int {
        const uint64_t tk = now_ns();
        std::vector<uint8_t> done(G.flight.size(), 0);
        size_t left = G.flight.size();
        while (left) {
            bool any = false;
            for (size_t j = 0; j < G.flight.size(); j++) {
                if (done[j] || (left > 1 && !be.ready(G.slot0 + (int)j))) continue;
                if (int rc = finish_job(G.flight[j], G.slot0 + (int)j)) return rc;
                done[j] = 1;
                left--;
                any = true;
            }
            if (!any) std::this_thread::yield();
        }
        G.flight.clear();
        out.wait_ns += now_ns() - tk;
        return AMBC_OK;
    };
    // decide as far as known, then ask for the next positions and launch
    auto advance = [&](Group& G) -> int {
        uint64_t tq = now_ns();
        // phase 1, in parallel and read-only: every walk's steps as far as its
        // positions are known; phase 2, in walk order: the steps into the table, a
        // walk stopping where an earlier one decided already (it joined that path:
        // the same decisions from there on) -- the sequential loop's outcome
        const size_t na = G.active.size();
        struct Trail { std::vector<std::pair<uint64_t, Decision>> steps; Walk end; bool open; };
        std::vector<Trail> trails(na);
        auto walk_range = [&](size_t a0, size_t a1) {
            Sizes scr;
            for (size_t a = a0; a < a1; a++) {
                Trail& tr = trails[a];
                tr.steps.clear();
                Walk w = G.active[a];
                tr.open = false;
                for (;;) {
                    PosTable::Rec* r = T.peek(w.pos);
                    if (r && r->decided) break;            // joined a decided path
                    const Sizes& z = sizes_in(w.pos, scr);
                    if (!r || !ready_z(z, *r)) { tr.open = true; break; }
                    const Decision dd = decide_z(w.pos, z, *r);
                    tr.steps.emplace_back(w.pos, dd);
                    if (dd.id == 255) break;               // the rest is raw: done
                    w.last = dd.s;
                    w.pos += dd.s;
                    if (w.pos >= n) break;
                }
                tr.end = w;
            }
        };
        if (na < 64 || pool.size() == 1) walk_range(0, na);
        else pool.run([&](unsigned t, unsigned Tn) { walk_range(na * t / Tn, na * (t + 1) / Tn); });
        std::vector<Walk> still;
        for (size_t a = 0; a < na; a++) {
            Trail& tr = trails[a];
            bool joined = false;
            for (const auto& st : tr.steps) {
                PosTable::Rec& r = T.at(st.first);
                if (r.decided) { joined = true; break; }
                r.decided = 1;
                r.dec = st.second;
            }
            if (joined || !tr.open) continue;
            PosTable::Rec* r = T.peek(tr.end.pos);
            if (r && r->decided) continue;                  // (decided by an earlier walk this round)
            still.push_back(tr.end);
        }
        // (two walks at one position: keep one)
        std::sort(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos < y.pos; });
        still.erase(std::unique(still.begin(), still.end(), [](const Walk& x, const Walk& y) { return x.pos == y.pos; }),
                    still.end());
        G.active.swap(still);
        out.t_dec += now_ns() - tq;
        tq = now_ns();
        if (G.active.empty()) return AMBC_OK;
        req_clear();
        hpos.clear();
        hsize.clear();
        // each walk's guess chain; many walks: on the pool, the records claimed by
        // atomic bit sets, the positions into per-thread buckets merged afterwards
        auto chain_of = [&](Walk& w, auto&& ask, auto&& rec_of) {
            uint64_t q = w.pos;
            int k = 0;
            // still on last round's chain: its requested prefix is skipped (with SPEC
            // 6 a walk re-asked for six positions a round, most of them known)
            if (!cfg.rechain && w.cs == w.last && w.cq > w.pos && (w.cq - w.pos) % w.last == 0) {
                k = (int)std::min<uint64_t>((w.cq - w.pos) / w.last, (uint64_t)SPEC + 1);
                q = w.pos + (uint64_t)k * w.last;
                // the walk's own position is always asked for again (its record
                // knows what is requested already): a speculative request there
                // may have been forgotten (a size check_size refuses), and the walk
                // would otherwise wait for it forever; host codecs skipped on a guess
                // are asked for here once the walk stands on it
                ask(w.pos, true);
                // (host codecs for the guesses within HSPEC that the skipped prefix holds)
                for (int kk = 1; kk < k && kk <= HSPEC; kk++) ask(w.pos + (uint64_t)kk * w.last, true);
            }
            for (; k <= SPEC && q < n; k++, q += w.last) {
                if (k && rec_of(q).decided) break;
                ask(q, k <= HSPEC);
            }
            w.cs = w.last;
            w.cq = q;
        };
        const size_t nw = G.active.size();
        if (nw < 64 || pool.size() == 1) {
            for (Walk& w : G.active) chain_of(w, request, [&](uint64_t q) -> PosTable::Rec& { return T.at(q); });
        } else {
            struct TL {
                std::vector<std::pair<ReqKey, std::vector<uint64_t>>> b;
                int in_idx[33];
                std::vector<uint64_t> hp;
                std::vector<uint32_t> hs;
            };
            std::vector<TL> tl(pool.size());
            pool.run([&](unsigned t, unsigned Tn) {
                TL& L = tl[t];
                for (int& x : L.in_idx) x = -1;
                Sizes scr;
                auto push = [&](bool in, int ci, ReqKey key, uint64_t pos) {
                    int bi = in ? L.in_idx[ci] : -1;
                    if (bi < 0) {
                        for (size_t b = 0; b < L.b.size() && bi < 0; b++)
                            if (L.b[b].first == key) bi = (int)b;
                        if (bi < 0) { L.b.emplace_back(key, std::vector<uint64_t>()); bi = (int)L.b.size() - 1; }
                        if (in) L.in_idx[ci] = bi;
                    }
                    L.b[(size_t)bi].second.push_back(pos);
                };
                auto ask = [&](uint64_t pos, bool host) {
                    const Sizes& z = sizes_in(pos, scr);
                    const bool in = &z == &inner;
                    PosTable::Rec& r = T.touch(pos);
                    if (needs_m(z) && !__atomic_load_n(&r.mhave, __ATOMIC_ACQUIRE) &&
                        !__atomic_exchange_n(&r.mreq, (uint8_t)1, __ATOMIC_ACQ_REL))
                        push(in, 32, {z.M, 1}, pos);
                    uint32_t want = 0, hwant = 0;
                    const uint32_t hhave = __atomic_load_n(&r.hhave, __ATOMIC_ACQUIRE);
                    const uint32_t have = __atomic_load_n(&r.have, __ATOMIC_ACQUIRE);
                    for (uint32_t i = 0; i < nc; i++) {
                        if (!((z.canon >> i) & 1)) continue;
                        if (hc && host && !((hhave >> i) & 1)) hwant |= 1u << i;
                        if (needs_o(z, i) && !((have >> i) & 1)) want |= 1u << i;
                    }
                    if (hwant) {
                        const uint32_t got = hwant & ~__atomic_fetch_or(&r.hreq, hwant, __ATOMIC_ACQ_REL);
                        for (uint32_t i = 0; i < nc; i++)
                            if ((got >> i) & 1) { L.hp.push_back(pos); L.hs.push_back(z.S[i]); }
                    }
                    if (want) {
                        const uint32_t got = want & ~__atomic_fetch_or(&r.req, want, __ATOMIC_ACQ_REL);
                        for (uint32_t i = 0; i < nc; i++)
                            if ((got >> i) & 1) push(in, (int)i, {z.S[i], 0}, pos);
                    }
                };
                for (size_t a = nw * t / Tn; a < nw * (t + 1) / Tn; a++)
                    chain_of(G.active[a], ask, [&](uint64_t q) -> PosTable::Rec& { return T.touch(q); });
            });
            for (TL& L : tl) {
                for (auto& b : L.b) {
                    std::vector<uint64_t>& dst = req_bucket(b.first);
                    dst.insert(dst.end(), b.second.begin(), b.second.end());
                }
                hpos.insert(hpos.end(), L.hp.begin(), L.hp.end());
                hsize.insert(hsize.end(), L.hs.begin(), L.hs.end());
            }
            for (int& x : req_in) x = -1;   // (bucket indices moved: the inner cache starts over)
        }
        // few walks left (the device idles behind one chunk's latency): each walk
        // also asks for every position its next step can reach, and a guess chain
        // from each, within BREADTH positions a round -- the next round then decides
        // at least two steps whatever size wins (breadth 0: off).  Budget: what
        // one round's latency hides, ~2048 chunks of 64 KiB ({1,2,3,4,5} 3.55-3.60 ->
        // 3.79-3.80 GB/s, {1,3,4,9} unchanged); with zlib-9, whose 64 KiB parse holds
        // a CU per chunk, about one chunk per CU: 256 (like_reference() 0 / 128 / 256
        // / 512 / 2048: 0.33 / 0.356 / 0.363 / 0.355 / 0.20 GB/s, profiles/r4_breadth_ab,
        // r5_breadth_ab)
        const uint64_t BREADTH = cfg.breadth >= 0 ? (uint64_t)cfg.breadth : (z9walk ? 256 : 2048);
        if (BREADTH && !G.active.empty() && G.active.size() * nc <= BREADTH) {
            const uint64_t per = BREADTH / G.active.size();
            for (const Walk& w : G.active) {
                const Sizes z = sizes_at(w.pos);           // (a copy: request() reuses the scratch)
                const uint32_t nsz = (uint32_t)__builtin_popcount(z.canon);
                const uint64_t depth = std::min<uint64_t>((uint64_t)SPEC + 1, std::max<uint64_t>(1, per / nsz));
                for (uint32_t i = 0; i < nc; i++) {
                    if (!((z.canon >> i) & 1) || z.S[i] == w.last) continue;   // (the main chain)
                    uint64_t q = w.pos + z.S[i];
                    for (uint64_t k = 0; k < depth && q < n; k++, q += z.S[i]) {
                        if (T.at(q).decided) break;
                        request(q, cfg.hbreadth);
                    }
                }
            }
        }
        std::vector<Job> jobs;
        // the input arrives in pieces (the backend's upload): chunks not all there yet
        // are forgotten like refused speculative ones and asked for again later (a
        // walk asks for its own position every round)
        const uint64_t av = be.avail();
        uint64_t need = ~0ull;     // the smallest input end a forgotten request needs
        auto forget = [&](const std::pair<uint32_t, int>& key, uint64_t q) {
            const Sizes& z = sizes_at(q);
            PosTable::Rec& rec = T.at(q);
            if (key.second == 1) rec.mreq = 0;
            for (uint32_t i = 0; i < nc; i++)
                if (z.S[i] == key.first) rec.req &= ~(1u << i);
        };
        for (auto& r : req) {
            if (av < n) {
                size_t k = 0;
                for (uint64_t q : r.second) {
                    if (q + r.first.first + 64 <= av) { r.second[k++] = q; continue; }
                    forget(r.first, q);
                    need = std::min<uint64_t>(need, q + r.first.first + 64);
                }
                r.second.resize(k);
                if (!k) continue;
            }
            const ambc_params* pk = r.first.second == 1 || !lzshare ? p : &po;
            if (int rc = be.check_size(pk, r.first.first)) {
                // only an error if a walk itself needs this size (not a speculative position)
                for (uint64_t q : r.second)
                    if (std::binary_search(G.active.begin(), G.active.end(), Walk{q, 0},
                                           [](const Walk& x, const Walk& y) { return x.pos < y.pos; }))
                        return rc;
                // speculative only: never decided from -- forget the requests
                for (uint64_t q : r.second) forget(r.first, q);
                continue;
            }
            jobs.emplace_back(r.first, std::move(r.second));
        }
        // (requests forgotten for the input: every walk asks its whole guess chain
        // again next round, so that its speculation resumes once the bytes are there)
        if (need != ~0ull)
            for (Walk& w : G.active) w.cs = 0;
        // the largest size first (slot 0, the high-priority stream)
        if (!cfg.noprio)
            std::stable_sort(jobs.begin(), jobs.end(), [](const Job& a, const Job& b) {
                return a.first.first != b.first.first ? a.first.first > b.first.first : a.first.second > b.first.second;
            });
        out.t_req += now_ns() - tq;
        if (!jobs.empty()) G.rounds++;
        // up to 8 batches at once, each on its own slot; more than 8: the earlier
        // ones are finished here, the last 8 fly
        const uint64_t tk = now_ns();
        // nothing to launch but requests waiting for the input: wait for it
        if (jobs.empty() && need != ~0ull && G.flight.empty())
            if (int rc = be.wait_avail(need)) return rc;
        for (size_t j0 = 0; j0 < jobs.size(); j0 += 8) {
            const size_t j1 = std::min(jobs.size(), j0 + 8);
            const uint64_t tl = now_ns();
            // the largest size first (its own high-priority stream), then the rest
            // smallest first: streams share hardware queues, and a 1 KiB batch
            // queued behind an 8 KiB Dictionary chain ended the round
            for (size_t x = 0; x < j1 - j0; x++) {
                const size_t j = cfg.launch_desc || x == 0 ? j0 + x : j1 - x;
                if (int rc = launch_job(jobs[j], G.slot0 + (int)(j - j0))) return rc;
            }
            out.t_launch += now_ns() - tl;
            if (j0 == 0)                           // the host codecs while the device works
                if (int rc = host_round()) return rc;
            if (j1 < jobs.size()) {
                for (size_t j = j0; j < j1; j++)
                    if (int rc = finish_job(jobs[j], G.slot0 + (int)(j - j0))) return rc;
            } else {
                // (the slots follow the launch positions: job j on slot0 + j - j0)
                for (size_t j = j0; j < j1; j++) G.flight.push_back(std::move(jobs[j]));
            }
        }
        if (jobs.empty())
            if (int rc = host_round()) return rc;
        out.wait_ns += now_ns() - tk;
        return AMBC_OK;
    };
    for (int gi = 0; gi < GROUPS; gi++)
        if (int rc = advance(grp[gi])) return rc;
    for (;;) {
        bool any = false;
        for (int gi = 0; gi < GROUPS; gi++) {
            Group& G = grp[gi];
            if (G.active.empty() && G.flight.empty()) continue;
            any = true;
            if (int rc = complete(G)) return rc;
            if (int rc = advance(G)) return rc;
        }
        if (!any) break;
    }
    for (int gi = 0; gi < GROUPS; gi++) out.steps = std::max(out.steps, grp[gi].rounds);

    // ---- the reference's walk from 0, read off the decisions ----
    out.path.clear();
    out.body = 0;
    uint64_t path_pos = 0;
    for (;;) {
        if (path_pos >= n) break;
        PosTable::Rec* r = T.peek(path_pos);
        if (!r || !r->decided) return fail(AMBC_E_DEVICE, "multi-size walk: undecided position on the path");
        const Decision dd = r->dec;
        if (dd.id == 255 && n - path_pos > 0xFFFFFFFFull)
            return fail(AMBC_E_RANGE, "raw remainder exceeds a u32 chunk field");
        out.path.push_back(WalkPkg{path_pos, dd.s, dd.plen, dd.id, dd.host, out.body});
        out.body += HDR + (uint64_t)dd.plen;
        if (dd.id == 255) break;
        path_pos += dd.s;
    }
    return AMBC_OK;
}

}  // namespace ambc
