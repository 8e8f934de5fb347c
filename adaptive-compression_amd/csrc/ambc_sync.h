// ambc_sync.h -- the host-side synchronisation of libambc_hip, kept free of HIP
// and RCCL types so that tests/native/sync_harness.cpp can drive the same code on
// the CPU under ThreadSanitizer and AddressSanitizer ("race
// detection"):
//
//   * WalkPool  -- the multi-size walk's spinning worker pool (ambc_multisize.cpp)
//   * Hub       -- the barrier of the host-memory transport (shards that share a
//                  device, ambc_shard.cpp's LocalTransport)
//   * AbortGate -- in-process RCCL ranks: enqueuers never wait on each other, and a
//                  failed rank's abort waits only for enqueues in progress, never
//                  for a collective (ambc_shard.cpp's RcclTransport)
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

namespace ambc {

// A few host threads for the walk's per-round host work (filling a batch's results
// into the position table, deciding every walk's steps): between two rounds the
// device waits for them (~1 ms a round for a thousand walks on one thread).  The
// workers spin briefly between tasks (the rounds come every few ms), then sleep.
// AMBC_MS_THREADS sets the process pool's count (1: all on the calling thread; 10
// by default where the host has the cores: {1,3,4,9} walk 40.2-41.4 -> 38.4 ms
// against 6, profiles/r4_walk_threads_ab3).  One task at a time: run() from
// several threads (walks on several devices of one process) take turns.
class WalkPool {
  public:
    static WalkPool& get() {
        static WalkPool pool(default_threads());
        return pool;
    }
    static unsigned default_threads() {
        const char* e = getenv("AMBC_MS_THREADS");
        return e ? (unsigned)std::max(1, atoi(e))
                 : std::min(10u, std::max(1u, std::thread::hardware_concurrency() / 2));
    }
    explicit WalkPool(unsigned T) {
        for (unsigned t = 1; t < T; t++) workers_.emplace_back([this, t] { loop(t); });
        pid_ = getpid();
    }
    WalkPool(const WalkPool&) = delete;
    WalkPool& operator=(const WalkPool&) = delete;
    unsigned size() const { return (unsigned)workers_.size() + 1; }
    // fn(t, T) for t in [0, T), T = size(); the caller runs t = 0
    void run(const std::function<void(unsigned, unsigned)>& fn) {
        const unsigned T = size();
        if (T == 1) { fn(0, 1); return; }
        if (getpid() != pid_) {   // a forked child has no workers: every slice here
            for (unsigned t = 0; t < T; t++) fn(t, T);
            return;
        }
        std::lock_guard<std::mutex> serial(run_mu_);   // one task at a time
        {
            std::lock_guard<std::mutex> g(mu_);
            task_ = &fn;
            pending_.store(T - 1);
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        fn(0, T);
        while (pending_.load() != 0) std::this_thread::yield();
        std::lock_guard<std::mutex> g(mu_);
        task_ = nullptr;
    }
    ~WalkPool() {
        if (getpid() != pid_) {   // (a forked child: the threads are the parent's; leave them be)
            new std::vector<std::thread>(std::move(workers_));
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true);
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void loop(unsigned t) {
        uint64_t seen = 0;
        for (;;) {
            // spin up to ~2 ms for the next task, then sleep on the condition variable
            const auto t0 = std::chrono::steady_clock::now();
            while (gen_.load() == seen && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2))
                std::this_thread::yield();
            const std::function<void(unsigned, unsigned)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_.load() != seen; });
                seen = gen_.load();
                if (stop_.load()) return;
                f = task_;
            }
            if (f) (*f)(t, size());
            pending_.fetch_sub(1);
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<unsigned> pending_{0};
    const std::function<void(unsigned, unsigned)>* task_ = nullptr;   // (under mu_)
    std::atomic<bool> stop_{false};
    pid_t pid_ = 0;
};

// W host threads meeting at a barrier; a failed thread releases every waiter
struct Hub {
    explicit Hub(int w) : W(w), vals(w), srcs(w, nullptr) {}
    std::mutex m;
    std::condition_variable cv;
    int W, arrived = 0;
    uint64_t gen = 0;
    bool failed = false;
    std::vector<std::vector<uint64_t>> vals;   // rank q writes vals[q] before wait(), reads all after
    std::vector<const uint8_t*> srcs;
    // false when some rank failed (every waiter returns)
    bool wait() {
        std::unique_lock<std::mutex> lk(m);
        if (failed) return false;
        const uint64_t g = gen;
        if (++arrived == W) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != g || failed; });
        return !failed;
    }
    void fail() {
        std::lock_guard<std::mutex> lk(m);
        failed = true;
        cv.notify_all();
    }
};

// In-process ranks enqueue collectives on their own communicators concurrently;
// a failed rank must abort every communicator of the group (that is what releases
// peers whose kernels wait for it), but never while another rank is inside an
// enqueue call on one of them.  The rule: no lock spans an enqueue.  An enqueuer
// counts itself in (`enter`), checks the abort flag, enqueues, counts itself out;
// the aborter raises the flag, waits until no enqueue is in progress, then aborts.
// (seq_cst on both sides: an enqueuer that saw the flag down is seen by the
// aborter's count.)  An enqueue returns without waiting for peers because the
// communicators are connected eagerly when they are created -- every collective
// kind at every size the calls use, and the gather's Send / Recv at its piece
// size (ambc_shard.cpp, connect_group) -- so the aborter's wait is short.  It is
// bounded all the same (AMBC_ABORT_WAIT_MS, default 20 s): an enqueue still
// inside its call by then is stuck on a peer that will never join, and only the
// abort can release it, so kill() runs anyway (abort() then returns false).
struct AbortGate {
    std::atomic<int> inflight{0};
    std::atomic<bool> aborted{false};
    std::mutex abort_mu;   // aborters only (one abort sequence runs)
    // true: the caller may enqueue and must call leave() afterwards
    bool enter() {
        inflight.fetch_add(1);
        if (aborted.load()) { inflight.fetch_sub(1); return false; }
        return true;
    }
    void leave() { inflight.fetch_sub(1); }
    static uint64_t default_wait_ms() {
        const char* e = getenv("AMBC_ABORT_WAIT_MS");
        return e && *e ? strtoull(e, nullptr, 10) : 20000;
    }
    // kill() runs once, after every enqueue in progress has left or after wait_ms
    // (false: it ran with an enqueue still inside); later enter()s fail
    template <typename F>
    bool abort(F&& kill, uint64_t wait_ms = default_wait_ms()) {
        std::lock_guard<std::mutex> g(abort_mu);
        if (aborted.exchange(true)) return true;
        const auto t0 = std::chrono::steady_clock::now();
        bool clean = true;
        while (inflight.load() != 0) {
            if (std::chrono::steady_clock::now() - t0 >= std::chrono::milliseconds(wait_ms)) { clean = false; break; }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        kill();
        return clean;
    }
    void reset() { aborted.store(false); }   // a fresh group (no rank thread running)
};

}  // namespace ambc
