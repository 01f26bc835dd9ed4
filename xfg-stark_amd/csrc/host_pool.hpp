// Process-wide pool of host threads for the per-proof host work of a proof unit (transcript replay,
// grinding and opening plans, serialisation, copy-out). The lane workers (prover.hip) run up to
// XFG_LANES units' host tails at once, each a loop over 8-64 independent proofs that used to run on
// the lane's own thread while its stream waited; parallel_for spreads such a loop over the pool.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace xfg {

class HostPool {
    struct Task {
        const std::function<void(int)>* fn = nullptr;
        int count = 0;
        int users = 0;  // pool threads inside work(), guarded by the pool mutex
        std::atomic<int> next{0}, done{0};
        std::mutex em;
        std::exception_ptr err;
    };
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<Task*> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;

    static void work(Task* t) {
        int i;
        while ((i = t->next.fetch_add(1)) < t->count) {
            try {
                (*t->fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> g(t->em);
                if (!t->err) t->err = std::current_exception();
            }
            t->done.fetch_add(1);
        }
    }
    void worker() {
        std::unique_lock<std::mutex> g(m_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (stop_) return;
            Task* t = q_.front();
            if (t->next.load() >= t->count) {  // every index claimed: the task leaves the queue
                q_.pop_front();
                continue;
            }
            t->users++;
            g.unlock();
            work(t);
            g.lock();
            if (--t->users == 0) done_cv_.notify_all();
        }
    }

   public:
    explicit HostPool(int n) {
        for (int k = 0; k < n; k++) th_.emplace_back([this] { worker(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // fn(0) .. fn(count - 1) on the calling thread and the pool, in any order; returns when every
    // call has returned and rethrows the first exception one of them threw
    void parallel_for(int count, const std::function<void(int)>& fn) {
        if (count <= 0) return;
        if (count == 1 || th_.empty()) {
            for (int i = 0; i < count; i++) fn(i);
            return;
        }
        Task t;
        t.fn = &fn;
        t.count = count;
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(&t);
        }
        cv_.notify_all();
        work(&t);
        std::unique_lock<std::mutex> g(m_);
        auto it = std::find(q_.begin(), q_.end(), &t);
        if (it != q_.end()) q_.erase(it);
        done_cv_.wait(g, [&] { return t.users == 0 && t.done.load() == count; });
        if (t.err) std::rethrow_exception(t.err);
    }
};

// XFG_HOST_THREADS (default 8; 0 = every loop on the calling lane worker, as before the pool).
// Never destroyed: lane workers of a context the process did not close may still use it while
// static destructors run at exit; its idle threads end with the process.
static inline HostPool& host_pool() {
    static HostPool* pool = new HostPool([] {
        const char* v = getenv("XFG_HOST_THREADS");
        return std::max(0, v && *v ? atoi(v) : 8);
    }());
    return *pool;
}

}  // namespace xfg
