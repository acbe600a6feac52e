// pool.h — the front-end's worker threads (rav1d's tile / frame worker threads,
// thread_task.rs): started once per decoder, shared by every frame in flight.
//
// run(n, fn) calls fn(0..n-1) on the calling thread and on free workers and returns when all
// calls have returned; batches of several frames queue in submission order, and the caller
// always takes tasks of its own batch, so a batch completes even with every worker busy. A
// worker that runs out of tasks spins briefly before sleeping: a frame's tile batches follow
// each other within a fraction of a millisecond, and waking a sleeping thread costs as much.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace av1 {

class WorkerPool {
public:
    explicit WorkerPool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
    }
    WorkerPool(const WorkerPool &) = delete;
    WorkerPool &operator=(const WorkerPool &) = delete;
    int workers() const { return (int)th_.size(); }

    // fn(i) for every i in [0, n); the first exception is rethrown here once all calls ended
    void run(int n, const std::function<void(int)> &fn) {
        if (n <= 0) return;
        Batch b;
        b.fn = &fn;
        b.n = n;
        if (n > 1 && !th_.empty()) {
            {
                std::lock_guard<std::mutex> g(m_);
                q_.push_back(&b);
                queued_.fetch_add(1, std::memory_order_release);
            }
            if (n - 1 >= (int)th_.size()) cv_.notify_all();
            else
                for (int i = 0; i < n - 1; i++) cv_.notify_one();
        }
        take(b);
        if (n > 1 && !th_.empty()) {
            {
                std::lock_guard<std::mutex> g(m_);
                unqueue(&b);
            }
            // workers that picked the batch may still be inside fn
            while (b.users.load(std::memory_order_acquire) || b.done.load(std::memory_order_acquire) < n)
                std::this_thread::yield();
        }
        if (b.ex) std::rethrow_exception(b.ex);
    }

private:
    struct Batch {
        const std::function<void(int)> *fn = nullptr;
        int n = 0;
        std::atomic<int> next{0}, done{0}, users{0};
        std::mutex exm;
        std::exception_ptr ex;
    };

    // run tasks of b until none is left
    static void take(Batch &b) {
        for (int i; (i = b.next.fetch_add(1, std::memory_order_relaxed)) < b.n;) {
            try {
                (*b.fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> g(b.exm);
                if (!b.ex) b.ex = std::current_exception();
            }
            b.done.fetch_add(1, std::memory_order_release);
        }
    }
    // (m_ held)
    void unqueue(Batch *b) {
        for (auto it = q_.begin(); it != q_.end(); ++it)
            if (*it == b) {
                q_.erase(it);
                queued_.fetch_sub(1, std::memory_order_release);
                return;
            }
    }
    // (m_ held) the oldest batch with tasks left, marked as used by this worker
    Batch *pick() {
        while (!q_.empty()) {
            Batch *b = q_.front();
            if (b->next.load(std::memory_order_relaxed) < b->n) {
                b->users.fetch_add(1, std::memory_order_acq_rel);
                return b;
            }
            q_.pop_front();   // exhausted: its caller finds it gone
            queued_.fetch_sub(1, std::memory_order_release);
        }
        return nullptr;
    }
    void loop() {
        using clk = std::chrono::steady_clock;
        for (;;) {
            // spin a little before sleeping (see above)
            const auto until = clk::now() + std::chrono::microseconds(300);
            while (!queued_.load(std::memory_order_acquire) && !stop_.load(std::memory_order_relaxed) &&
                   clk::now() < until)
                for (int k = 0; k < 64; k++) __builtin_ia32_pause();
            Batch *b;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || (b = pick()) != nullptr; });
                if (stop_) return;
            }
            take(*b);
            b->users.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Batch *> q_;
    std::atomic<int> queued_{0};
    std::atomic<bool> stop_{false};   // (set under m_, read by the spinning workers without it)
};

}  // namespace av1
