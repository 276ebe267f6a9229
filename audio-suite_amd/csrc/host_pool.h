// host_pool.h — the host worker pool of msg_render_batch (plan.h and the
// runtime records on the CPU).  Header-only so the host-sanitizer builds
// (host_san.cpp, tests/host_pool_tsan.cpp under ThreadSanitizer) compile the
// same code the product library runs.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <sched.h>
#include <thread>
#include <vector>

// Host worker pool for the per-preset planning of a batch (plan.h on the CPU).
// One process-wide pool that runs several callers' jobs at once: each caller
// (one render per context/stream) queues its job, takes part in it, and idle
// workers share out the oldest unfinished job, so three contexts planning
// concurrently keep every worker busy instead of two of them running inline.
// Size: MSGPU_HOST_THREADS, else the process's CPU affinity divided among the
// ranks of the node (LOCAL_WORLD_SIZE), at most 16 (one
// host pool per GPU).  Idle workers spin briefly before sleeping (a batch makes
// five pool calls; a condition-variable wake per call cost ~10-50 us).
class HostPool {
  public:
    static HostPool& get() {
        static HostPool pool;
        return pool;
    }
    int threads() const { return (int)workers_.size() + 1; }
    template <class F>
    void run(int count, F&& f) {
        if (count <= 0) return;
        if (workers_.empty() || count < 2) {
            for (int i = 0; i < count; ++i) f(i);
            return;
        }
        std::function<void(int)> fn(std::ref(f));
        Job job;
        job.fn = &fn;
        job.count = count;
        // items are claimed in chunks (about four per thread): per-item claims on
        // one counter cost more than a 0.3 us item (plan_sizes) under 16 threads
        job.chunk = std::max(1, count / (4 * threads()));
        {
            std::lock_guard<std::mutex> lk(m_);
            jobs_.push_back(&job);
            pending_.fetch_add(1);
        }
        cv_.notify_all();
        drain(job);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return job.done.load() == count && job.users == 0; });
        auto it = std::find(jobs_.begin(), jobs_.end(), &job);
        if (it != jobs_.end()) { jobs_.erase(it); pending_.fetch_sub(1); }
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int count = 0, chunk = 1;
        std::atomic<int> next{0}, done{0};
        int users = 0;                      // workers attached (under m_)
    };
    static int default_threads() {
        if (const char* e = getenv("MSGPU_HOST_THREADS")) return std::max(1, atoi(e));
        int cpus = 0;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        if (cpus <= 0) cpus = (int)std::thread::hardware_concurrency();
        int ranks = 1;
        if (const char* e = getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, atoi(e));
        return std::max(1, std::min(16, cpus / ranks));
    }
    HostPool() {
        const int n = default_threads();
        for (int i = 0; i + 1 < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    static void drain(Job& j) {
        const int c = j.chunk;
        for (int i0 = j.next.fetch_add(c); i0 < j.count; i0 = j.next.fetch_add(c)) {
            const int i1 = std::min(i0 + c, j.count);
            for (int i = i0; i < i1; ++i) (*j.fn)(i);
            j.done.fetch_add(i1 - i0);
        }
    }
    void loop() {
        for (;;) {
            for (int spin = 0; spin < 4000 && pending_.load(std::memory_order_relaxed) == 0; ++spin)
                __builtin_ia32_pause();
            Job* j = nullptr;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
                if (stop_) return;
                while (!jobs_.empty() && jobs_.front()->next.load() >= jobs_.front()->count) {
                    jobs_.pop_front();          // exhausted: its caller waits only for the attached workers
                    pending_.fetch_sub(1);
                }
                if (jobs_.empty()) continue;
                j = jobs_.front();
                ++j->users;
            }
            drain(*j);
            std::lock_guard<std::mutex> lk(m_);
            if (--j->users == 0 && j->done.load() == j->count) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job*> jobs_;
    std::atomic<int> pending_{0};
    bool stop_ = false;
};

