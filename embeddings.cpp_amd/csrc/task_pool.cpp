#include "task_pool.h"

#include <algorithm>

namespace emb {

TaskPool &TaskPool::instance()
{
    static TaskPool pool;
    return pool;
}

TaskPool::~TaskPool()
{
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_work_.notify_all();
    for (auto &t : threads_) t.join();
}

void TaskPool::grow(int n_workers)
{
    while ((int)threads_.size() < n_workers) {
        const int idx = (int)threads_.size();
        threads_.emplace_back([this, idx] { worker(idx); });
    }
}

void TaskPool::drain()
{
    for (;;) {
        const int64_t i = next_.fetch_add(1, std::memory_order_relaxed);
        if (i >= n_tasks_) return;
        (*fn_)(i);
    }
}

void TaskPool::worker(int idx)
{
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            // a worker joins a batch only when it is enlisted (idx < active_)
            cv_work_.wait(lk, [&] { return stop_ || (gen_ != seen && idx < active_); });
            if (stop_) return;
            seen = gen_;
        }
        drain();
        std::lock_guard<std::mutex> lk(mu_);
        if (--busy_ == 0) cv_done_.notify_one();
    }
}

void TaskPool::run(int64_t n_tasks, int n_threads, const std::function<void(int64_t)> &fn)
{
    if (n_tasks <= 0) return;
    n_threads = std::max(1, std::min<int>({n_threads, kMaxThreads, (int)std::min<int64_t>(n_tasks, kMaxThreads)}));
    if (n_threads == 1) {
        for (int64_t i = 0; i < n_tasks; ++i) fn(i);
        return;
    }
    std::lock_guard<std::mutex> run_lk(run_mu_);
    const int helpers = n_threads - 1;
    {
        std::lock_guard<std::mutex> lk(mu_);
        grow(helpers);
        fn_ = &fn;
        n_tasks_ = n_tasks;
        next_.store(0, std::memory_order_relaxed);
        active_ = helpers;
        busy_ = helpers;
        ++gen_;
    }
    cv_work_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return busy_ == 0; });
    active_ = 0;
    fn_ = nullptr;
}

}  // namespace emb
