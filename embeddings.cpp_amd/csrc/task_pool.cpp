#include "task_pool.h"

#include <algorithm>
#include <pthread.h>

namespace emb {

TaskPool &TaskPool::instance()
{
    static TaskPool pool;
    return pool;
}

TaskPool::TaskPool()
{
    // fork safety: no batch may be in flight across a fork (prepare takes both
    // locks, so a fork waits for a running batch); the child has none of the
    // parent's workers, so it drops their handles (leaked on purpose: joining or
    // destroying a std::thread of another process is undefined) and starts its
    // own on demand
    pthread_atfork([] { instance().before_fork(); }, [] { instance().after_fork(false); },
                   [] { instance().after_fork(true); });
}

void TaskPool::before_fork()
{
    run_mu_.lock();
    mu_.lock();
}

void TaskPool::after_fork(bool child)
{
    if (child) {
        if (!threads_.empty()) new std::vector<std::thread>(std::move(threads_));   // never joined, never freed
        threads_.clear();
        active_ = busy_ = 0;
        fn_ = nullptr;
        error_ = nullptr;
    }
    mu_.unlock();
    run_mu_.unlock();
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
        try {
            (*fn_)(i);
        } catch (...) {
            // the first exception of the batch is kept for run() to rethrow; the
            // remaining tasks are abandoned (no thread dies with it)
            std::lock_guard<std::mutex> lk(mu_);
            if (!error_) error_ = std::current_exception();
            next_.store(n_tasks_, std::memory_order_relaxed);
        }
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
        error_ = nullptr;
        ++gen_;
    }
    cv_work_.notify_all();
    drain();
    std::exception_ptr err;
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return busy_ == 0; });
        active_ = 0;
        fn_ = nullptr;
        err = error_;
        error_ = nullptr;
    }
    if (err) std::rethrow_exception(err);
}

}  // namespace emb
