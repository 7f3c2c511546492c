// Persistent host worker pool (tokenization of bert_encode_batch, bert.cpp:1402-1406
// runs it on one thread; here it runs on n_threads).  Workers are started once
// and parked on a condition variable between batches, so a call costs a wake-up
// instead of n thread creations; tasks are claimed dynamically (an atomic
// counter), the calling thread works too, and run() returns when every task is
// done.  One batch at a time: concurrent callers queue on the pool's mutex.  A
// task that throws ends the batch and run() rethrows the first exception in the
// caller; a forked child gets a fresh pool (pthread_atfork).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace emb {

class TaskPool {
public:
    static TaskPool &instance();
    ~TaskPool();

    // fn(i) for every i in [0, n_tasks) on up to n_threads threads (the caller
    // included); blocks until all are done, then rethrows a task's exception.
    void run(int64_t n_tasks, int n_threads, const std::function<void(int64_t)> &fn);

    static constexpr int kMaxThreads = 256;

private:
    TaskPool();
    void before_fork();
    void after_fork(bool child);
    void grow(int n_workers);
    void worker(int idx);
    void drain();

    std::mutex run_mu_;                    // one batch at a time
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::vector<std::thread> threads_;
    const std::function<void(int64_t)> *fn_ = nullptr;
    int64_t n_tasks_ = 0;
    std::atomic<int64_t> next_{0};
    int active_ = 0;                       // workers enlisted in the current batch
    int busy_ = 0;                         // enlisted workers not yet finished
    uint64_t gen_ = 0;                     // batch generation (wakes parked workers)
    bool stop_ = false;
    std::exception_ptr error_;             // first exception thrown by a task of the batch
};

}  // namespace emb
