// Micro-batching TCP embedding server.
//
// The wire protocol is the reference's examples/server.cpp:26-116, unchanged, so
// examples/sample_client.py talks to it as-is: on connect the server sends the
// native int32 n_embd; then every recv() of up to 32 KiB is one UTF-8 text and
// is answered with n_embd raw float32 (zeros when the text tokenizes past the
// model's n_max_tokens: the reference's refusal leaves its zero-initialised
// output vector as it was, server.cpp:113-115).
//
// The serving model differs.  The reference accepts one client at a time
// (listen backlog 1) and runs one bert_encode per recv.  Here every connection
// has its own thread, which tokenizes its text (bert_tokenize, host) and queues
// it; one batcher thread per GPU replica of the context (bertx_num_devices) takes
// queued texts (at most --max-batch) and sends them to the GPUs as ONE
// bert_forward_batch, so each replica can have a micro-batch in flight (the
// library routes a micro-batch whole to its least-loaded replica, bert_abi.cpp
// run_forward).  A batcher's window opens with the first queued text and closes
// when the clients that are not already waiting on an in-flight batch have queued
// their share of the free batchers (ceil(waiting clients / free batchers)), or
// --wait-us after it opened, whichever comes first (so a lone client never waits
// for a batch that cannot fill).  Per-sentence results do not depend on the batch
// they ride in (tests/test_gpu_forward.py batch invariance), so every reply equals
// the single-text result.
//
// usage: server -m MODEL [--port P] [-t N] [--max-batch B] [--wait-us U]
#include "bert.h"
#include "bert_hip.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Request {
    std::vector<int32_t> ids;
    int32_t n_tokens = 0;
    std::vector<float> emb;
    bool done = false;
};

class Batcher {
public:
    Batcher(bert_ctx *ctx, int n_threads, int max_batch, int wait_us, int n_batchers)
        : ctx_(ctx), n_threads_(n_threads), max_batch_(max_batch), wait_us_(wait_us), n_batchers_(n_batchers)
    {
    }

    // connection count: the batch threshold (a batch is full when every
    // connected client has a text in it)
    void connected(int delta)
    {
        std::lock_guard<std::mutex> g(mu_);
        clients_ += delta;
        cv_in_.notify_all();   // several batchers wait on cv_in_: wake the one whose window closed
    }

    // queues r and blocks until r->emb holds its embedding
    void run(Request *r)
    {
        std::unique_lock<std::mutex> lk(mu_);
        queue_.push_back(r);
        cv_in_.notify_all();
        cv_out_.wait(lk, [&] { return r->done; });
    }

    void loop()
    {
        std::vector<Request *> batch;
        std::vector<int32_t *> toks;
        std::vector<int32_t> lens;
        std::vector<float *> outs;
        for (;;) {
            batch.clear();
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_in_.wait(lk, [&] { return !queue_.empty(); });
                // the window opens with the first queued text and closes early once
                // the clients not waiting on an in-flight batch have queued this
                // batcher's share of them
                cv_in_.wait_for(lk, std::chrono::microseconds(wait_us_), [&] {
                    const int waiting = std::max(1, clients_ - in_flight_);
                    const int free = std::max(1, n_batchers_ - busy_);
                    const int full = std::min(max_batch_, (waiting + free - 1) / free);
                    return (int)queue_.size() >= full;
                });
                while (!queue_.empty() && (int)batch.size() < max_batch_) {
                    batch.push_back(queue_.front());
                    queue_.pop_front();
                }
                if (batch.empty()) continue;   // another batcher took them
                ++busy_;
                in_flight_ += (int)batch.size();
            }
            toks.clear();
            lens.clear();
            outs.clear();
            for (Request *r : batch) {
                toks.push_back(r->ids.data());
                lens.push_back(r->n_tokens);
                outs.push_back(r->emb.data());
            }
            bert_forward_batch(ctx_, n_threads_, (int32_t)batch.size(), toks.data(), lens.data(), outs.data());
            {
                std::lock_guard<std::mutex> g(mu_);
                for (Request *r : batch) r->done = true;
                --busy_;
                in_flight_ -= (int)batch.size();
            }
            cv_out_.notify_all();
            cv_in_.notify_all();   // a waiting batcher's share changed
        }
    }

private:
    bert_ctx *ctx_;
    int n_threads_, max_batch_, wait_us_, n_batchers_;
    int clients_ = 0;
    int busy_ = 0;        // batchers with a micro-batch on the GPUs
    int in_flight_ = 0;   // texts in those micro-batches
    std::mutex mu_;
    std::condition_variable cv_in_, cv_out_;
    std::deque<Request *> queue_;
};

bool send_all(int fd, const void *p, size_t n)
{
    const char *c = (const char *)p;
    while (n) {
        const ssize_t k = send(fd, c, n, MSG_NOSIGNAL);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

void serve(int fd, bert_ctx *ctx, Batcher *b)
{
    const int32_t n_embd = bert_n_embd(ctx), n_max = bert_n_max_tokens(ctx);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    b->connected(+1);
    if (send_all(fd, &n_embd, sizeof(n_embd))) {
        std::vector<char> buf((size_t)1 << 15);      // server.cpp:27
        for (;;) {
            const ssize_t k = recv(fd, buf.data(), buf.size(), 0);
            if (k <= 0) break;
            const std::string text(buf.data(), (size_t)k);
            Request r;
            r.ids.resize((size_t)n_max);
            bert_tokenize(ctx, text.c_str(), r.ids.data(), &r.n_tokens, n_max);
            r.emb.assign((size_t)n_embd, 0.0f);
            if (r.n_tokens > 0 && r.n_tokens <= n_max) b->run(&r);
            if (!send_all(fd, r.emb.data(), r.emb.size() * sizeof(float))) break;
        }
    }
    b->connected(-1);
    close(fd);
}

}  // namespace

int main(int argc, char **argv)
{
    int max_batch = 64, wait_us = 2000;
    std::vector<char *> rest;
    for (int i = 0; i < argc; ++i) {
        if (i > 0 && i + 1 < argc && !std::strcmp(argv[i], "--max-batch")) { max_batch = std::atoi(argv[++i]); continue; }
        if (i > 0 && i + 1 < argc && !std::strcmp(argv[i], "--wait-us")) { wait_us = std::atoi(argv[++i]); continue; }
        rest.push_back(argv[i]);
    }
    bert_params params;
    if (!bert_params_parse((int)rest.size(), rest.data(), params)) return 1;
    if (max_batch < 1) max_batch = 1;
    if (wait_us < 0) wait_us = 0;

    bert_ctx *ctx = bert_load_from_file(params.model);
    if (!ctx) {
        std::fprintf(stderr, "%s: failed to load model from '%s'\n", __func__, params.model);
        return 1;
    }
    const int srv = socket(AF_INET, SOCK_STREAM, 0);
    if (srv < 0) {
        std::perror("socket");
        return 1;
    }
    int one = 1;
    setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = INADDR_ANY;
    addr.sin_port = htons((uint16_t)params.port);
    if (bind(srv, (sockaddr *)&addr, sizeof(addr)) < 0 || listen(srv, 128) < 0) {
        std::perror("bind/listen");
        return 1;
    }
    std::printf("Server running on port %d: up to %d texts per GPU batch, %d us window, %d batcher(s)\n", params.port,
                max_batch, wait_us, std::max(1, (int)bertx_num_devices(ctx)));
    std::fflush(stdout);
    // one batcher (one micro-batch in flight) per GPU replica of the context
    const int n_batchers = std::max(1, (int)bertx_num_devices(ctx));
    Batcher batcher(ctx, params.n_threads, max_batch, wait_us, n_batchers);
    for (int i = 0; i < n_batchers; ++i) std::thread(&Batcher::loop, &batcher).detach();
    for (;;) {
        const int fd = accept(srv, nullptr, nullptr);
        if (fd < 0) {
            if (errno == EINTR || errno == ECONNABORTED) continue;
            std::perror("accept");
            return 1;
        }
        std::thread(serve, fd, ctx, &batcher).detach();
    }
}
