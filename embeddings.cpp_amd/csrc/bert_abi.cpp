// The drop-in C ABI (include/bert.h, reference bert.h:18-90) and the MI355X
// extensions (include/bert_hip.h): context lifetime, tokenization, batching,
// multi-GPU sharding of encode calls.  No CPU compute path: every forward runs
// on the HIP kernels, and fails loudly when no device is present.
#include "bert.h"
#include "bert_hip.h"
#include "ggml.h"

#include "engine.h"
#include "task_pool.h"
#include "tokenizer.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

using emb::Device;

namespace {

// A persistent host thread per replica (multi-replica contexts): run_forward posts
// a replica's share of a call to it instead of creating a std::thread per call.
class ReplicaWorker {
public:
    ReplicaWorker() : th_([this] { loop(); }) {}
    ~ReplicaWorker()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    void post(std::function<void()> f)
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    void loop()
    {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;   // stop_ with nothing queued
                f = std::move(q_.front());
                q_.pop_front();
            }
            // nothing may leave the worker thread (std::terminate); run_forward's
            // tasks catch their own failures, this is the last line
            try { f(); } catch (...) { emb::errorf("libbert: replica worker task failed\n"); }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace

struct bert_ctx {
    emb::HParams hp;
    emb::Vocab vocab;
    std::vector<std::unique_ptr<Device>> devices;
    bool host_only = false;
    // routing state of run_forward: the cost of the work routed to each replica and
    // not yet finished, and the rotation that breaks ties between equal loads
    std::mutex route_mu;
    std::vector<double> inflight;
    unsigned rr = 0;
    // declared after `devices`: destroyed (joined) before the replicas they drive
    std::vector<std::unique_ptr<ReplicaWorker>> workers;
};

namespace {

constexpr int64_t kChunkTokens = 1 << 17;   // tokens per device forward (workspace bound)
constexpr int kChunkSeqs = 4096;            // sentences per device forward (pool / output staging bound)
// A call is split only over replicas that are idle (no routed work in flight), and
// only while each share keeps at least kMinShareTokens.  The choice, from the
// measured per-share latency on one replica (scripts/share_curve.py,
// profiles/r05_share_curve.jsonl: bge-base q4_0, 128-token sentences through
// bert_forward_batch): the cost per token is 4.7x the large-batch asymptote at 128
// tokens, 1.8x at 4,096, 1.26x at 8,192 and 1.07x at 16,384.  The curve's own knee
// criterion (within 1.25x of the asymptote) gives 16,384; 8,192 is the smallest
// share for which a 2-way split still pays: a 16,384-token call takes 3.63 ms on one
// replica and 2.14 ms as two 8,192-token shares, while at 4,096 tokens per share
// (1.52 ms) the two half-size forwards buy 0.6 ms for a whole second replica.  A
// call that finds no idle replica goes whole to the least-loaded one, so concurrent
// callers (the server's batchers) land on different replicas instead of all
// splitting over all of them in lockstep.
constexpr int64_t kMinShareTokens = 8192;

std::vector<int> parse_device_list(int n_visible)
{
    std::vector<int> out;
    const char *env = std::getenv("BERT_DEVICES");
    if (!env || !*env) {
        for (int i = 0; i < n_visible; ++i) out.push_back(i);
        return out;
    }
    std::string s(env);
    size_t p = 0;
    while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        const std::string tok = s.substr(p, q - p);
        if (!tok.empty()) {
            const int v = std::atoi(tok.c_str());
            // a repeated ordinal is a second replica (own stream + workspace) on that device
            if (v >= 0 && v < n_visible) out.push_back(v);
        }
        p = q + 1;
    }
    return out;
}

// FLOP-proportional cost of one sentence of length L (GEMMs + attention).
double sentence_cost(const emb::HParams &hp, int L)
{
    const double d = hp.n_embd, f = hp.n_intermediate;
    return (double)L * (8.0 * d * d + 4.0 * d * f) + 4.0 * (double)L * L * d;
}

// Runs n sentences on the context's GPUs.  Routing (kMinShareTokens): the call
// uses k = min(idle replicas, sentences, tokens / kMinShareTokens) (at least 1)
// replicas, the k least-loaded by the cost still in flight on them (ties rotate,
// so consecutive small calls spread over the replicas too); its sentences are split over those k
// by cost, longest first to the least-loaded share (LPT).  Each replica walks its
// sentences in chunks of <= kChunkTokens on its persistent worker thread (the
// caller runs one share itself).  Results are independent of the routing and the
// split: every kernel computes a sentence from its own tokens only.
int run_forward(bert_ctx *ctx, const int32_t *const *toks, const int32_t *lens, float *const *outs, int n)
{
    if (ctx->devices.empty()) {
        emb::errorf("libbert: no HIP device in this context (BERT_HOST_ONLY); forward unavailable\n");
        return -1;
    }
    if (n <= 0) return 0;
    const int nd = (int)ctx->devices.size();
    std::vector<int> order((size_t)n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lens[a] > lens[b]; });
    int64_t tokens = 0;
    for (int i = 0; i < n; ++i) tokens += lens[i];
    std::vector<std::vector<int>> assign((size_t)nd);
    std::vector<double> load((size_t)nd, 0.0);
    std::vector<int> chosen((size_t)nd);
    {
        std::lock_guard<std::mutex> lk(ctx->route_mu);
        int64_t idle = 0;
        for (double w : ctx->inflight) idle += w == 0.0 ? 1 : 0;
        const int k = (int)std::max<int64_t>(1, std::min<int64_t>({idle, (int64_t)n, tokens / kMinShareTokens}));
        std::iota(chosen.begin(), chosen.end(), 0);
        const unsigned rot = ctx->rr;
        std::stable_sort(chosen.begin(), chosen.end(), [&](int a, int b) {
            if (ctx->inflight[(size_t)a] != ctx->inflight[(size_t)b]) return ctx->inflight[(size_t)a] < ctx->inflight[(size_t)b];
            return (unsigned)(a - (int)rot + nd) % nd < (unsigned)(b - (int)rot + nd) % nd;
        });
        chosen.resize((size_t)k);
        ctx->rr = (rot + (unsigned)k) % (unsigned)nd;
        for (int idx : order) {
            int best = chosen[0];
            for (int dv : chosen) if (load[(size_t)dv] < load[(size_t)best]) best = dv;
            assign[(size_t)best].push_back(idx);
            load[(size_t)best] += sentence_cost(ctx->hp, lens[idx]);
        }
        for (int dv : chosen) ctx->inflight[(size_t)dv] += load[(size_t)dv];
    }
    std::vector<int> rcs((size_t)nd, 0);
    auto work = [&](int dv) {
        Device &D = *ctx->devices[(size_t)dv];
        std::lock_guard<std::mutex> lk(D.mutex());
        const std::vector<int> &mine = assign[(size_t)dv];
        const auto t0 = std::chrono::steady_clock::now();
        int64_t toks_done = 0;
        struct Stamp {   // this call's share of the device: wall time, sentences, tokens
            Device &D; const std::chrono::steady_clock::time_point &t0; const std::vector<int> &mine; int64_t &toks;
            ~Stamp()
            {
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                D.set_last_call(ms, (int)mine.size(), toks);
            }
        } stamp{D, t0, mine, toks_done};
        std::vector<const int32_t *> tp;
        std::vector<int32_t> lp;
        std::vector<float *> op;
        size_t i = 0;
        while (i < mine.size()) {
            tp.clear(); lp.clear(); op.clear();
            int64_t tok = 0;
            while (i < mine.size() && (tp.empty() || (tok + lens[mine[i]] <= kChunkTokens &&
                                                       (int)tp.size() < kChunkSeqs))) {
                const int idx = mine[i++];
                tp.push_back(toks[idx]); lp.push_back(lens[idx]); op.push_back(outs[idx]);
                tok += lens[idx];
            }
            const int rc = D.forward_host(tp.data(), lp.data(), (int)tp.size(), op.data());
            if (rc != 0) { rcs[(size_t)dv] = rc; return; }
            toks_done += tok;
        }
    };
    auto finish = [&](int dv) {
        std::lock_guard<std::mutex> lk(ctx->route_mu);
        ctx->inflight[(size_t)dv] -= load[(size_t)dv];
        if (ctx->inflight[(size_t)dv] < 0.5) ctx->inflight[(size_t)dv] = 0.0;   // idle again (no float drift)
    };
    // One share, exception-safe: a failure (bad_alloc staging the chunk, a throwing
    // forward) becomes that share's rc, and `finish` always runs, so the replica
    // counts as idle again and no task outlives this frame with an exception.
    auto run_share = [&](int dv) noexcept {
        try {
            work(dv);
        } catch (const std::exception &ex) {
            emb::errorf("libbert: replica %d share failed: %s\n", dv, ex.what());
            rcs[(size_t)dv] = -1;
        } catch (...) {
            emb::errorf("libbert: replica %d share failed\n", dv);
            rcs[(size_t)dv] = -1;
        }
        finish(dv);
    };
    std::vector<int> used;
    for (int dv : chosen) if (!assign[(size_t)dv].empty()) used.push_back(dv);
    if (used.size() <= 1 || ctx->workers.size() != (size_t)nd) {
        for (int dv : used) run_share(dv);
    } else {
        // the other shares on their replicas' persistent workers, the first on this
        // thread; `left` counts only the tasks actually posted (a post that throws
        // runs its share here), and this frame outlives every posted task
        std::mutex mu;
        std::condition_variable cv;
        size_t left = 0;
        for (size_t i = 1; i < used.size(); ++i) {
            const int dv = used[i];
            {
                std::lock_guard<std::mutex> lk(mu);
                ++left;
            }
            try {
                ctx->workers[(size_t)dv]->post([&, dv] {
                    run_share(dv);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--left == 0) cv.notify_one();
                });
            } catch (...) {
                {
                    std::lock_guard<std::mutex> lk(mu);
                    --left;
                }
                run_share(dv);
            }
        }
        run_share(used[0]);
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
    for (int rc : rcs) if (rc != 0) {
        emb::errorf("libbert: forward failed (%d)\n", rc);
        return rc;
    }
    return 0;
}

// Tokenize n texts into ids[i * n_max ..] (lens[i] = bert_tokenize's count, which
// may exceed n_max: bert.cpp:386-387) on up to n_threads threads of the persistent
// pool; the stage bert_encode_batch runs first (bert.cpp:1402-1406, sequential in
// the reference).  Blocks of 8 texts per task.  False (after a message) when a
// task threw (e.g. bad_alloc growing a scratch buffer): nothing may unwind out of
// the C ABI, and the caller leaves its outputs untouched, as on every refusal.
bool tokenize_all(const bert_ctx *ctx, int n_threads, int n, const char *const *texts, int32_t n_max, int32_t *ids,
                  int32_t *lens)
{
    const int64_t n_blocks = ((int64_t)n + 7) / 8;
    try {
        emb::TaskPool::instance().run(n_blocks, n_threads, [&](int64_t blk) {
            const int e = (int)std::min<int64_t>(n, 8 * blk + 8);
            for (int i = (int)(8 * blk); i < e; ++i)
                lens[i] = ctx->vocab.tokenize(texts[i], n_max, ids + (size_t)i * n_max, n_max);
        });
    } catch (const std::exception &ex) {
        emb::errorf("libbert: tokenization failed: %s\n", ex.what());
        return false;
    } catch (...) {
        emb::errorf("libbert: tokenization failed\n");
        return false;
    }
    return true;
}

void print_usage(char **argv, const bert_params &p)
{
    std::fprintf(stderr, "usage: %s [options]\n\noptions:\n", argv[0]);
    std::fprintf(stderr, "  -h, --help            show this help message and exit\n");
    std::fprintf(stderr, "  -t N, --threads N     host threads (tokenizer pool) (default: %d)\n", p.n_threads);
    std::fprintf(stderr, "  -p PROMPT, --prompt PROMPT\n                        prompt text (default: %s)\n", p.prompt);
    std::fprintf(stderr, "  --port p              port to bind in server mode (default: %d)\n", p.port);
    std::fprintf(stderr, "  -m FNAME, --model FNAME\n                        model path (default: %s)\n", p.model);
    std::fprintf(stderr, "  environment: BERT_DEVICES=0,1,... (GPUs to use), BERT_HOST_ONLY=1\n\n");
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// ggml time shims (examples/main.cpp, test_batch_encode.cpp call these)
// ---------------------------------------------------------------------------
static std::chrono::steady_clock::time_point g_t0 = std::chrono::steady_clock::now();
void ggml_time_init(void) { g_t0 = std::chrono::steady_clock::now(); }
int64_t ggml_time_us(void)
{
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - g_t0).count();
}
int64_t ggml_time_ms(void) { return ggml_time_us() / 1000; }

// ---------------------------------------------------------------------------
// bert.h
// ---------------------------------------------------------------------------

bool bert_params_parse(int argc, char **argv, bert_params &params)
{
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has_val = i + 1 < argc;
        if ((a == "-t" || a == "--threads") && has_val) params.n_threads = std::stoi(argv[++i]);
        else if ((a == "-p" || a == "--prompt") && has_val) params.prompt = argv[++i];
        else if (a == "--port" && has_val) params.port = std::stoi(argv[++i]);
        else if ((a == "-m" || a == "--model") && has_val) params.model = argv[++i];
        else if (a == "-h" || a == "--help") { print_usage(argv, params); std::exit(0); }
        else {
            std::fprintf(stderr, "error: unknown argument: %s\n", a.c_str());
            print_usage(argv, params);
            std::exit(0);
        }
    }
    return true;
}

// The reference's loader reports and returns nullptr on every failure
// (bert.cpp:423-443, 684-750); so does this one: nothing thrown inside (a
// bad_alloc of the host repack, a std::system_error starting a worker thread)
// leaves the C ABI, and every partly built replica is released on the way out.
// All HIP calls of the load run on this thread, one replica after another; the
// weight uploads still overlap (async copies from one page-locked image on each
// replica's stream).  DESIGN §11 has the round-5 abort this replaces.
static bert_ctx *load_context(const char *fname)
{
    emb::infof("bert_load_from_file: loading model from '%s' - please wait ...\n", fname);
    if (emb::fault_inject("load")) throw std::runtime_error("BERT_FAULT_INJECT=load");
    emb::HostModel m;
    std::string err;
    if (!emb::load_model_file(fname, m, err, true)) {
        emb::errorf("bert_load_from_file: %s\n", err.c_str());
        return nullptr;
    }
    // declared before ctx: on a failure the replicas (ctx) are released first, and
    // each waits for its upload from the page-locked image before the image goes
    emb::ModelImage img;
    std::unique_ptr<bert_ctx> ctx(new bert_ctx);
    ctx->hp = m.hp;
    ctx->vocab.build(m.vocab);
    const char *ho = std::getenv("BERT_HOST_ONLY");
    const bool host_only = ho && *ho && std::strcmp(ho, "0") != 0;
    if (host_only) {
        ctx->host_only = true;
        emb::infof("bert_load_from_file: host-only context (tokenizer only, no forward)\n");
        return ctx.release();
    }
    const std::vector<int> devs = parse_device_list(emb::hip_device_count());
    // the host half of the load, once for all replicas: repack into one image
    if (!emb::build_model_image(m, img, err, !devs.empty())) {
        emb::errorf("bert_load_from_file: %s\n", err.c_str());
        return nullptr;
    }
    emb::trace("bert_load_from_file: '%s': image %zu bytes (%s), %zu replica(s)\n", fname, img.total,
               img.pinned() ? "page-locked" : "pageable", devs.size());
    { emb::HostModel none; std::swap(m.layers, none.layers); }   // the file tensors are no longer needed
    if (devs.empty()) {
        emb::errorf("bert_load_from_file: no HIP (gfx950) device available -- libbert.so has no CPU "
                    "compute path (set BERT_HOST_ONLY=1 for a tokenizer-only context)\n");
        return nullptr;
    }
    ctx->devices.reserve(devs.size());
    for (size_t i = 0; i < devs.size(); ++i) {
        if (devs.size() > 1) emb::trace("bert_load_from_file: replica %zu on device %d: create + upload\n", i, devs[i]);
        if (i == 1 && emb::fault_inject("replica1")) throw std::runtime_error("BERT_FAULT_INJECT=replica1");
        std::unique_ptr<Device> d(new Device(devs[i], img));   // owned before anything else can throw
        ctx->devices.push_back(std::move(d));
    }
    bool ok = true;
    for (auto &d : ctx->devices) {
        if (!d->finish_load()) {
            emb::errorf("bert_load_from_file: device %d initialisation failed\n", d->ordinal());
            ok = false;
        }
    }
    if (!ok) return nullptr;
    emb::trace("bert_load_from_file: %zu replica(s) uploaded\n", ctx->devices.size());
    ctx->inflight.assign(ctx->devices.size(), 0.0);
    if (ctx->devices.size() > 1) {
        if (emb::fault_inject("worker")) throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again), "BERT_FAULT_INJECT=worker");
        ctx->workers.reserve(ctx->devices.size());
        for (size_t i = 0; i < ctx->devices.size(); ++i) {
            std::unique_ptr<ReplicaWorker> w(new ReplicaWorker());   // joined by its destructor on any unwind
            ctx->workers.push_back(std::move(w));
        }
    }
    emb::infof("bert_load_from_file: MI355X engine on %zu HIP device(s)\n", ctx->devices.size());
    if (m.hp.ftype == emb::FMT_F32)
        emb::infof("bert_load_from_file: f32 file: f32 activations x f32 weights on the f32 MFMA chain "
                   "(as the reference multiplies them, bert.cpp:499-503)\n");
    return ctx.release();
}

struct bert_ctx *bert_load_from_file(const char *fname)
{
    try {
        return load_context(fname);
    } catch (const std::bad_alloc &) {
        emb::errorf("bert_load_from_file: out of host memory\n");
    } catch (const std::exception &ex) {
        emb::errorf("bert_load_from_file: load failed: %s\n", ex.what());
    } catch (...) {
        emb::errorf("bert_load_from_file: load failed\n");
    }
    return nullptr;
}

void bert_free(bert_ctx *ctx) { delete ctx; }

int32_t bert_n_embd(bert_ctx *ctx) { return ctx->hp.n_embd; }
int32_t bert_n_max_tokens(bert_ctx *ctx) { return ctx->hp.n_max_tokens; }
const char *bert_vocab_id_to_token(bert_ctx *ctx, bert_vocab_id id) { return ctx->vocab.id_to_token(id); }

void bert_tokenize(struct bert_ctx *ctx, const char *text, bert_vocab_id *tokens, int32_t *n_tokens,
                   int32_t n_max_tokens)
{
    *n_tokens = ctx->vocab.tokenize(text, n_max_tokens, tokens, n_max_tokens > 0 ? n_max_tokens : 0);
}

void bert_forward_batch(bert_ctx *ctx, int32_t n_threads, int32_t n_batch_size, bert_vocab_id **batch_tokens,
                        int32_t *n_tokens, float **batch_embeddings)
{
    (void)n_threads;
    if (!batch_embeddings || n_batch_size <= 0) return;   // reference memory-measurement mode: no output
    int32_t mx = 0;
    for (int i = 0; i < n_batch_size; ++i) mx = std::max(mx, n_tokens[i]);
    if (mx > ctx->hp.n_max_tokens) {
        emb::errorf("Too many tokens, maximum is %d\n", ctx->hp.n_max_tokens);
        return;
    }
    run_forward(ctx, batch_tokens, n_tokens, batch_embeddings, n_batch_size);
}

void bert_forward(struct bert_ctx *ctx, int32_t n_threads, bert_vocab_id *tokens, int32_t n_tokens, float *embeddings)
{
    bert_forward_batch(ctx, n_threads, 1, &tokens, &n_tokens, embeddings ? &embeddings : nullptr);
}

void bert_forward_fake_batch(bert_ctx *ctx, int32_t n_threads, int32_t n_batch_size, bert_vocab_id **batch_tokens,
                             int32_t *n_tokens, float **batch_embeddings)
{
    (void)n_threads;
    std::printf("using function bert_forward_fake_batch\n");
    if (!batch_embeddings || n_batch_size <= 0) return;
    // the reference stops at the first over-long input, after writing the ones before it
    int n_ok = 0;
    while (n_ok < n_batch_size && n_tokens[n_ok] <= ctx->hp.n_max_tokens) ++n_ok;
    run_forward(ctx, batch_tokens, n_tokens, batch_embeddings, n_ok);
    if (n_ok < n_batch_size) emb::errorf("Too many tokens, maximum is %d\n", ctx->hp.n_max_tokens);
}

void bert_encode_batch(struct bert_ctx *ctx, int32_t n_threads, int32_t n_batch_size, int32_t n_inputs,
                       const char **texts, float **embeddings)
{
    if (n_inputs <= 0) return;
    const int32_t N = ctx->hp.n_max_tokens;
    std::vector<int32_t> ids((size_t)n_inputs * N);
    std::vector<int32_t> lens((size_t)n_inputs);
    if (!tokenize_all(ctx, n_threads > 0 ? n_threads : 1, n_inputs, texts, N, ids.data(), lens.data())) return;
    // which inputs the reference's chunking refuses (bert.cpp:1408-1443)
    std::vector<char> ok((size_t)n_inputs, 1);
    if (n_batch_size == n_inputs || n_batch_size <= 0) {
        if (*std::max_element(lens.begin(), lens.end()) > N) {
            emb::errorf("Too many tokens, maximum is %d\n", N);
            return;
        }
    } else {
        std::vector<int> idx((size_t)n_inputs);
        std::iota(idx.begin(), idx.end(), 0);
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return lens[(size_t)a] < lens[(size_t)b]; });
        for (int s = 0; s < n_inputs; s += n_batch_size) {
            const int e = std::min(n_inputs, s + n_batch_size);
            if (lens[(size_t)idx[(size_t)e - 1]] > N) {
                emb::errorf("Too many tokens, maximum is %d\n", N);
                for (int j = s; j < e; ++j) ok[(size_t)idx[(size_t)j]] = 0;
            }
        }
    }
    std::vector<const int32_t *> tp;
    std::vector<int32_t> lp;
    std::vector<float *> op;
    for (int i = 0; i < n_inputs; ++i) {
        if (!ok[(size_t)i]) continue;
        tp.push_back(ids.data() + (size_t)i * N);
        lp.push_back(lens[(size_t)i]);
        op.push_back(embeddings[i]);
    }
    run_forward(ctx, tp.data(), lp.data(), op.data(), (int)tp.size());
}

void bert_encode(struct bert_ctx *ctx, int32_t n_threads, const char *texts, float *embeddings)
{
    bert_encode_batch(ctx, n_threads, 1, 1, &texts, &embeddings);
}

// ---------------------------------------------------------------------------
// bert_hip.h
// ---------------------------------------------------------------------------

int32_t bertx_num_devices(struct bert_ctx *ctx) { return (int32_t)ctx->devices.size(); }

int32_t bertx_device_ordinal(struct bert_ctx *ctx, int32_t slot)
{
    return (slot >= 0 && slot < (int32_t)ctx->devices.size()) ? ctx->devices[(size_t)slot]->ordinal() : -1;
}

void bertx_hparams(struct bert_ctx *ctx, int32_t *o)
{
    o[0] = ctx->hp.n_vocab; o[1] = ctx->hp.n_max_tokens; o[2] = ctx->hp.n_embd; o[3] = ctx->hp.n_intermediate;
    o[4] = ctx->hp.n_head; o[5] = ctx->hp.n_layer; o[6] = ctx->hp.ftype;
}

int32_t bertx_reserve(struct bert_ctx *ctx, int32_t slot, int32_t total_tokens, int32_t n_seqs)
{
    if (slot < 0 || slot >= (int32_t)ctx->devices.size()) return -1;
    Device &D = *ctx->devices[(size_t)slot];
    std::lock_guard<std::mutex> lk(D.mutex());
    emb::DeviceGuard g(D.ordinal());
    return D.reserve(total_tokens, n_seqs, ctx->hp.n_max_tokens) ? 0 : -1;
}

int32_t bertx_forward_device(struct bert_ctx *ctx, int32_t slot, const int32_t *d_ids, const int32_t *d_cu,
                             int32_t n_seqs, int32_t max_len, int32_t total_tokens, float *d_out, void *stream)
{
    if (slot < 0 || slot >= (int32_t)ctx->devices.size()) return -1;
    if (max_len > ctx->hp.n_max_tokens || max_len <= 0) return -4;
    Device &D = *ctx->devices[(size_t)slot];
    std::lock_guard<std::mutex> lk(D.mutex());
    emb::DeviceGuard g(D.ordinal());
    return D.forward(d_ids, d_cu, n_seqs, max_len, total_tokens, d_out, stream ? (hipStream_t)stream : D.stream());
}

void bertx_set_profiling(struct bert_ctx *ctx, int32_t on)
{
    for (auto &d : ctx->devices) d->set_profiling(on != 0);
}

void bertx_reset_stats(struct bert_ctx *ctx)
{
    for (auto &d : ctx->devices) d->reset_stats();
}

int32_t bertx_kernel_stats(struct bert_ctx *ctx, int32_t idx, const char **name, int64_t *launches, double *total_ms,
                           double *work, int32_t *work_is_flops)
{
    if (idx < 0 || idx >= emb::K_NUM_CLASSES) return -1;
    int64_t l = 0;
    double ms = 0, w = 0;
    for (auto &d : ctx->devices) {
        d->collect_stats();
        l += d->stats(idx).launches;
        ms += d->stats(idx).ms;
        w += d->stats(idx).work;
    }
    if (name) *name = emb::kclass_name(idx);
    if (launches) *launches = l;
    if (total_ms) *total_ms = ms;
    if (work) *work = w;
    if (work_is_flops)
        *work_is_flops = (idx == emb::K_EMBED_LN || idx == emb::K_LN_STATS || idx == emb::K_POOL_L2) ? 0 : 1;
    return 0;
}

int32_t bertx_device_last_call(struct bert_ctx *ctx, int32_t slot, double *wall_ms, int32_t *n_seqs,
                               int64_t *n_tokens)
{
    if (!ctx || slot < 0 || slot >= (int32_t)ctx->devices.size()) return -1;
    Device &D = *ctx->devices[(size_t)slot];
    std::lock_guard<std::mutex> lk(D.mutex());   // the stamps are written under it (run_forward)
    if (wall_ms) *wall_ms = D.last_call_ms();
    if (n_seqs) *n_seqs = D.last_call_seqs();
    if (n_tokens) *n_tokens = D.last_call_tokens();
    return 0;
}

int64_t bertx_device_calls(struct bert_ctx *ctx, int32_t slot)
{
    if (!ctx || slot < 0 || slot >= (int32_t)ctx->devices.size()) return -1;
    Device &D = *ctx->devices[(size_t)slot];
    std::lock_guard<std::mutex> lk(D.mutex());
    return D.calls();
}

int32_t bertx_quantize_file(const char *fin, const char *fout, int32_t itype)
{
    return emb::quantize_file(fin, fout, itype, false);
}

int32_t bertx_convert_hf(const char *dir_model, const char *fname_out, int32_t ftype)
{
    return emb::convert_hf_dir(dir_model, fname_out, ftype);
}

int32_t bertx_tokenize_batch(struct bert_ctx *ctx, int32_t n_threads, int32_t n_inputs, const char **texts,
                             int32_t n_max, int32_t *ids, int32_t *n_tokens)
{
    if (!ctx || n_inputs < 0 || n_max <= 0 || (n_inputs > 0 && (!texts || !ids || !n_tokens))) return -1;
    return tokenize_all(ctx, n_threads > 0 ? n_threads : 1, n_inputs, texts, n_max, ids, n_tokens) ? 0 : -1;
}

const char *bertx_version(void) { return "embeddings.cpp_amd 0.1 (gfx950)"; }

}  // extern "C"
