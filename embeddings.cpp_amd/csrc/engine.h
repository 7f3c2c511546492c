// Per-GPU engine: one weight replica, one workspace, one stream, one mutex.
// The forward is the reference's bert_forward_batch graph (bert.cpp:876-1097)
// as a fixed sequence of HIP launches over a packed (un-padded) token batch.
#pragma once

#include "host_common.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

namespace emb {

enum KClass : int32_t {
    K_EMBED_LN = 0, K_GEMM_QKV, K_ATTENTION, K_GEMM_O, K_LN_STATS, K_GEMM_FFN_UP, K_GEMM_FFN_DOWN, K_POOL_L2,
    K_NUM_CLASSES
};
const char *kclass_name(int k);

struct KStats {
    int64_t launches = 0;
    double ms = 0.0;
    double work = 0.0;     // FLOP (GEMM/attention) or bytes (memory-bound classes)
};

struct DevLayer {
    DevWeight qkv, o, up, down;
    float *b_o = nullptr, *b_down = nullptr;
    // LN fold (kernels.h) of the projections that read a LayerNorm'd stream:
    // c1 = W gamma, c2 = b + W beta of the LN in front (QKV: the previous layer's
    // output LN or the embedding LN; FFN-up: this layer's attention-output LN)
    float *c1_qkv = nullptr, *c2_qkv = nullptr, *c1_up = nullptr, *c2_up = nullptr;
    float *ln1_w = nullptr, *ln1_b = nullptr, *ln2_w = nullptr, *ln2_b = nullptr;
    // f32 files (the f32 chain, f32.hip): weights as the file rows [N][K] f32, QKV
    // fused [3d][d] with its bias [3d]
    const float *w32_qkv = nullptr, *w32_o = nullptr, *w32_up = nullptr, *w32_down = nullptr;
    const float *b_qkv = nullptr, *b_up = nullptr;
};

// Sets the calling thread's current HIP device for a scope and restores the
// previous one on exit (library calls must not move a host application's device).
class DeviceGuard {
public:
    explicit DeviceGuard(int ordinal)
    {
        if (hipGetDevice(&prev_) != hipSuccess) { (void)hipGetLastError(); prev_ = -1; }
        st_ = prev_ == ordinal ? hipSuccess : hipSetDevice(ordinal);
        if (prev_ == ordinal) prev_ = -1;
    }
    ~DeviceGuard() { if (prev_ >= 0) (void)hipSetDevice(prev_); }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
    bool ok() const { return st_ == hipSuccess; }
    hipError_t status() const { return st_; }

private:
    int prev_ = -1;
    hipError_t st_ = hipSuccess;
};

// A model's device image: every weight plane in its device layout (lane-order
// linear weights, LN-fold constants, embedding-table planes, the f32 chain's
// rows and tables), laid out at 256-B aligned offsets of one arena.  Built once
// on the host by build_model_image and uploaded to every replica, so N replicas
// cost one repack (reference: one read of the tensors, bert.cpp:650-766).
struct ModelImage {
    static constexpr size_t kNone = ~(size_t)0;
    struct Tab { size_t q = kNone, d = kNone, m = kNone; int fmt = 0, rows = 0, cols = 0; };
    struct Lin { size_t q = kNone, d = kNone, m = kNone; int N = 0, K = 0; };
    struct Layer {
        Lin qkv, o, up, down;
        size_t bo = kNone, bdown = kNone, c1q = kNone, c2q = kNone, c1u = kNone, c2u = kNone;
        size_t l1w = kNone, l1b = kNone, l2w = kNone, l2b = kNone;
        size_t w32q = kNone, w32o = kNone, w32u = kNone, w32d = kNone, bq = kNone, bu = kNone;
    };
    HParams hp;
    int wfmt = FMT_F16;
    bool f32 = false;
    Tab word, type, pos;
    size_t gelu = kNone, exp = kNone, lnw = kNone, lnb = kNone;
    std::vector<Layer> layers;
    // piece i: bytes [off[i], off[i] + len[i]) of the image (len 0: absent plane)
    std::vector<size_t> off, len;
    size_t total = 0;
    const uint8_t *bytes() const { return pinned_ ? pinned_ : host_.data(); }
    bool pinned() const { return pinned_ != nullptr; }

    ModelImage() = default;
    ~ModelImage();
    ModelImage(const ModelImage &) = delete;
    ModelImage &operator=(const ModelImage &) = delete;

private:
    friend bool build_model_image(const HostModel &m, ModelImage &img, std::string &err, bool pin);
    std::vector<uint8_t> host_;       // pageable image (when pinning failed or no device)
    uint8_t *pinned_ = nullptr;       // page-locked image (hipHostMalloc): async uploads
};

// Host work of a load, once per context: checks the shape, repacks every plane
// and concatenates them into the image (page-locked when `pin`).  False with a
// message in err; never throws (a bad_alloc becomes false).
bool build_model_image(const HostModel &m, ModelImage &img, std::string &err, bool pin);

class Device {
public:
    // Creates the replica's stream and completion event, allocates the weight
    // arena and issues the image upload on the replica's stream (async from a
    // page-locked image).  Call finish_load() before the first use.  All HIP calls
    // of a load are made by the loading thread (bert_load_from_file).
    Device(int ordinal, const ModelImage &img);
    ~Device();
    bool finish_load();   // waits for the upload; ok() from then on
    bool ok() const { return ok_; }
    int ordinal() const { return ordinal_; }
    hipStream_t stream() const { return stream_; }
    std::mutex &mutex() { return mu_; }

    // Grow the workspace so one forward of `tokens` packed tokens / `seqs`
    // sentences of at most `max_len` tokens fits (never called inside a timed
    // forward).  Waits for the replica's last forward, on whatever stream it ran.
    bool reserve(int64_t tokens, int64_t seqs, int max_len);

    // Device-resident forward (ids, cu, out on this GPU); async on `s`.  When
    // profiling is off and `s` is not the null stream, the launch sequence is
    // captured once per (pointers, shape, stream) into a HIP graph and replayed.
    // The workspace is shared by every forward of the replica: a forward on a
    // stream other than the previous forward's first waits (on the device) for
    // that forward's completion event, so calls on different streams never
    // overlap in the workspace.
    // len2_sum: sum of the squared sentence lengths when the caller knows them
    // (attention FLOP of the per-kernel stats), else -1.
    int forward(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int total_tokens, float *d_out,
                hipStream_t s, double len2_sum = -1.0);

    // Host-driven forward: packs tokens, H2D, forward, D2H, synchronous.
    // tokens[i] has lens[i] ids; out[i] receives n_embd floats.
    int forward_host(const int32_t *const *tokens, const int32_t *lens, int n, float *const *out);

    // profiling
    void set_profiling(bool on) { profiling_ = on; }
    void collect_stats();
    void reset_stats();
    const KStats &stats(int k) const { return stats_[k]; }

    const HParams &hp() const { return hp_; }

    // the last bert_forward_batch / bert_encode_batch call that ran on this replica
    // (bertx_device_last_call): host wall time of its forwards, sentences, tokens;
    // calls() counts the host-driven calls that ran here (bertx_device_calls)
    void set_last_call(double ms, int seqs, int64_t tokens)
    {
        lc_ms_ = ms; lc_seqs_ = seqs; lc_tokens_ = tokens; ++calls_;
    }
    int64_t calls() const { return calls_; }
    double last_call_ms() const { return lc_ms_; }
    int last_call_seqs() const { return lc_seqs_; }
    int64_t last_call_tokens() const { return lc_tokens_; }

private:
    struct PendingEv { int cls; hipEvent_t a, b; double work; };
    struct GraphKey {
        const void *ids, *cu, *out;
        hipStream_t s;
        int n_seqs, max_len, T;
        bool operator==(const GraphKey &o) const
        {
            return ids == o.ids && cu == o.cu && out == o.out && s == o.s && n_seqs == o.n_seqs &&
                   max_len == o.max_len && T == o.T;
        }
    };
    struct GraphEntry { GraphKey key; hipGraphExec_t exec; };
    int forward_ordered(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                        hipStream_t s);
    void order_after_last(hipStream_t s);   // stream s waits for the last forward (any stream)
    void mark_done(hipStream_t s);          // records the completion event of a forward on s
    int launch_all(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                   hipStream_t s, bool check);
    int launch_all_f32(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                       hipStream_t s);
    void drop_graphs();
    void bind(const ModelImage &img);   // device pointers of the image's planes
    bool uploading_ = false;
    void begin(int cls, hipStream_t s, hipEvent_t &a);
    void end(int cls, hipStream_t s, hipEvent_t a, double work);
    hipEvent_t get_event();

    bool ok_ = false;
    int ordinal_ = 0;
    HParams hp_;
    hipStream_t stream_ = nullptr;
    std::mutex mu_;

    // weights
    char *arena_ = nullptr;
    size_t arena_size_ = 0, arena_used_ = 0;
    DevTable word_, type_, pos_;
    float *ln_e_w_ = nullptr, *ln_e_b_ = nullptr;
    std::vector<DevLayer> layers_;
    int wfmt_ = FMT_F16;
    bool f32_ = false;              // ftype 0 file: the f32 chain (f32.hip)
    const uint16_t *gelu_tab_ = nullptr, *exp_tab_ = nullptr;   // f32 chain: the era's fp16 tables (host-built)

    // workspace
    int64_t cap_tokens_ = 0, cap_seqs_ = 0, cap_pool_ = 0;   // cap_pool_: pool partial rows (seqs x chunks)
    hipEvent_t done_ev_ = nullptr;          // completion of the last forward
    hipStream_t last_stream_ = nullptr;     // ... and the stream it ran on
    bool any_forward_ = false;
    char *ws_ = nullptr;
    uint16_t *z_ = nullptr;         // residual stream as z = y * gamma of its LN (f16, kernels.h)
    float2 *st_ = nullptr;          // (mean, 1/sigma) of y
    float2 *part_ = nullptr;        // [d/32][rows] group partials of the residual GEMMs
    int64_t rows_ = 0;              // workspace rows (part_ stride)
    uint16_t *qkv_ = nullptr, *att_ = nullptr, *ffn_ = nullptr;
    float *x32_ = nullptr, *z32_ = nullptr, *qkv32_ = nullptr, *att32_ = nullptr, *ffn32_ = nullptr;   // f32 chain
    int32_t *d_ids_ = nullptr, *d_cu_ = nullptr;
    float *d_out_ = nullptr;
    float *pool_part_ = nullptr;
    int32_t *h_ids_ = nullptr, *h_cu_ = nullptr;   // pinned staging
    float *h_out_ = nullptr;

    // HIP graphs of the launch sequence (cleared when the workspace moves)
    std::vector<GraphEntry> graphs_;
    std::vector<GraphKey> seen_once_;   // a shape is captured on its second use
    bool use_graphs_ = true;

    // profiling
    double lc_ms_ = 0.0;
    int lc_seqs_ = 0;
    int64_t lc_tokens_ = 0;
    int64_t calls_ = 0;

    bool profiling_ = false;
    double att_flop_ = 0.0;         // attention FLOP of the forward being launched
    std::vector<PendingEv> pending_;
    std::vector<hipEvent_t> free_events_;
    KStats stats_[K_NUM_CLASSES];
};

// HIP device count (0 when no runtime / no GPU); never throws.
int hip_device_count();

}  // namespace emb
