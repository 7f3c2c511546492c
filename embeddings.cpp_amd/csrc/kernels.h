// Device-side data layouts and kernel launchers (HIP, gfx950).
//
// HBM layout of one model replica (built by engine.cpp at load):
//   linear weights [N][K] ("lane order", gemm.hip): per K-step (64 k = quant
//            blocks 2ks, 2ks+1) and 32-feature group, 64 lane records; lane
//            l = 16g + f holds the four 16x16x32 A fragments u = 2a + s
//            (feature 32grp + 16a + f, block 2ks + s, elements 8g .. 8g+7):
//              q4_0/q4_1: 16 B (word u, element i at bit 4(i/2) + 16(i%2), so
//                    a mask and an OR with the f16 magic 0x6400 give an f16 pair)
//              q8_0: 32 B (8 B per u, (q ^ 0x80) in order e0 e2 e1 e3 per 4-group)
//              f16:  64 B; f32 files as f16 (hi, lo) pairs along a doubled K
//                    (hi = f16(w), lo = f16(w - hi)), X read twice
//            d (and m) f16 [ks][grp][f][u].  N % 32 == 0, K % 64 == 0.
//   QKV      the three projections are one [3d][d] weight (one GEMM, N = 3d)
//   tables   word/type/pos embeddings in the file's format; q blocks split
//            into an aligned 16/32 B plane + f16 d (+ m) planes.
// Activations (per device workspace, rows = packed tokens of all sentences,
// padded to whole GEMM tiles):
//   Z  [T][d] f16: the residual stream y kept PRE-LayerNorm and scaled by the
//      gamma of the LN that follows it, z = y * gamma ("LN fold", below), with
//      ST [T] (mean, 1/sigma) of y; QKV [T][3d], ATT [T][d], FFN [T][f] f16.
//
// LN fold.  Every consumer of a LayerNorm'd row LN(y) = gamma (y - mean) r + beta
// (r = 1/sigma) reads z = y * gamma and the row's (mean, r):
//   * a projection of it: LN(y) W^T + b = r (z W^T - mean c1) + c2 with the
//     per-feature constants c1 = W gamma, c2 = b + W beta (computed at load), so
//     the GEMM runs on z itself and applies r, mean in its epilogue;
//   * a residual add: LN(y) = r z - r mean gamma + beta, elementwise;
//   * the mean pool: the same expression per token.
// The statistics of a new stream y' come from the residual GEMM that produces
// it: each wave's 32 features of a row give (sum, squared deviations from their
// own mean) in its epilogue, and ln_stats combines them per row (Chan et al.).
// No kernel reads y' to normalise it.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace emb {

struct DevWeight {
    int32_t fmt = 0;   // FMT_F16, FMT_Q4_0, FMT_Q4_1, FMT_Q8_0
    int32_t N = 0, K = 0;
    int32_t kx = 0;    // 0: X has K columns; else X has kx = K/2 columns, read twice
                       // (f32 files: [hi | lo] f16 weight rows, engine.cpp)
    const void *qs = nullptr;       // values / nibbles / int8, lane order
    const uint16_t *d = nullptr;    // f16 scales
    const uint16_t *m = nullptr;    // f16 mins (q4_1)
};

struct DevTable {
    int32_t fmt = 0;   // FMT_F32, FMT_F16, FMT_Q4_0, FMT_Q4_1, FMT_Q8_0
    int32_t rows = 0, cols = 0;
    const void *qs = nullptr;       // f32/f16 values, or per-block 16 B (q4) / 32 B (q8) planes
    const uint16_t *d = nullptr;    // [rows][cols/32]
    const uint16_t *m = nullptr;
};

enum Epi : int32_t { EPI_BIAS_F16 = 0, EPI_BIAS_GELU_F16 = 1, EPI_BIAS_RES = 2 };

constexpr int GEMM_BM = 256;          // largest token tile: batches of >= GEMM_PAD_BIG tokens pad to it
constexpr int GEMM_PAD_BIG = 4096;
constexpr int GEMM_BM_MIN = 64;       // smaller batches pad to the 64-row tile
inline int gemm_rows(int T) { const int a = T >= GEMM_PAD_BIG ? GEMM_BM : GEMM_BM_MIN; return (T + a - 1) / a * a; }
constexpr int ATT_QT = 128;           // queries per attention workgroup (sentences > ATT_LDS_MAX)
constexpr int ATT_LDS_MAX = 512;      // sentences up to this length: whole K/V of a head in LDS

// LayerNorm bookkeeping of a GEMM epilogue (the LN fold above).
struct LnFold {
    // Input side (EPI_BIAS_F16 / EPI_BIAS_GELU_F16): X holds z of a LayerNorm'd
    // stream with per-row in_stats (mean, r); the result is r (acc - mean c1[n])
    // + bias[n], where the caller passes c2 as `bias`.  Null: plain acc + bias.
    const float2 *in_stats = nullptr;
    const float *c1 = nullptr;
    // Statistics fold (instead of in_stats; small batches): the residual GEMM's
    // partials of the input stream, in_part[g * in_part_stride + row] for its
    // in_G = d / 32 groups, combined by the GEMM itself (ln_stats_kernel's
    // arithmetic); the column-0 tiles store the rows' (mean, 1/sigma) to st_out.
    // Only where gemm_fold_ok says the chosen tile config has the LDS for it.
    const float2 *in_part = nullptr;
    int32_t in_part_stride = 0, in_G = 0;
    float2 *st_out = nullptr;
    // Residual side (EPI_BIAS_RES): `res` holds z of the previous LN (res_stats,
    // gamma res_g, beta res_b), the residual being LN(y) = r z - r mean gamma +
    // beta; res_stats null: the residual as stored.  With g_next the new stream
    // y' = residual + acc + bias is stored as f16(y' * g_next) and per (32-feature
    // group, row) partials (sum y', sum (y' - group mean)^2) go to
    // part[group * part_stride + row]; without it the output is f16(y').
    const float2 *res_stats = nullptr;
    const float *res_g = nullptr, *res_b = nullptr;
    const float *g_next = nullptr;
    float2 *part = nullptr;
    int32_t part_stride = 0;
};

// Y[m][n] = epi( sum_k X[m][k] W[n][k] ), X f16 [M][K] with M % 64 == 0 (tiles of
// 256, 128 or 64 rows: every row of every tile is computed and stored), Y f16 [M][N].
// EPI_BIAS_RES: Y = residual + acc + bias (f32 math), res may alias out (in place,
// element-wise).  Returns 0, or -1 for an unsupported shape.
int launch_gemm(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                const void *res, void *out, hipStream_t s, const LnFold &ln = LnFold());
// Tests/benches: tile config (0 = heuristic; the shipped configs are listed at
// gemm.hip launch_fmt: 2, 11, 3, 4, 16).  Per calling thread, so a test hook never
// changes a forward running on another thread.  g_gemm_ran: the config the
// calling thread's last launch_gemm actually dispatched (after fallbacks).
extern thread_local int g_gemm_cfg;
extern thread_local int g_gemm_ran;
// Whether launch_gemm of W over M rows can take the statistics fold (LnFold::in_part)
// for G partial groups: the tile config it will choose has the LDS for them.
bool gemm_fold_ok(const DevWeight &W, int32_t M, int32_t G);

// CU count of the calling thread's current HIP device (cached per ordinal).
int device_cu_count();

// z = f16((pos[i] + (type[0] + word[id])) * gamma) and the (mean, 1/sigma) of
// the f32 sum, for every valid token (bert.cpp:963-984).
void launch_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                     const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t d, uint16_t *z,
                     float2 *stats, hipStream_t s);

// stats[t] = (mean, 1/sqrt(var + 1e-5)) of rows t < rows from the G = d/32 group
// partials part[g * stride + t] a residual GEMM wrote (ggml_norm, bert.cpp:1048-1056).
// Returns -1 (nothing launched) unless d == 32 G with G <= 32.
int launch_ln_stats(const float2 *part, int32_t G, int32_t stride, int32_t rows, int32_t d, float2 *stats,
                     hipStream_t s);

// Benches only: attention kernel variant (bertx_bench_attention).
extern thread_local int g_att_variant;

// Per (sentence, head) softmax(Q K^T / sqrt(dh)) V over the sentence's own keys.
void launch_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                      int32_t d, uint16_t *out, hipStream_t s);

// out[b] = mean_{i<len} LN(y[start+i]) / ||.||  (bert.cpp:1087-1095), from z and
// the row statistics (LN fold).  Two stages: per-64-token-chunk partial sums into
// partial[n_seqs][pool_chunks][d], then sum + normalise.
int32_t pool_chunks(int32_t max_len);
void launch_pool_l2(const uint16_t *z, const float2 *stats, const float *ln_w, const float *ln_b, const int32_t *cu,
                    int32_t n_seqs, int32_t max_len, int32_t d, float *partial, float *out, hipStream_t s);

// ---- the f32 chain (ftype 0 files, f32.hip): every activation f32 [rows][width] ----
// x = LN(pos + (type + word)) with gamma/beta (bert.cpp:963-984).
void launch_f32_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                         const float *ln_b, const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                         int32_t d, float *x, hipStream_t s);
// In-place LayerNorm of rows [0, rows) (ggml_norm, f64 sums, eps 1e-5).
void launch_f32_ln(float *x, int32_t rows, int32_t d, const float *g, const float *b, hipStream_t s);
// Y[M][N] = epi(X[M][K] W[N][K]^T): 0 bias + acc, 1 era GELU(bias + acc) through the
// f16-indexed table gelu_tab [65536] (host_common.h era_tables, uploaded to the
// device), 2 (bias + acc) + res.  M % 64 == 0, K % 32 == 0; returns -1 otherwise.
int launch_f32_gemm(const float *X, int32_t M, const float *W, int32_t N, int32_t K, const float *bias, int32_t epi,
                    const float *res, float *Y, hipStream_t s, const uint16_t *gelu_tab);
// Per (sentence, head) softmax(Q K^T / sqrt(dh)) V with the era's fp16-table exp
// (exp_tab [65536] on the device), qkv f32 [T][3d] -> out f32 [T][d]; dh 32 or 64
// and the 16 score rows of max_len keys within the device's LDS, else -1.
int launch_f32_attention(const float *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                         int32_t d, float *out, hipStream_t s, const uint16_t *exp_tab);
// out[b] = mean_{i<len} x[start + i] / ||.|| (bert.cpp:1087-1095).
void launch_f32_pool(const float *x, const int32_t *cu, int32_t n_seqs, int32_t d, float *out, hipStream_t s);

// Diagnostics: *cnt += number of non-finite values in p[0..n) (f32, or f16 if f16).
void launch_count_nonfinite(const void *p, size_t n, int f16, unsigned *cnt, hipStream_t s);

}  // namespace emb
