// Device-side data layouts and kernel launchers (HIP, gfx950).
//
// HBM layout of one model replica (built by engine.cpp at load):
//   weights  [N][K] linear layers repacked "K-step major" (KS = 64 = two quant
//            blocks): element (n, k) lives in step ks = k/64 at
//            ((ks*N + n) * 64 + k%64) -- one K-step of a 128-row tile is one
//            contiguous, fully coalesced run of bytes.
//              f16 : 128 B per (ks, n) in MFMA A-fragment order: byte
//                    64h + 16kk + 2i holds k = 16kk + 8h + i (the lane of
//                    half h loads its 4 fragments as 64 contiguous bytes)
//              q4_0/q4_1: 32 B nibbles per (ks, n) in the MFMA A-fragment
//                    ("register") order of gemm_q.hip: word 4h + kk holds
//                    k = 16kk + 8h + i (i = 0..7), element i at bit
//                    4*(i/2) + 16*(i%2) so one AND/OR yields an f16 pair; the
//                    lane of half h loads its 4 words as one 16-B load.
//                    d (and m) f16 [ks][n][2] (blocks k<32, k>=32)
//              q8_0: 64 B per (ks, n): 8 bytes per (h, kk) at 32h + 8kk holding
//                    k = 16kk + 8h + i as (q ^ 0x80), order e0 e2 e1 e3 per
//                    4-group (pair extraction by mask); d f16 [ks][n][2]
//   QKV      the three projections are one [3d][d] weight (one GEMM, N = 3d)
//   tables   word/type/pos embeddings in the file's format; q blocks split
//            into an aligned 16/32 B plane + f16 d (+ m) planes.
// Activations (per device workspace, rows = packed tokens of all sentences):
//   YH [T][d] f16 residual stream kept PRE-LayerNorm + ST [T] (mean, 1/sigma)
//   of its last LN (the normalised row is recomputed where it is consumed),
//   XH [T][d] f16 normalised copy (GEMM input), QKV [T][3d] f16, ATT [T][d] f16,
//   FFN [T][f] f16.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace emb {

struct DevWeight {
    int32_t fmt = 0;   // FMT_F16 (also used for f32 files), FMT_Q4_0, FMT_Q4_1, FMT_Q8_0
    int32_t N = 0, K = 0;
    const void *qs = nullptr;       // values / nibbles / int8
    const uint16_t *d = nullptr;    // f16 scales [K/64][N][2]
    const uint16_t *m = nullptr;    // f16 mins (q4_1)
    int32_t layout = 0;             // 0: fragment order of gemm.hip, 1: lane order of gemm16.hip
};

struct DevTable {
    int32_t fmt = 0;   // FMT_F32, FMT_F16, FMT_Q4_0, FMT_Q4_1, FMT_Q8_0
    int32_t rows = 0, cols = 0;
    const void *qs = nullptr;       // f32/f16 values, or per-block 16 B (q4) / 32 B (q8) planes
    const uint16_t *d = nullptr;    // [rows][cols/32]
    const uint16_t *m = nullptr;
};

enum Epi : int32_t { EPI_BIAS_F16 = 0, EPI_BIAS_GELU_F16 = 1, EPI_BIAS_RES = 2 };

constexpr int GEMM_BM = 256;          // token rows per tile (M is padded to this)
constexpr int GEMM_BN = 128;          // output features per tile
constexpr int ATT_QT = 128;           // queries per attention workgroup (sentences > ATT_LDS_MAX)
constexpr int ATT_LDS_MAX = 512;      // sentences up to this length: whole K/V of a head in LDS

// Deferred LayerNorm: the residual stream is kept PRE-LN (f32) with each row's
// (mean, 1/sigma); a consumer that needs the normalised row recomputes it with
// ln_apply -- the expression the LN kernel itself uses for the f16 copy.
struct ResLN {
    const float2 *stats = nullptr;   // [rows] (mean, 1/sigma); nullptr: residual used as stored
    const float *w = nullptr, *b = nullptr;   // gamma, beta [n_embd]
    // Panel LayerNorm fused into the residual GEMM (gemm16, EPI_BIAS_RES): the
    // workgroup that finishes a 128-row token panel last (per-panel counter
    // `cnt`, zero between launches) normalises the panel's new pre-LN rows with
    // (nw, nb): xh = f16(LN(out)), st_out = (mean, 1/sigma) for rows < rows.
    // st_out may alias stats: every reader of the panel's old statistics has
    // counted in before the last workgroup overwrites them.
    uint32_t *cnt = nullptr;
    uint16_t *xh = nullptr;
    float2 *st_out = nullptr;
    const float *nw = nullptr, *nb = nullptr;
    int32_t rows = 0;
    int32_t pvar = 0;   // panel hand-off variant (gemm16.hip), BERT_PANEL_VARIANT
};
__host__ __device__ __forceinline__ float ln_apply(float v, float mean, float scale, float w, float b)
{
    return w * ((v - mean) * scale) + b;
}

// Y[m][n] = epi( sum_k X[m][k] W[n][k] ), X f16 [M][K] with M % GEMM_BM == 0.
// EPI_BIAS_RES: Y = LN(res) + acc + bias (f32 math; res and Y f16, the residual
// stream) with LN given by `rln` (identity if rln.stats is null); res may alias
// out (in place, element-wise).
// Returns 1 when the launch also ran the panel LayerNorm of rln (rln.cnt set,
// residual form of a gemm16 weight with N % 128 == 0 and N <= 1024), else 0
// (the caller then runs launch_layernorm itself).
int launch_gemm(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                const void *res, void *out, hipStream_t s, const ResLN &rln = ResLN());

// Weight layout 1 (gemm16.hip, v_mfma_f32_16x16x32_f16): per K-step (64 k =
// blocks 2ks, 2ks+1) and 32-feature group, 64 lane records; lane l = 16g + f
// holds fragments u = 2a + s (feature 32grp + 16a + f, block 2ks + s,
// elements 8g .. 8g+7): q4 16 B (word u, element i at bit 4(i/2) + 16(i%2)),
// q8 32 B (8 B per u, (q ^ 0x80) in order e0 e2 e1 e3 per 4-group), f16 64 B;
// d (and m) f16 [ks][grp][f][u].  N % 32 == 0.
int launch_gemm16(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                  const void *res, void *out, hipStream_t s, const ResLN &rln);
// Benches/tests: gemm16 tile config (0 = heuristic, 1 = 8 waves 256x256, 2 = 4 waves 256x128,
// 3 = 4 waves 128x128).
extern int g_gemm16_cfg;
int launch_gemm16_stamped(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                          const void *res, void *out, hipStream_t s, int cfg, uint64_t *stamps);
// Layout the engine repacks linear weights into (BERT_GEMM_LAYOUT overrides).
extern int g_weight_layout;

// Tests only: force the GEMM tile shape (128 / 256; 0 = heuristic).
extern int g_force_bn;
// Benches only: GEMM kernel variant (0 = heuristic, 2 = gemmqw everywhere).
extern int g_gemm_variant;
// Diagnostics: q4_0 gemmqw (wm waves along tokens) with per-wave s_memtime stamps.
int launch_gemm_q_stamped(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                          const void *res, void *out, hipStream_t s, int32_t wm, uint64_t *stamps,
                          int32_t diag);

// yh = f16(pos[i] + (type[0] + word[id])) (pre-LN), xh = f16(LN(yh)), stats, for
// every valid token (bert.cpp:963-984).
void launch_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                     const float *ln_b, const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                     int32_t d, uint16_t *yh, uint16_t *xh, float2 *stats, hipStream_t s);

// xh = f16(LN(yh)), stats = (mean, 1/sigma) per row, for T rows (yh f16).
void launch_layernorm(const uint16_t *yh, int32_t T, int32_t d, const float *w, const float *b, uint16_t *xh,
                      float2 *stats, hipStream_t s);

// Benches only: attention kernel variant (bertx_bench_attention).
extern int g_att_variant;

// Per (sentence, head) softmax(Q K^T / sqrt(dh)) V over the sentence's own keys.
void launch_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                      int32_t d, uint16_t *out, hipStream_t s);

// out[b] = mean_{i<len} LN(yh[start+i]) / ||.||  (bert.cpp:1087-1095).
// Two stages: per-64-token-chunk partial sums into partial[n_seqs][pool_chunks][d],
// then sum + normalise.
int32_t pool_chunks(int32_t max_len);
void launch_pool_l2(const uint16_t *yh, const ResLN &ln, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                    int32_t d, float *partial, float *out, hipStream_t s);

// Diagnostics: *cnt += number of non-finite values in p[0..n) (f32, or f16 if f16).
void launch_count_nonfinite(const void *p, size_t n, int f16, unsigned *cnt, hipStream_t s);

}  // namespace emb
