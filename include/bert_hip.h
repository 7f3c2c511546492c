/*
 * bert_hip.h — MI355X extensions of the bert.h ABI (libbert.so).
 *
 * Not part of the reference interface: these entry points exist for callers
 * that keep their data in HBM (zero-copy integration, bench.py), for live
 * per-kernel timing, for the native quantizer, and for per-kernel parity
 * tests.  Plain C types only (no torch / HIP types in the signatures); a
 * `stream` argument is a hipStream_t passed as void* (NULL = the context's own
 * stream for that device).
 */
#ifndef BERT_HIP_H
#define BERT_HIP_H

#include "bert.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Number of GPUs the context drives, and the HIP ordinal of slot i. */
BERT_API int32_t bertx_num_devices(struct bert_ctx *ctx);
BERT_API int32_t bertx_device_ordinal(struct bert_ctx *ctx, int32_t slot);

/* hparams {n_vocab, n_max_tokens, n_embd, n_intermediate, n_head, n_layer, ftype}. */
BERT_API void bertx_hparams(struct bert_ctx *ctx, int32_t *out7);

/*
 * Device-resident forward on GPU `slot`.  d_ids: int32[total_tokens] packed
 * sentences back to back; d_cu: int32[n_seqs+1] prefix offsets (d_cu[0] = 0,
 * d_cu[n_seqs] = total_tokens); d_out: float[n_seqs][n_embd].  All three are
 * device pointers on that GPU.  max_len must be >= every sentence length and
 * <= n_max_tokens.  Asynchronous on `stream`; returns 0 or a negative error.
 */
BERT_API int32_t bertx_forward_device(struct bert_ctx *ctx, int32_t slot,
                                      const int32_t *d_ids, const int32_t *d_cu,
                                      int32_t n_seqs, int32_t max_len, int32_t total_tokens,
                                      float *d_out, void *stream);

/* Make sure the workspace of `slot` can hold total_tokens (so a timed region
 * never allocates).  Returns 0 or a negative error. */
BERT_API int32_t bertx_reserve(struct bert_ctx *ctx, int32_t slot, int32_t total_tokens, int32_t n_seqs);

/*
 * Live kernel timing: when enabled, every launch is bracketed by hipEvents on
 * its stream and accumulated per kernel class.  bertx_kernel_stats fills the
 * class name, launch count, summed device milliseconds and summed algorithmic
 * work (FLOP for GEMM/attention classes, bytes for the memory-bound ones) for
 * class `idx` (returns 0, or -1 past the last class).  Stats cover launches
 * whose events have completed (call after a device synchronize).
 */
BERT_API void bertx_set_profiling(struct bert_ctx *ctx, int32_t on);
BERT_API void bertx_reset_stats(struct bert_ctx *ctx);
BERT_API int32_t bertx_kernel_stats(struct bert_ctx *ctx, int32_t idx, const char **name,
                                    int64_t *launches, double *total_ms, double *work,
                                    int32_t *work_is_flops);

/*
 * Multi-GPU balance of the last host-driven call that ran on GPU `slot`
 * (bert_forward_batch / bert_encode_batch, which route or shard sentences over the
 * context's GPUs by FLOP cost, reference entry point bert.cpp:1374-1444): its host
 * wall time for its share (staging, H2D, forward, D2H), its sentence and token
 * counts.  Returns 0, or -1 for a bad slot.
 */
BERT_API int32_t bertx_device_last_call(struct bert_ctx *ctx, int32_t slot, double *wall_ms, int32_t *n_seqs,
                                        int64_t *n_tokens);

/*
 * Number of host-driven calls (bert_forward_batch / bert_encode_batch shares) that
 * have run on replica `slot` since load, or -1 for a bad slot.  Routing rule of
 * those calls (bert_abi.cpp run_forward): a call of T tokens uses
 * k = clamp(min(idle replicas, T / 4096), 1, ...) replicas, the k least-loaded by the
 * work still in flight on them (ties rotate), split by cost; so a large batch
 * spreads over the idle replicas and a call that finds none idle (a concurrent
 * caller) goes whole to the least-loaded replica.
 */
BERT_API int64_t bertx_device_calls(struct bert_ctx *ctx, int32_t slot);

/* Native quantizer (mirrors models/quantize.cpp): f32/f16 file -> itype
 * 2 (q4_0), 3 (q4_1) or 8 (q8_0, extension).  Returns 0 on success. */
BERT_API int32_t bertx_quantize_file(const char *fname_in, const char *fname_out, int32_t itype);

/* Native converter (mirrors models/convert-to-ggml.py:1-113): a local HF
 * BERT directory (config.json, vocab.txt, model.safetensors or a sharded
 * model.safetensors.index.json) -> model file, ftype 0 (f32) or 1 (f16:
 * 2-D weights only).  Same bytes as the reference script writes.  Returns 0
 * on success. */
BERT_API int32_t bertx_convert_hf(const char *dir_model, const char *fname_out, int32_t ftype);

/*
 * Per-kernel parity hooks (host buffers in/out, run synchronously on device 0).
 * w_rows: the weight exactly as the model file stores it (N rows of K elements
 * in format `fmt` = 0,1,2,3,8).  x: f16 bits [M][K].  epi: 0 = +bias -> f16,
 * 1 = +bias, era GELU -> f16, 2 = +bias +res -> f16 (res f16 [M][N], the
 * residual-stream form; sum in f32, computed in place over res).  cfg: GEMM tile
 * config (0 = the production heuristic, 2 = 4 waves 256x128, 11 = the same with
 * the X pieces in one burst, 3 = 4 waves 128x128, 4 = 2 waves 64x64, 16 = 4 waves
 * 64x64 with wave-private X rings); a tile that does not divide the padded M falls
 * back to the next smaller one — bertx_test_gemm_ran() reports what ran.
 * Reference interface these kernels replace: ggml_mul_mat + ggml_add (+ ggml_gelu)
 * at bert.cpp:994-1016, 1040-1045, 1059-1072.
 */
BERT_API int32_t bertx_test_gemm(int32_t fmt, int32_t N, int32_t K, const void *w_rows,
                                 const float *bias, int32_t M, const uint16_t *x,
                                 int32_t epi, const void *res, void *out, int32_t cfg);

/*
 * The same GEMM with the LayerNorm bookkeeping of the forward (the "LN fold",
 * DESIGN.md §2; LayerNorm = bert.cpp:977-984, 1048-1056, 1074-1082):
 *  - in_stats (epi 0/1): x holds z = y * in_g of rows y with in_stats[M] =
 *    (mean, 1/sigma) float pairs; the result is LN(y) W^T + bias with LN's gamma
 *    in_g, beta in_b [K] (else NULL: plain x W^T + bias);
 *  - epi 2: res holds z = y * res_g with res_stats [M] (the residual is LN(y) with
 *    gamma res_g, beta res_b [N]), or the plain residual when res_stats is NULL;
 *    with g_next [N] the output is f16(y' * g_next) of the new stream y' =
 *    residual + x W^T + bias and st_out [M] receives y''s (mean, 1/sigma) as the
 *    forward computes them (epilogue partials + the statistics kernel).
 */
BERT_API int32_t bertx_test_gemm_ln(int32_t fmt, int32_t N, int32_t K, const void *w_rows, const float *bias,
                                    int32_t M, const uint16_t *x, const float *in_stats, const float *in_g,
                                    const float *in_b, int32_t epi, const uint16_t *res, const float *res_stats,
                                    const float *res_g, const float *res_b, const float *g_next, uint16_t *out,
                                    float *st_out, int32_t cfg);

/*
 * The statistics-fold form of the input-LN GEMM (epi 0/1; small batches, where the
 * forward drops the ln_stats launches): part holds the residual GEMM's partials of
 * the input rows, float pairs [K/32][M] (sum, squared deviations from the group
 * mean); the GEMM combines them per row with the statistics kernel's arithmetic
 * and then runs as bertx_test_gemm_ln with those in_stats; st_out [M] (mean,
 * 1/sigma) receives the combined statistics (the column-0 tiles' store), st_kernel
 * [M] (if not NULL) the statistics kernel's combine of the same partials.  Returns
 * -2 when the tile config has no fold form for this shape.
 */
BERT_API int32_t bertx_test_gemm_fold(int32_t fmt, int32_t N, int32_t K, const void *w_rows, const float *bias,
                                      int32_t M, const uint16_t *x, const float *part, const float *in_g,
                                      const float *in_b, int32_t epi, uint16_t *out, float *st_out, float *st_kernel,
                                      int32_t cfg);

/* The tile config the calling thread's last GEMM launch dispatched (after the
 * fallbacks above), so a test can assert which kernel it exercised. */
BERT_API int32_t bertx_test_gemm_ran(void);

/*
 * The f32 chain's GEMM (ftype 0 files: f32 activations x f32 weights on
 * v_mfma_f32_16x16x4_f32, reference ggml_mul_mat f32 x f32, bert.cpp:995):
 * w f32 [N][K] (file rows), x f32 [M][K], out f32 [M][N] = epi(x w^T):
 * epi 0 = bias + acc, 1 = era GELU(bias + acc) (fp16-table semantics), 2 =
 * (bias + acc) + res (res f32 [M][N]).  K % 32 == 0.  Returns 0 or -1.
 */
BERT_API int32_t bertx_test_gemm_f32(int32_t N, int32_t K, const float *w, const float *bias, int32_t M,
                                     const float *x, int32_t epi, const float *res, float *out);

/*
 * GEMM micro-benchmark on random operands (device 0): average device time of
 * `iters` launches of the GEMM for fmt / N / K / M / epi / cfg (as
 * bertx_test_gemm), in the forward's own forms: the LN fold on the input of
 * epi 0/1, the residual LN + next gamma + partial statistics for epi 2
 * (cfg | 0x100: the plain forms, for A/B).
 */
BERT_API int32_t bertx_bench_gemm(int32_t fmt, int32_t N, int32_t K, int32_t M, int32_t epi, int32_t cfg,
                                  int32_t iters, float *avg_us);

/*
 * Attention micro-benchmark on random operands (device 0): average device time
 * of `iters` launches for n_seqs sentences of `len` tokens, n_head heads of size
 * dh; variant 0 = the production kernels (attention_pp for 64 < L <= 512 at dh
 * 64, attention_short for L <= 64), 8 = attention_lds3 (the persistent 16-wave
 * kernel, bitwise the same), 7 = lds3 on at most 7 workgroups (many ragged items
 * per workgroup).
 */
BERT_API int32_t bertx_bench_attention(int32_t n_seqs, int32_t len, int32_t n_head, int32_t dh, int32_t variant,
                                       int32_t iters, float *avg_us);

/*
 * Attention parity hook (host buffers, device 0): qkv f16 bits [T][3d] as the
 * QKV GEMM writes it (packed tokens of n_seqs sentences, cu[n_seqs + 1] the
 * token offsets), out f16 [T][d] = per (sentence, head) softmax(Q K^T / sqrt(dh)) V
 * over the sentence's own keys (bert.cpp:1018-1036).  variant as
 * bertx_bench_attention; -1 = the streaming kernel (sentences > 512).
 */
BERT_API int32_t bertx_test_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t n_head,
                                      int32_t d, int32_t variant, uint16_t *out);

/*
 * The tokenization stage of bert_encode_batch on its own (bert.cpp:1402-1406 runs
 * it sequentially; here on n_threads threads of the library's persistent pool):
 * texts[i] -> ids[i * n_max .. + min(n_tokens[i], n_max)), n_tokens[i] =
 * bert_tokenize's count (which can exceed n_max, bert.cpp:386-387).  The same
 * function bert_encode_batch calls; for timing and bulk tokenization.  Returns 0
 * or -1.
 */
BERT_API int32_t bertx_tokenize_batch(struct bert_ctx *ctx, int32_t n_threads, int32_t n_inputs, const char **texts,
                                      int32_t n_max, int32_t *ids, int32_t *n_tokens);

BERT_API const char *bertx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BERT_HIP_H */
