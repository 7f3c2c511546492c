/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into libbert.so, never on the
 * product path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the timed CPU baseline.
 *
 * ggml-era arithmetic primitives that bert.cpp relies on.  ggml itself is an
 * un-vendored submodule (reference .gitmodules:1-3; /root/reference/ggml is
 * empty), so the semantics below are RESTATED from the published ggml
 * algorithms of the era bert.cpp was written against (mid-2023, inferred from
 * API use: ggml_scale taking a tensor bert.cpp:959, ggml_norm without eps
 * bert.cpp:978, stack ggml_cgraph bert.cpp:883).  Each item says what it
 * restates; all are "inferred" in the sense of SURVEY.md §8a.
 */
#ifndef EMB_ORACLE_GGML_ERA_H
#define EMB_ORACLE_GGML_ERA_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ggml_type ids of the era (the reference file stores them as per-tensor
 * "ftype", bert.cpp:720-742; header ftype 0..3 bert.cpp:500-521).  8 = Q8_0 is
 * the build's documented extension. */
enum { ERA_F32 = 0, ERA_F16 = 1, ERA_Q4_0 = 2, ERA_Q4_1 = 3, ERA_Q8_0 = 8 };

#define ERA_QK 32

/* block_q4_0 {fp16 d; u8 qs[16]}: element j = low nibble of qs[j], element
 * j+16 = high nibble; x = (q-8)*d. */
typedef struct { uint16_t d; uint8_t qs[16]; } era_block_q4_0;
/* block_q4_1 {fp16 d; fp16 m; u8 qs[16]}: x = q*d + m. */
typedef struct { uint16_t d; uint16_t m; uint8_t qs[16]; } era_block_q4_1;
/* block_q8_0 {fp16 d; i8 qs[32]}: x = q*d (activation side of q4_0, and the
 * build's q8_0 weight extension). */
typedef struct { uint16_t d; int8_t qs[32]; } era_block_q8_0;
/* block_q8_1 {f32 d; f32 s = d*sum(q); i8 qs[32]} (activation side of q4_1). */
typedef struct { float d; float s; int8_t qs[32]; } era_block_q8_1;

/* IEEE binary16 <-> binary32, round-to-nearest-even (what F16C _cvtss_sh(x,0)
 * and numpy astype(float16) both do; convert-to-ggml.py:96-99 uses numpy). */
uint16_t era_f32_to_f16(float f);
float    era_f16_to_f32(uint16_t h);

/* 65536-entry fp16 tables (ggml_init builds them once). */
void  era_init_tables(void);
/* ggml_vec_gelu_f32 with GGML_GELU_FP16: y = f16->f32(table_gelu[f32->f16(x)]),
 * table_gelu[i] = f16(0.5x(1+tanh(sqrt(2/pi) x (1 + 0.044715 x^2)))). */
float era_gelu(float x);
/* softmax exp: f16->f32(table_exp[f32->f16(x)]), table_exp[i] = f16(expf(i)). */
float era_exp(float x);

/* Row quantizers (ggml quantize_row_*_reference). */
void era_quantize_row_q4_0(const float *x, era_block_q4_0 *y, int k);
void era_quantize_row_q4_1(const float *x, era_block_q4_1 *y, int k);
void era_quantize_row_q8_0(const float *x, era_block_q8_0 *y, int k);
void era_quantize_row_q8_1(const float *x, era_block_q8_1 *y, int k);

/* Row dequantizers (ggml dequantize_row_*, used by get_rows). */
void era_dequantize_row(int type, const void *src, float *dst, int k);

/* Bytes of one row of k elements of `type`. */
size_t era_row_size(int type, int k);

#ifdef __cplusplus
}
#endif
#endif
