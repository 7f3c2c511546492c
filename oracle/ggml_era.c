/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ggml_era.h).  Restatement of the
 * ggml-era primitives bert.cpp calls; ggml is absent from /root/reference.
 */
#include "ggml_era.h"

#include <math.h>
#include <string.h>

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

uint16_t era_f32_to_f16(float f)
{
    uint32_t x = fbits(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    int32_t e = (int32_t)((x >> 23) & 0xffu);
    uint32_t m = x & 0x7fffffu;
    if (e == 255) return (uint16_t)(sign | 0x7c00u | (m ? 0x200u : 0u));
    int32_t he = e - 127 + 15;
    if (he >= 31) return (uint16_t)(sign | 0x7c00u);
    if (he <= 0) {
        if (he < -10) return (uint16_t)sign;
        m |= 0x800000u;
        int shift = 14 - he;
        uint32_t hm = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t hm = m >> 13;
    uint32_t rem = m & 0x1fffu;
    uint32_t h = sign | ((uint32_t)he << 10) | hm;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1u))) h++;
    return (uint16_t)h;
}

float era_f16_to_f32(uint16_t h)
{
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    if (e == 0) {
        if (m == 0) return bitsf(sign);
        /* subnormal: m * 2^-24 */
        float v = (float)m * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    if (e == 31) return bitsf(sign | 0x7f800000u | (m << 13));
    return bitsf(sign | ((e - 15 + 127) << 23) | (m << 13));
}

static uint16_t g_tab_gelu[65536];
static uint16_t g_tab_exp[65536];
static int g_tables_ready = 0;

void era_init_tables(void)
{
    if (g_tables_ready) return;
    const float k_a = 0.044715f;
    const float k_s = 0.79788456080286535587989211986876f; /* sqrt(2/pi) */
    for (uint32_t i = 0; i < 65536u; ++i) {
        float f = era_f16_to_f32((uint16_t)i);
        float g = 0.5f * f * (1.0f + tanhf(k_s * f * (1.0f + k_a * f * f)));
        g_tab_gelu[i] = era_f32_to_f16(g);
        g_tab_exp[i] = era_f32_to_f16(expf(f));
    }
    g_tables_ready = 1;
}

float era_gelu(float x) { return era_f16_to_f32(g_tab_gelu[era_f32_to_f16(x)]); }
float era_exp(float x)  { return era_f16_to_f32(g_tab_exp[era_f32_to_f16(x)]); }

void era_quantize_row_q4_0(const float *x, era_block_q4_0 *y, int k)
{
    const int nb = k / ERA_QK;
    for (int b = 0; b < nb; ++b) {
        const float *xb = x + b * ERA_QK;
        float amax = 0.0f, vmax = 0.0f;       /* signed value of largest |x| */
        for (int j = 0; j < ERA_QK; ++j) {
            if (amax < fabsf(xb[j])) { amax = fabsf(xb[j]); vmax = xb[j]; }
        }
        const float d = vmax / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = era_f32_to_f16(d);
        for (int j = 0; j < ERA_QK / 2; ++j) {
            const float a0 = xb[j] * id;
            const float a1 = xb[j + ERA_QK / 2] * id;
            int q0 = (int8_t)(a0 + 8.5f); if (q0 > 15) q0 = 15;
            int q1 = (int8_t)(a1 + 8.5f); if (q1 > 15) q1 = 15;
            y[b].qs[j] = (uint8_t)((uint8_t)q0 | ((uint8_t)q1 << 4));
        }
    }
}

void era_quantize_row_q4_1(const float *x, era_block_q4_1 *y, int k)
{
    const int nb = k / ERA_QK;
    for (int b = 0; b < nb; ++b) {
        const float *xb = x + b * ERA_QK;
        float vmin = 3.402823466e+38f, vmax = -3.402823466e+38f;
        for (int j = 0; j < ERA_QK; ++j) {
            if (xb[j] < vmin) vmin = xb[j];
            if (xb[j] > vmax) vmax = xb[j];
        }
        const float d = (vmax - vmin) / 15;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = era_f32_to_f16(d);
        y[b].m = era_f32_to_f16(vmin);
        for (int j = 0; j < ERA_QK / 2; ++j) {
            const float a0 = (xb[j] - vmin) * id;
            const float a1 = (xb[j + ERA_QK / 2] - vmin) * id;
            int q0 = (int8_t)(a0 + 0.5f); if (q0 > 15) q0 = 15;
            int q1 = (int8_t)(a1 + 0.5f); if (q1 > 15) q1 = 15;
            y[b].qs[j] = (uint8_t)((uint8_t)q0 | ((uint8_t)q1 << 4));
        }
    }
}

void era_quantize_row_q8_0(const float *x, era_block_q8_0 *y, int k)
{
    const int nb = k / ERA_QK;
    for (int b = 0; b < nb; ++b) {
        const float *xb = x + b * ERA_QK;
        float amax = 0.0f;
        for (int j = 0; j < ERA_QK; ++j) amax = fmaxf(amax, fabsf(xb[j]));
        const float d = amax / 127;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = era_f32_to_f16(d);
        for (int j = 0; j < ERA_QK; ++j) y[b].qs[j] = (int8_t)roundf(xb[j] * id);
    }
}

void era_quantize_row_q8_1(const float *x, era_block_q8_1 *y, int k)
{
    const int nb = k / ERA_QK;
    for (int b = 0; b < nb; ++b) {
        const float *xb = x + b * ERA_QK;
        float amax = 0.0f;
        for (int j = 0; j < ERA_QK; ++j) amax = fmaxf(amax, fabsf(xb[j]));
        const float d = amax / 127;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = d;
        int s = 0;
        for (int j = 0; j < ERA_QK; ++j) {
            y[b].qs[j] = (int8_t)roundf(xb[j] * id);
            s += y[b].qs[j];
        }
        y[b].s = (float)s * d;
    }
}

size_t era_row_size(int type, int k)
{
    switch (type) {
    case ERA_F32:  return (size_t)k * 4;
    case ERA_F16:  return (size_t)k * 2;
    case ERA_Q4_0: return (size_t)(k / ERA_QK) * sizeof(era_block_q4_0);
    case ERA_Q4_1: return (size_t)(k / ERA_QK) * sizeof(era_block_q4_1);
    case ERA_Q8_0: return (size_t)(k / ERA_QK) * sizeof(era_block_q8_0);
    default: return 0;
    }
}

void era_dequantize_row(int type, const void *src, float *dst, int k)
{
    switch (type) {
    case ERA_F32: memcpy(dst, src, (size_t)k * 4); break;
    case ERA_F16: {
        const uint16_t *h = (const uint16_t *)src;
        for (int i = 0; i < k; ++i) dst[i] = era_f16_to_f32(h[i]);
    } break;
    case ERA_Q4_0: {
        const era_block_q4_0 *b = (const era_block_q4_0 *)src;
        for (int i = 0; i < k / ERA_QK; ++i) {
            const float d = era_f16_to_f32(b[i].d);
            for (int j = 0; j < 16; ++j) {
                dst[i * 32 + j]      = (float)((int)(b[i].qs[j] & 0xf) - 8) * d;
                dst[i * 32 + j + 16] = (float)((int)(b[i].qs[j] >> 4) - 8) * d;
            }
        }
    } break;
    case ERA_Q4_1: {
        const era_block_q4_1 *b = (const era_block_q4_1 *)src;
        for (int i = 0; i < k / ERA_QK; ++i) {
            const float d = era_f16_to_f32(b[i].d);
            const float m = era_f16_to_f32(b[i].m);
            for (int j = 0; j < 16; ++j) {
                dst[i * 32 + j]      = (float)(b[i].qs[j] & 0xf) * d + m;
                dst[i * 32 + j + 16] = (float)(b[i].qs[j] >> 4) * d + m;
            }
        }
    } break;
    case ERA_Q8_0: {
        const era_block_q8_0 *b = (const era_block_q8_0 *)src;
        for (int i = 0; i < k / ERA_QK; ++i) {
            const float d = era_f16_to_f32(b[i].d);
            for (int j = 0; j < 32; ++j) dst[i * 32 + j] = (float)b[i].qs[j] * d;
        }
    } break;
    default: break;
    }
}
