// Embedding-table reads shared by the row kernels (norm.hip, f32.hip): tables
// stay in the file's format on the device (kernels.h DevTable), dequantized on
// read (reference get_rows, bert.cpp:963-974).
#pragma once

#include "device_common.h"
#include "host_common.h"
#include "kernels.h"

namespace emb {
namespace {

// 4 consecutive table values starting at column c (c % 4 == 0)
__device__ __forceinline__ f32x4 table4(const DevTable &t, int row, int c)
{
    f32x4 r;
    switch (t.fmt) {
    case FMT_F32: return *(const f32x4 *)((const float *)t.qs + (size_t)row * t.cols + c);
    case FMT_F16: {
        const h16x4 h = *(const h16x4 *)((const h16 *)t.qs + (size_t)row * t.cols + c);
        r[0] = h[0]; r[1] = h[1]; r[2] = h[2]; r[3] = h[3];
        return r;
    }
    case FMT_Q8_0: {
        const size_t b = (size_t)row * (t.cols / 32) + c / 32;
        const uint32_t w = *(const uint32_t *)((const int8_t *)t.qs + b * 32 + (c & 31));
        const float d = (float)as_h(t.d[b]);
        r[0] = (float)(int8_t)(w & 0xff) * d; r[1] = (float)(int8_t)((w >> 8) & 0xff) * d;
        r[2] = (float)(int8_t)((w >> 16) & 0xff) * d; r[3] = (float)(int8_t)(w >> 24) * d;
        return r;
    }
    default: {   // q4_0 / q4_1, file nibble order: element j<16 low nibble of byte j, j>=16 high of j-16
        const size_t b = (size_t)row * (t.cols / 32) + c / 32;
        const int j = c & 31;
        const uint32_t w = *(const uint32_t *)((const uint8_t *)t.qs + b * 16 + (j & 15));
        const int sh = j < 16 ? 0 : 4;
        const float d = (float)as_h(t.d[b]);
        const float mn = t.fmt == FMT_Q4_1 ? (float)as_h(t.m[b]) : 0.0f;
        const int o = t.fmt == FMT_Q4_1 ? 0 : 8;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = (int)((w >> (8 * e + sh)) & 15u) - o;
            r[e] = t.fmt == FMT_Q4_1 ? (float)q * d + mn : (float)q * d;
        }
        return r;
    }
    }
}

// The 32 values of quant block b (columns 32 b .. 32 b + 31) of a row, with
// table4's arithmetic per value, from whole-block loads (16 B of q4 nibbles, 32 B
// of q8, 64 / 128 B of f16 / f32) instead of one narrow load per 4 values.
__device__ __forceinline__ void table32(const DevTable &t, int row, int b, float (&r)[32])
{
    const size_t blk = (size_t)row * (t.cols / 32) + b;
    switch (t.fmt) {
    case FMT_F32: {
        const f32x4 *p = (const f32x4 *)((const float *)t.qs + blk * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const f32x4 v = p[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) r[4 * i + e] = v[e];
        }
        return;
    }
    case FMT_F16: {
        const h16x8 *p = (const h16x8 *)((const h16 *)t.qs + blk * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const h16x8 v = p[i];
#pragma unroll
            for (int e = 0; e < 8; ++e) r[8 * i + e] = v[e];
        }
        return;
    }
    case FMT_Q8_0: {
        const uint4 *p = (const uint4 *)((const int8_t *)t.qs + blk * 32);
        const uint4 w0 = p[0], w1 = p[1];
        const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float d = (float)as_h(t.d[blk]);
#pragma unroll
        for (int j = 0; j < 32; ++j) r[j] = (float)(int8_t)((w[j >> 2] >> (8 * (j & 3))) & 0xff) * d;
        return;
    }
    default: {   // q4_0 / q4_1: element j < 16 low nibble of byte j, j >= 16 high nibble of byte j - 16
        const uint4 q = *(const uint4 *)((const uint8_t *)t.qs + blk * 16);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
        const float d = (float)as_h(t.d[blk]);
        const float mn = t.fmt == FMT_Q4_1 ? (float)as_h(t.m[blk]) : 0.0f;
        const int o = t.fmt == FMT_Q4_1 ? 0 : 8;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int k = j & 15;
            const int qv = (int)((w[k >> 2] >> (8 * (k & 3) + (j < 16 ? 0 : 4))) & 15u) - o;
            r[j] = t.fmt == FMT_Q4_1 ? (float)qv * d + mn : (float)qv * d;
        }
        return;
    }
    }
}

}  // namespace
}  // namespace emb
