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

}  // namespace
}  // namespace emb
