// LayerNorm of token rows (ggml_norm, eps 1e-5, then * w + b; bert.cpp:977-984),
// shared by the row kernels (norm.hip) and the panel LayerNorm fused into the
// residual GEMM (gemm16.hip), so both produce the same bits.
// Layouts: ln_row -- one wave per row, lane owns 4 consecutive features per
// 256-wide slice (embeddings + LN); ln8_* / ln_rows -- 8 lanes per row (the LN
// kernel and the panel LN, which therefore give the same bits).
#pragma once

#include "device_common.h"
#include "kernels.h"

namespace emb {

// Writes the f16 GEMM input and the row's (mean, 1/sigma); the f32 normalised
// row itself is not stored -- the next residual epilogue recomputes it from the
// pre-LN row with ln_apply (kernels.h), the same expression as here.
template <int MAXV>
__device__ __forceinline__ void ln_row(f32x4 (&v)[MAXV], int d, int lane, const float *w, const float *b, h16 *xh,
                                       float2 *st)
{
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (c < d) s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    }
    const float mean = wave_sum(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (c < d) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { const float u = v[k][e] - mean; s2 += u * u; }
        }
    }
    const float scale = 1.0f / sqrtf(wave_sum(s2) / (float)d + 1e-5f);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (c >= d) continue;
        const f32x4 ww = *(const f32x4 *)(w + c), bb = *(const f32x4 *)(b + c);
        h16x4 yh;
#pragma unroll
        for (int e = 0; e < 4; ++e) yh[e] = (h16)ln_apply(v[k][e], mean, scale, ww[e], bb[e]);
        *(h16x4 *)(xh + c) = yh;
    }
    if (lane == 0) *st = float2{mean, scale};
}

// Sum over the 8 lanes of a row group (lanes 8r .. 8r+7) by three DPP moves
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror): VALU only, no LDS, and every
// lane of the group ends with the same bits (each step adds a commuted pair).
__device__ __forceinline__ float sum8(float v)
{
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
    return v;
}

// Rows by groups of 8 lanes: lane 8r + sub of a wave owns row r of the wave's 8,
// 16-B chunks k at features 8 sub + 64 k (k < d / 64; d % 64 == 0, d <= 64 NCH).
template <int NCH>
__device__ __forceinline__ void ln8_load(const h16 *__restrict__ y, int row, bool valid, int d, int sub,
                                         h16x8 (&v)[NCH])
{
    const h16 *p = y + (size_t)row * d + 8 * sub;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
        if (valid && 64 * k < d) v[k] = *(const h16x8 *)(p + 64 * k);
}

// ggml_norm (eps 1e-5, mean then centred variance) * w + b (bert.cpp:977-984) of
// the row held by this lane's group; writes the f16 GEMM input and (mean, 1/sigma).
// Every lane of the wave must call it (the sums cross lanes); `valid` = the row exists.
template <int NCH>
__device__ __forceinline__ void ln8_row(const h16x8 (&v)[NCH], int row, bool valid, int d, int sub,
                                        const float *__restrict__ w, const float *__restrict__ b,
                                        h16 *__restrict__ xh, float2 *__restrict__ st)
{
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
        if (64 * k < d) {
            float t = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) t += (float)v[k][e];
            s += t;
        }
    const float mean = sum8(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
        if (64 * k < d) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { const float u = (float)v[k][e] - mean; s2 += u * u; }
        }
    const float scale = 1.0f / sqrtf(sum8(s2) / (float)d + 1e-5f);
    if (!valid) return;
    h16 *o = xh + (size_t)row * d + 8 * sub;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        const int c = 8 * sub + 64 * k;
        if (64 * k >= d) continue;
        const f32x4 w0 = *(const f32x4 *)(w + c), w1 = *(const f32x4 *)(w + c + 4);
        const f32x4 b0 = *(const f32x4 *)(b + c), b1 = *(const f32x4 *)(b + c + 4);
        h16x8 yh;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            yh[e] = (h16)ln_apply((float)v[k][e], mean, scale, w0[e], b0[e]);
            yh[4 + e] = (h16)ln_apply((float)v[k][4 + e], mean, scale, w1[e], b1[e]);
        }
        *(h16x8 *)(o + 64 * k) = yh;
    }
    if (sub == 0) st[row] = float2{mean, scale};
}

// LN of rows [r_begin, r_end) of the f16 stream y [.][d] by NWV waves (this is
// wave `wave`), 8 rows per wave per pass, the next pass's loads issued before
// this pass's arithmetic.
template <int NCH, int NWV>
__device__ __forceinline__ void ln_rows(const h16 *__restrict__ y, int r_begin, int r_end, int d, int wave, int lane,
                                        const float *w, const float *b, h16 *xh, float2 *st)
{
    const int sub = lane & 7;
    int r = r_begin + 8 * wave + (lane >> 3);
    h16x8 cur[NCH], nxt[NCH];
    ln8_load<NCH>(y, r, r < r_end, d, sub, cur);
    for (int r0 = r_begin + 8 * wave; r0 < r_end; r0 += 8 * NWV) {
        const int rn = r + 8 * NWV;
        const bool more = r0 + 8 * NWV < r_end;      // wave-uniform
        if (more) ln8_load<NCH>(y, rn, rn < r_end, d, sub, nxt);
        ln8_row<NCH>(cur, r, r < r_end, d, sub, w, b, xh, st);
        if (!more) break;
#pragma unroll
        for (int k = 0; k < NCH; ++k) cur[k] = nxt[k];
        r = rn;
    }
}

}  // namespace emb
