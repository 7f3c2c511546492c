// HIP kernels of the BERT embedding forward for gfx950 (MI355X / CDNA4).
// Layouts: kernels.h.  Reference semantics: bert.cpp:827-1147.
#include "kernels.h"
#include "host_common.h"

#include <hip/hip_runtime.h>
#include <cmath>

namespace emb {

typedef _Float16 h16;
typedef h16 h16x8 __attribute__((ext_vector_type(8)));
typedef h16 h16x4 __attribute__((ext_vector_type(4)));
typedef h16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ h16x2 as_h2(uint32_t u) { return __builtin_bit_cast(h16x2, u); }
__device__ __forceinline__ h16 as_h(uint16_t u) { return __builtin_bit_cast(h16, u); }

// ggml-era GELU (tanh form) on an f16-rounded input, result rounded to f16:
// identical to ggml's table_gelu_f16 lookup (GGML_GELU_FP16), bert.cpp:1063.
__device__ __forceinline__ h16 gelu_era(float v)
{
    const float x = (float)(h16)v;
    const float a = 0.044715f, s = 0.79788456080286535587989211986876f;
    return (h16)(0.5f * x * (1.0f + tanhf(s * x * (1.0f + a * x * x))));
}

// 8 q4 nibbles (pair-interleaved word, kernels.h) -> 8 f16 = (q + off) * d  [+ m]
template <bool HAS_MIN>
__device__ __forceinline__ h16x8 dq4_word(uint32_t w, h16x2 off, h16x2 d2, h16x2 m2)
{
    h16x8 r;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t v = ((w >> (4 * p)) & 0x000F000Fu) | 0x64006400u;   // 1024 + q
        h16x2 h = as_h2(v) + off;                                          // exact small ints
        h = HAS_MIN ? h * d2 + m2 : h * d2;
        r[2 * p] = h[0];
        r[2 * p + 1] = h[1];
    }
    return r;
}

// 4 q8 bytes (q ^ 0x80, order e0 e2 e1 e3) -> 4 f16 = q * d
__device__ __forceinline__ void dq8_word(uint32_t w, h16x2 d2, h16 *o)
{
    const h16x2 off = {(h16)-1152.0f, (h16)-1152.0f};
    const h16x2 a = (as_h2((w & 0x00FF00FFu) | 0x64006400u) + off) * d2;
    const h16x2 b = (as_h2(((w >> 8) & 0x00FF00FFu) | 0x64006400u) + off) * d2;
    o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
}

// ---------------------------------------------------------------------------
// GEMM: Y[m][n] = epi(sum_k X[m][k] W[n][k]) with W dequantized into LDS.
// Block tile 128(m) x 128(n) x 64(k), 4 waves (2 x 2), wave tile 64 x 64 made
// of 2 x 2 v_mfma_f32_32x32x16_f16 tiles.  MFMA A = W rows (n), B = X rows
// (m): the accumulator lane is a token, its 16 registers are 4 runs of 4
// consecutive features, so the epilogue stores 8/16-byte row segments.
// One LDS double buffer; global loads of step k+1 are in flight while step k
// multiplies.
// ---------------------------------------------------------------------------

constexpr int BM = GEMM_BM, BN = GEMM_BN, BK = 64, LDS_STR = BK + 8;  // 144 B rows: conflict-free b128 reads

template <int FMT>
struct WStage;

template <>
struct WStage<FMT_F16> {
    uint4 v0, v1, v2, v3;
    __device__ __forceinline__ uint4 ld(const DevWeight &W, int n0, int ks, int tid, int i) const
    {
        const int n = n0 + (tid >> 3) + 32 * i;
        const h16 *p = (const h16 *)W.qs + ((size_t)ks * W.N + (n < W.N ? n : 0)) * 64 + (tid & 7) * 8;
        uint4 r = *(const uint4 *)p;
        if (n >= W.N) r = make_uint4(0, 0, 0, 0);
        return r;
    }
    __device__ __forceinline__ void load(const DevWeight &W, int n0, int ks, int tid)
    {
        v0 = ld(W, n0, ks, tid, 0); v1 = ld(W, n0, ks, tid, 1);
        v2 = ld(W, n0, ks, tid, 2); v3 = ld(W, n0, ks, tid, 3);
    }
    __device__ __forceinline__ void store(h16 *Ws, int tid) const
    {
        h16 *p = Ws + (tid >> 3) * LDS_STR + (tid & 7) * 8;
        *(uint4 *)(p) = v0;
        *(uint4 *)(p + 32 * LDS_STR) = v1;
        *(uint4 *)(p + 64 * LDS_STR) = v2;
        *(uint4 *)(p + 96 * LDS_STR) = v3;
    }
};

template <int FMT>
struct WStageQ4 {
    uint4 q;
    uint16_t d, m;
    __device__ void load(const DevWeight &W, int n0, int ks, int tid)
    {
        const int n = n0 + (tid >> 1), blk = tid & 1;
        if (n < W.N) {
            const size_t i = ((size_t)ks * W.N + n) * 2 + blk;
            q = *(const uint4 *)((const uint8_t *)W.qs + i * 16);
            d = W.d[i];
            m = FMT == FMT_Q4_1 ? W.m[i] : (uint16_t)0;
        } else {
            q = make_uint4(0, 0, 0, 0);
            d = 0; m = 0;
        }
    }
    __device__ void store(h16 *Ws, int tid) const
    {
        const h16 dd = as_h(d), mm = as_h(m);
        const h16x2 d2 = {dd, dd}, m2 = {mm, mm};
        const h16 o = FMT == FMT_Q4_1 ? (h16)-1024.0f : (h16)-1032.0f;
        const h16x2 off = {o, o};
        h16 *dst = Ws + (tid >> 1) * LDS_STR + (tid & 1) * 32;
        *(h16x8 *)(dst + 0) = dq4_word<FMT == FMT_Q4_1>(q.x, off, d2, m2);
        *(h16x8 *)(dst + 8) = dq4_word<FMT == FMT_Q4_1>(q.y, off, d2, m2);
        *(h16x8 *)(dst + 16) = dq4_word<FMT == FMT_Q4_1>(q.z, off, d2, m2);
        *(h16x8 *)(dst + 24) = dq4_word<FMT == FMT_Q4_1>(q.w, off, d2, m2);
    }
};
template <> struct WStage<FMT_Q4_0> : WStageQ4<FMT_Q4_0> {};
template <> struct WStage<FMT_Q4_1> : WStageQ4<FMT_Q4_1> {};

template <>
struct WStage<FMT_Q8_0> {
    uint4 q0, q1;
    uint16_t d;
    __device__ void load(const DevWeight &W, int n0, int ks, int tid)
    {
        const int n = n0 + (tid >> 1), blk = tid & 1;
        if (n < W.N) {
            const size_t i = ((size_t)ks * W.N + n) * 2 + blk;
            const uint4 *p = (const uint4 *)((const uint8_t *)W.qs + i * 32);
            q0 = p[0]; q1 = p[1];
            d = W.d[i];
        } else {
            q0 = q1 = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
            d = 0;
        }
    }
    __device__ void store(h16 *Ws, int tid) const
    {
        const h16 dd = as_h(d);
        const h16x2 d2 = {dd, dd};
        h16x8 r[4];
        h16 *o = (h16 *)r;
        const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) dq8_word(w[i], d2, o + 4 * i);
        h16 *dst = Ws + (tid >> 1) * LDS_STR + (tid & 1) * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) *(h16x8 *)(dst + 8 * i) = r[i];
    }
};

template <int FMT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(DevWeight W, const h16 *__restrict__ X, int M,
                                                      const float *__restrict__ bias,
                                                      const float *__restrict__ res, void *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) h16 smem[2][(BM + BN) * LDS_STR];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int K = W.K, N = W.N, KS = K / BK;

    uint4 x0, x1, x2, x3;
    WStage<FMT> ws;
    const h16 *xsrc = X + (size_t)(m0 + (tid >> 3)) * K + (tid & 7) * 8;
    const size_t xstep = (size_t)32 * K;
#define EMB_LOAD_X(ks_)                                                                                     \
    {                                                                                                       \
        const h16 *p_ = xsrc + (ks_) * BK;                                                                  \
        x0 = *(const uint4 *)(p_); x1 = *(const uint4 *)(p_ + xstep);                                       \
        x2 = *(const uint4 *)(p_ + 2 * xstep); x3 = *(const uint4 *)(p_ + 3 * xstep);                       \
    }
#define EMB_STORE_X(Xs_)                                                                                    \
    {                                                                                                       \
        h16 *p_ = (Xs_) + (tid >> 3) * LDS_STR + (tid & 7) * 8;                                             \
        *(uint4 *)(p_) = x0; *(uint4 *)(p_ + 32 * LDS_STR) = x1;                                            \
        *(uint4 *)(p_ + 64 * LDS_STR) = x2; *(uint4 *)(p_ + 96 * LDS_STR) = x3;                             \
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    EMB_LOAD_X(0)
    ws.load(W, n0, 0, tid);
    EMB_STORE_X(smem[0])
    ws.store(smem[0] + BM * LDS_STR, tid);
    __syncthreads();

    const int lr = lane & 31, lk = (lane >> 5) * 8;
    for (int ks = 0; ks < KS; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < KS) {
            EMB_LOAD_X(ks + 1)
            ws.load(W, n0, ks + 1, tid);
        }
        const h16 *Xs = smem[cur];
        const h16 *Ws = smem[cur] + BM * LDS_STR;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            const h16x8 a0 = *(const h16x8 *)(Ws + (wn * 64 + lr) * LDS_STR + kk * 16 + lk);
            const h16x8 a1 = *(const h16x8 *)(Ws + (wn * 64 + 32 + lr) * LDS_STR + kk * 16 + lk);
            const h16x8 b0 = *(const h16x8 *)(Xs + (wm * 64 + lr) * LDS_STR + kk * 16 + lk);
            const h16x8 b1 = *(const h16x8 *)(Xs + (wm * 64 + 32 + lr) * LDS_STR + kk * 16 + lk);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (ks + 1 < KS) {
            EMB_STORE_X(smem[cur ^ 1])
            ws.store(smem[cur ^ 1] + BM * LDS_STR, tid);
        }
        __syncthreads();
    }

    // epilogue: lane = token m, registers 4g..4g+3 = features n..n+3
    const int hi = lane >> 5;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int m = m0 + wm * 64 + j * 32 + lr;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = n0 + wn * 64 + i * 32 + 8 * g + 4 * hi;
                if (n >= N) continue;
                const float4 bb = *(const float4 *)(bias + n);
                const float v0 = acc[i][j][4 * g + 0], v1 = acc[i][j][4 * g + 1];
                const float v2 = acc[i][j][4 * g + 2], v3 = acc[i][j][4 * g + 3];
                if (EPI == EPI_BIAS_RES_F32) {
                    const float4 rr = *(const float4 *)(res + (size_t)m * N + n);
                    float4 o;
                    o.x = rr.x + (bb.x + v0); o.y = rr.y + (bb.y + v1);
                    o.z = rr.z + (bb.z + v2); o.w = rr.w + (bb.w + v3);
                    *(float4 *)((float *)out + (size_t)m * N + n) = o;
                } else {
                    h16x4 o;
                    if (EPI == EPI_BIAS_GELU_F16) {
                        o[0] = gelu_era(bb.x + v0); o[1] = gelu_era(bb.y + v1);
                        o[2] = gelu_era(bb.z + v2); o[3] = gelu_era(bb.w + v3);
                    } else {
                        o[0] = (h16)(bb.x + v0); o[1] = (h16)(bb.y + v1);
                        o[2] = (h16)(bb.z + v2); o[3] = (h16)(bb.w + v3);
                    }
                    *(h16x4 *)((h16 *)out + (size_t)m * N + n) = o;
                }
            }
        }
    }
}

template <int FMT>
static void gemm_dispatch_epi(const DevWeight &W, const uint16_t *X, int M, const float *bias, int epi,
                              const float *res, void *out, hipStream_t s)
{
    dim3 grid((W.N + BN - 1) / BN, M / BM);
    const h16 *x = (const h16 *)X;
    switch (epi) {
    case EPI_BIAS_F16: gemm_kernel<FMT, EPI_BIAS_F16><<<grid, 256, 0, s>>>(W, x, M, bias, res, out); break;
    case EPI_BIAS_GELU_F16: gemm_kernel<FMT, EPI_BIAS_GELU_F16><<<grid, 256, 0, s>>>(W, x, M, bias, res, out); break;
    default: gemm_kernel<FMT, EPI_BIAS_RES_F32><<<grid, 256, 0, s>>>(W, x, M, bias, res, out); break;
    }
}

void launch_gemm(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                 const float *res, void *out, hipStream_t s)
{
    switch (W.fmt) {
    case FMT_Q4_0: gemm_dispatch_epi<FMT_Q4_0>(W, X, M, bias, epi, res, out, s); break;
    case FMT_Q4_1: gemm_dispatch_epi<FMT_Q4_1>(W, X, M, bias, epi, res, out, s); break;
    case FMT_Q8_0: gemm_dispatch_epi<FMT_Q8_0>(W, X, M, bias, epi, res, out, s); break;
    default: gemm_dispatch_epi<FMT_F16>(W, X, M, bias, epi, res, out, s); break;
    }
}

// ---------------------------------------------------------------------------
// embeddings + LayerNorm: one wave per token
// ---------------------------------------------------------------------------

__device__ __forceinline__ float table_at(const DevTable &t, int row, int c)
{
    switch (t.fmt) {
    case FMT_F32: return ((const float *)t.qs)[(size_t)row * t.cols + c];
    case FMT_F16: return (float)as_h(((const uint16_t *)t.qs)[(size_t)row * t.cols + c]);
    case FMT_Q8_0: {
        const size_t b = (size_t)row * (t.cols / 32) + c / 32;
        return (float)((const int8_t *)t.qs)[b * 32 + (c & 31)] * (float)as_h(t.d[b]);
    }
    default: {  // q4_0 / q4_1: 16-byte plane in the file's nibble order
        const size_t b = (size_t)row * (t.cols / 32) + c / 32;
        const int j = c & 31;
        const uint8_t byte = ((const uint8_t *)t.qs)[b * 16 + (j & 15)];
        const int q = j < 16 ? (byte & 15) : (byte >> 4);
        if (t.fmt == FMT_Q4_1) return (float)q * (float)as_h(t.d[b]) + (float)as_h(t.m[b]);
        return (float)(q - 8) * (float)as_h(t.d[b]);
    }
    }
}

// ggml_norm (eps 1e-5, two-pass) * w + b over one row held as v[0..d/64) per lane
template <int NV>
__device__ __forceinline__ void ln_row(float (&v)[NV], int nv, int d, const float *w, const float *b, int lane,
                                       float *x32, h16 *xh)
{
    float s = 0.f;
    for (int k = 0; k < nv; ++k) s += v[k];
    const float mean = wave_sum(s) / (float)d;
    float s2 = 0.f;
    for (int k = 0; k < nv; ++k) { v[k] -= mean; s2 += v[k] * v[k]; }
    const float var = wave_sum(s2) / (float)d;
    const float scale = 1.0f / sqrtf(var + 1e-5f);
    for (int k = 0; k < nv; ++k) {
        const int c = lane + 64 * k;
        const float y = w[c] * (v[k] * scale) + b[c];
        x32[c] = y;
        xh[c] = (h16)y;
    }
}

__global__ __launch_bounds__(256) void embed_ln_kernel(DevTable word, DevTable type, DevTable pos,
                                                       const float *__restrict__ ln_w, const float *__restrict__ ln_b,
                                                       const int32_t *__restrict__ ids, const int32_t *__restrict__ cu,
                                                       int d, float *__restrict__ x32, h16 *__restrict__ xh)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int start = cu[b], len = cu[b + 1] - start;
    if (i >= len) return;
    const int t = start + i, id = ids[t];
    float v[16];
    const int nv = d / 64;
    for (int k = 0; k < nv; ++k) {
        const int c = lane + 64 * k;
        v[k] = table_at(pos, i, c) + (table_at(type, 0, c) + table_at(word, id, c));
    }
    ln_row<16>(v, nv, d, ln_w, ln_b, lane, x32 + (size_t)t * d, xh + (size_t)t * d);
}

__global__ __launch_bounds__(256) void layernorm_kernel(const float *__restrict__ y, int T, int d,
                                                        const float *__restrict__ w, const float *__restrict__ b,
                                                        float *__restrict__ x32, h16 *__restrict__ xh)
{
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= T) return;
    float v[16];
    const int nv = d / 64;
    const float *row = y + (size_t)t * d;
    for (int k = 0; k < nv; ++k) v[k] = row[lane + 64 * k];
    ln_row<16>(v, nv, d, w, b, lane, x32 + (size_t)t * d, xh + (size_t)t * d);
}

void launch_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                     const float *ln_b, const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                     int32_t d, float *x32, uint16_t *xh, hipStream_t s)
{
    dim3 grid((max_len + 3) / 4, n_seqs);
    embed_ln_kernel<<<grid, 256, 0, s>>>(word, type, pos, ln_w, ln_b, ids, cu, d, x32, (h16 *)xh);
}

void launch_layernorm(const float *y, int32_t T, int32_t d, const float *w, const float *b, float *x32,
                      uint16_t *xh, hipStream_t s)
{
    layernorm_kernel<<<(T + 3) / 4, 256, 0, s>>>(y, T, d, w, b, x32, (h16 *)xh);
}

// ---------------------------------------------------------------------------
// attention: flash-style, one workgroup = 128 queries of one (sentence, head),
// 4 waves x 32 queries.  S^T = K Q^T per 32-key block (query on the lane,
// keys in registers) -> online softmax in registers -> O^T += V^T P^T with
// the S accumulator reused as the B operand (no LDS round trip for P).
// Keys past the sentence end get probability exactly 0, as the reference's
// -1e5 mask does after its fp16 exp (bert.cpp:957-961, 1024-1025).
// ---------------------------------------------------------------------------

template <int DH>
__global__ __launch_bounds__(256) void attention_kernel(const h16 *__restrict__ qkv, const int32_t *__restrict__ cu,
                                                        int d, float sl2, h16 *__restrict__ out)
{
    constexpr int KT = 64, KSTR = DH + 8, VSTR = KT + 8;
    __shared__ __attribute__((aligned(16))) h16 Ks[KT * KSTR];
    __shared__ __attribute__((aligned(16))) h16 Vt[DH * VSTR];
    const int b = blockIdx.z, h = blockIdx.y;
    const int start = cu[b], len = cu[b + 1] - start;
    const int q0 = blockIdx.x * ATT_QT;
    if (q0 >= len) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int hi = lane >> 5, lq = lane & 31;
    const int ld = 3 * d;
    const int q = q0 + w * 32 + lq;

    h16x8 qf[DH / 16];
    const h16 *qrow = qkv + (size_t)(start + q) * ld + h * DH;
#pragma unroll
    for (int s = 0; s < DH / 16; ++s) qf[s] = *(const h16x8 *)(qrow + 16 * s + 8 * hi);

    f32x16 o[DH / 32];
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m_i = -INFINITY, l_i = 0.f;

    const int nkt = (len + KT - 1) / KT;
    for (int kt = 0; kt < nkt; ++kt) {
        const int k0 = kt * KT;
        __syncthreads();
        // K tile row-major (coalesced: chunk index fastest)
        for (int c = tid; c < KT * DH / 8; c += 256) {
            const int r = c / (DH / 8), ch = c % (DH / 8);
            *(uint4 *)(Ks + r * KSTR + ch * 8) = *(const uint4 *)(qkv + (size_t)(start + k0 + r) * ld + d + h * DH + ch * 8);
        }
        // V tile transposed into Vt[d][key] (key fastest across lanes: conflict-free 2-byte writes)
        for (int c = tid; c < KT * DH / 8; c += 256) {
            const int r = c % KT, ch = c / KT;
            const h16x8 vv = *(const h16x8 *)(qkv + (size_t)(start + k0 + r) * ld + 2 * d + h * DH + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * VSTR + r] = vv[e];
        }
        __syncthreads();

        f32x16 s[2];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
#pragma unroll
            for (int st = 0; st < DH / 16; ++st) {
                const h16x8 a = *(const h16x8 *)(Ks + (kh * 32 + lq) * KSTR + 16 * st + 8 * hi);
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[st], s[kh], 0, 0, 0);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = k0 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
                const float v = key < len ? s[kh][r] * sl2 : -INFINITY;
                s[kh][r] = v;
                mx = fmaxf(mx, v);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_i, mx);
        const float alpha = exp2f(m_i - m_new);
        float rs = 0.f;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = exp2f(s[kh][r] - m_new);
                s[kh][r] = p;
                rs += p;
            }
        rs += __shfl_xor(rs, 32, 64);
        l_i = l_i * alpha + rs;
        m_i = m_new;
#pragma unroll
        for (int t = 0; t < DH / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;

#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                h16x8 bp;
#pragma unroll
                for (int j = 0; j < 8; ++j) bp[j] = (h16)s[kh][8 * s2 + j];
#pragma unroll
                for (int t = 0; t < DH / 32; ++t) {
                    const h16 *vr = Vt + (32 * t + lq) * VSTR + 32 * kh + 16 * s2 + 4 * hi;
                    const h16x4 lo = *(const h16x4 *)vr;
                    const h16x4 up = *(const h16x4 *)(vr + 8);
                    const h16x8 a = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bp, o[t], 0, 0, 0);
                }
            }
        }
    }

    if (q < len) {
        const float inv = 1.0f / l_i;
        h16 *orow = out + (size_t)(start + q) * d + h * DH;
#pragma unroll
        for (int t = 0; t < DH / 32; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                h16x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (h16)(o[t][4 * g + e] * inv);
                *(h16x4 *)(orow + 32 * t + 8 * g + 4 * hi) = v;
            }
    }
}

void launch_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                      int32_t d, uint16_t *out, hipStream_t s)
{
    const int dh = d / n_head;
    const float sl2 = (1.0f / sqrtf((float)dh)) * 1.4426950408889634f;
    dim3 grid((max_len + ATT_QT - 1) / ATT_QT, n_head, n_seqs);
    if (dh == 64)
        attention_kernel<64><<<grid, 256, 0, s>>>((const h16 *)qkv, cu, d, sl2, (h16 *)out);
    else
        attention_kernel<32><<<grid, 256, 0, s>>>((const h16 *)qkv, cu, d, sl2, (h16 *)out);
}

// ---------------------------------------------------------------------------
// masked mean pool + L2 normalise: one workgroup per sentence
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void pool_l2_kernel(const float *__restrict__ x32, const int32_t *__restrict__ cu,
                                                      int d, float *__restrict__ out)
{
    __shared__ float part[4][1024];
    __shared__ float red[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int start = cu[b], len = cu[b + 1] - start;
    const float wt = 1.0f / (float)len;
    const int nch = d / 4;
    for (int ch = lane; ch < nch; ch += 64) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = w; i < len; i += 4) {
            const float4 x = *(const float4 *)(x32 + (size_t)(start + i) * d + 4 * ch);
            a.x += x.x * wt; a.y += x.y * wt; a.z += x.z * wt; a.w += x.w * wt;
        }
        *(float4 *)&part[w][4 * ch] = a;
    }
    __syncthreads();
    float ss = 0.f;
    float e[4];
    int ne = 0;
    for (int c = tid; c < d; c += 256) {
        const float v = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
        e[ne++] = v;
        ss += v * v;
    }
    ss = wave_sum(ss);
    if (lane == 0) red[w] = ss;
    __syncthreads();
    const float nrm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    ne = 0;
    for (int c = tid; c < d; c += 256) out[(size_t)b * d + c] = e[ne++] / nrm;
}

void launch_pool_l2(const float *x32, const int32_t *cu, int32_t n_seqs, int32_t d, float *out, hipStream_t s)
{
    pool_l2_kernel<<<n_seqs, 256, 0, s>>>(x32, cu, d, out);
}

}  // namespace emb
