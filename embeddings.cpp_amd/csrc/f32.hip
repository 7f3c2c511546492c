// The f32 forward (ftype 0 files): the reference multiplies f32 activations by
// f32 weights (bert.cpp:499-503; ggml_mul_mat f32 x f32 at bert.cpp:995), so
// these files run a separate chain of kernels whose every tensor is f32:
//   embeddings + LayerNorm -> per layer: QKV GEMM, attention, O-proj GEMM +
//   residual, LayerNorm, FFN-up GEMM + era GELU, FFN-down GEMM + residual,
//   LayerNorm -> mean pool + L2 divide.
// GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 products, k-ordered f32 FMA chain,
// MI355X f32 MFMA rate); LayerNorm sums in f64 as ggml_norm does; softmax and
// GELU follow the era's fp16 tables (exp(f16(s - max)) rounded to f16, sum in
// f64, bert.cpp:1025; gelu(f16(x)) rounded to f16, bert.cpp:1063) so the
// quantization the reference applies is applied here too.
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"
#include "table_read.h"

#include <atomic>
#include <cmath>

namespace emb {
namespace {

// ---------------------------------------------------------------- row helpers

__device__ __forceinline__ double wave_sum_d(double v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

constexpr int F32_MAXC = 4;   // float4 chunks per lane: d <= 1024

// ggml_norm (mean and centred variance summed in f64, eps 1e-5) then * gamma +
// beta (bert.cpp:977-984), of one row held as lane chunks c = 4 lane + 256 k.
__device__ __forceinline__ void ln_row(f32x4 (&v)[F32_MAXC], int d, int lane, const float *__restrict__ g,
                                       const float *__restrict__ b)
{
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k)
        if (4 * lane + 256 * k < d)
#pragma unroll
            for (int e = 0; e < 4; ++e) s += (double)v[k][e];
    const float mean = (float)(wave_sum_d(s) / d);
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k)
        if (4 * lane + 256 * k < d)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float c = v[k][e] - mean;
                v[k][e] = c;
                s2 += (double)(c * c);
            }
    const float var = (float)(wave_sum_d(s2) / d);
    const float scale = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < d) {
            const f32x4 gg = *(const f32x4 *)(g + c), bb = *(const f32x4 *)(b + c);
            // ggml_norm's y = c * scale, then ggml_mul (gamma) and ggml_add (beta):
            // three rounded ops, no contraction (bert.cpp:977-984, 1051-1055)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[k][e] = __fadd_rn(__fmul_rn(gg[e], __fmul_rn(v[k][e], scale)), bb[e]);
        }
    }
}

// One wave per token row: x = LN(pos[i] + (type[0] + word[id])) (bert.cpp:963-984).
__global__ __launch_bounds__(256) void f32_embed_ln_kernel(DevTable word, DevTable type, DevTable pos,
                                                           const float *__restrict__ ln_w,
                                                           const float *__restrict__ ln_b,
                                                           const int32_t *__restrict__ ids,
                                                           const int32_t *__restrict__ cu, int d, float *__restrict__ x)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int start = cu[b], len = cu[b + 1] - start;
    if (i >= len) return;   // whole waves
    const int t = start + i, id = ids[t];
    f32x4 v[F32_MAXC];
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < d) {
            const f32x4 w = table4(word, id, c), ty = table4(type, 0, c), p = table4(pos, i, c);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[k][e] = p[e] + (ty[e] + w[e]);
        }
    }
    ln_row(v, d, lane, ln_w, ln_b);
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < d) *(f32x4 *)(x + (size_t)t * d + c) = v[k];
    }
}

// In-place LayerNorm of rows [0, rows) (bert.cpp:1048-1056, 1074-1082).
__global__ __launch_bounds__(256) void f32_ln_kernel(float *__restrict__ x, int rows, int d,
                                                     const float *__restrict__ g, const float *__restrict__ b)
{
    const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= rows) return;
    f32x4 v[F32_MAXC];
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < d) v[k] = *(const f32x4 *)(x + (size_t)t * d + c);
    }
    ln_row(v, d, lane, g, b);
#pragma unroll
    for (int k = 0; k < F32_MAXC; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < d) *(f32x4 *)(x + (size_t)t * d + c) = v[k];
    }
}

// ---------------------------------------------------------------- GEMM

// The era's fp16 tables (GELU, exp), built on the host with libm at load
// (model_file.cpp era_tables) and indexed by the f16 bit pattern of the input:
// T(f16(x)), bit for bit the table ggml held.
__device__ __forceinline__ float era_table(const uint16_t *__restrict__ tab, float v)
{
    return (float)as_h(tab[__builtin_bit_cast(uint16_t, (h16)v)]);
}

// Y[m][n] = epi(sum_k X[m][k] W[n][k]) on 64 x 32 tiles, 4 waves of 32 x 16
// (2 v_mfma_f32_16x16x4_f32 tiles each), K in steps of 32 through LDS (rows
// padded to 33 floats), the next step's words loaded during this step's MFMAs.
// A = X (lane: row l & 15, k = l >> 4), B = W^T (k = l >> 4, feature l & 15); D
// lane: feature l & 15, tokens 4 (l >> 4) + r.  Every output is one k-ordered
// MFMA chain whatever the tile shape (so a sentence's bits do not depend on its
// batch); the tile is narrow because the f32 chain's batches are small (C1: one
// sentence): twice the workgroups of a 64 x 64 tile and half the MFMAs per wave
// and K-step (C1 711 -> 527 us with the double buffer alone).
// EPI: 0 bias + acc, 1 GELU table(bias + acc), 2 (bias + acc) + res (the
// reference's operand order, bert.cpp:1040-1045, 1066-1072).
constexpr int F32_BK = 32, F32_BN = 32;

template <int EPI>
__global__ __launch_bounds__(256) void f32_gemm_kernel(const float *__restrict__ X, const float *__restrict__ W,
                                                       const float *__restrict__ bias, const float *__restrict__ res,
                                                       float *__restrict__ Y, int N, int K, int nN,
                                                       const uint16_t *__restrict__ gelu_tab)
{
    __shared__ float xs[64][F32_BK + 1], ws[F32_BN][F32_BK + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m0 = (blockIdx.x / nN) * 64, n0 = (blockIdx.x % nN) * F32_BN;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 16;
    const int lr = tid >> 2, lc = (tid & 3) * 8;     // X loader: row lr, columns lc .. lc + 7
    const int wr = tid >> 3, wc = (tid & 7) * 4;     // W loader: row wr, columns wc .. wc + 3
    const bool wrow = n0 + wr < N;
    f32x4 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float *xp = X + (size_t)(m0 + lr) * K + lc;
    const float *wp = W + (size_t)(wrow ? n0 + wr : 0) * K + wc;
    f32x4 x0 = *(const f32x4 *)xp, x1 = *(const f32x4 *)(xp + 4);
    f32x4 w0 = {0.f, 0.f, 0.f, 0.f};
    if (wrow) w0 = *(const f32x4 *)wp;
    for (int k0 = 0; k0 < K; k0 += F32_BK) {
        __syncthreads();   // the previous step's fragment reads are done
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            xs[lr][lc + e] = x0[e]; xs[lr][lc + 4 + e] = x1[e];
            ws[wr][wc + e] = w0[e];
        }
        __syncthreads();
        if (k0 + F32_BK < K) {
            const int kn = k0 + F32_BK;
            x0 = *(const f32x4 *)(xp + kn);
            x1 = *(const f32x4 *)(xp + kn + 4);
            if (wrow) w0 = *(const f32x4 *)(wp + kn);
        }
#pragma unroll
        for (int kk = 0; kk < F32_BK; kk += 4) {
            const float bq = ws[wn + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float a = xs[wm + 16 * i + (lane & 15)][kk + (lane >> 4)];
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, acc[i], 0, 0, 0);
            }
        }
    }
    const int n = n0 + wn + (lane & 15);
    if (n >= N) return;
    const float bv = bias[n];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const size_t o = (size_t)(m0 + wm + 16 * i + 4 * (lane >> 4) + r) * N + n;
            float v = bv + acc[i][r];
            if (EPI == 1) v = era_table(gelu_tab, v);
            if (EPI == 2) v = v + res[o];
            Y[o] = v;
        }
}

// ---------------------------------------------------------------- attention

// One workgroup per (16 queries, head, sentence): scores of the 16 queries over
// the sentence's keys into LDS (f32 dot products, scaled by 1/sqrt(dh)), the
// era softmax per row (max, exp(f16(s - max)) rounded to f16, f64 sum, times
// 1/sum; bert.cpp:1018-1025), then P V (bert.cpp:1027-1036).  16 lanes per
// query row; K / V in 64-key tiles through LDS.  Padded keys do not exist here
// (packed sentences); the reference's mask makes theirs contribute exactly 0.
template <int DH>
__global__ __launch_bounds__(256) void f32_attention_kernel(const float *__restrict__ qkv, const int32_t *__restrict__ cu,
                                                            int d, int s_stride, float scale, float *__restrict__ out,
                                                            const uint16_t *__restrict__ exp_tab)
{
    extern __shared__ float smem[];
    float(*qs)[DH] = (float(*)[DH])smem;                      // [16][DH]
    float(*kv)[DH + 1] = (float(*)[DH + 1])(smem + 16 * DH);   // [64][DH + 1]
    float *S = smem + 16 * DH + 64 * (DH + 1);                 // [16][s_stride]
    const int q0 = blockIdx.x * 16, h = blockIdx.y, b = blockIdx.z;
    const int start = cu[b], len = cu[b + 1] - start;
    if (q0 >= len) return;   // whole workgroup
    const int tid = threadIdx.x, qi = tid >> 4, l16 = tid & 15;
    const size_t ld = 3 * (size_t)d;
    for (int i = tid; i < 16 * DH; i += 256) {
        const int r = i / DH, e = i % DH;
        qs[r][e] = q0 + r < len ? qkv[(size_t)(start + q0 + r) * ld + h * DH + e] : 0.f;
    }
    for (int k0 = 0; k0 < len; k0 += 64) {
        __syncthreads();
        for (int i = tid; i < 64 * DH; i += 256) {
            const int r = i / DH, e = i % DH;
            kv[r][e] = k0 + r < len ? qkv[(size_t)(start + k0 + r) * ld + d + h * DH + e] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kk = l16 + 16 * j;
            float a = 0.f;
#pragma unroll 8
            for (int e = 0; e < DH; ++e) a = fmaf(kv[kk][e], qs[qi][e], a);
            if (k0 + kk < len) S[qi * s_stride + k0 + kk] = a * scale;
        }
    }
    __syncthreads();
    float *row = S + qi * s_stride;
    float mx = -INFINITY;
    for (int k = l16; k < len; k += 16) mx = fmaxf(mx, row[k]);
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    double sum = 0.0;
    for (int k = l16; k < len; k += 16) {
        const float e = era_table(exp_tab, row[k] - mx);
        row[k] = e;
        sum += (double)e;
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = (float)(1.0 / sum);
    for (int k = l16; k < len; k += 16) row[k] *= inv;
    constexpr int NE = DH / 16;
    float o_acc[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) o_acc[j] = 0.f;
    for (int k0 = 0; k0 < len; k0 += 64) {
        __syncthreads();   // row updates visible; previous V tile consumed
        for (int i = tid; i < 64 * DH; i += 256) {
            const int r = i / DH, e = i % DH;
            kv[r][e] = k0 + r < len ? qkv[(size_t)(start + k0 + r) * ld + 2 * d + h * DH + e] : 0.f;
        }
        __syncthreads();
        const int kn = min(64, len - k0);
        for (int kk = 0; kk < kn; ++kk) {
            const float p = row[k0 + kk];
#pragma unroll
            for (int j = 0; j < NE; ++j) o_acc[j] = fmaf(p, kv[kk][l16 + 16 * j], o_acc[j]);
        }
    }
    if (q0 + qi < len)
#pragma unroll
        for (int j = 0; j < NE; ++j) out[(size_t)(start + q0 + qi) * d + h * DH + l16 + 16 * j] = o_acc[j];
}

// ---------------------------------------------------------------- pool

// out[b] = (sum_i x[i] * (1/len)) / ||.||  (bert.cpp:1087-1095), one workgroup
// per sentence, a thread per column; the norm's sum of squares in f64.
__global__ __launch_bounds__(256) void f32_pool_kernel(const float *__restrict__ x, const int32_t *__restrict__ cu,
                                                       int d, float *__restrict__ out)
{
    __shared__ double red[4];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int start = cu[b], len = cu[b + 1] - start;
    const float wt = 1.0f / (float)len;
    float e[4];
    double ss = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = tid + 256 * j;
        float a = 0.f;
        if (c < d) {
            // (unrolled: eight loads in flight; the fmaf chain keeps its token order)
#pragma unroll 8
            for (int i = 0; i < len; ++i) a = fmaf(x[(size_t)(start + i) * d + c], wt, a);
        }
        e[j] = a;
        ss += (double)(a * a);
    }
    ss = wave_sum_d(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const float nrm = sqrtf((float)((red[0] + red[1]) + (red[2] + red[3])));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = tid + 256 * j;
        if (c < d) out[(size_t)b * d + c] = e[j] / nrm;
    }
}

}  // namespace

void launch_f32_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                         const float *ln_b, const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                         int32_t d, float *x, hipStream_t s)
{
    f32_embed_ln_kernel<<<dim3((max_len + 3) / 4, n_seqs), 256, 0, s>>>(word, type, pos, ln_w, ln_b, ids, cu, d, x);
}

void launch_f32_ln(float *x, int32_t rows, int32_t d, const float *g, const float *b, hipStream_t s)
{
    if (rows > 0) f32_ln_kernel<<<(rows + 3) / 4, 256, 0, s>>>(x, rows, d, g, b);
}

int launch_f32_gemm(const float *X, int32_t M, const float *W, int32_t N, int32_t K, const float *bias, int32_t epi,
                    const float *res, float *Y, hipStream_t s, const uint16_t *gelu_tab)
{
    if (M % 64 || K % F32_BK || N <= 0 || M <= 0 || epi < 0 || epi > 2 || (epi == 2 && !res) ||
        (epi == 1 && !gelu_tab))
        return -1;
    const int nN = (N + F32_BN - 1) / F32_BN, grid = (M / 64) * nN;
    if (epi == 0) f32_gemm_kernel<0><<<grid, 256, 0, s>>>(X, W, bias, res, Y, N, K, nN, gelu_tab);
    else if (epi == 1) f32_gemm_kernel<1><<<grid, 256, 0, s>>>(X, W, bias, res, Y, N, K, nN, gelu_tab);
    else f32_gemm_kernel<2><<<grid, 256, 0, s>>>(X, W, bias, res, Y, N, K, nN, gelu_tab);
    return 0;
}

// Largest dynamic LDS one workgroup may request on the calling thread's device
// (cached per ordinal; gfx950: 160 KiB).
static size_t device_lds_limit()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) { (void)hipGetLastError(); return 65536; }
    if (dev < 64 && cache[dev].load(std::memory_order_relaxed) > 0) return (size_t)cache[dev].load(std::memory_order_relaxed);
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 65536;
    }
    if (dev < 64) cache[dev].store(n, std::memory_order_relaxed);
    return (size_t)n;
}

int launch_f32_attention(const float *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                         int32_t d, float *out, hipStream_t s, const uint16_t *exp_tab)
{
    const int dh = d / n_head;
    if (d % n_head || (dh != 32 && dh != 64) || max_len <= 0 || !exp_tab) return -1;
    const int s_stride = (max_len + 3) / 4 * 4;
    const size_t lds = sizeof(float) * (16 * (size_t)dh + 64 * (size_t)(dh + 1) + 16 * (size_t)s_stride);
    // the 16 score rows live in LDS: refuse (before launching anything) a length
    // whose rows do not fit the device's per-workgroup LDS
    if (lds > device_lds_limit()) return -1;
    const dim3 g((max_len + 15) / 16, n_head, n_seqs);
    const float scale = 1.0f / sqrtf((float)dh);
    if (dh == 64) f32_attention_kernel<64><<<g, 256, lds, s>>>(qkv, cu, d, s_stride, scale, out, exp_tab);
    else f32_attention_kernel<32><<<g, 256, lds, s>>>(qkv, cu, d, s_stride, scale, out, exp_tab);
    return 0;
}

void launch_f32_pool(const float *x, const int32_t *cu, int32_t n_seqs, int32_t d, float *out, hipStream_t s)
{
    f32_pool_kernel<<<n_seqs, 256, 0, s>>>(x, cu, d, out);
}

}  // namespace emb
