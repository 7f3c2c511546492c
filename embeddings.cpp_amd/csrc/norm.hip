// Memory-bound row kernels: embeddings + LayerNorm, LayerNorm, mean pool + L2.
// One wave per token row; each lane owns 4 consecutive features per 256-wide
// slice (16-B loads and stores), reductions by wave shuffles.
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"
#include "rowln.h"

#include <cmath>

namespace emb {

namespace {

constexpr int MAXV = 4;   // 4 slices x 256 features = n_embd <= 1024

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

__global__ __launch_bounds__(256) void embed_ln_kernel(DevTable word, DevTable type, DevTable pos,
                                                       const float *__restrict__ ln_w, const float *__restrict__ ln_b,
                                                       const int32_t *__restrict__ ids, const int32_t *__restrict__ cu,
                                                       int d, h16 *__restrict__ yh, h16 *__restrict__ xh,
                                                       float2 *__restrict__ stats)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int start = cu[b], len = cu[b + 1] - start;
    if (i >= len) return;
    const int t = start + i, id = ids[t];
    f32x4 v[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (c < d) {
            // pos + (type[0] + word[id])  (bert.cpp:968-973 operand order)
            const f32x4 w = table4(word, id, c), ty = table4(type, 0, c), p = table4(pos, i, c);
            h16x4 v16;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v16[e] = (h16)(p[e] + (ty[e] + w[e]));
                v[k][e] = (float)v16[e];       // LN of the stored (f16) residual value
            }
            *(h16x4 *)(yh + (size_t)t * d + c) = v16;            // pre-LN residual stream
        }
    }
    ln_row<MAXV>(v, d, lane, ln_w, ln_b, xh + (size_t)t * d, stats + t);
}

// 32 rows per 256-thread block, 8 lanes per row (as layernorm_kernel): lane sub
// of a row group gathers the 16-B chunks at features 8 sub + 64 k of the three
// tables, so a wave has 8 rows' gathers in flight (the one-wave-per-row kernel
// above has one), then ln8_row normalises the f16-rounded residual row.
__global__ __launch_bounds__(256) void embed_ln8_kernel(DevTable word, DevTable type, DevTable pos,
                                                        const float *__restrict__ ln_w, const float *__restrict__ ln_b,
                                                        const int32_t *__restrict__ ids, const int32_t *__restrict__ cu,
                                                        int d, h16 *__restrict__ yh, h16 *__restrict__ xh,
                                                        float2 *__restrict__ stats)
{
    const int b = blockIdx.y, sub = threadIdx.x & 7;
    const int i = blockIdx.x * 32 + (threadIdx.x >> 3);
    const int start = cu[b], len = cu[b + 1] - start;
    const bool valid = i < len;
    const int t = start + (valid ? i : 0);
    h16x8 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = h16x8{};
    if (valid) {
        const int id = ids[t];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int c = 8 * sub + 64 * k;
            if (64 * k >= d) continue;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                // pos + (type[0] + word[id])  (bert.cpp:968-973 operand order)
                const f32x4 w = table4(word, id, c + 4 * hf), ty = table4(type, 0, c + 4 * hf),
                            p = table4(pos, i, c + 4 * hf);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[k][4 * hf + e] = (h16)(p[e] + (ty[e] + w[e]));
            }
            *(h16x8 *)(yh + (size_t)t * d + c) = v[k];       // pre-LN residual stream
        }
    }
    ln8_row<16>(v, t, valid, d, sub, ln_w, ln_b, xh, stats);
}

// 32 rows per 256-thread block, 8 lanes per row (rowln.h ln8_*: the same
// arithmetic as the panel LN fused into the residual GEMM)
__global__ __launch_bounds__(256) void layernorm_kernel(const h16 *__restrict__ y, int T, int d,
                                                        const float *__restrict__ w, const float *__restrict__ b,
                                                        h16 *__restrict__ xh, float2 *__restrict__ stats)
{
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 32 + (threadIdx.x >> 3);
    h16x8 v[16];
    ln8_load<16>(y, t, t < T, d, lane & 7, v);
    ln8_row<16>(v, t, t < T, d, lane & 7, w, b, xh, stats);
}

// Persistent form (A/B via BERT_LN_BLOCKS, measured slower): block b normalises
// the 32-aligned row range [b rpb, min(T, (b + 1) rpb)), its 4 waves 8 rows each
// per pass with the next pass's loads issued before this pass's arithmetic
// (rowln.h ln_rows), so the reads and writes of one launch overlap.  The same
// ln8_row arithmetic as the one-pass kernel above, so the same bits.
template <int NCH>
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const h16 *__restrict__ y, int T, int d, int rpb,
                                                             const float *__restrict__ w, const float *__restrict__ b,
                                                             h16 *__restrict__ xh, float2 *__restrict__ stats)
{
    const int r0 = blockIdx.x * rpb;
    ln_rows<NCH, 4>(y, r0, min(T, r0 + rpb), d, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x & 63,
                    w, b, xh, stats);
}

// pool stage 1: partial column sums of 64-token chunks, weights 1/len
// (bert.cpp:1087-1089: sum_i X[i][c] * (1/len)).
constexpr int POOL_CHUNK = 64;

__global__ __launch_bounds__(256) void pool_partial_kernel(const h16 *__restrict__ y32, const float2 *__restrict__ stats,
                                                           const float *__restrict__ lw, const float *__restrict__ lb,
                                                           const int32_t *__restrict__ cu, int d, int n_chunks,
                                                           float *__restrict__ part)
{
    // thread t owns 8 columns (16-B loads) of every TT-th token of the chunk:
    // column group t % G (G = d / 8 <= 128), token lane t / G; the token lanes
    // are summed through LDS in a fixed order
    __shared__ f32x4 red[256][2];
    const int b = blockIdx.y, ch = blockIdx.x, tid = threadIdx.x;
    const int start = cu[b], len = cu[b + 1] - start;
    const int i0 = ch * POOL_CHUNK, i1 = min(len, i0 + POOL_CHUNK);
    const int G = d / 8, TT = 256 / G, cg = tid % G, tl = tid / G;
    const float wt = 1.0f / (float)len;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    if (tl < TT) {
        const int c = 8 * cg;
        const f32x4 w0 = *(const f32x4 *)(lw + c), w1 = *(const f32x4 *)(lw + c + 4);
        const f32x4 b0 = *(const f32x4 *)(lb + c), b1 = *(const f32x4 *)(lb + c + 4);
#pragma unroll 4
        for (int i = i0 + tl; i < i1; i += TT) {
            const h16x8 y = *(const h16x8 *)(y32 + (size_t)(start + i) * d + c);
            const float2 st = stats[start + i];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                a0[e] += ln_apply((float)y[e], st.x, st.y, w0[e], b0[e]) * wt;
                a1[e] += ln_apply((float)y[4 + e], st.x, st.y, w1[e], b1[e]) * wt;
            }
        }
    }
    red[tid][0] = a0;
    red[tid][1] = a1;
    __syncthreads();
    if (tid < G) {
        f32x4 s0 = red[tid][0], s1 = red[tid][1];
        for (int k = 1; k < TT; ++k) {
            s0 += red[tid + k * G][0];
            s1 += red[tid + k * G][1];
        }
        float *dst = part + ((size_t)b * n_chunks + ch) * d + 8 * tid;
        *(f32x4 *)dst = s0;
        *(f32x4 *)(dst + 4) = s1;
    }
}

// pool stage 2: sum the chunks, divide by the L2 norm (bert.cpp:1092-1095)
__global__ __launch_bounds__(256) void pool_final_kernel(const float *__restrict__ part, int d, int n_chunks,
                                                         float *__restrict__ out)
{
    __shared__ float red[4];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float e[4];
    float ss = 0.f;
    int ne = 0;
    for (int c = tid; c < d; c += 256) {
        float v = 0.f;
        for (int k = 0; k < n_chunks; ++k) v += part[((size_t)b * n_chunks + k) * d + c];
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

// diagnostics (BERT_CHECK_FINITE): count non-finite values of a buffer
__global__ void count_nonfinite_kernel(const void *p, size_t n, int f16, unsigned *cnt)
{
    unsigned c = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float v = f16 ? (float)((const h16 *)p)[i] : ((const float *)p)[i];
        c += !__builtin_isfinite(v);
    }
    if (c) atomicAdd(cnt, c);
}

}  // namespace

void launch_count_nonfinite(const void *p, size_t n, int f16, unsigned *cnt, hipStream_t s)
{
    count_nonfinite_kernel<<<1024, 256, 0, s>>>(p, n, f16, cnt);
}

void launch_embed_ln(const DevTable &word, const DevTable &type, const DevTable &pos, const float *ln_w,
                     const float *ln_b, const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                     int32_t d, uint16_t *yh, uint16_t *xh, float2 *stats, hipStream_t s)
{
    // the one-wave-per-row kernel by default; BERT_EMBED_LN8=1 (A/B) runs the
    // 8-lanes-per-row form, measured no faster (53.0 vs 51.9 us at C3, gpurun_out r01j:
    // the table gathers, not the row sums, bound it)
    static const bool rowwave = [] { const char *e = std::getenv("BERT_EMBED_LN8"); return !(e && *e == '1'); }();
    if (rowwave) {
        dim3 grid((max_len + 3) / 4, n_seqs);
        embed_ln_kernel<<<grid, 256, 0, s>>>(word, type, pos, ln_w, ln_b, ids, cu, d, (h16 *)yh, (h16 *)xh, stats);
        return;
    }
    dim3 grid((max_len + 31) / 32, n_seqs);
    embed_ln8_kernel<<<grid, 256, 0, s>>>(word, type, pos, ln_w, ln_b, ids, cu, d, (h16 *)yh, (h16 *)xh, stats);
}

void launch_layernorm(const uint16_t *yh, int32_t T, int32_t d, const float *w, const float *b, uint16_t *xh,
                      float2 *stats, hipStream_t s)
{
    if (T <= 0) return;
    // BERT_LN_BLOCKS (A/B): n > 0 runs the persistent form on n blocks (-1: two per
    // CU); default the one-pass kernel, measured faster in the forward at C3
    // (gpurun_out r01h: 21.8 vs 22.7 us at two blocks per CU)
    static const int nblk = [] {
        const char *e = std::getenv("BERT_LN_BLOCKS");
        const int n = e ? std::atoi(e) : 0;
        if (n >= 0) return n;
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return 2 * cus;
    }();
    if (nblk <= 0) {
        layernorm_kernel<<<(T + 31) / 32, 256, 0, s>>>((const h16 *)yh, T, d, w, b, (h16 *)xh, stats);
        return;
    }
    const int rpb = ((T + nblk - 1) / nblk + 31) & ~31;
    const int grid = (T + rpb - 1) / rpb;
    const h16 *y = (const h16 *)yh;
    h16 *o = (h16 *)xh;
    switch (d / 64) {
    case 6: layernorm_rows_kernel<6><<<grid, 256, 0, s>>>(y, T, d, rpb, w, b, o, stats); break;
    case 12: layernorm_rows_kernel<12><<<grid, 256, 0, s>>>(y, T, d, rpb, w, b, o, stats); break;
    default: layernorm_rows_kernel<16><<<grid, 256, 0, s>>>(y, T, d, rpb, w, b, o, stats); break;
    }
}

int32_t pool_chunks(int32_t max_len) { return (max_len + POOL_CHUNK - 1) / POOL_CHUNK; }

void launch_pool_l2(const uint16_t *yh, const ResLN &ln, const int32_t *cu, int32_t n_seqs, int32_t max_len,
                    int32_t d, float *partial, float *out, hipStream_t s)
{
    const int nc = pool_chunks(max_len);
    pool_partial_kernel<<<dim3(nc, n_seqs), 256, 0, s>>>((const h16 *)yh, ln.stats, ln.w, ln.b, cu, d, nc, partial);
    pool_final_kernel<<<n_seqs, 256, 0, s>>>(partial, d, nc, out);
}

}  // namespace emb
