// Memory-bound row kernels: embeddings + LayerNorm, the LayerNorm statistics
// of the residual stream, mean pool + L2 (the LN fold of kernels.h).
// Embeddings: one 32-lane group per token row, one 32-wide quant block per lane,
// reductions by shuffles.
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"
#include "table_read.h"

#include <cmath>
#include <cstdlib>

namespace emb {

namespace {


// One row per 32-lane group, one 32-wide quant block per lane (8 rows per 256-thread
// block, n_embd <= 1024): each lane reads its block of the three tables with a few
// wide loads (table_read.h) and keeps the 32 f32 values in registers, the two
// reductions are xor-shuffles inside the group.  No LDS and no barrier, so a row
// costs one dependent load chain (ids -> table rows) and the loads of every row in
// flight at once (the LDS-staged form with 16 rows per block: 48 us at C3, 16 us for
// one 32-token sentence).  TF >= 0: the three tables share format TF (the usual
// case; the format switch resolves at compile time and the kernel holds only that
// format's words: 4x the resident waves of the any-format form's 124 VGPRs).
template <int TF>
__device__ __forceinline__ void emb_table32(const DevTable &t, int row, int b, float (&r)[32])
{
    if constexpr (TF < 0) {
        table32(t, row, b, r);
    } else {
        DevTable u = t;
        u.fmt = TF;
        table32(u, row, b, r);
    }
}

__device__ __forceinline__ float sum32(float v)
{
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// resident waves per SIMD the register budget is held to (no spills at these)
constexpr int emb_occ(int tf) { return tf == FMT_Q4_0 || tf == FMT_F16 ? 8 : tf < 0 ? 4 : 6; }

template <int TF>
__global__ __launch_bounds__(256, emb_occ(TF)) void embed_ln_kernel(DevTable word, DevTable type, DevTable pos,
                                                       const float *__restrict__ ln_w, const int32_t *__restrict__ ids,
                                                       const int32_t *__restrict__ cu, int d, h16 *__restrict__ z,
                                                       float2 *__restrict__ stats)
{
    const int b = blockIdx.y, l32 = threadIdx.x & 31;
    const int start = cu[b], len = cu[b + 1] - start;
    const int i = blockIdx.x * 8 + (threadIdx.x >> 5);
    if (i >= len) return;                          // whole 32-lane groups: the shuffles stay in-group
    const int t = start + i;
    const bool act = l32 < d / 32;
    float v[32];
    float s = 0.f;
    if (act) {
        // pos + (type[0] + word[id]) in the reference's operand order (bert.cpp:968-973), f32
        // (one table at a time into a 32-value temporary: 64 live values, not 128)
        float tmp[32];
        emb_table32<TF>(word, ids[t], l32, v);
        emb_table32<TF>(type, 0, l32, tmp);
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] = tmp[e] + v[e];
        emb_table32<TF>(pos, i, l32, tmp);
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] = tmp[e] + v[e];
#pragma unroll
        for (int e = 0; e < 32; e += 4) s += (v[e] + v[e + 1]) + (v[e + 2] + v[e + 3]);
    }
    // ggml_norm (eps 1e-5, mean then centred variance; bert.cpp:977-984) of the f32 row
    const float mean = sum32(s) / (float)d;
    float s2 = 0.f;
    if (act) {
#pragma unroll
        for (int e = 0; e < 32; ++e) { const float u = v[e] - mean; s2 += u * u; }
    }
    const float r = 1.0f / sqrtf(sum32(s2) / (float)d + 1e-5f);
    if (act) {
        const f32x4 *g4 = (const f32x4 *)(ln_w + 32 * l32);
        h16x8 *dst = (h16x8 *)(z + (size_t)t * d + 32 * l32);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 g0 = g4[2 * q], g1 = g4[2 * q + 1];
            h16x8 zh;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                zh[e] = (h16)(v[8 * q + e] * g0[e]);
                zh[4 + e] = (h16)(v[8 * q + 4 + e] * g1[e]);
            }
            dst[q] = zh;                            // the stream as z = y * gamma (kernels.h LN fold)
        }
    }
    if (l32 == 0) stats[t] = float2{mean, r};
}

// Row statistics from the residual GEMM's 32-feature group partials (sum, M2 about
// the group mean): mean = sum / d, M2 = sum_g M2_g + (s_g - 32 mean)^2 / 32 (Chan
// et al.).  One thread per row, its G partials loaded at once (G <= 32, unrolled:
// every load in flight before the first add), 64-row blocks so short batches still
// spread over the CUs; reads part[g][rows] coalesced along the rows.
// Row block of workgroup b, XCD-aware: workgroups are dealt to the 8 XCDs round
// robin, and XCD x takes the x-th eighth of the row blocks -- the rows whose
// partials the residual GEMM's tiles on XCD x just wrote (gemm.hip remaps its
// tiles the same way, panel-major), and whose statistics the next GEMM's tiles
// on XCD x read: both stay in that XCD's L2.
__device__ __forceinline__ int xcd_block(int b, int nb)
{
    const int xcd = b & 7, qq = nb >> 3, rr = nb & 7;
    return (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
}

__global__ __launch_bounds__(64) void ln_stats_any(const float2 *__restrict__ part, int G, int stride, int rows,
                                                   int d, float2 *__restrict__ stats)
{
    const int t = xcd_block(blockIdx.x, gridDim.x) * 64 + threadIdx.x;
    if (t >= rows) return;
    float2 p[32];
#pragma unroll
    for (int g = 0; g < 32; ++g)
        if (g < G) p[g] = part[(size_t)g * stride + t];
    stats[t] = ln_row_stats<32>(p, G, d);
}

template <int G>
__global__ __launch_bounds__(64) void ln_stats_kernel(const float2 *__restrict__ part, int stride, int rows, int d,
                                                      float2 *__restrict__ stats)
{
    const int t = xcd_block(blockIdx.x, gridDim.x) * 64 + threadIdx.x;
    if (t >= rows) return;
    float2 p[G];
#pragma unroll
    for (int g = 0; g < G; ++g) p[g] = part[(size_t)g * stride + t];
    stats[t] = ln_row_stats<G>(p, G, d);
}

// pool stage 1: partial column sums of 64-token chunks, weights 1/len
// (bert.cpp:1087-1089: sum_i X[i][c] * (1/len)).
constexpr int POOL_CHUNK = 64;

// Column sums of chunk ch of sentence b: thread t owns 8 columns (16-B loads)
// of every TT-th token of the chunk: column group t % G (G = d / 8 <= 128),
// token lane t / G; the token lanes are summed through LDS in a fixed order,
// the result in (s0, s1) of threads t < G (columns 8t .. 8t + 7).
template <int UNR>
__device__ __forceinline__ void pool_chunk_sum(const h16 *__restrict__ z, const float2 *__restrict__ stats,
                                               const float *__restrict__ lw, const float *__restrict__ lb,
                                               const int32_t *__restrict__ cu, int d, int b, int ch, f32x4 &s0,
                                               f32x4 &s1)
{
    __shared__ f32x4 red[256][2];
    const int tid = threadIdx.x;
    const int start = cu[b], len = cu[b + 1] - start;
    const int i0 = ch * POOL_CHUNK, i1 = min(len, i0 + POOL_CHUNK);
    const int G = d / 8, TT = 256 / G, cg = tid % G, tl = tid / G;
    const float wt = 1.0f / (float)len;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    if (tl < TT) {
        const int c = 8 * cg;
        const f32x4 w0 = *(const f32x4 *)(lw + c), w1 = *(const f32x4 *)(lw + c + 4);
        const f32x4 b0 = *(const f32x4 *)(lb + c), b1 = *(const f32x4 *)(lb + c + 4);
#pragma unroll UNR
        for (int i = i0 + tl; i < i1; i += TT) {
            const h16x8 y = *(const h16x8 *)(z + (size_t)(start + i) * d + c);
            const float2 st = stats[start + i];
            const float r = st.y, t0 = -st.x * st.y;
            // LN(y) = r z - r mean gamma + beta (kernels.h LN fold)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                a0[e] += fmaf(r, (float)y[e], fmaf(t0, w0[e], b0[e])) * wt;
                a1[e] += fmaf(r, (float)y[4 + e], fmaf(t0, w1[e], b1[e])) * wt;
            }
        }
    }
    red[tid][0] = a0;
    red[tid][1] = a1;
    __syncthreads();
    if (tid < G) {
        s0 = red[tid][0];
        s1 = red[tid][1];
        for (int k = 1; k < TT; ++k) {
            s0 += red[tid + k * G][0];
            s1 += red[tid + k * G][1];
        }
    }
}

// Sum the n_chunks column-sum rows of one sentence (part[k * d + c]) and
// divide by the L2 norm (bert.cpp:1092-1095).
template <bool HOIST>
__device__ __forceinline__ void pool_normalize(const float *part, int d, int n_chunks, float *__restrict__ out)
{
    __shared__ float red[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float e[4];
    float ss = 0.f;
    int ne = 0;
    for (int c = tid; c < d; c += 256) {
        float v = 0.f;
        if constexpr (HOIST) {
            // global partials: the first 16 chunks' values loaded before the first
            // add (the serial load-add loop was 8 us at C3), summed in chunk order
            float pv[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < n_chunks) pv[k] = part[(size_t)k * d + c];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < n_chunks) v += pv[k];
            for (int k = 16; k < n_chunks; ++k) v += part[(size_t)k * d + c];
        } else {
            for (int k = 0; k < n_chunks; ++k) v += part[(size_t)k * d + c];
        }
        e[ne++] = v;
        ss += v * v;
    }
    ss = wave_sum(ss);
    if (lane == 0) red[w] = ss;
    __syncthreads();
    const float nrm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    ne = 0;
    for (int c = tid; c < d; c += 256) out[c] = e[ne++] / nrm;
}

// pool stage 1: partial column sums of 64-token chunks, weights 1/len
// (bert.cpp:1087-1089: sum_i X[i][c] * (1/len)).
__global__ __launch_bounds__(256) void pool_partial_kernel(const h16 *__restrict__ z, const float2 *__restrict__ stats,
                                                           const float *__restrict__ lw, const float *__restrict__ lb,
                                                           const int32_t *__restrict__ cu, int d, int n_chunks,
                                                           float *__restrict__ part)
{
    const int b = blockIdx.y, ch = blockIdx.x, tid = threadIdx.x;
    f32x4 s0, s1;
    pool_chunk_sum<8>(z, stats, lw, lb, cu, d, b, ch, s0, s1);   // 32 tokens per thread at L 512
    if (tid < d / 8) {
        float *dst = part + ((size_t)b * n_chunks + ch) * d + 8 * tid;
        *(f32x4 *)dst = s0;
        *(f32x4 *)(dst + 4) = s1;
    }
}

// pool stage 2: sum the chunks, divide by the L2 norm
__global__ __launch_bounds__(256) void pool_final_kernel(const float *__restrict__ part, int d, int n_chunks,
                                                         float *__restrict__ out)
{
    const int b = blockIdx.x;
    pool_normalize<true>(part + (size_t)b * n_chunks * d, d, n_chunks, out + (size_t)b * d);
}

// Batches of at most POOL_ONE_MAX chunks (max_len <= 256): both stages in one
// launch, a sentence's chunks summed one after another by its workgroup and the
// column sums kept in LDS instead of HBM -- the same arithmetic and order as the
// two kernels above (so the same bits), one launch fewer (C2: L 128).
constexpr int POOL_ONE_MAX = 4;
__global__ __launch_bounds__(256) void pool_one_kernel(const h16 *__restrict__ z, const float2 *__restrict__ stats,
                                                       const float *__restrict__ lw, const float *__restrict__ lb,
                                                       const int32_t *__restrict__ cu, int d, int n_chunks,
                                                       float *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) float cs[POOL_ONE_MAX * 1024];
    const int b = blockIdx.x, tid = threadIdx.x;
    for (int ch = 0; ch < n_chunks; ++ch) {
        f32x4 s0, s1;
        pool_chunk_sum<4>(z, stats, lw, lb, cu, d, b, ch, s0, s1);
        if (tid < d / 8) {
            *(f32x4 *)(cs + ch * d + 8 * tid) = s0;
            *(f32x4 *)(cs + ch * d + 8 * tid + 4) = s1;
        }
        __syncthreads();   // pool_chunk_sum's reduction buffer is reused by the next chunk
    }
    pool_normalize<false>(cs, d, n_chunks, out + (size_t)b * d);
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
                     const int32_t *ids, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t d, uint16_t *z,
                     float2 *stats, hipStream_t s)
{
    dim3 grid((max_len + 7) / 8, n_seqs);
    const int f = word.fmt == type.fmt && word.fmt == pos.fmt ? word.fmt : -1;
#define EMB_LAUNCH(TF) embed_ln_kernel<TF><<<grid, 256, 0, s>>>(word, type, pos, ln_w, ids, cu, d, (h16 *)z, stats)
    switch (f) {
    case FMT_F32: EMB_LAUNCH(FMT_F32); break;
    case FMT_F16: EMB_LAUNCH(FMT_F16); break;
    case FMT_Q4_0: EMB_LAUNCH(FMT_Q4_0); break;
    case FMT_Q4_1: EMB_LAUNCH(FMT_Q4_1); break;
    case FMT_Q8_0: EMB_LAUNCH(FMT_Q8_0); break;
    default: EMB_LAUNCH(-1); break;
    }
#undef EMB_LAUNCH
}

int launch_ln_stats(const float2 *part, int32_t G, int32_t stride, int32_t rows, int32_t d, float2 *stats,
                    hipStream_t s)
{
    // the kernels hold at most 32 partials per row (d <= 1024): a wider row would
    // silently drop groups, so it is refused
    if (G <= 0 || G > 32 || d != 32 * G) return -1;
    if (rows <= 0) return 0;
    const int nb = (rows + 63) / 64;
    switch (G) {
    case 12: ln_stats_kernel<12><<<nb, 64, 0, s>>>(part, stride, rows, d, stats); break;   // d 384
    case 16: ln_stats_kernel<16><<<nb, 64, 0, s>>>(part, stride, rows, d, stats); break;
    case 24: ln_stats_kernel<24><<<nb, 64, 0, s>>>(part, stride, rows, d, stats); break;   // d 768
    case 32: ln_stats_kernel<32><<<nb, 64, 0, s>>>(part, stride, rows, d, stats); break;   // d 1024
    default:
        // other widths (d % 64 == 0, d <= 1024): the same arithmetic (ln_row_stats)
        ln_stats_any<<<nb, 64, 0, s>>>(part, G, stride, rows, d, stats);
        break;
    }
    return 0;
}

int32_t pool_chunks(int32_t max_len) { return (max_len + POOL_CHUNK - 1) / POOL_CHUNK; }

void launch_pool_l2(const uint16_t *z, const float2 *stats, const float *ln_w, const float *ln_b, const int32_t *cu,
                    int32_t n_seqs, int32_t max_len, int32_t d, float *partial, float *out, hipStream_t s)
{
    const int nc = pool_chunks(max_len);
    // BERT_POOL_ONE=0: the two launches for every batch (A/B)
    static const bool one = [] { const char *e = std::getenv("BERT_POOL_ONE"); return !(e && *e == '0'); }();
    if (nc == 1 || (one && nc <= POOL_ONE_MAX && d <= 1024)) {
        pool_one_kernel<<<n_seqs, 256, 0, s>>>((const h16 *)z, stats, ln_w, ln_b, cu, d, nc, out);
        return;
    }
    pool_partial_kernel<<<dim3(nc, n_seqs), 256, 0, s>>>((const h16 *)z, stats, ln_w, ln_b, cu, d, nc, partial);
    pool_final_kernel<<<n_seqs, 256, 0, s>>>(partial, d, nc, out);
}

}  // namespace emb
