// Micro-benchmark for the q8 x q4 integer-dot question (the
// reference's own arithmetic for q4 weights is q8_0 / q8_1 activations x q4 block
// dots, ggml mul_mat at bert.cpp:995).  Register-only MFMA loops on every CU, 4
// waves per SIMD, random operands (DVFS depends on data), device-timed:
//   f16      v_mfma_f32_16x16x32_f16: the production GEMM's instruction (one quant
//            block of 32 k per MFMA, the block scale already in the f16 weights)
//   i8       v_mfma_i32_16x16x64_i8 with nothing else: the 2x ceiling, valid only
//            if both operands shared one scale per 64 k (they do not: blocks are 32)
//   i8_blk   the same instruction doing ONE 32-k block (the other half of K zero,
//            since per-block scales cannot ride inside the MFMA) and the scale
//            applied per block in f32: cvt i32 -> f32 and an FMA by d_w[n] d_x[m]
//            for each of the 4 outputs a lane holds (the products per lane: 4 MULs)
// Prints one JSON line per form: useful TFLOP/s (2 x M x N x useful K per MFMA).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int NACC = 8, ITERS = 4096;

__global__ __launch_bounds__(256) void k_f16(const float *seed, float *out)
{
    const int t = threadIdx.x;
    h16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)seed[(t + i) & 255]; b[i] = (_Float16)seed[(t * 3 + i) & 255]; }
    f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
    float s = 0.f;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + t] = s;
}

__global__ __launch_bounds__(256) void k_i8(const float *seed, float *out)
{
    const int t = threadIdx.x;
    i32x4 a, b;
    for (int i = 0; i < 4; ++i) { a[i] = (int)(seed[(t + i) & 255] * 1e6f); b[i] = (int)(seed[(t * 5 + i) & 255] * 1e6f); }
    i32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = i32x4{0, 0, 0, 0};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[j], 0, 0, 0);
    int s = 0;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + t] = (float)s;
}

__global__ __launch_bounds__(256) void k_i8_blk(const float *seed, float *out)
{
    const int t = threadIdx.x;
    i32x4 a, b[NACC];
    // one 32-k block per MFMA: the lanes holding k 32..63 carry zeros; a distinct B
    // operand per accumulator (as the token groups of a GEMM tile)
    const bool lo = (t & 63) < 32;
    for (int i = 0; i < 4; ++i) a[i] = lo ? (int)(seed[(t + i) & 255] * 1e6f) : 0;
    for (int j = 0; j < NACC; ++j)
        for (int i = 0; i < 4; ++i) b[j][i] = lo ? (int)(seed[(t * 5 + i + 7 * j) & 255] * 1e6f) : 0;
    f32x4 dw = {seed[t & 255], seed[(t + 1) & 255], seed[(t + 2) & 255], seed[(t + 3) & 255]};
    float dx = seed[(t + 7) & 255];
    f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < ITERS; ++it) {
        // the next K block: new operands (one VALU op keeps the MFMAs in the loop) and scales
        a[0] += it;
        dx = dx * 1.0000001f;
        f32x4 sc;
#pragma unroll
        for (int e = 0; e < 4; ++e) sc[e] = dw[e] * dx;
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            const i32x4 p = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[j], i32x4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][e] = __builtin_fmaf((float)p[e], sc[e], acc[j][e]);
        }
    }
    float s = 0.f;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + t] = s;
}

int main()
{
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 4;   // 4 workgroups x 4 waves per CU = 4 waves per SIMD
    float *seed = nullptr, *out = nullptr;
    (void)hipMalloc(&seed, 256 * 4);
    (void)hipMalloc(&out, (size_t)grid * 256 * 4);
    float h[256];
    unsigned st = 12345u;
    for (auto &v : h) { st = st * 1664525u + 1013904223u; v = ((st >> 8) / 16777216.0f - 0.5f) * 0.25f; }
    (void)hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const double waves = (double)grid * 4;
    struct Form { const char *name; void (*k)(const float *, float *); double flop_per_mfma; };
    const Form forms[] = {{"f16 v_mfma_f32_16x16x32_f16 (one q4 block per MFMA, scale in the weights)", k_f16,
                           2.0 * 16 * 16 * 32},
                          {"i8 v_mfma_i32_16x16x64_i8, no scales (ceiling: needs one scale per 64 k)", k_i8,
                           2.0 * 16 * 16 * 64},
                          {"i8_blk v_mfma_i32_16x16x64_i8 on one 32-k block + per-block f32 rescale", k_i8_blk,
                           2.0 * 16 * 16 * 32}};
    for (const Form &f : forms) {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(f.k, dim3(grid), dim3(256), 0, 0, seed, out);
        (void)hipEventRecord(a, 0);
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(f.k, dim3(grid), dim3(256), 0, 0, seed, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        const double flop = 5.0 * waves * ITERS * NACC * f.flop_per_mfma;
        std::printf("{\"form\": \"%s\", \"useful_tflops\": %.1f, \"ms\": %.3f}\n", f.name, flop / (ms * 1e-3) / 1e12,
                    ms / 5);
    }
    (void)hipFree(seed);
    (void)hipFree(out);
    return 0;
}
