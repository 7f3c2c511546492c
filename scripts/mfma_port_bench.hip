// Issue-port question for the GEMM's MFMA shape: an MFMA holds its SIMD's vector
// issue for 8 cycles (16 of v_mfma_f32_16x16x32_f16 or 32 of _32x32x16_f16), so
// with F VALU fillers per MFMA a 16x16x32 loop leaves 8 cycles for them and a
// 32x32x16 loop 24 for the same fillers per FLOP.  Register-only loops, random
// data, 2 waves per SIMD (as the production GEMM), fillers = independent
// v_fma_f32 (4 issue cycles each).  Prints one JSON line per (shape, fillers per
// 16x16x32-equivalent MFMA): TFLOP/s.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ITERS = 2048;

template <int F>
__device__ __forceinline__ void fill(float &x0, float &x1, float &x2, float &x3)
{
    if constexpr (F >= 1) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x0));
    if constexpr (F >= 2) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x1));
    if constexpr (F >= 3) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x2));
    if constexpr (F >= 4) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x3));
}

// 16 accumulators of 16x16x32 (a 32-feature x 128-token wave tile's half)
template <int F>
__global__ __launch_bounds__(256, 2) void k16(const float *seed, float *out)
{
    const int t = threadIdx.x;
    h16x8 a, b[8];
    for (int i = 0; i < 8; ++i) a[i] = (_Float16)seed[(t + i) & 255];
    for (int j = 0; j < 8; ++j)
        for (int i = 0; i < 8; ++i) b[j][i] = (_Float16)seed[(t * 3 + i + 5 * j) & 255];
    f32x4 acc[16];
    for (int j = 0; j < 16; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float x0 = seed[t & 255], x1 = x0 * 0.5f, x2 = x0 * 0.25f, x3 = x0 * 0.125f;
    for (int it = 0; it < ITERS; ++it) {
        a[0] += (_Float16)1.0f;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[j & 7], acc[j], 0, 0, 0);
            fill<F>(x0, x1, x2, x3);
        }
    }
    float s = x0 + x1 + x2 + x3;
    for (int j = 0; j < 16; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + t] = s;
}

// 4 accumulators of 32x32x16: the same outputs per wave, half the MFMAs per FLOP
// and twice the fillers per MFMA (2F)
template <int F>
__global__ __launch_bounds__(256, 2) void k32(const float *seed, float *out)
{
    const int t = threadIdx.x;
    h16x8 a, b[4];
    for (int i = 0; i < 8; ++i) a[i] = (_Float16)seed[(t + i) & 255];
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 8; ++i) b[j][i] = (_Float16)seed[(t * 3 + i + 5 * j) & 255];
    f32x16 acc[4];
    for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float x0 = seed[t & 255], x1 = x0 * 0.5f, x2 = x0 * 0.25f, x3 = x0 * 0.125f;
    for (int it = 0; it < ITERS; ++it) {
        a[0] += (_Float16)1.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[j & 3], acc[j & 3], 0, 0, 0);
            fill<F>(x0, x1, x2, x3);
            fill<F>(x0, x1, x2, x3);
        }
    }
    float s = x0 + x1 + x2 + x3;
    for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 16; ++r) s += acc[j][r];
    out[blockIdx.x * 256 + t] = s;
}

int main()
{
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 2;   // 2 workgroups x 4 waves per CU = 2 waves per SIMD
    float *seed = nullptr, *out = nullptr;
    (void)hipMalloc(&seed, 256 * 4);
    (void)hipMalloc(&out, (size_t)grid * 256 * 4);
    float h[256];
    unsigned st = 12345u;
    for (auto &v : h) { st = st * 1664525u + 1013904223u; v = ((st >> 8) / 16777216.0f - 0.5f) * 0.25f; }
    (void)hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double waves = (double)grid * 4;
    // FLOP per wave per iteration: 16 x (16x16x32) = 8 x (32x32x16) = 262144
    const double flop = 5.0 * waves * ITERS * 16 * 2.0 * 16 * 16 * 32;
    struct Form { const char *shape; int f; void (*k)(const float *, float *); };
    const Form forms[] = {{"16x16x32", 0, k16<0>}, {"16x16x32", 1, k16<1>}, {"16x16x32", 2, k16<2>},
                          {"16x16x32", 3, k16<3>}, {"16x16x32", 4, k16<4>}, {"32x32x16", 0, k32<0>},
                          {"32x32x16", 1, k32<1>}, {"32x32x16", 2, k32<2>}, {"32x32x16", 3, k32<3>},
                          {"32x32x16", 4, k32<4>}};
    for (int pass = 0; pass < 2; ++pass)
        for (const Form &f : forms) {
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(f.k, dim3(grid), dim3(256), 0, 0, seed, out);
            (void)hipEventRecord(e0, 0);
            for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(f.k, dim3(grid), dim3(256), 0, 0, seed, out);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::printf("{\"pass\": %d, \"shape\": \"%s\", \"fillers_per_16x16x32\": %d, \"tflops\": %.1f}\n", pass,
                        f.shape, f.f, flop / (ms * 1e-3) / 1e12);
        }
    (void)hipFree(seed);
    (void)hipFree(out);
    return 0;
}
