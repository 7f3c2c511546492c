// Device-side helpers shared by the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace emb {

typedef _Float16 h16;
typedef h16 h16x8 __attribute__((ext_vector_type(8)));
typedef h16 h16x4 __attribute__((ext_vector_type(4)));
typedef h16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// v_permlane32_swap: lanes l and l ^ 32 of a and b trade places (the s_nop
// covers the VALU-write -> permlane hazard the compiler does not see in asm)
__device__ __forceinline__ void swap32(float &a, float &b)
{
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
// x combined over both 32-lane halves (lanes l and l ^ 32)
__device__ __forceinline__ float halves_max(float x)
{
    float a = x, b = x;
    swap32(a, b);
    return fmaxf(a, b);
}
__device__ __forceinline__ float halves_sum(float x)
{
    float a = x, b = x;
    swap32(a, b);
    return a + b;
}

// LDS byte address of a pointer into __shared__ memory
__device__ __forceinline__ uint32_t lds_u32(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)p;
}

__device__ __forceinline__ h16x2 as_h2(uint32_t u) { return __builtin_bit_cast(h16x2, u); }
__device__ __forceinline__ h16 as_h(uint16_t u) { return __builtin_bit_cast(h16, u); }
// (x & vmask) | smagic as ONE v_and_or_b32: gfx9 VOP3 encodes no literal and reads at
// most one SGPR, so the compiler splits the two-constant form into v_and + v_or;
// here the mask lives in a VGPR (hoisted) and the magic in an SGPR.
__device__ __forceinline__ uint32_t and_or_vs(uint32_t x, uint32_t vmask, uint32_t smagic)
{
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(vmask), "s"(smagic));
    return r;
}

// ggml-era GELU (tanh form) on an f16-rounded input, result rounded to f16 --
// the value ggml's GGML_GELU_FP16 table holds (bert.cpp:1063).  Evaluated as
// 0.5 x (1 + tanh(u)) = x / (1 + exp(-2u)), well inside f16 rounding.
__device__ __forceinline__ h16 gelu_era(float v)
{
    const float x = (float)(h16)v;
    const float u2 = -2.0f * 1.4426950408889634f * 0.79788456080286535587989211986876f;   // -2 log2(e) sqrt(2/pi)
    const float e = __builtin_amdgcn_exp2f(u2 * x * (1.0f + 0.044715f * x * x));
    return (h16)(x * __builtin_amdgcn_rcpf(1.0f + e));
}

// Two GELUs in packed f16 (the epilogue form): x = f16(v) as the era table's
// input, then x * sigmoid(2u) with z = -2 log2(e) u evaluated in f16 pairs, one
// f16 exp2 and one f16 rcp per element.  Within 10 f16 ulps of the table
// (mean 0.5 ulp, |x| < 12); returns the two f16 results packed.
__device__ __forceinline__ uint32_t gelu2_era(float a, float b)
{
    const h16x2 x = {(h16)a, (h16)b};
    const h16 c0 = (h16)(-2.0f * 1.4426950408889634f * 0.7978845608028654f);
    const h16 c1 = (h16)(-2.0f * 1.4426950408889634f * 0.7978845608028654f * 0.044715f);
    const h16x2 C0 = {c0, c0}, C1 = {c1, c1}, ONE = {(h16)1.0f, (h16)1.0f};
    const h16x2 z = x * (x * x * C1 + C0);
    const h16x2 d = __builtin_elementwise_exp2(z) + ONE;
    h16x2 r;
    r.x = __builtin_amdgcn_rcph(d.x);
    r.y = __builtin_amdgcn_rcph(d.y);
    return __builtin_bit_cast(uint32_t, x * r);
}

// Eight GELUs (four f16 pairs, the epilogue form): the arithmetic of gelu2_era
// in one asm block, the four pairs interleaved so that no dependent
// instruction follows its producer directly (no hazard wait states), and the
// high halves of exp / rcp written in place by SDWA (no repacking).  o[i] =
// the f16 pair gelu(v[2i]), gelu(v[2i+1]).
__device__ __forceinline__ void gelu8_era(const float (&v)[8], uint32_t (&o)[4])
{
    const h16 c0 = (h16)(-2.0f * 1.4426950408889634f * 0.7978845608028654f);
    const h16 c1 = (h16)(-2.0f * 1.4426950408889634f * 0.7978845608028654f * 0.044715f);
    const uint32_t C1 = __builtin_bit_cast(uint32_t, h16x2{c1, c1});
    const uint32_t C0 = __builtin_bit_cast(uint32_t, h16x2{c0, c0});
    const uint32_t ONE = 0x3C003C00u;
    uint32_t x0, x1, x2, x3, t0, t1, t2, t3;
    asm volatile(
        "s_nop 1\n\t"
        "v_cvt_pk_f16_f32 %4, %12, %13\n\tv_cvt_pk_f16_f32 %5, %14, %15\n\t"
        "v_cvt_pk_f16_f32 %6, %16, %17\n\tv_cvt_pk_f16_f32 %7, %18, %19\n\t"
        "v_pk_mul_f16 %8, %4, %4\n\tv_pk_mul_f16 %9, %5, %5\n\t"
        "v_pk_mul_f16 %10, %6, %6\n\tv_pk_mul_f16 %11, %7, %7\n\t"
        "v_pk_fma_f16 %8, %8, %20, %21\n\tv_pk_fma_f16 %9, %9, %20, %21\n\t"
        "v_pk_fma_f16 %10, %10, %20, %21\n\tv_pk_fma_f16 %11, %11, %20, %21\n\t"
        "v_pk_mul_f16 %8, %8, %4\n\tv_pk_mul_f16 %9, %9, %5\n\t"
        "v_pk_mul_f16 %10, %10, %6\n\tv_pk_mul_f16 %11, %11, %7\n\t"
        "v_exp_f16_e32 %0, %8\n\tv_exp_f16_e32 %1, %9\n\tv_exp_f16_e32 %2, %10\n\tv_exp_f16_e32 %3, %11\n\t"
        "v_exp_f16_sdwa %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_exp_f16_sdwa %1, %9 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_exp_f16_sdwa %2, %10 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_exp_f16_sdwa %3, %11 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_pk_add_f16 %8, %0, %22\n\tv_pk_add_f16 %9, %1, %22\n\t"
        "v_pk_add_f16 %10, %2, %22\n\tv_pk_add_f16 %11, %3, %22\n\t"
        "v_rcp_f16_e32 %0, %8\n\tv_rcp_f16_e32 %1, %9\n\tv_rcp_f16_e32 %2, %10\n\tv_rcp_f16_e32 %3, %11\n\t"
        "v_rcp_f16_sdwa %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_rcp_f16_sdwa %1, %9 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_rcp_f16_sdwa %2, %10 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_rcp_f16_sdwa %3, %11 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
        "v_pk_mul_f16 %0, %4, %0\n\tv_pk_mul_f16 %1, %5, %1\n\t"
        "v_pk_mul_f16 %2, %6, %2\n\tv_pk_mul_f16 %3, %7, %3\n\t"
        "s_nop 1"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "s"(C1), "v"(C0),
          "v"(ONE));
}

// LDS-DMA: `size` bytes per lane from the per-lane global address `g` into
// LDS at (wave-uniform) `lds_base` + lane * size.
template <int SIZE>
__device__ __forceinline__ void glds(const void *g, void *lds_base)
{
    static_assert(SIZE == 4 || SIZE == 16, "LDS-DMA widths used here");
    if constexpr (SIZE == 16) __builtin_amdgcn_global_load_lds(g, (lds_void_t *)lds_base, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(g, (lds_void_t *)lds_base, 4, 0, 0);
}

// ds_read_b64_tr_b16: per 16-lane group, a 4-row x 16-column block of 16-bit
// values delivered column-major (lane i: column i of the 4 rows).  `p` is this
// lane's LDS byte address (lane 4q+p of the group: row q, columns 4p..4p+3).
typedef __fp16 fp16x4_tr __attribute__((vector_size(8)));
__device__ __forceinline__ h16x4 lds_read_tr16(const void *p)
{
    const fp16x4_tr v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_tr *)p);
    return __builtin_bit_cast(h16x4, v);
}

// (mean, 1/sigma) of a row of d = 32 G features from its G 32-feature group
// partials (sum, squared deviations about the group mean), Chan et al.:
// mean = sum / d, M2 = sum_g M2_g + (s_g - 32 mean)^2 / 32; eps 1e-5
// (ggml_norm, bert.cpp:1048-1056).  The arithmetic is pinned (explicit FMAs and
// rounded ops, no contraction left to the compiler, groups added in index
// order), so any other kernel that combines partials (the small-batch GEMM
// prologue form of profiles/r02_stats_fold_small_ab.log) gives the same bits.
template <int MAXG>
__device__ __forceinline__ float2 ln_row_stats(const float2 (&p)[MAXG], int G, int d)
{
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < MAXG; ++g)
        if (g < G) s = __fadd_rn(s, p[g].x);
    const float mean = __fdiv_rn(s, (float)d);
    float m2 = 0.f;
#pragma unroll
    for (int g = 0; g < MAXG; ++g)
        if (g < G) {
            const float dm = fmaf(-32.0f, mean, p[g].x);
            m2 = __fadd_rn(m2, fmaf(__fmul_rn(dm, dm), 1.0f / 32.0f, p[g].y));
        }
    return float2{mean, __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(__fdiv_rn(m2, (float)d), 1e-5f)))};
}

__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(N) through the builtin (not inline asm) so the compiler's
// waitcnt pass knows the loads older than the N youngest have retired and does
// not add its own conservative vmcnt(0) at their first use.  gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]; other counters
// left at their maximum (no wait).
template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
    asm volatile("" ::: "memory");
}

}  // namespace emb
