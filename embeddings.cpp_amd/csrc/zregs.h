// Lane-order weight fragments (kernels.h) for the 16x16x32 f16 MFMA
// GEMM (gemm.hip): one lane's raw words of one K-step (64 k,
// fragments u = 2a + s: features +16a, k-slice s) and their dequantization to
// f16 A fragments, (q - 8) d (q4_0), q d + m (q4_1), q d (q8_0) rounded once;
// and the permlane16 row exchange of the epilogues.
#pragma once

#include "device_common.h"
#include "host_common.h"

namespace emb {
namespace {

constexpr int ZK = 64;   // K per step (two k-slices of 32)

__device__ __forceinline__ uint4 zload16(const void *p) { return *(const uint4 *)p; }
__device__ __forceinline__ uint2 zload8(const void *p) { return *(const uint2 *)p; }
typedef uint32_t zu32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t zu32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void zpin(uint4 &q)
{
    zu32x4 v = __builtin_bit_cast(zu32x4, q);
    asm volatile("" : "+v"(v));
    q = __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ void zpin(uint2 &q)
{
    zu32x2 v = __builtin_bit_cast(zu32x2, q);
    asm volatile("" : "+v"(v));
    q = __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ h16 zh(uint2 v, int u)   // f16 number u (0..3) of an 8-byte word pair
{
    const uint32_t w = u < 2 ? v.x : v.y;
    return as_h((uint16_t)((u & 1) ? (w >> 16) : (w & 0xffffu)));
}

// One K-step of one lane's weight words: fragment (a, s) = features +16a,
// k-slice s (block 2ks+s), index u = 2a + s.
template <int FMT>
struct ZRegs;

template <int FMT>
struct ZRegsQ4 {
    uint4 q;           // word u: 8 nibbles, element i at bit 4*(i/2) + 16*(i%2)
    uint2 d, m;        // f16 scale (and min) of fragment u
    static constexpr int LOADS = FMT == FMT_Q4_1 ? 3 : 2;
    static constexpr int QB = 16;
    __device__ void load(const uint8_t *pq, const uint16_t *pd, const uint16_t *pm)
    {
        q = zload16(pq);
        d = zload8(pd);
        if (FMT == FMT_Q4_1) m = zload8(pm);
    }
    __device__ void pin_all() { zpin(q); zpin(d); if (FMT == FMT_Q4_1) zpin(m); }
    __device__ h16x8 frag(int u) const
    {
        const uint32_t w = u == 0 ? q.x : u == 1 ? q.y : u == 2 ? q.z : q.w;
        const h16 dh = zh(d, u);
        const h16x2 d2 = {dh, dh};
        h16x2 m2 = {(h16)0.0f, (h16)0.0f};
        if (FMT == FMT_Q4_1) { const h16 mh = zh(m, u); m2 = h16x2{mh, mh}; }
        // Pair p's nibbles sit at bits 4p'.. of each half (p' = p mod 2 after a shift
        // by 8 for p >= 2).  Bits 0-3 are the low mantissa bits of 0x6400 (1024,
        // ulp 1): 1024 + q; bits 4-7 are mantissa bits 4-7 of 0x5400 (64, ulp 1/16):
        // 64 + q.  So one shift per fragment instead of three; the offset add is exact
        // either way and the value (q - 8) d (q d + m) is rounded once, as before.
        const h16 o0 = FMT == FMT_Q4_1 ? (h16)-1024.0f : (h16)-1032.0f;
        const h16 o1 = FMT == FMT_Q4_1 ? (h16)-64.0f : (h16)-72.0f;
        const h16x2 off0 = {o0, o0}, off1 = {o1, o1};
        const uint32_t w8 = w >> 8;
        h16x8 a;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t x = p < 2 ? w : w8;
            h16x2 hh = (p & 1) ? as_h2(and_or_vs(x, 0x00F000F0u, 0x54005400u)) + off1
                               : as_h2(and_or_vs(x, 0x000F000Fu, 0x64006400u)) + off0;
            hh = FMT == FMT_Q4_1 ? hh * d2 + m2 : hh * d2;
            a[2 * p] = hh[0];
            a[2 * p + 1] = hh[1];
        }
        return a;
    }
};
template <> struct ZRegs<FMT_Q4_0> : ZRegsQ4<FMT_Q4_0> {};
template <> struct ZRegs<FMT_Q4_1> : ZRegsQ4<FMT_Q4_1> {};

template <>
struct ZRegs<FMT_Q8_0> {
    uint4 q0, q1;      // 8 bytes per fragment u at 8u: (q ^ 0x80), order e0 e2 e1 e3 per 4-group
    uint2 d;
    static constexpr int LOADS = 3;
    static constexpr int QB = 32;
    __device__ void load(const uint8_t *pq, const uint16_t *pd, const uint16_t *)
    {
        q0 = zload16(pq);
        q1 = zload16(pq + 16);
        d = zload8(pd);
    }
    __device__ void pin_all() { zpin(q0); zpin(q1); zpin(d); }
    __device__ h16x8 frag(int u) const
    {
        const uint32_t w0 = u == 0 ? q0.x : u == 1 ? q0.z : u == 2 ? q1.x : q1.z;
        const uint32_t w1 = u == 0 ? q0.y : u == 1 ? q0.w : u == 2 ? q1.y : q1.w;
        const h16 dh = zh(d, u);
        const h16x2 d2 = {dh, dh};
        const h16x2 off = {(h16)-1152.0f, (h16)-1152.0f};
        h16x8 a;
        // bytes 0 / 2 under the f16 magic 0x64 by one v_and_or_b32 (and_or_vs: the
        // plain C form compiled to v_and + v_or), bytes 1 / 3 by one v_perm_b32
        // (selector 5, 7 = the word's bytes 1, 3; 0 = a 0x64 byte of the magic
        // word) instead of a shift, an and and an or: 12 VALU per 8 weights as for
        // q4, not 19; the same f16 pairs 0x64XX
        const uint32_t mg = 0x64646464u;
        const h16x2 p0 = (as_h2(and_or_vs(w0, 0x00FF00FFu, 0x64006400u)) + off) * d2;
        const h16x2 p1 = (as_h2(__builtin_amdgcn_perm(w0, mg, 0x00070005u)) + off) * d2;
        const h16x2 p2 = (as_h2(and_or_vs(w1, 0x00FF00FFu, 0x64006400u)) + off) * d2;
        const h16x2 p3 = (as_h2(__builtin_amdgcn_perm(w1, mg, 0x00070005u)) + off) * d2;
        a[0] = p0[0]; a[1] = p0[1]; a[2] = p1[0]; a[3] = p1[1];
        a[4] = p2[0]; a[5] = p2[1]; a[6] = p3[0]; a[7] = p3[1];
        return a;
    }
};

template <>
struct ZRegs<FMT_F16> {
    uint4 q[4];        // fragment u: 8 f16
    static constexpr int LOADS = 4;
    static constexpr int QB = 64;
    __device__ void load(const uint8_t *pq, const uint16_t *, const uint16_t *)
    {
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = zload16(pq + 16 * i);
    }
    __device__ void pin_all()
    {
#pragma unroll
        for (int i = 0; i < 4; ++i) zpin(q[i]);
    }
    __device__ h16x8 frag(int u) const { return __builtin_bit_cast(h16x8, q[u]); }
};

// v_permlane16_swap_b32 x, y: rows (16 lanes) 1 and 3 of x trade places with rows
// 0 and 2 of y.  Inline asm: this compiler drops the builtin's second result
// (it reuses the first -- seen in the emitted code), and the asm needs the
// VALU-write -> permlane hazard's two wait states (s_nop 1) itself.
__device__ __forceinline__ void zswap(float &x, float &y)
{
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}

// The four exchanges (v[e], v[4 + e]) of one epilogue row pair behind a single
// hazard pad (their operands are accumulators the K loop wrote long before).
__device__ __forceinline__ void zswap4(float (&v)[8])
{
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %4\n\tv_permlane16_swap_b32 %1, %5\n\t"
                 "v_permlane16_swap_b32 %2, %6\n\tv_permlane16_swap_b32 %3, %7"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
}

}  // namespace
}  // namespace emb
