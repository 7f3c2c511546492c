// Flash-style self-attention for gfx950 (reference bert.cpp:1018-1036).
#include "device_common.h"
#include "diag_att_stamps.h"
#include "kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <utility>

namespace emb {

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
                                                        int d, int nqt, int nh, float sl2, h16 *__restrict__ out)
{
    constexpr int KT = 64, KSTR = DH + 8, VSTR = KT + 8;
    __shared__ __attribute__((aligned(16))) h16 Ks[KT * KSTR];
    __shared__ __attribute__((aligned(16))) h16 Vt[DH * VSTR];
    // XCD-aware order: the query tiles of one (sentence, head) get consecutive
    // logical ids on ONE XCD, so its K/V tiles are fetched into that XCD's L2
    // once instead of once per XCD (dispatch is round-robin over the 8 XCDs).
    const int nb = gridDim.x, bid = blockIdx.x, xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int qt = t % nqt, h = (t / nqt) % nh, b = t / (nqt * nh);
    const int start = cu[b], len = cu[b + 1] - start;
    const int q0 = qt * ATT_QT;
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
            uint4 kv = {0u, 0u, 0u, 0u};
            if (k0 + r < len) kv = *(const uint4 *)(qkv + (size_t)(start + k0 + r) * ld + d + h * DH + ch * 8);
            *(uint4 *)(Ks + r * KSTR + ch * 8) = kv;
        }
        // V tile transposed into Vt[d][key] (key fastest across lanes: conflict-free 2-byte writes)
        for (int c = tid; c < KT * DH / 8; c += 256) {
            const int r = c % KT, ch = c / KT;
            // keys past the sentence: zeros (their P is exactly 0; 0 * garbage could be NaN)
            h16x8 vv = {};
            if (k0 + r < len) vv = *(const h16x8 *)(qkv + (size_t)(start + k0 + r) * ld + 2 * d + h * DH + ch * 8);
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

// ---------------------------------------------------------------------------
// attention_lds: one workgroup per (sentence, head), up to 512 keys.  The
// sentence's whole K and V (<= 512 x DH f16 each, 128 KiB at DH 64) are
// brought into LDS ONCE by LDS-DMA; 16 waves x 32 queries then run with no
// further global loads and no barriers.
//   K image: [key][DH] rows, 16-B chunks XOR-swizzled by kswz(key) (via the
//            DMA source address), read as ds_read_b128 A fragments of S^T = K Q^T.
//   V image: [key][DH] rows, chunks XOR-swizzled by ((key >> 1) & 1) << 2, read
//            with ds_read_b64_tr_b16 as the transposed A fragments of
//            O^T += V^T P^T -- no transposing copy.
// Q is pre-scaled by log2(e)/sqrt(dh) (f16), so S comes out in the exp2 domain;
// keys past the sentence end are masked (only in the last 64-key block).
// ---------------------------------------------------------------------------
// K image chunk swizzle: the 16 lanes of a ds_read_b128 group read 16 rows
// ({0-3,12-15,20-27} + 32n) at one chunk; XOR with (row >> 1) & 7 (128-B rows)
// or (row >> 2) & 3 (64-B rows) puts them on 16 distinct 16-B bank slots.
template <int CH>
__device__ __forceinline__ int kswz(int row)
{
    return CH == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3);
}

template <int DH>
__global__ __launch_bounds__(1024) void attention_lds_kernel(const h16 *__restrict__ qkv,
                                                             const int32_t *__restrict__ cu, int d, int nh,
                                                             float sl2, h16 *__restrict__ out)
{
    constexpr int RB = DH * 2, CH = RB / 16, LMAX = ATT_LDS_MAX;
    __shared__ __attribute__((aligned(16))) char smem[2 * LMAX * RB];
    char *Kl = smem, *Vl = smem + LMAX * RB;
    const int h = blockIdx.x % nh, b = blockIdx.x / nh;
    const int start = cu[b], len = cu[b + 1] - start;
    if (len <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int hi = lane >> 5, lq = lane & 31;
    const int ld = 3 * d;
    const int nrows = (len + 63) & ~63;

    // ---- K and V of the sentence -> LDS (64 chunks of 16 B per wave-instruction) ----
    {
        const int ninstr = nrows * CH / 64;
        const h16 *kbase = qkv + (size_t)start * ld + d + h * DH;
        const h16 *vbase = kbase + d;
        for (int i = w; i < ninstr; i += 16) {
            const int g = i * 64 + lane, row = g / CH, pc = g % CH;
            const int srow = min(row, len - 1);          // rows past the end: finite copies, masked / P = 0
            const int ck = pc ^ kswz<CH>(row);
            const int cv = pc ^ ((((row >> 1) & 1) << 2) & (CH - 1));
            glds<16>(kbase + (size_t)srow * ld + ck * 8, Kl + i * 1024);
            glds<16>(vbase + (size_t)srow * ld + cv * 8, Vl + i * 1024);
        }
        wait_vmcnt<0>();
        __syncthreads();
    }

    const int q0 = 32 * w;
    if (q0 >= len) return;                                // no barrier follows
    const int q = q0 + lq;
    h16x8 qf[DH / 16];
    {
        const h16 *qrow = qkv + (size_t)(start + min(q, len - 1)) * ld + h * DH;
        const h16 s16 = (h16)sl2;
        const h16x8 sc = {s16, s16, s16, s16, s16, s16, s16, s16};
#pragma unroll
        for (int s = 0; s < DH / 16; ++s) qf[s] = *(const h16x8 *)(qrow + 16 * s + 8 * hi) * sc;
    }
    f32x16 o[DH / 32];
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    float m_i = -INFINITY, l_i = 0.f;

    // tr-read lane roles: group g = lane >> 4 reads rows r0 + (i >> 2), columns c0 + 4 (i & 3)
    const int gi = lane & 15, gq = gi >> 2, gp = gi & 3, gg = lane >> 4;

    for (int kb = 0; kb < nrows; kb += 64) {
        f32x16 s[2];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
            const int row = kb + 32 * kh + lq;
            const char *krow = Kl + row * RB;
#pragma unroll
            for (int st = 0; st < DH / 16; ++st) {
                const h16x8 a = *(const h16x8 *)(krow + (((2 * st + hi) ^ kswz<CH>(row)) << 4));
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[st], s[kh], 0, 0, 0);
            }
        }
        if (kb + 64 > len) {
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = kb + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
                    if (key >= len) s[kh][r] = -INFINITY;
                }
        }
        float mx = s[0][0];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kh][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_i, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_i - m_new);
        float rs = 0.f;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[kh][r] - m_new);
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
                const int r0 = kb + 32 * kh + 16 * s2 + 4 * (gg >> 1) + gq;
#pragma unroll
                for (int t = 0; t < DH / 32; ++t) {
                    const int c0 = 32 * t + 16 * (gg & 1) + 4 * gp;       // column of this lane's 8 bytes
                    const int ch = c0 >> 3;
                    const int rowa = r0, rowb = r0 + 8;
                    const h16x4 lo = lds_read_tr16(Vl + rowa * RB +
                                                   ((ch ^ ((((rowa >> 1) & 1) << 2) & (CH - 1))) << 4) + (c0 & 7) * 2);
                    const h16x4 up = lds_read_tr16(Vl + rowb * RB +
                                                   ((ch ^ ((((rowb >> 1) & 1) << 2) & (CH - 1))) << 4) + (c0 & 7) * 2);
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

// ---------------------------------------------------------------------------
// attention_lds3 (production, dh 64) keeps the attention_lds structure (whole
// K/V of a (sentence, head) in LDS, 16 waves x 32 queries, S^T = K Q^T with the
// query on the lane) with the softmax VALU cut to the exp, the row sum and the
// f16 packing per score:
//  * fixed offset: each query keeps an f16 offset c (the max of its first
//    block) and S - c comes out of the MFMA itself -- one extra MFMA per
//    32 keys multiplies a ones-column of K by a (-c)-row of Q.  softmax(S) =
//    exp2(S - c) / sum exp2(S - c) for any c, so the result is the function
//    of the running-max form.  No max is taken per block: a block whose
//    32-key partial row sum exceeds 2^ATT_SUMX (so some P may leave the safe
//    f16 range) is recomputed after moving c to the row max and rescaling O
//    and l -- rare, and it keeps every P <= 2^ATT_SUMX.
//  * the row sum stays per 32-lane half (no cross-lane op per block); the
//    halves are combined once, by v_permlane32_swap, at the end.
//  * LDS reads at base + immediate offsets (the swizzles of both images are
//    lane constants for 16-row-aligned blocks): six address adds per block.
// ---------------------------------------------------------------------------
constexpr int ATT_SUMX = 12;   // a block whose half-row sum passes 2^ATT_SUMX moves the offset

// ---------------------------------------------------------------------------
// Persistence: one workgroup per CU that walks the items (sentence, head)
// it = blockIdx.x, + gridDim.x, ..., so the K/V DMA of the next item runs
// under the current item's MFMAs instead of in front of them (a workgroup per
// item loads every item in the open: about 16 of 84 us at C3 were exposed loads).  The K/V
// image is two regions of 256 keys (A = key blocks 0-3, B = blocks 4-7):
//   B1 (every wave past the item's region-A blocks): the next item's region-A
//      K/V pieces are issued;
//   S  (every wave past its region-B blocks; the next item's Q rows loaded in
//      front of it): the item's rows are stored; the next item's region-B
//      pieces are issued once its Q has arrived (the loop top).
// The waits in front of B1 and S retire pieces issued half an item earlier; only
// a workgroup's first item waits for its loads in the open.  Per-phase cycles:
// ATT_STAMPS build, scripts/att_stamps.py.
// ---------------------------------------------------------------------------
// the lane id from an asm statement the compiler cannot hoist out of a loop
__device__ __forceinline__ int lane_id_opaque()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// LDS-DMA issued from asm: hipcc's waitcnt pass cannot see it, so it no longer
// puts a vmcnt(0) in front of the first LDS read after each issue (which retired
// the next item's region-A prefetch in the first block after B1).  The kernel's
// own waits in front of B1 and S are the only ones; no compiler-visible global
// load may be in flight across the block loop's back edge (its wait there would
// retire the hidden pieces too), and the compiler's waits for its own loads stay
// conservative (hidden younger loads only make its vmcnt(N) stricter).
__device__ __forceinline__ void glds16_hidden(const void *g, const void *lds)
{
    const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char *)lds;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m) : "memory", "m0");
#pragma clang diagnostic pop
}
// every vector-memory op retired: the builtin for the compiler's own loads, the
// asm copy for the hidden pieces
__device__ __forceinline__ void wait_all_vm()
{
    wait_vmcnt<0>();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


__global__ __launch_bounds__(1024) void attention_lds3_kernel(const h16 *__restrict__ qkv,
                                                              const int32_t *__restrict__ cu, int d, int nh,
                                                              int n_items, float sl2, h16 *__restrict__ out)
{
    constexpr int DH = 64, RB = DH * 2, LMAX = ATT_LDS_MAX, RH = LMAX / 2;
    static_assert(RH == 256, "a region is 32 pieces: two per wave");
    __shared__ __attribute__((aligned(16))) char smem[2 * LMAX * RB];
    char *Kl = smem;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hi = lane >> 5, lq = lane & 31;
    const int ld = 3 * d;

    struct Item { int start, len, h; };
    auto item = [&](int i) {
        const int b = i / nh;
        Item r;
        r.h = i - b * nh;
        r.start = cu[b];
        r.len = cu[b + 1] - r.start;
        return r;
    };
    // region r (rows 256 r .. 256 r + 255) of `it`: piece i = rows 8i .. 8i + 7;
    // wave w issues pieces 32 r + w and 32 r + w + 16 when they hold rows of the
    // sentence's 64-row blocks.  K swizzled by (row >> 1) & 7, V by
    // ((row >> 1) & 1) << 2 ; rows past the end are finite
    // copies (masked / P = 0).
    auto issue = [&](const Item &it, int r) {
        const int lane = lane_id_opaque();                // recomputed here: hoisted, its
        const int nrows = (it.len + 63) & ~63;            // derivatives spill around the block loop
        const h16 *kbase = qkv + (size_t)it.start * ld + d + it.h * DH;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = 32 * r + w + 16 * j;
            if (8 * i < nrows) {
                const int row = 8 * i + (lane >> 3), pc = lane & 7;
                const size_t so = (size_t)min(row, it.len - 1) * ld;
                glds16_hidden(kbase + so + (pc ^ ((row >> 1) & 7)) * 8, Kl + i * 1024);
                glds16_hidden(kbase + d + so + (pc ^ (((row >> 1) & 1) << 2)) * 8, Kl + LMAX * RB + i * 1024);
            }
        }
    };
    h16x8 qf[DH / 16];
    auto load_q = [&](const Item &it) {                   // raw rows; scaled at the item's start
        if (it.len <= 0) return;
        const int lane = lane_id_opaque(), hi = lane >> 5, lq = lane & 31;
        const h16 *qrow = qkv + (size_t)(it.start + min(32 * w + lq, it.len - 1)) * ld + it.h * DH;
#pragma unroll
        for (int s = 0; s < DH / 16; ++s) qf[s] = *(const h16x8 *)(qrow + 16 * s + 8 * hi);
    };

    // lane-constant LDS offsets (blocks are 64-row aligned)
    int koff[DH / 16];
#pragma unroll
    for (int st = 0; st < DH / 16; ++st) koff[st] = lq * RB + (((2 * st + hi) ^ ((lq >> 1) & 7)) << 4);
    const int gi = lane & 15, gq = gi >> 2, gp = gi & 3, gg = lane >> 4;
    const int vsw = ((gq >> 1) & 1) << 2;
    int voff[DH / 32];
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) {
        const int ch = 4 * t + 2 * (gg & 1) + (gp >> 1);
        voff[t] = (4 * (gg >> 1) + gq) * RB + ((ch ^ vsw) << 4) + 8 * (gp & 1);
    }
    const h16 one = (h16)1.0f, zero = (h16)0.0f;
    const h16x8 abias = {hi ? zero : one, zero, zero, zero, zero, zero, zero, zero};
    h16x8 bbias = {zero, zero, zero, zero, zero, zero, zero, zero};

    f32x16 o[DH / 32];
    float c = 0.f, l = 0.f;                               // offset (f16-exact), this half's row sum
    f32x16 s[2];
    int len = 0;                                          // the current item's

    auto qk = [&](int kb, bool bias) {
        int kbo[DH / 16];
#pragma unroll
        for (int st = 0; st < DH / 16; ++st) {
            kbo[st] = koff[st] + kb * RB;
            asm volatile("" : "+v"(kbo[st]));
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            if (bias) {
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(abias, bbias, f32x16{}, 0, 0, 0);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
            }
#pragma unroll
            for (int st = 0; st < DH / 16; ++st) {
                const h16x8 a = *(const h16x8 *)(Kl + kbo[st] + kh * 32 * RB);
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[st], s[kh], 0, 0, 0);
            }
        }
        if (kb + 64 > len) {
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = kb + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
                    if (key >= len) s[kh][r] = -INFINITY;
                }
        }
    };
    auto row_max = [&]() {                                // over both halves
        float mx = s[0][0];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = (kh ? 0 : 1); r < 16; ++r) mx = fmaxf(mx, s[kh][r]);
        return halves_max(mx);
    };
    auto shift_by = [&](float sh) {                       // scores -= sh
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kh][r] -= sh;
    };
    auto expsum = [&]() {                                 // s <- exp2(s); this half's sum
        float rs = 0.f;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[kh][r]);
                s[kh][r] = p;
                rs += p;
            }
        return rs;
    };
    auto pv = [&](int kb) {
        int vbo[DH / 32];
#pragma unroll
        for (int t = 0; t < DH / 32; ++t) {
            vbo[t] = voff[t] + kb * RB + LMAX * RB;
            asm volatile("" : "+v"(vbo[t]));
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                h16x8 bp;
#pragma unroll
                for (int j = 0; j < 8; ++j) bp[j] = (h16)s[kh][8 * s2 + j];
#pragma unroll
                for (int t = 0; t < DH / 32; ++t) {
                    const char *va = smem + vbo[t] + (32 * kh + 16 * s2) * RB;
                    const h16x4 lo = lds_read_tr16(va);
                    const h16x4 up = lds_read_tr16(va + 8 * RB);
                    const h16x8 a = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bp, o[t], 0, 0, 0);
                }
            }
        }
    };
    // Q K^T and softmax of block kb > 0 (the first block, peeled off the block loop
    // sets the offset to its row max)
    auto scores = [&](int kb) {                           // blocks after the first
        qk(kb, true);                                     // S - c
        float rs = expsum();
        if (__builtin_amdgcn_ballot_w64(rs > (float)(1 << ATT_SUMX))) {
            // rare: move c to the row max, rescale, redo the block
            qk(kb, true);
            const float m = row_max();
            const float sh = m > 0.f ? (float)(h16)(c + m) - c : 0.f;
            const float alpha = __builtin_amdgcn_exp2f(-sh);
            shift_by(sh);
            c += sh;
            bbias[0] = hi ? zero : (h16)(-c);
            l *= alpha;
#pragma unroll
            for (int t = 0; t < DH / 32; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
            rs = expsum();
        }
        l += rs;
    };

    int cur_i = blockIdx.x;
    if (cur_i >= n_items) return;                         // workgroup-uniform
    Item cur = item(cur_i);
    // the first item: Q and region A in the open; region B (issued at the loop
    // top) under region A's blocks, retired by B1's wait as in every later item
    load_q(cur);
    issue(cur, 0);
    wait_all_vm();
    __syncthreads();
    const h16 s16 = (h16)sl2;
    const h16x8 sc = {s16, s16, s16, s16, s16, s16, s16, s16};
    ASTAMP_ITEMS(nit);   // (stamps builds only, diag_att_stamps.h)
    for (;;) {
        ASTAMP(0, __builtin_amdgcn_s_memtime());
        const int nx_i = cur_i + (int)gridDim.x;
        const bool more = nx_i < n_items;                 // workgroup-uniform
        Item nx = {0, 0, 0};
        if (more) nx = item(nx_i);
        len = cur.len;
        const int nrows = (len + 63) & ~63;
        const bool active = 32 * w < len;                 // wave-uniform
        // unconditional resets: nothing of the block state stays live across items
#pragma unroll
        for (int st = 0; st < DH / 16; ++st) qf[st] *= sc;
        // the item's region B, issued after the first use of Q (the compiler's
        // wait for the Q loads retires every older piece); the empty asm keeps
        // the issue below that wait
        asm volatile("" ::"v"(qf[0]), "v"(qf[1]), "v"(qf[2]), "v"(qf[3]));
        issue(cur, 1);
#pragma unroll
        for (int t = 0; t < DH / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
        c = 0.f;
        l = 0.f;
        bbias[0] = zero;
        __builtin_amdgcn_s_setprio(3);                    // block 0: see the block loop
        if (active) {                                     // block 0: the offset is its row max (f16-rounded)
            qk(0, false);
            c = (float)(h16)row_max();
            shift_by(c);
            bbias[0] = hi ? zero : (h16)(-c);
            l = expsum();
            pv(0);
        }
        ASTAMP(1, __builtin_amdgcn_s_memtime());
        // blocks 1-7 in one loop (one inlined copy of the block code), B1 at the
        // region boundary
#pragma clang loop unroll(disable)
        for (int kb = 64; kb < LMAX; kb += 64) {
            if (kb == RH) {
                ASTAMP(2, __builtin_amdgcn_s_memtime());
                wait_all_vm();                            // this item's region-B pieces
                __syncthreads();                          // B1: region A is free
                ASTAMP(3, __builtin_amdgcn_s_memtime());
                if (more) issue(nx, 0);
            }
            // progress-based priority: the further a wave is past the last
            // barrier, the lower its priority, so the 4 waves of a SIMD reach the
            // next barrier together instead of in age order (the oldest wave of a
            // SIMD ran its 4 blocks 2x faster than the youngest and then waited
            // for it; 69.5 -> 65.8 us at C3, profiles/r02_att_stamps_prio.log)
            switch ((kb >> 6) & 3) {
            case 0: __builtin_amdgcn_s_setprio(3); break;
            case 1: __builtin_amdgcn_s_setprio(2); break;
            case 2: __builtin_amdgcn_s_setprio(1); break;
            default: __builtin_amdgcn_s_setprio(0); break;
            }
            if (active && kb < nrows) {
                scores(kb);
                pv(kb);
            }
        }
        ASTAMP(4, __builtin_amdgcn_s_memtime());
        // The item's rows are stored after the S barrier (storing them before S,
        // so a wave that finishes early writes while the slower ones still
        // compute, measured 2 us slower: the early stores queue in front of the
        // next item's region-A pieces, profiles/r03_attention_store_ab.log).  The
        // stores are bounds-checked buffer stores on every lane of an active wave
        // (rows past the sentence fall outside the resource and are dropped).  The
        // wait in front of S is exact: the next item's Q (4 loads) stays in
        // flight, every older piece (the next item's region A) is retired.
        if (more) load_q(nx);
        auto store_rows = [&]() {
            // lane (q, hi) holds dh 8m + 4 hi .. +3 of chunks m = 4t + g; one
            // v_permlane32_swap per dword of the chunk pair (2p, 2p + 1) gives lane
            // (q, 0) dh 16p .. 16p + 7 and lane (q, 1) dh 16p + 8 .. 16p + 15: four
            // 16-B stores per lane instead of eight 8-B ones (the store tail is
            // issue-bound; cdna_hip_programming.md T21).  Both lanes of a pair
            // hold the same query, so the swaps run on every lane.
            const float inv = 1.0f / halves_sum(l);
            const int q = 32 * w + lq;
            uint32_t pk[DH / 8][2];
#pragma unroll
            for (int m = 0; m < DH / 8; ++m)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int t = m >> 2, g = m & 3;
                    const h16x2 v = {(h16)(o[t][4 * g + 2 * k] * inv), (h16)(o[t][4 * g + 2 * k + 1] * inv)};
                    pk[m][k] = __builtin_bit_cast(uint32_t, v);
                }
#pragma unroll
            for (int p = 0; p < DH / 16; ++p)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * p][k], pk[2 * p + 1][k], false, false);
                    pk[2 * p][k] = r[0];
                    pk[2 * p + 1][k] = r[1];
                }
            // the item's rows [start, start + len) of `out` as the resource: a row
            // q >= len lies past num_records and its store is dropped
            const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(out + (size_t)cur.start * d), (short)0, cur.len * d * 2, 0x00020000);
            const int ob = (q * d + cur.h * DH + 8 * hi) * 2;
#pragma unroll
            for (int p = 0; p < DH / 16; ++p) {
                typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
                const u32x4v v = {pk[2 * p][0], pk[2 * p][1], pk[2 * p + 1][0], pk[2 * p + 1][1]};
                __builtin_amdgcn_raw_buffer_store_b128(v, ors, ob + 32 * p, 0, 0);
            }
        };
        static_assert(DH / 16 == 4, "four stores per active wave");
        if (more) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // the 4 Q loads younger
        else wait_all_vm();
        ASTAMP(5, __builtin_amdgcn_s_memtime());
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // no LDS read in flight into the store phase
        __syncthreads();                                  // S: region B is free
        if (active) store_rows();
        ASTAMP(6, __builtin_amdgcn_s_memtime());
        ASTAMP_ITEM_END(nit);
        if (!more) break;
        cur = nx;
        cur_i = nx_i;
    }
}

// ---------------------------------------------------------------------------
// Short sentences (max_len <= 64, the serving shape: examples/server.cpp:114 ->
// one text per bert_encode): one 2-wave workgroup per (sentence, head), the
// item's one 64-key block.  attention_lds3 runs such an item on 16 waves of which
// one or two have queries, through its region DMA and its B1 and S barriers;
// here the K/V rows are plain 16-B loads into the same swizzled LDS image and
// the block is lds3's block 0 instruction for instruction (the same MFMA chains
// in the same order, the f16 row-max offset, the exp2 sum, P.V, 1 / l), so a
// sentence gets the same bits from either kernel (batch-composition invariance:
// a short sentence alone takes this kernel, inside a longer batch lds3).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void attention_short_kernel(const h16 *__restrict__ qkv,
                                                              const int32_t *__restrict__ cu, int d, int nh,
                                                              float sl2, h16 *__restrict__ out)
{
    constexpr int DH = 64, RB = DH * 2, NK = 64, VB = NK * RB;
    __shared__ __attribute__((aligned(16))) char smem[2 * NK * RB];
    const int it = blockIdx.x, b = it / nh, h = it - b * nh;
    const int start = cu[b], len = cu[b + 1] - start;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int hi = lane >> 5, lq = lane & 31;
    const int ld = 3 * d;
    if (len <= 0) return;                                 // workgroup-uniform
    // the wave's Q rows first: their loads fly with the K / V loads below
    h16x8 qf[DH / 16];
    {
        const h16 *qrow = qkv + (size_t)(start + min(32 * w + lq, len - 1)) * ld + h * DH;
#pragma unroll
        for (int st = 0; st < DH / 16; ++st) qf[st] = *(const h16x8 *)(qrow + 16 * st + 8 * hi);
    }
    // K / V rows 0-63 (rows past the end: finite copies of the last row, masked /
    // P = 0), K chunk j of row r at chunk j ^ ((r >> 1) & 7), V at j ^ (((r >> 1) & 1) << 2)
    const h16 *kbase = qkv + (size_t)start * ld + d + h * DH;
#pragma unroll
    for (int k = 0; k < NK * 8 / 128; ++k) {
        const int c = tid + 128 * k, r = c >> 3, j = c & 7;
        const size_t so = (size_t)min(r, len - 1) * ld + 8 * j;
        const uint4 kv = *(const uint4 *)(kbase + so);
        const uint4 vv = *(const uint4 *)(kbase + d + so);
        *(uint4 *)(smem + r * RB + ((j ^ ((r >> 1) & 7)) << 4)) = kv;
        *(uint4 *)(smem + VB + r * RB + ((j ^ (((r >> 1) & 1) << 2)) << 4)) = vv;
    }
    __syncthreads();
    if (32 * w >= len) return;                            // wave-uniform: no queries
    const h16 s16 = (h16)sl2;
    const h16x8 sc = {s16, s16, s16, s16, s16, s16, s16, s16};
#pragma unroll
    for (int st = 0; st < DH / 16; ++st) qf[st] *= sc;
    // S^T = K Q^T for keys 0-63 (lds3 qk(0, false))
    f32x16 s[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
#pragma unroll
        for (int st = 0; st < DH / 16; ++st) {
            const int ko = lq * RB + (((2 * st + hi) ^ ((lq >> 1) & 7)) << 4) + kh * 32 * RB;
            const h16x8 a = *(const h16x8 *)(smem + ko);
            s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[st], s[kh], 0, 0, 0);
        }
    }
    if (NK > len) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
                if (key >= len) s[kh][r] = -INFINITY;
            }
    }
    // the offset: the row max, f16-rounded; P = exp2(S - c); this half's sum
    float mx = s[0][0];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = (kh ? 0 : 1); r < 16; ++r) mx = fmaxf(mx, s[kh][r]);
    const float c = (float)(h16)halves_max(mx);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kh][r] -= c;
    float l = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(s[kh][r]);
            s[kh][r] = p;
            l += p;
        }
    // O^T = V^T P^T (lds3 pv(0))
    const int gi = lane & 15, gq = gi >> 2, gp = gi & 3, gg = lane >> 4;
    const int vsw = ((gq >> 1) & 1) << 2;
    f32x16 o[DH / 32];
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            h16x8 bp;
#pragma unroll
            for (int j = 0; j < 8; ++j) bp[j] = (h16)s[kh][8 * s2 + j];
#pragma unroll
            for (int t = 0; t < DH / 32; ++t) {
                const int ch = 4 * t + 2 * (gg & 1) + (gp >> 1);
                const char *va = smem + VB + (4 * (gg >> 1) + gq) * RB + ((ch ^ vsw) << 4) + 8 * (gp & 1) +
                                 (32 * kh + 16 * s2) * RB;
                const h16x4 lo = lds_read_tr16(va);
                const h16x4 up = lds_read_tr16(va + 8 * RB);
                const h16x8 a = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bp, o[t], 0, 0, 0);
            }
        }
    }
    // rows out: lds3's store phase (1 / l, one permlane32 swap per dword of a
    // chunk pair, four 16-B bounds-checked stores per lane; rows >= len dropped)
    const float inv = 1.0f / halves_sum(l);
    const int q = 32 * w + lq;
    uint32_t pk[DH / 8][2];
#pragma unroll
    for (int m = 0; m < DH / 8; ++m)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int t = m >> 2, g = m & 3;
            const h16x2 v = {(h16)(o[t][4 * g + 2 * k] * inv), (h16)(o[t][4 * g + 2 * k + 1] * inv)};
            pk[m][k] = __builtin_bit_cast(uint32_t, v);
        }
#pragma unroll
    for (int p = 0; p < DH / 16; ++p)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * p][k], pk[2 * p + 1][k], false, false);
            pk[2 * p][k] = r[0];
            pk[2 * p + 1][k] = r[1];
        }
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc((void *)(out + (size_t)start * d), (short)0, len * d * 2, 0x00020000);
    const int ob = (q * d + h * DH + 8 * hi) * 2;
#pragma unroll
    for (int p = 0; p < DH / 16; ++p) {
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        const u32x4v v = {pk[2 * p][0], pk[2 * p][1], pk[2 * p + 1][0], pk[2 * p + 1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, ob + 32 * p, 0, 0);
    }
}

// ---------------------------------------------------------------------------
// attention_pp (production for 64 < L <= 512, dh 64; round 6): lds3's per-query
// arithmetic in two co-resident 8-wave workgroups per CU instead of one 16-wave
// workgroup, so one workgroup's per-unit phases (Q in, block 0, the row stores)
// run beside the other's steady blocks instead of stalling the whole CU.  A unit is
// half an item: 256 queries (8 waves x 32, wave w of half qh = lds3's wave
// 8 qh + w) over all of the sentence's keys; K and V stream through a 4-stage
// LDS ring of 64-key blocks (16 KiB a stage: 64 KiB per workgroup, two per CU),
// each wave issuing one K and one V piece per block, NS - 1 blocks ahead; a
// barrier per block publishes block j and frees block j - 1's stage.  The two
// halves of an item are consecutive units on one XCD, so the second reads K/V
// from that L2.  Every query runs lds3's block sequence (block 0 sets the f16
// offset, later blocks the biased QK^T, the ballot rescale, P.V) on the same
// wave composition, so the output has lds3's bits (the kernel tests compare them).
// (Round 6 also measured, all bitwise equal and slower: four 4-wave workgroups
// per CU with a 2-stage ring, a barrier per block pair, and a persistent form
// whose ring runs on across units; profiles/r06_attention_pp_ab.log.  A priority
// split between the co-resident workgroups: no effect, r06_attention_pp_prio_ab.log.)
__global__ __launch_bounds__(512, 4) void attention_pp_kernel(const h16 *__restrict__ qkv,
                                                              const int32_t *__restrict__ cu, int d, int nh,
                                                              float sl2, h16 *__restrict__ out)
{
    constexpr int NW = 8, NS = 4, DH = 64, RB = DH * 2, SB = 2 * 64 * RB, VO = 64 * RB;
    constexpr int UPI = 16 / NW, PW = 16 / NW;            // units per item, pieces per wave and block
    __shared__ __attribute__((aligned(16))) char smem[NS * SB];
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hi = lane >> 5, lq = lane & 31;
    const int ld = 3 * d;
    // XCD-aware bijective remap (as the GEMM tiles): each XCD a contiguous run of
    // units, so an item's two halves share its L2
    const int nb = gridDim.x, bid = blockIdx.x, xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int u = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int it = u / UPI, q0 = 32 * NW * (u - it * UPI);
    const int b = it / nh, h = it - b * nh;
    const int start = cu[b], len = cu[b + 1] - start;
    if (q0 >= len) return;                                // workgroup-uniform: no queries
    const int nblk = (len + 63) >> 6;
    const bool active = q0 + 32 * w < len;                // wave-uniform
    const h16 *kbase = qkv + (size_t)start * ld + d + h * DH;
    PST_DECL;   // (stamps builds only, diag_att_stamps.h)
    PST_SET(0, PST_NOW());

    // block j's K and V rows into stage j % NS: piece i < 8 is K rows 8i .. 8i + 7
    // of the block, 8 + i the same V rows (K swizzled by (row >> 1) & 7, V by
    // ((row >> 1) & 1) << 2, the row's parity within the block being its parity in
    // the sentence); wave w issues pieces w, w + NW, ...; rows past the end are
    // finite copies (masked / P = 0)
    auto issue = [&](int j) {
        const int ln = lane_id_opaque();
#pragma unroll
        for (int k = 0; k < PW; ++k) {
            const int i = w + NW * k, r8 = i & 7;
            const int row = 64 * j + 8 * r8 + (ln >> 3), pc = ln & 7;
            const size_t so = (size_t)min(row, len - 1) * ld;
            char *dst = smem + (j % NS) * SB + i * 1024;
            if (i < 8) glds16_hidden(kbase + so + (pc ^ ((row >> 1) & 7)) * 8, dst);
            else glds16_hidden(kbase + d + so + (pc ^ (((row >> 1) & 1) << 2)) * 8, dst);
        }
    };
    // the wave's Q rows by asm loads (hipcc's waitcnt pass does not see them, so it
    // puts no vmcnt(0) at their first use, which would retire every prologue
    // piece); then blocks 0-2 (always three: a block past the sentence is a
    // clamped copy into a stage no block reads), so block 0's wait below has one
    // constant count and is one asm tied to the Q registers (a wait per branch
    // let hipcc copy the registers in front of it, before the loads landed)
    h16x8 qf[DH / 16];
    {
        const h16 *qrow = qkv + (size_t)(start + min(q0 + 32 * w + lq, len - 1)) * ld + h * DH;
#pragma unroll
        for (int st = 0; st < DH / 16; ++st)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[st]) : "v"(qrow + 16 * st + 8 * hi) : "memory");
    }
#pragma unroll
    for (int j = 0; j < NS - 1; ++j) issue(j);

    // lane-constant LDS offsets within a stage (lds3's)
    int koff[DH / 16];
#pragma unroll
    for (int st = 0; st < DH / 16; ++st) koff[st] = lq * RB + (((2 * st + hi) ^ ((lq >> 1) & 7)) << 4);
    const int gi = lane & 15, gq = gi >> 2, gp = gi & 3, gg = lane >> 4;
    const int vsw = ((gq >> 1) & 1) << 2;
    int voff[DH / 32];
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) {
        const int ch = 4 * t + 2 * (gg & 1) + (gp >> 1);
        voff[t] = (4 * (gg >> 1) + gq) * RB + ((ch ^ vsw) << 4) + 8 * (gp & 1) + VO;
    }
    const h16 one = (h16)1.0f, zero = (h16)0.0f;
    const h16x8 abias = {hi ? zero : one, zero, zero, zero, zero, zero, zero, zero};
    h16x8 bbias = {zero, zero, zero, zero, zero, zero, zero, zero};
    f32x16 o[DH / 32];
    float c = 0.f, l = 0.f;
    f32x16 s[2];

    auto qk = [&](int kb, int sbase, bool bias) {
        int kbo[DH / 16];
#pragma unroll
        for (int st = 0; st < DH / 16; ++st) {
            kbo[st] = koff[st] + sbase;
            asm volatile("" : "+v"(kbo[st]));
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            if (bias) {
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(abias, bbias, f32x16{}, 0, 0, 0);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
            }
#pragma unroll
            for (int st = 0; st < DH / 16; ++st) {
                const h16x8 a = *(const h16x8 *)(smem + kbo[st] + kh * 32 * RB);
                s[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[st], s[kh], 0, 0, 0);
            }
        }
        if (kb + 64 > len) {
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = kb + 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * hi;
                    if (key >= len) s[kh][r] = -INFINITY;
                }
        }
    };
    auto row_max = [&]() {
        float mx = s[0][0];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = (kh ? 0 : 1); r < 16; ++r) mx = fmaxf(mx, s[kh][r]);
        return halves_max(mx);
    };
    auto shift_by = [&](float sh) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kh][r] -= sh;
    };
    auto expsum = [&]() {
        float rs = 0.f;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(s[kh][r]);
                s[kh][r] = p;
                rs += p;
            }
        return rs;
    };
    auto pv = [&](int sbase) {
        int vbo[DH / 32];
#pragma unroll
        for (int t = 0; t < DH / 32; ++t) {
            vbo[t] = voff[t] + sbase;
            asm volatile("" : "+v"(vbo[t]));
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                h16x8 bp;
#pragma unroll
                for (int j = 0; j < 8; ++j) bp[j] = (h16)s[kh][8 * s2 + j];
#pragma unroll
                for (int t = 0; t < DH / 32; ++t) {
                    const char *va = smem + vbo[t] + (32 * kh + 16 * s2) * RB;
                    const h16x4 lo = lds_read_tr16(va);
                    const h16x4 up = lds_read_tr16(va + 8 * RB);
                    const h16x8 a = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bp, o[t], 0, 0, 0);
                }
            }
        }
    };
    auto scores = [&](int kb, int sbase) {
        qk(kb, sbase, true);
        float rs = expsum();
        if (__builtin_amdgcn_ballot_w64(rs > (float)(1 << ATT_SUMX))) {
            qk(kb, sbase, true);
            const float m = row_max();
            const float sh = m > 0.f ? (float)(h16)(c + m) - c : 0.f;
            const float alpha = __builtin_amdgcn_exp2f(-sh);
            shift_by(sh);
            c += sh;
            bbias[0] = hi ? zero : (h16)(-c);
            l *= alpha;
#pragma unroll
            for (int t = 0; t < DH / 32; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
            rs = expsum();
        }
        l += rs;
    };

#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    const h16 s16 = (h16)sl2;
    const h16x8 sc = {s16, s16, s16, s16, s16, s16, s16, s16};
    // block j: this wave's pieces of it retired (blocks j + 1 .. j + NS - 2 may
    // fly), then the barrier publishes every wave's and frees block j - 1's stage,
    // then block j + NS - 1 is issued into that stage
    auto enter = [&](int j) {
        const int younger = min(NS - 2, nblk - 1 - j);   // blocks in flight behind block j
        if (j == 0) {   // the Q loads and block 0 (the oldest); blocks 1 .. NS - 2 may fly
            asm volatile("s_waitcnt vmcnt(%4)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3])
                         : "i"(PW * (NS - 2)) : "memory");
        } else if (younger >= 2) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PW * 2) : "memory");
        } else if (younger == 1) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PW) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
        if (j + NS - 1 < nblk) issue(j + NS - 1);
    };
    auto block0 = [&]() {                                 // lds3's block 0 (peeled)
        qk(0, 0, false);
        c = (float)(h16)row_max();
        shift_by(c);
        bbias[0] = hi ? zero : (h16)(-c);
        l = expsum();
        pv(0);
    };
    enter(0);
    PST_SET(1, PST_NOW());
#pragma unroll
    for (int st = 0; st < DH / 16; ++st) qf[st] *= sc;
    if (active) block0();
    PST_SET(2, PST_NOW());
#pragma clang loop unroll(disable)
    for (int j = 1; j < nblk; ++j) {
        PST_MARK();
        enter(j);
        PST_ADDW();
        PST_MARK();
        if (active) {
            const int sbase = (j % NS) * SB;
            scores(64 * j, sbase);
            pv(sbase);
        }
        PST_ADDC();
    }
    PST_SUMS();
    PST_SET(5, PST_NOW());
    // (short sentences: the clamped prologue copies may still fly; none may land
    // after the workgroup is gone)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!active) return;
    // lds3's store phase: 1 / l, one permlane32 swap per dword of a chunk pair,
    // four 16-B bounds-checked stores per lane (rows >= len dropped)
    const float inv = 1.0f / halves_sum(l);
    const int q = q0 + 32 * w + lq;
    uint32_t pk[DH / 8][2];
#pragma unroll
    for (int m = 0; m < DH / 8; ++m)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int t = m >> 2, g = m & 3;
            const h16x2 v = {(h16)(o[t][4 * g + 2 * k] * inv), (h16)(o[t][4 * g + 2 * k + 1] * inv)};
            pk[m][k] = __builtin_bit_cast(uint32_t, v);
        }
#pragma unroll
    for (int p = 0; p < DH / 16; ++p)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * p][k], pk[2 * p + 1][k], false, false);
            pk[2 * p][k] = r[0];
            pk[2 * p + 1][k] = r[1];
        }
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc((void *)(out + (size_t)start * d), (short)0, len * d * 2, 0x00020000);
    const int ob = (q * d + h * DH + 8 * hi) * 2;
#pragma unroll
    for (int p = 0; p < DH / 16; ++p) {
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        const u32x4v v = {pk[2 * p][0], pk[2 * p][1], pk[2 * p + 1][0], pk[2 * p + 1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, ob + 32 * p, 0, 0);
    }
    PST_SET(6, PST_NOW());
    PST_HWID();
}

thread_local int g_att_variant = 0;   // benches only (bertx_bench_attention), per calling thread

// BERT_ATT_SHORT=0: short batches through attention_lds3 as well (A/B)
static bool att_short_env()
{
    static const bool on = [] { const char *e = std::getenv("BERT_ATT_SHORT"); return !(e && *e == '0'); }();
    return on;
}

void launch_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t max_len, int32_t n_head,
                      int32_t d, uint16_t *out, hipStream_t s)
{
    const int dh = d / n_head;
    const float sl2 = (1.0f / sqrtf((float)dh)) * 1.4426950408889634f;
    if (max_len <= ATT_LDS_MAX && (dh == 64 || dh == 32)) {
        const dim3 g(n_seqs * n_head), blk(1024);
        if (dh == 64) {
            // 0: production (attention_lds3, persistent, one workgroup per CU); 7:
            // the same kernel on at most 7 workgroups (tests: many ragged items each)
            const int n_items = n_seqs * n_head;
            // short batches (max_len <= 64): one 2-wave workgroup per item, lds3's
            // block-0 arithmetic (the same bits); variant 8 forces lds3 (tests, A/B)
            if (max_len <= 64 && g_att_variant != 7 && g_att_variant != 8 && att_short_env()) {
                if (n_items > 0)
                    attention_short_kernel<<<n_items, 128, 0, s>>>((const h16 *)qkv, cu, d, n_head, sl2, (h16 *)out);
                return;
            }
            // 64 < max_len <= 512: attention_pp (two 8-wave workgroups per CU, half an
            // item each: 66.2-67.1 vs lds3 67.5-68.2 us at C3, the same bits,
            // profiles/r06_attention_pp_ab.log); variant 7 / 8 or BERT_ATT_PP=0 run
            // attention_lds3 (tests, A/B)
            static const bool pp_env = [] { const char *e = std::getenv("BERT_ATT_PP"); return !(e && *e == '0'); }();
            if (g_att_variant != 7 && g_att_variant != 8 && pp_env) {
                if (n_items > 0)
                    attention_pp_kernel<<<2 * n_items, 512, 0, s>>>((const h16 *)qkv, cu, d, n_head, sl2, (h16 *)out);
                return;
            }
            const int cap = g_att_variant == 7 ? 7 : device_cu_count();
            const int grid = n_items < cap ? n_items : cap;
            if (grid > 0)
                attention_lds3_kernel<<<grid, 1024, 0, s>>>((const h16 *)qkv, cu, d, n_head, n_items, sl2, (h16 *)out);
        } else {
            attention_lds_kernel<32><<<g, blk, 0, s>>>((const h16 *)qkv, cu, d, n_head, sl2, (h16 *)out);
        }
        return;
    }
    const int nqt = (max_len + ATT_QT - 1) / ATT_QT;
    const int grid = nqt * n_head * n_seqs;
    if (dh == 64)
        attention_kernel<64><<<grid, 256, 0, s>>>((const h16 *)qkv, cu, d, nqt, n_head, sl2, (h16 *)out);
    else
        attention_kernel<32><<<grid, 256, 0, s>>>((const h16 *)qkv, cu, d, nqt, n_head, sl2, (h16 *)out);
}

}  // namespace emb
