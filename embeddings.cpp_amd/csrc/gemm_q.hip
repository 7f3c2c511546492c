// Quantized-weight GEMM for gfx950:  Y[m][n] = epi( sum_k X[m][k] * W[n][k] )
// with W in q4_0 / q4_1 / q8_0 ("register" layout of kernels.h) and X f16.
//
// The weights never touch LDS.  Each lane loads, with one 16-B (q4) or two
// 16-B (q8) loads per 32-feature subtile and K-step, exactly the nibbles /
// int8 of its own MFMA A fragments (the repack puts them contiguous), and
// expands them to f16 in registers, interleaved with the MFMAs of the previous
// k-slice.  LDS carries only the activations: a 3-stage LDS-DMA ring (XOR
// swizzled on the source address), two K-steps ahead.  Bytes moved per FLOP:
// 32 KiB of X + 8 KiB of q4 per 256 x 256 x 64 step; the weight bytes are read
// twice per workgroup (two waves along the tokens share each weight row).
//
// Workgroup 8 waves = 2 (tokens) x 4 (features), tile 256 tokens x BN features,
// wave tile 128 tokens x BN/4 features: NI = BN/128 ... (BN/4)/32 A fragments
// and 4 B fragments per k-slice.  MFMA v_mfma_f32_32x32x16_f16, A = W rows,
// B = X rows (the accumulator lane is a token).
//
// Per K-step: W(ks+1) to the other register set (ordinary loads), then
// X(ks+2) by LDS-DMA, then an explicit `s_waitcnt vmcnt(loads issued)` -- a
// run-time no-op that tells the compiler the current set has landed, so its
// waitcnt pass adds no vmcnt(0) (which would drain the ring) before the MFMAs.
// The loop is branch-free (past the end the issues re-read step KS-1), so the
// compiler sees a fixed count on every path.  At the end of the step
// `s_waitcnt vmcnt(4)` retires everything but X(ks+2).
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"

namespace emb {

namespace {

constexpr int GM = GEMM_BM;   // 256 tokens per tile
constexpr int GK = 64;
constexpr int XS = 3;                        // X stages
constexpr int X_BYTES = GM * GK * 2;          // 32 KiB

__device__ __forceinline__ int swz(int r, int c) { return (r << 7) | ((c ^ ((r >> 1) & 7)) << 4); }

// Weight words are ordinary (compiler-visible) loads: the compiler must own the
// registers of an in-flight load (an asm load's destination can be reused by
// the register allocator before the data arrives).  They are issued before the
// step's LDS-DMA, so the compiler's wait at their first use (next step) only
// retires X(ks+2), which has had a whole step of MFMAs to land.
__device__ __forceinline__ uint4 gload16(const void *p) { return *(const uint4 *)p; }
__device__ __forceinline__ uint32_t gload4(const void *p) { return *(const uint32_t *)p; }
// pin: an empty volatile asm that "rewrites" the registers, so their uses
// cannot be scheduled above the (side-effecting) explicit wait before it.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pin(uint4 &q)
{
    u32x4 v = __builtin_bit_cast(u32x4, q);
    asm volatile("" : "+v"(v));
    q = __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ void pin(uint32_t &v) { asm volatile("" : "+v"(v)); }

template <int FMT>
struct QRegs;   // one K-step of this lane's weight words for one 32-feature subtile

template <int FMT>
struct QRegsQ4 {
    uint4 q;           // words kk = 0..3 of lane half h
    uint32_t d, m;     // scale (and min) dword: (block 0, block 1)
    static constexpr int LOADS = FMT == FMT_Q4_1 ? 3 : 2;
    __device__ void load(const uint8_t *pq, const uint32_t *pd, const uint32_t *pm)
    {
        q = gload16(pq);
        d = gload4(pd);
        if (FMT == FMT_Q4_1) m = gload4(pm);
    }
    __device__ void pin_all() { pin(q); pin(d); if (FMT == FMT_Q4_1) pin(m); }
    // A fragment of k-slice kk: 8 f16 = (q - 8) d  |  q d + m
    __device__ h16x8 frag(int kk) const
    {
        const uint32_t w = kk == 0 ? q.x : kk == 1 ? q.y : kk == 2 ? q.z : q.w;
        const uint16_t dh = kk < 2 ? (uint16_t)(d & 0xffffu) : (uint16_t)(d >> 16);
        const h16x2 d2 = {as_h(dh), as_h(dh)};
        h16x2 m2 = {(h16)0.0f, (h16)0.0f};
        if (FMT == FMT_Q4_1) {
            const uint16_t mh = kk < 2 ? (uint16_t)(m & 0xffffu) : (uint16_t)(m >> 16);
            m2 = h16x2{as_h(mh), as_h(mh)};
        }
        const h16 o = FMT == FMT_Q4_1 ? (h16)-1024.0f : (h16)-1032.0f;
        const h16x2 off = {o, o};
        h16x8 a;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            h16x2 hh = as_h2(((w >> (4 * p)) & 0x000F000Fu) | 0x64006400u) + off;
            hh = FMT == FMT_Q4_1 ? hh * d2 + m2 : hh * d2;
            a[2 * p] = hh[0];
            a[2 * p + 1] = hh[1];
        }
        return a;
    }
};
template <> struct QRegs<FMT_Q4_0> : QRegsQ4<FMT_Q4_0> {};
template <> struct QRegs<FMT_Q4_1> : QRegsQ4<FMT_Q4_1> {};

template <>
struct QRegs<FMT_Q8_0> {
    uint4 q0, q1;      // 8 bytes per k-slice: kk 0,1 in q0, kk 2,3 in q1
    uint32_t d;
    static constexpr int LOADS = 3;
    __device__ void load(const uint8_t *pq, const uint32_t *pd, const uint32_t *)
    {
        q0 = gload16(pq);
        q1 = gload16(pq + 16);
        d = gload4(pd);
    }
    __device__ void pin_all() { pin(q0); pin(q1); pin(d); }
    __device__ h16x8 frag(int kk) const
    {
        const uint32_t w0 = kk == 0 ? q0.x : kk == 1 ? q0.z : kk == 2 ? q1.x : q1.z;
        const uint32_t w1 = kk == 0 ? q0.y : kk == 1 ? q0.w : kk == 2 ? q1.y : q1.w;
        const uint16_t dh = kk < 2 ? (uint16_t)(d & 0xffffu) : (uint16_t)(d >> 16);
        const h16x2 d2 = {as_h(dh), as_h(dh)};
        const h16x2 off = {(h16)-1152.0f, (h16)-1152.0f};   // bytes (q ^ 0x80), order e0 e2 e1 e3
        h16x8 a;
        const h16x2 p0 = (as_h2((w0 & 0x00FF00FFu) | 0x64006400u) + off) * d2;
        const h16x2 p1 = (as_h2(((w0 >> 8) & 0x00FF00FFu) | 0x64006400u) + off) * d2;
        const h16x2 p2 = (as_h2((w1 & 0x00FF00FFu) | 0x64006400u) + off) * d2;
        const h16x2 p3 = (as_h2(((w1 >> 8) & 0x00FF00FFu) | 0x64006400u) + off) * d2;
        a[0] = p0[0]; a[1] = p0[1]; a[2] = p1[0]; a[3] = p1[1];
        a[4] = p2[0]; a[5] = p2[1]; a[6] = p3[0]; a[7] = p3[1];
        return a;
    }
};

template <int FMT, int EPI, int BN>
__global__ __launch_bounds__(512, 1) void gemmq_kernel(DevWeight W, const h16 *__restrict__ X,
                                                       const float *__restrict__ bias, const float *__restrict__ res,
                                                       void *__restrict__ out, int nN, int nTiles)
{
    constexpr int NI = BN / 128;                          // 32-feature subtiles per wave
    constexpr int ES = EPI == EPI_BIAS_RES_F32 ? BN * 4 + 16 : BN * 2 + 16;   // staging row bytes
    constexpr int LDS_BYTES = (XS * X_BYTES > GM * ES) ? XS * X_BYTES : GM * ES;
    constexpr int QB = FMT == FMT_Q8_0 ? 64 : 32;           // weight bytes per (step, feature)
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x, xcd = b & 7, qq = nTiles >> 3, rr = nTiles & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int m0 = (t / nN) * GM, n0 = (t % nN) * BN;
    const int K = W.K, N = W.N, KS = K / GK;
    const int wm = wave >> 2, wn = wave & 3, lr = lane & 31, hi = lane >> 5;

    // X LDS-DMA sources: 4 instructions per wave, rows 32w + 8i + lane/8
    const h16 *xp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 32 * wave + 8 * i + (lane >> 3);
        xp[i] = X + (size_t)(m0 + r) * K + (((lane & 7) ^ ((r >> 1) & 7)) * 8);
    }
#define EMB_ISSUE_X(ks_, stage_)                                                                    \
    {                                                                                               \
        char *dst_ = smem + (stage_) * X_BYTES + ((32 * wave) << 7);                                \
        glds<16>(xp[0] + (ks_) * GK, dst_);                                                         \
        glds<16>(xp[1] + (ks_) * GK, dst_ + (8 << 7));                                              \
        glds<16>(xp[2] + (ks_) * GK, dst_ + (16 << 7));                                             \
        glds<16>(xp[3] + (ks_) * GK, dst_ + (24 << 7));                                             \
    }
    // weight sources of this lane: subtile i rows n0 + wn*BN/4 + 32i + lr, lane half hi
    const uint8_t *wq[NI];
    const uint32_t *wd[NI], *wmn[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int n = min(n0 + wn * (BN / 4) + 32 * i + lr, N - 1);
        wq[i] = (const uint8_t *)W.qs + (size_t)n * QB + (QB / 2) * hi;
        wd[i] = (const uint32_t *)W.d + n;
        wmn[i] = FMT == FMT_Q4_1 ? (const uint32_t *)W.m + n : nullptr;
    }
    const size_t qstep = (size_t)N * QB, sstep = (size_t)N;

    f32x16 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // Two register sets of weight words, used alternately (loop unrolled by two
    // so no copy ties an in-flight load to the set being multiplied).
    QRegs<FMT> wA[NI], wB[NI];
    // prologue: W(0) to registers, X(0), X(1) to LDS; retire all but X(1)
#pragma unroll
    for (int i = 0; i < NI; ++i) wA[i].load(wq[i], wd[i], wmn[i]);
    EMB_ISSUE_X(0, 0)
    if (KS > 1) {
        EMB_ISSUE_X(1, 1)
        wait_vmcnt<4>();
    } else {
        wait_vmcnt<0>();
    }
    lds_barrier();

    const int sw = (lr >> 1) & 7;
    int rb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = (wm * 128 + 32 * j + lr) << 7;
    int st = 0;

// One K-step: load the next step's weights into NXT, LDS-DMA X(ks+2), MFMAs
// with CUR, retire everything but X(ks+2), barrier.
#define EMB_QSTEP(CUR, NXT, ks_)                                                                          \
    {                                                                                                     \
        const int ksx = (ks_);                                                                            \
        const int st2 = st == 0 ? 2 : st - 1;                                                             \
        /* Branch-free: past the end the issues re-read step KS-1 (L2 hits; the */                        \
        /* registers / stage they fill are never read).  With a fixed count of */                         \
        /* ops in flight, the wait below is a run-time no-op that tells the */                            \
        /* compiler CUR has landed, so it adds no vmcnt(0) before the MFMAs. */                           \
        {                                                                                                 \
            const int k1 = min(ksx + 1, KS - 1), k2 = min(ksx + 2, KS - 1);                               \
            _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                \
                NXT[i].load(wq[i] + k1 * qstep, wd[i] + k1 * sstep,                                       \
                            FMT == FMT_Q4_1 ? wmn[i] + k1 * sstep : nullptr);                             \
            EMB_ISSUE_X(k2, st2)                                                                          \
            wait_vmcnt<NI * QRegs<FMT>::LOADS + 4>();                                                     \
            _Pragma("unroll") for (int i = 0; i < NI; ++i) CUR[i].pin_all();                              \
        }                                                                                                 \
        const char *xs = smem + st * X_BYTES;                                                             \
        h16x8 bf[4];                                                                                      \
        {                                                                                                 \
            const int cx = (hi ^ sw) << 4;                                                                \
            _Pragma("unroll") for (int j = 0; j < 4; ++j) bf[j] = *(const h16x8 *)(xs + rb[j] + cx);      \
        }                                                                                                 \
        _Pragma("unroll") for (int kk = 0; kk < 4; ++kk)                                                  \
        {                                                                                                 \
            h16x8 nb[4];                                                                                  \
            if (kk < 3) {                                                                                 \
                const int cx = ((2 * kk + 2 + hi) ^ sw) << 4;                                             \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) nb[j] = *(const h16x8 *)(xs + rb[j] + cx);  \
            }                                                                                             \
            _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                \
            {                                                                                             \
                const h16x8 a = CUR[i].frag(kk);                                                          \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) acc[i][j] =                                 \
                    __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bf[j], acc[i][j], 0, 0, 0);                 \
            }                                                                                             \
            if (kk < 3) {                                                                                 \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) bf[j] = nb[j];                              \
            }                                                                                             \
        }                                                                                                 \
        wait_vmcnt<4>(); /* NXT and X(ks+1) landed; X(ks+2) may fly */                                  \
        lds_barrier();                                                                                    \
        st = st == 2 ? 0 : st + 1;                                                                        \
    }

    for (int ks = 0; ks < KS; ks += 2) {
        EMB_QSTEP(wA, wB, ks)
        if (ks + 1 < KS) EMB_QSTEP(wB, wA, ks + 1)
    }
#undef EMB_QSTEP

    // ---- epilogue: stage the tile in LDS, write whole rows ----
    wait_vmcnt<0>();   // the clamped tail re-reads still write LDS
    lds_barrier();
    if constexpr (EPI == EPI_BIAS_RES_F32) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = wm * 128 + 32 * j + lr;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = wn * (BN / 4) + 32 * i + 8 * g + 4 * hi;
                    f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                    *(f32x4 *)(smem + m * ES + n * 4) = v;
                }
            }
        lds_barrier();
        constexpr int CPR = BN / 4, RPI = 512 / CPR;
        const int nl = (tid % CPR) * 4, gn = n0 + nl;
        if (gn >= N) return;
        const f32x4 bb = *(const f32x4 *)(bias + gn);
#pragma unroll 4
        for (int it = 0; it < GM / RPI; ++it) {
            const int m = it * RPI + tid / CPR;
            const size_t gm = (size_t)(m0 + m);
            const f32x4 v = *(const f32x4 *)(smem + m * ES + nl * 4);
            const f32x4 r = *(const f32x4 *)(res + gm * N + gn);
            f32x4 o;
            o[0] = r[0] + (bb[0] + v[0]); o[1] = r[1] + (bb[1] + v[1]);
            o[2] = r[2] + (bb[2] + v[2]); o[3] = r[3] + (bb[3] + v[3]);
            *(f32x4 *)((float *)out + gm * N + gn) = o;
        }
    } else {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = wn * (BN / 4) + 32 * i + 8 * g + 4 * hi;
                const f32x4 bb = *(const f32x4 *)(bias + min(n0 + n, N - 4));
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int m = wm * 128 + 32 * j + lr;
                    h16x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = bb[e] + acc[i][j][4 * g + e];
                        o[e] = EPI == EPI_BIAS_GELU_F16 ? gelu_era(v) : (h16)v;
                    }
                    *(h16x4 *)(smem + m * ES + n * 2) = o;
                }
            }
        lds_barrier();
        constexpr int CPR = BN / 8, RPI = 512 / CPR;
        const int nl = (tid % CPR) * 8, gn = n0 + nl;
        if (gn >= N) return;
#pragma unroll 4
        for (int it = 0; it < GM / RPI; ++it) {
            const int m = it * RPI + tid / CPR;
            *(uint4 *)((h16 *)out + (size_t)(m0 + m) * N + gn) = *(const uint4 *)(smem + m * ES + nl * 2);
        }
    }
}

template <int FMT, int BN>
void dispatch_q_bn(const DevWeight &W, const h16 *x, int M, const float *bias, int epi, const float *res, void *out,
                   hipStream_t s)
{
    const int nN = (W.N + BN - 1) / BN, nTiles = (M / GM) * nN;
    if (epi == EPI_BIAS_F16)
        gemmq_kernel<FMT, EPI_BIAS_F16, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
    else if (epi == EPI_BIAS_GELU_F16)
        gemmq_kernel<FMT, EPI_BIAS_GELU_F16, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
    else if constexpr (BN == 128)
        gemmq_kernel<FMT, EPI_BIAS_RES_F32, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
}

}  // namespace

void launch_gemm_q(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi, const float *res,
                   void *out, hipStream_t s, int32_t force_bn)
{
    const h16 *x = (const h16 *)X;
    const bool wide = force_bn ? (force_bn == 256 && epi != EPI_BIAS_RES_F32 && W.N % 256 == 0)
                               : (epi != EPI_BIAS_RES_F32 && W.N % 256 == 0 && (long)(M / GM) * (W.N / 256) >= 512);
    switch (W.fmt) {
    case FMT_Q4_0:
        if (wide) dispatch_q_bn<FMT_Q4_0, 256>(W, x, M, bias, epi, res, out, s);
        else dispatch_q_bn<FMT_Q4_0, 128>(W, x, M, bias, epi, res, out, s);
        break;
    case FMT_Q4_1:
        if (wide) dispatch_q_bn<FMT_Q4_1, 256>(W, x, M, bias, epi, res, out, s);
        else dispatch_q_bn<FMT_Q4_1, 128>(W, x, M, bias, epi, res, out, s);
        break;
    default:
        if (wide) dispatch_q_bn<FMT_Q8_0, 256>(W, x, M, bias, epi, res, out, s);
        else dispatch_q_bn<FMT_Q8_0, 128>(W, x, M, bias, epi, res, out, s);
        break;
    }
}

}  // namespace emb
