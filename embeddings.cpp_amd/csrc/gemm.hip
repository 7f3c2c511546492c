// f16-weight GEMM for gfx950:  Y[m][n] = epi( sum_k X[m][k] * W[n][k] )
//   X  f16 [M][K] activations (tokens x features), M a multiple of 256
//   W  f16 [N][K] weights (f16 files; f32 files converted at load) in the
//      K-step-major layout of kernels.h.  Quantized weights: gemm_q.hip.
//
// Workgroup = 8 waves (4 along tokens x 2 along features), tile 256 tokens x BN
// features x 64 k per step, BN = 256 for the wide projections (QKV, FFN-up)
// and 128 for the N = n_embd ones.  The bytes a CU must pull per FLOP set the
// speed here (the L2 -> LDS fill rate, not the MFMA): a 256 x 256 step moves
// 32 KiB of X + 8 KiB of q4 weights for 8.4 MFLOP.
//   * X arrives by LDS-DMA (global_load_lds_dwordx4) into a ring of stages with
//     an XOR swizzle applied to the per-lane SOURCE address (the LDS image stays
//     lane-linear, as LDS-DMA requires).
//   * W: f16 tiles arrive the same way; q-format tiles arrive raw (nibbles /
//     int8 + the row's f16 scale dword, per lane) by LDS-DMA into a staging
//     area, and the lane that loaded a block expands it to f16 into the
//     swizzled W stage (its own vmcnt orders that read; no other lane needs it).
//   * Every global load of the K loop is LDS-DMA; the loop waits with a full
//     vmcnt(0) only where that is the exact wait, so no prefetch is drained
//     early, and barriers are raw s_barrier (a __syncthreads drains vmcnt).
//   * MFMA v_mfma_f32_32x32x16_f16; A = W rows, B = X rows, so the accumulator
//     lane is a token and its registers hold runs of 4 consecutive features.
//   * Epilogue through LDS: bias / GELU applied in registers and the tile
//     staged (f16, or f32 for the residual form), then written as whole rows,
//     16 B per lane.
//   * Tiles are remapped so blocks that share an XCD (b, b+8, ...) walk
//     consecutive tiles of the same X rows: the X panel stays in that XCD's L2.
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"

namespace emb {

int g_force_bn = 0;   // tests: force the tile width (0 = heuristic)

namespace {

constexpr int GM = GEMM_BM;   // 256 tokens per tile
constexpr int GK = 64;        // k per step (two quant blocks)

template <int BN>
struct Cfg {
    static constexpr int XS = BN == 256 ? 2 : 3;             // X stages
    static constexpr int NI = BN / 64;                      // 32-feature subtiles per wave
    static constexpr int X_BYTES = GM * GK * 2;              // 32 KiB
    static constexpr int W_BYTES = BN * GK * 2;              // 16 / 32 KiB
    static constexpr int OFF_X = 0;
    static constexpr int OFF_W = OFF_X + XS * X_BYTES;        // 2 stages
    static constexpr int OFF_RQ = OFF_W + 2 * W_BYTES;        // raw quant payload of one step
    static constexpr int RQ_BYTES = BN == 256 ? 16384 : 8192;
    static constexpr int OFF_RS = OFF_RQ + RQ_BYTES;          // raw scale dwords, one per lane
    static constexpr int OFF_RM = OFF_RS + 2048;              // raw min dwords (q4_1)
    static constexpr int LDS_BYTES = OFF_RM + 2048;
};

// Byte offset of 16-byte chunk c (0..7) of row r in a [rows][64 x f16] image.
// Two 128-B rows share a 256-B bank row; XOR with (r>>1)&7 spreads the 16 rows
// of a ds_read_b128 lane group over all 16 slots.
__device__ __forceinline__ int swz(int r, int c) { return (r << 7) | ((c ^ ((r >> 1) & 7)) << 4); }

// X tile: 256 rows x 128 B = 32 LDS-DMA instructions, 4 per wave.
struct XSrc {
    const h16 *p[4];
    __device__ void init(const h16 *X, int K, int m0, int wave, int lane)
    {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 32 * wave + 8 * i + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            p[i] = X + (size_t)(m0 + r) * K + c * 8;
        }
    }
    __device__ void issue(int ks, char *xs, int wave) const
    {
#pragma unroll
        for (int i = 0; i < 4; ++i) glds<16>(p[i] + ks * GK, xs + ((32 * wave + 8 * i) << 7));
    }
};

// ---- weight paths: issue() starts the LDS-DMA of step ks, expand() makes the
// f16 W stage out of the raw bytes this lane loaded ----
template <int FMT, int BN>
struct WPath;

template <int BN>
struct WPath<FMT_F16, BN> {   // f16 (f32 files are converted at load)
    static constexpr int NL = BN / 64;   // instructions per wave
    const h16 *p[NL];
    size_t step;
    __device__ void init(const DevWeight &W, int n0, int wave, int lane)
    {
        step = (size_t)W.N * GK;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int r = (BN / 8) * wave + 8 * i + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            p[i] = (const h16 *)W.qs + (size_t)min(n0 + r, W.N - 1) * GK + c * 8;
        }
    }
    __device__ void issue(int ks, char *wst, char *, int wave) const
    {
#pragma unroll
        for (int i = 0; i < NL; ++i) glds<16>(p[i] + ks * step, wst + (((BN / 8) * wave + 8 * i) << 7));
    }
    __device__ void expand(char *, const char *, int, int) const {}
};

// Ablation switches (diagnostic builds only; production instantiates ABL = 0).
enum : int { ABL_NO_LOADS = 1, ABL_NO_EXPAND = 2, ABL_NO_MFMA = 4, ABL_NO_EPILOGUE = 8 };

template <int FMT, int EPI, int BN, int ABL = 0>
__global__ __launch_bounds__(512, 1) void gemm_kernel(DevWeight W, const h16 *__restrict__ X,
                                                      const float *__restrict__ bias, const float *__restrict__ res,
                                                      void *__restrict__ out, int nN, int nTiles)
{
    using C = Cfg<BN>;
    constexpr int NI = C::NI;
    __shared__ __attribute__((aligned(16))) char smem[C::LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware bijective remap: blocks b, b+8, ... (one XCD) get consecutive tiles
    const int b = blockIdx.x, xcd = b & 7, q = nTiles >> 3, rr = nTiles & 7;
    const int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
    const int m0 = (t / nN) * GM, n0 = (t % nN) * BN;
    const int K = W.K, N = W.N, KS = K / GK;
    const int wm = wave & 3, wn = wave >> 2, lr = lane & 31, hi = lane >> 5;

    XSrc xsrc;
    xsrc.init(X, K, m0, wave, lane);
    WPath<FMT, BN> wp;
    wp.init(W, n0, wave, lane);

    f32x16 acc[NI][2];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // prologue: W(0) and X(0) landed (+ X(1) in flight with 3 stages)
    wp.issue(0, smem + C::OFF_W, smem, wave);
    xsrc.issue(0, smem + C::OFF_X, wave);
    wait_vmcnt<0>();
    wp.expand(smem + C::OFF_W, smem, wave, lane);
    if (C::XS == 3 && KS > 1) xsrc.issue(1, smem + C::OFF_X + C::X_BYTES, wave);
    lds_barrier();

    // Step ks (2 X stages): issue W(ks+1), X(ks+1) -> MFMAs on step ks -> vmcnt(0)
    //   -> expand W(ks+1) -> barrier.
    // Step ks (3 X stages): issue W(ks+1) -> MFMAs -> vmcnt(0) -> expand W(ks+1)
    //   -> issue X(ks+2) -> barrier.
    // Either way vmcnt(0) is the exact wait (the loads it waits for are needed
    // next), so the compiler's own conservative waits drain nothing early.
    const int sw = (lr >> 1) & 7;   // swizzle key of every row this lane reads
    int ra[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) ra[i] = (wn * (BN / 2) + 32 * i + lr) << 7;
    const int rb0 = (wm * 64 + lr) << 7, rb1 = (wm * 64 + 32 + lr) << 7;
    int xs_cur = 0;
    for (int ks = 0; ks < KS; ++ks) {
        const bool more = ks + 1 < KS;
        const int xs_nxt = xs_cur + 1 == C::XS ? 0 : xs_cur + 1;
        const int xs_nn = xs_nxt + 1 == C::XS ? 0 : xs_nxt + 1;
        if (more && !(ABL & ABL_NO_LOADS)) {
            wp.issue(ks + 1, smem + C::OFF_W + ((ks + 1) & 1) * C::W_BYTES, smem, wave);
            if (C::XS == 2) xsrc.issue(ks + 1, smem + C::OFF_X + xs_nxt * C::X_BYTES, wave);
        }
        const char *xs = smem + C::OFF_X + xs_cur * C::X_BYTES;
        const char *ws = smem + C::OFF_W + (ks & 1) * C::W_BYTES;
        h16x8 a[NI], b0, b1;
        {
            const int cx = (hi ^ sw) << 4;
#pragma unroll
            for (int i = 0; i < NI; ++i) a[i] = *(const h16x8 *)(ws + ra[i] + cx);
            b0 = *(const h16x8 *)(xs + rb0 + cx);
            b1 = *(const h16x8 *)(xs + rb1 + cx);
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            h16x8 na[NI], nb0, nb1;
            if (kk < 3) {   // next fragments in flight under this k-slice's MFMAs
                const int cx = ((2 * kk + 2 + hi) ^ sw) << 4;
#pragma unroll
                for (int i = 0; i < NI; ++i) na[i] = *(const h16x8 *)(ws + ra[i] + cx);
                nb0 = *(const h16x8 *)(xs + rb0 + cx);
                nb1 = *(const h16x8 *)(xs + rb1 + cx);
            }
            if constexpr (!(ABL & ABL_NO_MFMA)) {
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b0, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b1, acc[i][1], 0, 0, 0);
                }
                __builtin_amdgcn_s_setprio(0);
            } else {
#pragma unroll
                for (int i = 0; i < NI; ++i) asm volatile("" ::"v"(a[i]), "v"(b0), "v"(b1));
            }
            if (kk < 3) {
#pragma unroll
                for (int i = 0; i < NI; ++i) a[i] = na[i];
                b0 = nb0;
                b1 = nb1;
            }
        }
        if (more) {
            wait_vmcnt<0>();
            if constexpr (!(ABL & ABL_NO_EXPAND)) wp.expand(smem + C::OFF_W + ((ks + 1) & 1) * C::W_BYTES, smem, wave, lane);
            if (C::XS == 3 && ks + 2 < KS && !(ABL & ABL_NO_LOADS))
                xsrc.issue(ks + 2, smem + C::OFF_X + xs_nn * C::X_BYTES, wave);
            lds_barrier();
        }
        xs_cur = xs_nxt;
    }

    // ---- epilogue ----
    if constexpr ((ABL & ABL_NO_EPILOGUE) != 0) {   // keep the accumulators alive, store one word per lane
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) s += acc[i][0][r] + acc[i][1][r];
        ((float *)out)[(size_t)blockIdx.x * 512 + tid] = s;
        return;
    }
    lds_barrier();   // every wave is done with the operand stages
    if constexpr (EPI == EPI_BIAS_RES_F32) {
        // f32 staging: 256 rows x (BN*4 + 16) B, then res + (bias + acc) per 16-B chunk
        constexpr int ES = BN * 4 + 16;
        static_assert(GM * ES <= C::LDS_BYTES, "f32 staging must fit");
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int m = wm * 64 + j * 32 + lr;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = wn * (BN / 2) + i * 32 + 8 * g + 4 * hi;
                    f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                    *(f32x4 *)(smem + m * ES + n * 4) = v;
                }
            }
        lds_barrier();
        constexpr int CPR = BN / 4;              // 16-B chunks per row
        constexpr int RPI = 512 / CPR;           // rows per pass
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
        // bias (+ GELU) in registers, f16 staging: 256 rows x (BN*2 + 16) B
        constexpr int ES = BN * 2 + 16;
        static_assert(GM * ES <= C::LDS_BYTES, "f16 staging must fit");
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = wn * (BN / 2) + i * 32 + 8 * g + 4 * hi;
                const f32x4 bb = *(const f32x4 *)(bias + min(n0 + n, N - 4));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int m = wm * 64 + j * 32 + lr;
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
        constexpr int CPR = BN / 8;              // 16-B chunks (8 x f16) per row
        constexpr int RPI = 512 / CPR;
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
void dispatch_bn(const DevWeight &W, const h16 *x, int M, const float *bias, int epi, const float *res, void *out,
                 hipStream_t s)
{
    const int nN = (W.N + BN - 1) / BN, nTiles = (M / GM) * nN;
    if (epi == EPI_BIAS_F16)
        gemm_kernel<FMT, EPI_BIAS_F16, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
    else if (epi == EPI_BIAS_GELU_F16)
        gemm_kernel<FMT, EPI_BIAS_GELU_F16, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
    else if constexpr (BN == 128)   // the f32 residual tile only fits 128 wide
        gemm_kernel<FMT, EPI_BIAS_RES_F32, BN><<<nTiles, 512, 0, s>>>(W, x, bias, res, out, nN, nTiles);
}

template <int FMT>
void dispatch(const DevWeight &W, const uint16_t *X, int M, const float *bias, int epi, const float *res, void *out,
              hipStream_t s)
{
    const h16 *x = (const h16 *)X;
    // 256-wide tiles halve the bytes per FLOP; use them when they still fill
    // the chip (>= 2 rounds of 256 CUs) and the residual (f32) epilogue is not needed.
    const bool wide = g_force_bn ? (g_force_bn == 256 && epi != EPI_BIAS_RES_F32 && W.N % 256 == 0)
                                 : (epi != EPI_BIAS_RES_F32 && W.N % 256 == 0 && (long)(M / GM) * (W.N / 256) >= 512);
    if (wide) dispatch_bn<FMT, 256>(W, x, M, bias, epi, res, out, s);
    else dispatch_bn<FMT, 128>(W, x, M, bias, epi, res, out, s);
}

}  // namespace

// Diagnostic: f16-weight / EPI_BIAS_F16 GEMM with ablation switches, tile 128 or 256.
template <int BN, int ABL>
static void abl_one(const DevWeight &W, const h16 *x, int M, const float *bias, void *out, hipStream_t s)
{
    const int nN = (W.N + BN - 1) / BN, nTiles = (M / GM) * nN;
    gemm_kernel<FMT_F16, EPI_BIAS_F16, BN, ABL><<<nTiles, 512, 0, s>>>(W, x, bias, nullptr, out, nN, nTiles);
}

template <int BN>
static void abl_bn(const DevWeight &W, const h16 *x, int M, const float *bias, void *out, hipStream_t s, int abl)
{
    switch (abl) {
    case 0: abl_one<BN, 0>(W, x, M, bias, out, s); break;
    case 1: abl_one<BN, 1>(W, x, M, bias, out, s); break;
    case 2: abl_one<BN, 2>(W, x, M, bias, out, s); break;
    case 3: abl_one<BN, 3>(W, x, M, bias, out, s); break;
    case 4: abl_one<BN, 4>(W, x, M, bias, out, s); break;
    case 6: abl_one<BN, 6>(W, x, M, bias, out, s); break;
    case 8: abl_one<BN, 8>(W, x, M, bias, out, s); break;
    case 11: abl_one<BN, 11>(W, x, M, bias, out, s); break;
    default: abl_one<BN, 15>(W, x, M, bias, out, s); break;
    }
}

void launch_gemm_ablation(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, void *out,
                          hipStream_t s, int32_t abl, int32_t bn)
{
    if (bn == 256) abl_bn<256>(W, (const h16 *)X, M, bias, out, s, abl);
    else abl_bn<128>(W, (const h16 *)X, M, bias, out, s, abl);
}

void launch_gemm(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi, const float *res,
                 void *out, hipStream_t s)
{
    if (W.fmt == FMT_Q4_0 || W.fmt == FMT_Q4_1 || W.fmt == FMT_Q8_0)
        launch_gemm_q(W, X, M, bias, epi, res, out, s, g_force_bn);   // weights in registers (gemm_q.hip)
    else
        dispatch<FMT_F16>(W, X, M, bias, epi, res, out, s);
}

}  // namespace emb
