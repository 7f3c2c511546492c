// Linear layers on v_mfma_f32_16x16x32_f16 (gfx950), weights in the "lane
// order" layout (kernels.h, DevWeight::layout == 1).
//
// Same contraction and epilogues as gemm.hip -- Y[m][n] = epi(sum_k X[m][k]
// W[n][k]) -- with the 16x16x32 MFMA: A = 16 features x 32 k (one quant block
// per feature), B = 32 k x 16 tokens.  The 16x16x32 loop holds a higher clock
// under load than the 32x32x16 loop at the same cycles per FLOP
// (MI355X_MICROARCH.md, DVFS give-back item 7), and one A fragment is exactly
// one quant block, so each lane's scale is a single f16.
//
// Workgroup = NW waves, tile BM tokens x 32*NW features; wave w owns features
// n0 + 32w .. +31 (two A fragments, a = 0/1 for +0 / +16) and all BM tokens
// (NJ = BM/16 B fragments per k-slice, each feeding two MFMAs).  Weights
// never touch LDS: each lane loads its own fragment words (16 B q4, 32 B q8,
// 64 B f16 per K-step, plus 8 B of scales) into a 3-set register ring two
// K-steps ahead and expands them between MFMAs.  X goes through an NS-stage
// LDS ring by LDS-DMA with the XOR swizzle on the source address (chunk
// c ^ ((row>>1)&7)), which keeps the 16x16x32 B-operand row read
// (ds_read_b128, lanes = 16 rows x 4 chunks) conflict-free.
//   NW 8, BM 256, NS 3: one workgroup per CU (96 KiB LDS)
//   NW 4, BM 256, NS 2 / BM 128, NS 4: two per CU (64 KiB each), so one's
//   epilogue overlaps the other's MFMAs.
// Epilogue: accumulator pairs of adjacent 16-token groups are exchanged with
// v_permlane16_swap so each lane owns 8 consecutive features of one token
// (16-B loads of bias/residual/LN parameters and one 16-B store).
#include "device_common.h"
#include "host_common.h"
#include "kernels.h"
#include "rowln.h"
#include "zregs.h"

#include <cstdio>
#include <cstdlib>
#include <utility>

namespace emb {
extern int g_gemm16_flags;
#ifndef EMB_ZABL
#define EMB_ZABL 0
#endif
// diagnostics builds only: K-loop ablations (1 no X DMA, 2 no weight loads,
// 4 no barrier, 8 no dequant (q4), 16 no MFMA) -- wrong results, timing only
constexpr int ZABL = EMB_ZABL;

namespace {

// 16-B store that bypasses L1/L2 retention (sc1): the panel hand-off below
// (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores by the
// producer, agent-scope counter add, agent acquire by the consumer).
typedef uint32_t zu32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_sc1(void *p, uint4 v)
{
    const zu32x4v d = __builtin_bit_cast(zu32x4v, v);
    // the s_nop covers the "VALU writes the data VGPRs of a >8-byte VMEM store"
    // hazard, which the compiler's hazard recognizer does not see through asm
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

// PLN (residual form only): 0, or NSL = 256-feature slices of a row -- the panel
// LayerNorm of ResLN (kernels.h) runs in the workgroup that completes its
// BM-row token panel last.  Opt-in (BERT_PANEL_LN=1): measured slower than the
// separate LN kernel (profiles/r01_panel_ln_ab.log) -- one workgroup's LN of a
// 128 x d panel is bound by that CU's load/store bandwidth.  rln.pvar: 0 = tile
// staged in LDS and stored as whole 128-B lines with sc1, 1 = direct sc1 stores.
__device__ __forceinline__ uint32_t lds_u32(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)p;
}

// ds_read_b128 at base + OFF with the read's completion tracked by hand: the
// asm keeps the issue order (hipcc's scheduler otherwise moves every read down
// next to its MFMAs), zwait_lgkm ties the data to a counted s_waitcnt.
template <int OFF>
__device__ __forceinline__ h16x8 zds_read(uint32_t base)
{
    h16x8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF));
    return r;
}
template <int N>
__device__ __forceinline__ void zwait_lgkm(h16x8 &r)
{
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r) : "i"(N));
}

// One K-step's MFMAs with the B fragments (s, j) -> item i = s NJ + j read PF
// items ahead of their two MFMAs (a ring of PF + 1 fragments).
// NWAIT >= 0 (EMB_ZNF builds): the first-half A fragments come in as fa0 / fa1
// and the next step's are dequantized in this step's second half, after a
// vmcnt(NWAIT) that retires the next step's weight loads (issued a step ago).
template <int NJ, int PF, int NWAIT, class R, class H, int... I>
__device__ __forceinline__ void zmma_items(const R &cur, R &nxt, h16x8 &fa0, h16x8 &fa1, uint32_t b0, uint32_t b1,
                                           f32x4 (&acc)[2][NJ], H &&hook, std::integer_sequence<int, I...>)
{
    constexpr int NI = 2 * NJ;
    h16x8 bq[PF + 1];
    auto rd = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NI) bq[i % (PF + 1)] = zds_read<(i % NJ) << 11>(i < NJ ? b0 : b1);
    };
    auto pre = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < PF) rd(std::integral_constant<int, i>{});
    };
    (pre(std::integral_constant<int, I>{}), ...);
    h16x8 a0, a1;
    if constexpr (NWAIT >= 0) { a0 = fa0; a1 = fa1; }
    else { a0 = cur.frag(0); a1 = cur.frag(2); }
    auto item = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        rd(std::integral_constant<int, i + PF>{});
        constexpr int last = (i + PF < NI ? i + PF : NI - 1);
        zwait_lgkm<last - i>(bq[i % (PF + 1)]);
        if constexpr (i == NJ) { a0 = cur.frag(1); a1 = cur.frag(3); }
        if constexpr (NWAIT >= 0 && i == NJ + NJ / 2) {
            wait_vmcnt<NWAIT>();
            nxt.pin_all();
            fa0 = nxt.frag(0);
            fa1 = nxt.frag(2);
        }
        const h16x8 bf = bq[i % (PF + 1)];
        if constexpr (ZABL & 16) {
            asm volatile("" ::"v"(bf), "v"(a0), "v"(a1));
        } else {
            acc[0][i % NJ] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf, acc[0][i % NJ], 0, 0, 0);
            acc[1][i % NJ] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bf, acc[1][i % NJ], 0, 0, 0);
        }
        hook(ic);
    };
    (item(std::integral_constant<int, I>{}), ...);
}
// One K-step's MFMAs on dequantized fragments f[0..3] (f[s], f[2 + s] for the
// k-half s), B fragments read PF items ahead (ping-pong kernel).
template <int NJ, int PF, int... I>
__device__ __forceinline__ void zpmma(const h16x8 (&f)[4], uint32_t b0, uint32_t b1, f32x4 (&acc)[2][NJ],
                                      std::integer_sequence<int, I...>)
{
    constexpr int NI = 2 * NJ;
    h16x8 bq[PF + 1];
    auto rd = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NI) bq[i % (PF + 1)] = zds_read<(i % NJ) << 11>(i < NJ ? b0 : b1);
    };
    auto pre = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < PF) rd(std::integral_constant<int, i>{});
    };
    (pre(std::integral_constant<int, I>{}), ...);
    auto item = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        rd(std::integral_constant<int, i + PF>{});
        constexpr int last = (i + PF < NI ? i + PF : NI - 1);
        zwait_lgkm<last - i>(bq[i % (PF + 1)]);
        constexpr int s = i / NJ;
        const h16x8 bf = bq[i % (PF + 1)];
        acc[0][i % NJ] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[s], bf, acc[0][i % NJ], 0, 0, 0);
        acc[1][i % NJ] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[2 + s], bf, acc[1][i % NJ], 0, 0, 0);
    };
    (item(std::integral_constant<int, I>{}), ...);
}

// hook(integral_constant<int, i>) runs after item i's MFMAs (memory issue spread
// through the step, EMB_ZSPREAD)
template <int NJ, int PF, int NWAIT, class R, class H>
__device__ __forceinline__ void zmma_step(const R &cur, R &nxt, h16x8 &fa0, h16x8 &fa1, uint32_t xs, uint32_t cx0,
                                          uint32_t cx1, f32x4 (&acc)[2][NJ], H &&hook)
{
    zmma_items<NJ, PF, NWAIT>(cur, nxt, fa0, fa1, xs + cx0, xs + cx1, acc, hook,
                              std::make_integer_sequence<int, 2 * NJ>{});
}

#ifndef EMB_ZBUF
#define EMB_ZBUF 1
#endif
#ifndef EMB_ZNF
#define EMB_ZNF 0
#endif
#ifndef EMB_ZSPREAD
#define EMB_ZSPREAD 0
#endif
#ifndef EMB_ZPF
#define EMB_ZPF 4
#endif
constexpr int ZPF = EMB_ZPF;   // B-fragment read-ahead in the K loop (A/B builds; 0 = reads beside their MFMAs)

// STAMP (diagnostics builds only): s_memtime at start / after the prologue /
// after the K loop / at the end, s_memrealtime at start and end, and the CU,
// per wave into stamps[(blockIdx * NW + wave) * 8 ..] (bertx_bench_gemm -3).
// The tile body: workgroup b of a grid of nTiles tiles (nN column tiles from
// feature nb0 on), staging X in `smem` (NS * BM * 128 B of LDS).
template <int FMT, int EPI, int NW, int BM, int NS, int PLN = 0, bool STAMP = false>
__device__ __forceinline__ void gemmz_body(char *__restrict__ smem, const int b, DevWeight W,
                                           const h16 *__restrict__ X, const float *__restrict__ bias,
                                           const void *__restrict__ res, void *__restrict__ out, int nN,
                                           int nTiles, ResLN rln, int fl, uint64_t *__restrict__ stamps, int nb0)
{
    uint64_t ts[4], rt0 = 0;
    if constexpr (STAMP) { ts[0] = __builtin_amdgcn_s_memtime(); rt0 = __builtin_amdgcn_s_memrealtime(); }
    constexpr int BN = 32 * NW;
    constexpr int NJ = BM / 16;                 // 16-token B fragments per k-slice
    constexpr int XB = BM * ZK * 2;             // bytes per X stage
    constexpr int XG = XB / (64 * NW * 16);     // LDS-DMA instructions per wave per stage
    constexpr int QB = ZRegs<FMT>::QB;
    constexpr int LQ = ZRegs<FMT>::LOADS;
    constexpr int P = LQ + XG;                  // vector-memory ops issued per K-step per wave
    static_assert(NS >= 2 && NS <= 4 && XG >= 1, "X ring");
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int xcd = b & 7, qq = nTiles >> 3, rr = nTiles & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int m0 = (t / nN) * BM, n0 = nb0 + (t % nN) * BN;
    const int K = W.K, N = W.N, KS = K / ZK;
    // A/B (fl bits 2-4 = n): first-round workgroups on every other CU of an XCD
    // start n x 8k cycles late -- do the store bursts of tiles finishing together
    // bound the epilogue?
    if ((fl >> 2) & 7) {
        if (b < 256 * (8 / NW) && ((b >> 3) & 1)) {
            for (int i = 0; i < ((fl >> 2) & 7); ++i) __builtin_amdgcn_s_sleep(127);
        }
    }
    const int fr = lane & 15, g = lane >> 4;
    const int nw = n0 + 32 * wave;              // this wave's first feature
    const int grp = min(nw, N - 32) >> 5;       // its 32-feature weight group (clamped past N)

    // LDS-DMA sources: instruction i of this wave fills rows 8*XG*wave + 8i + lane/8;
    // the swizzle ((row>>1)&7) only differs between even and odd i (XG even)
    static_assert(XG % 2 == 0, "XG even");
#if EMB_ZBUF
    // as buffer loads: the tile's BM rows are the buffer (out-of-range reads give
    // 0), one 32-bit offset VGPR per parity of i, the row step in soffset
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(X + (size_t)m0 * K), (short)0, BM * K * 2, 0x00020000);
    uint32_t xvo[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 8 * XG * wave + 8 * i + (lane >> 3);
        xvo[i] = (uint32_t)(r * K + (((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2u;
    }
#define EMB_ISSUE_XZ(ks_, stage_)                                                                   \
    {                                                                                               \
        char *dst_ = smem + (stage_) * XB + ((8 * XG * wave) << 7);                                 \
        _Pragma("unroll") for (int i = 0; i < XG; ++i)                                              \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t *)(dst_ + (i << 10)), 16,     \
                                                     xvo[i & 1], ((i >> 1) * 16 * K + (ks_) * ZK) * 2, 0, 0); \
    }
#else
    const h16 *xp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 8 * XG * wave + 8 * i + (lane >> 3);
        xp[i] = X + (size_t)(m0 + r) * K + (((lane & 7) ^ ((r >> 1) & 7)) * 8);
    }
    const size_t xrow8 = (size_t)16 * K;        // 16 rows: i -> i + 2
#define EMB_ISSUE_XZ(ks_, stage_)                                                                   \
    {                                                                                               \
        char *dst_ = smem + (stage_) * XB + ((8 * XG * wave) << 7);                                 \
        _Pragma("unroll") for (int i = 0; i < XG; ++i)                                              \
            glds<16>(xp[i & 1] + (i >> 1) * xrow8 + (ks_) * ZK, dst_ + (i << 10));                  \
    }
#endif
    const uint8_t *wq = (const uint8_t *)W.qs + ((size_t)grp * 64 + lane) * QB;
    const uint16_t *wd = W.d + ((size_t)grp * 16 + fr) * 4;
    const uint16_t *wmn = FMT == FMT_Q4_1 ? W.m + ((size_t)grp * 16 + fr) * 4 : nullptr;
    const size_t qstep = (size_t)N * 2 * QB, sstep = (size_t)N * 2;

    f32x4 acc[2][NJ];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    ZRegs<FMT> w0, w1, w2;
    const int k1 = min(1, KS - 1);
    w0.load(wq, wd, wmn);
    EMB_ISSUE_XZ(0, 0)
    if constexpr (NS == 2) {
        w1.load(wq + k1 * qstep, wd + k1 * sstep, FMT == FMT_Q4_1 ? wmn + k1 * sstep : nullptr);
        wait_vmcnt<LQ>();
    } else if constexpr (NS == 3) {
        asm volatile("" ::: "memory");
        w1.load(wq + k1 * qstep, wd + k1 * sstep, FMT == FMT_Q4_1 ? wmn + k1 * sstep : nullptr);
        asm volatile("" ::: "memory");
        EMB_ISSUE_XZ(k1, 1)
        wait_vmcnt<P>();
    } else {
        EMB_ISSUE_XZ(k1, 1)
        asm volatile("" ::: "memory");
        w1.load(wq + k1 * qstep, wd + k1 * sstep, FMT == FMT_Q4_1 ? wmn + k1 * sstep : nullptr);
        asm volatile("" ::: "memory");
        EMB_ISSUE_XZ(min(2, KS - 1), 2)
        wait_vmcnt<P + XG>();
    }
    lds_barrier();
    if constexpr (STAMP) ts[1] = __builtin_amdgcn_s_memtime();

    const int sw = (fr >> 1) & 7;
    const int rbase = fr << 7;
    int st = 0;
    // EMB_ZNF: vmcnt that retires the next step's weights mid-step (see zmma_items):
    // the loads issued after them are one X stage (NS 2) or two (NS 3, 4) and one
    // weight set
    constexpr int ZNW = EMB_ZNF ? (NS == 2 ? XG + LQ : 2 * XG + LQ) : -1;
    // EMB_ZSPREAD (2-stage ring, buffer DMA): the step's memory issue spread
    // between its first-half MFMAs instead of bunched at the step start
    constexpr bool SPREAD = EMB_ZSPREAD > 0 && NS == 2 && EMB_ZBUF && ZPF > 0 && !EMB_ZNF && EMB_ZSPREAD * XG <= 2 * NJ;
    h16x8 fa0{}, fa1{};
    if constexpr (ZNW >= 0) {
        w0.pin_all();
        fa0 = w0.frag(0);
        fa1 = w0.frag(2);
    }

// One K-step with CUR's weights (see gemm.hip EMB_VSTEP for the wait logic).
#define EMB_ZSTEP(CUR, NXT, NXT2, ks_)                                                                         \
    {                                                                                                     \
        const int ksx = (ks_);                                                                            \
        {                                                                                                 \
            const int kx = min(ksx + NS - 1, KS - 1), k2 = min(ksx + 2, KS - 1);                          \
            const int sx = st == 0 ? NS - 1 : st - 1;                                                     \
            if constexpr (SPREAD) {                                                                       \
                /* W(ks) retired by the previous step's closing vmcnt */                                  \
            } else if constexpr (NS == 2) {                                                               \
                if constexpr (!(ZABL & 1)) EMB_ISSUE_XZ(kx, sx)                                           \
                asm volatile("" ::: "memory");                                                            \
                if constexpr (!(ZABL & 2))                                                                \
                NXT2.load(wq + k2 * qstep, wd + k2 * sstep, FMT == FMT_Q4_1 ? wmn + k2 * sstep : nullptr); \
                wait_vmcnt<2 * LQ + XG>();                                                                \
            } else {                                                                                      \
                NXT2.load(wq + k2 * qstep, wd + k2 * sstep, FMT == FMT_Q4_1 ? wmn + k2 * sstep : nullptr); \
                asm volatile("" ::: "memory");                                                            \
                EMB_ISSUE_XZ(kx, sx)                                                                      \
                wait_vmcnt<2 * P + (NS == 4 ? XG : 0)>();                                                 \
            }                                                                                             \
            CUR.pin_all();                                                                                \
        }                                                                                                 \
        const char *xs = smem + st * XB + rbase;                                                          \
        if constexpr (ZPF == 0) {                                                                         \
        _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                     \
        {                                                                                                 \
            const int cx = ((4 * s + g) ^ sw) << 4;                                                       \
            const h16x8 a0 = CUR.frag(s), a1 = CUR.frag(2 + s);                                           \
            _Pragma("unroll") for (int j = 0; j < NJ; ++j)                                                \
            {                                                                                             \
                const h16x8 bf = *(const h16x8 *)(xs + (j << 11) + cx);                                   \
                acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf, acc[0][j], 0, 0, 0);           \
                acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bf, acc[1][j], 0, 0, 0);           \
            }                                                                                             \
        }                                                                                                 \
        } else {                                                                                          \
            const int kxs = min(ksx + 1, KS - 1), k2s = min(ksx + 2, KS - 1);                             \
            char *dsts = smem + (st == 0 ? 1 : 0) * XB + ((8 * XG * wave) << 7);                          \
            auto hook = [&](auto ic) {                                                                    \
                constexpr int i = decltype(ic)::value;                                                    \
                if constexpr (SPREAD) {                                                                   \
                    /* the XG X pieces of step ks+1 after every EV-th item of the first half, */          \
                    /* then W(ks+2): the step's closing vmcnt(LQ) retires the pieces */                   \
                    constexpr int EV = EMB_ZSPREAD;                                                       \
                    if constexpr (i % EV == EV - 1 && i / EV < XG) {                                      \
                        constexpr int j = i / EV;                                                         \
                        asm volatile("" ::: "memory");                                                    \
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t *)(dsts + (j << 10)), 16, \
                                                                 xvo[j & 1], ((j >> 1) * 16 * K + kxs * ZK) * 2, 0, 0); \
                        asm volatile("" ::: "memory");                                                    \
                    }                                                                                     \
                    if constexpr (i == EV * XG - 1)                                                       \
                        NXT2.load(wq + k2s * qstep, wd + k2s * sstep, FMT == FMT_Q4_1 ? wmn + k2s * sstep : nullptr); \
                }                                                                                         \
            };                                                                                            \
            zmma_step<NJ, ZPF, ZNW>(CUR, NXT, fa0, fa1, lds_u32(xs), (g ^ sw) << 4, ((4 + g) ^ sw) << 4, acc, hook); \
        }                                                                                                 \
        if constexpr (NS == 2) wait_vmcnt<LQ>();                                                          \
        else if constexpr (NS == 3) wait_vmcnt<P>();                                                      \
        else wait_vmcnt<P + XG>();                                                                        \
        if constexpr (ZABL & 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                       \
        else lds_barrier();                                                                               \
        st = st == NS - 1 ? 0 : st + 1;                                                                   \
    }

    // A/B flag 1: the second half of an 8-wave workgroup (the arbitration loser
    // on every SIMD, MI355X_MICROARCH.md "Two waves per SIMD" item 4) at priority 1
    if ((fl & 1) && NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
    int ks = 0;
    for (; ks + 3 <= KS; ks += 3) {
        EMB_ZSTEP(w0, w1, w2, ks)
        EMB_ZSTEP(w1, w2, w0, ks + 1)
        EMB_ZSTEP(w2, w0, w1, ks + 2)
    }
    if (ks < KS) {
        EMB_ZSTEP(w0, w1, w2, ks)
        if (ks + 1 < KS) EMB_ZSTEP(w1, w2, w0, ks + 1)
    }
#undef EMB_ZSTEP
#undef EMB_ISSUE_XZ
    wait_vmcnt<0>();
    if constexpr (STAMP) ts[2] = __builtin_amdgcn_s_memtime();

    // ---- epilogue ----
    // acc[a][j] lane (g, fr): token m0 + 16j + fr, features nw + 16a + 4g + 0..3.
    // After the permlane16 exchange of (acc[a][j], acc[a][j+1]) the lane holds
    // token m0 + 16(j + (g&1)) + fr, features nw + 16a + 8(g>>1) + 0..7.
    if (nw >= N) return;                        // wave-uniform (N % 32 == 0)
    f32x4 bb[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const float *bp = bias + nw + 16 * a + 8 * (g >> 1);
        bb[a][0] = *(const f32x4 *)bp;
        bb[a][1] = *(const f32x4 *)(bp + 4);
    }
    f32x4 lw[2][2], lb[2][2];
    if (EPI == EPI_BIAS_RES && rln.stats) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int c = nw + 16 * a + 8 * (g >> 1);
            lw[a][0] = *(const f32x4 *)(rln.w + c);
            lw[a][1] = *(const f32x4 *)(rln.w + c + 4);
            lb[a][0] = *(const f32x4 *)(rln.b + c);
            lb[a][1] = *(const f32x4 *)(rln.b + c + 4);
        }
    }
    // residual form: every residual row chunk and LN statistic of up to 8 token
    // pairs in flight before the first use (one latency, not one per pair)
    constexpr int JC = NJ < 16 ? NJ : 8;        // token groups per prefetch chunk
#pragma unroll
    for (int jc = 0; jc < NJ; jc += JC) {
    uint4 rr[JC / 2][2];
    float2 sts[JC / 2];
    if constexpr (EPI == EPI_BIAS_RES) {
#pragma unroll
        for (int jp = 0; jp < JC / 2; ++jp) {
            const int tok = m0 + 16 * (jc + 2 * jp + (g & 1)) + fr;
            sts[jp] = rln.stats ? rln.stats[tok] : float2{0.f, 1.f};
#pragma unroll
            for (int a = 0; a < 2; ++a)
                rr[jp][a] = *(const uint4 *)((const h16 *)res + (size_t)tok * N + nw + 16 * a + 8 * (g >> 1));
        }
    }
#pragma unroll
    for (int j = jc; j < jc + JC; j += 2) {
        const int tok = m0 + 16 * (j + (g & 1)) + fr;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = acc[a][j][e];
                v[4 + e] = acc[a][j + 1][e];
                zswap(v[e], v[4 + e]);
            }
            const int c = nw + 16 * a + 8 * (g >> 1);
            const size_t o = (size_t)tok * N + c;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bb[a][e >> 2][e & 3];
            uint4 pk;
            uint32_t *pw = (uint32_t *)&pk;
            if constexpr (EPI == EPI_BIAS_RES) {
                const h16x8 rh = __builtin_bit_cast(h16x8, rr[(j - jc) >> 1][a]);
                const float2 stt = sts[(j - jc) >> 1];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float r = (float)rh[e];
                    if (rln.stats) r = ln_apply(r, stt.x, stt.y, lw[a][e >> 2][e & 3], lb[a][e >> 2][e & 3]);
                    v[e] += r;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    pw[e] = __builtin_bit_cast(uint32_t, h16x2{(h16)v[2 * e], (h16)v[2 * e + 1]});
            } else if constexpr (EPI == EPI_BIAS_GELU_F16) {
#pragma unroll
                for (int e = 0; e < 4; ++e) pw[e] = gelu2_era(v[2 * e], v[2 * e + 1]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    pw[e] = __builtin_bit_cast(uint32_t, h16x2{(h16)v[2 * e], (h16)v[2 * e + 1]});
            }
            if constexpr (PLN != 0) {
                if (rln.pvar == 1) store16_sc1((h16 *)out + o, pk);
                else {
                    // stage the tile in LDS (16-B chunk index swizzled by row & 15)
                    const int rw = tok - m0, ch = (c - n0) >> 3;
                    *(uint4 *)(smem + (rw << 8) + ((ch ^ (rw & 15)) << 4)) = pk;
                }
            } else {
                *(uint4 *)((h16 *)out + o) = pk;
            }
        }
    }
    }

    if constexpr (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ts[3] = __builtin_amdgcn_s_memtime();
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        if (lane == 0) {
            uint64_t *o = stamps + ((size_t)b * NW + wave) * 8;
            for (int i = 0; i < 4; ++i) o[i] = ts[i];
            o[4] = rt0; o[5] = rt1; o[6] = ((uint64_t)xcc << 32) | hw;
        }
    }

    if constexpr (EPI == EPI_BIAS_RES && PLN != 0) {
        if (rln.pvar != 1) {
            // whole 128-B lines from the staged tile: a row's 256 B by 16 lanes
            __syncthreads();
            const int ch = tid & 15;
#pragma unroll
            for (int i = 0; i < BM / 16; ++i) {
                const int rw = (tid >> 4) + 16 * i;
                const uint4 v = *(const uint4 *)(smem + (rw << 8) + ((ch ^ (rw & 15)) << 4));
                h16 *dst = (h16 *)out + (size_t)(m0 + rw) * N + n0 + 8 * ch;
                store16_sc1(dst, v);
            }
        }
        // every wave's stores of this tile have landed; then one counter add per
        // workgroup; the workgroup whose add completes the panel normalises it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        volatile int *flag = (volatile int *)smem;
        if (tid == 0) {
            uint32_t *c = rln.cnt + m0 / BM;
            const uint32_t old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == (uint32_t)(nN - 1);
            if (last) {
                __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // ready for the next launch
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            *flag = last;
        }
        __syncthreads();
        if (*flag)
            ln_rows<4 * PLN, NW>((const h16 *)out, m0, min(m0 + BM, rln.rows), N, wave, lane, rln.nw, rln.nb,
                             (h16 *)rln.xh, rln.st_out);
    }
}

template <int FMT, int EPI, int NW, int BM, int NS, int PLN = 0, bool STAMP = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void gemmz_kernel(DevWeight W, const h16 *__restrict__ X,
                                                               const float *__restrict__ bias,
                                                               const void *__restrict__ res, void *__restrict__ out,
                                                               int nN, int nTiles, ResLN rln, int fl,
                                                               uint64_t *__restrict__ stamps = nullptr)
{
    __shared__ __attribute__((aligned(16))) char smem[NS * BM * ZK * 2];
    gemmz_body<FMT, EPI, NW, BM, NS, PLN, STAMP>(smem, blockIdx.x, W, X, bias, res, out, nN, nTiles, rln, fl,
                                                 stamps, 0);
}

// The column split of z_split_cols in ONE launch: workgroups [0, nA) are 256 x 128
// tiles of features [0, nbB), the rest 128 x 128 tiles of features [nbB, N).  Both
// shapes stage 64 KiB and run two workgroups per CU, so the small tiles take the
// slots the large ones free, with no launch boundary between the two.
template <int FMT, int EPI>
__global__ __launch_bounds__(256, 2) void gemmz_split_kernel(DevWeight W, const h16 *__restrict__ X,
                                                            const float *__restrict__ bias,
                                                            const void *__restrict__ res, void *__restrict__ out,
                                                            int nNA, int nA, int nNB, int nB, int nbB, ResLN rln,
                                                            int fl)
{
    static_assert(2 * 256 * ZK * 2 == 4 * 128 * ZK * 2, "one LDS footprint for both shapes");
    __shared__ __attribute__((aligned(16))) char smem[2 * 256 * ZK * 2];
    const int b = blockIdx.x;
    if (b < nA)
        gemmz_body<FMT, EPI, 4, 256, 2>(smem, b, W, X, bias, res, out, nNA, nA, rln, fl, nullptr, 0);
    else
        gemmz_body<FMT, EPI, 4, 128, 4>(smem, b - nA, W, X, bias, res, out, nNB, nB, rln, fl, nullptr, nbB);
}

// Co-resident 4-wave workgroups the device holds at once (two per CU).
int z_slots()
{
    static const int slots = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return 2 * cus;
    }();
    return slots;
}

// Column split of the 256 x 128 form: a grid of P x nN tiles that is not whole
// rounds of the slots ends in a part-filled round whose workgroups run alone on
// their CUs (C3: FFN-down / O-proj 768 tiles = 1.5 rounds, QKV 2304 = 4.5).
// Returns the largest n1 < nN whose P x n1 tiles ARE whole rounds; the columns
// from 128 n1 on then run as 128 x 128 tiles (twice the tiles at half the work,
// so the last round is full).  The per-wave arithmetic is the same in both
// shapes: the output is bitwise that of the unsplit grid.  0 = no split.
// Measured in the forward at C3 (gpurun_out r01g): QKV 114 -> 119 us, FFN-down
// 149.4 -> 148.3, O-proj 59.3 -> 58.3, 8,927 -> 8,760 sentences/s -- the lone
// workgroups of the part-filled round run nearly twice as fast as paired ones,
// so that round costs far less than a full one.  For the residual forms alone
// (BERT_GEMM16_SPLIT=r) the evented kernel times improve (O-proj 60.2 -> 57.4,
// FFN-down 149.7 -> 148.5 us) but the graph-replayed forward does not (9,010 ->
// 8,888 sentences/s, three runs each, gpurun_out r01m).  Off by default:
// BERT_GEMM16_SPLIT=1 turns it on (A/B); tile config 5 forces it (tests).
int z_split_cols(int M, int N)
{
    const int P = M / 256, nN = N / 128, slots = z_slots();
    if ((long)P * nN % slots == 0) return 0;
    for (int n1 = nN - 1; n1 >= 1; --n1)
        if ((long)P * n1 % slots == 0) return n1;
    return 0;
}

template <int FMT>
void dispatch_split(const DevWeight &W, const h16 *x, int M, const float *bias, int epi, const void *res, void *out,
                    hipStream_t s, const ResLN &rln, int n1)
{
    const int nA = (M / 256) * n1, nbB = 128 * n1, nNB = (W.N - nbB + 127) / 128, nB = (M / 128) * nNB;
    const int fl = g_gemm16_flags;
    if (epi == EPI_BIAS_F16)
        gemmz_split_kernel<FMT, EPI_BIAS_F16><<<nA + nB, 256, 0, s>>>(W, x, bias, res, out, n1, nA, nNB, nB, nbB, rln, fl);
    else if (epi == EPI_BIAS_GELU_F16)
        gemmz_split_kernel<FMT, EPI_BIAS_GELU_F16><<<nA + nB, 256, 0, s>>>(W, x, bias, res, out, n1, nA, nNB, nB, nbB,
                                                                            rln, fl);
    else
        gemmz_split_kernel<FMT, EPI_BIAS_RES><<<nA + nB, 256, 0, s>>>(W, x, bias, res, out, n1, nA, nNB, nB, nbB, rln, fl);
}

// Epilogue straight from the accumulators (as gemmz_kernel without the panel
// LN): acc[a][j] lane (g, fr) = token m0 + 16j + fr, features nw + 16a + 4g + 0..3.
template <int EPI, int NJ>
__device__ __forceinline__ void zepilogue(f32x4 (&acc)[2][NJ], int m0, int nw, int N, int g, int fr,
                                          const float *__restrict__ bias, const void *__restrict__ res,
                                          void *__restrict__ out, const ResLN &rln)
{
    f32x4 bb[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const float *bp = bias + nw + 16 * a + 8 * (g >> 1);
        bb[a][0] = *(const f32x4 *)bp;
        bb[a][1] = *(const f32x4 *)(bp + 4);
    }
    f32x4 lw[2][2], lb[2][2];
    if (EPI == EPI_BIAS_RES && rln.stats) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int c = nw + 16 * a + 8 * (g >> 1);
            lw[a][0] = *(const f32x4 *)(rln.w + c);
            lw[a][1] = *(const f32x4 *)(rln.w + c + 4);
            lb[a][0] = *(const f32x4 *)(rln.b + c);
            lb[a][1] = *(const f32x4 *)(rln.b + c + 4);
        }
    }
    constexpr int JC = NJ < 16 ? NJ : 8;
#pragma unroll
    for (int jc = 0; jc < NJ; jc += JC) {
        uint4 rr[JC / 2][2];
        float2 sts[JC / 2];
        if constexpr (EPI == EPI_BIAS_RES) {
#pragma unroll
            for (int jp = 0; jp < JC / 2; ++jp) {
                const int tok = m0 + 16 * (jc + 2 * jp + (g & 1)) + fr;
                sts[jp] = rln.stats ? rln.stats[tok] : float2{0.f, 1.f};
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    rr[jp][a] = *(const uint4 *)((const h16 *)res + (size_t)tok * N + nw + 16 * a + 8 * (g >> 1));
            }
        }
#pragma unroll
        for (int j = jc; j < jc + JC; j += 2) {
            const int tok = m0 + 16 * (j + (g & 1)) + fr;
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = acc[a][j][e];
                    v[4 + e] = acc[a][j + 1][e];
                    zswap(v[e], v[4 + e]);
                }
                const size_t o = (size_t)tok * N + nw + 16 * a + 8 * (g >> 1);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += bb[a][e >> 2][e & 3];
                uint4 pk;
                uint32_t *pw = (uint32_t *)&pk;
                if constexpr (EPI == EPI_BIAS_RES) {
                    const h16x8 rh = __builtin_bit_cast(h16x8, rr[(j - jc) >> 1][a]);
                    const float2 stt = sts[(j - jc) >> 1];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float r = (float)rh[e];
                        if (rln.stats) r = ln_apply(r, stt.x, stt.y, lw[a][e >> 2][e & 3], lb[a][e >> 2][e & 3]);
                        v[e] += r;
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        pw[e] = __builtin_bit_cast(uint32_t, h16x2{(h16)v[2 * e], (h16)v[2 * e + 1]});
                } else if constexpr (EPI == EPI_BIAS_GELU_F16) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) pw[e] = gelu2_era(v[2 * e], v[2 * e + 1]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        pw[e] = __builtin_bit_cast(uint32_t, h16x2{(h16)v[2 * e], (h16)v[2 * e + 1]});
                }
                *(uint4 *)((h16 *)out + o) = pk;
            }
        }
    }
}

// Ping-pong GEMM (cfg 4): one 8-wave workgroup per CU, tile 256 tokens x 256
// features, each wave 32 features x 256 tokens.  The two waves of every SIMD
// (wave w and w + 4: halves A = waves 0-3, B = waves 4-7) alternate roles
// phase by phase, separated by s_barrier (MI355X_MICROARCH.md "Two waves per
// SIMD"): while one half runs a K-step's 64 MFMAs (B fragments from LDS), the
// other issues its share of the X LDS-DMA and weight loads two steps ahead and
// dequantizes its next step's A fragments, so the matrix pipe of each SIMD
// always has one wave feeding it.  Per K-step k (phase t = 2k, 2k + 1):
//   A: compute(k) | barrier | load(k + 2), dequant(k + 1) | barrier
//   B: load(k + 2), dequant(k) | barrier | compute(k) | barrier
// X(k + 2) overwrites the stage of X(k - 1), whose last reader (B) finished in
// phase 2k - 1; X(k) is complete (every wave's vmcnt, then a barrier) before
// phase 2k.  Weights ring of 3 sets per wave, stages NS = 3 (96 KB).
template <int FMT, int EPI>
__global__ __launch_bounds__(512, 1) void gemmp_kernel(DevWeight W, const h16 *__restrict__ X,
                                                       const float *__restrict__ bias, const void *__restrict__ res,
                                                       void *__restrict__ out, int nN, int nTiles, ResLN rln)
{
    constexpr int NW = 8, BM = 256, BN = 256, NJ = 16, NS = 3;
    constexpr int XB = BM * ZK * 2;             // 32 KB per stage
    constexpr int XG = XB / (64 * NW * 16);     // 4 DMA pieces per wave per stage
    constexpr int QB = ZRegs<FMT>::QB;
    constexpr int LQ = ZRegs<FMT>::LOADS;
    constexpr int PF = ZPF > 0 ? ZPF : 4;
    __shared__ __attribute__((aligned(16))) char smem[NS * XB];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int half = wave >> 2;
    const int b = blockIdx.x, xcd = b & 7, qq = nTiles >> 3, rr = nTiles & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int m0 = (t / nN) * BM, n0 = (t % nN) * BN;
    const int K = W.K, N = W.N, KS = K / ZK;
    const int fr = lane & 15, g = lane >> 4;
    const int nw = n0 + 32 * wave;
    const int grp = min(nw, N - 32) >> 5;

    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(X + (size_t)m0 * K), (short)0, BM * K * 2, 0x00020000);
    uint32_t xvo[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 8 * XG * wave + 8 * i + (lane >> 3);
        xvo[i] = (uint32_t)(r * K + (((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2u;
    }
    auto dma = [&](int ks, int stage) {
        char *dst = smem + stage * XB + ((8 * XG * wave) << 7);
#pragma unroll
        for (int i = 0; i < XG; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t *)(dst + (i << 10)), 16, xvo[i & 1],
                                                     ((i >> 1) * 16 * K + ks * ZK) * 2, 0, 0);
    };
    const uint8_t *wq = (const uint8_t *)W.qs + ((size_t)grp * 64 + lane) * QB;
    const uint16_t *wd = W.d + ((size_t)grp * 16 + fr) * 4;
    const uint16_t *wmn = FMT == FMT_Q4_1 ? W.m + ((size_t)grp * 16 + fr) * 4 : nullptr;
    const size_t qstep = (size_t)N * 2 * QB, sstep = (size_t)N * 2;
    auto wload = [&](ZRegs<FMT> &w, int ks) {
        w.load(wq + ks * qstep, wd + ks * sstep, FMT == FMT_Q4_1 ? wmn + ks * sstep : nullptr);
    };

    f32x4 acc[2][NJ];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    ZRegs<FMT> w0, w1, w2;
    const int k1 = min(1, KS - 1);
    wload(w0, 0);
    dma(0, 0);
    wload(w1, k1);
    dma(k1, 1);
    wait_vmcnt<0>();
    lds_barrier();

    const int sw = (fr >> 1) & 7;
    const int rbase = fr << 7;
    const uint32_t cx0 = (g ^ sw) << 4, cx1 = ((4 + g) ^ sw) << 4;
    h16x8 f[4];                                 // the next compute's A fragments
    auto deq = [&](ZRegs<FMT> &w) {
        w.pin_all();
#pragma unroll
        for (int u = 0; u < 4; ++u) f[u] = w.frag(u);
    };
    // load phase for step ks: W(ks + 2) and X(ks + 2) (skipped past the end),
    // then every older load of this wave retired
    auto load = [&](ZRegs<FMT> &wn2, int ks) {
        if (ks + 2 < KS) {
            wload(wn2, ks + 2);
            dma(ks + 2, (ks + 2) % NS);
            wait_vmcnt<LQ + XG>();
        } else {
            wait_vmcnt<0>();
        }
    };
    auto compute = [&](int ks) {
        const uint32_t xs = lds_u32(smem + (ks % NS) * XB + rbase);
        const ZRegs<FMT> &dummy = w0;
        (void)dummy;
        zpmma<NJ, PF>(f, xs + cx0, xs + cx1, acc, std::make_integer_sequence<int, 2 * NJ>{});
    };

    if (half == 0) {
        deq(w0);
        for (int ks = 0; ks < KS; ks += 3) {
            // three steps per trip so the weight sets rotate statically
            compute(ks);
            lds_barrier();
            load(w2, ks);
            if (ks + 1 < KS) deq(w1);
            lds_barrier();
            if (ks + 1 >= KS) break;
            compute(ks + 1);
            lds_barrier();
            load(w0, ks + 1);
            if (ks + 2 < KS) deq(w2);
            lds_barrier();
            if (ks + 2 >= KS) break;
            compute(ks + 2);
            lds_barrier();
            load(w1, ks + 2);
            if (ks + 3 < KS) deq(w0);
            lds_barrier();
        }
    } else {
        for (int ks = 0; ks < KS; ks += 3) {
            load(w2, ks);
            deq(w0);
            lds_barrier();
            compute(ks);
            lds_barrier();
            if (ks + 1 >= KS) break;
            load(w0, ks + 1);
            deq(w1);
            lds_barrier();
            compute(ks + 1);
            lds_barrier();
            if (ks + 2 >= KS) break;
            load(w1, ks + 2);
            deq(w2);
            lds_barrier();
            compute(ks + 2);
            lds_barrier();
        }
    }
    wait_vmcnt<0>();
    if (nw >= N) return;
    zepilogue<EPI, NJ>(acc, m0, nw, N, g, fr, bias, res, out, rln);
}

template <int FMT, int NW, int BM, int NS>
void dispatch_z(const DevWeight &W, const h16 *x, int M, const float *bias, int epi, const void *res, void *out,
                hipStream_t s, const ResLN &rln)
{
    constexpr int BN = 32 * NW;
    const int nN = (W.N + BN - 1) / BN, nTiles = (M / BM) * nN;
    if (epi == EPI_BIAS_F16)
        gemmz_kernel<FMT, EPI_BIAS_F16, NW, BM, NS><<<nTiles, 64 * NW, 0, s>>>(W, x, bias, res, out, nN, nTiles, rln, g_gemm16_flags);
    else if (epi == EPI_BIAS_GELU_F16)
        gemmz_kernel<FMT, EPI_BIAS_GELU_F16, NW, BM, NS><<<nTiles, 64 * NW, 0, s>>>(W, x, bias, res, out, nN, nTiles,
                                                                                   rln, g_gemm16_flags);
    else
        gemmz_kernel<FMT, EPI_BIAS_RES, NW, BM, NS><<<nTiles, 64 * NW, 0, s>>>(W, x, bias, res, out, nN, nTiles, rln, g_gemm16_flags);
}

template <int FMT>
int launch_z_fmt(const DevWeight &W, const h16 *x, int32_t M, const float *bias, int32_t epi, const void *res,
                 void *out, hipStream_t s, const ResLN &rln, int cfg)
{
    // residual form with the panel LayerNorm: 4 waves, 128 x 128 tiles (the
    // residual form's production shape), every workgroup storing whole tiles
    if (epi == EPI_BIAS_RES && rln.cnt && (cfg == 0 || cfg == 3) && W.N % 128 == 0 && W.N > 256 &&
        W.N <= 1024 && M % 128 == 0) {
        const int nN = W.N / 128, nTiles = (M / 128) * nN;
        auto go = [&](auto kern) {
            kern<<<nTiles, 256, 0, s>>>(W, x, bias, res, out, nN, nTiles, rln, g_gemm16_flags, nullptr);
            return 1;
        };
        if (W.N <= 512) return go(gemmz_kernel<FMT, EPI_BIAS_RES, 4, 128, 4, 2>);
        if (W.N <= 768) return go(gemmz_kernel<FMT, EPI_BIAS_RES, 4, 128, 4, 3>);
        return go(gemmz_kernel<FMT, EPI_BIAS_RES, 4, 128, 4, 4>);
    }
    // BERT_GEMM16_SPLIT: 1 every form, r the residual forms only, else none (A/B)
    static const int split_env = [] {
        const char *e = std::getenv("BERT_GEMM16_SPLIT");
        return !e ? 0 : *e == '1' ? 1 : *e == 'r' ? 2 : 0;
    }();
    const bool split = cfg == 5 || (cfg == 0 && (split_env == 1 || (split_env == 2 && epi == EPI_BIAS_RES)));
    if (cfg == 5) cfg = 2;
    if (cfg == 0) {
        // measured in the forward at C3 (gpurun_out cfg A/B, r01): 4-wave 256 x 128
        // tiles two per CU (each wave 32 features x 256 tokens, like the 8-wave
        // 256 x 256 tile, but the two co-resident workgroups drift apart, so one's
        // epilogue overlaps the other's MFMAs) beat 256 x 256 for QKV (127 -> 119 us)
        // and 128 x 128 for FFN-down (158 -> 153 us), tie on FFN-up and O-proj
        // BERT_GEMM16_CFG="wide,res" overrides the two choices (A/B)
        static const int2 pick = [] {
            int2 p{2, 2};
            if (const char *e = std::getenv("BERT_GEMM16_CFG")) std::sscanf(e, "%d,%d", &p.x, &p.y);
            return p;
        }();
        // below two 256 x 128 tiles per CU (small batches), 128 x 128 tiles
        const bool fills = M % 256 == 0 && W.N % 128 == 0 && (long)(M / 256) * (W.N / 128) >= 512;
        cfg = !fills ? 3 : epi != EPI_BIAS_RES ? pick.x : pick.y;
        if (cfg == 1 && W.N % 256) cfg = 2;
    }
    if (cfg == 4 && W.N % 256 == 0 && M % 256 == 0) {
        const int nN = W.N / 256, nt = (M / 256) * nN;
        if (epi == EPI_BIAS_F16) gemmp_kernel<FMT, EPI_BIAS_F16><<<nt, 512, 0, s>>>(W, x, bias, res, out, nN, nt, rln);
        else if (epi == EPI_BIAS_GELU_F16)
            gemmp_kernel<FMT, EPI_BIAS_GELU_F16><<<nt, 512, 0, s>>>(W, x, bias, res, out, nN, nt, rln);
        else gemmp_kernel<FMT, EPI_BIAS_RES><<<nt, 512, 0, s>>>(W, x, bias, res, out, nN, nt, rln);
        return 0;
    }
    if (cfg == 4) cfg = 2;
    if (cfg == 1) dispatch_z<FMT, 8, 256, 3>(W, x, M, bias, epi, res, out, s, rln);
    else if (cfg == 2) {
        const int n1 = split && M % 256 == 0 && W.N % 128 == 0 ? z_split_cols(M, W.N) : 0;
        if (n1 > 0) dispatch_split<FMT>(W, x, M, bias, epi, res, out, s, rln, n1);
        else dispatch_z<FMT, 4, 256, 2>(W, x, M, bias, epi, res, out, s, rln);
    }
    else dispatch_z<FMT, 4, 128, 4>(W, x, M, bias, epi, res, out, s, rln);
    return 0;
}

}  // namespace

// Diagnostics: gemm16 tile config cfg (1-3) with per-wave stamps into `stamps`
// (nTiles * NW * 8 uint64); returns the tile count in units of 8 waves.
int launch_gemm16_stamped(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                          const void *res, void *out, hipStream_t s, int cfg, uint64_t *stamps)
{
    const h16 *x = (const h16 *)X;
    auto go = [&](auto nwt, auto bmt, auto nst) {
        constexpr int NW = decltype(nwt)::value, BM = decltype(bmt)::value, NS = decltype(nst)::value;
        const int nN = (W.N + 32 * NW - 1) / (32 * NW), nt = (M / BM) * nN;
        if (epi == EPI_BIAS_F16)
            gemmz_kernel<FMT_Q4_0, EPI_BIAS_F16, NW, BM, NS, 0, true><<<nt, 64 * NW, 0, s>>>(
                W, x, bias, res, out, nN, nt, ResLN(), g_gemm16_flags, stamps);
        else if (epi == EPI_BIAS_GELU_F16)
            gemmz_kernel<FMT_Q4_0, EPI_BIAS_GELU_F16, NW, BM, NS, 0, true><<<nt, 64 * NW, 0, s>>>(
                W, x, bias, res, out, nN, nt, ResLN(), g_gemm16_flags, stamps);
        else
            gemmz_kernel<FMT_Q4_0, EPI_BIAS_RES, NW, BM, NS, 0, true><<<nt, 64 * NW, 0, s>>>(
                W, x, bias, res, out, nN, nt, ResLN(), g_gemm16_flags, stamps);
        return nt * NW / 8;
    };
    if (cfg == 1) return go(std::integral_constant<int, 8>(), std::integral_constant<int, 256>(), std::integral_constant<int, 3>());
    if (cfg == 2) return go(std::integral_constant<int, 4>(), std::integral_constant<int, 256>(), std::integral_constant<int, 2>());
    return go(std::integral_constant<int, 4>(), std::integral_constant<int, 128>(), std::integral_constant<int, 4>());
}

int g_gemm16_cfg = 0;
int g_gemm16_flags = [] { const char *e = std::getenv("BERT_GEMM16_FLAGS"); return e ? std::atoi(e) : 0; }();

int launch_gemm16(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi,
                  const void *res, void *out, hipStream_t s, const ResLN &rln)
{
    const h16 *x = (const h16 *)X;
    const int cfg = g_gemm16_cfg;
    switch (W.fmt) {
    case FMT_Q4_0: return launch_z_fmt<FMT_Q4_0>(W, x, M, bias, epi, res, out, s, rln, cfg);
    case FMT_Q4_1: return launch_z_fmt<FMT_Q4_1>(W, x, M, bias, epi, res, out, s, rln, cfg);
    case FMT_Q8_0: return launch_z_fmt<FMT_Q8_0>(W, x, M, bias, epi, res, out, s, rln, cfg);
    default: return launch_z_fmt<FMT_F16>(W, x, M, bias, epi, res, out, s, rln, cfg);
    }
}

}  // namespace emb
