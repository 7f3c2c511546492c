// Linear layers on v_mfma_f32_16x16x32_f16 (gfx950), weights in the lane-order
// layout of kernels.h (reference bert.cpp:994-1016, 1040-1045, 1059-1072).
//
// Y[m][n] = epi( sum_k X[m][k] W[n][k] ).  A = 16 features x 32 k (one quant
// block per feature, so each lane's scale is a single f16), B = 32 k x 16
// tokens.  The 16x16x32 loop holds a higher clock under load than the 32x32x16
// loop at the same cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7).
//
// Workgroup = NW waves, tile BM tokens x 32*NW features; wave w owns features
// n0 + 32w .. +31 (two A fragments, a = 0/1 for +0 / +16) and all BM tokens
// (NJ = BM/16 B fragments per k-slice, each feeding two MFMAs), so every
// dequantized A fragment feeds NJ MFMA pairs and every weight byte is loaded by
// exactly one wave.  Weights never touch LDS: each lane loads its own fragment
// words (16 B q4, 32 B q8, 64 B f16 per K-step, plus 8 B of scales) into a 3-set
// register ring two K-steps ahead and expands them between MFMAs.  X goes
// through an NS-stage LDS ring by LDS-DMA (buffer_load ... lds) with the XOR
// swizzle on the source address (chunk c ^ ((row>>1)&7)), which keeps the
// B-operand row read (ds_read_b128, lanes = 16 rows x 4 chunks) conflict-free.
//   NW 4, BM 256, NS 2 / BM 128, NS 4: two workgroups per CU (64 KiB each), so
//   one's epilogue overlaps the other's MFMAs;
//   NW 2, BM 64, NS 4 (64 x 64 tiles, 32 KiB): small batches, where the larger
//   tiles would leave CUs idle.
// Epilogue: accumulator pairs of adjacent 16-token groups are exchanged with
// v_permlane16_swap so each lane owns 8 consecutive features of one token
// (16-B loads of bias / residual / LN parameters and one 16-B store); the
// LayerNorm bookkeeping of kernels.h LnFold runs there.
#include "device_common.h"
#include "diag_gemm_stamps.h"
#include "host_common.h"
#include "kernels.h"
#include "zregs.h"

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <utility>
#include <atomic>
#include <type_traits>

namespace emb {


namespace {

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

// A weight load of a K-loop tail step stands in as LQ dword LDS-DMA pieces into a
// scratch slot: the same vmcnt events, no register written (the real loads'
// data would be dead and hipcc deletes them; a dead asm load into a VGPR could
// land after the register's reuse).  Issued from asm: invisible to hipcc's
// waitcnt pass, like every counted X piece (their waits are the kernel's own).
template <int N>
__device__ __forceinline__ void ztail_dma(const void *g, uint32_t lds)
{
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#pragma unroll
    for (int i = 0; i < N; ++i)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
#pragma clang diagnostic pop
}

// One K-step's worth of one lane's weight words for the wave's FA 32-feature
// groups (FA = 1: 32 features per wave, FA = 2: 64).
template <int FMT, int FA>
struct ZSet {
    ZRegs<FMT> r[FA];
    __device__ __forceinline__ void pin_all()
    {
#pragma unroll
        for (int f = 0; f < FA; ++f) r[f].pin_all();
    }
};

// One K-step's MFMAs: B fragments (s, j) -> item i = s NJ + j, read PF items
// ahead of their 2 FA MFMAs (a ring of PF + 1 fragments); A fragments
// dequantized from the register set `cur` (s = 0 first half, s = 1 second);
// acc[2 f + a] = features +32 f + 16 a.
// The first PF B-fragment reads of a K-step (zmma_items issues them itself
// unless PRE: then the caller issued them earlier with zmma_pre).
template <int NJ, int PF, int... I>
__device__ __forceinline__ void zmma_pre(h16x8 (&bq)[PF + 1], uint32_t b0, uint32_t b1, std::integer_sequence<int, I...>)
{
    auto rd = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < PF && i < 2 * NJ) bq[i % (PF + 1)] = zds_read<(i % NJ) << 11>(i < NJ ? b0 : b1);
    };
    (rd(std::integral_constant<int, I>{}), ...);
}

// ALLDQ: all four A fragments of a 32-feature group dequantized up front (short
// K-steps, where the mid-step dequantization sat on the critical path), else
// the second k-slice's at item NJ (fewer live registers).
template <int NJ, int FA, int PF, bool PRE, bool ALLDQ, class R, class H, int... I>
__device__ __forceinline__ void zmma_items(const R &cur, uint32_t b0, uint32_t b1, f32x4 (&acc)[2 * FA][NJ],
                                           const H &hook, h16x8 (&bq)[PF + 1], std::integer_sequence<int, I...> seq)
{
    constexpr int NI = 2 * NJ;
    auto rd = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NI) bq[i % (PF + 1)] = zds_read<(i % NJ) << 11>(i < NJ ? b0 : b1);
    };
    if constexpr (!PRE) zmma_pre<NJ, PF>(bq, b0, b1, seq);
    h16x8 af[2 * FA], af2[ALLDQ ? 2 * FA : 1];
#pragma unroll
    for (int f = 0; f < FA; ++f) { af[2 * f] = cur.r[f].frag(0); af[2 * f + 1] = cur.r[f].frag(2); }
    if constexpr (ALLDQ) {
#pragma unroll
        for (int f = 0; f < FA; ++f) { af2[2 * f] = cur.r[f].frag(1); af2[2 * f + 1] = cur.r[f].frag(3); }
    }
    auto item = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        hook(ic);                                     // (XI: an X piece of the next stage)
        rd(std::integral_constant<int, i + PF>{});
        constexpr int last = (i + PF < NI ? i + PF : NI - 1);
        zwait_lgkm<last - i>(bq[i % (PF + 1)]);
        if constexpr (i == NJ) {
            if constexpr (ALLDQ) {
#pragma unroll
                for (int u = 0; u < 2 * FA; ++u) af[u] = af2[u];
            } else {
#pragma unroll
                for (int f = 0; f < FA; ++f) { af[2 * f] = cur.r[f].frag(1); af[2 * f + 1] = cur.r[f].frag(3); }
            }
        }
        const h16x8 bf = bq[i % (PF + 1)];
#pragma unroll
        for (int u = 0; u < 2 * FA; ++u)
            acc[u][i % NJ] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[u], bf, acc[u][i % NJ], 0, 0, 0);
    };
    (item(std::integral_constant<int, I>{}), ...);
}

// Epilogue operands staged in LDS by the prologue (their load latency then
// hides under the K loop): up to four per-feature f32 arrays of the tile's BN
// features (bias, c1 | bias, res_g, res_b, g_next) and the BM rows' (mean,
// 1/sigma), each part a whole number of 1-KiB LDS-DMA pieces.
template <int EPI, bool LNF>
constexpr int zepi_arrays()
{
    return EPI == EPI_BIAS_RES ? (LNF ? 4 : 1) : (LNF ? 2 : 1);
}
constexpr int zkib(int bytes) { return (bytes + 1023) / 1024; }
template <int EPI, bool LNF, int BN, int BM, int GF = 0>
constexpr int zepi_lds()
{
    // GF > 0 (statistics fold): + the partials of up to GF 32-feature groups of the
    // tile's BM rows, [group][row] float2
    return 1024 * (zkib(zepi_arrays<EPI, LNF>() * BN * 4) + (LNF ? zkib(BM * 8) : 0) + zkib(GF * BM * 8));
}

// vmcnt accounting of the K loop, derived instead of hand-counted.  Each wave
// issues per K-step one weight group W(k) of LQ loads (into a register set of
// the WR-deep ring, WR - 1 steps ahead) and one X group X(k) of XG LDS-DMA loads
// (into the NS-stage LDS ring, NS - 1 steps ahead); vmcnt retires in issue
// order, so a wait that must see group G complete may leave at most the loads
// issued after G's last load in flight.  z_waits replays the issue order the
// kernel uses (its prologue, then per step the two groups in kernel order; the
// tail clamps k but still issues every load, so counts are the same on every
// path) and returns, for each wait, the minimum over steps of that count:
//   prologue: W(0) and X(0) complete (then the barrier publishes X(0));
//   front of step ks: W(ks) complete (the registers its MFMAs dequantize);
//   back of step ks: X(ks + 1) and W(ks + 1) complete (then the barrier
//   publishes X(ks + 1) to every wave before step ks + 1 reads it).
// The minimum matters: with a deeper ring the steps right after the prologue
// have fewer loads in flight behind W(ks) than the steady state (the prologue
// issues its groups in another order), so a constant read off the steady
// state leaves those W(ks) unretired ("the 4-set ring race").
struct ZWaits { int prologue, front, back; };

template <int NS, int WR, int LQ, int XG, int XI = 0>
constexpr ZWaits z_waits()
{
    constexpr int S = 16;                        // steps replayed (periodic long before)
    int kind[3 * S + 16] = {}, kk[3 * S + 16] = {}, ops[3 * S + 16] = {};
    int n = 0;
    auto add = [&](int kd, int k) { kind[n] = kd; kk[n] = k; ops[n] = kd == 0 ? LQ : XG; ++n; };
    auto after = [&](int kd, int k) {            // loads issued after group (kd, k)'s last load
        int last = -1;
        for (int i = 0; i < n; ++i)
            if (kind[i] == kd && kk[i] == k) last = i;
        int c = 0;
        for (int i = last + 1; i < n; ++i) c += ops[i];
        return last < 0 ? -1 : c;
    };
    auto mn = [](int a, int b) { return a < b ? a : b; };
    // prologue, in the kernel's order (gemmz_body)
    if (NS == 2) { add(0, 0); add(1, 0); add(0, 1); }
    else if (NS == 3) { add(0, 0); add(1, 0); add(0, 1); add(1, 1); }
    else { add(0, 0); add(1, 0); add(1, 1); add(0, 1); add(1, 2); }
    for (int j = 2; j < WR - 1; ++j) add(0, j);
    ZWaits w{mn(after(0, 0), after(1, 0)), 1 << 20, 1 << 20};
    for (int ks = 0; ks < S; ++ks) {
        if (XI) {
            // interleaved X: W(ks + WR - 1), the front wait, then X(ks + NS - 1)'s
            // pieces among the step's MFMAs, the back wait
            add(0, ks + WR - 1);
            w.front = mn(w.front, after(0, ks));
            add(1, ks + NS - 1);
        } else {
            if (NS == 2) { add(1, ks + 1); add(0, ks + WR - 1); }
            else { add(0, ks + WR - 1); add(1, ks + NS - 1); }
            w.front = mn(w.front, after(0, ks));
        }
        w.back = mn(w.back, mn(after(1, ks + 1), after(0, ks + 1)));
    }
    return w;
}

// The production ring (WR = 3) against the counts the kernel carried before the
// derivation (2P + XG in front, P + XG behind at NS 4): equal; at NS 2
// the old front count 2 LQ + XG also retired X(ks), already retired by the
// previous step's back wait, so the derived 2 (LQ + XG) waits for the same loads.
static_assert(z_waits<4, 3, 2, 4>().front == 2 * 6 + 4 && z_waits<4, 3, 2, 4>().back == 6 + 4 &&
                  z_waits<4, 3, 2, 4>().prologue == 6 + 4,
              "derived waits, 128x128 / 64x64 q4_0");
static_assert(z_waits<4, 3, 4, 4>().front == 2 * 8 + 4 && z_waits<4, 3, 4, 4>().back == 8 + 4,
              "derived waits, 64x64 f16");
static_assert(z_waits<2, 3, 2, 8>().front == 2 * (2 + 8) && z_waits<2, 3, 2, 8>().back == 2 &&
                  z_waits<2, 3, 2, 8>().prologue == 2,
              "derived waits, 256x128 q4_0");
// interleaved X pieces (NS 2): the front wait sees W(ks + 1), X(ks), W(ks + 2)
// behind W(ks); the back wait retires everything (X(ks + 1) was issued last)
static_assert(z_waits<2, 3, 2, 8, 1>().front == 8 + 2 * 2 && z_waits<2, 3, 2, 8, 1>().back == 0 &&
                  z_waits<2, 3, 2, 8, 1>().prologue == 2,
              "derived waits, 256x128 q4_0, interleaved X");
static_assert(z_waits<4, 3, 2, 4, 2>().front == 2 * 2 + 2 * 4 && z_waits<4, 3, 2, 4, 2>().back == 2 + 2 * 4,
              "derived waits, 128x128 / 64x64 q4_0, interleaved X");
// the 4-set ring: the steady state has 3P + XG behind W(ks) (q4_0: 22) but the
// two steps after the prologue only 3P (18)
static_assert(z_waits<4, 4, 2, 4>().front == 3 * 6 && z_waits<4, 4, 2, 4>().back == 2 * 6 &&
                  z_waits<4, 4, 2, 4>().prologue == 2 * 6,
              "derived waits, 4-set ring");

// The tile body: workgroup b of a grid of nTiles tiles (nN column tiles),
// staging X in `smem` (NS * BM * 128 B of LDS) and the epilogue operands
// behind it (zepi_lds).
template <int FMT, int EPI, bool LNF, int NW, int BM, int NS, int FA, int WR, int NT, int XI, int GF>
__device__ __forceinline__ void gemmz_body(char *__restrict__ smem, const int b, DevWeight W,
                                           const h16 *__restrict__ X, const float *__restrict__ bias,
                                           const void *__restrict__ res, void *__restrict__ out, int nN, int nTiles,
                                           const LnFold &ln)
{
    // NT waves along the tokens (each BM / NT of them), NW / NT along the features
    static_assert(NW % NT == 0 && (BM / NT) % 32 == 0, "wave grid");
    constexpr int NF = NW / NT;
    constexpr int BN = 32 * NF * FA;
    constexpr int NJ = BM / NT / 16;            // 16-token B fragments per k-slice (this wave's tokens)
    constexpr int PF = FA == 1 ? (NJ <= 4 ? 2 * NJ - 1 : 4) : 3;   // B-fragment read-ahead (items of 2 FA MFMAs)
    // X modes (XI): 0 one burst of pieces in front of the K-step's MFMAs, 1 / 2 the
    // pieces among them (every second / every B-fragment item); 3 / 4 as 0 / 2 into
    // a wave-private ring: each wave stages its own BM / NT token rows (the NF waves
    // that share them each load a copy), so no barrier couples the waves in the K
    // loop -- a wave's own covering vmcnt orders its ds_reads behind its pieces
    // (MI355X_MICROARCH.md, co-residence item 7)
    constexpr bool PRIV = XI >= 3;
    constexpr int XMODE = XI == 3 ? 0 : XI == 4 ? 2 : XI;
    constexpr int XB = BM * ZK * 2;             // bytes per shared X stage
    constexpr int XBW = (BM / NT) * ZK * 2;     // bytes per wave-private stage
    constexpr int RING = PRIV ? NW * NS * XBW : NS * XB;
    constexpr int XG = PRIV ? XBW / 1024 : XB / (64 * NW * 16);   // LDS-DMA instructions per wave per stage
    constexpr int LQ = ZRegs<FMT>::LOADS * FA;
    constexpr int QB = ZRegs<FMT>::QB;
    constexpr int P = LQ + XG;                  // vector-memory ops issued per K-step per wave
    static_assert(NS >= 2 && NS <= 4 && XG >= 2 && XG % 2 == 0, "X ring");
    static_assert(WR == 3 || WR == 4, "weight register ring: 3 or 4 sets");
    constexpr ZWaits ZW = z_waits<NS, WR, LQ, XG, XMODE>();
    static_assert(ZW.prologue >= 0 && ZW.front >= 0 && ZW.back >= 0 && ZW.front < 64 && P <= 63,
                  "vmcnt range (6 bits)");
    (void)P;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    ZSTAMP(0, __builtin_amdgcn_s_memtime());
    // XCD-aware bijective remap: consecutive tiles (same token panel) land on one
    // XCD's L2 (workgroups are dealt to the 8 XCDs round-robin)
    const int xcd = b & 7, qq = nTiles >> 3, rr = nTiles & 7;
    // (round 6 measured panel-group and snake orders of the tiles inside an XCD's
    // share: within noise, and without the remap -13 %; profiles/r06_gemm_raster_ab.log)
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int m0 = (t / nN) * BM, n0 = (t % nN) * BN;
    const int K = W.K, N = W.N, KS = K / ZK;
    const int KX = W.kx ? W.kx : K, KSX = KX / ZK;   // X columns (f32 hi/lo weights: K = 2 KX)
    const int fr = lane & 15, g = lane >> 4;
    const int mt = (BM / NT) * (wave / NF);     // this wave's first token row in the tile
    const int nw = n0 + 32 * FA * (wave % NF);  // this wave's first feature
    const int grp = min(nw, N - 32) >> 5;       // its first 32-feature weight group (clamped past N)
    // the wave's further groups (clamped past N; wave-uniform byte / element offsets)
    int gq[FA], gd[FA];
#pragma unroll
    for (int f = 0; f < FA; ++f) {
        const int gf = min(grp + f, N / 32 - 1) - grp;
        gq[f] = __builtin_amdgcn_readfirstlane(gf * 64 * QB);
        gd[f] = __builtin_amdgcn_readfirstlane(gf * 64);
    }

    // LDS-DMA of X as buffer loads: the tile's BM rows are the buffer (reads
    // past it give 0); instruction i of this wave fills rows 8*XG*wave + 8i +
    // lane/8; the swizzle ((row>>1)&7) only differs between even and odd i, so
    // one offset VGPR per parity and the row step in soffset
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(X + (size_t)m0 * KX), (short)0, BM * KX * 2, 0x00020000);
    uint32_t xvo[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (PRIV ? mt : 8 * XG * wave) + 8 * i + (lane >> 3);
        xvo[i] = (uint32_t)(r * KX + (((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2u;
    }
    auto issue_x_piece = [&](int ks, int stage, int i) {
        char *dst = PRIV ? smem + (wave * NS + stage) * XBW : smem + stage * XB + ((8 * XG * wave) << 7);
        const int kc = ks < KSX ? ks : ks - KSX;   // the X column block of K-step ks
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t *)(dst + (i << 10)), 16, xvo[i & 1],
                                                 ((i >> 1) * 16 * KX + kc * ZK) * 2, 0, 0);
    };
    auto issue_x = [&](int ks, int stage) {
#pragma unroll
        for (int i = 0; i < XG; ++i) issue_x_piece(ks, stage, i);
    };
    const uint8_t *wq = (const uint8_t *)W.qs + ((size_t)grp * 64 + lane) * QB;
    const uint16_t *wd = W.d + ((size_t)grp * 16 + fr) * 4;
    const uint16_t *wmn = FMT == FMT_Q4_1 ? W.m + ((size_t)grp * 16 + fr) * 4 : nullptr;
    const size_t qstep = (size_t)N * 2 * QB, sstep = (size_t)N * 2;
    auto wload = [&](ZSet<FMT, FA> &w, int ks) {
#pragma unroll
        for (int f = 0; f < FA; ++f)
            w.r[f].load(wq + ks * qstep + gq[f], wd + ks * sstep + gd[f],
                        FMT == FMT_Q4_1 ? wmn + ks * sstep + gd[f] : nullptr);
    };

    // epilogue operands -> LDS (wave 0; retired by the prologue's vmcnt wait,
    // published by its barrier)
    constexpr bool RES = EPI == EPI_BIAS_RES;
    constexpr int NA = zepi_arrays<EPI, LNF>();
    constexpr int FP = zkib(NA * BN * 4);       // pieces of the per-feature arrays
    constexpr int SP = LNF ? zkib(BM * 8) : 0;  // pieces of the row statistics
    float *const efeat = (float *)(smem + RING);
    float2 *const estat = (float2 *)(smem + RING + FP * 1024);
    const float2 *stp = RES ? ln.res_stats : ln.in_stats;
    // Statistics fold (GF > 0; small batches, engine.cpp): instead of the rows'
    // (mean, 1/sigma), the residual GEMM's 32-feature partials of the tile's rows
    // come in with the prologue (one load latency, beside X(0) and W(0)) and are
    // combined after the K loop with ln_stats_kernel's arithmetic -- no statistics
    // launch in front of this GEMM, same bits.
    constexpr bool FOLD = GF > 0;
    static_assert(!FOLD || (LNF && !RES && BM % 64 == 0), "fold: input-LN forms");
    float2 *const epart = (float2 *)(smem + RING + (FP + SP) * 1024);
    if constexpr (FOLD) {
        if (wave == 1 % NW) {
            // piece j, lane l: elements e = 128 j + 2 l, + 1 of [group][row] (BM rows per
            // group); one wave issues them all (spread over every wave, each wave's
            // K loop started later: B = 1 +2 us, profiles/r04_stats_fold_ab.log)
            const int G = ln.in_G, npc = (G * BM + 127) / 128;
#pragma unroll
            for (int j = 0; j < GF * BM / 128; ++j) {
                if (j < npc) {
                    const int e = 128 * j + 2 * lane, gg = min(e / BM, G - 1), r = e % BM;
                    glds<16>(ln.in_part + (size_t)gg * ln.in_part_stride + m0 + r, (char *)epart + j * 1024);
                }
            }
        }
    }
    if (wave == 0) {
        const float *arr[4] = {bias, RES ? ln.res_g : ln.c1, ln.res_b, ln.g_next};
#pragma unroll
        for (int i = 0; i < FP; ++i) {
            const int f = 256 * i + 4 * lane, ai = f / BN < NA ? f / BN : 0;
            glds<16>(arr[ai] + min(n0 + f % BN, N - 4), (char *)efeat + i * 1024);
        }
        if constexpr (!FOLD) {
#pragma unroll
            for (int i = 0; i < SP; ++i) {
                const int r = 128 * i + 2 * lane;
                glds<16>(stp + m0 + (r < BM ? r : 0), (char *)estat + i * 1024);
            }
        }
    }

    f32x4 acc[2 * FA][NJ];
#pragma unroll
    for (int a = 0; a < 2 * FA; ++a)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    ZSet<FMT, FA> w0, w1, w2, w3;
    const int k1 = min(1, KS - 1);
    wload(w0, 0);
    issue_x(0, 0);
    if constexpr (NS == 2) {
        wload(w1, k1);
    } else if constexpr (NS == 3) {
        asm volatile("" ::: "memory");
        wload(w1, k1);
        asm volatile("" ::: "memory");
        issue_x(k1, 1);
    } else {
        issue_x(k1, 1);
        asm volatile("" ::: "memory");
        wload(w1, k1);
        asm volatile("" ::: "memory");
        issue_x(min(2, KS - 1), 2);
    }
    if constexpr (WR == 4) {
        asm volatile("" ::: "memory");
        wload(w2, min(2, KS - 1));
    }
    wait_vmcnt<ZW.prologue>();
    lds_barrier();
    ZSTAMP(1, __builtin_amdgcn_s_memtime());

    const int sw = (fr >> 1) & 7;               // mt is a multiple of 32: the row swizzle is fr's
    const int rbase = PRIV ? fr << 7 : (mt + fr) << 7;
    int st = 0;
    // K-loop split (stamps builds only, diag_gemm_stamps.h): cycles in the load wait
    // in front of each K-step's MFMAs, and in the wait + barrier behind them
    ZClock zc;
    // One K-step with CUR's weights: issue X(ks + NS - 1) into the stage freed by
    // the previous step and W(ks + WR - 1) into the ring's free register set,
    // then the derived vmcnt (z_waits: what is provably still in flight; a
    // run-time no-op that stops hipcc's waitcnt pass from draining the ring with
    // vmcnt(0)); the K loop runs whole, unguarded WR-tuples so the count holds
    // on every path.
    // A tail step (the remainder after the whole WR-tuples) loads no weights it
    // will use: ztail_dma stands in for them, so the counts hold.
    const uint32_t scratch = lds_u32(smem + RING + zepi_lds<EPI, LNF, BN, BM, GF>());
    auto wload_or_tail = [&](ZSet<FMT, FA> &nxt, int kw, auto tail) {
        if constexpr (decltype(tail)::value) ztail_dma<LQ>(wq + kw * qstep, scratch);
        else wload(nxt, kw);
    };
    auto kstep = [&](ZSet<FMT, FA> &cur, ZSet<FMT, FA> &nxt, int ks, auto tail) {
        const int kx = min(ks + NS - 1, KS - 1), kw = min(ks + WR - 1, KS - 1);
        const int sx = st == 0 ? NS - 1 : st - 1;
        // XI: X(ks + 1)'s XG pieces among the first XG * XS items (one every XS), so
        // the CU's texture path takes a wave's pieces between its MFMAs instead of
        // in one burst in front of them
        constexpr int XS = XMODE == 1 && 2 * NJ / XG >= 2 ? 2 : 1;   // mode 2: one per item (measured best), 1: every second
        auto hook = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (XMODE && i % XS == 0 && i / XS < XG) issue_x_piece(kx, sx, i / XS);
        };
        if constexpr (PRIV) {
            // private rings: X(ks) was retired by this wave's previous back wait (or
            // the prologue), so the step's B reads go out before its loads and front
            // wait (their latency under the wait), and all four A fragments are
            // dequantized up front; nothing between the reads and the items'
            // lgkmcnt waits may use the LDS / scalar-memory counter
            const uint32_t xs = lds_u32(smem + (wave * NS + st) * XBW + rbase);
            const uint32_t b0 = xs + ((g ^ sw) << 4), b1 = xs + (((4 + g) ^ sw) << 4);
            h16x8 bq[PF + 1];
            zmma_pre<NJ, PF>(bq, b0, b1, std::make_integer_sequence<int, 2 * NJ>{});
            wload_or_tail(nxt, kw, tail);
            if constexpr (!XMODE) {
                asm volatile("" ::: "memory");
                issue_x(kx, sx);
            }
            wait_vmcnt<ZW.front>();
            cur.pin_all();
            zmma_items<NJ, FA, PF, true, true>(cur, b0, b1, acc, hook, bq, std::make_integer_sequence<int, 2 * NJ>{});
            wait_vmcnt<ZW.back>();
        } else {
            if constexpr (XMODE) {
                wload_or_tail(nxt, kw, tail);
                wait_vmcnt<ZW.front>();
            } else if constexpr (NS == 2) {
                // (NS 2: the front slot holds the cycles of the X pieces' issue instead of the wait)
                zc.mark();
                issue_x(kx, sx);
                asm volatile("" ::: "memory");
                zc.add_front();
                wload_or_tail(nxt, kw, tail);
                wait_vmcnt<ZW.front>();
            } else {
                wload_or_tail(nxt, kw, tail);
                asm volatile("" ::: "memory");
                issue_x(kx, sx);
                zc.mark();
                wait_vmcnt<ZW.front>();
                zc.add_front();
            }
            cur.pin_all();
            const uint32_t xs = lds_u32(smem + st * XB + rbase);
            h16x8 bq[PF + 1];
            zmma_items<NJ, FA, PF, false, false>(cur, xs + ((g ^ sw) << 4), xs + (((4 + g) ^ sw) << 4), acc, hook, bq,
                                                 std::make_integer_sequence<int, 2 * NJ>{});
            zc.mark();
            wait_vmcnt<ZW.back>();
            lds_barrier();
            zc.add_back();
        }
        st = st == NS - 1 ? 0 : st + 1;
    };
    int ks = 0;
    constexpr std::false_type body{};
    constexpr std::true_type tail{};
    if constexpr (WR == 3) {
        for (; ks + 3 <= KS; ks += 3) {
            kstep(w0, w2, ks, body);
            kstep(w1, w0, ks + 1, body);
            kstep(w2, w1, ks + 2, body);
        }
        if (ks < KS) {
            kstep(w0, w2, ks, tail);
            if (ks + 1 < KS) kstep(w1, w0, ks + 1, tail);
        }
    } else {
        for (; ks + 4 <= KS; ks += 4) {
            kstep(w0, w3, ks, body);
            kstep(w1, w0, ks + 1, body);
            kstep(w2, w1, ks + 2, body);
            kstep(w3, w2, ks + 3, body);
        }
        if (ks < KS) {
            kstep(w0, w3, ks, tail);
            if (ks + 1 < KS) kstep(w1, w0, ks + 1, tail);
            if (ks + 2 < KS) kstep(w2, w1, ks + 2, tail);
        }
    }
    // (Round 2's "4-set ring race": the tail steps' real weight loads feed no later
    // step, so hipcc deleted them as dead, and a tail step's back wait -- counted
    // with them behind X(ks + 1) -- left the last LQ pieces of X(ks + 1) in flight
    // across the barrier: the NS 2 ring at KS % 3 == 2, the 4-set ring at
    // KS % 4 == 2.  The tail now issues ztail_dma pieces in their place.)
    // Both counters drained in front of the epilogue: the K loop's B-fragment reads
    // are asm (zds_read) with hand-counted lgkmcnt waits the compiler cannot see, so
    // without an explicit lgkmcnt(0) here an asm read still in flight could land in
    // a register hipcc hands to the epilogue (round 3's pipelined private-ring
    // variant faulted exactly so; scripts/check_drain.py checks the
    // shipped code objects for this wait).
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (FOLD) {
        // row tid's statistics from its G partials (ln_row_stats: the statistics
        // kernel's arithmetic and order), into estat; the column-0 tiles also store
        // them for the residual GEMM that reads this stream next (LnFold::st_out)
        if (tid < BM) {
            const int G = ln.in_G;
            // (LDS reads from asm on the 32-bit LDS address: hipcc's generic-pointer
            // form of these loads next to ln_row_stats' division sequence fails
            // instruction selection on gfx950 -- "operand has incorrect register class";
            // read as 64-bit integers: a float2 tied through an asm operand came out
            // with its halves mixed)
            const uint32_t pa = lds_u32(epart) + 8u * tid;
            unsigned long long pr[GF];
#pragma unroll
            for (int gg = 0; gg < GF; ++gg) {
                pr[gg] = 0ull;
                if (gg < G) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(pr[gg]) : "v"(pa), "i"(gg * BM * 8));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float2 pp[GF];
#pragma unroll
            for (int gg = 0; gg < GF; ++gg) {   // (each value tied to after the wait)
                asm volatile("" : "+v"(pr[gg]));
                pp[gg] = __builtin_bit_cast(float2, pr[gg]);
            }
            const float2 rs = ln_row_stats<GF>(pp, G, 32 * G);
            estat[tid] = rs;
            if (n0 == 0 && ln.st_out) ln.st_out[m0 + tid] = rs;
        }
        lds_barrier();
    }
    ZSTAMP(2, __builtin_amdgcn_s_memtime());
    ZSTAMP_KSPLIT(zc);

    // ---- epilogue ----
    // acc[2 fa + a][j] lane (g, fr): token m0 + 16j + fr, features nw + 32fa + 16a + 4g + 0..3.
    // After the permlane16 exchange of (acc[a][j], acc[a][j+1]) the lane holds
    // token m0 + 16(j + (g&1)) + fr, features nw + 16a + 8(g>>1) + 0..7; lane
    // l ^ 32 holds the other 16 of the wave's 32 features of the same token.
#pragma unroll
    for (int fa = 0; fa < FA; ++fa) {
        const int nwf = nw + 32 * fa;               // this pass: features nwf .. nwf + 31
        if (nwf >= N) return;                       // wave-uniform (N % 32 == 0)
        const int cb = nwf + 8 * (g >> 1);          // feature of v[0][0]; v[1][*] at cb + 16
        auto col8 = [&](int ai, f32x4 (&o)[2][2]) {   // per-feature array ai, from LDS
            const float *p = efeat + ai * BN + (cb - n0);
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                o[a][0] = *(const f32x4 *)(p + 16 * a);
                o[a][1] = *(const f32x4 *)(p + 16 * a + 4);
            }
        };
        f32x4 bb[2][2];
        col8(0, bb);
        constexpr bool lni = !RES && LNF;           // input LayerNorm folded
        constexpr bool rln = RES && LNF;            // residual given as z = y * gamma of an LN ...
        constexpr bool nxt = RES && LNF;            // ... and z' = y' * g_next + partial statistics out
        f32x4 c1[2][2], rg[2][2], gn[2][2];
        if (lni) col8(1, c1);
        if (rln) {
            // the residual LN's beta joins the bias: v = acc + r z + (t gamma + (bias + beta))
            f32x4 rb[2][2];
            col8(1, rg);
            col8(2, rb);
#pragma unroll
            for (int a = 0; a < 2; ++a) { bb[a][0] += rb[a][0]; bb[a][1] += rb[a][1]; }
        }
        if (nxt) col8(3, gn);
        constexpr bool use_st = LNF;
        // token pairs j = 2 jp, 2 jp + 1 (after the exchange each lane holds one
        // token of the pair); the residual rows of PW pairs stay in flight ahead
        // of their use (a sliding window: one load latency per tile, not per pair)
        constexpr int NP = NJ / 2, PW = NP < 4 ? NP : 4;
        uint4 rr[PW][2];
        auto ldres = [&](int jp) {
            const int tok = m0 + mt + 16 * (2 * jp + (g & 1)) + fr;
#pragma unroll
            for (int a = 0; a < 2; ++a)
                rr[jp % PW][a] = *(const uint4 *)((const h16 *)res + (size_t)tok * N + cb + 16 * a);
        };
        if constexpr (RES) {
#pragma unroll
            for (int jp = 0; jp < PW; ++jp) ldres(jp);
        }
#pragma unroll
        for (int jp = 0; jp < NP; ++jp) {
            {
                const int j = 2 * jp;
                const int tok = m0 + mt + 16 * (j + (g & 1)) + fr;
                const float2 stt = use_st ? estat[tok - m0] : float2{0.f, 1.f};
                uint4 rcur[2] = {};
                if constexpr (RES) {
                    rcur[0] = rr[jp % PW][0];
                    rcur[1] = rr[jp % PW][1];
                    if (jp + PW < NP) ldres(jp + PW);
                }
                // (mean, 1/sigma) -> v = r x + t with t = -mean / sigma
                const float sr = stt.y, st0 = -stt.x * stt.y;
                float v[2][8];
#pragma unroll
                for (int a = 0; a < 2; ++a) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[a][e] = acc[2 * fa + a][j][e];
                        v[a][4 + e] = acc[2 * fa + a][j + 1][e];
                    }
                    zswap4(v[a]);
                }
                if constexpr (!RES) {
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float bv = bb[a][e >> 2][e & 3];
                            // input LN fold: LN(y) W^T + b = r (z W^T - mean c1) + c2
                            v[a][e] = lni ? fmaf(sr, v[a][e], fmaf(st0, c1[a][e >> 2][e & 3], bv)) : v[a][e] + bv;
                        }
                } else {
#pragma unroll
                    for (int a = 0; a < 2; ++a) {
                        const h16x8 rh = __builtin_bit_cast(h16x8, rcur[a]);
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float z = (float)rh[e], bv = bb[a][e >> 2][e & 3];
                            // LN(y) = r z - r mean gamma + beta with z = y gamma (the stored stream)
                            v[a][e] += rln ? fmaf(sr, z, fmaf(st0, rg[a][e >> 2][e & 3], bv)) : z + bv;
                        }
                    }
                    if (nxt) {
                        // this token's 32 features of the new stream y': sum and squared
                        // deviations from their own mean (combined per row by ln_stats)
                        float s = 0.f;
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int e = 0; e < 8; ++e) s += v[a][e];
                        s = halves_sum(s);
                        const float mg = s * (1.0f / 32.0f);
                        float q = 0.f;
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int e = 0; e < 8; ++e) { const float u = v[a][e] - mg; q = fmaf(u, u, q); }
                        q = halves_sum(q);
                        if (g < 2) ln.part[(size_t)(nwf >> 5) * ln.part_stride + tok] = float2{s, q};
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int e = 0; e < 8; ++e) v[a][e] *= gn[a][e >> 2][e & 3];
                    }
                }
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    uint4 pk;
                    uint32_t *pw = (uint32_t *)&pk;
                    if constexpr (EPI == EPI_BIAS_GELU_F16) {
                        uint32_t o4[4];
                        gelu8_era(v[a], o4);
#pragma unroll
                        for (int e = 0; e < 4; ++e) pw[e] = o4[e];
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            pw[e] = __builtin_bit_cast(uint32_t, h16x2{(h16)v[a][2 * e], (h16)v[a][2 * e + 1]});
                    }
                    h16 *const dst = (h16 *)out + (size_t)tok * N + cb + 16 * a;
                    // plain stores: the next kernel reads the output from L2
                    // (nt / write-through policies measured -18..-22 % on the C3
                    // forward, profiles/r05i_gemm_store_policy_ab.log)
                    *(uint4 *)dst = pk;
                }
            }
        }
    }
}

template <int FMT, int EPI, bool LNF, int NW, int BM, int NS, int FA, int WR, int NT, int XI, int OCC, int GF>
__global__ __launch_bounds__(64 * NW, OCC * NW / 4) void gemmz_kernel(DevWeight W, const h16 *__restrict__ X,
                                                               const float *__restrict__ bias,
                                                               const void *__restrict__ res, void *__restrict__ out,
                                                               int nN, int nTiles, LnFold ln)
{
    __shared__ __attribute__((aligned(16))) char smem[(XI >= 3 ? NW / NT : 1) * NS * BM * ZK * 2 + zepi_lds<EPI, LNF, 32 * (NW / NT) * FA, BM, GF>() +
                                                      256];   // + the tail steps' scratch slot (ztail_dma)
    // a grid smaller than nTiles walks the tiles b, b + grid, ... (persistent;
    // the host only launches it so when every wave of every tile has features,
    // so no wave leaves the body early and the barrier between tiles is reached
    // by all)
    for (int b = blockIdx.x; b < nTiles; b += gridDim.x) {
        gemmz_body<FMT, EPI, LNF, NW, BM, NS, FA, WR, NT, XI, GF>(smem, b, W, X, bias, res, out, nN, nTiles, ln);
        ZSTAMP(3, __builtin_amdgcn_s_memtime());
        if (b + (int)gridDim.x < nTiles) lds_barrier();   // LDS (X ring, epilogue operands) reused
    }
}

// OCC: workgroups per CU the launch bounds ask registers for (2: two co-resident
// tiles; 3: three, at most 168 VGPRs per wave)
template <int FMT, int NW, int BM, int NS, int FA = 1, int WR = 3, int NT = 1, int XI = 0, int OCC = 2, int GF = 0>
void dispatch_z(const DevWeight &W, const h16 *x, int M, const float *bias, int epi, const void *res, void *out,
                hipStream_t s, const LnFold &ln, bool lnf)
{
    constexpr int BN = 32 * (NW / NT) * FA;
    const int nN = (W.N + BN - 1) / BN, nTiles = (M / BM) * nN;
    // Persistent when a launch is at most two rounds of two workgroups per CU
    // (the N = d GEMMs at C3: 768 tiles = 1.5 rounds): 2 workgroups per CU walk
    // the tiles, so a slot's second tile starts without a new dispatch (O-proj
    // 53.7 -> 51.6 us, FFN-down 140.4 -> 136.6 us; the 4.5- and 6-round GEMMs
    // measured 1-2 us slower so, profiles/r02_gemm_persist_ab.log).  Whole
    // column tiles only.  BERT_GEMM_PERSIST = k forces k per CU, 0 = off.
    static const int persist_env = [] { const char *e = std::getenv("BERT_GEMM_PERSIST"); return e ? std::atoi(e) : -1; }();

    const int cus = device_cu_count();
    const int persist = persist_env >= 0 ? persist_env : (nTiles <= 2 * OCC * cus ? OCC : 0);
    int grid = nTiles;
    if (persist > 0 && W.N % BN == 0) grid = std::min(nTiles, persist * cus);
    auto go = [&](auto kern) { kern<<<grid, 64 * NW, 0, s>>>(W, x, bias, res, out, nN, nTiles, ln); };
    if constexpr (GF > 0) {
        // statistics fold: the input-LN forms only (launch_fmt checked epi / lnf)
        if (epi == EPI_BIAS_F16) go(gemmz_kernel<FMT, EPI_BIAS_F16, true, NW, BM, NS, FA, WR, NT, XI, OCC, GF>);
        else go(gemmz_kernel<FMT, EPI_BIAS_GELU_F16, true, NW, BM, NS, FA, WR, NT, XI, OCC, GF>);
    } else if (epi == EPI_BIAS_F16) {
        if (lnf) go(gemmz_kernel<FMT, EPI_BIAS_F16, true, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
        else go(gemmz_kernel<FMT, EPI_BIAS_F16, false, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
    } else if (epi == EPI_BIAS_GELU_F16) {
        if (lnf) go(gemmz_kernel<FMT, EPI_BIAS_GELU_F16, true, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
        else go(gemmz_kernel<FMT, EPI_BIAS_GELU_F16, false, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
    } else {
        if (lnf) go(gemmz_kernel<FMT, EPI_BIAS_RES, true, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
        else go(gemmz_kernel<FMT, EPI_BIAS_RES, false, NW, BM, NS, FA, WR, NT, XI, OCC, 0>);
    }
}

// The shipped tile configs (round 4 pruned the A/B zoo to these; every config
// computes each output with the same MFMA sequence, so all give the same bits):
//   2   4 waves 256 x 128, X pieces among the MFMAs   large batches (production)
//   11  4 waves 256 x 128, X pieces in one burst       the large regime's A/B form
//   3   4 waves 128 x 128                              one tile per CU
//   4   2 waves 64 x 64                                small batches, >= half the CUs
//   16  4 waves 64 x 64, 2 along the tokens, wave-private X rings
//                                                      small batches, < half the CUs
// A config whose row tile does not divide M falls back to the next smaller tile.
// The tile config a launch of N features over M rows runs (cfg 0: the heuristic),
// after the fallbacks for tiles that do not divide M.
int pick_cfg(int N, int M, int cfg, int fmt)
{
    if (cfg == 0) {
        // the largest tile that still gives every CU work: 256 x 128 tiles two per CU
        // (measured fastest at C3 once there are two per CU, profiles/r01_gemm16_sweep.log),
        // else 128 x 128 once they cover half the CUs (one such tile per CU beats the
        // 64 x 64 tiles that would spread over all of them: MiniLM QKV at M 2,048 7.3 vs
        // 8.6 us, bge-base FFN-up at M 1,024 11.2 vs 14.7 us, profiles/r06_cfg34_crossover.log),
        // else 64 x 64 (small batches)
        const long n128 = (N + 127) / 128, cus = device_cu_count();
        // small batches: 64-row tiles.  Quantized weights on 4 waves (2 along the
        // tokens: every SIMD of a CU works, each wave's K-step and dequantization
        // half as long; B = 1, L = 32: 632 -> 571 us) with wave-private X rings (no
        // barrier in the K loop: 582 -> 567 us, profiles/r03_gemm_private_ab.log) --
        // round 6: at every M up to the 128 x 128 threshold, not only below half the
        // CUs (bge-base FFN-down at M 1,024 16.8 vs 20.9 us); f16 weights (nothing
        // to dequantize, four weight loads per K-step) on 2 waves, 0.5-2 us faster
        // at every width and M (profiles/r06_cfg_small_sweep.log).  Same bits either way.
        const int small = fmt == FMT_F16 ? 4 : 16;
        cfg = (M % 256 == 0 && (M / 256) * n128 >= 2 * cus) ? 2 : (M % 128 == 0 && 2 * (M / 128) * n128 >= cus) ? 3 : small;
    }
    if ((cfg == 2 || cfg == 11) && M % 256) cfg = 3;
    if (cfg == 3 && M % 128) cfg = 4;
    if (cfg != 2 && cfg != 11 && cfg != 3 && cfg != 16) cfg = 4;
    return cfg;
}

// Statistics-fold capacity (LnFold::in_part) of a config for N features over M
// rows: the partial groups its LDS holds (cfg 3 keeps two workgroups per CU with
// 12: d <= 384, and holds 24 on one workgroup per CU where its tiles are at most
// one per CU; the 64-row forms 24: d <= 768); 0 = no fold form (the 256-row
// large-batch tiles).
int fold_cap(int cfg, int N, int M)
{
    if (cfg == 3) return (long)(M / 128) * ((N + 127) / 128) <= device_cu_count() ? 24 : 12;
    return (cfg == 4 || cfg == 16) ? 24 : 0;
}

template <int FMT>
int launch_fmt(const DevWeight &W, const h16 *x, int32_t M, const float *bias, int32_t epi, const void *res,
               void *out, hipStream_t s, LnFold ln, bool lnf, int cfg)
{
    cfg = pick_cfg(W.N, M, cfg, FMT);
    if (ln.in_part) {
        // statistics fold: the caller made sure the config has the capacity
        // (gemm_fold_ok); anything else is an error, never a silent fallback
        if (!lnf || epi == EPI_BIAS_RES || ln.in_G <= 0 || ln.in_G > fold_cap(cfg, W.N, M) ||
            32 * ln.in_G != (W.kx ? W.kx : W.K))
            return -1;
        switch (cfg) {
        case 3:
            // (the 24-group form: 91 KiB of LDS, one workgroup per CU)
            if (ln.in_G <= 12) dispatch_z<FMT, 4, 128, 4, 1, 3, 1, 0, 2, 12>(W, x, M, bias, epi, res, out, s, ln, lnf);
            else dispatch_z<FMT, 4, 128, 4, 1, 3, 1, 0, 1, 24>(W, x, M, bias, epi, res, out, s, ln, lnf);
            break;
        case 16: dispatch_z<FMT, 4, 64, 4, 1, 3, 2, 3, 2, 24>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
        default: dispatch_z<FMT, 2, 64, 4, 1, 3, 1, 0, 2, 24>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
        }
        return cfg;
    }
    // 256 x 128: the X pieces among the MFMAs (one per B-fragment item from the
    // K-step's start; +1.2-1.6 % on the C3 forward over one burst in front of them,
    // profiles/r03_gemm_xi_ab.log); cfg 11 keeps the burst form for A/B
    switch (cfg) {
    case 2: dispatch_z<FMT, 4, 256, 2, 1, 3, 1, 2>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
    case 11: dispatch_z<FMT, 4, 256, 2>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
    case 3: dispatch_z<FMT, 4, 128, 4>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
    case 16: dispatch_z<FMT, 4, 64, 4, 1, 3, 2, 3>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
    default: dispatch_z<FMT, 2, 64, 4>(W, x, M, bias, epi, res, out, s, ln, lnf); break;
    }
    return cfg;
}

}  // namespace

thread_local int g_gemm_cfg = 0;
thread_local int g_gemm_ran = 0;

// the config a forward launch asks for: the calling thread's test hook, else the
// BERT_GEMM_CFG A/B hook, else 0 (the heuristic)
static int forward_cfg()
{
    static const int env_cfg = [] { const char *e = std::getenv("BERT_GEMM_CFG"); return e ? std::atoi(e) : 0; }();
    return g_gemm_cfg ? g_gemm_cfg : env_cfg;
}

bool gemm_fold_ok(const DevWeight &W, int32_t M, int32_t G)
{
    return G > 0 && M > 0 && M % 64 == 0 && 32 * G == (W.kx ? W.kx : W.K) &&
           G <= fold_cap(pick_cfg(W.N, M, forward_cfg(), W.fmt), W.N, M);
}

// CUs of the calling thread's current device, cached per ordinal (a context may
// hold devices in different partition modes; launches size persistent grids
// and tile configs by the device they run on)
int device_cu_count()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) { (void)hipGetLastError(); return 256; }
    if (dev < 64) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < 64) cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

int launch_gemm(const DevWeight &W, const uint16_t *X, int32_t M, const float *bias, int32_t epi, const void *res,
                void *out, hipStream_t s, const LnFold &ln)
{
    const h16 *x = (const h16 *)X;
    if (W.N % 32 || W.K % ZK || M % 64 || M <= 0 || (W.kx && (W.kx % ZK || 2 * W.kx != W.K))) return -1;
    // the LN fold runs whole or not at all: input (mean, 1/sigma) + c1, or residual
    // LN + next gamma + partials
    const bool res_ln = ln.res_stats && ln.res_g && ln.res_b && ln.g_next && ln.part;
    if (epi == EPI_BIAS_RES && !res_ln && (ln.res_stats || ln.g_next)) return -1;
    if (epi != EPI_BIAS_RES && (ln.in_stats || ln.in_part) && !ln.c1) return -1;
    if (ln.in_stats && ln.in_part) return -1;
    const bool lnf = epi == EPI_BIAS_RES ? res_ln : (ln.in_stats || ln.in_part);
    const LnFold lnx = ln;
    const int cfg = forward_cfg();
    switch (W.fmt) {
    case FMT_Q4_0: g_gemm_ran = launch_fmt<FMT_Q4_0>(W, x, M, bias, epi, res, out, s, lnx, lnf, cfg); break;
    case FMT_Q4_1: g_gemm_ran = launch_fmt<FMT_Q4_1>(W, x, M, bias, epi, res, out, s, lnx, lnf, cfg); break;
    case FMT_Q8_0: g_gemm_ran = launch_fmt<FMT_Q8_0>(W, x, M, bias, epi, res, out, s, lnx, lnf, cfg); break;
    default: g_gemm_ran = launch_fmt<FMT_F16>(W, x, M, bias, epi, res, out, s, lnx, lnf, cfg); break;
    }
    return g_gemm_ran < 0 ? -1 : 0;
}

}  // namespace emb
