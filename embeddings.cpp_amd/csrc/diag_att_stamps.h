// Cycle stamps of the attention kernel (attention.hip, its only includer): the
// diagnostics-only part; diag_gemm_stamps.h is the GEMM's.
//
// The production kernels (gemm.hip, attention.hip) carry named stamp points --
// ZSTAMP / ZSTAMP_KSPLIT / ZClock for the GEMM, ASTAMP / ASTAMP_ITEM for the
// attention -- and nothing else.  Only this header knows whether a build records
// them: a diagnostics build (make EXTRA=-DGEMM_STAMPS or -DATT_STAMPS
// BUILD=build/stamps, scripts/gemm_stamps.py, scripts/att_stamps.py) gets the
// device arrays, the s_memtime reads and the host readers bertx_gemm_stamps /
// bertx_att_stamps; every other build gets empty inline functions and macros
// that compile to nothing (the shipped code objects hold no stamp code).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace emb {

// ---------------------------------------------------------------------------
// Attention (attention_lds3): per wave and item (at most 4 items per workgroup)
// slots 0-6 = item start / after block 0 / B1's arrival / after B1 / block loop
// end / after S / after the stores, 7 = HW_ID.  ASTAMP needs `lane`, `w` and the
// item counter of ASTAMP_ITEMS in scope.
// ---------------------------------------------------------------------------
#ifdef ATT_STAMPS
__device__ unsigned long long g_att_stamps[1 << 17];
#define ASTAMP_ITEMS(nit) int nit = 0
#define ASTAMP(k, v) do { if (lane == 0 && nit < 4) g_att_stamps[(((size_t)blockIdx.x * 16 + w) * 4 + nit) * 8 + (k)] = (v); } while (0)
#define ASTAMP_ITEM_END(nit)                                                                    \
    do {                                                                                        \
        ASTAMP(7, (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11))); \
        ++(nit);                                                                                \
    } while (0)
extern "C" __attribute__((visibility("default"))) int bertx_att_stamps(unsigned long long *host, size_t n)
{
    if (n > (1u << 17)) n = 1u << 17;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_stamps), n * 8) == hipSuccess ? 0 : -1;
}
#else
#define ASTAMP_ITEMS(nit) do { } while (0)
#define ASTAMP(k, v) do { } while (0)
#define ASTAMP_ITEM_END(nit) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// attention_pp: per workgroup (unit) and wave, slots 0 unit start, 1 after block
// 0's wait + barrier, 2 after block 0, 3 / 4 cycles summed over blocks >= 1 in
// the wait + barrier + issue / in the block's compute, 5 after the block loop,
// 6 after the stores, 7 HW_ID.  PST_* need `lane` and `w` in scope.
// ---------------------------------------------------------------------------
#ifdef ATT_STAMPS
#define PST_DECL unsigned long long pst_t = 0, pst_w = 0, pst_c = 0
#define PST_SET(k, v) do { if (lane == 0) g_att_stamps[((size_t)blockIdx.x * 8 + w) * 8 + (k)] = (v); } while (0)
#define PST_NOW() __builtin_amdgcn_s_memtime()
#define PST_MARK() (pst_t = __builtin_amdgcn_s_memtime())
#define PST_ADDW() (pst_w += __builtin_amdgcn_s_memtime() - pst_t)
#define PST_ADDC() (pst_c += __builtin_amdgcn_s_memtime() - pst_t)
#define PST_SUMS() do { PST_SET(3, pst_w); PST_SET(4, pst_c); } while (0)
#define PST_HWID() PST_SET(7, (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)))
#else
#define PST_DECL do { } while (0)
#define PST_SET(k, v) do { } while (0)
#define PST_NOW() 0
#define PST_MARK() do { } while (0)
#define PST_ADDW() do { } while (0)
#define PST_ADDC() do { } while (0)
#define PST_SUMS() do { } while (0)
#define PST_HWID() do { } while (0)
#endif

}  // namespace emb
