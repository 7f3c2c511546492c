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

}  // namespace emb
