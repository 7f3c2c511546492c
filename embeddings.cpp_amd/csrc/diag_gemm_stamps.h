// Cycle stamps of the GEMM kernels (gemm.hip, its only includer): the
// diagnostics-only part; diag_att_stamps.h is the attention's.
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
// GEMM: per wave-tile slots 0-3 = start / after the prologue / after the K loop
// / after the epilogue, 4-5 = HW_ID / XCC_ID, 6-7 = the K loop's front-wait
// (NS 2: X-piece issue) and back-wait + barrier cycles
// ---------------------------------------------------------------------------
#ifdef GEMM_STAMPS
__device__ unsigned long long g_gemm_stamps[1 << 18];
#define ZSTAMP(i, v) do { if ((threadIdx.x & 63) == 0) g_gemm_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (i)] = (v); } while (0)
struct ZClock {
    unsigned long long front = 0, back = 0, t = 0;
    __device__ __forceinline__ void mark() { t = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void add_front() { front += __builtin_amdgcn_s_memtime() - t; }
    __device__ __forceinline__ void add_back() { back += __builtin_amdgcn_s_memtime() - t; }
};
#define ZSTAMP_KSPLIT(zc)                                                          \
    do {                                                                           \
        ZSTAMP(4, __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)));        \
        ZSTAMP(5, __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)));       \
        ZSTAMP(6, (zc).front);                                                     \
        ZSTAMP(7, (zc).back);                                                      \
    } while (0)
extern "C" __attribute__((visibility("default"))) int bertx_gemm_stamps(unsigned long long *host, size_t n)
{
    if (n > (1u << 18)) n = 1u << 18;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), n * 8) == hipSuccess ? 0 : -1;
}
#else
#define ZSTAMP(i, v) do { } while (0)
struct ZClock {
    __device__ __forceinline__ void mark() {}
    __device__ __forceinline__ void add_front() {}
    __device__ __forceinline__ void add_back() {}
};
#define ZSTAMP_KSPLIT(zc) do { (void)(zc); } while (0)
#endif

}  // namespace emb
