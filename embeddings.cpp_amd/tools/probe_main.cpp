// bert_probe: a fixed number of device-resident forwards of one synthetic batch,
// with no Python or torch in the process -- the program bench.py runs under
// `rocprofv3 --pmc` to read this run's HBM counters (FETCH_SIZE / WRITE_SIZE)
// per kernel launch.  Token ids as bertpy.synthetic_ids: [CLS] + uniform ids in
// [1000, n_vocab) + [SEP].
//
// usage: bert_probe MODEL N_SEQS SEQ_LEN [STEPS=3] [WARMUP=1]
// prints one line: {"n_seqs":..,"seq_len":..,"steps":..,"us_per_forward":..}
#include "bert.h"
#include "bert_hip.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "bert_probe: %s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main(int argc, char **argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s MODEL N_SEQS SEQ_LEN [STEPS=3] [WARMUP=1]\n", argv[0]);
        return 2;
    }
    const int B = std::atoi(argv[2]), L = std::atoi(argv[3]);
    const int steps = argc > 4 ? std::atoi(argv[4]) : 3, warm = argc > 5 ? std::atoi(argv[5]) : 1;
    if (B <= 0 || L <= 0 || steps <= 0 || warm < 0) return 2;
    bert_ctx *ctx = bert_load_from_file(argv[1]);
    if (!ctx) return 1;
    int32_t hp[7];
    bertx_hparams(ctx, hp);
    if (L > hp[1]) {
        std::fprintf(stderr, "bert_probe: seq_len %d > n_max_tokens %d\n", L, hp[1]);
        return 2;
    }
    const int T = B * L, d = hp[2];
    std::vector<int32_t> ids((size_t)T), cu((size_t)B + 1);
    uint64_t st = 7;
    for (int b = 0; b < B; ++b) {
        cu[(size_t)b] = b * L;
        for (int i = 0; i < L; ++i) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            ids[(size_t)b * L + i] = 1000 + (int32_t)((st >> 33) % (uint64_t)(hp[0] - 1000));
        }
        ids[(size_t)b * L] = 101;
        ids[(size_t)b * L + L - 1] = 102;
    }
    cu[(size_t)B] = T;
    if (bertx_reserve(ctx, 0, T, B) != 0) return 1;
    int32_t *d_ids = nullptr, *d_cu = nullptr;
    float *d_out = nullptr;
    hipStream_t s = nullptr;
    CK(hipSetDevice(bertx_device_ordinal(ctx, 0)));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipMalloc((void **)&d_ids, ids.size() * 4));
    CK(hipMalloc((void **)&d_cu, cu.size() * 4));
    CK(hipMalloc((void **)&d_out, (size_t)B * d * 4));
    CK(hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_cu, cu.data(), cu.size() * 4, hipMemcpyHostToDevice));
    for (int i = 0; i < warm; ++i)
        if (bertx_forward_device(ctx, 0, d_ids, d_cu, B, L, T, d_out, s) != 0) return 1;
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i)
        if (bertx_forward_device(ctx, 0, d_ids, d_cu, B, L, T, d_out, s) != 0) return 1;
    CK(hipStreamSynchronize(s));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::vector<float> out((size_t)B * d);
    CK(hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost));
    double nrm = 0;
    for (int c = 0; c < d; ++c) nrm += (double)out[(size_t)c] * out[(size_t)c];
    std::printf("{\"n_seqs\": %d, \"seq_len\": %d, \"steps\": %d, \"warmup\": %d, \"us_per_forward\": %.2f, "
                "\"norm0\": %.6f}\n",
                B, L, steps, warm, us / steps, nrm);
    (void)hipFree(d_ids);
    (void)hipFree(d_cu);
    (void)hipFree(d_out);
    (void)hipStreamDestroy(s);
    bert_free(ctx);
    return 0;
}
