// Launch floor of a captured forward: a HIP graph of 63 kernels (the B 1 forward's
// count) replayed back to back, for kernels that do nothing, kernels of one
// 64-thread workgroup that store one value, and 1024-thread / 256-workgroup
// shapes like the forward's.  Prints one JSON line per shape: microseconds per
// replay and per kernel.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_store(float *p) { if (threadIdx.x == 0) p[blockIdx.x] = 1.0f; }

int main()
{
    float *buf = nullptr;
    (void)hipMalloc(&buf, 1 << 20);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    struct Shape { const char *name; int grid, block; };
    const Shape shapes[] = {{"1 x 64", 1, 64}, {"36 x 128", 36, 128}, {"256 x 256", 256, 256}, {"12 x 1024", 12, 1024},
                            {"1024 x 256", 1024, 256}};
    for (const Shape &sh : shapes) {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < 63; ++i) hipLaunchKernelGGL(k_store, dim3(sh.grid), dim3(sh.block), 0, s, buf);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int i = 0; i < 20; ++i) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        const int reps = 200;
        (void)hipEventRecord(a, s);
        for (int i = 0; i < reps; ++i) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        std::printf("{\"shape\": \"%s\", \"kernels\": 63, \"us_per_replay\": %.1f, \"us_per_kernel\": %.2f}\n", sh.name,
                    ms * 1e3 / reps, ms * 1e3 / reps / 63);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    (void)hipFree(buf);
    return 0;
}
