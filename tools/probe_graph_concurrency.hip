// Does a HIP graph run independent kernel nodes concurrently on this stack?
// Two single-block kernels that each spin ~200 us: serial ~400 us, concurrent ~200 us.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(long long cycles, int *out) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    int *d;
    CK(hipMalloc(&d, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const long long cyc = 200000LL * 100;   // ~200 us at 100 MHz clock64? calibrated below
    // calibrate: one kernel alone
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    long long c = cyc;
    void *args[] = {&c, &d};
    CK(hipEventRecord(a, s));
    CK(hipLaunchKernel((const void *)spin, dim3(1), dim3(64), args, 0, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float one = 0;
    CK(hipEventElapsedTime(&one, a, b));
    for (int mode = 0; mode < 2; ++mode) {
        hipGraph_t g;
        CK(hipGraphCreate(&g, 0));
        hipKernelNodeParams kp = {};
        kp.func = (void *)spin;
        kp.gridDim = dim3(1);
        kp.blockDim = dim3(64);
        kp.kernelParams = args;
        hipGraphNode_t n1, n2;
        CK(hipGraphAddKernelNode(&n1, g, nullptr, 0, &kp));
        if (mode == 0) CK(hipGraphAddKernelNode(&n2, g, nullptr, 0, &kp));      // independent
        else CK(hipGraphAddKernelNode(&n2, g, &n1, 1, &kp));                    // chained
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%s: one kernel %.3f ms, graph of two %.3f ms\n", mode == 0 ? "independent" : "chained", one, ms);
    }
    return 0;
}
