// Probe: which way of timing a kernel inside a HIP graph works on this ROCm.
// (a) hipEventRecord during capture; (b) hipEventRecordWithFlags(External)
// during capture; (c) manual graph: kernel nodes + hipGraphAddEventRecordNode;
// (d) eager events. Prints elapsed ms or the error for each.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(float *x, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        float v = x[i];
        for (int k = 0; k < 2000; ++k) v = v * 0.999f + 0.001f;
        x[i] = v;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("  %s -> %s\n", #x, hipGetErrorString(e_)); ok = false; } } while (0)

int main() {
    const int n = 1 << 20;
    float *x;
    (void)hipMalloc(&x, n * sizeof(float));
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    bool ok;
    for (int variant = 0; variant < 2; ++variant) {
        ok = true;
        printf("variant %c (capture, %s)\n", 'a' + variant, variant ? "WithFlags External" : "hipEventRecord");
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        if (variant == 0) CK(hipEventRecord(e0, s)); else CK(hipEventRecordWithFlags(e0, s, hipEventRecordExternal));
        hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, x, n);
        if (variant == 0) CK(hipEventRecord(e1, s)); else CK(hipEventRecordWithFlags(e1, s, hipEventRecordExternal));
        CK(hipStreamEndCapture(s, &g));
        if (ok) CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        if (ok) CK(hipGraphLaunch(ge, s));
        if (ok) CK(hipStreamSynchronize(s));
        float ms = -1;
        if (ok) CK(hipEventElapsedTime(&ms, e0, e1));
        printf("  ok=%d ms=%f\n", ok, ms);
        if (ge) (void)hipGraphExecDestroy(ge);
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
    }
    {
        ok = true;
        printf("variant c (manual graph, event record nodes)\n");
        hipGraph_t g;
        CK(hipGraphCreate(&g, 0));
        hipGraphNode_t ne0, nk, ne1;
        CK(hipGraphAddEventRecordNode(&ne0, g, nullptr, 0, e0));
        hipKernelNodeParams kp = {};
        int nn = n;
        void *args[] = {&x, &nn};
        kp.func = (void *)spin;
        kp.gridDim = dim3(n / 256);
        kp.blockDim = dim3(256);
        kp.sharedMemBytes = 0;
        kp.kernelParams = args;
        kp.extra = nullptr;
        CK(hipGraphAddKernelNode(&nk, g, &ne0, 1, &kp));
        CK(hipGraphAddEventRecordNode(&ne1, g, &nk, 1, e1));
        hipGraphExec_t ge = nullptr;
        if (ok) CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        float ms = -1;
        for (int r = 0; r < 3 && ok; ++r) {
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("  replay %d ok=%d ms=%f\n", r, ok, ms);
        }
        (void)hipGetLastError();
    }
    {
        ok = true;
        printf("variant d (eager)\n");
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, x, n);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = -1;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("  ok=%d ms=%f\n", ok, ms);
    }
    return 0;
}
