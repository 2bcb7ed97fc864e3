// Latency probe (diagnostic, not part of the library): one wave per SIMD runs
// dependent chains of the instruction kinds on the ragged assignment's path
// iteration and reports s_memtime cycles per chain step. Build:
// hipcc --offload-arch=gfx950 -O3 tools/probe_latency.hip -o tools/probe_latency
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t now() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ int dpp_any(int v) {
    return __builtin_amdgcn_update_dpp(0x7fffffff, v, kCtrl, kRowMask, 0xf, false);
}
__device__ __forceinline__ int min32_i(int v) {
    v = min(v, dpp_any<0xB1>(v));
    v = min(v, dpp_any<0x4E>(v));
    v = min(v, dpp_any<0x141>(v));
    v = min(v, dpp_any<0x140>(v));
    v = min(v, dpp_any<0x142, 0xa>(v));
    return __builtin_amdgcn_readlane(v, 31);
}
constexpr int kIt = 256, kSlots = 8;
#define OPAQUE_V(x) asm volatile("" : "+v"(x))
#define OPAQUE_S(x) asm volatile("" : "+s"(x))

__global__ void probe(uint64_t *out, int seed) {
    const int lane = threadIdx.x & 63;
    uint64_t t0, t1;
    uint64_t *o = out + (size_t)blockIdx.x * kSlots;
    // (0) DPP min over 32 lanes + readlane, result feeds the next key
    int x = (lane * 7 + seed) & 1023;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {
        OPAQUE_V(x);
        const int m = min32_i(x);
        x = (x ^ m) + 1;
    }
    t1 = now();
    if (lane == 0) o[0] = t1 - t0 + (x & 0);
    // (1) three dependent f64 adds, SGPR operands
    double d = lane * 0.5 + seed, s = 0.25 + seed;

    t0 = now();
    for (int k = 0; k < kIt; ++k) {
        OPAQUE_V(d);
        d = ((s + d) - s) - 1e-30;
    }
    t1 = now();
    if (lane == 0) o[1] = t1 - t0 + (d > 1e300 ? 1 : 0);
    // (2) readlane whose lane index is the previous readlane's result
    int idx = seed & 31;
    const int val = (lane * 5 + 3) & 31;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {

        idx = __builtin_amdgcn_readlane(val, idx);
    }
    t1 = now();
    if (lane == 0) o[2] = t1 - t0 + (idx & 0);
    // (3) VALU compare -> ballot -> s_ff1 -> readlane -> next compare
    int y = (lane * 13 + seed) & 63, tgt = 5;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {

        const uint64_t b = __builtin_amdgcn_ballot_w64(y == tgt) | (1ull << 63);
        const int j = __builtin_ctzll(b);
        tgt = (__builtin_amdgcn_readlane(y, j) + 1) & 63;
    }
    t1 = now();
    if (lane == 0) o[3] = t1 - t0 + (tgt & 0);
    // (4) four dependent int VALU ops
    int z = lane;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {
        OPAQUE_V(z);
        z = z * 3 + 1;
        z = z ^ 5;
        z = z >> 1;
    }
    t1 = now();
    if (lane == 0) o[4] = t1 - t0 + (z & 0);
    // (5) empty loop (one opaque VGPR per iteration)
    int w = seed;
    t0 = now();
    for (int k = 0; k < kIt; ++k) OPAQUE_V(w);
    t1 = now();
    if (lane == 0) o[5] = t1 - t0 + (w & 0);
    // (6) uniform branch on a ballot each iteration (taken every other time)
    int q = lane;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {
        OPAQUE_V(q);
        if (__builtin_amdgcn_ballot_w64(((q + k) & 1) == 0) & 1) q += 3;
        else q -= 1;
    }
    t1 = now();
    if (lane == 0) o[6] = t1 - t0 + (q & 0);
    // (7) register-indexed read (s_set_gpr_idx) with the index from the value
    float arr[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) arr[i] = (float)((lane + i * 7) & 31);
    int ri = seed & 31;
    t0 = now();
    for (int k = 0; k < kIt; ++k) {

        const float f = arr[ri];
        ri = __builtin_amdgcn_readfirstlane((int)f);
    }
    t1 = now();
    if (lane == 0) o[7] = t1 - t0 + (ri & 0);
}

// VALU issue rate: every wave runs 4 independent chains of integer VALU ops;
// cycles per SIMD per VALU instruction = wave cycles / (instructions x waves
// resident on the SIMD). Also reports the shader clock (s_memtime ticks per
// s_memrealtime tick x 100 MHz).
__global__ void issue(uint64_t *out, int seed) {
    float a = threadIdx.x, b = a + seed, c = a * 0.5f, d = a * 3;
    uint64_t r0, t0, t1, r1;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
    t0 = now();
    for (int k = 0; k < 1024; ++k) {
        OPAQUE_V(a);
        a = __builtin_fmaf(a, 0.999f, 0.5f); b = __builtin_fmaf(b, 0.998f, 0.25f);
        c = __builtin_fmaf(c, 0.997f, 0.125f); d = __builtin_fmaf(d, 0.996f, 0.0625f);
        a = __builtin_fmaf(a, 0.999f, b); b = __builtin_fmaf(b, 0.998f, c);
        c = __builtin_fmaf(c, 0.997f, d); d = __builtin_fmaf(d, 0.996f, a);
    }
    t1 = now();
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[w * 2] = t1 - t0;
        out[w * 2 + 1] = r1 - r0;
    }
    if (a + b + c + d == 1.2345f) out[0] = 0;
}

int main() {
    const char *names[kSlots] = {"dpp min32 + readlane", "3x f64 add (dependent)", "readlane(idx from readlane)",
                                 "cmp->ballot->ff1->readlane", "3 dependent int VALU", "empty loop",
                                 "ballot -> uniform branch", "movrel read -> readfirstlane"};
    const int max_blocks = 256 * 4;
    uint64_t *d = nullptr;
    if (hipMalloc(&d, (size_t)max_blocks * kSlots * sizeof(uint64_t)) != hipSuccess) return 1;
    static uint64_t h[max_blocks * kSlots];
    for (int per_cu : {1, 4}) {
        const int blocks = 256 * per_cu;
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, d, 1);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(h, d, (size_t)blocks * kSlots * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 3;
        printf("%d one-wave blocks per CU:\n", per_cu);
        for (int k = 0; k < kSlots; ++k) {
            double s = 0;
            for (int b = 0; b < blocks; ++b) s += (double)h[b * kSlots + k];
            printf("  %-32s %7.1f cycles per iteration\n", names[k], s / blocks / kIt);
        }
    }
    // issue rate at 1, 2, 4, 8 waves per SIMD (blocks of 256 threads: one wave per SIMD each)
    uint64_t *d2 = nullptr;
    const int max_w = 256 * 4 * 8;
    if (hipMalloc(&d2, (size_t)max_w * 2 * sizeof(uint64_t)) != hipSuccess) return 4;
    static uint64_t h2[max_w * 2];
    for (int per_simd : {1, 2, 4, 8}) {
        const int blocks = 256 * per_simd;   // 4 waves per block, one per SIMD
        hipLaunchKernelGGL(issue, dim3(blocks), dim3(256), 0, 0, d2, 1);
        if (hipDeviceSynchronize() != hipSuccess) return 5;
        const int waves = blocks * 4;
        if (hipMemcpy(h2, d2, (size_t)waves * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 6;
        double cyc = 0, rt = 0;
        for (int w = 0; w < waves; ++w) { cyc += (double)h2[w * 2]; rt += (double)h2[w * 2 + 1]; }
        cyc /= waves; rt /= waves;
        // 1024 iterations x 8 v_fma_f32
        printf("%d waves/SIMD: %.0f cycles per wave, %.2f cycles per VALU per SIMD, clock %.2f GHz\n", per_simd, cyc,
               cyc / (1024.0 * 8.0 * per_simd), cyc / rt * 0.1);
    }
    return 0;
}
