// Issue-throughput probe (diagnostic, not part of the library): with W waves
// per SIMD on every CU, each wave runs blocks of 8 independent SALU, VALU or
// mixed instructions; reports instructions per shader cycle per SIMD and per
// CU: all instructions of the grid / SIMDs / (kernel wall time from HIP events
// x the shader clock, the median over waves of s_memtime / s_memrealtime). Answers whether the
// scalar ALU is a per-CU resource (one SALU per cycle shared by the 4 SIMDs)
// or per SIMD, which decides what the rollouts' SALU counts cost.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_issue.hip -o tools/probe_issue
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__device__ __forceinline__ uint64_t now() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
constexpr int kIt = 16384;

#define S8(a, b, c, d, e, f, g, h)                                                                            \
    asm volatile("s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\ts_add_u32 %3, %3, 1\n\t" \
                 "s_add_u32 %4, %4, 1\n\ts_add_u32 %5, %5, 1\n\ts_add_u32 %6, %6, 1\n\ts_add_u32 %7, %7, 1"      \
                 : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h)::"scc")
#define V8(a, b, c, d, e, f, g, h)                                                                            \
    asm volatile("v_add_f32 %0, 1.0, %0\n\tv_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2\n\tv_add_f32 %3, 1.0, %3\n\t" \
                 "v_add_f32 %4, 1.0, %4\n\tv_add_f32 %5, 1.0, %5\n\tv_add_f32 %6, 1.0, %6\n\tv_add_f32 %7, 1.0, %7" \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h))
// a VALU instruction that writes an SGPR (the sweep's ballots / readlanes)
#define R8(x, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_readlane_b32 %0, %8, 1\n\tv_readlane_b32 %1, %8, 2\n\tv_readlane_b32 %2, %8, 3\n\t"         \
                 "v_readlane_b32 %3, %8, 4\n\tv_readlane_b32 %4, %8, 5\n\tv_readlane_b32 %5, %8, 6\n\t"         \
                 "v_readlane_b32 %6, %8, 7\n\tv_readlane_b32 %7, %8, 8"                                         \
                 : "=s"(a), "=s"(b), "=s"(c), "=s"(d), "=s"(e), "=s"(f), "=s"(g), "=s"(h) : "v"(x))

// a VOP3 compare writing an SGPR pair (a ballot)
#define C8(x, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_cmp_lt_f32_e64 %0, %8, 1.0\n\tv_cmp_lt_f32_e64 %1, %8, 2.0\n\tv_cmp_lt_f32_e64 %2, %8, 4.0\n\t" \
                 "v_cmp_lt_f32_e64 %3, %8, 0.5\n\tv_cmp_lt_f32_e64 %4, %8, -1.0\n\tv_cmp_lt_f32_e64 %5, %8, -2.0\n\t" \
                 "v_cmp_lt_f32_e64 %6, %8, -4.0\n\tv_cmp_lt_f32_e64 %7, %8, -0.5"                              \
                 : "=s"(a), "=s"(b), "=s"(c), "=s"(d), "=s"(e), "=s"(f), "=s"(g), "=s"(h) : "v"(x))
// v_writelane: an SGPR into one lane of a VGPR
#define W8(s, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_writelane_b32 %0, %8, 1\n\tv_writelane_b32 %1, %8, 2\n\tv_writelane_b32 %2, %8, 3\n\t"         \
                 "v_writelane_b32 %3, %8, 4\n\tv_writelane_b32 %4, %8, 5\n\tv_writelane_b32 %5, %8, 6\n\t"         \
                 "v_writelane_b32 %6, %8, 7\n\tv_writelane_b32 %7, %8, 8"                                         \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(s))
// v_cndmask with an SGPR-pair lane mask (reads an SGPR pair)
#define M8(m, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_cndmask_b32_e64 %0, %0, 1.0, %8\n\tv_cndmask_b32_e64 %1, %1, 1.0, %8\n\tv_cndmask_b32_e64 %2, %2, 1.0, %8\n\t" \
                 "v_cndmask_b32_e64 %3, %3, 1.0, %8\n\tv_cndmask_b32_e64 %4, %4, 1.0, %8\n\tv_cndmask_b32_e64 %5, %5, 1.0, %8\n\t" \
                 "v_cndmask_b32_e64 %6, %6, 1.0, %8\n\tv_cndmask_b32_e64 %7, %7, 1.0, %8"                     \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(m))
// s_nop (issue slot only)
#define N8() asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0")
// ds_read_b64 of one LDS address for every lane (a broadcast)
#define D8(p, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:8\n\tds_read_b64 %2, %8 offset:16\n\t"           \
                 "ds_read_b64 %3, %8 offset:24\n\tds_read_b64 %4, %8 offset:32\n\tds_read_b64 %5, %8 offset:40\n\t" \
                 "ds_read_b64 %6, %8 offset:48\n\tds_read_b64 %7, %8 offset:56\n\ts_waitcnt lgkmcnt(0)"        \
                 : "=v"(a), "=v"(b), "=v"(c), "=v"(d), "=v"(e), "=v"(f), "=v"(g), "=v"(h) : "v"(p))

// plain VALU with a 32-bit SGPR source operand
#define A8(s, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_add_f32 %0, %8, %0\n\tv_add_f32 %1, %8, %1\n\tv_add_f32 %2, %8, %2\n\tv_add_f32 %3, %8, %3\n\t" \
                 "v_add_f32 %4, %8, %4\n\tv_add_f32 %5, %8, %5\n\tv_add_f32 %6, %8, %6\n\tv_add_f32 %7, %8, %7" \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(s))
// VOPC compares into VCC, each consumed by a v_cndmask_b32_e32 (VCC)
#define K4(x, a, b, c, d)                                                                                     \
    asm volatile("v_cmp_lt_f32_e32 vcc, %4, %0\n\tv_cndmask_b32_e32 %0, %0, %4, vcc\n\t"                          \
                 "v_cmp_lt_f32_e32 vcc, %4, %1\n\tv_cndmask_b32_e32 %1, %1, %4, vcc\n\t"                          \
                 "v_cmp_lt_f32_e32 vcc, %4, %2\n\tv_cndmask_b32_e32 %2, %2, %4, vcc\n\t"                          \
                 "v_cmp_lt_f32_e32 vcc, %4, %3\n\tv_cndmask_b32_e32 %3, %3, %4, vcc"                                \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x) : "vcc")
// v_addc with an SGPR-pair carry in (the shl1_add_lane accumulation)
#define Q8(m, a, b, c, d, e, f, g, h)                                                                         \
    asm volatile("v_addc_co_u32_e64 %0, s[100:101], %0, %0, %8\n\tv_addc_co_u32_e64 %1, s[100:101], %1, %1, %8\n\t" \
                 "v_addc_co_u32_e64 %2, s[100:101], %2, %2, %8\n\tv_addc_co_u32_e64 %3, s[100:101], %3, %3, %8\n\t" \
                 "v_addc_co_u32_e64 %4, s[100:101], %4, %4, %8\n\tv_addc_co_u32_e64 %5, s[100:101], %5, %5, %8\n\t" \
                 "v_addc_co_u32_e64 %6, s[100:101], %6, %6, %8\n\tv_addc_co_u32_e64 %7, s[100:101], %7, %7, %8" \
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(m) : "s100", "s101")

template <int kKind>
__global__ __launch_bounds__(256) void probe(uint64_t *cyc, float *sink, int seed) {
    __shared__ double lds[64];
    if (threadIdx.x < 64) lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, s4 = seed + 4, s5 = seed + 5, s6 = seed + 6,
             s7 = seed + 7;
    float v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6,
          v7 = v0 + 7;
    uint32_t u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6,
             u7 = u0 + 7;
    const uint64_t t0 = now(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < kIt; ++k) {
        if constexpr (kKind == 0 || kKind == 2) S8(s0, s1, s2, s3, s4, s5, s6, s7);
        if constexpr (kKind == 1 || kKind == 2) V8(v0, v1, v2, v3, v4, v5, v6, v7);
        if constexpr (kKind == 3) R8(v0, s0, s1, s2, s3, s4, s5, s6, s7);
        if constexpr (kKind == 4) {
            uint64_t m0, m1, m2, m3, m4, m5, m6, m7;
            C8(v0, m0, m1, m2, m3, m4, m5, m6, m7);
            s0 ^= (uint32_t)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7) & 0;
        }
        if constexpr (kKind == 5) W8(s0, v0, v1, v2, v3, v4, v5, v6, v7);
        if constexpr (kKind == 6) M8((uint64_t)s0 | ((uint64_t)s1 << 32), v0, v1, v2, v3, v4, v5, v6, v7);
        if constexpr (kKind == 7) N8();
        if constexpr (kKind == 9) A8(s0, v0, v1, v2, v3, v4, v5, v6, v7);
        if constexpr (kKind == 10) {
            K4(v7, v0, v1, v2, v3);
            K4(v6, v4, v5, v1, v2);
        }
        if constexpr (kKind == 11) Q8((uint64_t)s0 | ((uint64_t)s1 << 32), u0, u1, u2, u3, u4, u5, u6, u7);
        if constexpr (kKind == 12) {
            double d0, d1, d2, d3, d4, d5, d6, d7;
            const uint32_t a = (uint32_t)(uintptr_t)lds + (threadIdx.x & 7) * 8;
            D8(a, d0, d1, d2, d3, d4, d5, d6, d7);
            v0 += (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
        }
        if constexpr (kKind == 13) {
            S8(s0, s1, s2, s3, s4, s5, s6, s7);
            A8(s7, v0, v1, v2, v3, v4, v5, v6, v7);
        }
        if constexpr (kKind == 14) {
            V8(v0, v1, v2, v3, v4, v5, v6, v7);
            A8(s7, u0, u1, u2, u3, u4, u5, u6, u7);
        }
        if constexpr (kKind == 15) {
            uint64_t m0, m1, m2, m3, m4, m5, m6, m7;
            S8(s0, s1, s2, s3, s4, s5, s6, s7);
            C8(v0, m0, m1, m2, m3, m4, m5, m6, m7);
            s0 ^= (uint32_t)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7) & 0;
        }
        if constexpr (kKind == 8) {
            double d0, d1, d2, d3, d4, d5, d6, d7;
            const uint32_t a = (uint32_t)(uintptr_t)lds;
            D8(a, d0, d1, d2, d3, d4, d5, d6, d7);
            v0 += (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
        }
    }
    const uint64_t t1 = now(), r1 = __builtin_amdgcn_s_memrealtime();
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * wave] = t1 - t0;
        cyc[2 * wave + 1] = r1 - r0;
    }
    sink[blockIdx.x * 256 + threadIdx.x] =
        v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + (float)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7) +
        (float)(u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
}

int main() {
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[] = {"salu", "valu", "salu+valu", "v_readlane->sgpr", "v_cmp->sgpr", "v_writelane",
                           "v_cndmask(sgpr)", "s_nop", "ds_read_b64 bcast", "v_add(sgpr src)", "v_cmp vcc+cndmask",
                           "v_addc(sgpr cin)", "ds_read_b64 8addr", "salu+v_add(sgpr)", "valu+v_add(sgpr)",
                           "salu+v_cmp->sgpr"};
    const int per_kind[] = {8, 8, 16, 8, 8, 8, 8, 8, 8, 8, 16, 8, 8, 16, 16, 16};
    for (int wps : {8}) {   // waves per SIMD: blocks of 4 waves, wps blocks per CU
        const int blocks = n_cu * wps, waves = blocks * 4;
        uint64_t *cyc;
        float *sink;
        hipMalloc(&cyc, 2 * waves * sizeof(uint64_t));
        hipMalloc(&sink, blocks * 256 * sizeof(float));
        for (int kind = 13; kind < 16; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {   // first run warms the clocks
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipEventRecord(e0);
                switch (kind) {
                    case 0: probe<0><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 1: probe<1><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 2: probe<2><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 3: probe<3><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 4: probe<4><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 5: probe<5><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 6: probe<6><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 7: probe<7><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 8: probe<8><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 9: probe<9><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 10: probe<10><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 11: probe<11><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 12: probe<12><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 13: probe<13><<<blocks, 256>>>(cyc, sink, rep); break;
                    case 14: probe<14><<<blocks, 256>>>(cyc, sink, rep); break;
                    default: probe<15><<<blocks, 256>>>(cyc, sink, rep); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                std::vector<uint64_t> h(2 * waves);
                hipMemcpy(h.data(), cyc, 2 * waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
                std::vector<double> clk(waves);
                for (int w = 0; w < waves; ++w) clk[w] = (double)h[2 * w] / (double)h[2 * w + 1] * 0.1;   // GHz
                std::sort(clk.begin(), clk.end());
                const double ghz = clk[waves / 2];
                const double insts = (double)kIt * per_kind[kind] * waves;
                const double per_simd = insts / (4.0 * n_cu) / (ms * 1e6 * ghz), per_cu = per_simd * 4;
                if (rep == 1)
                    printf("waves/SIMD %d  %-17s  %.3f inst/cyc/SIMD  %.3f inst/cyc/CU  (%.3f ms, clock %.2f GHz)\n",
                           wps, names[kind], per_simd, per_cu, ms, ghz);
                hipEventDestroy(e0);
                hipEventDestroy(e1);
            }
        }
        hipFree(cyc);
        hipFree(sink);
    }
    return 0;
}
