// Granule staleness across XCDs: does an agent-scope
// load on one XCD keep returning an old granule after a workgroup on another
// XCD has stored a new one, and for how long; which load / memory forms fix it.
//
// One launch of 1 + R workgroups of one wave: workgroup 0 writes, the others
// read (blocks are dealt round-robin over the 8 XCDs, so readers 1..7 sit on
// other XCDs than the writer and reader 8 on its own; each records XCC_ID).
// Per round r = 1..ROUNDS:
//   every reader loads the granule with the load form under test (so that
//   line is in its XCD's L2 when the form caches there) and expects r - 1,
//   then arrives on a counter (agent-scope atomic add: executed at memory);
//   the writer waits for all arrivals (polling with a returning atomic add of
//   0, never a cacheable load) and stores r with an agent-scope relaxed store
//   (sc1: write-through);
//   every reader polls with the form under test until it reads r or 200 us
//   pass, and records the s_memrealtime ticks (100 MHz) it took, or -1.
// Load forms: 0 agent-scope relaxed (`sc1`, the rollouts' form), 1
// system-scope relaxed (`sc0 sc1`), 2 agent acquire fence (`buffer_inv sc1`)
// before each agent-scope load, 3 returning atomic add of 0 (memory-side).
// Memory: 0 hipMalloc, 1 hipDeviceMallocUncached, 2 hipDeviceMallocFinegrained.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_stale.hip -o tools/probe_stale
// Run:   tools/probe_stale   (prints one JSON object per memory x form)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kReaders = 15, kRounds = 64;
constexpr uint64_t kTimeout = 20000;   // 200 us at 100 MHz

typedef __attribute__((address_space(1))) uint64_t gu64;

template <int kForm>
__device__ __forceinline__ uint64_t rd(uint64_t *g) {
    if constexpr (kForm == 0) return __hip_atomic_load((gu64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (kForm == 1) return __hip_atomic_load((gu64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (kForm == 2) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        return __hip_atomic_load((gu64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return __hip_atomic_fetch_add((gu64 *)g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int kForm>
__global__ void probe(uint64_t *gran, uint64_t *arrive, int64_t *lat, int *xcc) {
    const int b = blockIdx.x;
    if (threadIdx.x != 0) return;
    xcc[b] = (int)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u);
    for (int r = 1; r <= kRounds; ++r) {
        if (b == 0) {
            const uint64_t want = (uint64_t)kReaders * r;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_fetch_add((gu64 *)arrive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100 * kTimeout) return;   // a reader is gone
                __builtin_amdgcn_s_sleep(4);
            }
            __builtin_amdgcn_s_sleep(20);   // the readers are polling by now
            __hip_atomic_store((gu64 *)gran, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            (void)rd<kForm>(gran);   // the line into this XCD's L2 (as the form caches it)
            __hip_atomic_fetch_add((gu64 *)arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int64_t got = -1;
            for (;;) {
                const uint64_t x = rd<kForm>(gran);
                const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
                if (x >= (uint64_t)r) { got = (int64_t)dt; break; }
                if (dt > kTimeout) break;
            }
            lat[(b - 1) * kRounds + (r - 1)] = got;
            // the next round needs every reader past this one: wait for the
            // writer's next store only after all readers have arrived again
        }
    }
}

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

template <int kForm>
void run(int mem) {
    uint64_t *buf = nullptr;
    const size_t bytes = 4096;
    if (mem == 0) CK(hipMalloc(&buf, bytes));
    if (mem == 1) CK(hipExtMallocWithFlags((void **)&buf, bytes, hipDeviceMallocUncached));
    if (mem == 2) CK(hipExtMallocWithFlags((void **)&buf, bytes, hipDeviceMallocFinegrained));
    CK(hipMemset(buf, 0, bytes));
    int64_t *lat;
    int *xcc;
    CK(hipMalloc(&lat, sizeof(int64_t) * kReaders * kRounds));
    CK(hipMalloc(&xcc, sizeof(int) * (kReaders + 1)));
    CK(hipDeviceSynchronize());
    // granule and counter on different 4 KiB halves' lines
    hipLaunchKernelGGL(probe<kForm>, dim3(kReaders + 1), dim3(64), 0, 0, buf, buf + 256, lat, xcc);
    CK(hipDeviceSynchronize());
    int64_t h[kReaders * kRounds];
    int hx[kReaders + 1];
    CK(hipMemcpy(h, lat, sizeof h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hx, xcc, sizeof hx, hipMemcpyDeviceToHost));
    // per reader: rounds timed out, and the median / max ticks of the others
    printf("{\"mem\": \"%s\", \"form\": \"%s\", \"writer_xcc\": %d, \"readers\": [",
           mem == 0 ? "hipMalloc" : mem == 1 ? "uncached" : "finegrained",
           kForm == 0 ? "agent_load_sc1" : kForm == 1 ? "system_load" : kForm == 2 ? "acquire_fence+agent_load"
                                                                                  : "atomic_add0",
           hx[0]);
    for (int r = 0; r < kReaders; ++r) {
        int stale = 0;
        int64_t v[kRounds];
        int n = 0;
        for (int k = 0; k < kRounds; ++k) {
            const int64_t x = h[r * kRounds + k];
            if (x < 0) ++stale; else v[n++] = x;
        }
        for (int i = 1; i < n; ++i)
            for (int j = i; j > 0 && v[j] < v[j - 1]; --j) { int64_t t = v[j]; v[j] = v[j - 1]; v[j - 1] = t; }
        printf("%s{\"xcc\": %d, \"timed_out\": %d, \"median_ticks\": %lld, \"max_ticks\": %lld}", r ? ", " : "",
               hx[r + 1], stale, n ? (long long)v[n / 2] : -1LL, n ? (long long)v[n - 1] : -1LL);
    }
    printf("]}\n");
    CK(hipFree(buf));
    CK(hipFree(lat));
    CK(hipFree(xcc));
}

int main() {
    for (int mem = 0; mem < 3; ++mem) {
        run<0>(mem);
        run<1>(mem);
        run<2>(mem);
        run<3>(mem);
    }
    return 0;
}
