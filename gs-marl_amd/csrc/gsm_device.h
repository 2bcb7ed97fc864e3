// Device helpers shared by the segmented, tile and ragged kernel families.
#pragma once
#include "gsm_internal.h"
#include "gsm_philox.h"

namespace gsm {

enum { kModeStep = 0, kModeReset = 1, kModeObserve = 2 };

// v_writelane_b32: replace lane `lane` of `old` with the wave-uniform `src`
// (the LLVM intrinsic has no clang builtin; bound by name so the compiler
// still schedules it and resolves its hazards)
__device__ uint32_t writelane_u32(uint32_t src, uint32_t lane, uint32_t old) __asm("llvm.amdgcn.writelane.i32");

// 2*own + (this lane's bit of `lanes`): one v_addc per column (the compiler
// builds own |= bit << j from a select and a shift-or)
__device__ __forceinline__ uint32_t shl1_add_lane(uint32_t own, uint64_t lanes) {
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(own), "s"(lanes));
    return r;
}

// The launch's DevParams read back from the kernarg segment at the point of
// use: fields loaded through this view are fresh scalar loads there (the asm
// hides that the pointer is the one read at kernel entry), so base pointers
// used only by a kernel's final stores do not hold SGPRs across the kernel.
// Valid in kernels whose first argument is the DevParams (all of them).
typedef const __attribute__((address_space(4))) DevParams KernargParams;
__device__ __forceinline__ KernargParams &late_params() {
    KernargParams *kp = (KernargParams *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *kp;
}

// v_cndmask with a wave-uniform lane mask held in SGPRs (a ballot, a bit
// set): lanes whose bit of m is set take a, the others b. The mask is used as
// is, without the per-lane bit extraction (v_and + v_cmp) the compiler emits
// for a select on ((m >> lane) & 1).
__device__ __forceinline__ uint32_t sel_lanes(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ int sel_lanes(uint64_t m, int a, int b) {
    return (int)sel_lanes(m, (uint32_t)a, (uint32_t)b);
}
__device__ __forceinline__ double sel_lanes(uint64_t m, double a, double b) {
    const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
    const uint32_t lo = sel_lanes(m, (uint32_t)ua, (uint32_t)ub);
    const uint32_t hi = sel_lanes(m, (uint32_t)(ua >> 32), (uint32_t)(ub >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Orders LDS traffic between the lanes of one wave: LDS ops of a wave execute
// in order, so only compiler motion has to be fenced.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// --- DPP wave collectives (gfx9 DPP: quad_perm, row mirrors, row_shr, row_bcast)
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, kCtrl, kRowMask, 0xf, true);
}
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, kRowMask, 0xf, true));
}
// sum over the 64 lanes, returned wave-uniform
__device__ __forceinline__ int wave_total(int v) {
    v += dpp_i<0xB1>(v);          // quad_perm [1,0,3,2]
    v += dpp_i<0x4E>(v);          // quad_perm [2,3,0,1]
    v += dpp_i<0x141>(v);         // row_half_mirror
    v += dpp_i<0x140>(v);         // row_mirror: every lane holds its row's sum
    v += dpp_i<0x142, 0xa>(v);    // row_bcast:15 -> rows 1, 3
    v += dpp_i<0x143, 0xc>(v);    // row_bcast:31 -> rows 2, 3 (lane 63 = total)
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ float wave_total(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    v += dpp_f<0x142, 0xa>(v);
    v += dpp_f<0x143, 0xc>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// inclusive scan over the 64 lanes (Hillis-Steele in rows of 16, then row broadcasts)
__device__ __forceinline__ int wave_scan(int v) {
    v += dpp_i<0x111>(v);         // row_shr:1
    v += dpp_i<0x112>(v);         // row_shr:2
    v += dpp_i<0x114>(v);         // row_shr:4
    v += dpp_i<0x118>(v);         // row_shr:8
    v += dpp_i<0x142, 0xa>(v);
    v += dpp_i<0x143, 0xc>(v);
    return v;
}

// In-kernel phase stamps for diagnostic builds (-DGSM_STAMPS): lane 0 of each
// wave records s_memtime at phase boundaries into p.stamps[wave][k]. Never
// compiled into the product library.
#ifdef GSM_STAMPS
#define GSM_STAMP(p, wave_id, k)                                                                  \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        unsigned long long t_;                                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if ((p).stamps && (threadIdx.x & 63) == 0) (p).stamps[(int64_t)(wave_id)*16 + (k)] = t_;  \
    } while (0)
#define GSM_RSTAMP(p, wave_id, k)                                                                 \
    do {                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        unsigned long long t_;                                                                    \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        if ((p).stamps && (threadIdx.x & 63) == 0) (p).stamps[(int64_t)(wave_id)*16 + (k)] = t_;  \
    } while (0)
// cycles since t0 (a GSM_TNOW) added to p.stamps[wave][k] (vector atomic)
#define GSM_TNOW(var)                                                                             \
    unsigned long long var;                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0)
#define GSM_ACC(p, wave_id, k, t0)                                                                \
    do {                                                                                          \
        GSM_TNOW(t1_);                                                                            \
        if ((p).stamps && (threadIdx.x & 63) == 0)                                                \
            __hip_atomic_fetch_add((p).stamps + (int64_t)(wave_id)*16 + (k), t1_ - (t0),          \
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                   \
    } while (0)
#define GSM_SET(p, wave_id, k, val)                                                               \
    do {                                                                                          \
        if ((p).stamps && (threadIdx.x & 63) == 0) (p).stamps[(int64_t)(wave_id)*16 + (k)] = (val); \
    } while (0)
#else
#define GSM_STAMP(p, wave_id, k) do { (void)(wave_id); } while (0)
#define GSM_RSTAMP(p, wave_id, k) do { (void)(wave_id); } while (0)
#define GSM_TNOW(var) do { } while (0)
#define GSM_ACC(p, wave_id, k, t0) do { (void)(wave_id); } while (0)
#define GSM_SET(p, wave_id, k, val) do { (void)(wave_id); } while (0)
#endif

// number of set bits of `mask` below this lane
__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// compact collider index (agents [0,N), obstacles [N,M)) -> entity index
__device__ __forceinline__ int collider_entity(int c, int N) { return c < N ? c : N + c; }

__device__ __forceinline__ float2 layout_pos(const DevParams &p, uint32_t gid, uint32_t ep,
                                             uint32_t e) {
    // keys in VGPRs: the (cold) reset path otherwise holds Philox's whole
    // wave-uniform key schedule in SGPRs, which set the step kernels' SGPR
    // count and hence their occupancy
    uint32_t k0 = p.seed_lo, k1 = p.seed_hi;
    asm volatile("" : "+v"(k0), "+v"(k1));
    const Philox4 x = philox4x32_10(e, ep, gid, kTagLayout, k0, k1);
    return make_float2(u01(x.x0) * p.twoL - p.L, u01(x.x1) * p.twoL - p.L);
}

// Environment._set_action + apply_action_force (App. A S5).
__device__ __forceinline__ float2 action_force(const DevParams &p, int64_t a) {
    float ux, uy;
    if (p.action_fmt == 0) {
        const float *q = (const float *)p.actions + a * 5;
        ux = q[1] - q[2];
        uy = q[3] - q[4];
    } else if (p.action_fmt == 1) {
        const int k = ((const int32_t *)p.actions)[a];
        ux = (float)(k == 1) - (float)(k == 2);
        uy = (float)(k == 3) - (float)(k == 4);
    } else {
        const float2 q = ((const float2 *)p.actions)[a];
        ux = q.x;
        uy = q.y;
    }
    return make_float2(ux * p.sens, uy * p.sens);
}

// App. A S16 (degenerate states). nonfinite2: a position with a NaN/inf
// coordinate. strict_bad: in strict mode, whether agent `a`'s contact force is
// NaN as in MPE — a collider c != self at d2 = 0 (MPE: delta / dist = 0 / 0)
// or any agent of the env at a non-finite position (MPE evaluates every pair,
// so one NaN agent reaches every agent's force). `pos_of(c)` gives collider
// c's position (agents first); O(M) per agent — strict mode is a checking
// mode, the default path never runs it.
constexpr uint8_t kDegCoincident = 1, kDegNonfinite = 2;   // gsm.h GSM_DEGENERATE_*
__device__ __forceinline__ bool nonfinite2(float2 a) {
    return !(__builtin_isfinite(a.x) && __builtin_isfinite(a.y));
}
template <typename PosOf>
__device__ __forceinline__ bool strict_bad(int self, float2 a, int N, int M, PosOf pos_of) {
    bool bad = nonfinite2(a);
    for (int c = 0; c < M; ++c) {
        const float2 q = pos_of(c);
        const float dx = a.x - q.x, dy = a.y - q.y;
        bad |= (c != self && dx * dx + dy * dy == 0.0f) || (c < N && nonfinite2(q));
    }
    return bad;
}

// MPE get_collision_force magnitude / d for one pair inside the cutoff:
//   F/d = c * k * softplus(-(d - dmin)/k) / d.
// Written as pen = max(D, 0) + k*log1p(exp(-|D|/k)), D = dmin - d: the
// dominant term max(D, 0) is exact and the transcendental part is a
// correction < k*ln2, so the hardware v_exp/v_log/v_rcp/v_sqrt (<= 1 ulp)
// keep |F| within ~2e-7 relative (positions/velocities stay within the 1e-6
// parity bar). The raw base-2 v_exp_f32 / v_log_f32 are used
// directly: 1 + e lies in (1, 2], so the library log's denormal scaling
// (a dozen VALU per pair) is never needed, and an exp2 underflow is e = 0.
template <typename Params>   // DevParams or its kernarg view (late_params)
__device__ __forceinline__ float contact_scale(const Params &p, float d2, float dmin) {
    constexpr float kLog2e = 1.44269504088896341f, kLn2 = 0.693147180559945309f;
    const float d = __builtin_amdgcn_sqrtf(d2);
    const float D = dmin - d;
    const float e = __builtin_amdgcn_exp2f(-fabsf(D) * (p.inv_k * kLog2e));   // in [0, 1]
    const float pen = fmaxf(D, 0.0f) + (p.k * kLn2) * __builtin_amdgcn_logf(1.0f + e);
    return p.cf * pen * __builtin_amdgcn_rcpf(d);
}

// ---- fused rollout hand-offs (gsm_seg_kernels.hip / gsm_tile_kernels.hip)
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr uint64_t kRollSpinTicks = 20000000ull;   // s_memrealtime ticks (100 MHz): 0.2 s

// Every granule access of the rollouts' hand-offs goes through gran_ld /
// gran_st (relaxed agent-scope: write-through, L1 bypassed). Several are
// issued unconditionally at clamped addresses (a load under a branch makes
// the compiler drain the memory counter at every later wait), so a wrong
// clamp reads outside the allocation — once past its end into another
// page (a GPU memory fault, round 4), once inside its page slack, unnoticed.
// The checked build (-DGSM_CHECKED, tools/build_variant.sh; never the
// product library) tests every such address against the slot's allocation
// [roll.gran, roll.gran_end): one outside sets the sticky status word to
// kStatusOutOfBounds and is redirected to the first granule, so the tests
// (which fail on any non-zero status) name it without faulting the GPU.
constexpr uint32_t kStatusOutOfBounds = 6u;
#ifdef GSM_CHECKED
__device__ __forceinline__ const uint64_t *gran_chk(const uint64_t *g) {
    KernargParams &q = late_params();
    if (__builtin_expect(g < q.roll.gran || g >= q.roll.gran_end, 0)) {
        __hip_atomic_store((gu32 *)q.roll.status, kStatusOutOfBounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return q.roll.gran;
    }
    return g;
}
// any other hand-off word of the slot's allocation (chunk sums, pacing
// counters, the eager step's epoch replicas): the same test
template <typename T>
__device__ __forceinline__ T *hand_chk(T *g) {
    KernargParams &q = late_params();
    const char *c = (const char *)g;
    if (__builtin_expect(c < (const char *)q.roll.gran || c + sizeof(T) > (const char *)q.roll.gran_end, 0)) {
        __hip_atomic_store((gu32 *)q.roll.status, kStatusOutOfBounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return (T *)q.roll.gran;
    }
    return g;
}
#else
__device__ __forceinline__ const uint64_t *gran_chk(const uint64_t *g) { return g; }
template <typename T>
__device__ __forceinline__ T *hand_chk(T *g) { return g; }
#endif
__device__ __forceinline__ uint64_t gran_ld(const uint64_t *g) {
    return __hip_atomic_load((const gu64 *)gran_chk(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_st(uint64_t *g, uint64_t v) {
    __hip_atomic_store((gu64 *)gran_chk(g), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one granule, polled until its tag matches (cold path)
__device__ __forceinline__ uint64_t roll_wait(const uint64_t *g, uint32_t tag, uint32_t *status) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint64_t x = gran_ld(g);
        if ((uint32_t)(x >> 32) == tag) return x;
        if (__hip_atomic_load((gu32 *)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
            __builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks) {
            __hip_atomic_store((gu32 *)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return (uint64_t)tag << 32;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Environment._set_action + apply_action_force of a rollout step: agent index
// `a` of action row `row` (roll.actions + row * stride), runtime format.
template <typename Params>   // DevParams or its kernarg view (late_params)
__device__ __forceinline__ float2 roll_action_force(const Params &p, int row, int64_t a) {
    const char *base = p.roll.actions + (int64_t)row * p.roll.stride;
    float ux, uy;
    if (p.action_fmt == 0) {
        const float *q = (const float *)base + a * 5;
        ux = q[1] - q[2];
        uy = q[3] - q[4];
    } else if (p.action_fmt == 1) {
        const int k = ((const int32_t *)base)[a];
        ux = (float)(k == 1) - (float)(k == 2);
        uy = (float)(k == 3) - (float)(k == 4);
    } else {
        const float2 q = ((const float2 *)base)[a];
        ux = q.x;
        uy = q.y;
    }
    return make_float2(ux * p.sens, uy * p.sens);
}

// ---- granule tags of the rollouts' CSR hand-offs
// A granule is 8 bytes {tag32 << 32 | value32}, stored and loaded with relaxed
// agent-scope atomics (write-through, no fence). tag32 = epoch20 << 12 |
// (step + 1): the launch epoch (20 bits, DevParams::Roll::epoch: assigned by
// the host to every launch from one process-wide counter) and the step within
// the launch (K <= kRollMaxSteps). No granule left in memory by another
// launch — of this graph, or of a graph freed before this one was allocated
// at the same address — carries a tag of this launch until 2^20 launches
// later (observed before per-launch epochs: a memset / store-initialised
// allocation still showed an agent-scope load the granules of the previous
// graph's last replay). Tag 0 is never valid (step + 1 >= 1), so zeroed
// memory never matches.
__device__ __forceinline__ uint32_t roll_epoch_tag(uint32_t epoch) { return (epoch & 0xfffffu) << 12; }

// ---- per-wave CSR hand-off of the one-env-per-wave rollouts
// (the ragged rollout, gsm_ragged_kernels.hip; `depth` = the lag between a
// step and the packing of its edges, >= 2). The packed CSR offset of env (=
// wave) w at step s is the sum of the edge counts of every wave before it.
// Three levels of tagged granules:
//   agg[s][w]  wave w's edge count at step s, published right after its sweep;
//   grp[s][g]  the sum of agg[s][64g .. 64g+63], published by wave 64g+63 in
//              iteration s + 1;
//   offset     sum of grp[s][g' < w/64] + sum of agg[s][64(w/64) .. w-1],
//              loaded and summed in iteration s + depth, when step s's edges
//              are packed.
// Every granule a wave reads was published at least one iteration before it
// is needed, so no wave normally waits; there are no barriers. A wave waits
// only on waves of lower index (dispatched before it), so the launch always
// progresses; every wait is bounded (kRollSpinTicks, then a sticky status
// word).
struct Xfer {
    uint64_t *agg;      // [K][W]
    uint64_t *grp;      // [K][NG]
    uint32_t *status;
    int W, NG;          // waves of the grid, groups of 64 waves
    uint32_t etag;      // roll_epoch_tag(epoch)
    __device__ __forceinline__ uint32_t tag(int s) const { return etag | (uint32_t)(s + 1); }
};
__device__ __forceinline__ uint64_t xfer_ld(const uint64_t *g) { return gran_ld(g); }
__device__ __forceinline__ void xfer_st(uint64_t *g, uint32_t tag, uint32_t v) { gran_st(g, (uint64_t)tag << 32 | v); }
// The value of a granule loaded as x from g on lanes `act`, once its tag is
// `tag` (re-polled until it is: the cold path); 0 on other lanes.
__device__ __forceinline__ uint32_t xfer_settle(uint64_t x, const uint64_t *g, bool act, uint32_t tag,
                                                uint32_t *status) {
    bool bad = act && (uint32_t)(x >> 32) != tag;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        do {
            __builtin_amdgcn_s_sleep(2);
            if (bad) x = xfer_ld(g);
            bad = act && (uint32_t)(x >> 32) != tag;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks ||
                __hip_atomic_load((gu32 *)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                __hip_atomic_store((gu32 *)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bad = false;
            }
        } while (__builtin_amdgcn_ballot_w64(bad) != 0);
    }
    return act ? (uint32_t)x : 0u;
}
// Granules wave w needs for step s's offset, loaded at clamped (always valid)
// addresses with the lane predicates applied when they are settled.
struct XferOff {
    uint64_t a, g0, g1;
};
__device__ __forceinline__ XferOff xfer_off_load(const Xfer &x, int s, int w, int lane) {
    const int g = w >> 6, r = w & 63;
    const uint64_t *ag = x.agg + (int64_t)s * x.W + (g << 6);
    const uint64_t *gg = x.grp + (int64_t)s * x.NG;
    const int gl = g > 0 ? g - 1 : 0;
    XferOff o;
    o.a = xfer_ld(ag + min(lane, r > 0 ? r - 1 : 0));
    o.g0 = xfer_ld(gg + min(lane, gl));
    o.g1 = g > kWave ? xfer_ld(gg + min(lane + kWave, gl)) : 0ull;   // wave-uniform branch
    return o;
}
// The same loads with none under a branch (g1 always loaded): for a loop
// that keeps them in flight across other loads' waits
__device__ __forceinline__ XferOff xfer_off_load_all(const Xfer &x, int s, int w, int lane) {
    const int g = w >> 6, r = w & 63;
    const uint64_t *ag = x.agg + (int64_t)s * x.W + (g << 6);
    const uint64_t *gg = x.grp + (int64_t)s * x.NG;
    const int gl = g > 0 ? g - 1 : 0;
    XferOff o;
    o.a = xfer_ld(ag + min(lane, r > 0 ? r - 1 : 0));
    o.g0 = xfer_ld(gg + min(lane, gl));
    o.g1 = xfer_ld(gg + min(lane + kWave, gl));
    return o;
}
__device__ __forceinline__ int xfer_off_settle(const Xfer &x, const XferOff &o, int s, int w, int lane) {
    const int g = w >> 6, r = w & 63, gl = g > 0 ? g - 1 : 0;
    const uint32_t tag = x.tag(s);
    const uint64_t *ag = x.agg + (int64_t)s * x.W + (g << 6);
    const uint64_t *gg = x.grp + (int64_t)s * x.NG;
    uint32_t v = xfer_settle(o.a, ag + min(lane, r > 0 ? r - 1 : 0), lane < r, tag, x.status);
    v += xfer_settle(o.g0, gg + min(lane, gl), lane < g, tag, x.status);
    if (g > kWave) v += xfer_settle(o.g1, gg + min(lane + kWave, gl), lane + kWave < g, tag, x.status);
    return wave_total((int)v);
}
// Group sum of step s by the group's last wave (w & 63 == 63): the other 63
// members' granules plus its own count. The load is issued by every wave (a
// load under a branch drains the memory counter at later waits); its index
// stays inside step s's row also for a wave of a partial last group, whose
// result is never used (the checked build caught the unclamped form reading
// past the allocation at the last step of a 16-wave grid).
// Only the group's last wave uses the result: every other wave's lanes all
// load one granule (one memory request instead of eight: the granules are
// uncached, so each request goes to HBM).
__device__ __forceinline__ const uint64_t *xfer_grp_addr(const Xfer &x, int s, int w, int lane) {
    return x.agg + (int64_t)s * x.W + min((w & ~63) + min(lane, (w & 63) == 63 ? 62 : 0), x.W - 1);
}
__device__ __forceinline__ uint64_t xfer_grp_load(const Xfer &x, int s, int w, int lane) {
    return xfer_ld(xfer_grp_addr(x, s, w, lane));
}
__device__ __forceinline__ void xfer_grp_publish(const Xfer &x, uint64_t l, int s, int w, int lane, int own) {
    const uint32_t tag = x.tag(s);
    const uint32_t v = xfer_settle(l, xfer_grp_addr(x, s, w, lane), lane < 63, tag, x.status);
    const int sum = wave_total((int)v) + own;
    if (lane == 0) xfer_st(x.grp + (int64_t)s * x.NG + (w >> 6), tag, (uint32_t)sum);
}

// ---- pacing of the rollouts (round 5; gsm_roll_seg_kernel, gsm_roll_tile_kernel)
// A SIMD issues its ready waves oldest first below the user priority
// (s_setprio), and a CU holds several workgroups of a rollout (eight at H),
// dispatched one residency rank at a time (blockIdx / 256 at H). Measured per
// CU, the rank-0 workgroup finished a 20-step launch at 109 us and rank 7 at
// 210 us, in exact rank order on every CU, and the same without any hand-off
// (profiles/r5_pace): the last ranks' final steps run on a CU already half
// empty. Some order between ranks helps the look-back — a workgroup finds
// the inclusive prefixes of the rank before it already published — but not
// twelve steps of it. So each workgroup counts its finished steps into its
// CU's counter (one atomic add per step, the counter loaded back beside the
// next step's look-back loads; its rank = the arrivals before its own, read
// at entry) and sets its waves' priority from its own
// steps against a target: the CU's mean plus (c - rank) x q / 4 steps,
// c = (arrivals - 1) / 2 — ahead of the target by half a step or more 0,
// behind by as much 2, else 1. Priority only orders issue: outputs are
// unchanged. A counter is one 32-bit word: arrivals in the top 8 bits, steps
// in the low 24 (8 workgroups x 4094 steps < 2^24).
constexpr uint32_t kPaceArrive = 1u << 24;
__device__ __forceinline__ uint32_t pace_key() {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);          // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;   // XCC_ID
    return (xcc << 8 | ((hw >> 13) & 7u) << 5 | ((hw >> 12) & 1u) << 4 | ((hw >> 8) & 15u)) * kPaceStride;
}
// the level from the CU counter as loaded after this workgroup's `done`-th
// step was added to it
// (diagnostic variants: -DGSM_PACE_T=t moves the thresholds to t/8 of a step,
// -DGSM_PACE_LEVELS=4 adds a fourth level, behind by less than the threshold)
#ifndef GSM_PACE_T
#define GSM_PACE_T 4
#endif
#ifndef GSM_PACE_LEVELS
#define GSM_PACE_LEVELS 3
#endif
__device__ __forceinline__ int pace_level(uint32_t fv, int done, int rank, int q) {
    const int arr = (int)(fv >> 24), tot = (int)(fv & (kPaceArrive - 1));
    // 8 x arrivals x (own steps - the CU's mean - (c - rank) x q / 4)
    const int x = 8 * (done * arr - tot) - arr * (arr - 1 - 2 * rank) * q;
    if constexpr (GSM_PACE_LEVELS == 4)
        return x >= GSM_PACE_T * arr ? 0 : x >= 0 ? 1 : x > -GSM_PACE_T * arr ? 2 : 3;
    return x >= GSM_PACE_T * arr ? 0 : x <= -GSM_PACE_T * arr ? 2 : 1;
}
__device__ __forceinline__ void pace_set(int lvl) {   // lvl wave-uniform
    if (lvl == 0)
        __builtin_amdgcn_s_setprio(0);
    else if (lvl == 1)
        __builtin_amdgcn_s_setprio(1);
    else if (GSM_PACE_LEVELS == 3 || lvl == 2)
        __builtin_amdgcn_s_setprio(2);
    else
        __builtin_amdgcn_s_setprio(3);
}

// the priority of a rollout's first iterations, before the pace levels take
// over (gsm_roll_seg_kernel; -DGSM_START_PRIO=0: none, the A/B baseline)
#ifndef GSM_START_PRIO
#define GSM_START_PRIO 1
#endif
template <int kLvl>
__device__ __forceinline__ void start_prio() {
    if constexpr (GSM_START_PRIO != 0) __builtin_amdgcn_s_setprio(kLvl);
}

// ---- one-hop CSR prefix of the one-env-per-wave segmented rollout (round 5)
// The packed offset of workgroup w's edges of step s is the sum of the edge
// counts of every workgroup before it. Two kinds of words per step:
//   agg[s][w]  workgroup w's count, a tagged granule;
//   sum[s][c]  chunk c = workgroups [64c, 64c + 64): {arrivals32, sum32}, formed
//              by one agent-scope atomic add (1 << 32 | count) of each member
//              (the chunk words `cs` u64 apart: spread over memory lines).
// offset(w) = sum[s][c'] over the chunks c' < w / 64 (each complete: arrivals
// 64) + agg[s][w'] over w's chunk-mates w' < w: ONE load per lane and no
// chain. (A decoupled look-back resolves through the predecessors' inclusive
// prefixes, each published after its own walk: workgroups that reach a step
// together wait on each other hop by hop, and only a skew of whole steps
// between the CU's dispatch ranks hid that — DESIGN.md §4.) The rollout reads
// a step's words two iterations after publishing them, so they are complete
// at the first load unless a workgroup trails by two steps (then re-polled).
// The sum words carry no tag: each launch uses one half of a double buffer
// and zeroes the other, which the slot's next launch uses.
__device__ __forceinline__ void prefix_publish(uint64_t *agg_s, uint64_t *sum_s, int cs, int w, uint32_t tag,
                                               uint32_t v) {
    gran_st(agg_s + w, (uint64_t)tag << 32 | v);
    (void)__hip_atomic_fetch_add((gu64 *)hand_chk(sum_s + (int64_t)(w / kPrefixChunk) * cs), 1ull << 32 | v,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Workgroup w's exclusive prefix of step s (ONE wave; wave-uniform result).
// Lane l loads chunk sum l (l < w / 64) and chunk-mate 64(w / 64) + l's
// aggregate (l < w % 64), at clamped addresses inside the step's rows; a word
// not yet complete is re-polled (bounded: kRollSpinTicks, then the sticky
// status word and a zero contribution).
__device__ __forceinline__ int roll_prefix(const uint64_t *agg_s, const uint64_t *sum_s, int cs, uint32_t tag,
                                           uint32_t *status, int lane) {
    int w = (int)blockIdx.x;
    asm volatile("" : "+s"(w));   // no window predicates hoisted into a rollout's loop (SGPR pairs)
    const int c = w / kPrefixChunk, r = w % kPrefixChunk;
    const uint64_t *sp = hand_chk(sum_s + (int64_t)min(lane, c > 0 ? c - 1 : 0) * cs);
    const uint64_t *ap = agg_s + c * kPrefixChunk + min(lane, r > 0 ? r - 1 : 0);
    uint64_t sv = __hip_atomic_load((const gu64 *)sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t av = gran_ld(ap);
    const bool use_s = lane < c, use_a = lane < r;
    bool sb = use_s && (uint32_t)(sv >> 32) != (uint32_t)kPrefixChunk;
    bool ab = use_a && (uint32_t)(av >> 32) != tag;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(sb || ab) != 0, 0)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        do {
            __builtin_amdgcn_s_sleep(8);
            if (sb) sv = __hip_atomic_load((const gu64 *)sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (ab) av = gran_ld(ap);
            sb = use_s && (uint32_t)(sv >> 32) != (uint32_t)kPrefixChunk;
            ab = use_a && (uint32_t)(av >> 32) != tag;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks ||
                __hip_atomic_load((gu32 *)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                __hip_atomic_store((gu32 *)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sb = ab = false;
            }
        } while (__builtin_amdgcn_ballot_w64(sb || ab) != 0);
    }
    return wave_total((int)((use_s ? (uint32_t)sv : 0u) + (use_a ? (uint32_t)av : 0u)));
}

// Decoupled look-back over the preceding workgroups (ONE wave; wave-uniform
// result): windows of 64 predecessors, nearest first; the nearest one whose
// inclusive prefix is published ends the walk (its inclusive + the aggregates
// of those in between), otherwise the window's aggregates are added and the
// walk moves on. Aggregates were published an iteration earlier, so the walk
// never waits on an inclusive prefix; an aggregate read early is re-polled.
// (Reading several windows per round before using the first, so a long walk
// pays one load latency per round, was measured slower at H — four windows
// every round: 10.2 vs 9.8 us per step; eight per round after a first single
// window: 8.6 vs 8.4 — and for the one-launch eager step)
__device__ __forceinline__ int roll_lookback(const uint64_t *agg_k, const uint64_t *inc_k, uint32_t tag,
                                             uint32_t *status, int lane) {
    int acc = 0;
    int first = (int)blockIdx.x;
    asm volatile("" : "+s"(first));   // no window predicates hoisted into a rollout's loop (SGPR pairs)
    for (int hi = first; hi > 0; hi -= kWave) {
        const int idx = hi - 1 - lane;                      // lane 0 = nearest predecessor
        const int ci = idx >= 0 ? idx : 0;
        const bool valid = idx >= 0;
        const uint64_t xi = gran_ld(inc_k + ci);
        uint64_t a = gran_ld(agg_k + ci);
        const uint64_t have = __ballot(valid && (uint32_t)(xi >> 32) == tag);
        const int j = have ? __builtin_ctzll(have) : kWave;   // wave-uniform
        // aggregates of lanes < j (all valid lanes when no inclusive was found)
        const bool need = valid && lane < j;
        if (need && (uint32_t)(a >> 32) != tag) a = roll_wait(agg_k + ci, tag, status);
        int v = need ? (int)(uint32_t)a : 0;
        if (lane == j) v = (int)(uint32_t)xi;
        acc += wave_total(v);
        if (have) return acc;
    }
    return acc;
}

}  // namespace gsm
