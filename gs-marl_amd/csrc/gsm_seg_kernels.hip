// gsm_seg_kernels.hip — segmented kernels for envs with M = N + No <= 64
// colliders: the headline 24-agent navigation path and every BASELINE config
// except the 96-agent one.
//
// Lane layout. A wave holds G = min(64 / M, 16) envs ("segments" of M
// lanes); lane (seg, m) owns row m of its env in compact collider order
// (m < N: agent m = entity m; m >= N: obstacle m-N = entity N+m). The G envs'
// positions live in LDS.
//
// Observation pass (post-physics positions). The radius adjacency is
// symmetric, so a wave-uniform sweep over the N *agent* columns j suffices:
//   * the ballot over lanes of  rad(m, j) = 0 < d2 <= R2  is agent row j's
//     full mask; lane j captures its segment's slice (v_writelane when G = 1);
//   * obstacle rows set their agent bits per lane; their obstacle-obstacle
//     bits are static within an episode and are carried in the stored row
//     masks (a reset or an observe recomputes them with a full sweep);
//   * the ballot of  d2 < dmin2  gives agent j's collision count (popcount),
//   * the ballot of  0 < d2 < (dmin + cutoff)^2  gives agent j's contact
//     candidates, stored for the NEXT step's force pass (same positions).
// All predicates use d2 = dx*dx + dy*dy without FMA (bit-exact contract).
//
// Physics pass (pre-step positions): agent lane i sums the contact force of
// its stored candidates only (ascending collider index), then integrates.
//
// Emission (gsm_emit_seg_kernel): row masks -> per-row counts in entity order
// (agent rows, goal rows, obstacle rows) -> lane scan -> each lane writes its
// row (agent columns, own goal, obstacle columns); agent lanes also write the
// goal rows. CSR offsets come from the per-workgroup sums of the step kernel:
// no atomics, no inter-workgroup waiting, deterministic. In a graph chain the
// same emission runs at the top of the NEXT step kernel (kLag: the previous
// step's positions and masks are that kernel's inputs; block_emit), so a
// step costs one launch.
//
// With one env per wave (G = 1, e.g. 24 agents) the segment collectives are
// DPP wave scans/reductions and per-env scalars are scalar loads.
#include <type_traits>

#include "gsm_device.h"

namespace gsm {

template <typename T>
__device__ __forceinline__ T seg_scan(T v, int m) {   // inclusive scan within a segment
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const T u = __shfl_up(v, o);
        if (m >= o) v += u;
    }
    return v;
}

__device__ __forceinline__ int row_entity(int m, int N) { return m < N ? m : N + m; }

template <int kN, int kNo>
constexpr int envs_per_wave() {
    return kN > 0 ? ((kWave / (kN + kNo)) > kMaxSegEnvsPerWave ? kMaxSegEnvsPerWave : kWave / (kN + kNo))
                  : 0;
}

// compile-time shape when kN > 0, runtime otherwise
template <int kN, int kNo>
struct Shape {
    int N, No, M, E, G;
    __device__ __forceinline__ explicit Shape(const DevParams &p) {
        if constexpr (kN > 0) {
            N = kN;
            No = kNo;
            M = kN + kNo;
            E = 2 * kN + kNo;
            G = envs_per_wave<kN, kNo>();
        } else {
            N = p.N;
            No = p.No;
            M = p.N + p.No;
            E = p.E;
            G = p.G;
        }
    }
};

struct Lane {
    int lane, seg, m, b, base, wave;    // base = first lane of the segment
    bool live, agent;
};

template <int kN, int kNo>
__device__ __forceinline__ Lane seg_lane(const DevParams &p, const Shape<kN, kNo> &s) {
    Lane L;
    L.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    L.lane = threadIdx.x & 63;
    if constexpr (envs_per_wave<kN, kNo>() == 1) {
        L.seg = 0;
        L.base = 0;
        L.m = L.lane;
        L.b = blockIdx.x * kWavesPerBlock + L.wave;          // wave-uniform
        L.live = L.lane < s.M && L.b < p.B;
    } else {
        L.seg = L.lane / s.M;
        L.base = L.seg * s.M;
        L.m = L.lane - L.base;
        L.b = (blockIdx.x * kWavesPerBlock + L.wave) * s.G + L.seg;
        L.live = L.seg < s.G && L.b < p.B;
    }
    L.agent = L.live && L.m < s.N;
    return L;
}

// a wave-uniform 64-bit ballot restricted to this lane's segment, delivered
// to the lane whose row index is j (other lanes keep `old`)
template <int kG>
__device__ __forceinline__ uint64_t capture(uint64_t ballot, int j, const Lane &L, uint64_t segmask,
                                            uint64_t old) {
    if constexpr (kG == 1) {
        const uint64_t v = ballot & segmask;
        const uint32_t lo = writelane_u32((uint32_t)v, (uint32_t)j, (uint32_t)old);
        const uint32_t hi = writelane_u32((uint32_t)(v >> 32), (uint32_t)j, (uint32_t)(old >> 32));
        return ((uint64_t)hi << 32) | lo;
    } else {
        const uint64_t mine = (ballot >> L.base) & segmask;
        return L.m == j ? mine : old;
    }
}
template <int kG>
__device__ __forceinline__ int capture_count(uint64_t ballot, int j, const Lane &L, uint64_t segmask,
                                             int old) {
    if constexpr (kG == 1) {
        return (int)writelane_u32((uint32_t)__popcll(ballot & segmask), (uint32_t)j, (uint32_t)old);
    } else {
        const int mine = __popcll((ballot >> L.base) & segmask);
        return L.m == j ? mine : old;
    }
}

// sum over the lanes of this lane's segment (every lane of the segment gets it)
template <int kG, typename T>
__device__ __forceinline__ T seg_total(T v, const Lane &L, int M) {
    if constexpr (kG == 1) {
        return wave_total(v);
    } else {
        return __shfl(seg_scan(v, L.m), L.base + M - 1);
    }
}

// agent-column bits of one row: 32 bits suffice when N <= 32 is known
template <int kN>
using OwnBits = typename std::conditional<(kN > 0 && kN <= 32), uint32_t, uint64_t>::type;

// low 16 bits of a, low 16 bits of b above them (one s_pack_ll_b32_b16)
__device__ __forceinline__ uint32_t pack_lo16(uint64_t a, uint64_t b) {
    uint32_t r;
    asm("s_pack_ll_b32_b16 %0, %1, %2" : "=s"(r) : "s"((uint32_t)a), "s"((uint32_t)b));
    return r;
}

// One env per wave (32 < M <= 64, compile-time even N <= 32): the sweep with
// the fewest instructions per agent column j.
//   * the agent positions are re-staged as column pairs [x_j x_j+1 y_j y_j+1]
//     (s_xy, 16 B per pair) so one ds_read_b128 and five packed-f32 VALU give
//     the squared distances of two columns; the next group's pairs are read
//     while this group is processed;
//   * lanes >= M carry a far-away position, so no ballot needs a segment mask;
//   * two ballots on plain float compares: rad' (d2 <= R2) and near
//     (d2 < cut2: contact candidates plus the self and coincident pairs);
//     three v_writelanes (low words; the two high words packed when M <= 48);
//   * obstacle rows accumulate their agent bits with one v_addc per column
//     (column order reversed, so one v_bfrev at the end);
//   * the walk over each agent row's near bits counts collisions
//     (d2 < dmin2 implies d2 < cut2) and finds coincident pairs (d2 = 0);
//     self bits are dropped, and a wave holding a coincident pair (never
//     seen in practice) recomputes its rows with the exact 0 < d2 <= R2;
//   * kForce (fused rollout): the same walk also forms the NEXT step's
//     contact forces — the candidates are exactly these near bits at these
//     positions (d2 != 0), so *force = finit() (the next step's action force,
//     formed only here so it holds no registers during the column loop) plus
//     the contact terms in ascending collider order, the operations and order
//     of the step kernel's force pass (bit-identical).
template <int kN, int kNo, bool kForce = false, typename FInit = int, typename Params = DevParams>
__device__ __forceinline__ void obs_sweep_g1(const Params &p, const Lane &L, const float2 *sp, float *s_xy,
                                             float2 pm, bool full, uint64_t oo, uint64_t &row, uint64_t &cand,
                                             int &ccnt, bool &coinc, float2 *force = nullptr, FInit finit = 0) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    constexpr int N = kN, M = kN + kNo;
    static_assert(M > 32 && M <= 64 && N <= 32 && N % 2 == 0, "one env per wave, agent bits in the low word");
    constexpr bool kPack = M <= 48;
    constexpr uint64_t abits = (1ull << N) - 1;
    const bool obst = L.live && L.m >= N;
    if (L.agent) {
        const int at = (L.m >> 1) * 4 + (L.m & 1);
        s_xy[at] = pm.x;
        s_xy[at + 2] = pm.y;
    }
    if (!L.live) pm = make_float2(1.0e18f, 1.0e18f);        // d2 ~ 1e36: every predicate false
    const float R2 = p.R2, cut2 = obst ? p.cut2_ao : p.cut2_aa;
    const uint64_t r0 = (!full && obst) ? (oo & ~abits) : 0ull;
    uint32_t r_lo = (uint32_t)r0, r_hi = (uint32_t)(r0 >> 32);
    uint32_t c_lo = 0, c_hi = 0, hi = kPack ? (r_hi & 0xffffu) : 0u;
    uint32_t own = 0;                                       // bit N-1-j = rad'(lane, j)
    wave_sync();
    auto column = [&](int j, float d2) {
        const uint64_t b_rad = __ballot(d2 <= R2);
        const uint64_t b_near = __ballot(d2 < cut2);
        own = shl1_add_lane(own, b_rad);
        r_lo = writelane_u32((uint32_t)b_rad, (uint32_t)j, r_lo);
        c_lo = writelane_u32((uint32_t)b_near, (uint32_t)j, c_lo);
        if constexpr (kPack) {
            hi = writelane_u32(pack_lo16(b_rad >> 32, b_near >> 32), (uint32_t)j, hi);
        } else {
            r_hi = writelane_u32((uint32_t)(b_rad >> 32), (uint32_t)j, r_hi);
            c_hi = writelane_u32((uint32_t)(b_near >> 32), (uint32_t)j, c_hi);
        }
    };
    const f32x2 px = {pm.x, pm.x}, py = {pm.y, pm.y};
    auto pair = [&](int j, float4 Q) {
        const f32x2 dx = px - (f32x2){Q.x, Q.y};
        const f32x2 dy = py - (f32x2){Q.z, Q.w};
        const f32x2 d2 = dx * dx + dy * dy;
        column(j, d2.x);
        column(j + 1, d2.y);
    };
    // pairs in groups of kU, the next group read while this one is processed
    constexpr int kP = N / 2, kU = 2;
    const float4 *xy4 = (const float4 *)s_xy;
    float4 qn[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) qn[u] = xy4[u < kP ? u : kP - 1];
    for (int g = 0; g < kP; g += kU) {
        float4 q[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) q[u] = qn[u];
        if (g + kU < kP) {
#pragma unroll
            for (int u = 0; u < kU; ++u) qn[u] = xy4[g + kU + u < kP ? g + kU + u : kP - 1];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (kP % kU == 0 || g + u < kP) pair(2 * (g + u), q[u]);
    }
    own = __builtin_bitreverse32(own) >> (32 - N);
    if constexpr (kPack) {
        r_hi = hi & 0xffffu;
        c_hi = hi >> 16;
    }
    uint64_t r = ((uint64_t)r_hi << 32) | r_lo;
    const uint64_t near = ((uint64_t)c_hi << 32) | c_lo;
    if (obst) r = (r & ~abits) | own;                       // agent bits of obstacle rows
    if (L.agent) r &= ~(1ull << L.m);                      // self
    if (full) {
        // obstacle columns: obstacle-obstacle bits (the agent-obstacle bits
        // of agent rows were captured above)
#pragma unroll 2
        for (int k = N; k < M; ++k) {
            const float2 q = sp[N + k];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            const float d2 = dx * dx + dy * dy;
            if (obst && d2 > 0.0f && d2 <= p.R2) r |= 1ull << k;
        }
    }
    // collisions and contact candidates of agent rows from the near bits
    int cc = 0;
    uint64_t c = 0;
    bool coincident = false;
    if (L.agent) {
        uint64_t w = near & ~(1ull << L.m);
        c = w;
        float Fx = 0.0f, Fy = 0.0f;
        if constexpr (kForce) {
            const float2 f0 = finit();
            Fx = f0.x;
            Fy = f0.y;
        }
        const float dmin_aa = p.dmin_aa, dmin_ao = p.dmin_ao;   // both read before the walk
        while (w) {
            const int k = __builtin_ctzll(w);
            w &= w - 1;
            const float2 q = sp[k < N ? k : N + k];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            const float d2 = dx * dx + dy * dy;
            cc += d2 < (k < N ? p.dmin2_aa : p.dmin2_ao) ? 1 : 0;
            if (d2 == 0.0f) {
                c &= ~(1ull << k);
                coincident = true;
            } else if (kForce) {
                const float f = contact_scale(p, d2, k < N ? dmin_aa : dmin_ao);
                Fx += f * dx;
                Fy += f * dy;
            }
        }
        if constexpr (kForce) *force = make_float2(Fx, Fy);
    }
    coinc = __any(coincident);   // the env (= the wave) holds a coincident pair (App. A S16)
    if (__builtin_expect(coinc, 0)) {
        // exact agent-column bits of every row (and obstacle columns of agent
        // rows): rad' also holds coincident pairs
        uint64_t ex = 0;
        for (int k = 0; k < (L.agent ? M : N); ++k) {
            const float2 q = sp[k < N ? k : N + k];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            const float d2 = dx * dx + dy * dy;
            if (d2 > 0.0f && d2 <= p.R2) ex |= 1ull << k;
        }
        if (L.agent) r = ex;
        else if (obst) r = (r & ~abits) | ex;
    }
    row = r;
    cand = c;
    ccnt = cc;
}

// Observation sweep (file header). row/cand/ccnt are per lane: row = radius
// row mask (compact bits), cand = contact candidates (agent lanes),
// ccnt = collisions of agent lanes (self excluded), coinc = the lane's env
// holds a coincident pair with an agent (d2 = 0, App. A S16). With full =
// false the obstacle-obstacle bits are taken from `oo` (the cached masks).
// kForce: see obs_sweep_g1 (only with that sweep: sweep_walks_near).
template <int kN, int kNo>
constexpr bool sweep_walks_near(int G) {
    return G == 1 && kN > 0 && kN <= 32 && kN % 2 == 0 && kN + kNo > 32;
}
// Params: DevParams, or its kernarg view (late_params: the constants are then
// scalar loads at the sweep, not SGPRs held across a rollout's loop)
template <int kN, int kNo, int kG, bool kForce = false, typename FInit = int, typename Params = DevParams>
__device__ __forceinline__ void obs_sweep(const Params &p, const Shape<kN, kNo> &s, const Lane &L,
                                          const float2 *sp, float *s_xy, float2 pm, bool full, uint64_t oo,
                                          uint64_t &row, uint64_t &cand, int &ccnt, bool &coinc,
                                          float2 *force = nullptr, FInit finit = 0) {
    static_assert(!kForce || sweep_walks_near<kN, kNo>(kG), "contact forces only in the near-bit walk");
    if constexpr (sweep_walks_near<kN, kNo>(kG)) {
        // (a variant forming each row's bits by VGPR integer arithmetic, off the
        // scalar issue path as the ragged sweep does, measured slower here:
        // 10.2 vs 9.0 us per step at H)
        obs_sweep_g1<kN, kNo, kForce>(p, L, sp, s_xy, pm, full, oo, row, cand, ccnt, coinc, force, finit);
        return;
    }
    const int N = s.N, M = s.M;
    const uint64_t segmask = M >= 64 ? ~0ull : ((1ull << M) - 1);
    const uint64_t abits = N >= 64 ? ~0ull : ((1ull << N) - 1);
    const bool obst = L.m >= N;
    (void)abits;
    const float dmin2 = obst ? p.dmin2_ao : p.dmin2_aa;   // lane m vs an agent column
    // For a non-negative float d2 the bit pattern is monotone, so with
    // t = bits(d2) - 1 (d2 = +0 wraps to 0xffffffff):
    //   0 < d2 <= R2    <=>  t <u bits(R2)
    //   0 < d2 < cut2   <=>  t <u bits(cut2) - 1      (same predicates, one compare each)
    const uint32_t r2b = __float_as_uint(p.R2);
    const uint32_t cutb = __float_as_uint(obst ? p.cut2_ao : p.cut2_aa) - 1u;
    uint64_t r = (!full && obst) ? (oo & segmask & ~abits) : 0ull;
    uint64_t c = 0;
    OwnBits<kN> own = 0;                                    // per-lane agent bits (obstacle rows)
    int cc = 0;
    // lanes at d2 = 0 from an agent column other than their own row (wave-
    // uniform, scalar ops only): b_col holds d2 < dmin2 (self and coincident
    // pairs included), b_cand 0 < d2 < cut2 with cut2 > dmin2, so
    // b_col & ~b_cand is exactly d2 = 0; the self lanes of column j are the
    // segments' lanes j
    uint64_t zero = 0, selves = 0;
    for (int g = 0; g < (kG == 1 ? 1 : s.G); ++g) selves |= 1ull << (g * M);
#pragma unroll 4
    for (int j = 0; j < N; ++j) {
        const float2 q = sp[j];
        const float dx = pm.x - q.x, dy = pm.y - q.y;
        const float d2 = dx * dx + dy * dy;
        const uint32_t t = __float_as_uint(d2) - 1u;
        const bool rad = t < r2b;
        const uint64_t b_rad = __ballot(rad);
        const uint64_t b_cand = __ballot(t < cutb);
        const uint64_t b_col = __ballot(d2 < dmin2);
        own |= (OwnBits<kN>)rad << j;
        zero |= b_col & ~b_cand & ~(selves << j);
        r = capture<kG>(b_rad, j, L, segmask, r);
        c = capture<kG>(b_cand, j, L, segmask, c);
        cc = capture_count<kG>(b_col, j, L, segmask, cc);
    }
    if (obst) r |= own;                                     // agent bits of obstacle rows
    if (full) {
        // obstacle columns: obstacle-obstacle bits (the agent-obstacle bits
        // of agent rows were captured above)
        for (int k = N; k < M; ++k) {
            const float2 q = sp[N + k];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            const float d2 = dx * dx + dy * dy;
            if (obst && d2 > 0.0f && d2 <= p.R2) r |= 1ull << k;
        }
    }
    row = r;
    cand = c;
    ccnt = cc - (nonfinite2(pm) ? 0 : 1);                   // the self pair (d2 = 0 < dmin2; NaN if pm is not finite)
    coinc = ((zero >> L.base) & segmask) != 0;
}

// Environment._set_action for a compile-time action format (kFmt < 0: runtime)
template <int kFmt>
__device__ __forceinline__ float2 action_force_t(const DevParams &p, int64_t a) {
    if constexpr (kFmt < 0) {
        return action_force(p, a);
    } else {
        float ux, uy;
        if constexpr (kFmt == 0) {
            const float *q = (const float *)p.actions + a * 5;
            ux = q[1] - q[2];
            uy = q[3] - q[4];
        } else if constexpr (kFmt == 1) {
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
}

// node-feature row of entity e: vx vy px py gx-px gy-py type
__device__ __forceinline__ void store_row(float *nf, float2 v, float2 pos, float2 grel, float type) {
    nf[0] = v.x;
    nf[1] = v.y;
    nf[2] = pos.x;
    nf[3] = pos.y;
    nf[4] = grel.x;
    nf[5] = grel.y;
    nf[6] = type;
}

// Writes the env's edges from the lanes' radius row masks, given the env's
// global offset: row offsets in entity order (agent rows, goal rows,
// obstacle rows) by a segment scan of the row counts, then each lane writes
// its row (agent columns, own goal, obstacle columns); agent lanes also
// write the goal rows.
template <int kN, int kNo, int kG>
__device__ __forceinline__ void emit_rows(const Shape<kN, kNo> &s, const Lane &L, const float2 *s_pos,
                                          uint64_t mask, int64_t env_off, const EdgeSink &out,
                                          bool checked = true) {
    const int N = s.N, E = s.E;
    const int m = L.m;
    const int64_t eb = L.live ? L.b : 0;
    // row offsets in entity order: agent rows, goal rows, obstacle rows
    const int c = __popcll(mask) + (L.agent ? 1 : 0);
    int incl, a_total;
    if constexpr (kG == 1) {
        incl = wave_scan(c);
        a_total = __builtin_amdgcn_readlane(incl, N - 1);
    } else {
        incl = seg_scan(c, m);
        a_total = __shfl(incl, L.base + N - 1);
    }
    // Stores are addressed from a wave-uniform base (the offset of the wave's
    // first env: envs are in order) plus a 32-bit byte offset, the SGPR-base
    // + VGPR-offset store form; edge offsets fit in 32 bits (edge capacity
    // < 2^31, gsm_query_sizes).
    const uint32_t wb_lo = __builtin_amdgcn_readfirstlane((uint32_t)env_off);
    const uint32_t wb_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)env_off >> 32));
    const int64_t wbase = (int64_t)(((uint64_t)wb_hi << 32) | wb_lo);
    uint32_t o = (uint32_t)(env_off - wbase) + (uint32_t)(incl - c + (m >= N ? N : 0));
    const uint32_t goal_at = (uint32_t)(env_off - wbase) + (uint32_t)(a_total + m);
    if (!L.live || wbase >= out.cap) return;

    const float2 pm = s_pos[row_entity(m, N)];
    const uint32_t cap = (uint32_t)(out.cap - wbase);   // redirected outputs may be smaller than the worst case
    char *src = (char *)(out.index + wbase), *dst = (char *)(out.index + out.cap + wbase);
    char *attr = (char *)(out.attr + wbase);
    const int32_t g0 = (int32_t)(eb * E);
    const int32_t gs = g0 + row_entity(m, N);
    const uint64_t agent_bits = N >= 64 ? ~0ull : ((1ull << N) - 1);
    // the same walk with and without the capacity test (an env that fits
    // entirely, the normal case, stores unchecked)
    auto walk = [&](auto chk) {
        constexpr bool kChecked = decltype(chk)::value;
        auto put = [&](uint32_t at, int32_t a, int32_t b, float d) {
            if (!kChecked || at < cap) {
                const uint32_t byte = at << 2;
                *(int32_t *)(src + byte) = a;
                *(int32_t *)(dst + byte) = b;
                *(float *)(attr + byte) = d;
            }
        };
        auto edge_to = [&](int j, int32_t col) {     // lane's row -> entity j (staged position)
            const float2 q = s_pos[j];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            put(o++, gs, col, __builtin_amdgcn_sqrtf(dx * dx + dy * dy));
        };
        if constexpr (kG == 1 && kN > 0 && kN <= 32 && kN + kNo > 32) {
            // one walk over the whole row (its length is the longest row of
            // the wave, not the longest agent part plus the longest obstacle
            // part); an agent row's own-goal edge sits between its agent and
            // obstacle columns, so columns >= N shift by one
            const uint32_t gshift = L.agent ? 1u : 0u;
            if (L.agent) {
                const float2 q = s_pos[N + m];
                const float dx = pm.x - q.x, dy = pm.y - q.y;
                put(o + (uint32_t)__popcll(mask & agent_bits), gs, g0 + N + m,
                    __builtin_amdgcn_sqrtf(dx * dx + dy * dy));
            }
            uint64_t w = mask;
            while (w) {
                const int j = __builtin_ctzll(w);
                w &= w - 1;
                const bool ob = j >= kN;
                const int ent = ob ? kN + j : j;
                const float2 q = s_pos[ent];
                const float dx = pm.x - q.x, dy = pm.y - q.y;
                put(o + (ob ? gshift : 0u), gs, g0 + ent, __builtin_amdgcn_sqrtf(dx * dx + dy * dy));
                ++o;
            }
        } else if constexpr (kN > 0 && kN <= 32 && kNo <= 32) {
            // compile-time shape with both halves in 32 bits
            uint32_t lo = (uint32_t)(mask & agent_bits), hi = (uint32_t)(mask >> kN);
            while (lo) {
                const int j = __builtin_ctz(lo);
                lo &= lo - 1;
                edge_to(j, g0 + j);
            }
            if (L.agent) edge_to(N + m, g0 + N + m);       // agent m -> its goal
            while (hi) {
                const int j = __builtin_ctz(hi);
                hi &= hi - 1;
                edge_to(2 * N + j, g0 + 2 * N + j);
            }
        } else {
            uint64_t lo = mask & agent_bits, hi = mask & ~agent_bits;
            while (lo) {
                const int j = __builtin_ctzll(lo);
                lo &= lo - 1;
                edge_to(j, g0 + j);
            }
            if (L.agent) edge_to(N + m, g0 + N + m);       // agent m -> its goal
            while (hi) {
                const int j = __builtin_ctzll(hi);
                hi &= hi - 1;
                edge_to(N + j, g0 + N + j);
            }
        }
        if (L.agent) {                                      // goal row: goal m -> agent m
            const float2 g = s_pos[N + m];
            const float dx = pm.x - g.x, dy = pm.y - g.y;
            put(goal_at, g0 + N + m, gs, __builtin_amdgcn_sqrtf(dx * dx + dy * dy));
        }
    };
    if (checked) walk(std::true_type{});
    else walk(std::false_type{});
}

// One env per wave (compile-time shape, N <= 31 agent bits and <= 32
// obstacle bits): the env's edge list is first expanded into LDS as
// (source entity | destination entity << 8) words in CSR order — per lane a
// few instructions per set bit of its row, so the row-length imbalance across
// lanes costs little — then written by all 64 lanes, edge e by lane e mod 64:
// distances from the staged positions and three coalesced stores per 64 edges.
// The expansion needs no global offset, so it runs before the workgroup's
// prefix exchange (block_emit) and fills the wait at its barrier.
// stage_rows returns the env's edge count, or -1 (nothing staged) when the
// list exceeds the scratch.
template <int kN, int kNo>
__device__ __forceinline__ int stage_rows(const Lane &L, uint32_t *s_scr, int scr_cap, uint64_t mask) {
    constexpr int N = kN;
    static_assert(N <= 31 && kNo <= 32, "agent and obstacle column bits in one word each");
    const int m = L.m;
    const uint64_t mk = L.live ? mask : 0ull;
    const uint32_t lo = (uint32_t)mk & ((1u << N) - 1u), hi = (uint32_t)(mk >> N);
    const int c = __popc(lo) + __popc(hi) + (L.agent ? 1 : 0);
    const int incl = wave_scan(c);
    const int a_total = __builtin_amdgcn_readlane(incl, N - 1);
    const int total = __builtin_amdgcn_readlane(incl, 63) + N;
    if (total > scr_cap) return -1;
    uint32_t *at = s_scr + (incl - c + (m >= N ? N : 0));
    const uint32_t src = (uint32_t)row_entity(m, N);
    for (uint32_t w = lo; w; w &= w - 1) *at++ = src | ((uint32_t)__builtin_ctz(w) << 8);
    if (L.agent) {
        *at++ = src | ((uint32_t)(N + m) << 8);             // agent m -> its goal
        s_scr[a_total + m] = (uint32_t)(N + m) | ((uint32_t)m << 8);   // goal row
    }
    for (uint32_t w = hi; w; w &= w - 1) *at++ = src | ((uint32_t)(2 * N + __builtin_ctz(w)) << 8);
    wave_sync();
    return total;
}
template <int kN, int kNo>
__device__ __forceinline__ void write_staged(const Lane &L, const float2 *s_pos, const uint32_t *s_scr, int total,
                                             int64_t env_off, const EdgeSink &out) {
    constexpr int E = 2 * kN + kNo;
    const int64_t eb = L.b;
    const int32_t g0 = (int32_t)(eb * E);
    if (out.cap < ((int64_t)1 << 29)) {
        // SGPR base (the sink's arrays) + 32-bit VGPR byte offset (the env's
        // offset and the edge): no 64-bit scalar address arithmetic per env
        // (8 * cap < 2^32 bytes)
        const uint32_t wb = (uint32_t)env_off, cap4 = (uint32_t)out.cap * 4u;
        char *const isrc = (char *)out.index, *const attr = (char *)out.attr;
        for (int e = L.lane; e < total; e += kWave) {
            const uint32_t w = s_scr[e];
            const uint32_t a = w & 0xffu, b = w >> 8;
            const float2 pa = s_pos[a], pb = s_pos[b];
            const float dx = pa.x - pb.x, dy = pa.y - pb.y;
            uint32_t byte = (wb + (uint32_t)e) << 2;
            asm("" : "+v"(byte));   // keeps the stores in SGPR-base + 32-bit-offset form
            *(int32_t *)(isrc + byte) = g0 + (int32_t)a;
            *(int32_t *)(isrc + (byte + cap4)) = g0 + (int32_t)b;
            *(float *)(attr + byte) = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
        }
        return;
    }
    const uint32_t wb_lo = __builtin_amdgcn_readfirstlane((uint32_t)env_off);
    const uint32_t wb_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)env_off >> 32));
    const int64_t wbase = (int64_t)(((uint64_t)wb_hi << 32) | wb_lo);
    char *isrc = (char *)(out.index + wbase), *idst = (char *)(out.index + out.cap + wbase);
    char *attr = (char *)(out.attr + wbase);
    for (int e = L.lane; e < total; e += kWave) {
        const uint32_t w = s_scr[e];
        const uint32_t a = w & 0xffu, b = w >> 8;
        const float2 pa = s_pos[a], pb = s_pos[b];
        const float dx = pa.x - pb.x, dy = pa.y - pb.y;
        uint32_t byte = (uint32_t)e << 2;
        asm("" : "+v"(byte));
        *(int32_t *)(isrc + byte) = g0 + (int32_t)a;
        *(int32_t *)(idst + byte) = g0 + (int32_t)b;
        *(float *)(attr + byte) = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
    }
}

// CSR offsets of a workgroup's envs: its edge counts (lane k < envs of the
// block: env first+k) and the sum of the preceding workgroups' edge sums
// (int4 loads spread over the workgroup's threads). Loads only; the sums are
// reduced in block_emit after the caller's other loads are in flight.
struct BlockPrefix {
    int cnt_k, acc;
};
// Loads at clamped addresses, predicates on the values (see seg_load): the
// first 2 * kBlock int4 words of preceding sums (2048 workgroups, 8192
// one-env-per-wave envs) need no loop; `any16` is any >= 16-byte buffer,
// read in place of block_sum when no whole int4 word precedes this block.
__device__ __forceinline__ BlockPrefix block_prefix_loads(const int32_t *block_sum, const int32_t *edge_count,
                                                          int B, int G, const void *any16) {
    BlockPrefix r{0, 0};
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int first = blockIdx.x * kWavesPerBlock * G;
    const int nblk = min(kWavesPerBlock * G, B - first);
    const int ck = edge_count[first + min(lane, nblk - 1)];
    r.cnt_k = lane < nblk ? ck : 0;
    const int nb = (int)blockIdx.x, n4 = nb >> 2, nb4 = n4 << 2;
    const int4 *bs4 = n4 > 0 ? (const int4 *)block_sum : (const int4 *)any16;
    const int kc = n4 > 0 ? n4 - 1 : 0;
    const int4 q0 = bs4[min(tid, kc)], q1 = bs4[min(tid + kBlock, kc)];
    const int tl = block_sum[min(nb4 + tid, max(nb - 1, 0))];
    r.acc = (tid < n4 ? q0.x + q0.y + q0.z + q0.w : 0) + (tid + kBlock < n4 ? q1.x + q1.y + q1.z + q1.w : 0) +
            (tid < nb - nb4 ? tl : 0);
    for (int k = tid + 2 * kBlock; k < n4; k += kBlock) {   // more than 2048 preceding workgroups
        const int4 q = bs4[k];
        r.acc += q.x + q.y + q.z + q.w;
    }
    return r;
}

// Workgroup-wide (every wave of the block must call it: one barrier): the
// env's global offset from the loaded prefix, its edge_ptr entry, then its
// edges. s_red: kWavesPerBlock ints of LDS.
template <int kN, int kNo, int kG>
__device__ __forceinline__ void block_emit(const DevParams &p, const Shape<kN, kNo> &s, const Lane &L,
                                           const float2 *s_pos, uint64_t mask, BlockPrefix pre, int *s_red,
                                           int64_t *edge_ptr, const EdgeSink &out, uint32_t *s_scr,
                                           int scr_cap) {
    const int first = blockIdx.x * kWavesPerBlock * s.G;
    // one env per wave, compile-time shape: the env's list is staged in LDS
    // before the prefix exchange (needs only local counts)
    constexpr bool kStaged = kG == 1 && kN > 0 && kN <= 31 && kNo <= 32;
    int staged = -1;
    if constexpr (kStaged) {
        if (L.b < p.B) staged = stage_rows<kN, kNo>(L, s_scr, scr_cap, mask);
    }
    const int acc = wave_total(pre.acc);
    const int incl_k = wave_scan(pre.cnt_k);     // envs of this block in order
    if (L.lane == 0) s_red[L.wave] = acc;
    __syncthreads();
    int64_t base = 0;
    for (int q = 0; q < kWavesPerBlock; ++q) base += s_red[q];
    int my_cnt, before;
    if constexpr (kG == 1) {
        my_cnt = __builtin_amdgcn_readlane(pre.cnt_k, L.wave);
        before = __builtin_amdgcn_readlane(incl_k, L.wave) - my_cnt;
    } else {
        const int kk = L.live ? L.b - first : 0;
        my_cnt = __shfl(pre.cnt_k, kk);
        before = __shfl(incl_k, kk) - my_cnt;
    }
    const int64_t env_off = base + before;
    if (L.live && L.m == 0) {
        edge_ptr[L.b] = env_off;
        if (L.b == p.B - 1) edge_ptr[p.B] = env_off + my_cnt;
    }
    if constexpr (kStaged) {
        // wave-uniform: the staged path when the env's list fit the scratch
        // and fits the outputs (a redirected slot may be smaller than the
        // worst case)
        if (staged >= 0 && env_off + staged <= out.cap) {
            write_staged<kN, kNo>(L, s_pos, s_scr, staged, env_off, out);
            return;
        }
    }
    emit_rows<kN, kNo, kG>(s, L, s_pos, mask, env_off, out, env_off + my_cnt > out.cap);
}

// ---------------------------------------------------------------------------
// Global inputs of one env for a one-env-per-wave (G = 1) wave, loaded into
// registers before the first wait. (Processing two envs per wave in turn with
// the second's loads in flight measured slower: DESIGN.md §8.)
struct SegIn {
    float2 x0, x1, v, u;
    uint64_t cand_prev, oo;
    int t, ep;
    float2 acc;
    float4 araw;   // the lane's action as loaded (seg_load_finish turns it into u)
};

// Every load is unconditional, at clamped (always valid) addresses, with the
// lane/mode predicates applied to the values afterwards: a load under a
// divergent branch ends in a wait for its data at the branch join, which
// serialised the state loads into several HBM round trips.
template <int kN, int kNo, int kFmt, bool kLag>
__device__ __forceinline__ SegIn seg_load(const DevParams &p, const Shape<kN, kNo> &s, const Lane &L) {
    static_assert(kN > 0 && kFmt >= 0, "compile-time shape and action format");
    constexpr int N = kN, E = 2 * kN + kNo, M = kN + kNo;
    SegIn in;
    const int64_t eb = L.b < p.B ? L.b : p.B - 1;                  // wave-uniform
    const uint32_t lane = (uint32_t)L.lane;
    const uint32_t ma = lane < (uint32_t)N ? lane : N - 1, mm = lane < (uint32_t)M ? lane : M - 1;
    const float2 *pos_b = p.pos + eb * E;
    in.x0 = pos_b[lane < (uint32_t)E ? lane : E - 1];
    in.x1 = E > kWave ? pos_b[lane + kWave < (uint32_t)E ? lane + kWave : E - 1] : make_float2(0.0f, 0.0f);
    in.t = p.step_count[eb];
    in.ep = p.episode[eb];
    in.acc = p.ep_acc[eb];
    in.v = p.vel[eb * N + ma];
    // reset / observe launches may carry no actions: read node features instead
    // (28 B per entity >= any action format's bytes per agent), never used
    const bool step = p.mode == kModeStep;
    const int64_t ai = eb * N + ma;
    if constexpr (kFmt == 0) {
        const float *q = (step ? (const float *)p.actions : p.node_feat) + ai * 5;
        in.araw = make_float4(q[1], q[2], q[3], q[4]);
    } else if constexpr (kFmt == 1) {
        const int32_t *q = step ? (const int32_t *)p.actions : (const int32_t *)p.node_feat;
        in.araw = make_float4(__int_as_float(q[ai]), 0.0f, 0.0f, 0.0f);
    } else {
        const float2 *q = step ? (const float2 *)p.actions : (const float2 *)p.node_feat;
        const float2 a = q[ai];
        in.araw = make_float4(a.x, a.y, 0.0f, 0.0f);
    }
    in.cand_prev = p.contact_mask[eb * N + ma];
    in.oo = p.row_mask[eb * M + mm];
    return in;
}

// the lane/mode predicates and the action force, once the loads are issued
template <int kN, int kNo, int kFmt, bool kLag>
__device__ __forceinline__ void seg_load_finish(const DevParams &p, const Lane &L, SegIn &in) {
    const bool step = p.mode == kModeStep;
    const float4 a = in.araw;
    float ux, uy;
    if constexpr (kFmt == 0) {
        ux = a.x - a.y;
        uy = a.z - a.w;
    } else if constexpr (kFmt == 1) {
        const int k = __float_as_int(a.x);
        ux = (float)(k == 1) - (float)(k == 2);
        uy = (float)(k == 3) - (float)(k == 4);
    } else {
        ux = a.x;
        uy = a.y;
    }
    const bool ag_step = L.agent && step;
    in.u = ag_step ? make_float2(ux * p.sens, uy * p.sens) : make_float2(0.0f, 0.0f);
    in.cand_prev = ag_step ? in.cand_prev : 0ull;
    if (!L.agent) in.v = make_float2(0.0f, 0.0f);
    // obstacle rows: cached obstacle-obstacle bits; lagged emission: every
    // row (the previous step's masks)
    in.oo = (L.live && (kLag || L.m >= kN) && step) ? in.oo : 0ull;
    if (L.b >= p.B) {
        in.t = in.ep = 0;
        in.acc = make_float2(0.0f, 0.0f);
    }
}

// One env (G = 1) or one wave's G envs: everything after the loads. Returns
// the wave's edge count (the sum over its envs).
template <int kN, int kNo, int kFmt, bool kLag>
__device__ __forceinline__ int seg_env(const DevParams &p, const Shape<kN, kNo> &s, const Lane &L,
                                       unsigned char *wave_lds, const SegIn &in, int64_t wid,
                                       BlockPrefix lag_pre, int *s_lag) {
    constexpr int kG = envs_per_wave<kN, kNo>();
    const int N = s.N, E = s.E, M = s.M, G = s.G;
    const int segc = L.seg < G ? L.seg : G - 1;             // clamp idle lanes' addresses
    float2 *s_pos = (float2 *)wave_lds + segc * E;
    float *s_nf = (float *)((float2 *)wave_lds + G * E);    // [G][E][7]
    const int m = L.m;
    const bool obst = L.live && m >= N;
    const bool wave_live = kG == 1 ? L.b < p.B : true;
    // per-env base pointers: wave-uniform (scalar) when G = 1; lane offsets
    // below are 32-bit
    const int64_t eb = kG == 1 ? (wave_live ? L.b : 0) : (L.live ? L.b : 0);
    const uint32_t um = (uint32_t)m;

    SegIn inf = in;
    if constexpr (kG == 1) seg_load_finish<kN, kNo, kFmt, kLag>(p, L, inf);
    int t = inf.t, ep = inf.ep;
    float2 acc = inf.acc;
    float2 v = inf.v, u = inf.u;
    uint64_t cand_prev = inf.cand_prev, oo = inf.oo;
    if constexpr (kG == 1) {
        if (wave_live) {
            if (L.lane < E) s_pos[L.lane] = in.x0;
            if (L.lane + kWave < E) s_pos[L.lane + kWave] = in.x1;
        }
    } else {
        if (L.live) {
            for (int e = m; e < E; e += M) s_pos[e] = p.pos[eb * E + e];
            t = p.step_count[L.b];
            ep = p.episode[L.b];
            acc = p.ep_acc[L.b];
        }
        if (L.agent) {
            v = p.vel[eb * N + m];
            if (p.mode == kModeStep) {
                u = action_force_t<kFmt>(p, eb * N + m);
                cand_prev = p.contact_mask[eb * N + m];
            }
        }
        if ((kLag ? L.live : obst) && p.mode == kModeStep) oo = p.row_mask[eb * M + m];
    }
    bool reset = L.live && p.mode == kModeReset && (p.env_mask == nullptr || p.env_mask[L.b] != 0);
    wave_sync();
    GSM_STAMP(p, wid, 1);
    if constexpr (kLag) {
        // the previous step's edges: its positions (staged above) and row masks
        // scratch: the staged node-feature / column-pair area (free until the sweep)
        KernargParams &q = late_params();
        block_emit<kN, kNo, kG>(p, s, L, s_pos, oo, lag_pre, s_lag, q.lag.edge_ptr,
                                EdgeSink{q.lag.edge_index, q.lag.edge_attr, q.lag.cap}, (uint32_t *)s_nf,
                                (p.wave_lds_step - 8 * G * E) / 4);
    }
    GSM_STAMP(p, wid, 2);

    // scenario.reset_world (Philox layout, App. A S14) for the lanes' envs
    auto relayout = [&]() {
        if (reset) {
            ep = (p.mode == kModeReset && p.reseed ? -1 : ep) + 1;
            t = 0;
            acc = make_float2(0.0f, 0.0f);
            v = make_float2(0.0f, 0.0f);
            const uint32_t gid = (uint32_t)(p.env_base + L.b);
            for (int e = m; e < E; e += M) s_pos[e] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)e);
        }
        wave_sync();
    };
    if (__any(reset)) relayout();

    bool done = false;
    if (p.mode == kModeStep) {
        // apply_environment_force over the candidates found on these positions
        // by the previous observation pass, then integrate_state (App. A S6)
        // physics constants read here (kernarg view), not held from the entry
        KernargParams &pc = late_params();
        if (L.agent) {
            const float2 pi = s_pos[m];
            float Fx = u.x, Fy = u.y;
            uint64_t cm = cand_prev;
            // (both constants read before the loop: a per-lane select of the
            // two kernarg fields compiles to a vector load and a vmcnt wait
            // per contact)
            const float dmin_aa = pc.dmin_aa, dmin_ao = pc.dmin_ao;
            while (cm) {
                const int c = __builtin_ctzll(cm);
                cm &= cm - 1;
                const bool ag = c < N;
                const float2 pj = s_pos[row_entity(c, N)];
                const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                const float d2 = dx * dx + dy * dy;
                const float f = contact_scale(pc, d2, ag ? dmin_aa : dmin_ao);
                Fx += f * dx;
                Fy += f * dy;
            }
            if (pc.strict && strict_bad(m, pi, N, M, [&](int c) { return s_pos[row_entity(c, N)]; })) {
                Fx = __builtin_nanf("");   // App. A S16 strict: MPE's 0/0 force
                Fy = __builtin_nanf("");
            }
            const float dt = pc.dt, max_speed = pc.max_speed;
            v.x = v.x * pc.omd;
            v.y = v.y * pc.omd;
            v.x = v.x + (Fx * pc.inv_mass) * dt;
            v.y = v.y + (Fy * pc.inv_mass) * dt;
            if (max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > max_speed) {
                    v.x = v.x / sp * max_speed;
                    v.y = v.y / sp * max_speed;
                }
            }
            float2 np;
            np.x = pi.x + v.x * dt;
            np.y = pi.y + v.y * dt;
            s_pos[m] = np;
        }
        wave_sync();
        t += 1;
        done = L.live && t >= pc.EL;
    }
    GSM_STAMP(p, wid, 3);

    // ---- observation pass on the post-physics positions
    const bool full = p.mode != kModeStep;                  // reset / observe: recompute obstacle pairs
    float2 pm = s_pos[row_entity(m, N)];
    uint64_t row, cand;
    int ccnt;
    bool coinc;
    obs_sweep<kN, kNo, kG>(p, s, L, s_pos, s_nf, pm, full, oo, row, cand, ccnt, coinc);
    GSM_STAMP(p, wid, 4);

    // reward / cost callbacks
    float r = 0.0f;
    if (L.agent) {
        const float2 g = s_pos[N + m];
        const float dx = pm.x - g.x, dy = pm.y - g.y;
        r = -__builtin_amdgcn_sqrtf(dx * dx + dy * dy);
    }
    float rsum = seg_total<kG>(r, L, M);
    const int ci = L.agent ? ccnt : 0;
    const int csum = seg_total<kG>(ci, L, M);
    if (L.agent) {
        KernargParams &q = late_params();
        (q.reward + eb * N)[um] = p.shared_reward ? rsum : r;
        (q.cost + eb * N)[um] = (float)ci;
    }
    if (p.shared_reward) rsum *= (float)N;
    bool relaid = reset;                                    // layout changed in this launch
    if (p.mode == kModeStep) {
        if (L.live) {
            acc.x += rsum;
            acc.y += (float)csum;
        }
        if (done && p.auto_reset) {
            reset = true;
            if (m == 0) p.ep_last[L.b] = acc;
        }
        if (__any(reset)) {
            // auto-reset: new layout, then the graph part of the observation again
            relayout();
            const float2 pm2 = s_pos[row_entity(m, N)];
            uint64_t row2, cand2;
            int cc2;
            bool coinc2;
            obs_sweep<kN, kNo, kG>(p, s, L, s_pos, s_nf, pm2, true, 0ull, row2, cand2, cc2, coinc2);
            if (reset) {
                pm = pm2;
                row = row2;
                cand = cand2;
                coinc = coinc2;
            }
            relaid = reset;
        }
    }
    if (!L.live) row = 0;
    GSM_STAMP(p, wid, 5);

    // ---- outputs and state. Node features: agent rows every step; goal and
    // obstacle rows (static within an episode) only when the layout is new or
    // on an observe. Rows are staged in LDS and stored lane-linear.
    // base pointers of the final stores: read here, not held from the entry
    KernargParams &q = late_params();
    float2 *const pos_b = q.pos + eb * E;
    float2 *const vel_b = q.vel + eb * N;
    const bool any_statics = p.mode != kModeStep || p.nf_full || __any(relaid);
    // one env per wave: rows go straight to HBM (each lane its 28-byte row,
    // the wave's rows contiguous); G > 1: staged in LDS, stored lane-linear
    constexpr bool kDirectNf = kG == 1;
    if (L.live) {
        float *nf = kDirectNf ? q.node_feat + eb * E * 7 : s_nf + segc * E * 7;
        if (L.agent) {
            const float2 g = s_pos[N + m];
            store_row(nf + m * 7, v, pm, make_float2(g.x - pm.x, g.y - pm.y), 0.0f);
            if (any_statics)
                store_row(nf + (N + m) * 7, make_float2(0.0f, 0.0f), g, make_float2(0.0f, 0.0f), 1.0f);
        } else if (any_statics) {
            store_row(nf + (N + m) * 7, make_float2(0.0f, 0.0f), pm, make_float2(0.0f, 0.0f), 2.0f);
        }
        if (relaid) {
            for (int e = m; e < E; e += M) pos_b[(uint32_t)e] = s_pos[e];
        } else if (L.agent && p.mode == kModeStep) {
            pos_b[um] = pm;
        }
        if (L.agent && (p.mode == kModeStep || relaid)) vel_b[um] = v;
        if (L.agent) (q.contact_mask + eb * N)[um] = cand;
        (q.row_mask + eb * M)[um] = row;
    }
    if constexpr (!kDirectNf) {
        wave_sync();
        const int b0 = kG == 1 ? L.b : (blockIdx.x * kWavesPerBlock + L.wave) * G;
        for (int g = 0; g < G; ++g) {
            if (b0 + g >= p.B) break;
            // per env, not per lane: idle lanes of the env's wave copy too
            const bool full_rows = p.mode != kModeStep || p.nf_full || (kG == 1 ? __any(relaid) : __shfl(relaid, g * M));
            const int len = (full_rows ? E : N) * 7;
            float *dst = q.node_feat + (int64_t)(b0 + g) * E * 7;
            const float *src = s_nf + g * E * 7;
            for (int q = L.lane; q < len; q += kWave) dst[(uint32_t)q] = src[q];
        }
    }

    GSM_STAMP(p, wid, 6);
    // App. A S16 flags of the final state: a coincident pair (from the sweep),
    // an agent at a non-finite position
    uint8_t deg = 0;
    if (q.degenerate) {
        const uint64_t nb = __ballot(L.agent && nonfinite2(pm));
        const uint64_t segm = M >= 64 ? ~0ull : ((1ull << M) - 1);
        deg = (uint8_t)((coinc ? kDegCoincident : 0) | (((nb >> L.base) & segm) ? kDegNonfinite : 0));
    }
    // edge count (radius rows + goal edges both ways)
    const int edges = __popcll(row) + ((L.live && m == 0) ? 2 * N : 0);
    int wave_edges;
    if constexpr (kG == 1) {
        wave_edges = wave_total(edges);
        if (wave_live && L.lane == 0) {
            q.step_count[L.b] = t;
            q.episode[L.b] = ep;
            q.ep_acc[L.b] = acc;
            q.done[L.b] = done ? 1 : 0;
            q.edge_count[L.b] = wave_edges;
            if (q.degenerate) q.degenerate[L.b] = deg;
        }
    } else {
        wave_edges = wave_sum(edges);
        const int env_edges = seg_total<kG>(edges, L, M);
        if (L.live && m == 0) {
            q.step_count[L.b] = t;
            q.episode[L.b] = ep;
            q.ep_acc[L.b] = acc;
            q.done[L.b] = done ? 1 : 0;
            q.edge_count[L.b] = env_edges;
            if (q.degenerate) q.degenerate[L.b] = deg;
        }
    }
    GSM_STAMP(p, wid, 7);
    return wave_edges;
}

template <int kN, int kNo, int kFmt, bool kLag>
__global__ __launch_bounds__(kBlock) void gsm_step_seg_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Shape<kN, kNo> s(p);
    constexpr int kG = envs_per_wave<kN, kNo>();
    const Lane L = seg_lane(p, s);
    const int wave = L.wave;
    unsigned char *wave_lds = smem + wave * p.wave_lds_step;
    const int64_t wid = (int64_t)blockIdx.x * kWavesPerBlock + wave;
    int *s_bc = (int *)(smem + kWavesPerBlock * p.wave_lds_step);
    int *s_lag = s_bc + kWavesPerBlock;
    GSM_RSTAMP(p, wid, 8);
    GSM_STAMP(p, wid, 0);
    // (the loads issued at priority 3: a late workgroup's state requests go
    // out at once instead of after the older waves' compute, then 1)
    start_prio<3>();
    {
        SegIn in{};
        if constexpr (kG == 1) in = seg_load<kN, kNo, kFmt, kLag>(p, s, L);
        BlockPrefix lag_pre{0, 0};
        if constexpr (kLag) lag_pre = block_prefix_loads(p.lag.block_sum, p.lag.edge_count, p.B, s.G, p.pos);
        start_prio<1>();
        const int edges = seg_env<kN, kNo, kFmt, kLag>(p, s, L, wave_lds, in, wid, lag_pre, s_lag);
        if (L.lane == 0) s_bc[wave] = edges;
        __syncthreads();
        if (threadIdx.x == 0) {
            int q = 0;
            for (int k = 0; k < kWavesPerBlock; ++k) q += s_bc[k];
            late_params().block_edge_sum[blockIdx.x] = q;
        }
    }
    GSM_RSTAMP(p, wid, 9);
}

// ---------------------------------------------------------------------------
template <int kN, int kNo>
__global__ __launch_bounds__(kBlock) void gsm_emit_seg_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Shape<kN, kNo> s(p);
    constexpr int kG = envs_per_wave<kN, kNo>();
    const Lane L = seg_lane(p, s);
    const int E = s.E, M = s.M, G = s.G;
    const int wave = L.wave;
    const int segc = L.seg < G ? L.seg : G - 1;
    float2 *s_pos = (float2 *)(smem + wave * p.wave_lds_emit) + segc * E;
    int *s_red = (int *)(smem + kWavesPerBlock * p.wave_lds_emit);
    const int m = L.m;
    const int64_t eb = L.live ? L.b : 0;
    const int64_t wid = (int64_t)(gridDim.x + blockIdx.x) * kWavesPerBlock + wave;
    GSM_RSTAMP(p, wid, 8);
    GSM_STAMP(p, wid, 0);

    // every global load first (positions, row masks, the block's edge counts,
    // the preceding blocks' sums; at priority 3, as in the step kernel), then
    // the first wait
    start_prio<3>();
    const BlockPrefix pre = block_prefix_loads(p.block_edge_sum, p.edge_count, p.B, G, p.pos);
    uint64_t mask = 0;
    float2 x0 = make_float2(0.0f, 0.0f), x1 = x0;
    if constexpr (kG == 1) {
        if (L.b < p.B) {
            const float2 *src = p.pos + (int64_t)L.b * E;
            if (L.lane < E) x0 = src[L.lane];
            if (L.lane + kWave < E) x1 = src[L.lane + kWave];
            if (L.live) mask = p.row_mask[eb * M + m];
        }
    } else if (L.live) {
        mask = p.row_mask[eb * M + m];
    }
    start_prio<1>();
    if constexpr (kG == 1) {
        if (L.b < p.B) {
            if (L.lane < E) s_pos[L.lane] = x0;
            if (L.lane + kWave < E) s_pos[L.lane + kWave] = x1;
        }
    } else if (L.live) {
        for (int e = m; e < E; e += M) s_pos[e] = p.pos[eb * E + e];
    }
    GSM_STAMP(p, wid, 1);
    block_emit<kN, kNo, kG>(p, s, L, s_pos, mask, pre, s_red, p.edge_ptr,
                            EdgeSink{p.edge_index, p.edge_attr, p.edge_capacity}, (uint32_t *)(s_pos + E),
                            (p.wave_lds_emit - 8 * G * E) / 4);
    GSM_STAMP(p, wid, 4);
    GSM_RSTAMP(p, wid, 9);
}

// ---------------------------------------------------------------------------
// Fused rollout: K consecutive steps of a graph chain in ONE launch (one env
// per wave, compile-time shape). Each wave keeps its env's state
// on chip across the steps — positions in LDS, velocity / contact candidates /
// row masks in registers, counters in SGPRs — so a step issues no state loads,
// and the launch boundary between steps (≈5.5 µs of fixed latency per launch
// at any batch) is paid once per K steps.
//
// Iteration k (step t = t_first + k): physics, observation sweep, reward /
// cost, auto-reset and every store of step t exactly as gsm_step_seg_kernel
// (same operations in the same order: bit-identical outputs); the
// workgroup's edge sum of step t is published as an 8-byte {tag, sum}
// granule (tag = roll_epoch_tag(epoch) | (k + 1); one relaxed agent-scope store:
// write-through, no fence); then the edges of step t - 1 are emitted from the
// positions and row masks kept from the previous iteration, at the CSR offset
// found by a decoupled look-back over the preceding workgroups' granules
// (relaxed agent-scope loads, every tag checked). Aggregates were published
// one iteration earlier, so the walk normally never waits. A workgroup waits
// only on workgroups with smaller index (dispatched before it), so the chain
// always progresses; every wait is bounded (kRollSpinTicks, then
// p.roll.status is set and the launch drains). A tail after the loop emits the
// last step's edges; the last workgroup then advances the launch epoch. In
// the bound buffers the earlier steps' edges go to a library scratch: a
// workgroup may trail its successors by several steps, so only the last
// step's edges may land in the shared outputs. (A barrier-free variant with
// per-wave granules and emission two steps behind, gsm_device.h Xfer,
// measured slower here: 9.95 vs 9.40 µs per step)
// all 8 waves per SIMD resident (2048 workgroups at 8192 envs: one residency round)
#define GSM_ROLL_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
// a lane's action of the given step row, as loaded (decoded by roll_force)
// (32-bit byte offsets from the kernarg base: capture_roll requires the
// action rows to span < 2^32 bytes, so no 64-bit scalar arithmetic per step)
template <int kN, int kFmt, typename Params>   // DevParams or its kernarg view
__device__ __forceinline__ float4 roll_action_load(const Params &p, int row, int64_t eb, uint32_t ma) {
    const char *base = p.roll.actions;
    const uint32_t rb = (uint32_t)row * (uint32_t)p.roll.stride, ai = (uint32_t)eb * (uint32_t)kN + ma;
    if constexpr (kFmt == 0) {
        const float *q = (const float *)(base + (rb + ai * 20u));
        return make_float4(q[1], q[2], q[3], q[4]);
    } else if constexpr (kFmt == 1) {
        return make_float4(__int_as_float(*(const int32_t *)(base + (rb + ai * 4u))), 0.0f, 0.0f, 0.0f);
    } else {
        const float2 a = *(const float2 *)(base + (rb + ai * 8u));
        return make_float4(a.x, a.y, 0.0f, 0.0f);
    }
}
template <int kFmt, typename Params>
__device__ __forceinline__ float2 roll_force(const Params &p, float4 a, bool agent) {
    float ux, uy;
    if constexpr (kFmt == 0) {
        ux = a.x - a.y;
        uy = a.z - a.w;
    } else if constexpr (kFmt == 1) {
        const int k = __float_as_int(a.x);
        ux = (float)(k == 1) - (float)(k == 2);
        uy = (float)(k == 3) - (float)(k == 4);
    } else {
        ux = a.x;
        uy = a.y;
    }
    return agent ? make_float2(ux * p.sens, uy * p.sens) : make_float2(0.0f, 0.0f);
}

// LDS per wave of the segmented rollout: [positions E][positions E][positions
// E] rounded to 16 B, [staging scratch 28 E] rounded to 16 B, [next forces N]
// [row masks of 64 lanes]. Buffer j at j * 8 E: one multiply per use (a select
// between two bases cost four scalar instructions per use).
constexpr int roll_lds_scr(int E) { return (24 * E + 15) & ~15; }
constexpr int roll_lds_force(int E) { return roll_lds_scr(E) + ((28 * E + 15) & ~15); }
constexpr int roll_lds_wave(int N, int E) { return roll_lds_force(E) + 8 * N + 8 * kWave; }

// kSlots: per-step outputs at base + k * stride (a rollout buffer); else every
// step into the bound buffers (the strides are 0 and fold away).
// kEager: the one-launch eager step (gsm_step, K = 1 at compile time). Its
// hand-off epoch lives in device memory (p.roll.dev_epoch: kEpochReps
// replicas), read by every workgroup at entry and advanced by the grid's last
// workgroup once its final prefix is complete — by then every workgroup has
// published its count, so has read the epoch — and the chunk-sum half is the
// epoch's parity. No per-launch host state: a stream capture of env.step
// (torch.cuda.graph around a policy and the step) records this launch and
// every replay takes the next epoch.
template <int kN, int kNo, int kFmt, bool kSlots, bool kEager = false>
__global__ __launch_bounds__(kBlock) GSM_ROLL_ATTR void gsm_roll_seg_kernel(DevParams p) {
    static_assert(kN > 0 && kN <= 31 && kNo <= 32 && kFmt >= 0, "compile-time shape, staged emission");
    static_assert(!(kSlots && kEager), "the eager step writes the bound or redirected outputs");
    constexpr int N = kN, M = kN + kNo, E = 2 * kN + kNo;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Shape<kN, kNo> s(p);
    // one env per wave whatever the config's G (the step kernels may pack
    // several small envs into a wave; here a wave's latency chain per step is
    // the bound, so one env each)
    Lane L0;
    L0.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    L0.lane = threadIdx.x & 63;
    L0.seg = 0;
    L0.base = 0;
    L0.m = L0.lane;
    L0.b = blockIdx.x * kWavesPerBlock + L0.wave;
    L0.live = L0.lane < M && L0.b < p.B;
    L0.agent = L0.live && L0.m < N;
    const int wave = L0.wave;
    // Positions rotate through three LDS buffers: step k reads buffer k % 3
    // and writes the agents' new positions into buffer (k + 1) % 3, so the
    // positions after step k - 2, which iteration k emits the edges of, are
    // still in the third; goals and obstacles (static within an episode) are
    // kept in all three. Compile-time layout (roll_kernel_lds): [positions] x 3,
    // [staging scratch], [the next step's agent forces], [the row masks of
    // step k - 2].
    constexpr int wstride = roll_lds_wave(N, E);
    unsigned char *wave_lds = smem + wave * wstride;
    float2 *const s_buf0 = (float2 *)wave_lds;
    float2 *const s_buf1 = s_buf0 + E;
    float2 *const s_buf2 = s_buf1 + E;
    float *s_nf = (float *)(wave_lds + roll_lds_scr(E));
    float2 *s_force = (float2 *)(wave_lds + roll_lds_force(E));
    uint64_t *const s_row = (uint64_t *)(s_force + N);
    // positions before step j, by j % 3
    auto pos_buf = [&](int j3) { return s_buf0 + j3 * E; };
    int *s_bc = (int *)(smem + kWavesPerBlock * wstride);   // [3][waves]: per-env edge counts by step % 3
    int *s_red = s_bc + 3 * kWavesPerBlock;                 // [4]: the workgroup's offset, pace level, rank, pad
    int *s_pre = s_red + 4;                                 // [3][waves]: exclusive prefix of the counts
    constexpr int scr_cap = 7 * E;   // words of staging scratch
    const bool wave_live = L0.b < p.B;
    const int64_t eb = wave_live ? L0.b : 0;
    GSM_RSTAMP(p, L0.b, 0);   // diagnostic builds: the launch's timeline per wave
    GSM_SET(p, L0.b, 9, (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                  // HW_ID
                            ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32));   // XCC_ID
    // start priorities (the pace levels take over from iteration 2): the
    // entry at 3, so that a late workgroup's state loads issue at once; step 0
    // at 2 and step 1 at 1, so that no wave runs a later step while one on its
    // SIMD is still in an earlier one — oldest-first issue alone let a CU's
    // rank-0 workgroup finish step 0 at 4.9 us and rank 7 at 21.5 us, and
    // iteration 2's emission waits for step 0 of every workgroup
    start_prio<3>();
    // this launch's epoch (eager: from device memory, a replica per 64
    // workgroups' neighbourhood; else a launch argument)
    uint32_t epoch;
    if constexpr (kEager)
        epoch = __builtin_amdgcn_readfirstlane(__hip_atomic_load(
            (gu32 *)hand_chk(p.roll.dev_epoch + (blockIdx.x % kEpochReps) * kEpochStride), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
    else
        epoch = p.roll.epoch;
    // the chunk sums of this launch and the half zeroed for the next one
    // (eager: by the epoch's parity; else set per launch by the host)
    auto csum_of = [&](KernargParams &q) -> uint64_t * {
        if constexpr (kEager) return (epoch & 1u) ? q.roll.csum_next : q.roll.csum;
        else return q.roll.csum;
    };
    auto csum_next_of = [&](KernargParams &q) -> uint64_t * {
        if constexpr (kEager) return (epoch & 1u) ? q.roll.csum : q.roll.csum_next;
        else return q.roll.csum_next;
    };
    // pacing: this workgroup's CU counter (the arrival now, a step after each
    // step; its address re-formed at each use, no SGPRs held across the loop),
    // and the counters of the slot's next launch zeroed (none for one step)
    auto pacing = [] {
        if constexpr (kEager) return false;
        else return late_params().roll.pace != nullptr;
    };
    auto pace_ctr = [] { return (gu32 *)hand_chk(late_params().roll.pace + pace_key()); };
    uint32_t pace_v = 0;   // thread 0: the arrivals before its own
    // one-hop prefix: chunks of 64 workgroups, their sums `cs` u64 apart; the
    // slot's next launch's chunk sums zeroed
    const int nc = ((int)gridDim.x + kPrefixChunk - 1) / kPrefixChunk;
    auto zero_next_csums = [&] {
        KernargParams &qz = late_params();
        const int cs = qz.roll.csum_stride, n = (kEager ? 1 : qz.roll.K) * nc;
        uint64_t *const cz = csum_next_of(qz);
        for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
            __hip_atomic_store((gu64 *)hand_chk(cz + (int64_t)i * cs), 0ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // (eager: behind the state loads, so that they need not wait for the
    // epoch load that picks the half)
    if constexpr (!kEager) zero_next_csums();
    if (pacing()) {
        KernargParams &qz = late_params();
        for (int i = blockIdx.x * kBlock + threadIdx.x; i < kPaceKeys; i += gridDim.x * kBlock)
            __hip_atomic_store((gu32 *)hand_chk(qz.roll.pace_next + i * kPaceStride), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0)
            pace_v = __hip_atomic_fetch_add(pace_ctr(), kPaceArrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---- the state before step t_first and step t_first's actions
    // (p.actions); the edges of that state were emitted by whatever ran before
    SegIn in = seg_load<kN, kNo, kFmt, true>(p, s, L0);
    if constexpr (kEager) zero_next_csums();   // (the state loads in flight: only the epoch is waited for)
    seg_load_finish<kN, kNo, kFmt, true>(p, L0, in);
    int t = in.t, ep = in.ep;
    float2 acc = in.acc, v = in.v, u = in.u;
    uint64_t cand_prev = in.cand_prev, oo = in.oo;
    if (wave_live) {
        if (L0.lane < E) s_buf0[L0.lane] = s_buf1[L0.lane] = s_buf2[L0.lane] = in.x0;
        if (L0.lane + kWave < E) s_buf0[L0.lane + kWave] = s_buf1[L0.lane + kWave] = s_buf2[L0.lane + kWave] = in.x1;
    }
    if (threadIdx.x == 0) s_red[2] = (int)(pace_v >> 24);   // the rank on the CU (its load waited above)
    wave_sync();
    start_prio<2>();
    GSM_RSTAMP(p, L0.b, 1);
    // apply_environment_force: the action force plus the contact terms of the
    // candidates in ascending collider order
    auto add_contacts = [&](const float2 *s_pos, float2 F, float2 pi, uint64_t cm, const KernargParams &pc) {
        // (both constants read before the loop: a per-lane select of the two
        // kernarg fields compiles to a vector load and a vmcnt wait per contact)
        const float dmin_aa = pc.dmin_aa, dmin_ao = pc.dmin_ao;
        while (cm) {
            const int c = __builtin_ctzll(cm);
            cm &= cm - 1;
            const bool ag = c < N;
            const float2 pj = s_pos[row_entity(c, N)];
            const float dx = pi.x - pj.x, dy = pi.y - pj.y;
            const float d2 = dx * dx + dy * dy;
            const float f = contact_scale(pc, d2, ag ? dmin_aa : dmin_ao);
            F.x += f * dx;
            F.y += f * dy;
        }
        return F;
    };
    // With the near-bit walk (kFused) each step's sweep forms the next step's
    // force at the positions it reads (obs_sweep_g1 kForce), so the loop runs
    // one pass over the pairs per step; the force waits in LDS (s_force) for
    // the next integration; the first step's force is formed here.
    constexpr bool kFused = sweep_walks_near<kN, kNo>(1);
    if constexpr (kFused) {
        if (L0.agent) s_force[L0.m] = add_contacts(s_buf0, u, s_buf0[L0.m], cand_prev, late_params());
    }

    const int K = kEager ? 1 : p.roll.K, n_act = p.roll.n_actions;
    const uint32_t etag = roll_epoch_tag(epoch);            // this launch's tag base
    int arow = p.roll.t_first % n_act;                      // action row of the current step
    uint8_t deg = 0;                                        // App. A S16 flags of the final state
    // The edges of step t_first + j (j < K), emitted two iterations later
    // (iteration j + 2; the last two steps' by the tail after the loop): its
    // positions kept in buffer pj3, its row masks `mask`, this workgroup's
    // counts of it in s_bc[cj3]. `done`: the steps this workgroup has added to
    // its CU's pace counter (0: no pacing here, the tail).
    auto emit_step = [&](const int j, const int pj3, const int cj3, const uint64_t mask, const int done,
                         const Lane &L) {
        const int *cb = s_bc + cj3 * kWavesPerBlock;   // this workgroup's counts of step j
        // the env's list staged first (needs only its own row counts)
        GSM_TNOW(te0);
        const int staged = wave_live ? stage_rows<kN, kNo>(L, (uint32_t *)s_nf, scr_cap, mask) : -1;
        GSM_ACC(p, L.b, 14, te0);   // diagnostic builds: staging (emission, below, adds to it)
        GSM_TNOW(te1);
        // wave 0 forms the workgroup's offset (one hop: the chunk sums and its
        // chunk-mates' counts, published two iterations ago) and hands it to
        // the other waves, with its CU's pace counter loaded beside it
        if (wave == 0) {
            KernargParams &qe = late_params();
            const uint32_t pv = done > 0 ? __hip_atomic_load(pace_ctr(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            const int cs = qe.roll.csum_stride;
            const int ex = roll_prefix(qe.roll.gran + (int64_t)j * gridDim.x, csum_of(qe) + (int64_t)j * nc * cs, cs,
                                       etag | (uint32_t)(j + 1), qe.roll.status, L.lane);
            // eager: the grid's last workgroup, its prefix complete, has seen
            // every other workgroup's count published — each read the epoch
            // before — so the next launch's epoch goes out now
            if constexpr (kEager) {
                if (blockIdx.x == gridDim.x - 1 && L.lane < kEpochReps)
                    __hip_atomic_store((gu32 *)hand_chk(qe.roll.dev_epoch + L.lane * kEpochStride), (epoch + 1u) & 0xfffffu,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the pace level formed here once for the workgroup (wave-uniform
            // SALU work that every wave repeated before)
            const int lvl = done > 0 ? pace_level((uint32_t)__builtin_amdgcn_readfirstlane(pv), done,
                                                  __builtin_amdgcn_readfirstlane(s_red[2]), qe.roll.pace_q)
                                     : 1;
            if (L.lane == 0) {
                s_red[0] = ex;
                s_red[1] = lvl;
            }
        }
        GSM_ACC(p, L.b, 12, te1);   // the prefix (wave 0)
        GSM_TNOW(te2);
        __syncthreads();
        GSM_ACC(p, L.b, 13, te2);   // waiting for it
        GSM_TNOW(te3);
        if (done > 0) pace_set(__builtin_amdgcn_readfirstlane(s_red[1]));
        // (the prefix formed once by thread 0, not w < wave selects: those
        // are loop-invariant lane masks the compiler holds in SGPR pairs)
        const int before = s_pre[cj3 * kWavesPerBlock + wave];
        const int my_cnt = cb[wave];
        int64_t env_off = (int64_t)s_red[0] + before;
        // (an offset past the capacity is a legal overflow of a small slot:
        // edge_ptr keeps it, the writes below stop at the capacity)
        if (env_off < 0) {   // a broken hand-off: never write out of bounds
            if (L.lane == 0)
                __hip_atomic_store((gu32 *)late_params().roll.status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            env_off = late_params().ro.cap;
        }
        if (wave_live) {
            KernargParams &qs = late_params();
            if (L.lane == 0) {
                int64_t *const eptr = qs.ro.eptr + (kSlots ? j * qs.ro.ep_s : 0);
                eptr[L.b] = env_off;
                if (L.b == qs.B - 1) eptr[qs.B] = env_off + my_cnt;
            }
            const EdgeSink out = roll_edge_sink<kSlots>(qs, j, K);
            const float2 *s_prev = pos_buf(pj3);                // positions after step j
            if (staged >= 0 && env_off + staged <= out.cap)
                write_staged<kN, kNo>(L, s_prev, (uint32_t *)s_nf, staged, env_off, out);
            else
                emit_rows<kN, kNo, 1>(s, L, s_prev, mask, env_off, out, env_off + my_cnt > out.cap);
        }
        wave_sync();
        GSM_ACC(p, L.b, 14, te3);
    };
    int r3 = 0;                 // k % 3
    bool relaid_prev = false;   // the previous iteration re-laid the env out (wave-uniform)
    for (int k = 0; k < K; ++k) {
        // lane-derived values re-formed every iteration (an asm barrier): held
        // across the loop they would pin their hoisted addresses in VGPRs
        Lane L = L0;
        asm volatile("" : "+v"(L.lane), "+v"(L.m));
        const int m = L.m;
        GSM_TNOW(tw0);
        const uint32_t um = (uint32_t)m, ma = L.lane < N ? (uint32_t)L.lane : N - 1;
        // the next step's actions, in flight during this step
        const int nrow = arow + 1 == n_act ? 0 : arow + 1;
        const float4 anext = roll_action_load<kN, kFmt>(late_params(), nrow, eb, ma);

        // apply_environment_force + integrate_state (as gsm_step_seg_kernel):
        // from s_cur into s_pos
        const int r3n = r3 == 2 ? 0 : r3 + 1;   // (k + 1) % 3
        const float2 *const s_cur = pos_buf(r3);
        float2 *const s_pos = pos_buf(r3n);
        KernargParams &pc = late_params();
        if (L.agent) {
            const float2 pi = s_cur[m];
            float Fx, Fy;
            if constexpr (kFused) {
                const float2 F = s_force[m];
                Fx = F.x;
                Fy = F.y;
            } else {
                const float2 Fc = add_contacts(s_cur, u, pi, cand_prev, pc);
                Fx = Fc.x;
                Fy = Fc.y;
            }
            if (pc.strict && strict_bad(m, pi, N, M, [&](int c) { return s_cur[row_entity(c, N)]; })) {
                Fx = __builtin_nanf("");
                Fy = __builtin_nanf("");
            }
            const float dt = pc.dt, max_speed = pc.max_speed;
            v.x = v.x * pc.omd;
            v.y = v.y * pc.omd;
            v.x = v.x + (Fx * pc.inv_mass) * dt;
            v.y = v.y + (Fy * pc.inv_mass) * dt;
            if (max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > max_speed) {
                    v.x = v.x / sp * max_speed;
                    v.y = v.y / sp * max_speed;
                }
            }
            float2 np;
            np.x = pi.x + v.x * dt;
            np.y = pi.y + v.y * dt;
            s_pos[m] = np;
        }
        wave_sync();
        if (k == 0) GSM_RSTAMP(p, L.b, 2);
        t += 1;
        const bool done = L.live && t >= pc.EL;

        // observation pass on the post-physics positions
        float2 pm = s_pos[row_entity(m, N)];
        uint64_t row, cand;
        int ccnt;
        bool coinc;
        // (kFused: the next step's force, formed by the sweep's walk)
        auto unext = [&]() { return roll_force<kFmt>(late_params(), anext, true); };
        float2 Fn = make_float2(0.0f, 0.0f);
        obs_sweep<kN, kNo, 1, kFused>(late_params(), s, L, s_pos, s_nf, pm, false, oo, row, cand, ccnt, coinc, &Fn,
                                      unext);
        if (k == 0) GSM_RSTAMP(p, L.b, 3);

        // reward / cost
        float r = 0.0f;
        if (L.agent) {
            const float2 g = s_pos[N + m];
            const float dx = pm.x - g.x, dy = pm.y - g.y;
            r = -__builtin_amdgcn_sqrtf(dx * dx + dy * dy);
        }
        float rsum = wave_total(r);
        const int ci = L.agent ? ccnt : 0;
        const int csum = wave_total(ci);
        if (L.agent) {
            // (32-bit byte offsets from the kernarg base: SGPR base + VGPR
            // offset stores, no 64-bit scalar address arithmetic per store)
            KernargParams &q = late_params();
            const uint32_t off = ((uint32_t)eb * (uint32_t)N + um) * 4u;
            *(float *)((char *)(q.ro.rew + (kSlots ? k * q.ro.rc_s : 0)) + off) = q.shared_reward ? rsum : r;
            *(float *)((char *)(q.ro.cost + (kSlots ? k * q.ro.rc_s : 0)) + off) = (float)ci;
        }
        if (late_params().shared_reward) rsum *= (float)N;
        if (L.live) {
            acc.x += rsum;
            acc.y += (float)csum;
        }
        bool reset = false;
        if (done && late_params().auto_reset) {
            reset = true;
            if (m == 0) late_params().ep_last[L.b] = acc;
        }
        GSM_TNOW(tr0);
        if (__any(reset)) {
            // auto-reset: scenario.reset_world, then the graph part again
            if (reset) {
                ep = ep + 1;
                t = 0;
                acc = make_float2(0.0f, 0.0f);
                v = make_float2(0.0f, 0.0f);
                const uint32_t gid = (uint32_t)(late_params().env_base + L.b);
                for (int e = m; e < E; e += M) s_pos[e] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)e);
            }
            wave_sync();
            const float2 pm2 = s_pos[row_entity(m, N)];
            uint64_t row2, cand2;
            int cc2;
            bool coinc2;
            float2 Fn2 = make_float2(0.0f, 0.0f);
            obs_sweep<kN, kNo, 1, kFused>(late_params(), s, L, s_pos, s_nf, pm2, true, 0ull, row2, cand2, cc2,
                                          coinc2, &Fn2, unext);
            if (reset) {
                pm = pm2;
                row = row2;
                cand = cand2;
                coinc = coinc2;
                Fn = Fn2;
            }
        }
        GSM_ACC(p, L.b, 15, tr0);   // diagnostic builds: the re-layout (and the test for it)
        const bool relaid = reset;
        if (!L.live) row = 0;
        if constexpr (kFused) {
            if (L.agent) s_force[m] = Fn;
        }

        // the step's observation outputs (node features, reward / cost above,
        // done; edges one iteration on); the simulator state (positions,
        // velocities, masks, counters) stays on chip and is stored once, after
        // the loop
        KernargParams &q = late_params();
        const bool any_statics = q.nf_full || __any(relaid);
        if constexpr (kSlots) {
            // (a rollout buffer: every slot's rows in full; the nested form
            // measured 1.4% faster there, profiles/r5_ab/store_blocks)
            if (L.live) {
                float *nf = q.ro.nf + k * q.ro.nf_s + eb * E * 7;
                if (L.agent) {
                    const float2 g = s_pos[N + m];
                    store_row(nf + m * 7, v, pm, make_float2(g.x - pm.x, g.y - pm.y), 0.0f);
                    if (any_statics)
                        store_row(nf + (N + m) * 7, make_float2(0.0f, 0.0f), g, make_float2(0.0f, 0.0f), 1.0f);
                } else if (any_statics) {
                    store_row(nf + (N + m) * 7, make_float2(0.0f, 0.0f), pm, make_float2(0.0f, 0.0f), 2.0f);
                }
            }
        } else {
            // one store block per row kind, its values selected by bit masks
            // (plain VALU; nested lane branches cost ~20 exec-mask SALU per
            // step): agent lanes their agent row (v, p, goal - p, 0), obstacle
            // lanes with statics their obstacle row (0, p, 0, 2) — v is 0
            // there — then agent lanes with statics their goal row (0, goal, 0, 1)
            const uint32_t am = (uint32_t)((int)(um - (uint32_t)N) >> 31);   // ~0 on agent lanes
            const float2 g = s_pos[N + (um & am)];
            const float2 gr = make_float2(__uint_as_float(__float_as_uint(g.x - pm.x) & am),
                                          __uint_as_float(__float_as_uint(g.y - pm.y) & am));
            const float type = __uint_as_float(~am & 0x40000000u);           // 0 or 2
            char *nfb = (char *)q.ro.nf;
            const uint32_t env_el = (uint32_t)eb * (uint32_t)(E * 7);
            if (L.live && (L.agent || any_statics))
                store_row((float *)(nfb + (env_el + (um + (~am & (uint32_t)N)) * 7u) * 4u), v, pm, gr, type);
            if (L.agent && any_statics)
                store_row((float *)(nfb + (env_el + (um + (uint32_t)N) * 7u) * 4u), make_float2(0.0f, 0.0f), g,
                          make_float2(0.0f, 0.0f), 1.0f);
        }
        if (k == K - 1 && q.degenerate) {
            const uint64_t nb = __ballot(L.agent && nonfinite2(pm));
            deg = (uint8_t)((coinc ? kDegCoincident : 0) | (nb ? kDegNonfinite : 0));
        }
        const int edges = __popcll(row) + ((L.live && m == 0) ? 2 * N : 0);
        const int wave_edges = wave_total(edges);
        if (wave_live && L.lane == 0) {
            (q.ro.done + (kSlots ? k * q.ro.done_s : 0))[L.b] = done ? 1 : 0;
            if (kSlots || k == K - 1) (q.ro.ecount + (kSlots ? k * q.ro.ec_s : 0))[L.b] = wave_edges;
        }

        // publish the workgroup's edge sum of step t
        if (L.lane == 0) s_bc[r3 * kWavesPerBlock + wave] = wave_edges;
        GSM_ACC(p, L.b, 10, tw0);   // the step's work
        GSM_TNOW(tw1);
        __syncthreads();
        GSM_ACC(p, L.b, 11, tw1);   // the publish barrier
        if (threadIdx.x == 0) {
            int sum = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) {
                s_pre[r3 * kWavesPerBlock + w] = sum;
                sum += s_bc[r3 * kWavesPerBlock + w];
            }
            const int cs = q.roll.csum_stride;
            prefix_publish(q.roll.gran + (int64_t)k * gridDim.x, csum_of(q) + (int64_t)k * nc * cs, cs,
                           (int)blockIdx.x, etag | (uint32_t)(k + 1), (uint32_t)sum);
            // the last step's sums for the emit launch that follows, in the
            // config's workgroup layout: with G envs per wave the last of the
            // G rollout workgroups of a slot adds the others' granules
            if (k == K - 1) {
                const int G = q.G, r = (int)blockIdx.x;
                if (G == 1) {
                    q.block_edge_sum[r] = sum;
                } else {
                    const int first = (r / G) * G, last = min(first + G, (int)gridDim.x) - 1;
                    if (r == last) {
                        const uint64_t *gk = q.roll.gran + (int64_t)k * gridDim.x;
                        const uint32_t tag = etag | (uint32_t)(k + 1);
                        int tot = sum;
                        for (int j = first; j < r; ++j) {
                            uint64_t x = gran_ld(gk + j);
                            if ((uint32_t)(x >> 32) != tag) x = roll_wait(gk + j, tag, q.roll.status);
                            tot += (int)(uint32_t)x;
                        }
                        q.block_edge_sum[r / G] = tot;
                    }
                }
            }
        }
        if (k == K - 1) GSM_RSTAMP(p, L.b, 4);
        // the edges of step t - 2 (row masks kept in s_row, positions after
        // it in buffer (k + 2) % 3, its counts in s_bc[(k + 1) % 3])
        if (k >= 2) emit_step(k - 2, r3n == 2 ? 0 : r3n + 1, r3n, s_row[L.lane], pacing() ? k : 0, L);
        // this workgroup's step into its CU's pace counter (read back in the
        // next iteration's emission)
        if (threadIdx.x == 0 && pacing())
            (void)__hip_atomic_fetch_add(pace_ctr(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == 0) start_prio<1>();
        // keep step t - 1's row masks for the next iteration's emission and
        // step t's for its sweep
        s_row[L.lane] = oo;
        oo = row;
        cand_prev = L.agent ? cand : 0ull;
        // A re-layout (iteration k) puts the new episode's statics into
        // buffer (k + 1) % 3; the other two still hold the old ones, which the
        // emissions of steps t - 2 and t - 1 (this and the next iteration)
        // read. So they are copied into buffer (k + 2) % 3 now, after this
        // iteration's emission, and into buffer k % 3 = (k + 3) % 3 at the end
        // of the next iteration, after its emission: each before the sweep
        // that reads it.
        const bool relaid_now = __any(relaid);
        if (__builtin_expect(relaid_now || relaid_prev, 0)) {
            float2 *const dst = pos_buf(r3n == 2 ? 0 : r3n + 1);
            for (int e = N + m; e < E; e += kWave) dst[e] = s_pos[e];
        }
        relaid_prev = relaid_now;
        if constexpr (!kFused) u = roll_force<kFmt>(late_params(), anext, L.agent);
        arow = nrow;
        r3 = r3n;
        wave_sync();
    }
    // the final state (what the next launch or an eager step reads), stored
    // before the tail: its emissions wait for the last steps' offsets, and
    // these stores need none
    KernargParams &q = late_params();
    if (wave_live) {
        float2 *const pos_b = q.pos + eb * E;
        const float2 *const s_pos = pos_buf(r3);
        // (eager: the goal / obstacle rows change only with a re-layout — for
        // K = 1 the last iteration's, relaid_prev — so otherwise the agents'
        // rows only: 384 of 576 bytes per env less at 24 agents)
        const int n_rows = (kEager && !relaid_prev) ? N : E;
        if (L0.lane < n_rows) pos_b[L0.lane] = s_pos[L0.lane];
        if (L0.lane + kWave < n_rows) pos_b[L0.lane + kWave] = s_pos[L0.lane + kWave];
        if (L0.agent) {
            (q.vel + eb * N)[L0.lane] = v;
            (q.contact_mask + eb * N)[L0.lane] = cand_prev;
        }
        if (L0.live) (q.row_mask + eb * M)[L0.lane] = oo;
        if (L0.lane == 0) {
            q.step_count[L0.b] = t;
            q.episode[L0.b] = ep;
            q.ep_acc[L0.b] = acc;
            if (q.degenerate) q.degenerate[L0.b] = deg;
        }
    }
    {   // the tail: the last two steps' edges (r3 = K % 3)
        Lane L = L0;
        asm volatile("" : "+v"(L.lane), "+v"(L.m));
        GSM_RSTAMP(p, L.b, 5);
        const int rm1 = r3 == 0 ? 2 : r3 - 1;   // (K - 1) % 3
        // Wave 0 hands each emission's offset over in s_red[0] before the
        // emission's barrier. In the loop the publish barrier lies between
        // two emissions; here they are adjacent, so a barrier first: no wave
        // may still be about to read the previous emission's offset when
        // wave 0 writes the next one (a wave held back by its priority would
        // otherwise write step K - 2's edges at step K - 1's offset)
        if (K >= 2) {
            __syncthreads();
            emit_step(K - 2, rm1, rm1 == 0 ? 2 : rm1 - 1, s_row[L.lane], 0, L);
        }
        GSM_RSTAMP(p, L.b, 6);
        __syncthreads();
        emit_step(K - 1, r3, rm1, oo, 0, L);
        GSM_RSTAMP(p, L.b, 7);
    }
    GSM_RSTAMP(p, L0.b, 8);
}

// ---------------------------------------------------------------------------
// Fused rollout of SMALL envs (M = N + No <= 16; C2: 3 agents + 3 obstacles),
// four envs per wave in 16-lane segments. One env per wave left
// 58 of 64 lanes idle at C2 and paid every per-step wave-level instruction —
// reductions, stores, the hand-off, most of them on the CU's shared scalar
// issue path — once per env; here once per four. Lane (seg, m):
// env (blockIdx * 4 + wave) * 4 + seg, collider row m (agents [0, N), obstacle
// m >= N = entity N + m). Per-env values live in every lane of the segment;
// segment sums and scans are 16-lane DPP row operations (plain VALU). The
// pair sweep forms each row's bits by VGPR integer arithmetic on d2
// (gsm_ragged_kernels.hip ragged_sweep) over all M columns, so obstacle rows
// need no cached obstacle-obstacle bits. Every output, the operations and
// their order are those of gsm_step_seg_kernel + gsm_emit_seg_kernel for the
// same envs (G = 4 there too: a workgroup holds the same 16 envs, so the last
// step's workgroup sums are the config's block_edge_sum directly).
constexpr int kPackSeg = 16, kPackG = kWave / kPackSeg;   // lanes per env, envs per wave
constexpr int kPackDepth = 5;   // iterations between a step and the writing of its edges
template <int kN, int kNo>
constexpr int pack_lds_wave() { return (kPackDepth + 1) * 8 * kPackG * (2 * kN + kNo) + 8 * kPackG * kN; }
template <int kCtrl>
__device__ __forceinline__ int dpp_row0(int v) {   // DPP within 16-lane rows, 0 shifted in
    return __builtin_amdgcn_update_dpp(0, v, kCtrl, 0xf, 0xf, true);
}
__device__ __forceinline__ int seg_sum16(int v) {   // every lane: its 16-lane row's sum
    v += dpp_row0<0xB1>(v);
    v += dpp_row0<0x4E>(v);
    v += dpp_row0<0x141>(v);
    v += dpp_row0<0x140>(v);
    return v;
}
__device__ __forceinline__ float seg_sum16(float v) {
    v += __int_as_float(dpp_row0<0xB1>(__float_as_int(v)));
    v += __int_as_float(dpp_row0<0x4E>(__float_as_int(v)));
    v += __int_as_float(dpp_row0<0x141>(__float_as_int(v)));
    v += __int_as_float(dpp_row0<0x140>(__float_as_int(v)));
    return v;
}
__device__ __forceinline__ int seg_scan16(int v) {   // inclusive scan within the 16-lane row
    v += dpp_row0<0x111>(v);
    v += dpp_row0<0x112>(v);
    v += dpp_row0<0x114>(v);
    v += dpp_row0<0x118>(v);
    return v;
}

// (four envs per wave: C2's 4096 envs are 1024 waves, one per SIMD; up to
// 128 VGPRs, four waves per SIMD, keep 16384 envs in one residency round)
template <int kN, int kNo, int kFmt, bool kSlots>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void gsm_roll_pack_kernel(DevParams p) {
    constexpr int N = kN, M = kN + kNo, E = 2 * kN + kNo;
    static_assert(M <= kPackSeg && E <= kPackSeg, "one 16-lane segment per env");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, seg = lane >> 4, m = lane & (kPackSeg - 1);
    const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kPackG + seg;   // this lane's env
    const bool env_live = b < p.B;
    const bool live = env_live && m < M, agent = live && m < N;
    const int64_t eb = env_live ? b : 0;
    // LDS per wave: positions [kPackDepth + 1][G][E] in rotation — buffer
    // `cur` holds the positions before step k, step k writes all of its env's
    // rows into the next (agents integrated, goals / obstacles carried or
    // relaid), and the others still hold the positions after steps k - 2 ..
    // k - kPackDepth (this iteration writes step k - kPackDepth's edges) —
    // then the next step's forces [G][N]
    float2 *const s_w = (float2 *)(smem + wave * pack_lds_wave<kN, kNo>());
    auto pos_buf = [&](int i) { return s_w + i * kPackG * E + seg * E; };   // this env's rows in buffer i
    float2 *const s_force = s_w + (kPackDepth + 1) * kPackG * E + seg * N;
    int *s_bc = (int *)(smem + kWavesPerBlock * pack_lds_wave<kN, kNo>());   // [waves]: the last step's counts
    const int ent = m < N ? m : N + m;                                       // this lane's collider entity
    const int wid = blockIdx.x * kWavesPerBlock + wave;                     // (diagnostic stamps)
    (void)wid;

    // ---- the state before step t_first
    const float2 *pos_g = p.pos + eb * E;
    float2 x = env_live && m < E ? pos_g[m] : make_float2(0.0f, 0.0f);   // lane m: entity m
    float2 v = agent ? p.vel[eb * N + m] : make_float2(0.0f, 0.0f);
    int t = env_live ? p.step_count[eb] : 0, ep = env_live ? p.episode[eb] : 0;
    float2 acc = env_live ? p.ep_acc[eb] : make_float2(0.0f, 0.0f);
    uint32_t cand_prev = agent ? (uint32_t)p.contact_mask[eb * N + m] : 0u;
    const float4 a0 = roll_action_load<kN, kFmt>(p, p.roll.t_first % p.roll.n_actions, eb, agent ? m : 0);
    if (env_live && m < E) pos_buf(0)[m] = x;
    wave_sync();

    // one pass over the env's M columns from the positions at `s` (lane m:
    // row m): radius row bits, contact candidates (agent rows), collisions
    // (agent rows, own column excluded), an agent-column coincidence; with
    // kForce the contact forces of the candidates added to *F in ascending
    // collider order (the step kernel's force pass: same operations)
    auto sweep = [&](const float2 *sp, float2 pm, uint32_t &rad, uint32_t &cand, int &cnt, bool &zero_agent,
                     float2 *F) {
        KernargParams &q = late_params();
        uint32_t r2b1 = __float_as_uint(q.R2) + 1u;
        asm volatile("" : "+v"(r2b1));
        // (the candidate threshold is the PAIR's: agent-agent for agent columns
        // of an agent row, agent-obstacle otherwise)
        uint32_t cut_aa = __float_as_uint(q.cut2_aa), cut_ao = __float_as_uint(q.cut2_ao);
        asm volatile("" : "+v"(cut_aa), "+v"(cut_ao));
        uint32_t rw = 0, cw = 0, nz = 0;
#pragma unroll
        for (int c = M - 1; c >= 0; --c) {   // descending: column c ends at bit c
            const float2 qc = sp[c < N ? c : N + c];
            const float dx = pm.x - qc.x, dy = pm.y - qc.y;
            const uint32_t a = __float_as_uint(__builtin_fabsf(dx * dx) + __builtin_fabsf(dy * dy));
            const uint32_t na = 0u - a;
            const uint32_t cb = (c < N && m < N) ? cut_aa : cut_ao;   // c compile-time; m < N per lane
            rw = __builtin_amdgcn_alignbit(rw, na & (a - r2b1), 31);
            cw = __builtin_amdgcn_alignbit(cw, na & (a - cb), 31);
            nz = __builtin_amdgcn_alignbit(nz, na, 31);
        }
        constexpr uint32_t colmask = (1u << M) - 1u, amask = (1u << N) - 1u;
        const uint32_t self = 1u << m;
        const uint32_t zero = ~nz & colmask & ~self;
        zero_agent = live && (zero & amask) != 0u;
        rad = live ? rw & colmask : 0u;
        cand = agent ? cw & colmask : 0u;
        int n = agent ? __popc(zero) : 0;
        if (agent) {
            float Fx = F ? F->x : 0.0f, Fy = F ? F->y : 0.0f;
            const float dmin2_aa = q.dmin2_aa, dmin2_ao = q.dmin2_ao, dmin_aa = q.dmin_aa, dmin_ao = q.dmin_ao;
            for (uint32_t w = cand; w; w &= w - 1u) {
                const int c = __builtin_ctz(w);
                const bool ag = c < N;
                const float2 qc = sp[ag ? c : N + c];
                const float dx = pm.x - qc.x, dy = pm.y - qc.y;
                const float d2 = dx * dx + dy * dy;
                n += d2 < (ag ? dmin2_aa : dmin2_ao) ? 1 : 0;
                if (F) {
                    const float f = contact_scale(q, d2, ag ? dmin_aa : dmin_ao);
                    Fx += f * dx;
                    Fy += f * dy;
                }
            }
            if (F) *F = make_float2(Fx, Fy);
        }
        cnt = n;
    };

    {   // the forces of step t_first: its action, then the stored candidates
        float2 F = roll_force<kFmt>(late_params(), a0, agent);
        if (agent) {
            const float2 pi = x;   // lane m < N: agent m = entity m
            const float dmin_aa = late_params().dmin_aa, dmin_ao = late_params().dmin_ao;
            for (uint32_t w = cand_prev; w; w &= w - 1u) {
                const int c = __builtin_ctz(w);
                const bool ag = c < N;
                const float2 pj = pos_buf(0)[ag ? c : N + c];
                const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                const float d2 = dx * dx + dy * dy;
                const float f = contact_scale(late_params(), d2, ag ? dmin_aa : dmin_ao);
                F.x += f * dx;
                F.y += f * dy;
            }
            s_force[m] = F;
        }
    }

    const int K = p.roll.K, n_act = p.roll.n_actions;
    int arow = p.roll.t_first % n_act;
    // CSR hand-off per wave (gsm_device.h Xfer: each wave publishes its four
    // envs' edge count of step k in iteration k, the last wave of each group
    // of 64 their group sum in iteration k + 2, and step k's edges are written
    // in iteration k + 5 at the offset those give) — no workgroup barrier and
    // no look-back walk in the loop. A hand-off hop under load takes 2-3 us
    // (MI355X_MICROARCH.md handoff-1to1) and a C2 step about 3: every granule
    // a wave reads was published at least an iteration before it is loaded,
    // and the offset loads are issued two iterations before the one that uses
    // them (the group loads one), at the end of an iteration behind the next
    // step's action load (the vector memory counter drains in order, so that
    // load's wait leaves them in flight). (Edges two or three iterations
    // late with the loads at the iteration's start, or four with them one
    // iteration ahead: the offset still settled in ~1900-2200 cycles per
    // step, profiles/r4_stamps.)
    const int w = blockIdx.x * kWavesPerBlock + wave;      // this wave's index in the grid
    const bool glast = (w & 63) == 63;                      // publishes its group's sums
    auto xf = [&]() -> Xfer {
        KernargParams &q = late_params();
        Xfer x;
        x.W = q.roll.xW;
        x.NG = q.roll.xNG;
        x.agg = q.roll.gran;
        x.grp = x.agg + (int64_t)q.roll.K * x.W;
        x.status = q.roll.status;
        x.etag = roll_epoch_tag(q.roll.epoch);
        return x;
    };
    uint32_t row_m1 = 0, row_m2 = 0, row_m3 = 0, row_m4 = 0, row_m5 = 0;   // radius row bits of steps k - 1 .. k - 5
    int cnt_m1 = 0, cnt_m2 = 0;                                // this wave's edge counts of steps k - 1, k - 2
    uint32_t cand_keep = cand_prev;
    bool coinc = false;
    static_assert(kPackDepth == 5, "the row ring below");
    auto ring = [](int i) { return i >= kPackDepth + 1 ? i - (kPackDepth + 1) : i; };
    int cur = 0;   // the buffer holding the positions before step k (those after step k - 5: cur + 2)

    // the edges of step j (positions in buffer `pb`, rows `row`) at the wave's
    // offset `woff`: each env after the wave's earlier envs
    auto emit = [&](const int j, const int pb, const uint32_t row, const int woff) {
        GSM_TNOW(te2);
        KernargParams &qs = late_params();
        // rows in entity order: agent rows (agent columns, own goal, obstacle
        // columns), goal rows, obstacle rows (agent then obstacle columns)
        const int c = live ? __popc(row) + (agent ? 1 : 0) : 0;
        const int incl = seg_scan16(c);
        const int a_total = seg_sum16(agent ? c : 0);
        // env totals (segment sums plus the N goal rows) and the wave's
        // exclusive prefix over its envs
        const int e_tot = env_live ? seg_sum16(c) + N : 0;
        const int t0 = __builtin_amdgcn_readlane(e_tot, 0), t1 = __builtin_amdgcn_readlane(e_tot, 16),
                  t2 = __builtin_amdgcn_readlane(e_tot, 32);
        const int before = (seg > 0 ? t0 : 0) + (seg > 1 ? t1 : 0) + (seg > 2 ? t2 : 0);
        int64_t env_off = (int64_t)woff + before;
        if (woff < 0) {   // a broken hand-off: never write out of bounds
            if (lane == 0)
                __hip_atomic_store((gu32 *)qs.roll.status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            env_off = qs.ro.cap;
        }
        if (env_live && m == 0) {
            int64_t *const eptr = qs.ro.eptr + (kSlots ? j * qs.ro.ep_s : 0);
            eptr[b] = env_off;
            if (b == qs.B - 1) eptr[qs.B] = env_off + e_tot;
        }
        const EdgeSink out = roll_edge_sink<kSlots>(qs, j, K);
        const float2 *sp = pos_buf(pb);
        const int32_t g0 = (int32_t)(eb * E);
        // every column's position read up front (M independent LDS reads in
        // flight at once), then the row's edges in column order from
        // registers: no LDS read waited on inside the per-edge chain (one
        // wave per SIMD here: nothing else hides those latencies)
        float2 qc[M];
#pragma unroll
        for (int cc = 0; cc < M; ++cc) qc[cc] = sp[cc < N ? cc : N + cc];
        const float2 gq = sp[N + (m < N ? m : 0)];
        if (live) {
            int64_t o = env_off + (incl - c) + (m >= N ? N : 0);
            const float2 a = sp[ent];
            auto put = [&](int64_t at, int dst, float2 qd) {
                if (at < out.cap) {
                    const float dx = a.x - qd.x, dy = a.y - qd.y;
                    out.index[at] = g0 + ent;
                    out.index[out.cap + at] = g0 + dst;
                    out.attr[at] = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
                }
            };
#pragma unroll
            for (int cc = 0; cc < N; ++cc)
                if ((row >> cc) & 1u) put(o++, cc, qc[cc]);
            if (agent) {
                put(o++, N + m, gq);                                 // agent m -> its goal
                const float dx = gq.x - a.x, dy = gq.y - a.y;
                const int64_t at = env_off + a_total + m;            // goal row: goal m -> agent m
                if (at < out.cap) {
                    out.index[at] = g0 + N + m;
                    out.index[out.cap + at] = g0 + m;
                    out.attr[at] = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
                }
            }
#pragma unroll
            for (int cc = N; cc < M; ++cc)
                if ((row >> cc) & 1u) put(o++, N + cc, qc[cc]);
        }
        GSM_ACC(late_params(), wid, 4, te2);   // diagnostic builds: emission
    };

    GSM_RSTAMP(p, wid, 8);
    // the first iteration's next-step actions and hand-off loads (the loads
    // unconditional, at valid addresses: a load under a branch leaves the
    // compiler's count of outstanding loads unknown at the join, and every
    // later wait becomes a full drain)
    int nrow = arow + 1 == n_act ? 0 : arow + 1;
    float4 anext = roll_action_load<kN, kFmt>(late_params(), nrow, eb, agent ? m : 0);
    // (the offset loads two iterations ahead: xo for this iteration, xo2 for
    // the next — one iteration of a C2 step was shorter than such a load)
    XferOff xo = xfer_off_load_all(xf(), 0, w, lane);
    XferOff xo2 = xfer_off_load_all(xf(), 0, w, lane);
    uint64_t gl = xfer_grp_load(xf(), 0, w, lane);
    for (int k = 0; k < K; ++k) {
        GSM_TNOW(tc0);
        const float2 *const s_cur = pos_buf(cur);
        float2 *const s_pos = pos_buf(ring(cur + 1));
        KernargParams &pc = late_params();
        // apply_environment_force (formed by the previous sweep) + integrate_state;
        // goals and obstacles carried into the step's buffer
        if (agent) {
            const float2 pi = s_cur[m];
            const float2 F0 = s_force[m];
            float Fx = F0.x, Fy = F0.y;
            if (pc.strict && strict_bad(m, pi, N, M, [&](int c) { return s_cur[c < N ? c : N + c]; })) {
                Fx = __builtin_nanf("");
                Fy = __builtin_nanf("");
            }
            const float dt = pc.dt, max_speed = pc.max_speed;
            v.x = v.x * pc.omd;
            v.y = v.y * pc.omd;
            v.x = v.x + (Fx * pc.inv_mass) * dt;
            v.y = v.y + (Fy * pc.inv_mass) * dt;
            if (max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > max_speed) {
                    v.x = v.x / sp * max_speed;
                    v.y = v.y / sp * max_speed;
                }
            }
            s_pos[m] = make_float2(pi.x + v.x * dt, pi.y + v.y * dt);
        } else if (env_live && m < E) {
            s_pos[m] = s_cur[m];
        }
        wave_sync();
        t += 1;
        const bool done = env_live && t >= pc.EL;

        // observation on the post-physics positions (and the next step's forces)
        float2 pm = live ? s_pos[ent] : make_float2(0.0f, 0.0f);
        uint32_t rad, cand;
        int cnt;
        bool za;
        float2 Fn = roll_force<kFmt>(late_params(), anext, agent);
        sweep(s_pos, pm, rad, cand, cnt, za, &Fn);
        // reward / cost
        float r = 0.0f;
        if (agent) {
            const float2 g = s_pos[N + m];
            const float dx = pm.x - g.x, dy = pm.y - g.y;
            r = -__builtin_amdgcn_sqrtf(dx * dx + dy * dy);
        }
        float rsum = seg_sum16(r);
        const int csum = seg_sum16(agent ? cnt : 0);
        {
            KernargParams &q = late_params();
            if (agent) {
                (q.ro.rew + (kSlots ? k * q.ro.rc_s : 0) + eb * N)[m] = q.shared_reward ? rsum : r;
                (q.ro.cost + (kSlots ? k * q.ro.rc_s : 0) + eb * N)[m] = (float)cnt;
            }
            if (q.shared_reward) rsum *= (float)N;
        }
        if (env_live) {
            acc.x += rsum;
            acc.y += (float)csum;
        }
        const bool reset = done && late_params().auto_reset;
        if (reset && m == 0) late_params().ep_last[b] = acc;
        if (__any(reset)) {
            // auto-reset: scenario.reset_world for the segments whose env is done
            if (reset) {
                ep = ep + 1;
                t = 0;
                acc = make_float2(0.0f, 0.0f);
                v = make_float2(0.0f, 0.0f);
                const uint32_t gid = (uint32_t)(late_params().env_base + b);
                if (m < E) s_pos[m] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)m);
            }
            wave_sync();
            if (reset) {
                pm = live ? s_pos[ent] : make_float2(0.0f, 0.0f);
                Fn = roll_force<kFmt>(late_params(), anext, agent);
                sweep(s_pos, pm, rad, cand, cnt, za, &Fn);
            }
        }
        coinc = (seg_sum16(za ? 1 : 0) != 0);
        if (agent) s_force[m] = Fn;

        // node features: agent rows every step, goal / obstacle rows on a new layout
        KernargParams &q = late_params();
        const bool statics = q.nf_full || reset;
        float *nf = q.ro.nf + (kSlots ? k * q.ro.nf_s : 0) + eb * E * 7;
        if (agent) {
            const float2 g = s_pos[N + m];
            store_row(nf + m * 7, v, pm, make_float2(g.x - pm.x, g.y - pm.y), 0.0f);
        }
        if (env_live && statics && m >= N && m < E) {
            const float2 a = s_pos[m];
            store_row(nf + m * 7, make_float2(0.0f, 0.0f), a, make_float2(0.0f, 0.0f), m < 2 * N ? 1.0f : 2.0f);
        }
        const int edges = seg_sum16(live ? (int)__popc(rad) : 0) + 2 * N;
        if (env_live && m == 0) {
            (q.ro.done + (kSlots ? k * q.ro.done_s : 0))[b] = done ? 1 : 0;
            if (kSlots || k == K - 1) (q.ro.ecount + (kSlots ? k * q.ro.ec_s : 0))[b] = edges;
        }
        // publish the wave's count of this step, then (a group's last wave)
        // the group sum of the previous step
        const int ev = env_live ? edges : 0;
        const int wcnt = __builtin_amdgcn_readlane(ev, 0) + __builtin_amdgcn_readlane(ev, 16) +
                         __builtin_amdgcn_readlane(ev, 32) + __builtin_amdgcn_readlane(ev, 48);
        GSM_ACC(late_params(), wid, 0, tc0);   // diagnostic builds: the step's work
        GSM_TNOW(tc1);
        if (lane == 0) xfer_st(xf().agg + (int64_t)k * xf().W + w, xf().tag(k), (uint32_t)wcnt);
        if (k >= 2 && glast) xfer_grp_publish(xf(), gl, k - 2, w, lane, cnt_m2);
        GSM_ACC(late_params(), wid, 1, tc1);   // publish
        // the edges of step k - 5
        if (k >= kPackDepth) {
            GSM_TNOW(te0);
            const int woff = xfer_off_settle(xf(), xo, k - kPackDepth, w, lane);
            GSM_ACC(late_params(), wid, 3, te0);   // the offset settled
            emit(k - kPackDepth, ring(cur + 2), row_m5, woff);
        }
        row_m5 = row_m4;
        row_m4 = row_m3;
        row_m3 = row_m2;
        row_m2 = row_m1;
        row_m1 = rad;
        cnt_m2 = cnt_m1;
        cnt_m1 = wcnt;
        cand_keep = cand;
        cur = ring(cur + 1);
        arow = nrow;
        // the next iteration's next-step actions, then its hand-off loads
        nrow = arow + 1 == n_act ? 0 : arow + 1;
        anext = roll_action_load<kN, kFmt>(late_params(), nrow, eb, agent ? m : 0);
        xo = xo2;
        xo2 = xfer_off_load_all(xf(), k + 2 >= kPackDepth ? k + 2 - kPackDepth : 0, w, lane);
        gl = xfer_grp_load(xf(), k + 1 >= 2 ? k - 1 : 0, w, lane);
        wave_sync();
    }
    // the tail: the group sums of the last two steps, then the edges of the
    // last five (the first two tail iterations' offset loads and the first's
    // group load were issued by the loop)
    const int fin = cur;   // positions after the last step
    const int last_cnt = cnt_m1;
    const uint32_t last_row = row_m1;
    for (int k = K; k < K + kPackDepth; ++k) {
        if (k > K) {
            xo = k == K + 1 ? xo2 : xfer_off_load_all(xf(), k >= kPackDepth ? k - kPackDepth : 0, w, lane);
            // (clamped to a step of this launch: the load is unconditional, and
            // past the last step it would read beyond the granule allocation)
            gl = xfer_grp_load(xf(), min(max(k - 2, 0), K - 1), w, lane);
        }
        if (k - 2 >= 0 && k - 2 < K && glast) xfer_grp_publish(xf(), gl, k - 2, w, lane, cnt_m2);
        if (k >= kPackDepth)
            emit(k - kPackDepth, ring(cur + 2), row_m5, xfer_off_settle(xf(), xo, k - kPackDepth, w, lane));
        row_m5 = row_m4;
        row_m4 = row_m3;
        row_m3 = row_m2;
        row_m2 = row_m1;
        cnt_m2 = cnt_m1;
        cur = ring(cur + 1);
    }
    GSM_RSTAMP(p, wid, 9);
    // the last step's sums in the config's workgroup layout (G = 4: the same
    // 16 envs per workgroup), for the emit launch that may follow
    if (lane == 0) s_bc[wave] = last_cnt;
    __syncthreads();
    KernargParams &q = late_params();
    if (threadIdx.x == 0 && K >= 1) q.block_edge_sum[blockIdx.x] = s_bc[0] + s_bc[1] + s_bc[2] + s_bc[3];
    // the final state (what the next launch or an eager step reads)
    const float2 *const s_fin = pos_buf(fin);
    if (env_live && m < E) q.pos[eb * E + m] = s_fin[m];
    if (agent) {
        q.vel[eb * N + m] = v;
        q.contact_mask[eb * N + m] = cand_keep;
    }
    if (live) q.row_mask[eb * M + m] = last_row;
    if (env_live && m == 0) {
        q.step_count[b] = t;
        q.episode[b] = ep;
        q.ep_acc[b] = acc;
    }
    if (q.degenerate) {
        const bool nf_agent = agent && nonfinite2(s_fin[m]);
        const bool nfe = seg_sum16(nf_agent ? 1 : 0) != 0;
        if (env_live && m == 0) q.degenerate[b] = (uint8_t)((coinc ? kDegCoincident : 0) | (nfe ? kDegNonfinite : 0));
    }
}

// ---------------------------------------------------------------------------
// The same rollout of small envs with each stepping wave's edge emission on a
// wave of its own (round 6; C2). gsm_roll_pack_kernel's waves are alone on
// their SIMDs (C2's 1024 waves, one per SIMD) and each runs one serial chain
// per step: ~2430 cycles of step, ~1900 of edge emission (15 scattered stores
// per lane) and ~1650 settling the CSR offset (uncached granule loads under
// load, profiles/r4_stamps/stamps_c2.json) — nothing hides any of it. Here a
// workgroup holds its four stepping waves (the same 16 envs, the same per-wave
// hand-off granules) and four emitting waves, one per stepper and on its SIMD:
// a stepper publishes each step's positions (a ring of kPack2Ring LDS buffers)
// and radius row bits (a ring of row words) and moves on; its emitter waits for
// them, settles the offset (its loads for step j + 1 in flight while it emits
// step j) and writes the edges. The two chains overlap. A stepper waits only
// before reusing a ring slot its emitter has not finished (kPack2Ring - 2 steps
// of slack); an emitter waits on its own stepper and, through the granules, on
// steppers of lower index — every wait bounded (kRollSpinTicks, then the
// sticky status word). Hand-offs between the two waves are LDS words: the data
// written, lgkmcnt(0), then the count; the reader re-reads the count with
// s_sleep and reads the data after it. Outputs, operations and their order are
// gsm_roll_pack_kernel's (bit-identical: tests/test_gpu_roll.py).
constexpr int kPack2Ring = 8;   // LDS ring slots: the stepper may run kPack2Ring - 2 steps ahead
#ifndef GSM_PACK2_APREF
#define GSM_PACK2_APREF 3   // steps of actions in flight in a stepper
#endif
#ifndef GSM_PACK2_LAG
#define GSM_PACK2_LAG 3   // steps the stepper is ahead when its emitter starts a step (< kPack2Ring - 2)
#endif
static_assert(GSM_PACK2_LAG + 2 < kPack2Ring, "the stepper must not wait for its lagging emitter");
#ifndef GSM_PACK2_EMITTERS
#define GSM_PACK2_EMITTERS 1   // emitting waves per stepping wave (steps dealt round robin; 2: 2.43, 3: 2.50 vs 2.29 us, profiles/r6_ab/c2_emitters)
#endif
constexpr int kPack2Emitters = GSM_PACK2_EMITTERS;
constexpr int kPack2Block = kWave * kWavesPerBlock * (1 + kPack2Emitters);
template <int kN, int kNo>
constexpr int pack2_lds_stepper() {
    return kPack2Ring * 8 * kPackG * (2 * kN + kNo) + 8 * kPackG * kN + kPack2Ring * 4 * kWave;
}
__device__ __forceinline__ int lds_count_ld(const volatile int *c) {
    asm volatile("" ::: "memory");
    const int v = *c;
    asm volatile("" ::: "memory");
    return v;
}
__device__ __forceinline__ void lds_count_st(volatile int *c, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the data before the count
    *c = v;
}
// wait until *c >= want (wave-uniform); false if the bounded wait gave up
__device__ __forceinline__ bool lds_count_wait(const volatile int *c, int want, uint32_t *status) {
    if (__builtin_expect(lds_count_ld(c) >= want, 1)) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (lds_count_ld(c) >= want) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks) {
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store((gu32 *)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
}

template <int kN, int kNo, int kFmt, bool kSlots>
// (two workgroups per CU: 8192 envs in one residency round)
__global__ __launch_bounds__(kPack2Block) __attribute__((amdgpu_waves_per_eu(2 * (1 + kPack2Emitters)))) void
gsm_roll_pack2_kernel(
    DevParams p) {
    constexpr int N = kN, M = kN + kNo, E = 2 * kN + kNo;
    static_assert(M <= kPackSeg && E <= kPackSeg, "one 16-lane segment per env");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool stepper = wv < kWavesPerBlock;
    // emitter (wv - 4) serves stepper (wv - 4) % 4 and emits its steps
    // j = par (mod kPack2Emitters)
    const int wave = stepper ? wv : (wv - kWavesPerBlock) % kWavesPerBlock;   // the stepper this wave is, or emits for
    const int par = stepper ? 0 : (wv - kWavesPerBlock) / kWavesPerBlock;
    const int lane = threadIdx.x & 63, seg = lane >> 4, m = lane & (kPackSeg - 1);
    const int64_t b = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * kPackG + seg;   // this lane's env
    const bool env_live = b < p.B;
    const bool live = env_live && m < M, agent = live && m < N;
    const int64_t eb = env_live ? b : 0;
    // LDS per stepper: positions [kPack2Ring][G][E] (slot (j + 1) % ring holds
    // the positions after step j, slot 0 those before the launch's first
    // step), the next step's forces [G][N], radius row bits [kPack2Ring][64];
    // then per stepper the steps published and the steps emitted
    unsigned char *const s_st = smem + wave * pack2_lds_stepper<kN, kNo>();
    float2 *const s_w = (float2 *)s_st;
    auto pos_buf = [&](int i) { return s_w + i * kPackG * E + seg * E; };   // this env's rows in slot i
    float2 *const s_force = s_w + kPack2Ring * kPackG * E + seg * N;
    uint32_t *const s_rows = (uint32_t *)(s_w + kPack2Ring * kPackG * E + kPackG * N);
    int *const s_bc = (int *)(smem + kWavesPerBlock * pack2_lds_stepper<kN, kNo>());   // [waves]
    volatile int *const s_done = s_bc + kWavesPerBlock;       // [waves] steps published
    volatile int *const s_emit = s_done + kWavesPerBlock;     // [waves][emitters] last step emitted + 1
    const int ent = m < N ? m : N + m;                        // this lane's collider entity
    const int w = blockIdx.x * kWavesPerBlock + wave;        // the stepper's index in the grid (granules)
    const int K = p.roll.K;
    auto xf = [&]() -> Xfer {
        KernargParams &q = late_params();
        Xfer x;
        x.W = q.roll.xW;
        x.NG = q.roll.xNG;
        x.agg = q.roll.gran;
        x.grp = x.agg + (int64_t)q.roll.K * x.W;
        x.status = q.roll.status;
        x.etag = roll_epoch_tag(q.roll.epoch);
        return x;
    };
    if (lane == 0 && stepper) {
        s_done[wave] = 0;
        for (int e = 0; e < kPack2Emitters; ++e) s_emit[wave * kPack2Emitters + e] = 0;
    }
    __syncthreads();
    // (diagnostic stamps, tools/stamps_c2_roll.py: per stepper wave w, slots
    // 0-2 its step / publish / ring wait, 3-5 its emitter's wait for the step /
    // offset settle / emission, 8-11 start and end of both)
    GSM_RSTAMP(p, w, stepper ? 8 : 10);

    if (!stepper) {
        // ---- the emitter: the edges of every step of its stepper's envs
        auto emit = [&](const int j, const float2 *sp, const uint32_t row, const int woff) {
            KernargParams &qs = late_params();
            const int c = live ? __popc(row) + (agent ? 1 : 0) : 0;
            const int incl = seg_scan16(c);
            const int a_total = seg_sum16(agent ? c : 0);
            const int e_tot = env_live ? seg_sum16(c) + N : 0;
            const int t0 = __builtin_amdgcn_readlane(e_tot, 0), t1 = __builtin_amdgcn_readlane(e_tot, 16),
                      t2 = __builtin_amdgcn_readlane(e_tot, 32);
            const int before = (seg > 0 ? t0 : 0) + (seg > 1 ? t1 : 0) + (seg > 2 ? t2 : 0);
            int64_t env_off = (int64_t)woff + before;
            if (woff < 0) {   // a broken hand-off: never write out of bounds
                if (lane == 0)
                    __hip_atomic_store((gu32 *)qs.roll.status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                env_off = qs.ro.cap;
            }
            // (the bound edge_ptr holds the last step's offsets: with several
            // emitters per stepper an earlier step's could land after it, so
            // in the bound buffers only the last step writes them)
            if (env_live && m == 0 && (kSlots || j == K - 1)) {
                int64_t *const eptr = qs.ro.eptr + (kSlots ? j * qs.ro.ep_s : 0);
                eptr[b] = env_off;
                if (b == qs.B - 1) eptr[qs.B] = env_off + e_tot;
            }
            const EdgeSink out = roll_edge_sink<kSlots>(qs, j, K);
            const int32_t g0 = (int32_t)(eb * E);
            float2 qc[M];
#pragma unroll
            for (int cc = 0; cc < M; ++cc) qc[cc] = sp[cc < N ? cc : N + cc];
            const float2 gq = sp[N + (m < N ? m : 0)];
            const float2 a = sp[ent];
            return [=](void) {
                // (the positions are in registers here: the slot may be reused
                // as soon as the emitted count is out)
                if (!live) return;
                int64_t o = env_off + (incl - c) + (m >= N ? N : 0);
                auto put = [&](int64_t at, int dst, float2 qd) {
                    if (at < out.cap) {
                        const float dx = a.x - qd.x, dy = a.y - qd.y;
                        out.index[at] = g0 + ent;
                        out.index[out.cap + at] = g0 + dst;
                        out.attr[at] = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
                    }
                };
#pragma unroll
                for (int cc = 0; cc < N; ++cc)
                    if ((row >> cc) & 1u) put(o++, cc, qc[cc]);
                if (agent) {
                    put(o++, N + m, gq);                                 // agent m -> its goal
                    const float dx = gq.x - a.x, dy = gq.y - a.y;
                    const int64_t at = env_off + a_total + m;            // goal row: goal m -> agent m
                    if (at < out.cap) {
                        out.index[at] = g0 + N + m;
                        out.index[out.cap + at] = g0 + m;
                        out.attr[at] = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
                    }
                }
#pragma unroll
                for (int cc = N; cc < M; ++cc)
                    if ((row >> cc) & 1u) put(o++, N + cc, qc[cc]);
            };
        };
        // Step j is emitted once the stepper has finished step j + kPack2Lag
        // (or the launch's last): the group sums of step j + 1, published by
        // the groups' last steppers in their iteration j + 3, are then normally
        // complete when this emission's loads for step j + 1 are issued, so the
        // next settle does not re-poll a granule (an uncached round trip each)
        XferOff xo = xfer_off_load_all(xf(), par < K ? par : 0, w, lane);
        for (int j = par; j < K; j += kPack2Emitters) {
            GSM_TNOW(te0);
            if (!lds_count_wait(s_done + wave, min(j + 1 + GSM_PACK2_LAG, K), late_params().roll.status)) break;
            GSM_ACC(late_params(), w, 3, te0);
            GSM_TNOW(te1);
            const uint32_t row = s_rows[(j % kPack2Ring) * kWave + lane];
            const int woff = xfer_off_settle(xf(), xo, j, w, lane);
            GSM_ACC(late_params(), w, 5, te1);
            GSM_TNOW(te2);
            // the next step's offset loads, in flight during this emission
            xo = xfer_off_load_all(xf(), j + kPack2Emitters < K ? j + kPack2Emitters : j, w, lane);
            auto write = emit(j, pos_buf((j + 1) % kPack2Ring), row, woff);
            if (lane == 0) lds_count_st(s_emit + wave * kPack2Emitters + par, j + 1);   // positions in registers
            write();
            GSM_ACC(late_params(), w, 4, te2);
        }
        GSM_RSTAMP(p, w, 11);
    } else {
        // ---- the stepper: gsm_roll_pack_kernel's loop without the emission
        const float2 *pos_g = p.pos + eb * E;
        float2 x = env_live && m < E ? pos_g[m] : make_float2(0.0f, 0.0f);
        float2 v = agent ? p.vel[eb * N + m] : make_float2(0.0f, 0.0f);
        int t = env_live ? p.step_count[eb] : 0, ep = env_live ? p.episode[eb] : 0;
        float2 acc = env_live ? p.ep_acc[eb] : make_float2(0.0f, 0.0f);
        uint32_t cand_prev = agent ? (uint32_t)p.contact_mask[eb * N + m] : 0u;
        const float4 a0 = roll_action_load<kN, kFmt>(p, p.roll.t_first % p.roll.n_actions, eb, agent ? m : 0);
        if (env_live && m < E) pos_buf(0)[m] = x;
        wave_sync();
        auto sweep = [&](const float2 *sp, float2 pm, uint32_t &rad, uint32_t &cand, int &cnt, bool &zero_agent,
                         float2 *F) {
            KernargParams &q = late_params();
            uint32_t r2b1 = __float_as_uint(q.R2) + 1u;
            asm volatile("" : "+v"(r2b1));
            uint32_t cut_aa = __float_as_uint(q.cut2_aa), cut_ao = __float_as_uint(q.cut2_ao);
            asm volatile("" : "+v"(cut_aa), "+v"(cut_ao));
            uint32_t rw = 0, cw = 0, nz = 0;
#pragma unroll
            for (int c = M - 1; c >= 0; --c) {
                const float2 qc = sp[c < N ? c : N + c];
                const float dx = pm.x - qc.x, dy = pm.y - qc.y;
                const uint32_t a = __float_as_uint(__builtin_fabsf(dx * dx) + __builtin_fabsf(dy * dy));
                const uint32_t na = 0u - a;
                const uint32_t cb = (c < N && m < N) ? cut_aa : cut_ao;
                rw = __builtin_amdgcn_alignbit(rw, na & (a - r2b1), 31);
                cw = __builtin_amdgcn_alignbit(cw, na & (a - cb), 31);
                nz = __builtin_amdgcn_alignbit(nz, na, 31);
            }
            constexpr uint32_t colmask = (1u << M) - 1u, amask = (1u << N) - 1u;
            const uint32_t self = 1u << m;
            const uint32_t zero = ~nz & colmask & ~self;
            zero_agent = live && (zero & amask) != 0u;
            rad = live ? rw & colmask : 0u;
            cand = agent ? cw & colmask : 0u;
            int n = agent ? __popc(zero) : 0;
            if (agent) {
                float Fx = F ? F->x : 0.0f, Fy = F ? F->y : 0.0f;
                const float dmin2_aa = q.dmin2_aa, dmin2_ao = q.dmin2_ao, dmin_aa = q.dmin_aa, dmin_ao = q.dmin_ao;
                for (uint32_t wd = cand; wd; wd &= wd - 1u) {
                    const int c = __builtin_ctz(wd);
                    const bool ag = c < N;
                    const float2 qc = sp[ag ? c : N + c];
                    const float dx = pm.x - qc.x, dy = pm.y - qc.y;
                    const float d2 = dx * dx + dy * dy;
                    n += d2 < (ag ? dmin2_aa : dmin2_ao) ? 1 : 0;
                    if (F) {
                        const float f = contact_scale(q, d2, ag ? dmin_aa : dmin_ao);
                        Fx += f * dx;
                        Fy += f * dy;
                    }
                }
                if (F) *F = make_float2(Fx, Fy);
            }
            cnt = n;
        };
        {   // the forces of step t_first: its action, then the stored candidates
            float2 F = roll_force<kFmt>(late_params(), a0, agent);
            if (agent) {
                const float2 pi = x;
                const float dmin_aa = late_params().dmin_aa, dmin_ao = late_params().dmin_ao;
                for (uint32_t wd = cand_prev; wd; wd &= wd - 1u) {
                    const int c = __builtin_ctz(wd);
                    const bool ag = c < N;
                    const float2 pj = pos_buf(0)[ag ? c : N + c];
                    const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                    const float d2 = dx * dx + dy * dy;
                    const float f = contact_scale(late_params(), d2, ag ? dmin_aa : dmin_ao);
                    F.x += f * dx;
                    F.y += f * dy;
                }
                s_force[m] = F;
            }
        }
        const int n_act = p.roll.n_actions;
        int arow = p.roll.t_first % n_act;
        const bool glast = (w & 63) == 63;
        int cnt_m1 = 0, cnt_m2 = 0;
        uint32_t cand_keep = cand_prev, last_row = 0;
        bool coinc = false;
        // The next steps' actions are loaded GSM_PACK2_APREF steps ahead: in
        // gsm_roll_pack_kernel the emission filled the time between an action
        // load and its use in the next iteration's sweep; without it a load one
        // step ahead would be waited for every step (an HBM round trip)
        float4 apf[GSM_PACK2_APREF];
        int prow = arow;   // the row of the last prefetched step
#pragma unroll
        for (int d = 0; d < GSM_PACK2_APREF; ++d) {
            prow = prow + 1 == n_act ? 0 : prow + 1;
            apf[d] = roll_action_load<kN, kFmt>(late_params(), prow, eb, agent ? m : 0);
        }
        uint64_t gl = xfer_grp_load(xf(), 0, w, lane);
        for (int k = 0; k < K; ++k) {
            const float4 anext = apf[0];   // step k + 1's actions
            const float2 *const s_cur = pos_buf(k % kPack2Ring);
            float2 *const s_pos = pos_buf((k + 1) % kPack2Ring);
            // the slot about to be written held step k + 1 - ring's positions:
            // emitted before it is reused
            GSM_TNOW(tw0);
            if (k >= kPack2Ring) {   // step k - ring, emitted by emitter (k - ring) mod emitters
                const int jo = k - kPack2Ring;
                (void)lds_count_wait(s_emit + wave * kPack2Emitters + jo % kPack2Emitters, jo + 1,
                                     late_params().roll.status);
            }
            GSM_ACC(late_params(), w, 2, tw0);
            GSM_TNOW(tc0);
            KernargParams &pc = late_params();
            if (agent) {
                const float2 pi = s_cur[m];
                const float2 F0 = s_force[m];
                float Fx = F0.x, Fy = F0.y;
                if (pc.strict && strict_bad(m, pi, N, M, [&](int c) { return s_cur[c < N ? c : N + c]; })) {
                    Fx = __builtin_nanf("");
                    Fy = __builtin_nanf("");
                }
                const float dt = pc.dt, max_speed = pc.max_speed;
                v.x = v.x * pc.omd;
                v.y = v.y * pc.omd;
                v.x = v.x + (Fx * pc.inv_mass) * dt;
                v.y = v.y + (Fy * pc.inv_mass) * dt;
                if (max_speed > 0.0f) {
                    const float sp = sqrtf(v.x * v.x + v.y * v.y);
                    if (sp > max_speed) {
                        v.x = v.x / sp * max_speed;
                        v.y = v.y / sp * max_speed;
                    }
                }
                s_pos[m] = make_float2(pi.x + v.x * dt, pi.y + v.y * dt);
            } else if (env_live && m < E) {
                s_pos[m] = s_cur[m];
            }
            wave_sync();
            t += 1;
            const bool done = env_live && t >= pc.EL;
            float2 pm = live ? s_pos[ent] : make_float2(0.0f, 0.0f);
            uint32_t rad, cand;
            int cnt;
            bool za;
            float2 Fn = roll_force<kFmt>(late_params(), anext, agent);
            sweep(s_pos, pm, rad, cand, cnt, za, &Fn);
            float r = 0.0f;
            if (agent) {
                const float2 g = s_pos[N + m];
                const float dx = pm.x - g.x, dy = pm.y - g.y;
                r = -__builtin_amdgcn_sqrtf(dx * dx + dy * dy);
            }
            float rsum = seg_sum16(r);
            const int csum = seg_sum16(agent ? cnt : 0);
            {
                KernargParams &q = late_params();
                if (agent) {
                    (q.ro.rew + (kSlots ? k * q.ro.rc_s : 0) + eb * N)[m] = q.shared_reward ? rsum : r;
                    (q.ro.cost + (kSlots ? k * q.ro.rc_s : 0) + eb * N)[m] = (float)cnt;
                }
                if (q.shared_reward) rsum *= (float)N;
            }
            if (env_live) {
                acc.x += rsum;
                acc.y += (float)csum;
            }
            const bool reset = done && late_params().auto_reset;
            if (reset && m == 0) late_params().ep_last[b] = acc;
            if (__any(reset)) {
                if (reset) {
                    ep = ep + 1;
                    t = 0;
                    acc = make_float2(0.0f, 0.0f);
                    v = make_float2(0.0f, 0.0f);
                    const uint32_t gid = (uint32_t)(late_params().env_base + b);
                    if (m < E) s_pos[m] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)m);
                }
                wave_sync();
                if (reset) {
                    pm = live ? s_pos[ent] : make_float2(0.0f, 0.0f);
                    Fn = roll_force<kFmt>(late_params(), anext, agent);
                    sweep(s_pos, pm, rad, cand, cnt, za, &Fn);
                }
            }
            coinc = (seg_sum16(za ? 1 : 0) != 0);
            if (agent) s_force[m] = Fn;
            // the step's row bits for the emitter, then the step published to it
            s_rows[(k % kPack2Ring) * kWave + lane] = rad;
            if (lane == 0) lds_count_st(s_done + wave, k + 1);
            KernargParams &q = late_params();
            const bool statics = q.nf_full || reset;
            float *nf = q.ro.nf + (kSlots ? k * q.ro.nf_s : 0) + eb * E * 7;
            if (agent) {
                const float2 g = s_pos[N + m];
                store_row(nf + m * 7, v, pm, make_float2(g.x - pm.x, g.y - pm.y), 0.0f);
            }
            if (env_live && statics && m >= N && m < E) {
                const float2 a = s_pos[m];
                store_row(nf + m * 7, make_float2(0.0f, 0.0f), a, make_float2(0.0f, 0.0f), m < 2 * N ? 1.0f : 2.0f);
            }
            const int edges = seg_sum16(live ? (int)__popc(rad) : 0) + 2 * N;
            if (env_live && m == 0) {
                (q.ro.done + (kSlots ? k * q.ro.done_s : 0))[b] = done ? 1 : 0;
                if (kSlots || k == K - 1) (q.ro.ecount + (kSlots ? k * q.ro.ec_s : 0))[b] = edges;
            }
            const int ev = env_live ? edges : 0;
            const int wcnt = __builtin_amdgcn_readlane(ev, 0) + __builtin_amdgcn_readlane(ev, 16) +
                             __builtin_amdgcn_readlane(ev, 32) + __builtin_amdgcn_readlane(ev, 48);
            GSM_ACC(late_params(), w, 0, tc0);
            GSM_TNOW(tc1);
            if (lane == 0) xfer_st(xf().agg + (int64_t)k * xf().W + w, xf().tag(k), (uint32_t)wcnt);
            if (k >= 2 && glast) xfer_grp_publish(xf(), gl, k - 2, w, lane, cnt_m2);
            GSM_ACC(late_params(), w, 1, tc1);
            cnt_m2 = cnt_m1;
            cnt_m1 = wcnt;
            cand_keep = cand;
            last_row = rad;
#pragma unroll
            for (int d = 0; d + 1 < GSM_PACK2_APREF; ++d) apf[d] = apf[d + 1];
            prow = prow + 1 == n_act ? 0 : prow + 1;
            apf[GSM_PACK2_APREF - 1] = roll_action_load<kN, kFmt>(late_params(), prow, eb, agent ? m : 0);
            gl = xfer_grp_load(xf(), k + 1 >= 2 ? k - 1 : 0, w, lane);
            wave_sync();
        }
        // the group sums of the last two steps (the first's load issued by the loop)
        for (int k = K; k < K + 2; ++k) {
            if (k > K) gl = xfer_grp_load(xf(), min(max(k - 2, 0), K - 1), w, lane);
            if (k - 2 >= 0 && k - 2 < K && glast) xfer_grp_publish(xf(), gl, k - 2, w, lane, cnt_m2);
            cnt_m2 = cnt_m1;
        }
        // the final state (what the next launch or an eager step reads)
        KernargParams &q = late_params();
        const float2 *const s_fin = pos_buf(K % kPack2Ring);
        if (env_live && m < E) q.pos[eb * E + m] = s_fin[m];
        if (agent) {
            q.vel[eb * N + m] = v;
            q.contact_mask[eb * N + m] = cand_keep;
        }
        if (live) q.row_mask[eb * M + m] = last_row;
        if (env_live && m == 0) {
            q.step_count[b] = t;
            q.episode[b] = ep;
            q.ep_acc[b] = acc;
        }
        if (q.degenerate) {
            const bool nf_agent = agent && nonfinite2(s_fin[m]);
            const bool nfe = seg_sum16(nf_agent ? 1 : 0) != 0;
            if (env_live && m == 0) q.degenerate[b] = (uint8_t)((coinc ? kDegCoincident : 0) | (nfe ? kDegNonfinite : 0));
        }
        if (lane == 0) s_bc[wave] = cnt_m1;   // the last step's count
        GSM_RSTAMP(p, w, 9);
    }
    // the last step's sums in the config's workgroup layout (G = 4: the same
    // 16 envs per workgroup), for the emit launch that may follow
    __syncthreads();
    if (threadIdx.x == 0 && K >= 1) late_params().block_edge_sum[blockIdx.x] = s_bc[0] + s_bc[1] + s_bc[2] + s_bc[3];
}

// Specialisations with compile-time shapes (segment arithmetic folded, G = 1
// collectives for 24 agents) and action formats; anything else runs the
// runtime-shape instantiation.
#define GSM_SEG_SHAPES(X) X(3, 3) X(24, 24)
// rollout shapes: BASELINE's (3, 24 agents) and the reference's zero-shot
// navigation sizes 6 and 12 (readme.md:75)
#define GSM_ROLL_SHAPES(X) X(3, 3) X(6, 6) X(12, 12) X(24, 24)

template <bool LAG>
static const void *pick_step_seg(const DevParams &p) {
#define GSM_PICK(n, no)                                                                       \
    if (p.N == n && p.No == no && p.G == envs_per_wave<n, no>()) {                           \
        switch (p.action_fmt) {                                                               \
            case 0: return reinterpret_cast<const void *>(&gsm_step_seg_kernel<n, no, 0, LAG>); \
            case 1: return reinterpret_cast<const void *>(&gsm_step_seg_kernel<n, no, 1, LAG>); \
            default: return reinterpret_cast<const void *>(&gsm_step_seg_kernel<n, no, 2, LAG>); \
        }                                                                                     \
    }
    GSM_SEG_SHAPES(GSM_PICK)
#undef GSM_PICK
    return reinterpret_cast<const void *>(&gsm_step_seg_kernel<0, 0, -1, LAG>);
}
const void *step_seg_kernel_fn(const DevParams &p) { return pick_step_seg<false>(p); }
const void *lag_step_seg_kernel_fn(const DevParams &p) { return pick_step_seg<true>(p); }

// small shapes run four envs per wave (gsm_roll_pack_kernel)
#define GSM_PACK_SHAPES(X) X(3, 3)
bool roll_packed(const DevParams &p) {
#define GSM_PICK(n, no) if (p.N == n && p.No == no) return true;
    GSM_PACK_SHAPES(GSM_PICK)
#undef GSM_PICK
    return false;
}
int roll_seg_envs_per_block(const DevParams &p) { return roll_packed(p) ? kWavesPerBlock * kPackG : kWavesPerBlock; }
// the packed small-env rollout with its emission on waves of its own
// (gsm_roll_pack2_kernel: 512-thread workgroups, two per CU at most, so up to
// 8192 envs in one residency round; larger batches keep gsm_roll_pack_kernel;
// GSM_PACK_SPLIT=0 keeps it everywhere, an A/B knob)
bool roll_pack_split(const DevParams &p) {
    static const bool on = [] {
        const char *e = getenv("GSM_PACK_SPLIT");
        return !(e && *e && atoi(e) == 0);
    }();
    return on && roll_packed(p) && p.B <= 512 * kWavesPerBlock * kPackG;
}
int roll_block_threads(const DevParams &p) { return roll_pack_split(p) ? kPack2Block : block_threads(p); }

template <bool kSlots, bool kEager = false>
static const void *pick_roll_seg(const DevParams &p) {
    if constexpr (kEager) {   // (one env per wave only: the packed rollout keeps host epochs)
        if (roll_packed(p)) return nullptr;
    } else {
        const bool split = roll_pack_split(p);
#define GSM_PICK(n, no)                                                                                     \
    if (p.N == n && p.No == no) {                                                                           \
        switch (p.action_fmt) {                                                                             \
            case 0: return split ? reinterpret_cast<const void *>(&gsm_roll_pack2_kernel<n, no, 0, kSlots>)  \
                                 : reinterpret_cast<const void *>(&gsm_roll_pack_kernel<n, no, 0, kSlots>);  \
            case 1: return split ? reinterpret_cast<const void *>(&gsm_roll_pack2_kernel<n, no, 1, kSlots>)  \
                                 : reinterpret_cast<const void *>(&gsm_roll_pack_kernel<n, no, 1, kSlots>);  \
            default: return split ? reinterpret_cast<const void *>(&gsm_roll_pack2_kernel<n, no, 2, kSlots>) \
                                  : reinterpret_cast<const void *>(&gsm_roll_pack_kernel<n, no, 2, kSlots>); \
        }                                                                                                   \
    }
        GSM_PACK_SHAPES(GSM_PICK)
#undef GSM_PICK
    }
#define GSM_PICK(n, no)                                                                          \
    if (p.N == n && p.No == no) {                                                                \
        switch (p.action_fmt) {                                                                  \
            case 0: return reinterpret_cast<const void *>(&gsm_roll_seg_kernel<n, no, 0, kSlots, kEager>); \
            case 1: return reinterpret_cast<const void *>(&gsm_roll_seg_kernel<n, no, 1, kSlots, kEager>); \
            default: return reinterpret_cast<const void *>(&gsm_roll_seg_kernel<n, no, 2, kSlots, kEager>); \
        }                                                                                        \
    }
    GSM_ROLL_SHAPES(GSM_PICK)
#undef GSM_PICK
    return nullptr;
}
const void *roll_seg_kernel_fn(const DevParams &p, bool slots) {
    if (p.path != kPathSeg) return nullptr;
    return slots ? pick_roll_seg<true>(p) : pick_roll_seg<false>(p);
}
const void *roll_seg_eager_kernel_fn(const DevParams &p) {
    if (p.path != kPathSeg) return nullptr;
    return pick_roll_seg<false, true>(p);
}
size_t roll_kernel_lds(const DevParams &p) {
#define GSM_PICK(n, no)                                                                             \
    if (p.N == n && p.No == no)                                                                     \
        return roll_pack_split(p) ? (size_t)kWavesPerBlock * pack2_lds_stepper<n, no>() + 4 * kWavesPerBlock * (2 + kPack2Emitters) \
                                  : (size_t)kWavesPerBlock * pack_lds_wave<n, no>() + 4 * kWavesPerBlock;
    GSM_PACK_SHAPES(GSM_PICK)
#undef GSM_PICK
    return (size_t)kWavesPerBlock * roll_lds_wave(p.N, p.E) + 4 * (6 * kWavesPerBlock + 4);
}

const void *emit_seg_kernel_fn(const DevParams &p) {
#define GSM_PICK(n, no) \
    if (p.N == n && p.No == no && p.G == envs_per_wave<n, no>()) \
        return reinterpret_cast<const void *>(&gsm_emit_seg_kernel<n, no>);
    GSM_SEG_SHAPES(GSM_PICK)
#undef GSM_PICK
    return reinterpret_cast<const void *>(&gsm_emit_seg_kernel<0, 0>);
}

}  // namespace gsm
