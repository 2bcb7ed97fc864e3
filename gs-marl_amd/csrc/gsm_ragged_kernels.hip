// gsm_ragged_kernels.hip — ragged batches: navigation, polygon and line envs
// with per-env agent counts in one padded batch (SURVEY.md §8 row a12,
// config C4; semantics in oracle/ragged_ref.py and DESIGN.md §3).
//
//  gsm_step_ragged_kernel  one wave64 per env (N_env <= 32, colliders <= 64).
//                          Lane l holds collider l (agents, then navigation
//                          obstacles) and target l (goal / centre / line end).
//                          World.step physics as the other paths; then, for
//                          polygon/line, the per-step linear sum assignment
//                          of agents to formation slots (scipy's
//                          shortest-augmenting-path solver, restated in
//                          oracle/lsa_ref.py) run one column per lane in
//                          float64 so the assignment equals scipy's, ties
//                          included; reward, collision cost, auto-reset,
//                          node features, radius row masks, edge count.
//  gsm_emit_ragged_kernel  same env->wave mapping: per-lane row emission from
//                          the row masks, the agent<->target edges inserted
//                          in entity order.
//
// Storage per env (E = N_max + T_max + O_max rows): agents [0, N_max),
// targets [N_max, N_max + T_max), obstacles [N_max + T_max, E); rows past the
// env's own counts are padding (node type -1, position 0).
#include <math.h>

#include <mutex>
#include <vector>

#include "gsm_device.h"

namespace gsm {

__constant__ float2 c_unit[kRaggedTable];           // (cos, sin)(2*pi*j/n) at tri(n) + j
__constant__ float c_linet[kRaggedTable];           // j/(n-1) (n == 1: 0.5) at tri(n) + j
__constant__ float c_halfw[kRaggedMaxAgents + 1];   // sqrt(n/3)

__host__ __device__ __forceinline__ int tri(int n) { return n * (n - 1) / 2; }

__device__ __forceinline__ float rl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float2 rl_f2(float2 v, int l) { return make_float2(rl_f(v.x, l), rl_f(v.y, l)); }
__device__ __forceinline__ double rl_d(double v, int l) {
    const long long bits = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// DPP reductions over lanes [0, 32) (the assignment never uses more): within
// rows of 16 via quad perms and half-row / row mirrors, then row 0 broadcast
// into row 1 (row_bcast:15); lane 31 holds the result. Lanes a control does
// not write keep their own value (old = src).
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
    const long long bits = __double_as_longlong(v);
    const int lo = (int)(uint32_t)bits, hi = (int)(uint32_t)(bits >> 32);
    const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, kCtrl, kRowMask, 0xf, false);
    const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, kCtrl, kRowMask, 0xf, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi2 << 32) | (uint32_t)lo2));
}
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ int dpp_keep(int v) {
    return __builtin_amdgcn_update_dpp(v, v, kCtrl, kRowMask, 0xf, false);
}
// exact minimum (values are never NaN; -0 and +0 compare equal downstream)
__device__ __forceinline__ double min32(double v) {
    v = fmin(v, dpp_d<0xB1>(v));          // quad_perm [1,0,3,2]
    v = fmin(v, dpp_d<0x4E>(v));          // quad_perm [2,3,0,1]
    v = fmin(v, dpp_d<0x141>(v));         // row_half_mirror
    v = fmin(v, dpp_d<0x140>(v));         // row_mirror
    v = fmin(v, dpp_d<0x142, 0xa>(v));    // row_bcast:15 -> rows 1, 3
    return rl_d(v, 31);
}
__device__ __forceinline__ int max32(int v) {
    v = max(v, dpp_keep<0xB1>(v));
    v = max(v, dpp_keep<0x4E>(v));
    v = max(v, dpp_keep<0x141>(v));
    v = max(v, dpp_keep<0x140>(v));
    v = max(v, dpp_keep<0x142, 0xa>(v));
    return __builtin_amdgcn_readlane(v, 31);
}
// DPP source whose unwritten lanes read INT_MAX, the identity of min: the
// compiler folds each move into its v_min_i32_dpp
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
// float -> int with the same order for every non-NaN value
__device__ __forceinline__ int f32_order_key(float f) {
    const int b = __float_as_int(f);
    return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ int first_lane(uint64_t m) { return __builtin_ctzll(m); }

struct RShape {
    int N, scn, T, O, M, Tper;   // agents, scenario, targets, obstacles, colliders, targets per agent
    float L, twoL;               // layout half-width
};

template <typename Params>
__device__ __forceinline__ RShape make_shape(const Params &p, int N, int scn) {
    RShape s;
    s.N = N;
    s.scn = scn;
    s.T = scn == kScnNav ? N : (scn == kScnPolygon ? 1 : 2);
    s.O = scn == kScnNav ? N : 0;
    s.M = N + s.O;
    s.Tper = scn == kScnLine ? 2 : 1;
    s.L = p.fixed_L > 0.0f ? p.fixed_L : c_halfw[N];
    s.twoL = s.L * 2.0f;
    return s;
}

// N_env and scenario of global env id gid (oracle/ragged_ref.py: env_shapes)
template <typename Params>
__device__ __forceinline__ RShape draw_shape(const Params &p, int b) {
    const int64_t gid = p.env_base + b;
    int N = p.N, scn = p.scenario;
    if (p.scenario == kScnMixed) {
        const Philox4 x = philox4x32_10(0u, 0u, (uint32_t)gid, kTagShape, p.seed_lo, p.seed_hi);
        N = p.n_min + (int)(((uint64_t)x.x0 * (uint64_t)(p.N - p.n_min + 1)) >> 32);
        scn = (int)((uint64_t)gid % 3u);
    }
    return make_shape(p, N, scn);
}

template <typename Params>
__device__ __forceinline__ float2 layout_at(const Params &p, const RShape &s, uint32_t gid, uint32_t ep,
                                            uint32_t e) {
    const Philox4 x = philox4x32_10(e, ep, gid, kTagLayout, p.seed_lo, p.seed_hi);
    return make_float2(u01(x.x0) * s.twoL - s.L, u01(x.x1) * s.twoL - s.L);
}

// storage row of collider l (agents, then obstacles)
template <typename Params>
__device__ __forceinline__ int collider_row(const Params &p, const RShape &s, int l) {
    return l < s.N ? l : p.N + p.T + (l - s.N);
}

// ---- the pair sweep (lane = collider row m, one pass over the env's
// collider columns c). Every predicate of the step is a function of
// d2 = dx*dx + dy*dy, formed here by VGPR-only integer arithmetic on its bits
// and shifted into per-lane row words (v_alignbit: word = word << 1 | sign),
// with no compare, ballot, lane write or SGPR operand: those all issue through
// the CU's scalar path (~1 instruction per CU and cycle, shared by its four
// SIMDs — tools/probe_issue.hip), which the rest of the step
// already fills. With a = bits(|dx*dx| + |dy*dy|) (non-negative, NaN above
// every finite threshold) and na = -a (negative iff d2 > 0):
//   0 < d2 <= R2     sign(na & (a - (bits(R2) + 1)))
//   0 < d2 < cut2    sign(na & (a - bits(cut2)))
//   d2 != 0          sign(na)
// Columns run in descending order within each 32-bit word, so column c ends at
// bit c mod 32. Collisions (d2 < dmin2 for c != m) are the other zero columns
// plus the candidates with d2 < dmin2 (dmin2 < cut2), counted by the walk over
// the candidate bits, which also forms contact forces where asked for (the
// candidates are exactly the pairs the MPE force loop sums, in ascending c).
struct RowBits {
    uint32_t rad[2], cand[2], nz[2];   // columns [32w, 32w + 32) of word w
};
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t shift_in_sign(uint32_t word, uint32_t x) {
    return __builtin_amdgcn_alignbit(word, x, 31);   // (word << 1) | (x >> 31)
}
// pm: the lane's own position; agent columns c < N at s_pos[c], obstacle
// columns c >= N at s_pos[orow + c] (the storage rows, orow = N_max + T_max - N)
template <typename Params>
__device__ __forceinline__ RowBits ragged_sweep(const Params &p, const float2 *s_pos, float2 pm, int N, int M,
                                                int orow) {
    // thresholds held in VGPRs (opaque to the compiler): a VALU operand in an
    // SGPR would put every column's instruction on the scalar path
    uint32_t r2b1 = __float_as_uint(p.R2) + 1u, cut_aa = __float_as_uint(p.cut2_aa),
             cut_ao = __float_as_uint(p.cut2_ao);
    asm volatile("" : "+v"(r2b1), "+v"(cut_aa), "+v"(cut_ao));
    int zv = 0;                                   // a VGPR zero: column indices kept per lane
    asm volatile("" : "+v"(zv));
    const f32x2 P = {pm.x, pm.y};
    RowBits rb = {{0u, 0u}, {0u, 0u}, {0u, 0u}};
    auto column = [&](float2 q, uint32_t cutb, int w) {
        const f32x2 d = P - (f32x2){q.x, q.y};
        const f32x2 sq = d * d;
        const uint32_t a = __float_as_uint(__builtin_fabsf(sq.x) + __builtin_fabsf(sq.y));
        const uint32_t na = 0u - a;
        rb.rad[w] = shift_in_sign(rb.rad[w], na & (a - r2b1));
        rb.cand[w] = shift_in_sign(rb.cand[w], na & (a - cutb));
        rb.nz[w] = shift_in_sign(rb.nz[w], na);
    };
    // columns [lo, hi) of one class from row base + c, descending
    auto range = [&](int lo, int hi, int base, uint32_t cutb, int w) {
        int r = base + hi - 1 + zv;
        int c = hi - 1;
        for (; c - 1 >= lo; c -= 2, r -= 2) {
            const float2 q1 = s_pos[r], q0 = s_pos[r - 1];
            column(q1, cutb, w);
            column(q0, cutb, w);
        }
        if (c >= lo) column(s_pos[r], cutb, w);
    };
    if (M > 32) {
        const int mid = min(max(N, 32), M);
        range(mid, M, orow, cut_ao, 1);
        range(32, mid, 0, cut_aa, 1);
    }
    const int hi0 = min(M, 32), mid0 = min(N, hi0);
    range(mid0, hi0, orow, cut_ao, 0);
    range(0, mid0, 0, cut_aa, 0);
    return rb;
}
// The sweep's per-lane results for lane (row) m: the radius row mask, the
// collision count (agent rows), contact candidates' forces added to *F when
// kForce, and whether the row has another collider at d2 = 0 in an agent
// column (App. A S16)
template <bool kForce, typename Params>
__device__ __forceinline__ uint64_t ragged_rows(const Params &p, const float2 *s_pos, float2 pm, int N, int M,
                                                int orow, int lane, int *cnt, bool *zero_agent, float2 *F) {
    const RowBits rb = ragged_sweep(p, s_pos, pm, N, M, orow);
    const uint64_t colmask = M >= 64 ? ~0ull : ((1ull << M) - 1ull);
    const uint64_t self = 1ull << (lane & 63);
    const uint64_t rad = ((uint64_t)rb.rad[1] << 32 | rb.rad[0]) & colmask;
    const uint64_t zero = ~((uint64_t)rb.nz[1] << 32 | rb.nz[0]) & colmask & ~self;
    const uint64_t amask = N >= 64 ? ~0ull : ((1ull << N) - 1ull);
    *zero_agent = lane < M && (zero & amask) != 0;
    int n = 0;
    if (lane < N) {
        n = __popcll(zero);
        uint64_t cm = ((uint64_t)rb.cand[1] << 32 | rb.cand[0]) & colmask;
        float Fx = 0.0f, Fy = 0.0f;
        if constexpr (kForce) {
            Fx = F->x;
            Fy = F->y;
        }
        const float dmin2_aa = p.dmin2_aa, dmin2_ao = p.dmin2_ao, dmin_aa = p.dmin_aa, dmin_ao = p.dmin_ao;
        while (cm) {
            const int c = __builtin_ctzll(cm);
            cm &= cm - 1;
            const bool ag = c < N;
            const float2 q = s_pos[ag ? c : orow + c];
            const float dx = pm.x - q.x, dy = pm.y - q.y;
            const float d2 = dx * dx + dy * dy;
            n += d2 < (ag ? dmin2_aa : dmin2_ao) ? 1 : 0;
            if constexpr (kForce) {
                const float f = contact_scale(p, d2, ag ? dmin_aa : dmin_ao);
                Fx += f * dx;
                Fy += f * dy;
            }
        }
        if constexpr (kForce) *F = make_float2(Fx, Fy);
    }
    *cnt = n;
    return lane < M ? rad : 0ull;
}

// slot j (< N) of a polygon/line env from its target positions (lanes 0/1)
template <typename Params>
__device__ __forceinline__ float2 slot_of(const Params &p, const RShape &s, int lane, float2 tp) {
    const int j = lane < s.N ? lane : 0;
    if (s.scn == kScnPolygon) {
        const float2 c = rl_f2(tp, 0);
        const float2 u = c_unit[tri(s.N) + j];
        const float ox = p.form_r * u.x, oy = p.form_r * u.y;
        return make_float2(c.x + ox, c.y + oy);
    }
    const float2 l0 = rl_f2(tp, 0), l1 = rl_f2(tp, 1);
    const float tj = c_linet[tri(s.N) + j];
    const float ex = l1.x - l0.x, ey = l1.y - l0.y;
    return make_float2(l0.x + ex * tj, l0.y + ey * tj);
}

// Per-env warm-start state of the assignment (optional caller buffers,
// gsm_buffers.lsa_v / lsa_col / lsa_stats): the column duals and the matching
// of the env's last assignment, and (hits, solves) counters.
struct LsaWarm {
    double *v;        // [N_max] column duals
    int32_t *col;     // [N_max] column of each row (-1: none)
    int32_t *stats;   // [2] certified warm starts, assignments solved
};

// Square linear sum assignment of N <= 32 agents (rows) to N slots (columns)
// with lane k holding row k and column k. C[i][j] = |p_i - slot_j| in fp32
// (staged in LDS), all dual arithmetic in float64. Returns the lane's column
// (row `lane`), and its cost in *own. The result is scipy's
// linear_sum_assignment(C), ties included:
//
//  * warm start (w.v != nullptr): the previous step's column duals v and
//    matching. Row duals u_i = min_j (C[i][j] - v_j) make every reduced cost
//    r_ij = C[i][j] - u_i - v_j >= 0; each row keeps its previous column when
//    that column attains its minimum (r = 0); the other rows are matched by
//    scipy's augmenting step (below) from this feasible partial state. The
//    result is accepted only with a certificate that it is the UNIQUE optimum:
//    r >= -1e-11 everywhere and |r| <= 1e-11 on the matching, and no
//    alternating cycle among the tight pairs (r <= 1e-9). Any other
//    assignment differs from this one by cycles, each using a pair with
//    r > 1e-9, so it costs at least 1e-9 - N * 1e-11 more (float64 rounding
//    here and in scipy is ~1e-14), and scipy, which returns an optimum,
//    returns this one. Without the certificate (ties, or a state the warm
//    start cannot use):
//  * cold: scipy's rectangular_lsap recurrence from scratch (oracle/lsa_ref.py),
//    rows in order, with its tie rules.
#ifdef GSM_STAMPS   // diagnostic builds: s_memtime at the assignment's phase boundaries
#define LSA_T(k)                                                                   \
    do {                                                                           \
        unsigned long long t_;                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        if (tm && lane == 0) tm[k] = t_;                                           \
    } while (0)
#else
#define LSA_T(k) do { } while (0)
#endif
// LDS of the assignment (lsa_lds_bytes): C row-major at an odd stride S
// (row i, column j at i*S + j: a lane per row reads column j of 32 rows from
// 32 distinct banks), the column duals, and a column -> row scratch.
struct LsaLds {
    float *cost;   // [roundup8(N_max)][S]
    double *v;     // [32] column duals
    double *u;     // [32] row duals
    int *keep;     // [32]
    int S;
};
__device__ __forceinline__ LsaLds lsa_lds(unsigned char *lds, int nmax) {
    const int S = lsa_stride(nmax);
    const int cb = (lsa_cost_bytes(nmax) + 15) & ~15;
    return LsaLds{(float *)lds, (double *)(lds + cb), (double *)(lds + cb + 8 * kRaggedMaxAgents),
                  (int *)(lds + cb + 16 * kRaggedMaxAgents), S};
}

// kColLds: the path loop reads C[i][lane] from the LDS copy instead of a
// 32-register column (the rollout kernel's 64-VGPR budget; one LDS read on the
// loop's chain, same values: identical results).
// s_agent: the agents' positions in LDS (rows 0..N-1: the staged storage
// rows), read as broadcasts when the cost matrix is built
#ifndef GSM_LSA_ROLL_CHUNK
#define GSM_LSA_ROLL_CHUNK 4
#endif
template <bool kColLds = false>
__device__ int wave_lsa(int N, int lane, float2 pa, float2 slot, const float2 *s_agent, const LsaLds &sl, float *own,
                        LsaWarm w, int *iters = nullptr, uint64_t *tm = nullptr) {
    const bool col = lane < N;
    float *const s_cost = sl.cost;
    const int S = sl.S;
    // a non-finite agent position (strict mode, App. A S16; or a caller-written
    // state) has no assignment (scipy raises on such a cost matrix): slot -1,
    // cost NaN
    if (__any(col && nonfinite2(pa))) {
        *own = __builtin_nanf("");
        return -1;
    }
    // column `lane` of C held in registers, C[i][lane] picked by the
    // wave-uniform row i (s_set_gpr_idx): no LDS round trip in the path loop;
    // the LDS copy serves the row-parallel passes and the final cost lookup.
    // Rows in groups of 8 with no per-row branch, so the (correctly rounded)
    // square roots of a group are independent instructions; rows >= N of the
    // last group are computed and never read by the path loop (the column
    // pass gives them u = -inf). Columns N..roundup8(N)-1 of every row hold
    // +inf, so the row passes run whole chunks of 8 with no per-column test.
    float ccol[kColLds ? 1 : kRaggedMaxAgents];
    const int n8 = (N + 7) & ~7;
    const bool pad = !col && lane < n8;
#pragma unroll
    for (int i0 = 0; i0 < kRaggedMaxAgents; i0 += 8) {
        if (i0 < N) {
            float c8[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float2 pi = s_agent[i0 + k];
                const float dx = pi.x - slot.x, dy = pi.y - slot.y;
                c8[k] = sqrtf(dx * dx + dy * dy);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (col || pad) s_cost[(i0 + k) * S + lane] = col ? c8[k] : __builtin_inff();
                if constexpr (!kColLds) ccol[i0 + k] = c8[k];
            }
        } else if constexpr (!kColLds) {
#pragma unroll
            for (int k = 0; k < 8; ++k) ccol[i0 + k] = 0.0f;
        }
    }
    const int ccl = col ? lane : 0;   // kColLds: this lane's column (lanes past N read column 0, never used)
    // LDS operands per wait in the warm start's row / column passes: 8, or 4
    // in the rollout (kColLds), whose 64-VGPR budget spilled the 8-wide chunk's
    // 24 registers to scratch inside the step loop — private lines of every
    // wave, evicted from L2 to HBM
    constexpr int kPassChunk = kColLds ? GSM_LSA_ROLL_CHUNK : 8;
    wave_sync();
    LSA_T(0);
    const double kInf = __builtin_inf();
    double u = 0.0, v = 0.0;
    int col4row = -1, row4col = -1;
    const uint64_t colmask = N >= 64 ? ~0ull : ((1ull << N) - 1);

    // scipy's augmenting step for row `cur` from the current duals and
    // matching: shortest augmenting path, dual update, augmentation. Returns
    // false if no free column was reached (never for finite costs).
    auto augment = [&](int cur) -> bool {
        double spc = kInf;
        // 32-bit order key of spc (below), kept beside it: the key of a new r
        // is formed alongside the comparison instead of after the select;
        // INT_MAX once the column leaves `remaining`
        int key = sel_lanes(colmask, f32_order_key(__builtin_inff()), 0x7fffffff);
        int path = -1;
        int rpos = N - 1 - lane;     // position in scipy's `remaining` list (filled in reverse)
        int nrem = N;
        double minVal = 0.0;
        int i = cur, sink = -1;
        // Wave-uniform bit sets: columns still in `remaining`, rows visited.
        // The iteration has no divergent branch; its chain is: dual of row i
        // and C[i][j] -> reduced cost -> 32-bit minimum key -> (the unique
        // minimum, else an exact f64 reduction among the near ones) -> the
        // column's row.
        uint64_t remm = colmask, srm = 0;
#ifdef GSM_STAMPS
        unsigned long long ta_, tb_, tc_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ta_)::"memory");
#endif
        // a square problem reaches a free column within N scans; the bound
        // only guarantees termination should the invariants ever break
        // One loop exit per iteration (a free column reached, or the guard);
        // the exact-tie reduction is the only other branch and is rare.
        int guard = 0, r4c, jsel;
        do {
#ifdef GSM_STAMPS   // diagnostic builds: path iterations
            if (iters) ++*iters;
#endif
            srm |= 1ull << i;
            const double ui = rl_d(u, i);
            const float cij = kColLds ? s_cost[i * S + ccl] : ccol[i];
            const double r = minVal + (double)cij - ui - v;
            // selects on SGPR lane masks (remm, the update ballot), no per-lane
            // bit extraction on the chain
            const int rkey = f32_order_key((float)r + 0.0f);
            const uint64_t upd = __builtin_amdgcn_ballot_w64(r < spc) & remm;
            path = sel_lanes(upd, i, path);
            spc = sel_lanes(upd, r, spc);
            key = sel_lanes(upd, rkey, key);
            // scipy scans `remaining` in order and keeps the first minimum
            // unless a later equal one is unassigned: the last unassigned
            // minimum in scan order if any, else the first minimum. The
            // minimum is found over a 32-bit key first (spc rounded to float:
            // monotone; -0 folded into +0; in integer order) with one DPP
            // reduction: the lanes whose key equals the smallest key hold
            // every exact minimum, so a single such lane IS the minimum and
            // several (near or exact ties) take the f64 reduction among them;
            // exact ties then take one more reduction over key = 64 + pos
            // (unassigned) or 63 - pos (assigned), larger key winning.
            // Lanes outside `remaining` carry INT_MAX, above every finite key.
            const int kmin = min32_i(key);
            // Columns are lanes 0..31 (N <= 32): 32-bit masks keep the test in
            // SALU. An empty `near` (impossible for finite costs) selects lane
            // 63, whose row4col is -1, and the sink check below rejects it.
            const uint32_t near = (uint32_t)(__builtin_amdgcn_ballot_w64(key == kmin) & remm);
            jsel = near ? __builtin_ctz(near) : 63;
            double m;
            if (__builtin_expect((near & (near - 1)) != 0u, 0)) {   // several near: exact f64 minimum
                m = min32(sel_lanes((uint64_t)near, spc, kInf));
                const uint64_t cand = __builtin_amdgcn_ballot_w64(spc == m) & remm;
                jsel = first_lane(cand);
                if (cand & (cand - 1)) {
                    const int tkey = sel_lanes(cand, row4col == -1 ? 64 + rpos : 63 - rpos, -1);
                    const int kb = max32(tkey);
                    jsel = first_lane(__builtin_amdgcn_ballot_w64(tkey == kb));
                }
            } else {
                m = rl_d(spc, jsel);
            }
            minVal = m;
            r4c = __builtin_amdgcn_readlane(row4col, jsel);
            const int at = __builtin_amdgcn_readlane(rpos, jsel);
            remm &= ~(1ull << jsel);
            key = sel_lanes(1ull << jsel, 0x7fffffff, key);
            nrem -= 1;
            // remaining[index] = remaining[--n]: the lane at the last position
            // moves to jsel's
            rpos = sel_lanes(__builtin_amdgcn_ballot_w64(rpos == nrem) & remm, at, rpos);
            i = r4c;
        } while (r4c >= 0 && ++guard < N);
        if (r4c < 0 && jsel < N) sink = jsel;
#ifdef GSM_STAMPS
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tb_)::"memory");
#endif
        if (sink < 0) return false;   // unreachable for finite costs
        const bool SR = (srm >> lane) & 1, SC = ((colmask & ~remm) >> lane) & 1;
        // dual update (before augmenting: col4row is the previous matching)
        const double spc_c = __shfl(spc, col4row < 0 ? 0 : col4row);
        if (lane == cur) u += minVal;
        else if (SR) u += minVal - spc_c;
        if (SC) v -= minVal - spc;
        // augment along path[] from the sink back to row `cur`
        int j = sink;
        for (int guard = 0; guard <= N; ++guard) {
            const int pi_ = __builtin_amdgcn_readlane(path, j);
            if (lane == j) row4col = pi_;
            const int nj = __builtin_amdgcn_readlane(col4row, pi_);
            if (lane == pi_) col4row = j;
            j = nj;
            if (pi_ == cur) break;
        }
#ifdef GSM_STAMPS   // path-loop and update cycles, summed over the augments
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tc_)::"memory");
        if (tm && lane == 0) {
            tm[6] += tb_ - ta_;
            tm[7] += tc_ - tb_;
        }
#endif
        return true;
    };

    // uniqueness certificate of the current matching and duals: dual
    // feasibility and complementary slackness (to rounding), then no
    // alternating cycle of tight pairs (r <= 1e-9) — the graph with an arc
    // from row i to the row holding column j for every tight unmatched (i, j)
    // is acyclic (peeled sink by sink)
    auto certified = [&](double tau = 1e-9) -> bool {
        // row-parallel: lane i checks row i against the column duals in LDS,
        // by VGPR arithmetic only (no per-column compare or select): the
        // smallest reduced cost over all columns (>= -1e-11 together with
        // |r| <= 1e-11 on the matched column is the same test as per column),
        // and the tight bits r <= tau as the sign of r - succ(tau), shifted in
        // (columns past N hold +inf: never tight)
        if (lane < kRaggedMaxAgents) sl.v[lane] = col ? v : 0.0;
        wave_sync();
        bool good = true;
        uint32_t tight = 0;   // lane i: tight unmatched columns of row i
        if (col) {
            const float *crow = s_cost + lane * S;
            const int ci = col4row;
            const double tau1 = __longlong_as_double(__double_as_longlong(tau) + 1);   // succ(tau), tau > 0
            double rmin = kInf;
            for (int j0 = n8 - 4; j0 >= 0; j0 -= 4) {   // descending: column j ends at bit j
                float cr[4];
                double vj[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    cr[k] = crow[j0 + k];
                    vj[k] = sl.v[j0 + k];
                }
#pragma unroll
                for (int k = 3; k >= 0; --k) {
                    const double r = (double)cr[k] - u - vj[k];
                    rmin = fmin(rmin, r);
                    const uint32_t hi = (uint32_t)((uint64_t)__double_as_longlong(r - tau1) >> 32);
                    tight = __builtin_amdgcn_alignbit(tight, hi, 31);
                }
            }
            const double rc = ci >= 0 ? (double)crow[ci] - u - sl.v[ci] : 0.0;
            good = rmin >= -1e-11 && fabs(rc) <= 1e-11;
            if (ci >= 0) tight &= ~(1u << ci);
        }
        if (!__all(good)) {
#ifdef GSM_STAMPS   // diagnostic builds: why the certificate failed (bits 24+)
            if (iters) *iters |= 2 << 24;
#endif
            return false;
        }
        uint64_t rows = colmask, cols = colmask;   // rows not yet peeled, their columns
        for (int it = 0; it < N && rows; ++it) {
            const bool sink = ((rows >> lane) & 1) && !(tight & (uint32_t)cols);
            const uint64_t sinks = __builtin_amdgcn_ballot_w64(sink);
            if (!sinks) break;                   // every remaining row is on a cycle
            rows &= ~sinks;
            cols &= ~__builtin_amdgcn_ballot_w64(col && row4col >= 0 && ((sinks >> row4col) & 1));
        }
#ifdef GSM_STAMPS
        if (iters && tau == 1e-9) *iters |= (rows == 0 ? 1 : 3) << 24;
#endif
        return rows == 0;
    };

    bool solved = false;
    if (w.v) {
        const double v0 = col ? w.v[lane] : 0.0;    // column duals: lane = column
        const int c0 = col ? w.col[lane] : -1;      // previous matching: lane = row
        if (__all(!col || __builtin_isfinite(v0))) {
            // feasible row duals from the previous v; rows whose previous
            // column still attains their minimum keep it, the others are
            // re-matched by scipy's augmenting step. (Keeping the whole
            // previous matching and restoring feasibility by Bellman-Ford on
            // v certified only 5% of N = 24 polygon steps under random
            // actions — the optimum moves — and cost more than it saved.)
            // Row-parallel: lane i scans row i of C in LDS (independent
            // iterations; u_i = min_j (C[i][j] - v_j) is exact in any order).
            v = v0;
            if (lane < kRaggedMaxAgents) {
                sl.v[lane] = v0;
                sl.keep[lane] = -1;
            }
            wave_sync();
            // lane i: u_i = min_j (C[i][j] - v_j) and rc = C[i][c0_i] - v_c0
            double rc = kInf;
            auto row_pass = [&]() -> double {
                double m = kInf;
                if (col) {
                    const float *crow = s_cost + lane * S;
                    // chunks of 8 columns: every LDS read of a chunk is issued
                    // before the first use (one wait per chunk); columns past
                    // N hold +inf (and v = 0): r = +inf, no per-column test
                    // (the minimum by v_min_f64: no zero of either sign
                    // arises, C - v is +0 when equal, and no NaN)
                    for (int j0 = 0; j0 < n8; j0 += kPassChunk) {
                        float cr[kPassChunk];
                        double vj[kPassChunk];
#pragma unroll
                        for (int k = 0; k < kPassChunk; ++k) {
                            cr[k] = crow[j0 + k];
                            vj[k] = sl.v[j0 + k];
                        }
#pragma unroll
                        for (int k = 0; k < kPassChunk; ++k) m = fmin(m, (double)cr[k] - vj[k]);
                    }
                    // the previous column's reduced cost, the same expression as in the scan
                    rc = (c0 >= 0 && c0 < N) ? (double)crow[c0] - sl.v[c0] : kInf;
                }
                return m;
            };
            double m = row_pass();
            // one column reduction (Jonker-Volgenant's): raise each v_j to its
            // column minimum of C[i][j] - u_i (duals stay feasible), then the
            // row minima again. Fewer rows lose their previous column: 12.2 ->
            // 8.9 of 24 in a polygon simulation (oracle/lsa_ref.py duals,
            // random actions); further rounds keep 8.9.
            // (rows past N get u = -inf: r = +inf, no per-row test)
            if (lane < kRaggedMaxAgents) sl.u[lane] = col ? m : -kInf;
            wave_sync();
            if (col) {
                double cm = kInf;
                for (int i0 = 0; i0 < n8; i0 += kPassChunk) {   // chunks of rows, reads first
                    float cc[kPassChunk];
                    double ui[kPassChunk];
#pragma unroll
                    for (int k = 0; k < kPassChunk; ++k) {
                        cc[k] = s_cost[(i0 + k) * S + lane];
                        ui[k] = sl.u[i0 + k];
                    }
#pragma unroll
                    for (int k = 0; k < kPassChunk; ++k) cm = fmin(cm, (double)cc[k] - ui[k]);
                }
                v = cm;
            }
            wave_sync();
            if (lane < kRaggedMaxAgents) sl.v[lane] = v;
            wave_sync();
            m = row_pass();
            u = col ? m : 0.0;
            // a row keeps its previous column when that column attains its
            // minimum (c0 is a matching, so no column is claimed twice; a
            // duplicate would keep one claimant, any one: the result is used
            // only if certified unique)
            const bool want = col && c0 >= 0 && c0 < N && rc == m;
            if (want) sl.keep[c0] = lane;
            wave_sync();
            const bool kept = want && sl.keep[c0] == lane;
            col4row = kept ? c0 : -1;
            row4col = col ? sl.keep[lane] : -1;
            const uint64_t freerows = __builtin_amdgcn_ballot_w64(col && !kept);
#ifdef GSM_STAMPS   // diagnostic builds: rows the warm start re-augments (high half)
            if (iters) *iters += __popcll(freerows) << 16;
#endif
            LSA_T(1);
            bool ok = true;
            for (uint64_t fr = freerows; fr && ok; fr &= fr - 1) ok = augment(first_lane(fr));
            LSA_T(2);
            solved = ok && certified();
            LSA_T(3);
#ifdef GSM_STAMPS   // diagnostic: would a 1e-13 tight threshold certify it? (code 4)
            if (ok && !solved && iters && ((*iters >> 24) & 0xff) == 3 && certified(1e-13)) *iters += 1 << 24;
#endif
        }
        if (w.stats && lane == 0) {
            w.stats[0] += solved ? 1 : 0;
            w.stats[1] += 1;
        }
    }
    if (!solved) {
        // The cold recurrence is normally the tail of its launch (an env whose
        // warm start could not be certified: exact float32 ties).
        // It runs at raised wave priority so that, until the other waves of
        // its SIMD finish, its dependent chain is issued first (priority only
        // orders issue: results are unchanged; C4 -0.9% per step).
        __builtin_amdgcn_s_setprio(3);
        u = 0.0;
        v = 0.0;
        col4row = -1;
        row4col = -1;
        for (int cur = 0; cur < N; ++cur)
            if (!augment(cur)) break;
        __builtin_amdgcn_s_setprio(0);
    }
    if (w.v && col) {
        w.v[lane] = v;
        w.col[lane] = col4row;
    }
    *own = col && col4row >= 0 ? s_cost[lane * S + col4row] : 0.0f;
    return col ? col4row : -1;
}

// ---------------------------------------------------------------------------
// step kernel
// ---------------------------------------------------------------------------
// `stage` runs once the step's own loads of the env state have been issued
// (the lagged kernel stages the previous step's emission inputs there)
template <class Stage>
__device__ int ragged_env_step(const DevParams &p, const int b, const int lane, unsigned char *lds, Stage &&stage) {
    const int Nmax = p.N, Tmax = p.T, Emax = p.E, Mmax = p.M;
    const int64_t eb = b;
    const LsaLds s_lsa = lsa_lds(lds, Nmax);                    // assignment scratch
    float2 *s_pos = (float2 *)(lds + lsa_lds_bytes(Nmax));      // [E] staged rows
    float2 *pos_b = p.pos + eb * Emax;
    const bool do_reset = p.mode == kModeReset && (p.env_mask == nullptr || p.env_mask[b] != 0);
    const LsaWarm lsa_warm{p.lsa_v ? p.lsa_v + eb * Nmax : nullptr, p.lsa_col ? p.lsa_col + eb * Nmax : nullptr,
                           p.lsa_stats ? p.lsa_stats + 2 * eb : nullptr};
    int t = p.step_count[b];
    int ep = p.episode[b];
    float2 acc = p.ep_acc[b];
    RShape s;
    float2 cp = make_float2(0.0f, 0.0f), tp = cp, v = cp;   // collider pos, target pos, agent vel
    bool relaid = false;

    // scenario.reset_world with the Philox layout: compact entity index =
    // agents, targets, obstacles (a navigation env lays out like the same env
    // of a navigation batch of N_env agents)
    auto relayout = [&]() {
        ep = (p.mode == kModeReset && p.reseed ? -1 : ep) + 1;
        t = 0;
        acc = make_float2(0.0f, 0.0f);
        s = draw_shape(p, b);
        const uint32_t gid = (uint32_t)(p.env_base + b);
        cp = make_float2(0.0f, 0.0f);
        tp = cp;
        v = cp;
        if (lane < s.M) cp = layout_at(p, s, gid, (uint32_t)ep, lane < s.N ? lane : s.N + s.T + (lane - s.N));
        if (lane < s.T) tp = layout_at(p, s, gid, (uint32_t)ep, s.N + lane);
        relaid = true;
    };
    if (do_reset) {
        relayout();
    } else {
        const int32_t sh = p.env_shape[b];
        s = make_shape(p, sh & 0xFF, sh >> 8);
        if (lane < s.M) cp = pos_b[collider_row(p, s, lane)];
        if (lane < s.T) tp = pos_b[Nmax + lane];
        if (lane < s.N) v = p.vel[eb * Nmax + lane];
    }
    stage();

    // the env's colliders and targets at their storage rows of s_pos (the
    // column loops of the pair sweep read them)
    const int orow = Nmax + Tmax;   // obstacle column c at s_pos[orow - N + c]
    auto stage_rows = [&]() {
        if (lane < s.M) s_pos[collider_row(p, s, lane)] = cp;
        if (lane < s.T) s_pos[Nmax + lane] = tp;
        wave_sync();
    };
    bool done = false;
    if (p.mode == kModeStep) {
        // _set_action + apply_environment_force + integrate_state (App. A S3-S6):
        // the action force, then the contacts of the candidate pairs in
        // ascending collider order (ragged_rows)
        float2 F = make_float2(0.0f, 0.0f);
        if (lane < s.N) F = action_force(p, eb * Nmax + lane);
        stage_rows();
        {
            int unused_n;
            bool unused_z;
            (void)ragged_rows<true>(p, s_pos, cp, s.N, s.M, orow - s.N, lane, &unused_n, &unused_z, &F);
        }
        wave_sync();   // s_pos is re-staged after the integration
        float Fx = F.x, Fy = F.y;
        if (p.strict) {   // App. A S16 strict: MPE's 0/0 force (every lane runs the readlanes)
            const bool bad = strict_bad(lane, cp, s.N, s.M, [&](int c) { return rl_f2(cp, c); });
            if (lane < s.N && bad) {
                Fx = __builtin_nanf("");
                Fy = __builtin_nanf("");
            }
        }
        if (lane < s.N) {
            v.x = v.x * p.omd;
            v.y = v.y * p.omd;
            v.x = v.x + (Fx / p.mass) * p.dt;
            v.y = v.y + (Fy / p.mass) * p.dt;
            if (p.max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > p.max_speed) {
                    v.x = v.x / sp * p.max_speed;
                    v.y = v.y / sp * p.max_speed;
                }
            }
            cp.x = cp.x + v.x * p.dt;
            cp.y = cp.y + v.y * p.dt;
        }
        t += 1;
        done = t >= p.EL;
    }

    // collision cost (agent lanes) and radius row masks (collider lanes)
    // (+ coinc: a collider other than the lane's own at d2 = 0 with an agent
    // on either side, App. A S16)
    bool coinc = false;
    auto pair_sweep = [&](int *cnt) {
        stage_rows();
        bool z;
        const uint64_t rm = ragged_rows<false>(p, s_pos, cp, s.N, s.M, orow - s.N, lane, cnt, &z, nullptr);
        coinc = __any(z);
        return rm;
    };
    int cnt = 0;
    uint64_t rmask = pair_sweep(&cnt);
    if (lane >= s.N) cnt = 0;

    // reward: navigation -|p_i - g_i|; polygon/line -C[i][sigma_i]
    float2 slot = make_float2(0.0f, 0.0f);
    int sigma = -1;
    float r = 0.0f;
    if (s.scn == kScnNav) {
        if (lane < s.N) {
            const float dx = cp.x - tp.x, dy = cp.y - tp.y;
            r = -sqrtf(dx * dx + dy * dy);
        }
    } else {
        slot = slot_of(p, s, lane, tp);
        float own;
        int nit = 0;
        GSM_STAMP(p, b, 0);
#ifdef GSM_STAMPS
        sigma = wave_lsa(s.N, lane, cp, slot, s_pos, s_lsa, &own, lsa_warm, &nit, p.stamps ? p.stamps + (int64_t)b * 16 + 4 : nullptr);
#else
        sigma = wave_lsa(s.N, lane, cp, slot, s_pos, s_lsa, &own, lsa_warm, &nit);
#endif
        GSM_STAMP(p, b, 1);
#ifdef GSM_STAMPS
        if (p.stamps && lane == 0) p.stamps[(int64_t)b * 16 + 2] = (uint64_t)nit;
#endif
        r = -own;
    }
    // output base pointers read here (kernarg view), not held across the assignment
    KernargParams &kq = late_params();
    float2 *const pos_out = kq.pos + eb * Emax;
    float rsum = wave_sum(lane < s.N ? r : 0.0f);
    if (p.shared_reward) {
        r = rsum;
        rsum *= (float)s.N;
    }
    if (lane < Nmax) {
        kq.reward[eb * Nmax + lane] = lane < s.N ? r : 0.0f;
        kq.cost[eb * Nmax + lane] = (float)cnt;
    }
    const int csum = wave_sum(cnt);

    if (p.mode == kModeStep) {
        acc.x += rsum;
        acc.y += (float)csum;
        if (done && p.auto_reset) {
            if (lane == 0) kq.ep_last[b] = acc;
            relayout();
            // observation of the new layout
            rmask = pair_sweep(&cnt);
            if (s.scn != kScnNav) {
                slot = slot_of(p, s, lane, tp);
                float own;
                sigma = wave_lsa(s.N, lane, cp, slot, s_pos, s_lsa, &own, lsa_warm);
            }
        }
    }

    // node features [v, p, target - p, type]; target = own goal / assigned slot
    const bool full = p.mode != kModeStep || relaid;   // positions / velocities of every row
    const bool full_nf = full || p.nf_full;              // static node-feature rows
    float2 tgt = tp;
    if (s.scn != kScnNav) {
        const int src = sigma < 0 ? 0 : sigma;
        tgt = make_float2(__shfl(slot.x, src), __shfl(slot.y, src));
    }
    if (lane < s.N) {
        float *nf = kq.node_feat + (eb * Emax + lane) * 7;
        nf[0] = v.x;
        nf[1] = v.y;
        nf[2] = cp.x;
        nf[3] = cp.y;
        nf[4] = tgt.x - cp.x;
        nf[5] = tgt.y - cp.y;
        if (full_nf) nf[6] = 0.0f;
    }
    if (lane < Nmax) kq.assign[eb * Nmax + lane] = (lane < s.N && s.scn != kScnNav) ? sigma : -1;

    if (full_nf) {
        // every storage row: positions (padding 0) and the static node rows
        for (int q = lane; q < Emax; q += kWave) s_pos[q] = make_float2(0.0f, 0.0f);
        wave_sync();
        if (lane < s.M) s_pos[collider_row(p, s, lane)] = cp;
        if (lane < s.T) s_pos[Nmax + lane] = tp;
        wave_sync();
        for (int q = lane; q < Emax; q += kWave) {
            const float2 pq = s_pos[q];
            if (full) pos_out[q] = pq;
            if (q < s.N) continue;   // live agent rows written above
            float type;
            if (q < Nmax) type = -1.0f;
            else if (q < Nmax + Tmax) type = q - Nmax < s.T ? 1.0f : -1.0f;
            else type = q - Nmax - Tmax < s.O ? 2.0f : -1.0f;
            float *nf = kq.node_feat + (eb * Emax + q) * 7;
            nf[0] = 0.0f;
            nf[1] = 0.0f;
            nf[2] = pq.x;
            nf[3] = pq.y;
            nf[4] = 0.0f;
            nf[5] = 0.0f;
            nf[6] = type;
        }
    }
    if (full) {
        if (lane < Nmax) kq.vel[eb * Nmax + lane] = lane < s.N ? v : make_float2(0.0f, 0.0f);
    } else if (lane < s.N) {
        pos_out[lane] = cp;
        kq.vel[eb * Nmax + lane] = v;
    }

    if (lane < s.M) kq.row_mask[eb * Mmax + lane] = rmask;
    const int edges = wave_sum((int)__popcll(rmask)) + 2 * s.N * s.Tper;
    const bool nonfin = __any(lane < s.N && nonfinite2(cp));
    if (lane == 0) {
        if (kq.degenerate)
            kq.degenerate[b] = (uint8_t)((coinc ? kDegCoincident : 0) | (nonfin ? kDegNonfinite : 0));
        kq.step_count[b] = t;
        kq.episode[b] = ep;
        kq.ep_acc[b] = acc;
        kq.done[b] = done ? 1 : 0;
        kq.edge_count[b] = edges;
        if (relaid) kq.env_shape[b] = s.N | (s.scn << 8);
    }
#ifdef GSM_STAMPS
    if (p.stamps && lane == 0) p.stamps[(int64_t)b * 16 + 3] = (uint64_t)(s.N | (s.scn << 8));
#endif
    return edges;
}

template <typename Params>
__device__ void ragged_env_emit_rows(const Params &p, const int b, const int lane, const int64_t off,
                                     const float2 *s_pos, const RShape &s, uint64_t mask, const EdgeSink &out);

// kLag (graph chains, gsm_abi.hip capture_impl): the kernel also emits the
// edges of the PREVIOUS step of its workgroup's envs — functions of this
// launch's input positions, row masks and shapes — into the previous step's
// outputs (p.lag), at the offsets given by the previous launch's
// per-workgroup sums (p.lag.block_sum, env-block order; this launch writes
// its own sums to the other half). This replaces the separate emit launch of
// that step. The kernel's time is set by its slowest env's assignment
// (DESIGN.md §4), so the emission is kept off that env's path: each wave
// stages its env's emission inputs in LDS (while its own state loads are in
// flight), and the waves that finish their step first claim the workgroup's
// four emissions (an LDS counter) — normally the slowest wave claims none.
struct RaggedLagLds {
    int *job, *ready;   // next emission to claim; per wave: inputs staged
    int *cnt, *shape;   // per wave: previous edge count and shape word
    uint64_t *rm;       // [4][64] previous row masks
    float2 *pos;        // [4][E_max] previous positions
};
// at smem + 4 * wave_lds_step + 32 (gsm_kernels.hip step_kernel_lds)
__device__ __forceinline__ RaggedLagLds ragged_lag_lds(unsigned char *base, int E) {
    RaggedLagLds l;
    l.job = (int *)base;
    l.ready = l.job + 4;
    l.cnt = l.job + 8;
    l.shape = l.job + 12;
    l.rm = (uint64_t *)(base + 64);
    l.pos = (float2 *)(base + 64 + 8 * kWave * kWavesPerBlock);
    (void)E;
    return l;
}

template <bool kLag>
__global__ __launch_bounds__(kBlock) void gsm_step_ragged_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave-uniform: env shape, loops and assignment state stay scalar
    // env block of this workgroup (mixed: heaviest first, gsm_abi.hip update_block_order)
    const int blk = p.block_order ? p.block_order[blockIdx.x] : (int)blockIdx.x;
    const int b = blk * kWavesPerBlock + wave;
    const int first = blk * kWavesPerBlock;
    const int nlive = min(kWavesPerBlock, p.B - first);
    int *s_bc = (int *)(smem + kWavesPerBlock * p.wave_lds_step);
    const RaggedLagLds L = ragged_lag_lds(smem + kWavesPerBlock * p.wave_lds_step + 32, p.E);
    int32_t sh = 0;
    uint64_t rm = 0;
    float2 q0 = make_float2(0.0f, 0.0f), q1 = q0;
    int ck = 0;
    if constexpr (kLag) {
        // the emission inputs (E_max <= 3 * 32 rows: two per lane), loaded
        // before the step's: the step's first wait covers them
        const int64_t eb = b < p.B ? b : 0;
        sh = p.env_shape[eb];
        rm = lane < p.M ? p.row_mask[eb * p.M + lane] : 0ull;
        q0 = lane < p.E ? p.pos[eb * p.E + lane] : q0;
        q1 = lane + kWave < p.E ? p.pos[eb * p.E + lane + kWave] : q1;
        ck = p.lag.edge_count[eb];
        if (threadIdx.x < 2 * kWavesPerBlock) L.job[threadIdx.x] = 0;   // job and ready[]
        // LDS only: the barrier does not wait for the loads above
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // the wave's own env's inputs into LDS, before its step overwrites them
    // (every read of a previous edge count or row mask precedes that write)
    auto stage = [&]() {
        if constexpr (kLag) {
            float2 *sp = L.pos + wave * p.E;
            if (lane < p.E) sp[lane] = q0;
            if (lane + kWave < p.E) sp[lane + kWave] = q1;
            L.rm[wave * kWave + lane] = rm;
            if (lane == 0) {
                L.cnt[wave] = ck;
                L.shape[wave] = sh;
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the rows land before the flag
            if (lane == 0) __hip_atomic_store(&L.ready[wave], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    int edges = 0;
    GSM_RSTAMP(p, b, 8);
    if (b < p.B) edges = ragged_env_step(p, b, lane, smem + wave * p.wave_lds_step, stage);
    else stage();
    GSM_RSTAMP(p, b, 9);
    if constexpr (kLag) {
        // claim the workgroup's emissions until none is left
        int j = lane == 0 ? __hip_atomic_fetch_add(L.job, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
        j = __builtin_amdgcn_readfirstlane(j);
        if (j < nlive) {
            // every wave's inputs staged (set early in every wave's step;
            // bounded wait: should it ever run out, nothing is emitted from
            // unstaged LDS and the sticky status word says so)
            bool staged = false;
            for (int spin = 0; spin < (1 << 20) && !staged; ++spin) {
                const int r = lane < nlive ? __hip_atomic_load(&L.ready[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) : 1;
                staged = __all(r != 0);
                if (!staged) __builtin_amdgcn_s_sleep(2);
            }
            if (!staged) {
                if (lane == 0 && p.roll.status)
                    __hip_atomic_store((gu32 *)p.roll.status, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                j = nlive;
            }
            // exclusive prefix of the preceding workgroups' previous sums
            int acc = 0;
#pragma unroll 8
            for (int k = lane; k < blk; k += kWave) acc += p.lag.block_sum[k];
            const int64_t base = wave_sum(acc);
            const int cl = lane < nlive ? L.cnt[lane] : 0;
            while (j < nlive) {
                const int bj = first + j;
                const int64_t off = base + wave_sum(lane < j ? cl : 0);
                if (lane == 0) {
                    p.lag.edge_ptr[bj] = off;
                    if (bj == p.B - 1) p.lag.edge_ptr[p.B] = off + __builtin_amdgcn_readlane(cl, j);
                }
                const int32_t shj = L.shape[j];
                const RShape s = make_shape(p, shj & 0xFF, shj >> 8);
                ragged_env_emit_rows(p, bj, lane, off, L.pos + j * p.E, s, lane < s.M ? L.rm[j * kWave + lane] : 0ull,
                                     EdgeSink{p.lag.edge_index, p.lag.edge_attr, p.lag.cap});
                j = lane == 0 ? __hip_atomic_fetch_add(L.job, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
                j = __builtin_amdgcn_readfirstlane(j);
            }
        }
    }
    if (lane == 0) s_bc[wave] = edges;
    __syncthreads();
    if (threadIdx.x == 0) {
        int sum = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) sum += s_bc[w];
        p.block_edge_sum[blk] = sum;
    }
}

// ---------------------------------------------------------------------------
// edge emitter
// ---------------------------------------------------------------------------
// env b's edges at global offset `off` from its positions staged in LDS
// (s_pos, all E_max rows) and its collider lanes' row masks
template <typename Params>
__device__ void ragged_env_emit_rows(const Params &p, const int b, const int lane, const int64_t off,
                                     const float2 *s_pos, const RShape &s, const uint64_t mask,
                                     const EdgeSink &out) {
    const int Nmax = p.N, Tmax = p.T, Emax = p.E;
    const int64_t eb = b;
    int32_t *const src = out.index;
    int32_t *const dst = out.index + out.cap;
    const int32_t g0 = (int32_t)(eb * Emax);
    const int cnt = __popcll(mask) + (lane < s.N ? s.Tper : 0);
    const int incl = wave_scan(cnt);
    const int agent_total = s.N > 0 ? __builtin_amdgcn_readlane(incl, s.N - 1) : 0;
    // row order: agent rows, target rows (N*Tper edges), obstacle rows
    int64_t o = off + (incl - cnt) + (lane >= s.N ? s.N * s.Tper : 0);
    auto put = [&](int a_row, float2 a, int d_row) {
        if (o < out.cap) {   // redirected outputs may be smaller than the worst case
            const float2 q = s_pos[d_row];
            const float dx = a.x - q.x, dy = a.y - q.y;
            src[o] = g0 + a_row;
            dst[o] = g0 + d_row;
            out.attr[o] = sqrtf(dx * dx + dy * dy);
        }
        ++o;
    };
    if (lane < s.M) {
        const int row = collider_row(p, s, lane);
        const float2 a = s_pos[row];
        const uint64_t amask = s.N >= 64 ? ~0ull : ((1ull << s.N) - 1ull);
        uint64_t am = mask & amask, om = mask & ~amask;
        while (am) {
            const int c = __builtin_ctzll(am);
            am &= am - 1;
            put(row, a, c);
        }
        if (lane < s.N) {
            if (s.scn == kScnNav) {
                put(row, a, Nmax + lane);
            } else {
                put(row, a, Nmax);
                if (s.Tper == 2) put(row, a, Nmax + 1);
            }
        }
        while (om) {
            const int c = __builtin_ctzll(om);
            om &= om - 1;
            put(row, a, Nmax + Tmax + (c - s.N));
        }
    }
    // target rows: goal i -> agent i; centre / line ends -> every agent
    if (lane < s.N) {
        const int64_t tb = off + agent_total;
        if (s.scn == kScnNav) {
            o = tb + lane;
            put(Nmax + lane, s_pos[Nmax + lane], lane);
        } else {
            o = tb + lane;
            put(Nmax, s_pos[Nmax], lane);
            if (s.Tper == 2) {
                o = tb + s.N + lane;
                put(Nmax + 1, s_pos[Nmax + 1], lane);
            }
        }
    }
}

__device__ void ragged_env_emit(const DevParams &p, const int b, const int lane, const int64_t off,
                                unsigned char *lds, const EdgeSink &out) {
    const int64_t eb = b;
    float2 *s_pos = (float2 *)lds;
    const int32_t sh = p.env_shape[b];
    const RShape s = make_shape(p, sh & 0xFF, sh >> 8);
    for (int q = lane; q < p.E; q += kWave) s_pos[q] = p.pos[eb * p.E + q];
    const uint64_t mask = lane < s.M ? p.row_mask[eb * p.M + lane] : 0ull;
    wave_sync();
    ragged_env_emit_rows(p, b, lane, off, s_pos, s, mask, out);
}

__global__ __launch_bounds__(kBlock) void gsm_emit_ragged_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int *s_red = (int *)(smem + kWavesPerBlock * p.wave_lds_emit);
    // exclusive prefix of the step kernel's per-workgroup edge sums
    int acc = 0;
    for (int k = threadIdx.x; k < (int)blockIdx.x; k += kBlock) acc += p.block_edge_sum[k];
    acc = wave_sum(acc);
    if (lane == 0) s_red[wave] = acc;
    __syncthreads();
    int64_t off = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) off += s_red[w];
    const int b0 = blockIdx.x * kWavesPerBlock;
    for (int w = 0; w < wave && b0 + w < p.B; ++w) off += p.edge_count[b0 + w];
    const int b = b0 + wave;
    if (b >= p.B) return;
    if (lane == 0) {
        p.edge_ptr[b] = off;
        if (b == p.B - 1) p.edge_ptr[p.B] = off + p.edge_count[b];
    }
    ragged_env_emit(p, b, lane, off, smem + wave * p.wave_lds_emit, EdgeSink{p.edge_index, p.edge_attr, p.edge_capacity});
}

// ---- the ragged rollout's compact edge lists. A step's edges are first
// expanded, in CSR order, into (source row | destination row << 8) words — rows
// of the env's storage layout — by every lane walking the set bits of its own
// row mask: per bit a v_ffbl, the word and an LDS or HBM write at the row's
// next offset; a lane whose row is exhausted writes a spare word instead (the
// address picked by a bit mask, no compare), so the walk runs the wave's
// longest row with no per-lane branch. Written out (and packed `depth` steps
// later) by all 64 lanes, edge e by lane e mod 64.
__device__ __forceinline__ int ffbl_or_neg(uint32_t x) {   // lowest set bit, -1 for 0
    int r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ int wave_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
// The env's edges of one step in CSR order (agent rows: agent columns, the
// agent's target edges, obstacle columns; target rows; obstacle rows: agent
// then obstacle columns), each through put(at, src_row, dst_row) with
// at < total, or at = spare for a lane with nothing to write. Returns total.
template <typename Params, typename Put>
__device__ __forceinline__ int ragged_expand(const Params &p, const RShape &s, int lane, uint64_t mask,
                                             uint32_t spare, Put &&put) {
    const int Nmax = p.N, orow = p.N + p.T - s.N;
    const uint32_t abits = s.N >= 32 ? ~0u : ((1u << s.N) - 1u);
    const uint32_t am = (uint32_t)mask & abits, om0 = (uint32_t)mask & ~abits, om1 = (uint32_t)(mask >> 32);
    const bool agent = lane < s.N;
    const int na = __popc(am), no0 = __popc(om0), no1 = __popc(om1);
    const int cnt = na + no0 + no1 + (agent ? s.Tper : 0);
    const int incl = wave_scan(cnt);
    const int agent_total = s.N > 0 ? __builtin_amdgcn_readlane(incl, s.N - 1) : 0;
    const int total = __builtin_amdgcn_readlane(incl, kWave - 1) + s.N * s.Tper;
    uint32_t o = (uint32_t)(incl - cnt + (agent ? 0 : s.N * s.Tper));
    const uint32_t src = (uint32_t)(agent ? lane : orow + lane);
    auto walk = [&](uint32_t wd, int n_it, uint32_t rowbase) {
        for (int i = 0; i < n_it; ++i) {
            const int c = ffbl_or_neg(wd);
            const uint32_t none = (uint32_t)(c >> 31);   // all ones once the row is exhausted
            wd &= wd - 1u;
            // (an exhausted row's lane writes the spare word, from a valid row)
            put((none & spare) | (~none & o), src, rowbase + ((uint32_t)c & ~none));
            o += 1u + none;
        }
    };
    walk(am, wave_max(na), 0u);
    if (agent) {   // the agent's own target edges, between its agent and obstacle columns
        if (s.scn == kScnNav) {
            put(o++, src, (uint32_t)(Nmax + lane));
        } else {
            put(o++, src, (uint32_t)Nmax);
            if (s.Tper == 2) put(o++, src, (uint32_t)(Nmax + 1));
        }
    }
    walk(om0, wave_max(no0), (uint32_t)orow);
    walk(om1, wave_max(no1), (uint32_t)(orow + 32));
    if (agent) {   // target rows: goal i -> agent i; centre / line ends -> every agent
        const uint32_t tb = (uint32_t)agent_total;
        if (s.scn == kScnNav) {
            put(tb + lane, (uint32_t)(Nmax + lane), (uint32_t)lane);
        } else {
            put(tb + lane, (uint32_t)Nmax, (uint32_t)lane);
            if (s.Tper == 2) put(tb + s.N + lane, (uint32_t)(Nmax + 1), (uint32_t)lane);
        }
    }
    return total;
}

// ---------------------------------------------------------------------------
// Fused rollout of a ragged batch (GSM_GRAPH_ROLL; config C4)
// ---------------------------------------------------------------------------
// K steps of a graph chain in ONE launch, one env per wave (the wave's index
// in the grid IS its env: identity order), every env's state on chip across
// the steps: collider / target positions and velocities in registers, shape
// and counters in SGPRs; the assignment's warm-start state stays in its
// global buffers. Each step runs exactly the operations of
// ragged_env_step (physics, radius sweep, per-step assignment, reward, cost,
// auto-reset, node features): bit-identical outputs.
//
// What a per-step launch cannot do: let an env run ahead of the others. The
// only thing envs share is the packed CSR offset of their edges, which needs
// the edge counts of every earlier env. So a wave writes its env's edges of
// step t into a slab of its own (fixed stride, in HBM) right after its sweep,
// publishes its count (gsm_device.h Xfer, per-wave granules, group sums), and
// packs the slab into the CSR outputs `depth` steps later, from granules
// loaded at the top of that iteration. A wave whose assignment falls back to
// the cold recurrence (an exact float32 tie) falls behind by a
// few steps without holding anyone: its successors wait only if it is more
// than `depth` steps behind. No barriers. A tail packs the last `depth`
// steps. In the bound buffers the earlier steps' edges go to the library
// scratch (roll_edge_sink): only the last step's may land in the shared
// outputs.
// ---- SIMD-balanced placement (ragged mixed batches). A launch is as slow
// as its most loaded SIMD: every env trails the others by at most `depth`
// steps, and a SIMD's eight waves share its issue. With env e on wave e, a
// SIMD's load is the sum of eight random envs' costs (N from 3 to 24,
// navigation or polygon/line: max / mean ~1.7 over 1024 SIMDs). So each wave
// first learns which SIMD it runs on (HW_ID, XCC_ID), and once every wave has
// registered the envs are dealt by cost: sorted descending (p.roll.place,
// host), stratum r (the wave's rank among its SIMD's waves) holds the
// S = place_S envs r*S .. r*S+S-1, snaked over the SIMDs (SIMD i takes entry
// i of even strata, S-1-i of odd ones). Each SIMD then holds one env of every
// cost stratum. Waits on envs handled by any wave are safe only when every
// wave is resident; that is decided from the registrations: all W arrive
// within kPlaceWaitTicks and exactly place_S SIMDs hold them with no SIMD
// above place_R -> dealt; else (another kernel holds CUs: partial
// residency) env = wave index, whose waits are on earlier-dispatched waves
// only. The decision is identity as soon as the arrival count has not grown
// for kPlaceStallTicks (the non-resident workgroups cannot arrive before the
// resident ones finish), at the latest after kPlaceWaitTicks. Registration
// uses returning atomics only, each wave waits for its own (and makes them
// visible at agent scope) before the workgroup barrier that precedes the
// arrival count, and the deciding wave acquires after it has seen every
// arrival; the words are tagged with this launch's epoch, so nothing needs
// clearing except the arrival / SIMD counters, which the grid's last wave
// zeroes at the end of the launch. A wrong decision cannot go unnoticed:
// every env is claimed by a tagged exchange (a second claim sets status 4, a
// missing env times its successors out), and a dealt slot outside the
// placement table (r >= place_R, i >= place_S, env >= the grid's waves) sets
// status 5 and runs the wave's own index instead of reading past the table.
constexpr uint64_t kPlaceWaitTicks = 40000;    // 400 us of s_memrealtime
constexpr uint64_t kPlaceStallTicks = 5000;    // 50 us without a new arrival
constexpr uint32_t kPlaceIdentity = 1, kPlaceDealt = 2;
__device__ __forceinline__ uint64_t place_ld(const uint64_t *g) {   // a wave-uniform atomic load
    const uint64_t x = gran_ld(g);
    return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32 |
           __builtin_amdgcn_readfirstlane((uint32_t)x);
}
__device__ __forceinline__ uint64_t *place_area(const KernargParams &q) {
    return q.roll.gran + (int64_t)q.roll.K * (q.roll.xW + q.roll.xNG);   // (roll.gran is past the header)
}
// Registration counters are spread over kGroups words (XCC x shader engine)
// so that no word takes more than ~128 atomics per launch.
__device__ int roll_place(const int wg_wave, const uint32_t epoch) {
    KernargParams &q = late_params();
    if (q.roll.place == nullptr) return wg_wave;
    const int lane = threadIdx.x & 63;
    const uint32_t ptag = roll_epoch_tag(epoch) | 0xfffu;
    uint64_t *const A = place_area(q);
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);          // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;   // XCC_ID
    const uint32_t grp = (xcc << 3) | ((hw >> 13) & 7u);                    // XCC, shader engine
    const int key = (int)((grp << 7) | (((hw >> 12) & 1u) << 6) | (((hw >> 8) & 15u) << 2) | ((hw >> 4) & 3u));
    const uint32_t slot = hw & 15u;
    const int R = q.roll.place_R, S = q.roll.place_S;
    if (lane == 0) {   // returning atomics only (results used): each completes before the next is issued
        gu64 *mk = (gu64 *)(A + PlaceArea::kMask + key);
        uint64_t x = __hip_atomic_load(mk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), have;
        for (;;) {
            have = (uint32_t)(x >> 32) == ptag ? x : (uint64_t)ptag << 32;
            if (__hip_atomic_compare_exchange_strong(mk, &x, have | (1ull << slot), __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
        const int before = __popc((uint32_t)have);
        uint64_t sink = 0;
        if (before == 0) {   // the SIMD's first wave: its index within the group
            const uint64_t il = __hip_atomic_fetch_add((gu64 *)(A + PlaceArea::kNsimd + 8 * grp), 1ull,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sink ^= __hip_atomic_exchange((gu64 *)(A + PlaceArea::kRank + key), (uint64_t)ptag << 32 | (uint32_t)il,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (before + 1 > R)
            sink ^= __hip_atomic_exchange((gu64 *)(A + PlaceArea::kBad), (uint64_t)ptag << 32, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(sink));   // the returned values are used: returning atomics
    }
    // each wave's registration complete and visible at agent scope before the
    // workgroup's arrival is counted
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();   // the workgroup's waves have registered: one arrival for all four
    if (threadIdx.x == 0) {
        const uint64_t o = __hip_atomic_fetch_add((gu64 *)(A + PlaceArea::kArrive + 8 * grp), 1ull,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(o));
    }
    // The decision, by workgroup 0's first wave (dispatched first, so always
    // resident): it polls the arrival counters and publishes to one replica
    // of the decision per counter group; every other wave polls its group's
    // replica only (8192 waves polling the counters themselves kept the
    // registrations waiting ~300 us).
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t dec = 0;
    if (wg_wave == 0) {
        int seen = -1;
        uint64_t t_seen = t0;
        for (;;) {
            const uint64_t a = gran_ld(A + PlaceArea::kArrive + 8 * lane);
            const int arrived = wave_total((int)a);
            const uint64_t tn = __builtin_amdgcn_s_memrealtime();
            if (arrived == (int)gridDim.x) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every registration before the reads below
                const uint64_t n = gran_ld(A + PlaceArea::kNsimd + 8 * lane);
                const uint64_t bad = place_ld(A + PlaceArea::kBad);
                dec = (wave_total((int)n) == S && (uint32_t)(bad >> 32) != ptag && !q.roll.place_force)
                          ? kPlaceDealt : kPlaceIdentity;
                break;
            }
            if (arrived != seen) {
                seen = arrived;
                t_seen = tn;
            }
            // partial residency: the arrivals stopped (the rest are waiting
            // for resident workgroups to finish), or the outer bound
            if (tn - t_seen > kPlaceStallTicks || tn - t0 > kPlaceWaitTicks) {
                dec = kPlaceIdentity;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        const uint64_t o = __hip_atomic_exchange((gu64 *)(A + PlaceArea::kMode + 8 * lane),
                                                 (uint64_t)ptag << 32 | dec, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(o));
    } else {
        for (;;) {
            const uint64_t m = place_ld(A + PlaceArea::kMode + 8 * grp);
            if ((uint32_t)(m >> 32) == ptag) {
                dec = (uint32_t)m;
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks) {
                if (lane == 0)
                    __hip_atomic_store((gu32 *)q.roll.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dec = kPlaceIdentity;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    dec = __builtin_amdgcn_readfirstlane(dec);
    GSM_SET(q, wg_wave, 12, (uint64_t)dec);   // diagnostic builds: the decision and its wait
    GSM_SET(q, wg_wave, 13, __builtin_amdgcn_s_memrealtime() - t0);
    if (dec != kPlaceDealt) return wg_wave;
    // stratum r: the wave's rank among its SIMD's waves; i: the SIMD's index
    // (SIMDs of lower groups first)
    const uint64_t mk = place_ld(A + PlaceArea::kMask + key);
    uint64_t rk = place_ld(A + PlaceArea::kRank + key);
    while ((uint32_t)(rk >> 32) != ptag) {   // published before its wave arrived: normally at once
        __builtin_amdgcn_s_sleep(1);
        rk = place_ld(A + PlaceArea::kRank + key);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kRollSpinTicks) {
            if (lane == 0) __hip_atomic_store((gu32 *)q.roll.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return wg_wave;
        }
    }
    const uint64_t nx = lane < (int)grp ? gran_ld(A + PlaceArea::kNsimd + 8 * lane) : 0ull;
    const int i = __builtin_amdgcn_readfirstlane((int)(uint32_t)rk + wave_total((int)nx));
    const int r = __popc((uint32_t)mk & ((1u << slot) - 1u));
    // a dealt slot is inside the table by construction (exactly S SIMDs, none
    // above R waves); checked anyway, so that a wrong decision can never read
    // past the table or run an env index outside the grid
    if (r >= R || i < 0 || i >= S) {
        if (lane == 0) __hip_atomic_store((gu32 *)q.roll.status, 5u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return wg_wave;
    }
    const int pos = r * S + ((r & 1) ? S - 1 - i : i);
    const int env = __builtin_amdgcn_readfirstlane(q.roll.place[pos]);
    if (env < 0 || env >= q.roll.xW) {
        if (lane == 0) __hip_atomic_store((gu32 *)q.roll.status, 5u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return wg_wave;
    }
    if (lane == 0) {
        const uint32_t old = __hip_atomic_exchange((gu32 *)((uint32_t *)(A + PlaceArea::kClaim) + env), ptag,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == ptag) __hip_atomic_store((gu32 *)q.roll.status, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return env;
}

// per wave after the step kernel's LDS: the lane state stashed across the
// assignment, the next step's forces, the row masks, the counts (N_max = 24
// mixed: 3616 + 1328 B per wave, 19.8 KB per workgroup: eight workgroups per
// CU, so 8192 envs take one residency round)
constexpr int kRaggedRollWaveLds = 16 * kRaggedMaxAgents + 8 * kRaggedMaxAgents + 8 * kWave +
                                   ((4 * (kRaggedRollMaxDepth + 1) + 15) & ~15);
template <bool kSlots>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void gsm_roll_ragged_kernel(
    DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t epoch = p.roll.epoch;
    // the env this wave runs (SIMD-balanced placement, or the wave's index)
    const int w = __builtin_amdgcn_readfirstlane(roll_place((int)blockIdx.x * kWavesPerBlock + wave, epoch));
    const int Nmax = p.N, Tmax = p.T, Emax = p.E;
    const bool live = w < p.B;
    const int64_t eb = live ? w : 0;
    unsigned char *lds = smem + wave * (p.wave_lds_step + kRaggedRollWaveLds);
    const LsaLds s_lsa = lsa_lds(lds, Nmax);                    // assignment scratch
    float2 *s_pos = (float2 *)(lds + lsa_lds_bytes(Nmax));      // [E] staged rows
    float4 *s_stash = (float4 *)(lds + p.wave_lds_step);        // [32] lane state across the assignment
    float2 *s_fn = (float2 *)(s_stash + kRaggedMaxAgents);       // [32] the next step's forces
    uint64_t *s_rm = (uint64_t *)(s_fn + kRaggedMaxAgents);      // [64]
    int *s_cnt = (int *)(s_rm + kWave);                          // [depth + 1] the env's edge counts by step
    const int D = p.roll.depth, K = p.roll.K, n_act = p.roll.n_actions;
    int lane = threadIdx.x & 63;
    GSM_RSTAMP(p, w, 0);
#ifdef GSM_STAMPS   // diagnostic builds: where the wave runs
    GSM_SET(p, w, 8, (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4));    // HW_ID
    GSM_SET(p, w, 9, (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20));   // XCC_ID
#endif

    // ---- the state before step t_first
    int t = 0, ep = 0;
    float2 acc = make_float2(0.0f, 0.0f), cp = acc, tp = acc, v = acc;
    RShape s = make_shape(p, 0, kScnNav);                       // an idle wave: no agents, no edges
    if (live) {
        t = p.step_count[eb];
        ep = p.episode[eb];
        acc = p.ep_acc[eb];
        const int32_t sh = p.env_shape[eb];
        s = make_shape(p, sh & 0xFF, sh >> 8);
        const float2 *pos_b = p.pos + eb * Emax;
        if (lane < s.M) cp = pos_b[collider_row(p, s, lane)];
        if (lane < s.T) tp = pos_b[Nmax + lane];
        if (lane < s.N) v = p.vel[eb * Nmax + lane];
    }
    auto xf = [&]() -> Xfer {
        KernargParams &q = late_params();
        Xfer x;
        x.W = q.roll.xW;
        x.NG = q.roll.xNG;
        x.agg = q.roll.gran;   // (past the allocation's 16-byte header already)
        x.grp = x.agg + (int64_t)q.roll.K * x.W;
        x.status = q.roll.status;
        x.etag = roll_epoch_tag(epoch);
        return x;
    };
    // launch parameters read at the point of use (late_params): held across
    // the loop they would not fit the 78-SGPR / 64-VGPR budget
    auto P = [&]() -> KernargParams & { return late_params(); };
    // the env's edge slab at ring position j (step mod depth + 1): slab_e + 1
    // (source row | destination row << 8) words (the last one a spare), then
    // as many f32 distances
    struct Slab {
        uint32_t *word;
        float *attr;
    };
    auto slab_of = [&](const int j) -> Slab {
        KernargParams &q = late_params();
        const int64_t per = 2 * ((int64_t)q.roll.slab_e + 1);
        int32_t *base = q.roll.slab + ((int64_t)j * q.B + eb) * per;
#ifdef GSM_CHECKED   // (gsm_device.h gran_chk) the env's slab inside the slab allocation
        if (base < q.roll.slab || base + per > q.roll.slab_end) {
            __hip_atomic_store((gu32 *)q.roll.status, kStatusOutOfBounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base = q.roll.slab;
        }
#endif
        return Slab{(uint32_t *)base, (float *)(base + q.roll.slab_e + 1)};
    };
    int ring = 0;                    // k mod (depth + 1): the slab / count of the current step
    const bool glast = (w & 63) == 63;
    int arow = p.roll.t_first % n_act;
    int cur_edges = 0;              // the env's edge count of the current step
    uint64_t rmask = 0;             // row masks of the current step (collider lanes)
    bool coinc = false, relaid_any = false;

    // The forces of a step act at the positions the previous step's sweep
    // reads, so one pass over the collider pairs serves both: the sweep of
    // step k also forms the forces of step k + 1. Fn: the agent's force for
    // the next integration — _set_action's force first, then the contacts in
    // collider order, the NaN of App. A S16 strict mode last (the operations
    // and order of ragged_env_step's physics: bit-identical). It waits in LDS
    // (s_fn) until that integration: held in registers across the step it
    // would spill.
    // radius row masks and collision counts (as ragged_env_step) and, with
    // `nxt`, the forces of the step whose actions are in row `row`
    // (the env's colliders and targets staged at their storage rows of s_pos:
    // the sweep's column loops and the emission read them)
    auto pair_sweep = [&](int *cnt, const bool nxt, const int row) {
        if (lane < s.M) s_pos[collider_row(P(), s, lane)] = cp;
        if (lane < s.T) s_pos[Nmax + lane] = tp;
        wave_sync();
        float2 F = make_float2(0.0f, 0.0f);
        if (nxt && lane < s.N) F = roll_action_force(late_params(), row, eb * Nmax + lane);
        bool z;
        const uint64_t rm = ragged_rows<true>(P(), s_pos, cp, s.N, s.M, Nmax + Tmax - s.N, lane, cnt, &z, &F);
        if (nxt && P().strict) {
            const bool bad = strict_bad(lane, cp, s.N, s.M, [&](int c) { return rl_f2(cp, c); });
            if (lane < s.N && bad) F = make_float2(__builtin_nanf(""), __builtin_nanf(""));
        }
        if (nxt && lane < kRaggedMaxAgents) s_fn[lane] = F;
        coinc = __any(z);
        return rm;
    };
    // step k's edge count published, its edges written to the env's slab
    // (from the positions the sweep staged)
    auto publish = [&](const int k) {   // at ring position `ring`
        const int edges = wave_sum((int)__popcll(rmask)) + 2 * s.N * s.Tper;
        if (lane == 0) {
            const Xfer x = xf();
            xfer_st(x.agg + (int64_t)k * x.W + w, x.tag(k), (uint32_t)edges);
            s_cnt[ring] = edges;
        }
        if (live) {
            const Slab sl = slab_of(ring);
            // the assignment's LDS is free here (before this step's assignment,
            // or after the reset's): the list is expanded there when it fits
            uint32_t *const scr = (uint32_t *)lds;
            const int cap = lsa_lds_bytes(Nmax) / 4 - 1;   // the last word is the spare
            if (edges <= cap) {
                (void)ragged_expand(P(), s, lane, rmask, (uint32_t)cap,
                                    [&](uint32_t at, uint32_t a, uint32_t b) { scr[at] = a | b << 8; });
                wave_sync();
                for (int e = lane; e < edges; e += kWave) {
                    const uint32_t wd = scr[e];
                    const float2 pa = s_pos[wd & 0xffu], pb = s_pos[wd >> 8];
                    const float dx = pa.x - pb.x, dy = pa.y - pb.y;
                    sl.word[e] = wd;
                    sl.attr[e] = sqrtf(dx * dx + dy * dy);
                }
            } else {   // straight into the slab (its spare word at slab_e)
                const uint32_t spare = (uint32_t)P().roll.slab_e;
                (void)ragged_expand(P(), s, lane, rmask, spare, [&](uint32_t at, uint32_t a, uint32_t b) {
                    const float2 pa = s_pos[a], pb = s_pos[b];
                    const float dx = pa.x - pb.x, dy = pa.y - pb.y;
                    sl.word[at] = a | b << 8;
                    sl.attr[at] = sqrtf(dx * dx + dy * dy);
                });
            }
        }
        wave_sync();
        cur_edges = edges;
    };
    // step j's edges packed into the CSR outputs at offset `off`
    auto pack = [&](const int j, const int off_in) {   // step j = k - depth: ring position ring + 1
        const int jr = ring == D ? 0 : ring + 1;
        const int cnt = s_cnt[jr];
        int64_t off = off_in;
        if (off < 0) {   // a broken hand-off: never write out of bounds
            if (lane == 0) __hip_atomic_store((gu32 *)P().roll.status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            off = P().ro.cap;
        }
        if (!live) return;
        KernargParams &q = late_params();
        if (lane == 0) {
            int64_t *const eptr = q.ro.eptr + (kSlots ? j * q.ro.ep_s : 0);
            eptr[w] = off;
            if (w == q.B - 1) eptr[q.B] = off + cnt;
        }
        const Slab src = slab_of(jr);
        const EdgeSink dst = roll_edge_sink<kSlots>(q, j, K);
#ifdef GSM_CHECKED   // the slab's words read below lie inside it
        if (cnt > q.roll.slab_e + 1 && lane == 0)
            __hip_atomic_store((gu32 *)q.roll.status, kStatusOutOfBounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        int32_t g0 = (int32_t)(eb * Emax);   // the env's first global node id
        asm volatile("" : "+v"(g0));
        for (int e = lane; e < cnt; e += kWave) {
            if (off + e < dst.cap) {   // a redirected slot may be smaller than the worst case
                const uint32_t wd = src.word[e];
                dst.index[off + e] = g0 + (int32_t)(wd & 0xffu);
                dst.index[dst.cap + off + e] = g0 + (int32_t)(wd >> 8);
                dst.attr[off + e] = src.attr[e];
            }
        }
    };

    {   // the forces of step t_first (its actions, the contacts at the loaded positions)
        int unused;
        (void)pair_sweep(&unused, true, arow);
    }
    for (int k = 0; k < K; ++k) {
        lane = threadIdx.x & 63;
        asm volatile("" : "+v"(lane));
        GSM_TNOW(tk0);
        // (the hand-off's granules are loaded where they are used: published
        // steps earlier, they normally land without a wait, and held across
        // the assignment they would cost the 64-VGPR budget scratch spills)
        // integrate_state (App. A S5-S6) with the forces the previous sweep formed
        const float2 F = lane < kRaggedMaxAgents ? s_fn[lane] : make_float2(0.0f, 0.0f);
        const float Fx = F.x, Fy = F.y;
        const int arow_next = arow + 1 == n_act ? 0 : arow + 1;
        if (lane < s.N) {
            v.x = v.x * P().omd;
            v.y = v.y * P().omd;
            v.x = v.x + (Fx / P().mass) * P().dt;
            v.y = v.y + (Fy / P().mass) * P().dt;
            if (P().max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > P().max_speed) {
                    v.x = v.x / sp * P().max_speed;
                    v.y = v.y / sp * P().max_speed;
                }
            }
            cp.x = cp.x + v.x * P().dt;
            cp.y = cp.y + v.y * P().dt;
        }
        t += 1;
        const bool done = live && t >= P().EL;
        // a group's last wave: the group sum of step k - 1
        GSM_ACC(late_params(), w, 3, tk0);
        GSM_TNOW(tk1);
        if (k >= 1 && glast) xfer_grp_publish(xf(), xfer_grp_load(xf(), k - 1, w, lane), k - 1, w, lane, cur_edges);
        GSM_ACC(late_params(), w, 5, tk1);
        GSM_TNOW(tk2);

        int cnt = 0;
        rmask = pair_sweep(&cnt, k + 1 < K, arow_next);
        if (lane >= s.N) cnt = 0;
        const bool will_reset = done && P().auto_reset;
        if (!will_reset) publish(k);   // ahead of the assignment

        // reward: navigation -|p_i - g_i|; polygon/line -C[i][sigma_i]
        float2 slot = make_float2(0.0f, 0.0f);
        int sigma = -1;
        float r = 0.0f;
        auto assign = [&]() {
            slot = slot_of(P(), s, lane, tp);
            float own;
            KernargParams &q = late_params();
            const LsaWarm lw{q.lsa_v ? q.lsa_v + eb * Nmax : nullptr, q.lsa_col ? q.lsa_col + eb * Nmax : nullptr,
                             q.lsa_stats ? q.lsa_stats + 2 * eb : nullptr};
            // the lane state the assignment does not read waits in LDS (the
            // 64-VGPR budget: held in registers it would spill to scratch)
            // (agents and targets sit in lanes < 32: N_max <= 32; lanes past
            // them hold zeros)
            if (lane < kRaggedMaxAgents) s_stash[lane] = make_float4(v.x, v.y, tp.x, tp.y);
            s_rm[lane] = rmask;
            sigma = wave_lsa<true>(s.N, lane, cp, slot, s_pos, s_lsa, &own, lw);
            const float4 st = lane < kRaggedMaxAgents ? s_stash[lane] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            v = make_float2(st.x, st.y);
            tp = make_float2(st.z, st.w);
            rmask = s_rm[lane];
            return own;
        };
        if (s.scn == kScnNav) {
            if (lane < s.N) {
                const float dx = cp.x - tp.x, dy = cp.y - tp.y;
                r = -sqrtf(dx * dx + dy * dy);
            }
        } else {
            GSM_ACC(late_params(), w, 4, tk2);   // sweep + publish
            GSM_TNOW(tk3);
            r = -assign();
            GSM_ACC(late_params(), w, 6, tk3);   // assignment
        }
        float rsum = wave_sum(lane < s.N ? r : 0.0f);
        if (P().shared_reward) {
            r = rsum;
            rsum *= (float)s.N;
        }
        {
            KernargParams &q = late_params();
            if (live && lane < Nmax) {   // (an idle wave's eb aliases env 0)
                (q.ro.rew + (kSlots ? k * q.ro.rc_s : 0))[eb * Nmax + lane] = lane < s.N ? r : 0.0f;
                (q.ro.cost + (kSlots ? k * q.ro.rc_s : 0))[eb * Nmax + lane] = (float)cnt;
            }
        }
        const int csum = wave_sum(cnt);
        acc.x += rsum;
        acc.y += (float)csum;
        bool relaid = false;
        if (will_reset) {
            // auto-reset: scenario.reset_world (as ragged_env_step's relayout),
            // then the observation of the new layout
            if (lane == 0) late_params().ep_last[eb] = acc;
            ep = ep + 1;
            t = 0;
            acc = make_float2(0.0f, 0.0f);
            s = draw_shape(P(), w);
            const uint32_t gid = (uint32_t)(P().env_base + w);
            cp = make_float2(0.0f, 0.0f);
            tp = cp;
            v = cp;
            if (lane < s.M) cp = layout_at(P(), s, gid, (uint32_t)ep, lane < s.N ? lane : s.N + s.T + (lane - s.N));
            if (lane < s.T) tp = layout_at(P(), s, gid, (uint32_t)ep, s.N + lane);
            relaid = relaid_any = true;
            rmask = pair_sweep(&cnt, k + 1 < K, arow_next);
            if (s.scn != kScnNav) (void)assign();
            publish(k);
        }

        // node features [v, p, target - p, type]; target = own goal / assigned slot
        const bool full_nf = relaid || P().nf_full;
        float2 tgt = tp;
        if (s.scn != kScnNav) {
            const int src = sigma < 0 ? 0 : sigma;
            tgt = make_float2(__shfl(slot.x, src), __shfl(slot.y, src));
        }
        KernargParams &q = late_params();
        float *const nfb = q.ro.nf + (kSlots ? k * q.ro.nf_s : 0) + eb * Emax * 7;
        if (live && lane < s.N) {
            float *nf = nfb + lane * 7;
            nf[0] = v.x;
            nf[1] = v.y;
            nf[2] = cp.x;
            nf[3] = cp.y;
            nf[4] = tgt.x - cp.x;
            nf[5] = tgt.y - cp.y;
            if (full_nf) nf[6] = 0.0f;
        }
        if (live && lane < Nmax) {
            int32_t *const asg = q.ro.asg + (kSlots ? k * q.ro.as_s : 0);
            asg[eb * Nmax + lane] = (lane < s.N && s.scn != kScnNav) ? sigma : -1;
        }
        if (live && full_nf) {
            // the static rows of every storage row (padding: 0, type -1)
            for (int qq = lane; qq < Emax; qq += kWave) s_pos[qq] = make_float2(0.0f, 0.0f);
            wave_sync();
            if (lane < s.M) s_pos[collider_row(P(), s, lane)] = cp;
            if (lane < s.T) s_pos[Nmax + lane] = tp;
            wave_sync();
            for (int qq = lane; qq < Emax; qq += kWave) {
                if (qq < s.N) continue;   // live agent rows written above
                const float2 pq = s_pos[qq];
                float type;
                if (qq < Nmax) type = -1.0f;
                else if (qq < Nmax + Tmax) type = qq - Nmax < s.T ? 1.0f : -1.0f;
                else type = qq - Nmax - Tmax < s.O ? 2.0f : -1.0f;
                float *nf = nfb + qq * 7;
                nf[0] = 0.0f;
                nf[1] = 0.0f;
                nf[2] = pq.x;
                nf[3] = pq.y;
                nf[4] = 0.0f;
                nf[5] = 0.0f;
                nf[6] = type;
            }
            wave_sync();
        }
        if (live && lane == 0) {
            (q.ro.done + (kSlots ? k * q.ro.done_s : 0))[eb] = done ? 1 : 0;
            if (kSlots || k == K - 1) (q.ro.ecount + (kSlots ? k * q.ro.ec_s : 0))[eb] = cur_edges;
        }
        if (k == K - 1 && q.degenerate && lane == 0) {}   // flags written with the final state
        // the edges of step k - depth
        GSM_TNOW(tk4);
        if (k >= D) pack(k - D, xfer_off_settle(xf(), xfer_off_load(xf(), k - D, w, lane), k - D, w, lane));
        GSM_ACC(late_params(), w, 7, tk4);
        arow = arow_next;
        ring = ring == D ? 0 : ring + 1;
    }
    GSM_RSTAMP(late_params(), w, 1);
    // ---- the tail: the last group sums, the last `depth` steps' edges, the
    // last step's edge sums per env block (later eager emit launches)
    for (int k = K; k < K + D; ++k) {
        XferOff xo{0ull, 0ull, 0ull};
        uint64_t xl = 0;
        if (k >= D) xo = xfer_off_load(xf(), k - D, w, lane);
        if (k == K) {
            if (glast) xl = xfer_grp_load(xf(), K - 1, w, lane);
            // block_edge_sum of env block w / 4: its last env adds the others' counts
            const int cfirst = w & ~(kWavesPerBlock - 1);
            if (w == min(cfirst + kWavesPerBlock, P().B) - 1) {
                const Xfer x = xf();
                const uint64_t *g = x.agg + (int64_t)(K - 1) * x.W + cfirst + min(lane, max(w - cfirst - 1, 0));
                const uint32_t cv = xfer_settle(xfer_ld(g), g, lane < w - cfirst, x.tag(K - 1), x.status);
                const int tot = wave_total((int)cv) + cur_edges;
                if (lane == 0) late_params().block_edge_sum[w / kWavesPerBlock] = tot;
            }
            if (glast) xfer_grp_publish(xf(), xl, K - 1, w, lane, cur_edges);
        }
        if (k >= D) pack(k - D, xfer_off_settle(xf(), xo, k - D, w, lane));
        ring = ring == D ? 0 : ring + 1;
    }
    // The grid's last wave has read (directly or through the group sums) a
    // granule of this launch from every wave, so every wave has registered
    // and decided: the placement counters for the next launch (one per lane),
    // and this launch's decision counted
    if (w == xf().W - 1 && late_params().roll.place) {
        KernargParams &q = late_params();
        uint64_t *const A = place_area(q);
        __hip_atomic_store((gu64 *)(A + PlaceArea::kArrive + 8 * lane), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gu64 *)(A + PlaceArea::kNsimd + 8 * lane), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t m = place_ld(A + PlaceArea::kMode);   // (replica 0)
        const bool dealt = (uint32_t)(m >> 32) == (roll_epoch_tag(epoch) | 0xfffu) && (uint32_t)m == kPlaceDealt;
        if (lane == 0)
            __hip_atomic_fetch_add((gu32 *)(q.roll.status + (dealt ? 2 : 1)), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    GSM_RSTAMP(late_params(), w, 2);
    // ---- the final state (what the next launch or an eager step reads)
    if (!live) return;
    KernargParams &q = late_params();
    float2 *const pos_b = q.pos + eb * Emax;
    if (relaid_any) {   // every storage row (padding 0), as a reset writes them
        for (int qq = lane; qq < Emax; qq += kWave) s_pos[qq] = make_float2(0.0f, 0.0f);
        wave_sync();
        if (lane < s.M) s_pos[collider_row(p, s, lane)] = cp;
        if (lane < s.T) s_pos[Nmax + lane] = tp;
        wave_sync();
        for (int qq = lane; qq < Emax; qq += kWave) pos_b[qq] = s_pos[qq];
        if (lane < Nmax) q.vel[eb * Nmax + lane] = lane < s.N ? v : make_float2(0.0f, 0.0f);
    } else if (lane < s.N) {
        pos_b[lane] = cp;
        q.vel[eb * Nmax + lane] = v;
    }
    if (lane < s.M) q.row_mask[eb * p.M + lane] = rmask;
    const bool nonfin = __any(lane < s.N && nonfinite2(cp));
    if (lane == 0) {
        if (q.degenerate) q.degenerate[eb] = (uint8_t)((coinc ? kDegCoincident : 0) | (nonfin ? kDegNonfinite : 0));
        q.step_count[eb] = t;
        q.episode[eb] = ep;
        q.ep_acc[eb] = acc;
        if (relaid_any) q.env_shape[eb] = s.N | (s.scn << 8);
    }
}

const void *roll_ragged_kernel_fn(const DevParams &p, bool slots) {
    if (p.path != kPathRagged) return nullptr;
    return slots ? reinterpret_cast<const void *>(&gsm_roll_ragged_kernel<true>)
                 : reinterpret_cast<const void *>(&gsm_roll_ragged_kernel<false>);
}
size_t roll_ragged_kernel_lds(const DevParams &p) {
    return (size_t)kWavesPerBlock * (p.wave_lds_step + kRaggedRollWaveLds);
}

const void *step_ragged_kernel_fn() { return reinterpret_cast<const void *>(&gsm_step_ragged_kernel<false>); }
const void *lag_step_ragged_kernel_fn() { return reinterpret_cast<const void *>(&gsm_step_ragged_kernel<true>); }
const void *emit_ragged_kernel_fn() { return reinterpret_cast<const void *>(&gsm_emit_ragged_kernel); }

// Host side: the tables come from float64 libm and are rounded to fp32 once,
// exactly as oracle/ragged_ref.py forms them (math.cos/sin/sqrt, same
// operation order), so slots and half-widths agree bit for bit.
hipError_t upload_ragged_tables() {
    static std::mutex mu;
    static bool done[256] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    if (dev >= 0 && dev < 256 && done[dev]) return hipSuccess;
    std::vector<float2> unit(kRaggedTable);
    std::vector<float> lt(kRaggedTable);
    float hw[kRaggedMaxAgents + 1];
    hw[0] = 0.0f;
    for (int n = 1; n <= kRaggedMaxAgents; ++n) {
        hw[n] = (float)sqrt(n / 3.0);
        for (int j = 0; j < n; ++j) {
            const double a = 2.0 * M_PI * j / n;
            unit[tri(n) + j] = make_float2((float)cos(a), (float)sin(a));
            lt[tri(n) + j] = n == 1 ? 0.5f : (float)((double)j / (double)(n - 1));
        }
    }
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_unit), unit.data(), sizeof(float2) * kRaggedTable);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_linet), lt.data(), sizeof(float) * kRaggedTable);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_halfw), hw, sizeof hw);
    if (e == hipSuccess && dev >= 0 && dev < 256) done[dev] = true;
    return e;
}

}  // namespace gsm
