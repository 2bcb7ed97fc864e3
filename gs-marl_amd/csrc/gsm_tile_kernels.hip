// gsm_tile_kernels.hip — navigation envs with more than 64 colliders
// (BASELINE config C3: 96 agents, 96 obstacles -> 192 colliders, 288 entities).
//
// One 512-thread workgroup (8 waves) per env: a wave per env would leave one
// wave per SIMD at C3 (1024 envs on 1024 SIMDs) with nothing to hide the
// O(M^2) pair loops' latency. Entity positions live in LDS; the work is split
// over the workgroup:
//
//  gsm_step_tile_kernel  force pass over the contact candidates recorded by
//                        the previous step's sweep (sparse: pairs within the
//                        contact cutoff), integrate, then one sweep over all
//                        collider rows (wave w: rows w, w+8, ...; lanes =
//                        64-collider chunks) ballots the radius adjacency,
//                        the next contact candidates and the collisions into
//                        mask words (row_mask / contact_mask, W = ceil(M/64)
//                        words per row). Node features: agent rows every
//                        step, static rows on layout change.
//  gsm_emit_tile_kernel  thread = a contiguous run of rows; counts from the
//                        mask popcounts, a workgroup scan, then each thread
//                        walks its rows' set bits and writes the row-major
//                        COO edges with their distances.
//
// Same arithmetic contract as the other paths (d2 = dx*dx + dy*dy without
// contraction, squared predicates).
#include "gsm_device.h"

namespace gsm {

constexpr int kTileWaves = kTileBlock / kWave;

// workgroup sums (every thread gets the total); s_red holds kTileWaves slots
__device__ __forceinline__ int tile_sum(int v, int *s_red) {
    const int wave = threadIdx.x >> 6;
    v = wave_total(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[wave] = v;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int w = 0; w < kTileWaves; ++w) t += s_red[w];
    return t;
}
__device__ __forceinline__ float tile_sum(float v, float *s_red) {
    const int wave = threadIdx.x >> 6;
    v = wave_total(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[wave] = v;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < kTileWaves; ++w) t += s_red[w];
    return t;
}

// Post-step sweep over every collider row r (wave w takes rows w, w+8, ...):
// lane l of chunk k holds collider c = 64k + l; one ballot per (row, chunk)
// and predicate yields the row's words of
//   rad     c != r, 0 < d2 <= R^2           -> row_mask  [B][M][W]
//   contact c != r, 0 < d2 < cut^2 (agents) -> contact_mask [B][N][W]
//            (the next step's force pass visits only these pairs: its
//             pre-step positions are exactly these post-step positions)
//   collide c != r, d2 < dmin^2 (agents)    -> cost (popcount)
// Row positions are held one per lane and broadcast with v_readlane (no LDS
// in the inner loop); words are gathered into lane j (the wave's j-th row of
// the group) with v_writelane and stored by that lane. Obstacle rows keep
// their obstacle-only words (static within an episode) when `keep_oo`.
// Returns this thread's share of the directed radius pair count and leaves
// agent collision counts in s_cost.
template <int kW>   // mask words per row; 0 = runtime p.W
__device__ __forceinline__ int obs_sweep(const DevParams &p, const float2 *s_pos, int *s_cost, int64_t eb,
                                         bool keep_oo, int *s_coinc) {
    const int N = p.N, M = p.M, W = kW > 0 ? kW : p.W;
    constexpr int kR = kW > 0 ? kW : 1;     // words held in registers per pass
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int rows_w = (M - wave + kTileWaves - 1) / kTileWaves;   // rows r = wave + 8j
    const int arows_w = N > wave ? (N - wave + kTileWaves - 1) / kTileWaves : 0;   // agent rows first
    uint64_t *const rmask = p.row_mask + eb * M * W;
    uint64_t *const cmask = p.contact_mask + eb * N * W;
    // obstacle rows recompute only the chunks holding agent columns when the
    // obstacle-only words are still valid (same layout as the last sweep)
    const int kc_obst = keep_oo ? (N + 63) / 64 : W;
    // t = bits(d2) - 1:  0 < d2 <= R^2 <=> t <u bits(R^2);  0 < d2 < cut^2 <=>
    // t <u bits(cut^2) - 1 (d2 is never negative). Both exclude the row's own
    // column (d2 = 0) by themselves; lanes past M hold an infinite position.
    const uint32_t R2b = (uint32_t)__float_as_int(p.R2);
    int pairs = 0;   // per lane: set bits of the words it stores / keeps
    bool zc = false;   // an agent row with a collider other than itself at d2 = 0 (App. A S16)
    for (int g0 = 0; g0 < rows_w; g0 += kWave) {
        const int ng = min(kWave, rows_w - g0);
        const int ja = min(ng, max(0, arows_w - g0));   // rows [0, ja) of the group are agent rows
        const int rl = wave + kTileWaves * (g0 + lane);
        const float2 rowp = lane < ng ? s_pos[collider_entity(rl, N)] : make_float2(0.0f, 0.0f);
        uint32_t cnt = 0;   // lane j: collisions of its row (own column included)
        for (int k0 = 0; k0 < W; k0 += kR) {
            float2 q[kR];
            float dmin2[kR];
            uint32_t cutb[kR];
            uint32_t rad_lo[kR], rad_hi[kR], con_lo[kR], con_hi[kR];
#pragma unroll
            for (int u = 0; u < kR; ++u) {
                const int c = 64 * (k0 + u) + lane;
                q[u] = c < M ? s_pos[collider_entity(c, N)] : make_float2(__builtin_inff(), __builtin_inff());
                dmin2[u] = c < N ? p.dmin2_aa : p.dmin2_ao;
                cutb[u] = (uint32_t)__float_as_int(c < N ? p.cut2_aa : p.cut2_ao) - 1u;
                con_lo[u] = con_hi[u] = 0;
                uint64_t old = 0;
                if (k0 + u >= kc_obst && k0 + u < W && lane >= ja && lane < ng)
                    old = rmask[(int64_t)rl * W + k0 + u];   // obstacle-only word: unchanged
                rad_lo[u] = (uint32_t)old;
                rad_hi[u] = (uint32_t)(old >> 32);
            }
            for (int j = 0; j < ja; ++j) {   // agent rows: radius, contact, collision
                const float ax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rowp.x), j));
                const float ay = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rowp.y), j));
                uint32_t ncol = 0;
#pragma unroll
                for (int u = 0; u < kR; ++u) {
                    if (kW == 0 && k0 + u >= W) break;
                    const float dx = ax - q[u].x, dy = ay - q[u].y;
                    const float d2 = dx * dx + dy * dy;
                    const uint32_t tb = (uint32_t)__float_as_int(d2) - 1u;
                    const uint64_t rad = __builtin_amdgcn_ballot_w64(tb < R2b);
                    const uint64_t con = __builtin_amdgcn_ballot_w64(tb < cutb[u]);
                    ncol += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(d2 < dmin2[u]));
                    const int rj = wave + kTileWaves * (g0 + j), cb = 64 * (k0 + u);
                    const uint64_t self = (rj >= cb && rj < cb + 64) ? 1ull << (rj - cb) : 0ull;
                    zc |= (__builtin_amdgcn_ballot_w64(d2 == 0.0f) & ~self) != 0;
                    rad_lo[u] = writelane_u32((uint32_t)rad, (uint32_t)j, rad_lo[u]);
                    rad_hi[u] = writelane_u32((uint32_t)(rad >> 32), (uint32_t)j, rad_hi[u]);
                    con_lo[u] = writelane_u32((uint32_t)con, (uint32_t)j, con_lo[u]);
                    con_hi[u] = writelane_u32((uint32_t)(con >> 32), (uint32_t)j, con_hi[u]);
                }
                cnt = writelane_u32(__builtin_amdgcn_readlane(cnt, j) + ncol, (uint32_t)j, cnt);
            }
            const int kc = min(kR, kc_obst - k0);   // chunks computed for obstacle rows
            for (int j = ja; j < ng; ++j) {  // obstacle rows: radius only
                const float ax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rowp.x), j));
                const float ay = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rowp.y), j));
#pragma unroll
                for (int u = 0; u < kR; ++u) {
                    if (u >= kc) break;
                    const float dx = ax - q[u].x, dy = ay - q[u].y;
                    const float d2 = dx * dx + dy * dy;
                    const uint32_t tb = (uint32_t)__float_as_int(d2) - 1u;
                    const uint64_t rad = __builtin_amdgcn_ballot_w64(tb < R2b);
                    rad_lo[u] = writelane_u32((uint32_t)rad, (uint32_t)j, rad_lo[u]);
                    rad_hi[u] = writelane_u32((uint32_t)(rad >> 32), (uint32_t)j, rad_hi[u]);
                }
            }
            if (lane < ng) {
#pragma unroll
                for (int u = 0; u < kR; ++u) {
                    const int k = k0 + u;
                    if (kW == 0 && k >= W) break;
                    pairs += __popc(rad_lo[u]) + __popc(rad_hi[u]);
                    if (lane >= ja && k >= kc_obst) continue;   // kept word: already stored
                    rmask[(int64_t)rl * W + k] = ((uint64_t)rad_hi[u] << 32) | rad_lo[u];
                    if (lane < ja) cmask[(int64_t)rl * W + k] = ((uint64_t)con_hi[u] << 32) | con_lo[u];
                }
            }
        }
        if (lane < ja) s_cost[rl] = (int)cnt - (nonfinite2(rowp) ? 0 : 1);   // minus the row's own column (NaN row: d2 NaN)
    }
    if (zc) *s_coinc = 1;
    return pairs;
}

// Symmetric sweep (when its LDS fits, p.tile_sym): lanes are ROWS and the
// loop runs over agent COLUMNS, as on the one-env-per-wave path. A unit is
// (row chunk c, 8 agent columns j0..j0+7): per column j the wave ballots the
// rows m of chunk c with rad'(m, j) = d2 <= R^2 and near(m, j) = d2 < cut^2 —
// by symmetry agent row j's words c of the radius and contact-candidate
// masks. Each agent pair is evaluated once per (chunk, column) instead of
// once from each side, on column pairs staged for packed-f32 distances
// (s_xy: [x_j x_j+1 y_j y_j+1]); obstacle rows collect their agent-column
// bits with one v_addc per column (a byte per unit), their obstacle-obstacle
// bits stay cached (keep_oo) or are recomputed on a new layout. Agent rows
// then walk their near bits: collisions (d2 < dmin^2 implies d2 < cut^2) and
// the stored candidates without the self and coincident pairs; a coincident
// pair anywhere in the env (never seen in practice) re-derives every row with
// the exact 0 < d2 <= R^2. Same outputs as obs_sweep.
struct TileSymLds {
    float *xy;        // [ceil(N/2)][4]
    uint64_t *arow;   // [N][2W]: radius words, then near words of agent rows
    uint64_t *own;    // [No][W]: agent-column bits of obstacle rows
    int *flag;        // coincident pair seen
};

__device__ __forceinline__ uint64_t agent_bits_of_word(int N, int k) {   // agent columns of mask word k
    const int lo = 64 * k;
    return N <= lo ? 0ull : (N >= lo + 64 ? ~0ull : ((1ull << (N - lo)) - 1ull));
}

// rout: where the row masks go; rkeep: where the cached obstacle-obstacle
// words are read (keep_oo) — the same buffer except in the fused rollout,
// which double-buffers the masks in LDS (the previous step's are emitted
// later); cout: where the contact words go (LDS in the rollout)
// kN > 0: a compiled shape (kN agents, kNo obstacles), else the config's
#define GSM_TILE_SHAPE(p)                                                 \
    const int N = kN > 0 ? kN : (p).N, No = kN > 0 ? kNo : (p).No;        \
    const int M = N + No, E = 2 * N + No;                                 \
    const int W = kN > 0 ? (kN + kNo + 63) / 64 : (p).W;                  \
    (void)M, (void)E, (void)W, (void)No
template <int kN = 0, int kNo = 0>
__device__ __forceinline__ int obs_sweep_sym(const DevParams &p, const float2 *s_pos, const TileSymLds &S,
                                             int *s_cost, int64_t eb, bool keep_oo, uint64_t *rout = nullptr,
                                             const uint64_t *rkeep = nullptr, uint64_t *cout = nullptr) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    GSM_TILE_SHAPE(p);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int NB8 = (N + 7) >> 3, NP = (N + 1) >> 1;
    const float2 far = make_float2(1.0e18f, 1.0e18f);       // d2 ~ 1e36: every predicate false
    for (int j = tid; j < 2 * NP; j += kTileBlock) {
        const float2 a = j < N ? s_pos[j] : far;
        const int at = (j >> 1) * 4 + (j & 1);
        S.xy[at] = a.x;
        S.xy[at + 2] = a.y;
    }
    for (int k = tid; k < No * W; k += kTileBlock) S.own[k] = 0ull;
    if (tid == 0) *S.flag = 0;
    __syncthreads();
    const float R2 = p.R2;
    const int U = W * NB8;
    GSM_TNOW(ts0);
    for (int u = wave; u < U; u += kTileWaves) {
        const int c = u / NB8, jb = u - c * NB8;
        const int m = 64 * c + lane;
        const bool live = m < M, obst = live && m >= N;
        const float2 pm = live ? s_pos[collider_entity(m, N)] : far;
        const float cut2 = obst ? p.cut2_ao : p.cut2_aa;
        const f32x2 px = {pm.x, pm.x}, py = {pm.y, pm.y};
        const int j0 = 8 * jb, nc = min(8, N - j0);
        const float4 *xy4 = (const float4 *)S.xy + (j0 >> 1);
        uint32_t rlo = 0, rhi = 0, nlo = 0, nhi = 0, own = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (2 * q >= nc) break;
            const float4 Q = xy4[q];
            const f32x2 dx = px - (f32x2){Q.x, Q.y}, dy = py - (f32x2){Q.z, Q.w};
            const f32x2 d2 = dx * dx + dy * dy;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 2 * q + h;
                if (k >= nc) break;
                const float dd = h ? d2.y : d2.x;
                const uint64_t br = __builtin_amdgcn_ballot_w64(dd <= R2);
                const uint64_t bn = __builtin_amdgcn_ballot_w64(dd < cut2);
                own = shl1_add_lane(own, br);
                rlo = writelane_u32((uint32_t)br, (uint32_t)k, rlo);
                rhi = writelane_u32((uint32_t)(br >> 32), (uint32_t)k, rhi);
                nlo = writelane_u32((uint32_t)bn, (uint32_t)k, nlo);
                nhi = writelane_u32((uint32_t)(bn >> 32), (uint32_t)k, nhi);
            }
        }
        if (lane < nc) {
            uint64_t *ar = S.arow + (int64_t)(j0 + lane) * 2 * W;
            ar[c] = ((uint64_t)rhi << 32) | rlo;
            ar[W + c] = ((uint64_t)nhi << 32) | nlo;
        }
        // obstacle row m, agent columns j0.. j0+nc-1: byte jb of its words
        if (obst) ((uint8_t *)(S.own + (int64_t)(m - N) * W))[jb] = (uint8_t)(__builtin_bitreverse32(own) >> (32 - nc));
    }
    GSM_ACC(p, blockIdx.x * kTileWaves + wave, 1, ts0);   // diagnostic builds: column pass
    __syncthreads();
    uint64_t *const rmask = rout ? rout : p.row_mask + eb * M * W;
    const uint64_t *const rprev = rkeep ? rkeep : rmask;
    const bool rewrite = rprev != rmask;                    // every word is written
    uint64_t *const cmask = cout ? cout : p.contact_mask + eb * N * W;
    int pairs = 0, coinc = 0;
    for (int r = tid; r < M; r += kTileBlock) {
        const float2 a = s_pos[collider_entity(r, N)];
        if (r < N) {
            const uint64_t *ar = S.arow + (int64_t)r * 2 * W;
            int cnt = 0;
#pragma unroll 1
            for (int k = 0; k < W; ++k) {
                const uint64_t self = k == (r >> 6) ? 1ull << (r & 63) : 0ull;
                const uint64_t rad = ar[k] & ~self;
                uint64_t near = ar[W + k] & ~self, cand = near;
                while (near) {
                    const int b = __builtin_ctzll(near);
                    near &= near - 1;
                    const int ci = 64 * k + b;
                    const float2 q = s_pos[collider_entity(ci, N)];
                    const float dx = a.x - q.x, dy = a.y - q.y;
                    const float d2 = dx * dx + dy * dy;
                    cnt += d2 < (ci < N ? p.dmin2_aa : p.dmin2_ao) ? 1 : 0;
                    if (d2 == 0.0f) {
                        cand &= ~(1ull << b);
                        coinc = 1;
                    }
                }
                rmask[(int64_t)r * W + k] = rad;
                cmask[(int64_t)r * W + k] = cand;
                pairs += __popcll(rad);
            }
            s_cost[r] = cnt;
        } else {
            const uint64_t *ow = S.own + (int64_t)(r - N) * W;
#pragma unroll 1
            for (int k = 0; k < W; ++k) {
                const uint64_t am = agent_bits_of_word(N, k);
                uint64_t oo = 0;
                if (keep_oo) {
                    oo = rprev[(int64_t)r * W + k] & ~am;   // obstacle-obstacle bits: static in an episode
                } else {
                    const int c1 = min(64 * k + 64, M);
                    for (int ci = max(64 * k, N); ci < c1; ++ci) {
                        const float2 q = s_pos[collider_entity(ci, N)];
                        const float dx = a.x - q.x, dy = a.y - q.y;
                        const float d2 = dx * dx + dy * dy;
                        if (d2 > 0.0f && d2 <= R2) oo |= 1ull << (ci - 64 * k);
                    }
                }
                const uint64_t w = (ow[k] & am) | oo;
                if (am || !keep_oo || rewrite) rmask[(int64_t)r * W + k] = w;
                pairs += __popcll(w);
            }
        }
    }
    if (coinc) *S.flag = 1;
    __syncthreads();
    if (*S.flag) {
        // exact rows: rad' also held the coincident pairs (agent columns of
        // every row, obstacle columns of agent rows; obstacle-obstacle bits
        // are exact already)
        pairs = 0;
        for (int r = tid; r < M; r += kTileBlock) {
            const float2 a = s_pos[collider_entity(r, N)];
            for (int k = 0; k < W; ++k) {
                const uint64_t am = agent_bits_of_word(N, k);
                uint64_t w = r < N ? 0ull : rmask[(int64_t)r * W + k] & ~am;
                const int c1 = min(64 * k + 64, r < N ? M : N);
                for (int ci = 64 * k; ci < c1; ++ci) {
                    const float2 q = s_pos[collider_entity(ci, N)];
                    const float dx = a.x - q.x, dy = a.y - q.y;
                    const float d2 = dx * dx + dy * dy;
                    if (d2 > 0.0f && d2 <= R2) w |= 1ull << (ci - 64 * k);
                }
                rmask[(int64_t)r * W + k] = w;
                pairs += __popcll(w);
            }
        }
    }
    return pairs;
}

__device__ __forceinline__ int obs_sweep_any(const DevParams &p, const float2 *s_pos, int *s_cost, int64_t eb,
                                             bool keep_oo, int *s_coinc) {
    switch (p.W) {
        case 2: return obs_sweep<2>(p, s_pos, s_cost, eb, keep_oo, s_coinc);
        case 3: return obs_sweep<3>(p, s_pos, s_cost, eb, keep_oo, s_coinc);
        case 4: return obs_sweep<4>(p, s_pos, s_cost, eb, keep_oo, s_coinc);
        default: return obs_sweep<0>(p, s_pos, s_cost, eb, keep_oo, s_coinc);
    }
}

// 8 waves per SIMD: four 512-thread workgroups per CU, so C3's 1024 envs run
// in one residency round (the compiler's default, 106 SGPRs, allowed 7 waves
// and three workgroups per CU). Fits without scratch (78 SGPRs, 58 VGPRs);
// step kernel 23.4 -> 22.0 us at C3.
#define GSM_TILE_ATTR __attribute__((amdgpu_waves_per_eu(8)))
// ---------------------------------------------------------------------------
// edge emitter
// ---------------------------------------------------------------------------
// Row r's edges in entity order from its radius mask words: agent rows ->
// agents, own goal (always), obstacles; goal rows -> own agent; obstacle rows
// -> agents, obstacles. kWrite = false only counts.
template <bool kWrite, int kN = 0, int kNo = 0>
__device__ __forceinline__ int row_edges(const DevParams &p, const EdgeSink &out, const float2 *s_pos,
                                         const uint64_t *rmask, int r, int64_t off, int32_t g0) {
    GSM_TILE_SHAPE(p);
    if (r >= N && r < 2 * N) {   // goal row: goal i -> agent i
        if (kWrite && off < out.cap) {
            const float2 a = s_pos[r], q = s_pos[r - N];
            const float dx = a.x - q.x, dy = a.y - q.y;
            out.index[off] = g0 + r;
            out.index[out.cap + off] = g0 + r - N;
            out.attr[off] = sqrtf(dx * dx + dy * dy);
        }
        return 1;
    }
    const int m = r < N ? r : r - N;             // collider row
    const uint64_t *row = rmask + (int64_t)m * W;
    if (!kWrite) {
        int n = r < N ? 1 : 0;
        for (int k = 0; k < W; ++k) n += __popcll(row[k]);
        return n;
    }
    const float2 a = s_pos[r];
    int n = 0;
    auto put = [&](int dst) {
        if (off + n < out.cap) {   // redirected outputs may be smaller than the worst case
            const float2 q = s_pos[dst];
            const float dx = a.x - q.x, dy = a.y - q.y;
            out.index[off + n] = g0 + r;
            out.index[out.cap + off + n] = g0 + dst;
            out.attr[off + n] = sqrtf(dx * dx + dy * dy);
        }
        ++n;
    };
    bool goal_done = r >= N;
#pragma unroll 1
    for (int k = 0; k < W; ++k) {
        uint64_t bits = row[k];
        while (bits) {
            const int c = 64 * k + __builtin_ctzll(bits);
            bits &= bits - 1;
            if (!goal_done && c >= N) {   // own goal sits between agents and obstacles
                put(N + r);
                goal_done = true;
            }
            put(collider_entity(c, N));
        }
    }
    if (!goal_done) put(N + r);
    return n;
}

// Row r's edges in entity order as (source | destination << 16) entity-id
// words at `at` (the staged form of row_edges<true>); returns the end.
template <int kN = 0, int kNo = 0>
__device__ __forceinline__ uint32_t *expand_row(const DevParams &p, const uint64_t *rmask, int r, uint32_t *at) {
    GSM_TILE_SHAPE(p);
    const uint32_t src = (uint32_t)r;
    if (r >= N && r < 2 * N) {   // goal row: goal i -> agent i
        *at = src | ((uint32_t)(r - N) << 16);
        return at + 1;
    }
    const uint64_t *row = rmask + (int64_t)(r < N ? r : r - N) * W;
    bool goal_done = r >= N;
#pragma unroll 1
    for (int k = 0; k < W; ++k) {
        for (uint64_t bits = row[k]; bits; bits &= bits - 1) {
            const int c = 64 * k + __builtin_ctzll(bits);
            if (!goal_done && c >= N) {   // own goal sits between agents and obstacles
                *at++ = src | ((uint32_t)(N + r) << 16);
                goal_done = true;
            }
            *at++ = src | ((uint32_t)collider_entity(c, N) << 16);
        }
    }
    if (!goal_done) *at++ = src | ((uint32_t)(N + r) << 16);
    return at;
}

// Env b's edges (workgroup-wide: barriers): each thread takes a contiguous
// run of rows, counts them from the mask words, a workgroup scan gives the
// run offsets. The env's global offset `off` is the sum of the threads'
// `before` partials (edge counts of earlier envs), reduced in the same LDS
// exchange as the scan (one barrier) and returned in *off_out. When the env's
// edges fit the LDS scratch s_scr (scr_cap words) and the outputs, the runs
// are first expanded into s_scr in CSR order and then written by every
// thread, edge e by thread e mod 512 — coalesced stores and no row-length
// imbalance; otherwise each thread writes its runs directly (bounded by the
// output capacity). s_red: 2 * kTileWaves ints.
template <int kN = 0, int kNo = 0>
__device__ __forceinline__ void emit_env(const DevParams &p, const EdgeSink &out, const float2 *s_pos,
                                         const uint64_t *rmask, int before, int64_t *off_out, int *s_red,
                                         uint32_t *s_scr, int scr_cap, int32_t g0) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    GSM_TILE_SHAPE(p);
    const int R = (E + kTileBlock - 1) / kTileBlock;
    const int r0 = tid * R, r1 = min(E, r0 + R);
    int mine = 0;
    for (int r = r0; r < r1; ++r) mine += row_edges<false, kN, kNo>(p, out, s_pos, rmask, r, 0, g0);
    const int incl = wave_scan(mine);
    const int btot = wave_total(before);
    if (lane == 63) s_red[wave] = incl;
    if (lane == 0) s_red[kTileWaves + wave] = btot;
    __syncthreads();
    int64_t off = 0;
#pragma unroll
    for (int w = 0; w < kTileWaves; ++w) off += s_red[kTileWaves + w];
    *off_out = off;
    int base = incl - mine, total = 0;
#pragma unroll
    for (int w = 0; w < kTileWaves; ++w) {
        const int t = s_red[w];
        base += w < wave ? t : 0;
        total += t;
    }
    if (total <= scr_cap && off + total <= out.cap) {   // workgroup-uniform
        uint32_t *at = s_scr + base;
        for (int r = r0; r < r1; ++r) at = expand_row<kN, kNo>(p, rmask, r, at);
        __syncthreads();
        int32_t *src = out.index + off, *dst = out.index + out.cap + off;
        float *attr = out.attr + off;
        for (int e = tid; e < total; e += kTileBlock) {
            const uint32_t w = s_scr[e];
            const uint32_t a = w & 0xffffu, b = w >> 16;
            const float2 pa = s_pos[a], pb = s_pos[b];
            const float dx = pa.x - pb.x, dy = pa.y - pb.y;
            src[e] = g0 + (int32_t)a;
            dst[e] = g0 + (int32_t)b;
            attr[e] = sqrtf(dx * dx + dy * dy);
        }
    } else {
        int64_t o = off + base;
        for (int r = r0; r < r1; ++r) o += row_edges<true, kN, kNo>(p, out, s_pos, rmask, r, o, g0);
    }
}

__global__ __launch_bounds__(kTileBlock) GSM_TILE_ATTR void gsm_step_tile_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, E = p.E, W = p.W;
    float2 *s_pos = (float2 *)smem;           // [E]
    float2 *s_vel = s_pos + E;                // [N]
    float2 *s_np = s_vel + N;                 // [N] integrated agent positions
    int *s_cost = (int *)(s_np + N);          // [N]
    int *s_ired = s_cost + N;                 // [4 * kTileWaves] reduction slots
    float *s_fred = (float *)(s_ired + 4 * kTileWaves);
    int *s_deg = (int *)(s_fred + kTileWaves);   // [2] coincident pair (unsymmetric sweep), non-finite agent
    // symmetric sweep scratch (p.tile_sym), 16-byte aligned after the above
    TileSymLds sym;
    {
        unsigned char *q = smem + ((8 * E + 8 * N + 8 * N + 4 * N + 20 * kTileWaves + 8 + 15) & ~15);
        sym.xy = (float *)q;
        q += 16 * ((N + 1) / 2);
        sym.arow = (uint64_t *)q;
        q += 16 * N * W;
        sym.own = (uint64_t *)q;
        q += 8 * p.No * W;
        sym.flag = (int *)q;
    }
    const int64_t eb = b;

    // Issue every global read of the step up front (positions, velocities,
    // this thread's agent action and contact-candidate words) so their
    // latencies overlap instead of chaining through the phases below.
    constexpr int kPre = 4;   // contact words prefetched per agent (W <= 4)
    const bool step_mode = p.mode == kModeStep;
    uint64_t cw[kPre] = {0, 0, 0, 0};
    float2 u0 = make_float2(0.0f, 0.0f);
    if (step_mode && tid < N) {
        u0 = action_force(p, eb * N + tid);
        const uint64_t *cm = p.contact_mask + (eb * N + tid) * W;
#pragma unroll
        for (int k = 0; k < kPre; ++k)
            if (k < W) cw[k] = cm[k];
    }
    for (int e = tid; e < E; e += kTileBlock) s_pos[e] = p.pos[eb * E + e];
    for (int i = tid; i < N; i += kTileBlock) s_vel[i] = p.vel[eb * N + i];
    int t = p.step_count[b];
    int ep = p.episode[b];
    float2 acc = p.ep_acc[b];
    const bool do_reset = p.mode == kModeReset && (p.env_mask == nullptr || p.env_mask[b] != 0);
    bool relaid = false;
    if (tid == 0) s_deg[0] = s_deg[1] = 0;
    __syncthreads();

    auto relayout = [&]() {   // scenario.reset_world with the Philox layout
        ep = (p.mode == kModeReset && p.reseed ? -1 : ep) + 1;
        t = 0;
        acc = make_float2(0.0f, 0.0f);
        const uint32_t gid = (uint32_t)(p.env_base + b);
        __syncthreads();
        if (tid == 0) s_deg[0] = 0;   // the flags describe the new layout
        for (int e = tid; e < E; e += kTileBlock) s_pos[e] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)e);
        for (int i = tid; i < N; i += kTileBlock) s_vel[i] = make_float2(0.0f, 0.0f);
        relaid = true;
        __syncthreads();
    };
    if (do_reset) relayout();

    bool done = false;
    if (p.mode == kModeStep) {
        // apply_environment_force over the contact candidates of the previous
        // sweep (every pair within the cutoff), then integrate_state (App. A S3-S6)
        const uint64_t *cm = p.contact_mask + eb * N * W;
        for (int i = tid; i < N; i += kTileBlock) {
            const bool pre = i == tid;   // first agent of the thread: prefetched above
            const float2 pi = s_pos[i];
            const float2 u = pre ? u0 : action_force(p, eb * N + i);
            float fx = 0.0f, fy = 0.0f;
            auto visit = [&](int k, uint64_t bits) {
                while (bits) {
                    const int c = 64 * k + __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const bool ag = c < N;
                    const float2 pj = s_pos[collider_entity(c, N)];
                    const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                    const float d2 = dx * dx + dy * dy;
                    const float f = contact_scale(p, d2, ag ? p.dmin_aa : p.dmin_ao);
                    fx += f * dx;
                    fy += f * dy;
                }
            };
#pragma unroll
            for (int k = 0; k < kPre; ++k)
                if (k < W) visit(k, pre ? cw[k] : cm[(int64_t)i * W + k]);
            for (int k = kPre; k < W; ++k) visit(k, cm[(int64_t)i * W + k]);
            float Fx = u.x + fx, Fy = u.y + fy;
            if (p.strict && strict_bad(i, pi, N, p.M, [&](int c) { return s_pos[collider_entity(c, N)]; })) {
                Fx = __builtin_nanf("");   // App. A S16 strict: MPE's 0/0 force
                Fy = __builtin_nanf("");
            }
            float2 v = s_vel[i];
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
            s_vel[i] = v;
            s_np[i] = make_float2(pi.x + v.x * p.dt, pi.y + v.y * p.dt);
        }
        __syncthreads();   // every pre-step position read
        for (int i = tid; i < N; i += kTileBlock) s_pos[i] = s_np[i];
        __syncthreads();
        t += 1;
        done = t >= p.EL;
    }

    // observation sweep of the post-step state: masks, collision counts, pairs
    int pairs = p.tile_sym ? obs_sweep_sym(p, s_pos, sym, s_cost, eb, p.mode == kModeStep && !relaid)
                           : obs_sweep_any(p, s_pos, s_cost, eb, p.mode == kModeStep && !relaid, s_deg);
    // reward and cost callbacks, episode accounting. The workgroup sums of
    // reward, collisions, directed radius pairs and the non-finite flag share
    // one LDS exchange (an auto-reset, rare, re-sweeps and exchanges again).
    auto nonfinite_part = [&]() {
        int bad = 0;
        if (p.degenerate)
            for (int i = tid; i < N; i += kTileBlock) bad |= nonfinite2(s_pos[i]) ? 1 : 0;
        return bad;
    };
    float rpart = 0.0f;
    for (int i = tid; i < N; i += kTileBlock) {
        const float2 a = s_pos[i], g = s_pos[N + i];
        const float dx = a.x - g.x, dy = a.y - g.y;
        rpart += -sqrtf(dx * dx + dy * dy);
    }
    __syncthreads();   // s_cost from the sweep; the exchange slots are free
    int cpart = 0;
    for (int i = tid; i < N; i += kTileBlock) {
        const int cnt = s_cost[i];
        p.cost[eb * N + i] = (float)cnt;
        cpart += cnt;
        if (!p.shared_reward) {
            const float2 a = s_pos[i], g = s_pos[N + i];
            const float dx = a.x - g.x, dy = a.y - g.y;
            p.reward[eb * N + i] = -sqrtf(dx * dx + dy * dy);
        }
    }
    {
        const float rw = wave_total(rpart);
        const int cw = wave_total(cpart), pw = wave_total(pairs), bw = wave_total(nonfinite_part());
        if ((tid & 63) == 0) {
            const int w = tid >> 6;
            s_fred[w] = rw;
            s_ired[w] = cw;
            s_ired[kTileWaves + w] = pw;
            s_ired[2 * kTileWaves + w] = bw;
        }
    }
    __syncthreads();
    float rsum = 0.0f;
    int csum = 0, bad = 0;
    pairs = 0;
#pragma unroll
    for (int w = 0; w < kTileWaves; ++w) {
        rsum += s_fred[w];
        csum += s_ired[w];
        pairs += s_ired[kTileWaves + w];
        bad |= s_ired[2 * kTileWaves + w];
    }
    if (p.shared_reward) {
        for (int i = tid; i < N; i += kTileBlock) p.reward[eb * N + i] = rsum;
        rsum *= (float)N;
    }

    if (p.mode == kModeStep) {
        acc.x += rsum;
        acc.y += (float)csum;
        if (done && p.auto_reset) {
            if (tid == 0) p.ep_last[b] = acc;
            relayout();
            pairs = p.tile_sym ? obs_sweep_sym(p, s_pos, sym, s_cost, eb, false)
                               : obs_sweep_any(p, s_pos, s_cost, eb, false, s_deg);
            pairs = tile_sum(pairs, s_ired);
            bad = tile_sum(nonfinite_part(), s_ired + 3 * kTileWaves);
        }
    }

    // node features [E][7] = [vx vy px py gx-px gy-py type]: agent rows every
    // step (one thread per row), goal/obstacle rows only on layout change
    float *nf = p.node_feat + eb * E * 7;
    const bool full = p.mode != kModeStep || relaid || p.nf_full;
    for (int i = tid; i < N; i += kTileBlock) {
        const float2 v = s_vel[i], a = s_pos[i], g = s_pos[N + i];
        float *row = nf + (int64_t)i * 7;
        row[0] = v.x;
        row[1] = v.y;
        row[2] = a.x;
        row[3] = a.y;
        row[4] = g.x - a.x;
        row[5] = g.y - a.y;
        if (full) row[6] = 0.0f;
    }
    if (full) {
        for (int e = N + tid; e < E; e += kTileBlock) {
            const float2 a = s_pos[e];
            float *row = nf + (int64_t)e * 7;
            row[0] = 0.0f;
            row[1] = 0.0f;
            row[2] = a.x;
            row[3] = a.y;
            row[4] = 0.0f;
            row[5] = 0.0f;
            row[6] = e < 2 * N ? 1.0f : 2.0f;
        }
    }
    // state
    if (p.mode == kModeStep || do_reset) {
        const int ne = relaid ? E : N;
        for (int e = tid; e < ne; e += kTileBlock) p.pos[eb * E + e] = s_pos[e];
        for (int i = tid; i < N; i += kTileBlock) p.vel[eb * N + i] = s_vel[i];
    }
    const int edges = pairs + 2 * N;   // directed radius edges + agent<->goal
    if (tid == 0) {
        p.step_count[b] = t;
        p.episode[b] = ep;
        p.ep_acc[b] = acc;
        p.done[b] = done ? 1 : 0;
        p.edge_count[b] = edges;
        p.block_edge_sum[b] = edges;
        if (p.degenerate) {
            const int co = p.tile_sym ? *sym.flag : s_deg[0];
            p.degenerate[b] = (uint8_t)((co ? kDegCoincident : 0) | (bad ? kDegNonfinite : 0));
        }
    }
}

__global__ __launch_bounds__(kTileBlock) void gsm_emit_tile_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int E = p.E;
    float2 *s_pos = (float2 *)smem;
    int *s_red = (int *)(s_pos + E);          // [2 * kTileWaves]
    uint32_t *s_scr = (uint32_t *)(s_red + 2 * kTileWaves);   // staged edge words
    const int scr_cap = (p.wave_lds_emit - 8 * E - 8 * kTileWaves) / 4;
    const int64_t eb = b;
    // global offset: edges of envs [0, b)  (host keeps totals < 2^31), reduced
    // inside emit_env with the row-count scan
    int before = 0;
    for (int k = tid; k < b; k += kTileBlock) before += p.edge_count[k];
    for (int e = tid; e < E; e += kTileBlock) s_pos[e] = p.pos[eb * E + e];
    int64_t off;   // (emit_env's exchange barrier also publishes the staged positions)
    emit_env(p, EdgeSink{p.edge_index, p.edge_attr, p.edge_capacity}, s_pos, p.row_mask + eb * p.M * p.W, before,
             &off, s_red, s_scr, scr_cap, (int32_t)(eb * E));
    if (tid == 0) {
        p.edge_ptr[b] = off;
        if (b == p.B - 1) p.edge_ptr[p.B] = off + p.edge_count[b];
    }
}

// ---------------------------------------------------------------------------
// Fused rollout on the tile path (one 512-thread workgroup per env; C3):
// K steps of a graph in one launch, as gsm_roll_seg_kernel.
// Positions, velocities, contact words and row masks stay in LDS; the row
// masks alternate between two LDS buffers (step k writes k & 1) so step
// k-1's masks survive step k's sweep and are emitted after it at the offset
// found by the look-back over per-env granules (one env per workgroup); the
// masks go to global memory once, after the loop (the emit launch that
// follows reads the last step's). The step's
// outputs (node features, reward, cost, done) are written every step, the
// state once after the loop. Same operations as gsm_step_tile_kernel in the
// same order: bit-identical outputs.
constexpr int kRollTileScr = 1536;   // staged edge words (C3: ~390 edges per env; else direct writes)

size_t roll_tile_kernel_lds(const DevParams &p) {
    return (size_t)p.wave_lds_step + 16 * (size_t)p.E + 16 + 8 * kTileWaves + 4 * kRollTileScr +
           8 * (size_t)p.W * (3 * p.M + p.N);
}

// kN > 0: compiled for kN agents and kNo obstacles (C3: 96 + 96), so the
// shape is immediates throughout the loop instead of values held in SGPRs
// (at 8 waves per SIMD those spilled to VGPR lanes: a v_readlane at every use)
template <bool kSlots, int kN = 0, int kNo = 0>   // kSlots: per-step outputs at base + k * stride (a rollout buffer)
__global__ __launch_bounds__(kTileBlock) GSM_TILE_ATTR void gsm_roll_tile_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    GSM_TILE_SHAPE(p);
    float2 *const s_p0 = (float2 *)smem;      // [E] position buffer 0 (of three, below)
    float2 *s_vel = s_p0 + E;                 // [N]
    float2 *s_np = s_vel + N;                 // [N] integrated agent positions
    int *s_cost = (int *)(s_np + N);          // [N]
    int *s_ired = s_cost + N;                 // [4 * kTileWaves] reduction slots
    float *s_fred = (float *)(s_ired + 4 * kTileWaves);
    int *s_deg = (int *)(s_fred + kTileWaves);   // [2] (unsymmetric sweep's coincident flag), unused here
    TileSymLds sym;
    {
        unsigned char *q = smem + ((8 * E + 8 * N + 8 * N + 4 * N + 20 * kTileWaves + 8 + 15) & ~15);
        sym.xy = (float *)q;
        q += 16 * ((N + 1) / 2);
        sym.arow = (uint64_t *)q;
        q += 16 * N * W;
        sym.own = (uint64_t *)q;
        q += 8 * No * W;
        sym.flag = (int *)q;
    }
    // Positions rotate through three LDS buffers (buffer j % 3 holds the
    // positions before step j): step k reads buffer k % 3 and writes its
    // agents' new positions into buffer (k + 1) % 3, and iteration k emits
    // step k - 2's edges from buffer (k - 1) % 3 — no per-step copy of the
    // positions and two workgroup barriers fewer per step than a single
    // buffer plus a saved copy. Goals and obstacles (static within an
    // episode) are kept in all three: copied at entry and, after a
    // re-layout, into the next buffer at the end of this iteration and the
    // one after (each after the emission that still reads the old ones)
    float2 *s_prv = (float2 *)(smem + p.wave_lds_step);    // buffers 1 and 2
    auto pbuf = [&](int j3) -> float2 * { return j3 == 0 ? s_p0 : s_prv + (j3 - 1) * E; };
    int *s_x = (int *)(s_prv + 2 * E);                     // [4]
    int *s_red = s_x + 4;                                  // [2 * kTileWaves] emit_env exchange
    uint32_t *s_scr = (uint32_t *)(s_red + 2 * kTileWaves);
    uint64_t *s_rm = (uint64_t *)(s_scr + kRollTileScr);   // [3][M][W] row masks, step k at k % 3
    uint64_t *s_cm = s_rm + 3 * M * W;                     // [N][W] contact words
    const int64_t eb = b;
    const int32_t g0 = (int32_t)(eb * E);
    for (int w = tid; w < M * W; w += kTileBlock) s_rm[2 * M * W + w] = p.row_mask[eb * M * W + w];
    for (int w = tid; w < N * W; w += kTileBlock) s_cm[w] = p.contact_mask[eb * N * W + w];

    for (int e = tid; e < E; e += kTileBlock) {
        const float2 x = p.pos[eb * E + e];
        s_p0[e] = x;
        s_prv[e] = x;
        s_prv[E + e] = x;
    }
    bool relaid_prev = false;   // the previous iteration re-laid the env out
    for (int i = tid; i < N; i += kTileBlock) s_vel[i] = p.vel[eb * N + i];
    int t = p.step_count[b];
    int ep = p.episode[b];
    float2 acc = p.ep_acc[b];
    if (tid == 0) s_deg[0] = s_deg[1] = 0;
    // pacing (gsm_device.h pace_level): this workgroup's CU counter (its
    // arrival now, a step after each step, its rank = the arrivals before it;
    // the address re-formed at each use), the slot's next counters zeroed
    auto pacing = [] { return late_params().roll.pace != nullptr; };
    auto pace_ctr = [] { return (gu32 *)hand_chk(late_params().roll.pace + pace_key()); };
    // the one-hop CSR prefix (gsm_device.h roll_prefix): chunks of 64
    // workgroups; the slot's next launch's chunk sums zeroed
    const int nc = ((int)gridDim.x + kPrefixChunk - 1) / kPrefixChunk;
    {
        KernargParams &qz = late_params();
        const int cs = qz.roll.csum_stride, n = qz.roll.K * nc;
        for (int i = b * kTileBlock + tid; i < n; i += gridDim.x * kTileBlock)
            __hip_atomic_store((gu64 *)hand_chk(qz.roll.csum_next + (int64_t)i * cs), 0ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (pacing()) {
        KernargParams &qz = late_params();
        for (int i = b * kTileBlock + tid; i < kPaceKeys; i += gridDim.x * kTileBlock)
            __hip_atomic_store((gu32 *)hand_chk(qz.roll.pace_next + i * kPaceStride), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (tid == 0)
            s_x[3] = (int)(__hip_atomic_fetch_add(pace_ctr(), kPaceArrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >>
                           24);
    }
    const int K = p.roll.K, n_act = p.roll.n_actions;
    const uint32_t etag = roll_epoch_tag(p.roll.epoch);     // this launch's tag base
    int arow = p.roll.t_first % n_act;
    int edges_m1 = 0, edges_m2 = 0, last_edges = 0, bad = 0;   // edge counts of steps k - 1, k - 2, K - 1
    int r3 = 0;                                               // k % 3
    __syncthreads();

    // iterations 0..K-1 run step k and emit step k-2; iterations K and K+1
    // (the tail) only emit steps K-2 and K-1
    // Inside the loop the launch's flags and constants are read through the
    // kernarg view at their use (late_params()): read from `p` the compiler
    // hoists them out of the loop and holds them in SGPRs, spilled to VGPR
    // lanes at 8 waves per SIMD (gsm_roll_seg_kernel).
    GSM_RSTAMP(p, b * kTileWaves + (tid >> 6), 8);
    for (int k = 0; k <= K + 1; ++k) {
        // thread-derived values re-formed every iteration (an asm barrier): held
        // across the loop their hoisted addresses would pin VGPRs
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int wave = tid >> 6, lane = tid & 63;
        const int wid = b * kTileWaves + wave;   // (diagnostic stamps)
        (void)wid;
        GSM_TNOW(tp0);
        const int r3n = r3 == 2 ? 0 : r3 + 1, r3p = r3 == 0 ? 2 : r3 - 1;   // (k + 1) % 3, (k - 1) % 3
        const float2 *const s_cur = pbuf(r3);   // positions before step k
        float2 *const s_pos = pbuf(r3n);        // after it (agents written by the physics)
        uint64_t *const rout = s_rm + r3 * M * W;
        const uint64_t *const rkeep = s_rm + r3p * M * W;   // the previous step's masks
        const uint64_t *const remit = s_rm + r3n * M * W;   // step k - 2's masks (emitted this iteration)
        int edges = 0;
        // step k - 2's CSR offset: the one-hop prefix (published an iteration
        // ago by every workgroup in step: one load per lane) by the last wave,
        // idle in the physics below (agents 0..N-1 on the first threads), so
        // its latency overlaps the step; read by the emission after the step
        // (s_x[2], published by the step's barriers); the CU's pace counter
        // loaded beside it
        if (k > 0 && wave == kTileWaves - 1) {
            GSM_TNOW(tp4);
            KernargParams &q = late_params();
            const uint32_t pv = k < K && pacing() ? __hip_atomic_load(pace_ctr(), __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT)
                                                  : 0u;
            int ex = 0;
            if (k >= 2) {
                const int cs = q.roll.csum_stride;
                ex = roll_prefix(q.roll.gran + (int64_t)(k - 2) * gridDim.x, q.roll.csum + (int64_t)(k - 2) * nc * cs,
                                 cs, etag | (uint32_t)(k - 1), q.roll.status, lane);
            }
            // the pace level formed once here for the workgroup (it was the
            // same wave-uniform SALU work repeated by all eight waves)
            const int lvl = k < K && pacing() ? pace_level((uint32_t)__builtin_amdgcn_readfirstlane(pv), k,
                                                            __builtin_amdgcn_readfirstlane(s_x[3]), q.roll.pace_q)
                                              : 0;   // (the tail: level 0, as pace_level of a zero counter)
            if (lane == 0) {
                s_x[1] = lvl;
                // (an offset past the capacity is a legal overflow of a small
                // slot: edge_ptr keeps it, emit_env stops its writes at the
                // capacity)
                if (ex < 0) {   // a broken hand-off: never write out of bounds
                    __hip_atomic_store((gu32 *)late_params().roll.status, 2u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    ex = (int)min(late_params().ro.cap, (int64_t)0x7fffffff);
                }
                s_x[2] = ex;
            }
            GSM_ACC(late_params(), wid, 5, tp4);   // the prefix (last wave)
        }
        if (k >= K) __syncthreads();   // (the tail: no step; s_x[2] for the emission)
        bool relaid = false;
        if (k < K) {
        auto relayout = [&]() {   // scenario.reset_world with the Philox layout
            ep = ep + 1;
            t = 0;
            acc = make_float2(0.0f, 0.0f);
            const uint32_t gid = (uint32_t)(late_params().env_base + b);
            __syncthreads();
            for (int e = tid; e < E; e += kTileBlock) s_pos[e] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)e);
            for (int i = tid; i < N; i += kTileBlock) s_vel[i] = make_float2(0.0f, 0.0f);
            relaid = true;
            __syncthreads();
        };
        // apply_environment_force + integrate_state (as gsm_step_tile_kernel)
        const uint64_t *cm = s_cm;
        for (int i = tid; i < N; i += kTileBlock) {
            const float2 pi = s_cur[i];
            const float2 u = roll_action_force(late_params(), arow, eb * N + i);
            float fx = 0.0f, fy = 0.0f;
            // (both read before the loop: a per-lane select of two kernarg
            // fields compiles to a vector load and a vmcnt wait per contact)
            const float dmin_aa = late_params().dmin_aa, dmin_ao = late_params().dmin_ao;
            for (int kw = 0; kw < W; ++kw) {
                uint64_t bits = cm[(int64_t)i * W + kw];
                while (bits) {
                    const int c = 64 * kw + __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const bool ag = c < N;
                    const float2 pj = s_cur[collider_entity(c, N)];
                    const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                    const float d2 = dx * dx + dy * dy;
                    const float f = contact_scale(late_params(), d2, ag ? dmin_aa : dmin_ao);
                    fx += f * dx;
                    fy += f * dy;
                }
            }
            float Fx = u.x + fx, Fy = u.y + fy;
            if (late_params().strict && strict_bad(i, pi, N, M, [&](int c) { return s_cur[collider_entity(c, N)]; })) {
                Fx = __builtin_nanf("");
                Fy = __builtin_nanf("");
            }
            float2 v = s_vel[i];
            v.x = v.x * late_params().omd;
            v.y = v.y * late_params().omd;
            v.x = v.x + (Fx / late_params().mass) * late_params().dt;
            v.y = v.y + (Fy / late_params().mass) * late_params().dt;
            if (late_params().max_speed > 0.0f) {
                const float sp = sqrtf(v.x * v.x + v.y * v.y);
                if (sp > late_params().max_speed) {
                    v.x = v.x / sp * late_params().max_speed;
                    v.y = v.y / sp * late_params().max_speed;
                }
            }
            s_vel[i] = v;
            s_pos[i] = make_float2(pi.x + v.x * late_params().dt, pi.y + v.y * late_params().dt);
        }
        __syncthreads();
        // this workgroup's pace level (from the counter the last wave loaded
        // at the top of the iteration, published by the barrier above)
        if (k > 0 && pacing()) pace_set(__builtin_amdgcn_readfirstlane(s_x[1]));
        t += 1;
        const bool done = t >= late_params().EL;
        GSM_ACC(late_params(), wid, 0, tp0);   // physics
        GSM_TNOW(tp1);
        int pairs = obs_sweep_sym<kN, kNo>(p, s_pos, sym, s_cost, eb, true, rout, rkeep, s_cm);
        GSM_ACC(late_params(), wid, 2, tp1);   // sweep (column pass: 1)
        GSM_TNOW(tp2);
        auto nonfinite_part = [&]() {
            int bd = 0;
            if (late_params().degenerate)
                for (int i = tid; i < N; i += kTileBlock) bd |= nonfinite2(s_pos[i]) ? 1 : 0;
            return bd;
        };
        float rpart = 0.0f;
        for (int i = tid; i < N; i += kTileBlock) {
            const float2 a = s_pos[i], g = s_pos[N + i];
            const float dx = a.x - g.x, dy = a.y - g.y;
            rpart += -sqrtf(dx * dx + dy * dy);
        }
        __syncthreads();
        int cpart = 0;
        for (int i = tid; i < N; i += kTileBlock) {
            const int cnt = s_cost[i];
            late_params().ro.cost[(kSlots ? k * late_params().ro.rc_s : 0) + eb * N + i] = (float)cnt;
            cpart += cnt;
            if (!late_params().shared_reward) {
                const float2 a = s_pos[i], g = s_pos[N + i];
                const float dx = a.x - g.x, dy = a.y - g.y;
                late_params().ro.rew[(kSlots ? k * late_params().ro.rc_s : 0) + eb * N + i] = -sqrtf(dx * dx + dy * dy);
            }
        }
        {
            const float rw = wave_total(rpart);
            const int cw = wave_total(cpart), pw = wave_total(pairs), bw = wave_total(nonfinite_part());
            if (lane == 0) {
                s_fred[wave] = rw;
                s_ired[wave] = cw;
                s_ired[kTileWaves + wave] = pw;
                s_ired[2 * kTileWaves + wave] = bw;
            }
        }
        __syncthreads();
        float rsum = 0.0f;
        int csum = 0;
        bad = 0;
        pairs = 0;
#pragma unroll
        for (int w = 0; w < kTileWaves; ++w) {
            rsum += s_fred[w];
            csum += s_ired[w];
            pairs += s_ired[kTileWaves + w];
            bad |= s_ired[2 * kTileWaves + w];
        }
        if (late_params().shared_reward) {
            for (int i = tid; i < N; i += kTileBlock) late_params().ro.rew[(kSlots ? k * late_params().ro.rc_s : 0) + eb * N + i] = rsum;
            rsum *= (float)N;
        }
        acc.x += rsum;
        acc.y += (float)csum;
        GSM_ACC(late_params(), wid, 3, tp2);   // reward / cost and the exchange
        if (done && late_params().auto_reset) {
            if (tid == 0) late_params().ep_last[b] = acc;
            relayout();
            pairs = obs_sweep_sym<kN, kNo>(p, s_pos, sym, s_cost, eb, false, rout, rkeep, s_cm);
            pairs = tile_sum(pairs, s_ired);
            bad = tile_sum(nonfinite_part(), s_ired + 3 * kTileWaves);
        }
        // the step's observation outputs: agent node rows, static rows on a new layout
        GSM_TNOW(tp3);
        float *nf = late_params().ro.nf + (kSlots ? k * late_params().ro.nf_s : 0) + eb * E * 7;
        const bool full = relaid || late_params().nf_full;
        for (int i = tid; i < N; i += kTileBlock) {
            const float2 v = s_vel[i], a = s_pos[i], g = s_pos[N + i];
            float *row = nf + (int64_t)i * 7;
            row[0] = v.x;
            row[1] = v.y;
            row[2] = a.x;
            row[3] = a.y;
            row[4] = g.x - a.x;
            row[5] = g.y - a.y;
            if (full) row[6] = 0.0f;
        }
        if (full) {
            for (int e = N + tid; e < E; e += kTileBlock) {
                const float2 a = s_pos[e];
                float *row = nf + (int64_t)e * 7;
                row[0] = 0.0f;
                row[1] = 0.0f;
                row[2] = a.x;
                row[3] = a.y;
                row[4] = 0.0f;
                row[5] = 0.0f;
                row[6] = e < 2 * N ? 1.0f : 2.0f;
            }
        }
        edges = pairs + 2 * N;   // directed radius edges + agent<->goal
        if (tid == 0) {
            KernargParams &q = late_params();
            q.ro.done[(kSlots ? k * q.ro.done_s : 0) + b] = done ? 1 : 0;
            if (kSlots || k == K - 1) q.ro.ecount[(kSlots ? k * q.ro.ec_s : 0) + b] = edges;
            const int cs = q.roll.csum_stride;
            prefix_publish(q.roll.gran + (int64_t)k * gridDim.x, q.roll.csum + (int64_t)k * nc * cs, cs, b,
                           etag | (uint32_t)(k + 1), (uint32_t)edges);
            if (pacing()) (void)__hip_atomic_fetch_add(pace_ctr(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        GSM_ACC(late_params(), wid, 4, tp3);   // node features, publish
        }   // k < K
        // step k - 2's edges at the offset of the prefix (its positions in
        // buffer (k - 1) % 3, its masks in buffer (k - 2) % 3)
        const float2 *const s_pk = pbuf(r3p);
        if (k >= 2) {
            GSM_TNOW(tp5);
            int64_t off;
            emit_env<kN, kNo>(p, roll_edge_sink<kSlots>(late_params(), k - 2, K), s_pk, remit,
                              tid == 0 ? s_x[2] : 0, &off, s_red, s_scr, kRollTileScr, g0);
            GSM_ACC(late_params(), wid, 6, tp5);   // emission
            if (tid == 0) {
                KernargParams &q = late_params();
                int64_t *const eptr = q.ro.eptr + (kSlots ? (k - 2) * q.ro.ep_s : 0);
                eptr[b] = off;
                if (b == late_params().B - 1) eptr[late_params().B] = off + edges_m2;
            }
        }
        if (k < K) {
            GSM_TNOW(tp6);
            // the emission's reads of buffer (k - 1) % 3 and of the staged
            // words done before the next step writes that buffer
            __syncthreads();
            // after a re-layout (this iteration or the previous one) the new
            // goals / obstacles into the buffer the next step writes its
            // agents into (its old ones were read by this emission)
            if (relaid || relaid_prev) {
                float2 *const dst = pbuf(r3n == 2 ? 0 : r3n + 1);
                for (int e = N + tid; e < E; e += kTileBlock) dst[e] = s_pos[e];
            }
            relaid_prev = relaid;
            arow = arow + 1 == n_act ? 0 : arow + 1;
            if (k == K - 1) last_edges = edges;
            GSM_ACC(late_params(), wid, 7, tp6);   // hand-over to the next step
        }
        edges_m2 = edges_m1;
        edges_m1 = edges;
        r3 = r3n;
    }
    GSM_RSTAMP(p, b * kTileWaves + (tid >> 6), 9);
    // the final state (what the next launch or an eager step reads)
    for (int e = tid; e < E; e += kTileBlock) p.pos[eb * E + e] = pbuf(K % 3)[e];
    const int rl = (K - 1) % 3;   // the last step's masks
    for (int w = tid; w < M * W; w += kTileBlock) p.row_mask[eb * M * W + w] = s_rm[rl * M * W + w];
    for (int w = tid; w < N * W; w += kTileBlock) p.contact_mask[eb * N * W + w] = s_cm[w];
    for (int i = tid; i < N; i += kTileBlock) p.vel[eb * N + i] = s_vel[i];
    if (tid == 0) {
        p.step_count[b] = t;
        p.episode[b] = ep;
        p.ep_acc[b] = acc;
        p.block_edge_sum[b] = last_edges;
        if (p.degenerate) p.degenerate[b] = (uint8_t)((*sym.flag ? kDegCoincident : 0) | (bad ? kDegNonfinite : 0));
    }
}

const void *roll_tile_kernel_fn(const DevParams &p, bool slots) {
    if (p.path != kPathTile || !p.tile_sym) return nullptr;
    // (a C3-compiled instantiation, <96, 96>, trades the runtime shape's SGPR
    // spills — 132 -> 106 — for 22 VGPR spills to scratch at the 64-VGPR
    // budget of 8 waves per SIMD: not used)
    return slots ? reinterpret_cast<const void *>(&gsm_roll_tile_kernel<true>)
                 : reinterpret_cast<const void *>(&gsm_roll_tile_kernel<false>);
}

const void *step_tile_kernel_fn() { return reinterpret_cast<const void *>(&gsm_step_tile_kernel); }
const void *emit_tile_kernel_fn() { return reinterpret_cast<const void *>(&gsm_emit_tile_kernel); }

}  // namespace gsm
