// gsm_kernels.hip — batched MultiAgentGraphConstrainEnv step path for gfx950.
//
// Two kernels per env.step:
//
//  gsm_step_kernel   one wave64 per env, 4 envs per workgroup. Loads the env's
//                    entity positions into LDS and does, in order:
//                      _set_action + World.step() (core.py, SOURCES.txt:14):
//                        action force, pairwise soft contact, semi-implicit
//                        Euler integrate_state;
//                      reward / collision cost / done (scenario callbacks,
//                        SOURCES.txt:21-22; readme.md:34-41,101);
//                      auto-reset with a Philox layout (App. A S14);
//                      node features and the env's edge count.
//  gsm_emit_edges_kernel
//                    same env->wave mapping; its global edge offset is the
//                    prefix of the step kernel's per-workgroup edge sums, then
//                    one __ballot per (row, 64 candidates) writes the row-major
//                    COO edges with their distances.
//
// Bit-exactness contract: every +,-,x that feeds an integer output (collision
// counts, edge predicates) is done in fp32 without contraction (the library is
// built with -ffp-contract=off) in the same order as oracle/batch_ref.py's fp32
// mode: d2 = dx*dx + dy*dy, collide iff d2 < dmin*dmin, edge iff 0 < d2 <= R*R.
#include "gsm_device.h"

namespace gsm {

// ---------------------------------------------------------------------------
// step kernel
// ---------------------------------------------------------------------------
__device__ int env_step(const DevParams &p, const int b, const int lane, unsigned char *lds) {
    const int N = p.N, E = p.E, M = p.M, S = p.S, SN = S * N;
    float2 *s_pos = (float2 *)lds;            // [E]
    float2 *s_vel = s_pos + E;                // [N]
    float2 *s_part = s_vel + N;               // [S][N] partial forces
    int *s_icnt = (int *)(s_part + SN);       // [S][N] partial collision counts
    const int64_t eb = b;

    for (int e = lane; e < E; e += kWave) s_pos[e] = p.pos[eb * E + e];
    for (int i = lane; i < N; i += kWave) s_vel[i] = p.vel[eb * N + i];
    int t = p.step_count[b];
    int ep = p.episode[b];
    float2 acc = p.ep_acc[b];
    bool do_reset = p.mode == kModeReset && (p.env_mask == nullptr || p.env_mask[b] != 0);
    bool done = false;
    // scenario.reset_world with the Philox layout (App. A S14): new episode
    auto relayout = [&]() {
        ep = (p.mode == kModeReset && p.reseed ? -1 : ep) + 1;
        t = 0;
        acc = make_float2(0.0f, 0.0f);
        const uint32_t gid = (uint32_t)(p.env_base + b);
        for (int e = lane; e < E; e += kWave) s_pos[e] = layout_pos(p, gid, (uint32_t)ep, (uint32_t)e);
        for (int i = lane; i < N; i += kWave) s_vel[i] = make_float2(0.0f, 0.0f);
        wave_sync();
    };
    wave_sync();
    if (do_reset) relayout();

    if (p.mode == kModeStep) {
        // apply_environment_force: lane (i, s) sums the contact forces on
        // agent i from colliders c = s, s+S, ... (self excluded).
        for (int w = lane; w < SN; w += kWave) {
            const int i = w % N, s = w / N;
            const float2 pi = s_pos[i];
            float fx = 0.0f, fy = 0.0f;
            for (int c = s; c < M; c += S) {
                if (c == i) continue;
                const bool ag = c < N;
                const float2 pj = s_pos[collider_entity(c, N)];
                const float dx = pi.x - pj.x, dy = pi.y - pj.y;
                const float d2 = dx * dx + dy * dy;
                if (d2 < (ag ? p.cut2_aa : p.cut2_ao) && d2 > 0.0f) {
                    const float f = contact_scale(p, d2, ag ? p.dmin_aa : p.dmin_ao);
                    fx += f * dx;
                    fy += f * dy;
                }
            }
            s_part[s * N + i] = make_float2(fx, fy);
        }
        wave_sync();
        // integrate_state (App. A S6): damping, F/m*dt, speed clamp, p += v*dt
        for (int i = lane; i < N; i += kWave) {
            const float2 u = action_force(p, eb * N + i);
            float Fx = u.x, Fy = u.y;
            for (int s = 0; s < S; ++s) {
                const float2 q = s_part[s * N + i];
                Fx += q.x;
                Fy += q.y;
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
            float2 pi = s_pos[i];
            pi.x = pi.x + v.x * p.dt;
            pi.y = pi.y + v.y * p.dt;
            s_vel[i] = v;
            s_pos[i] = pi;
        }
        wave_sync();
        t += 1;
        done = t >= p.EL;
    }

    // reward callback: -|p_i - g_i| ; cost callback: collisions of agent i
    float rsum = 0.0f;
    for (int i = lane; i < N; i += kWave) {
        const float2 a = s_pos[i], g = s_pos[N + i];
        const float dx = a.x - g.x, dy = a.y - g.y;
        const float r = -sqrtf(dx * dx + dy * dy);
        rsum += r;
        if (!p.shared_reward) p.reward[eb * N + i] = r;
    }
    rsum = wave_sum(rsum);
    if (p.shared_reward) {
        for (int i = lane; i < N; i += kWave) p.reward[eb * N + i] = rsum;
        rsum *= (float)N;
    }
    for (int w = lane; w < SN; w += kWave) {
        const int i = w % N, s = w / N;
        const float2 pi = s_pos[i];
        int cnt = 0;
        for (int c = s; c < M; c += S) {
            if (c == i) continue;
            const float2 pj = s_pos[collider_entity(c, N)];
            const float dx = pi.x - pj.x, dy = pi.y - pj.y;
            const float d2 = dx * dx + dy * dy;
            cnt += d2 < (c < N ? p.dmin2_aa : p.dmin2_ao);
        }
        s_icnt[s * N + i] = cnt;
    }
    wave_sync();
    int csum = 0;
    for (int i = lane; i < N; i += kWave) {
        int cnt = 0;
        for (int s = 0; s < S; ++s) cnt += s_icnt[s * N + i];
        p.cost[eb * N + i] = (float)cnt;
        csum += cnt;
    }
    csum = wave_sum(csum);

    if (p.mode == kModeStep) {
        acc.x += rsum;
        acc.y += (float)csum;
        if (done && p.auto_reset) {
            do_reset = true;
            if (lane == 0) p.ep_last[b] = acc;
        }
    }
    if (do_reset && p.mode == kModeStep) relayout();

    // node features [E][7]: vx vy px py gx-px gy-py type
    float *nf = p.node_feat + eb * E * 7;
    for (int q = lane; q < E * 7; q += kWave) {
        const int e = q / 7, col = q - e * 7;
        const float2 pe = s_pos[e];
        float v;
        switch (col) {
            case 0: v = e < N ? s_vel[e].x : 0.0f; break;
            case 1: v = e < N ? s_vel[e].y : 0.0f; break;
            case 2: v = pe.x; break;
            case 3: v = pe.y; break;
            case 4: v = e < N ? s_pos[N + e].x - pe.x : 0.0f; break;
            case 5: v = e < N ? s_pos[N + e].y - pe.y : 0.0f; break;
            default: v = e < N ? 0.0f : (e < 2 * N ? 1.0f : 2.0f); break;
        }
        nf[q] = v;
    }

    // edge count: unordered pairs among agents+obstacles with 0 < d2 <= R2,
    // enumerated circulantly (m, m+t mod M), t = 1..M/2 (each pair once).
    const int half = M >> 1;
    int pairs = 0;
    for (int tt = 1; tt <= half; ++tt) {
        const int mend = (2 * tt == M) ? half : M;
        for (int m = lane; m < mend; m += kWave) {
            int m2 = m + tt;
            if (m2 >= M) m2 -= M;
            const float2 a = s_pos[collider_entity(m, N)], c = s_pos[collider_entity(m2, N)];
            const float dx = a.x - c.x, dy = a.y - c.y;
            const float d2 = dx * dx + dy * dy;
            pairs += (d2 > 0.0f) & (d2 <= p.R2);
        }
    }
    const int edges = 2 * wave_sum(pairs) + 2 * N;

    // state + per-env outputs
    const bool moved = p.mode == kModeStep || do_reset;
    if (moved) {
        const int ne = do_reset ? E : N;
        for (int e = lane; e < ne; e += kWave) p.pos[eb * E + e] = s_pos[e];
        for (int i = lane; i < N; i += kWave) p.vel[eb * N + i] = s_vel[i];
    }
    if (lane == 0) {
        p.step_count[b] = t;
        p.episode[b] = ep;
        p.ep_acc[b] = acc;
        p.done[b] = done ? 1 : 0;
        p.edge_count[b] = edges;
    }
    return edges;
}

__global__ __launch_bounds__(kBlock) void gsm_step_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.x * kWavesPerBlock + wave;
    int edges = 0;
    if (b < p.B) edges = env_step(p, b, lane, smem + wave * p.wave_lds_step);
    int *s_bc = (int *)(smem + kWavesPerBlock * p.wave_lds_step);
    if (lane == 0) s_bc[wave] = edges;
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += s_bc[w];
        p.block_edge_sum[blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// edge emitter
// ---------------------------------------------------------------------------
struct EdgeSink {
    int32_t *src, *dst;
    float *attr;
};

// One (row, 64-candidate chunk): ballot the predicate, write the set lanes at
// off + rank, return the chunk's edge count.
__device__ __forceinline__ int emit_chunk(const EdgeSink &k, int64_t off, bool pred,
                                          int32_t gsrc, int32_t gdst, float d2) {
    const uint64_t mask = __ballot(pred);
    if (pred) {
        const int64_t o = off + lanes_below(mask);
        k.src[o] = gsrc;
        k.dst[o] = gdst;
        k.attr[o] = sqrtf(d2);
    }
    return __popcll(mask);
}

__device__ void env_emit(const DevParams &p, const int b, const int lane, int64_t off,
                         unsigned char *lds) {
    const int N = p.N, No = p.No, E = p.E;
    float2 *s_pos = (float2 *)lds;
    const int64_t eb = b;
    for (int e = lane; e < E; e += kWave) s_pos[e] = p.pos[eb * E + e];
    wave_sync();
    const EdgeSink k{p.edge_index, p.edge_index + p.edge_capacity, p.edge_attr};
    const int32_t g0 = (int32_t)(eb * E);

    // agent rows: candidates agents [0,N), own goal, obstacles (entity order)
    const int KA = N + 1 + No;
    for (int i = 0; i < N; ++i) {
        const float2 a = s_pos[i];
        for (int c0 = 0; c0 < KA; c0 += kWave) {
            const int l = c0 + lane;
            bool pred = false;
            int dst = 0;
            float d2 = 0.0f;
            if (l < KA) {
                dst = l < N ? l : (l == N ? N + i : N + l - 1);
                const float2 q = s_pos[dst];
                const float dx = a.x - q.x, dy = a.y - q.y;
                d2 = dx * dx + dy * dy;
                pred = l == N || (l != i && d2 > 0.0f && d2 <= p.R2);
            }
            off += emit_chunk(k, off, pred, g0 + i, g0 + dst, d2);
        }
    }
    // goal rows: goal i -> agent i
    for (int i = lane; i < N; i += kWave) {
        const float2 g = s_pos[N + i], a = s_pos[i];
        const float dx = g.x - a.x, dy = g.y - a.y;
        const float d2 = dx * dx + dy * dy;
        k.src[off + i] = g0 + N + i;
        k.dst[off + i] = g0 + i;
        k.attr[off + i] = sqrtf(d2);
    }
    off += N;
    // obstacle rows: candidates agents, obstacles (self excluded)
    const int KO = N + No;
    for (int o = 0; o < No; ++o) {
        const int src = 2 * N + o;
        const float2 a = s_pos[src];
        for (int c0 = 0; c0 < KO; c0 += kWave) {
            const int l = c0 + lane;
            bool pred = false;
            int dst = 0;
            float d2 = 0.0f;
            if (l < KO) {
                dst = collider_entity(l, N);
                const float2 q = s_pos[dst];
                const float dx = a.x - q.x, dy = a.y - q.y;
                d2 = dx * dx + dy * dy;
                pred = dst != src && d2 > 0.0f && d2 <= p.R2;
            }
            off += emit_chunk(k, off, pred, g0 + src, g0 + dst, d2);
        }
    }
}

__global__ __launch_bounds__(kBlock) void gsm_emit_edges_kernel(DevParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int *s_red = (int *)(smem + kWavesPerBlock * p.wave_lds_emit);
    // exclusive prefix of the step kernel's per-workgroup edge sums
    // (host guarantees edge_capacity < 2^31, so int32 sums cannot overflow)
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
    env_emit(p, b, lane, off, smem + wave * p.wave_lds_emit);
}

int grid_blocks(const DevParams &p) {
    const int per_block = kWavesPerBlock * p.G;
    return (p.B + per_block - 1) / per_block;
}
const void *step_kernel_fn(const DevParams &p) {
    if (p.path == kPathRagged) return step_ragged_kernel_fn();
    return p.path == kPathSeg ? step_seg_kernel_fn(p) : reinterpret_cast<const void *>(&gsm_step_kernel);
}
const void *emit_kernel_fn(const DevParams &p) {
    if (p.path == kPathRagged) return emit_ragged_kernel_fn();
    return p.path == kPathSeg ? emit_seg_kernel_fn(p) : reinterpret_cast<const void *>(&gsm_emit_edges_kernel);
}
size_t step_kernel_lds(const DevParams &p) { return (size_t)kWavesPerBlock * p.wave_lds_step + 16; }
size_t emit_kernel_lds(const DevParams &p) { return (size_t)kWavesPerBlock * p.wave_lds_emit + 16; }

static hipError_t launch_fn(const void *fn, const DevParams &p, size_t lds, hipStream_t s) {
    (void)hipGetLastError();   // report this launch's error only
    void *args[] = {const_cast<DevParams *>(&p)};
    const hipError_t e = hipLaunchKernel(fn, dim3(grid_blocks(p)), dim3(kBlock), args, lds, s);
    return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_step_kernel(const DevParams &p, hipStream_t s) {
    return launch_fn(step_kernel_fn(p), p, step_kernel_lds(p), s);
}

hipError_t launch_emit_kernel(const DevParams &p, hipStream_t s) {
    return launch_fn(emit_kernel_fn(p), p, emit_kernel_lds(p), s);
}

hipError_t launch_step(const DevParams &p, hipStream_t s) {
    hipError_t e = launch_step_kernel(p, s);
    if (e != hipSuccess) return e;
    return launch_emit_kernel(p, s);
}

}  // namespace gsm
