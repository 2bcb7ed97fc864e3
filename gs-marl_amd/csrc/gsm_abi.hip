// gsm_abi.hip — extern "C" boundary of libgsm.so (declared in include/gsm.h).
//
// Host-only bookkeeping: validate the config, derive the fp32 constants the
// kernels use (same fp32 operations as oracle/batch_ref.py:Spec), borrow the
// caller's device buffers, launch, and optionally capture whole multi-step
// rollouts into a HIP graph. No allocation and no synchronisation happens in
// gsm_step / gsm_reset / gsm_observe.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "gsm.h"
#include "gsm_internal.h"
#include "gsm_philox.h"

struct gsm_handle {
    gsm_config cfg;
    gsm_sizes sz;
    gsm::DevParams dp;      // constants + bound buffers
    bool bound = false;
    std::string err;
    // graph capture
    hipStream_t cap_stream = nullptr;
    int32_t *bsum_alt = nullptr;   // second half of the per-workgroup edge-sum double buffer (lagged emission)
    int32_t *block_order = nullptr;   // ragged mixed: workgroup -> env block, heaviest first
    int32_t *order_host = nullptr;    // pinned staging of block_order's async upload
    int32_t *place_order = nullptr;   // ragged mixed: the rollout's placement order (inside block_order)
    hipEvent_t order_copied = nullptr;   // recorded after the last upload (staging free again)
    struct Slot {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        std::vector<hipEvent_t> events;   // timing event-record nodes
        int steps = 0;
        int kern = 0;
        bool each = false;
        uint64_t *gran = nullptr;     // fused rollout: a 16-byte header, then the edge-sum granules
        void *gran_base = nullptr;    // its allocation (gran_malloc: the granules end at its end)
        // one-env-per-wave segmented rollout: the chunk sums of its one-hop
        // CSR prefix (two halves of csum_half words inside gran) and its pace
        // counters (two halves of kPaceKeys x kPaceStride u32; nullptr: pacing
        // off); a launch uses half (launches & 1) and zeroes the other for the
        // slot's next launch
        uint64_t *csum = nullptr;
        int64_t csum_half = 0;
        uint32_t *pace = nullptr;
        uint32_t launches = 0;
        uint32_t last_epoch = 0xffffffffu;   // the epoch of the slot's previous launch
        bool roll = false;            // the graph is one rollout launch
        // A rollout graph without timing events is one kernel node: launched
        // directly (the same kernel, grid and arguments) — a plain dispatch
        // costs the host less than a graph launch; the graph is kept for
        // gsm_graph_info and as the record of what runs.
        bool direct = false;
        const void *fn = nullptr;
        dim3 grid, block;
        unsigned lds = 0;
        gsm::DevParams args;
    } slots[GSM_GRAPH_SLOTS];
    uint32_t *roll_status = nullptr;  // fused rollout: a bounded wait gave up (sticky until read)
    void *edge_scratch = nullptr;     // fused rollout in the bound buffers: edges of all but the last step
    void *slab = nullptr;             // ragged rollout: per-env edge slabs (depth + 1 steps)
    size_t slab_bytes = 0;
    // the stream of the last rollout-slot launch: rollout slots share the
    // handle's scratch (edge scratch, slabs) and state, so launches on
    // another stream first wait for it (gsm_graph_launch)
    hipStream_t roll_stream = nullptr;
    bool roll_launched = false;
    hipEvent_t roll_done = nullptr;   // recorded behind every rollout-slot launch
    uint32_t eager_last_epoch = 0xffffffffu;   // the eager one-launch step's previous epoch
    uint64_t *eager_csum = nullptr;           // its chunk-sum halves (segmented: inside eager_gran)
    int64_t eager_csum_half = 0;
    uint32_t eager_launches = 0;
    uint32_t *eager_epoch = nullptr;  // the segmented one-launch step's device-side epoch (inside eager_gran)
    bool eager_dev_epoch = true;      // GSM_EAGER_DEV_EPOCH=0 (an A/B knob): host epochs outside captures
    // gsm_step as a one-step rollout launch (step + its edges in one kernel):
    // -1 not yet decided for this config, 0 no (two launches), 1 yes
    int eager_roll = -1;
    uint64_t *eager_gran = nullptr;   // its granules (K = 1)
    uint64_t *eager_gran_end = nullptr;
    void *eager_base = nullptr;       // their allocation
};

namespace {

thread_local std::string g_err;

int fail(gsm_handle *h, int code, const std::string &msg) {
    if (h) h->err = msg;
    g_err = msg;
    return code;
}

int hip_fail(gsm_handle *h, hipError_t e, const char *where) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: hipError %d (%s)", where, (int)e, hipGetErrorString(e));
    return fail(h, GSM_EHIP, buf);
}

int align16(int x) { return (x + 15) & ~15; }

// Ragged mixed batches: the step kernel's workgroups take their env blocks
// heaviest first, so the long assignment chains (polygon/line envs with many
// agents) start in the first residency round instead of waiting behind light
// envs. Cost of an env ~ N_env^2 for polygon/line (assignment path
// iterations), N_env for navigation; a block costs its heaviest env. The
// order only schedules: every output is the same under any order (each
// workgroup writes its own env block's slots). Recomputed when the seed that
// draws the env shapes changes (never per step). The upload is stream-ordered
// on the caller's stream `s` (from pinned staging), so kernels enqueued on it
// before the reseed finish with the old order and every later one sees the new
// order; the staging buffer is reused only after the previous upload read it.
//
// The same upload carries the ragged rollout's placement order (after the nb
// block entries): the grid's W = 4 * ceil(B / 4) envs by descending cost per
// step, linear in N_env per family: polygon / line a + b N, navigation
// c + d N, from scans of the C4 launch time (`tools/gpu.sh envsweep TAG c4
// GSM_PLACE_MODEL a,b,c,d`). Round 3 (navigation sweep on the scalar path):
// 63 + 27 N and 55 + 18 N (20 + 7 N: 39.4 us per step, 55 + 18 N: 36.9,
// 70 + 24 N: 38.9). Round 4, with the navigation sweep and the assignment's
// passes off the scalar path the navigation envs cost a fraction of an
// assignment env and the assignment's cost is flatter in N
// (profiles/r4_stamps/stamps_c4.json): 200 + 20 N and 10 + 3 N, 27.2 us per
// step against 29.4 for the round-3 weights (profiles/r4_place); padding envs
// (b >= B) last. roll_place (gsm_ragged_kernels.hip) deals them to the
// SIMDs in strata.
constexpr int kXcds = 8;   // MI355X: 8 XCDs of 32 CUs
int update_block_order(gsm_handle *h, hipStream_t s) {
    const gsm::DevParams &p = h->dp;
    if (p.path != gsm::kPathRagged || p.scenario != gsm::kScnMixed) return GSM_OK;
    const int nb = h->sz.n_blocks, per = h->sz.envs_per_block;
    const int W = (p.B + gsm::kWavesPerBlock - 1) / gsm::kWavesPerBlock * gsm::kWavesPerBlock;
    std::vector<int64_t> key(nb), cost(W, 0);
    // cost units per env and step: polygon/line a + b N, navigation c + d N,
    // the C4 rollout's best of a scan (tools/gpu.sh envsweep,
    // GSM_PLACE_MODEL="a,b,c,d" overrides)
    int64_t ma = 200, mb = 20, mc = 10, md = 3;
    if (const char *ev = getenv("GSM_PLACE_MODEL")) {
        long long x[4];
        if (sscanf(ev, "%lld,%lld,%lld,%lld", &x[0], &x[1], &x[2], &x[3]) == 4) {
            ma = x[0];
            mb = x[1];
            mc = x[2];
            md = x[3];
        }
    }
    for (int b = 0; b < p.B; ++b) {
        const int64_t gid = p.env_base + b;
        const gsm::Philox4 x = gsm::philox4x32_10(0u, 0u, (uint32_t)gid, gsm::kTagShape, p.seed_lo, p.seed_hi);
        const int n = p.n_min + (int)(((uint64_t)x.x0 * (uint64_t)(p.N - p.n_min + 1)) >> 32);
        const bool lsa = (gid % 3) != gsm::kScnNav;
        cost[b] = lsa ? ma + mb * (int64_t)n : mc + md * (int64_t)n;
        const int64_t ce = lsa ? (int64_t)n * n : n;
        if (b / per < nb && ce > key[b / per]) key[b / per] = ce;
    }
    std::vector<int32_t> order(nb + W);
    for (int k = 0; k < nb; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.begin() + nb, [&](int32_t a, int32_t b) { return key[a] > key[b]; });
    for (int k = 0; k < W; ++k) order[nb + k] = k;
    // XCD-local dealing (round 5): roll_place gives SIMD i (XCD-major: the
    // SIMDs of XCD x are i in [x S/8, (x+1) S/8)) entry i of even strata and
    // S - 1 - i of odd ones. Each XCD takes a contiguous block of W/8 envs, its
    // own cost order cut into strata of S/8 and snaked over its SIMDs, so envs
    // next to each other in memory (their per-env outputs and CSR edges share
    // cache lines) are written from one XCD's L2 instead of up to eight, each
    // writing back its own partial copy of the line. GSM_PLACE_XCD=0: one cost
    // order over the whole grid (round 4).
    int n_cu = 0, dev = 0;
    const char *px = getenv("GSM_PLACE_XCD");
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 0;
    const int S = 4 * n_cu, SX = S / kXcds;
    if (!(px && atoi(px) == 0) && S > 0 && S % kXcds == 0 && W % S == 0) {
        const int R = W / S, WX = W / kXcds;
        std::vector<int32_t> blk(WX);
        for (int x = 0; x < kXcds; ++x) {
            for (int k = 0; k < WX; ++k) blk[k] = x * WX + k;
            std::stable_sort(blk.begin(), blk.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
            for (int r = 0; r < R; ++r)
                for (int il = 0; il < SX; ++il) {
                    const int i = x * SX + il;                   // the SIMD
                    const int j = (r & 1) ? S - 1 - i : i;       // its table entry in stratum r
                    const int e = (r & 1) ? SX - 1 - il : il;    // snaked within the XCD
                    order[nb + (size_t)r * S + j] = blk[(size_t)r * SX + e];
                }
        }
    } else {
        std::stable_sort(order.begin() + nb, order.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
    }
    const size_t bytes = (size_t)(nb + W) * sizeof(int32_t);
    hipError_t e = hipSuccess;
    if (!h->block_order) {
        e = hipMalloc(&h->block_order, bytes);
        if (e != hipSuccess) {
            h->block_order = nullptr;
            return hip_fail(h, e, "hipMalloc (block order)");
        }
        e = hipHostMalloc((void **)&h->order_host, bytes, hipHostMallocDefault);
        if (e != hipSuccess) {
            h->order_host = nullptr;
            return hip_fail(h, e, "hipHostMalloc (block order staging)");
        }
        e = hipEventCreateWithFlags(&h->order_copied, hipEventDisableTiming);
        if (e != hipSuccess) {
            h->order_copied = nullptr;
            return hip_fail(h, e, "hipEventCreate (block order)");
        }
    } else {
        e = hipEventSynchronize(h->order_copied);   // the previous upload has read the staging
        if (e != hipSuccess) return hip_fail(h, e, "hipEventSynchronize (block order)");
    }
    memcpy(h->order_host, order.data(), bytes);
    e = hipMemcpyAsync(h->block_order, h->order_host, bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(h, e, "hipMemcpyAsync (block order)");
    e = hipEventRecord(h->order_copied, s);
    if (e != hipSuccess) return hip_fail(h, e, "hipEventRecord (block order)");
    h->dp.block_order = h->block_order;
    h->place_order = h->block_order + nb;
    return GSM_OK;
}

int check_config(const gsm_config *c, std::string *why) {
    if (!c) { *why = "config is NULL"; return GSM_EINVAL; }
    if (c->abi_version != GSM_ABI_VERSION) {
        *why = "abi_version mismatch (library " + std::to_string(GSM_ABI_VERSION) + ", caller " +
               std::to_string(c->abi_version) + ")";
        return GSM_EINVAL;
    }
    if (c->scenario < GSM_SCEN_NAVIGATION || c->scenario > GSM_SCEN_MIXED) {
        *why = "unsupported scenario";
        return GSM_EINVAL;
    }
    if (c->n_envs < 1) { *why = "n_envs must be >= 1"; return GSM_EINVAL; }
    if (c->n_agents < 1 || c->n_agents > 1024) { *why = "n_agents must be in [1, 1024]"; return GSM_EINVAL; }
    if (c->n_obstacles < 0 || c->n_obstacles > 1024) { *why = "n_obstacles must be in [0, 1024]"; return GSM_EINVAL; }
    if (c->episode_length < 1) { *why = "episode_length must be >= 1"; return GSM_EINVAL; }
    const bool ragged = c->scenario != GSM_SCEN_NAVIGATION;
    if (!(c->dt > 0) || !(c->mass > 0) || !(c->contact_margin > 0)) {
        *why = "dt, mass and contact_margin must be > 0";
        return GSM_EINVAL;
    }
    if (ragged ? !(c->world_half >= 0) : !(c->world_half > 0)) {
        *why = "world_half must be > 0 (ragged scenarios: >= 0, 0 = sqrt(N_env/3) per env)";
        return GSM_EINVAL;
    }
    if (ragged) {
        if (c->n_agents > GSM_RAGGED_MAX_AGENTS) {
            *why = "polygon/line/mixed: n_agents must be <= GSM_RAGGED_MAX_AGENTS (32)";
            return GSM_EINVAL;
        }
        if (c->scenario == GSM_SCEN_MIXED ? c->n_obstacles != c->n_agents : c->n_obstacles != 0) {
            *why = "mixed needs n_obstacles == n_agents (navigation envs); polygon/line need n_obstacles == 0";
            return GSM_EINVAL;
        }
        if (c->scenario == GSM_SCEN_MIXED && (c->n_agents_min < 1 || c->n_agents_min > c->n_agents)) {
            *why = "mixed needs 1 <= n_agents_min <= n_agents";
            return GSM_EINVAL;
        }
        if (!(c->formation_radius >= 0) || !isfinite(c->formation_radius)) {
            *why = "formation_radius must be a finite value >= 0";
            return GSM_EINVAL;
        }
    }
    if (!(c->damping >= 0 && c->damping <= 1)) { *why = "damping must be in [0, 1]"; return GSM_EINVAL; }
    if (!(c->sense_radius >= 0) || !(c->contact_cutoff > 0)) {
        *why = "sense_radius must be >= 0 and contact_cutoff > 0";
        return GSM_EINVAL;
    }
    return GSM_OK;
}

// kernel family and envs per wave for a config
void choose_path(const gsm_config *c, int *path, int *G) {
    const int M = c->n_agents + c->n_obstacles;
    if (c->scenario != GSM_SCEN_NAVIGATION) {
        *path = gsm::kPathRagged;
        *G = 1;
    } else if (M <= gsm::kWave) {
        *path = gsm::kPathSeg;
        // as many envs per wave as fit (at most kMaxSegEnvsPerWave), but no
        // fewer waves than one workgroup per CU (256 x 4): a small batch of
        // small envs is latency-bound, and packing it into fewer waves leaves
        // CUs idle
        int g = gsm::kWave / M;
        g = g > gsm::kMaxSegEnvsPerWave ? gsm::kMaxSegEnvsPerWave : g;
        const int64_t fill = c->n_envs / 1024;
        *G = fill < g ? (fill < 1 ? 1 : (int)fill) : g;
    } else {
        *path = gsm::kPathTile;
        *G = 1;
    }
}

// target rows per env: navigation goals = N, polygon centre 1, line ends 2,
// mixed = N (its navigation envs)
int targets_of(const gsm_config *c) {
    switch (c->scenario) {
        case GSM_SCEN_POLYGON: return 1;
        case GSM_SCEN_LINE: return 2;
        default: return c->n_agents;
    }
}

void fill_sizes(const gsm_config *c, gsm_sizes *s) {
    const int N = c->n_agents, No = c->n_obstacles, M = N + No, T = targets_of(c);
    int path, G;
    choose_path(c, &path, &G);
    s->n_entities = N + T + No;
    s->node_feat_dim = 7;
    s->obs_dim = 6;
    s->envs_per_block = path == gsm::kPathTile ? 1 : gsm::kWavesPerBlock * G;
    s->n_blocks = (c->n_envs + s->envs_per_block - 1) / s->envs_per_block;
    // radius edges among colliders + the agent <-> target edges (2 per agent
    // per target it is tied to: own goal / centre: 1, line ends: 2)
    int max_edges = M * (M - 1) + 2 * N;
    if (c->scenario == GSM_SCEN_LINE) max_edges = N * (N - 1) + 4 * N;
    if (c->scenario == GSM_SCEN_MIXED && N * (N - 1) + 4 * N > max_edges) max_edges = N * (N - 1) + 4 * N;
    s->max_edges_per_env = max_edges;
    s->n_colliders = M;
    s->n_targets = T;
    s->mask_words = path == gsm::kPathTile ? (M + 63) / 64 : 1;
    s->edge_capacity = (int64_t)c->n_envs * s->max_edges_per_env;
}

// fp32 constants, formed exactly like oracle/batch_ref.py:Spec (fp32 mode).
void derive(const gsm_config *c, gsm::DevParams *p) {
    memset(p, 0, sizeof *p);
    const int N = c->n_agents, No = c->n_obstacles;
    p->B = c->n_envs;
    p->N = N;
    p->No = No;
    p->T = targets_of(c);
    p->E = N + p->T + No;
    p->M = N + No;
    p->scenario = c->scenario;
    p->n_min = c->scenario == GSM_SCEN_MIXED ? c->n_agents_min : N;
    choose_path(c, &p->path, &p->G);
    p->W = p->path == gsm::kPathTile ? (p->M + 63) / 64 : 1;
    p->EL = c->episode_length;
    p->auto_reset = c->auto_reset != 0;
    p->shared_reward = c->shared_reward != 0;
    p->seed_lo = (uint32_t)(c->seed & 0xFFFFFFFFull);
    p->seed_hi = (uint32_t)(c->seed >> 32);
    p->env_base = c->env_base;
    p->strict = c->strict_degenerate != 0;
    if (p->path == gsm::kPathRagged) {
        // assignment scratch (cost matrix, duals) + staged entity positions [E]
        p->wave_lds_step = align16(gsm::lsa_lds_bytes(N) + 8 * p->E);
        p->wave_lds_emit = align16(8 * p->E);
    } else if (p->path == gsm::kPathSeg) {
        // positions + staged node-feature rows of the wave's G envs
        p->wave_lds_step = align16(8 * p->G * p->E + 28 * p->G * p->E);
        // one env per wave: + the staged edge list (stage_rows)
        p->wave_lds_emit = align16(p->G == 1 ? 36 * p->E : 8 * p->G * p->E);
    } else {
        // tile: whole-workgroup LDS: positions, velocities, new positions, costs, reductions,
        // the two degenerate-state flags;
        // + the symmetric sweep's column pairs, agent-row words and obstacle-row
        // agent bits when they fit in 32 KB (gsm_tile_kernels.hip: obs_sweep_sym)
        p->wave_lds_step = align16(8 * p->E + 8 * N + 8 * N + 4 * N + 20 * (gsm::kTileBlock / gsm::kWave) + 8);
        const int sym = 16 * ((N + 1) / 2) + 16 * N * p->W + 8 * No * p->W + 16;
        p->tile_sym = sym <= 32768;
        if (p->tile_sym) p->wave_lds_step += sym;
        // emit: positions, reductions and the staged edge words (gsm::kTileEmitScr)
        p->wave_lds_emit = align16(8 * p->E + 4 * (gsm::kTileBlock / gsm::kWave) + 4 * gsm::kTileEmitScr);
    }
    const float L = c->world_half;
    p->L = L;
    p->twoL = L * 2.0f;
    p->fixed_L = p->path == gsm::kPathRagged ? (L > 0.0f ? L : 0.0f) : L;
    p->form_r = c->formation_radius;
    p->dt = c->dt;
    p->omd = 1.0f - c->damping;
    p->mass = c->mass;
    p->inv_mass = 1.0f / c->mass;
    p->cf = c->contact_force;
    p->k = c->contact_margin;
    p->inv_k = 1.0f / c->contact_margin;
    p->sens = c->sensitivity;
    p->max_speed = c->max_speed;
    const float R = c->sense_radius;
    p->R2 = R * R;
    const float sa = c->agent_size, so = c->obstacle_size;
    p->dmin_aa = sa + sa;
    p->dmin_ao = sa + so;
    p->dmin2_aa = p->dmin_aa * p->dmin_aa;
    p->dmin2_ao = p->dmin_ao * p->dmin_ao;
    // beyond d - dmin > cutoff*k the pair force is below cf*k*exp(-cutoff)
    // (4e-19 at the default cutoff 40): skipped (contact cutoff)
    const float caa = p->dmin_aa + c->contact_cutoff * c->contact_margin;
    const float cao = p->dmin_ao + c->contact_cutoff * c->contact_margin;
    p->cut2_aa = caa * caa;
    p->cut2_ao = cao * cao;
}

hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Point a launch's outputs at `o` (NULL members keep the bound buffers).
int redirect(gsm_handle *h, gsm::DevParams *p, const gsm_outputs *o) {
    if (!o) return GSM_OK;
    if (o->edge_index && o->edge_capacity < 1)
        return fail(h, GSM_EINVAL, "redirected edge_index needs edge_capacity >= 1");
    if (o->edge_index && o->edge_capacity >= (int64_t)1 << 31)
        return fail(h, GSM_EINVAL, "edge_capacity must be < 2^31");
    if (!!o->edge_index != !!o->edge_attr)
        return fail(h, GSM_EINVAL, "edge_index and edge_attr are redirected together");
    if (o->node_feat) p->node_feat = o->node_feat;
    if (o->reward) p->reward = o->reward;
    if (o->cost) p->cost = o->cost;
    if (o->done) p->done = o->done;
    if (o->edge_count) p->edge_count = o->edge_count;
    if (o->edge_ptr) p->edge_ptr = o->edge_ptr;
    if (o->edge_index) {
        p->edge_index = o->edge_index;
        p->edge_attr = o->edge_attr;
        p->edge_capacity = o->edge_capacity;
    }
    if (o->assign) p->assign = o->assign;
    p->nf_full = 1;
    return GSM_OK;
}

uint32_t next_launch_epoch();
hipError_t clear_status(gsm_handle *h);
// u64 words between the chunk sums of the segmented rollout's one-hop prefix
// (gsm_device.h roll_prefix): each on a 64-byte line of its own
constexpr int kCsumStride = 8;
// a launch epoch other than `last` (the previous launch of the same granules:
// the process-wide counter wraps after 2^20 launches, and an idle slot's
// granules still carry its last launch's tags), recorded as the new last
uint32_t fresh_epoch(uint32_t &last) {
    uint32_t e = next_launch_epoch();
    if (e == last) e = next_launch_epoch();
    last = e;
    return e;
}

// The rollout granules (in-launch hand-off words, gsm_device.h) are allocated
// uncached: an agent-scope load of a granule line that this XCD's L2 still
// holds from an earlier read can be served stale until the line leaves the
// L2, and the hand-off then re-polls. Same box, one run each (profiles/
// r4_gran): C2 3.44 -> 3.16 us per step, H 8.46 -> 8.31, C3 and C4 within
// noise. GSM_GRAN_MEM = "hip" / "fine" selects hipMalloc / fine-grained (A/B).
//
// The used bytes are placed at the END of a whole number of 4 KiB pages
// (*gran = *base + the slack): an access past the last granule leaves the
// allocation instead of reading its own slack unnoticed (gsm_device.h
// gran_chk; the checked build tests every address against the end).
hipError_t gran_malloc(void **base, uint64_t **gran, size_t bytes) {
    const size_t alloc = (bytes + 4095) & ~(size_t)4095;
    const char *ev = getenv("GSM_GRAN_MEM");
    hipError_t e;
    if (ev && !strcmp(ev, "hip"))
        e = hipMalloc(base, alloc);
    else if (ev && !strcmp(ev, "fine"))
        e = hipExtMallocWithFlags(base, alloc, hipDeviceMallocFinegrained);
    else
        e = hipExtMallocWithFlags(base, alloc, hipDeviceMallocUncached);
    if (e != hipSuccess) {
        *base = nullptr;
        *gran = nullptr;
        return e;
    }
    *gran = (uint64_t *)((char *)*base + (alloc - bytes));
    return hipSuccess;
}

// gsm_step as ONE launch: the config's fused rollout kernel with K = 1 (the
// step, then its edges at the CSR offset of the in-launch prefix) instead of
// the step kernel + the emit kernel — the same operations, so the same outputs
// (tests/test_gpu_roll.py), when the grid fits one residency round (decided
// once per handle). The default for the one-env-per-wave segmented rollout
// (navigation with 6, 12 or 24 agents: 15.4 vs 16.5 us per step at H, 13.1 vs
// 15.5 at 12 x 8192; DESIGN.md §4, profiles/r5_ab/eager_forms); the packed
// small-env and tile rollouts keep the two launches unless
// GSM_EAGER_ONE_LAUNCH=1 (there the pair was faster: C2 8.7 vs 9.4, C3 27.9
// vs 29.6 us), and GSM_EAGER_ONE_LAUNCH=0 keeps them everywhere. The ragged
// path always runs two launches.
constexpr int kEagerIneligible = 1;
// Decided once per handle, at gsm_bind (the hand-off granules allocated and
// zeroed there, so that no step allocates or synchronises): h->eager_roll 1
// when the config has a rollout kernel whose grid fits one residency round
// and the one launch is wanted (above), else 0.
int eager_setup(gsm_handle *h) {
    gsm::DevParams p = h->dp;
    p.action_fmt = GSM_ACT_INDEX;   // (every format's kernel has the same LDS and occupancy)
    h->eager_roll = 0;
    if (p.path == gsm::kPathRagged) return GSM_OK;
    const bool tile = p.path == gsm::kPathTile;
    const void *fn = tile ? gsm::roll_tile_kernel_fn(p, false) : gsm::roll_seg_kernel_fn(p, false);
    if (!fn) return GSM_OK;
    const int per_blk = tile ? 1 : gsm::roll_seg_envs_per_block(p);
    const int nb = tile ? gsm::step_grid_blocks(p) : (p.B + per_blk - 1) / per_blk;
    const size_t lds = tile ? gsm::roll_tile_kernel_lds(p) : gsm::roll_kernel_lds(p);
    const char *ev = getenv("GSM_EAGER_ONE_LAUNCH");
    const bool want = ev && *ev ? atoi(ev) != 0 : !tile && !gsm::roll_packed(p);
    if (!want) return GSM_OK;
    const size_t nc = ((size_t)nb + gsm::kPrefixChunk - 1) / gsm::kPrefixChunk;
    if (nc > (size_t)gsm::kWave) return GSM_OK;   // roll_prefix: one chunk sum per lane
    const char *de = getenv("GSM_EAGER_DEV_EPOCH");
    h->eager_dev_epoch = !(de && *de && atoi(de) == 0);
    int dev = 0, per_cu = 0, n_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, gsm::roll_block_threads(p), lds);
    if (e != hipSuccess) return hip_fail(h, e, "occupancy query (eager rollout)");
    if ((int64_t)per_cu * n_cu < nb) return GSM_OK;
    // (tile path: aggregates + inclusive prefixes per workgroup;
    // segmented: aggregates + two halves of chunk sums; packed small envs:
    // per-wave counts + group sums)
    const size_t xw = (size_t)nb * gsm::kWavesPerBlock;
    const size_t words = std::max({2 * (size_t)nb, (size_t)nb + 2 * nc * kCsumStride,
                                   xw + (xw + gsm::kWave - 1) / gsm::kWave});
    // then the segmented step's device-side epoch replicas
    const size_t epoch_bytes = (size_t)gsm::kEpochReps * gsm::kEpochStride * sizeof(uint32_t);
    const size_t bytes = 16 + words * sizeof(uint64_t) + epoch_bytes;
    if (h->eager_base) {   // (a retried setup)
        (void)hipFree(h->eager_base);
        h->eager_base = nullptr;
        h->eager_gran = nullptr;
    }
    e = gran_malloc(&h->eager_base, &h->eager_gran, bytes);
    h->eager_gran_end = h->eager_gran ? (uint64_t *)((char *)h->eager_gran + bytes) : nullptr;
    h->eager_csum = h->eager_gran ? h->eager_gran + 2 + nb : nullptr;
    h->eager_csum_half = (int64_t)(nc * kCsumStride);
    h->eager_epoch = h->eager_gran ? (uint32_t *)((char *)h->eager_gran + bytes - epoch_bytes) : nullptr;
    if (e != hipSuccess) { h->eager_gran = nullptr; return hip_fail(h, e, "hipMalloc (eager granules)"); }
    e = gsm::launch_granule_init(h->eager_gran, bytes, 0u, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e == hipSuccess) {   // the first epoch: a fresh one of the process-wide sequence, in every replica
        std::vector<uint32_t> ep((size_t)gsm::kEpochReps * gsm::kEpochStride, 0u);
        const uint32_t e0 = next_launch_epoch();
        for (int r = 0; r < gsm::kEpochReps; ++r) ep[(size_t)r * gsm::kEpochStride] = e0;
        e = hipMemcpy(h->eager_epoch, ep.data(), epoch_bytes, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !h->roll_status) {
        e = hipMalloc(&h->roll_status, 16);
        if (e == hipSuccess) e = clear_status(h);
        if (e != hipSuccess) h->roll_status = nullptr;
    }
    if (e != hipSuccess) return hip_fail(h, e, "eager rollout setup");
    h->eager_roll = 1;
    return GSM_OK;
}

int launch_step_roll(gsm_handle *h, gsm::DevParams p, hipStream_t s) {
    if (h->eager_roll < 0) {   // (gsm_bind decides it; kept for a handle bound before)
        const int rc = eager_setup(h);
        if (rc) return rc;
    }
    if (h->eager_roll == 0 || p.path == gsm::kPathRagged) return kEagerIneligible;
    const bool tile = p.path == gsm::kPathTile;
    // one env per wave: the kernel takes its epoch and chunk-sum half from
    // device memory and advances them itself (gsm_roll_seg_kernel kEager), so
    // the launch holds no per-launch host state and may be recorded into a
    // stream capture (torch.cuda.graph around a policy + env.step). The tile
    // and packed small-env forms take both from the host per launch: on a
    // capturing stream they give way to the two launches, which hold none.
    const void *fn = tile ? nullptr : gsm::roll_seg_eager_kernel_fn(p);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
    if (fn && !capturing && !h->eager_dev_epoch) fn = nullptr;
    const bool dev_epoch = fn != nullptr;
    if (!dev_epoch) {
        if (capturing) return kEagerIneligible;
        fn = tile ? gsm::roll_tile_kernel_fn(p, false) : gsm::roll_seg_kernel_fn(p, false);
    }
    if (!fn) return kEagerIneligible;   // (the action format may differ per call: checked every time)
    const int per_blk = tile ? 1 : gsm::roll_seg_envs_per_block(p);
    const int nb = tile ? gsm::step_grid_blocks(p) : (p.B + per_blk - 1) / per_blk;
    const size_t lds = tile ? gsm::roll_tile_kernel_lds(p) : gsm::roll_kernel_lds(p);
    // the step's outputs: the bound (or redirected) buffers, its edges too
    p.ro = gsm::DevParams::RollOut{p.node_feat, p.reward, p.cost, p.done, p.edge_count, p.edge_ptr, p.edge_index,
                                   p.edge_attr, 0, 0, 0, 0, 0, 0, 0, p.edge_capacity, nullptr, nullptr, p.assign, 0};
    const int xW = nb * gsm::kWavesPerBlock, xNG = (xW + gsm::kWave - 1) / gsm::kWave;
    // (one step: no pacing)
    p.roll = gsm::DevParams::Roll{(const char *)p.actions, 0, 1, 0, 1, xW, xNG, 0, 0, 0, h->eager_gran + 2,
                                  h->roll_status, dev_epoch ? 0u : fresh_epoch(h->eager_last_epoch)};
    // (device epoch: the halves in a fixed order, the kernel picks by the
    // epoch's parity; else this launch's half by the host's launch parity)
    const int par = dev_epoch ? 0 : (int)(h->eager_launches & 1u);
    p.roll.csum = h->eager_csum + par * h->eager_csum_half;
    p.roll.csum_next = h->eager_csum + (1 - par) * h->eager_csum_half;
    p.roll.csum_stride = kCsumStride;
    p.roll.gran_end = h->eager_gran_end;
    p.roll.dev_epoch = dev_epoch ? h->eager_epoch : nullptr;
    void *args[] = {&p};
    const hipError_t e = hipLaunchKernel(fn, dim3(nb), dim3(gsm::roll_block_threads(p)), args, (unsigned)lds, s);
    if (e != hipSuccess) return hip_fail(h, e, "hipLaunchKernel (one-step rollout)");
    ++h->eager_launches;   // (only a launched step takes a half: a failed one leaves the order as it was)
    return GSM_OK;
}

int launch(gsm_handle *h, int mode, const void *actions, int fmt, const uint8_t *mask, int reseed,
           hipStream_t s, const gsm_outputs *out = nullptr) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!h->bound) return fail(h, GSM_ESTATE, "gsm_bind has not been called");
    if (mode == GSM_MODE_STEP) {
        if (!actions) return fail(h, GSM_EINVAL, "actions is NULL");
        if (fmt < GSM_ACT_ONEHOT || fmt > GSM_ACT_CONT) return fail(h, GSM_EINVAL, "bad action_fmt");
    }
    gsm::DevParams p = h->dp;
    const int rc = redirect(h, &p, out);
    if (rc) return rc;
    p.mode = mode;
    p.actions = actions;
    p.action_fmt = fmt;
    p.env_mask = mask;
    p.reseed = reseed;
    if (mode == GSM_MODE_STEP) {
        const int r = launch_step_roll(h, p, s);
        if (r != kEagerIneligible) return r;
    }
    const hipError_t e = gsm::launch_step(p, s);
    if (e != hipSuccess) return hip_fail(h, e, "kernel launch");
    return GSM_OK;
}

void drop_slot(gsm_handle::Slot &s) {
    if (s.exec) (void)hipGraphExecDestroy(s.exec);
    if (s.graph) (void)hipGraphDestroy(s.graph);
    for (hipEvent_t ev : s.events) (void)hipEventDestroy(ev);
    if (s.gran_base) (void)hipFree(s.gran_base);
    s.gran_base = nullptr;
    s.gran = nullptr;
    s.csum = nullptr;
    s.csum_half = 0;
    s.pace = nullptr;
    s.launches = 0;
    s.roll = false;
    s.direct = false;
    s.fn = nullptr;
    s.exec = nullptr;
    s.graph = nullptr;
    s.events.clear();
    s.steps = 0;
    s.kern = 0;
    s.each = false;
}

void drop_graph(gsm_handle *h) {
    for (auto &s : h->slots) drop_slot(s);
}

bool bad_slot(int32_t slot) { return slot < 0 || slot >= GSM_GRAPH_SLOTS; }

// The epoch of every rollout launch in the process (DevParams::Roll::epoch):
// one counter, started at a random point so that a granule left in device
// memory by an earlier process does not carry the first epochs of this one.
// A granule of launch L can match only launch L + 2^20 (gsm_device.h
// roll_epoch_tag), whatever graph or allocation either belongs to.
uint32_t next_launch_epoch() {
    static std::atomic<uint32_t> next{[] {
        uint64_t x = (uint64_t)time(nullptr) * 0x9E3779B97F4A7C15ull ^ (uint64_t)getpid() * 0xBF58476D1CE4E5B9ull;
        x ^= x >> 31;
        return (uint32_t)x;
    }()};
    return next.fetch_add(1u) & 0xfffffu;
}

// the status word is read by agent-scope loads in the kernels: cleared by the
// same kind of stores (gsm_kernels.hip launch_granule_init), synchronously
hipError_t clear_status(gsm_handle *h) {
    hipError_t e = gsm::launch_granule_init(h->roll_status, 16, 0u, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    return e;
}

}  // namespace

// A per-step output field of the slots: every slot redirected at a constant
// stride (base, stride), or none (the bound buffer, stride 0).
template <typename T>
static bool slot_field(const gsm_outputs *o, int n, T *gsm_outputs::*f, T **base, int64_t *stride) {
    T *const b0 = o[0].*f;
    if (!b0) {
        for (int j = 1; j < n; ++j)
            if (o[j].*f) return false;
        return true;
    }
    const int64_t st = n > 1 ? (int64_t)(o[1].*f - b0) : 0;
    for (int j = 0; j < n; ++j)
        if (o[j].*f != b0 + j * st) return false;
    *base = b0;
    *stride = st;
    return true;
}

extern "C" {

int gsm_abi_version(void) { return GSM_ABI_VERSION; }

int gsm_query_sizes(const gsm_config *cfg, gsm_sizes *out) {
    std::string why;
    const int rc = check_config(cfg, &why);
    if (rc) return fail(nullptr, rc, why);
    if (!out) return fail(nullptr, GSM_EINVAL, "sizes is NULL");
    fill_sizes(cfg, out);
    if (out->edge_capacity >= (int64_t)1 << 31 ||
        (int64_t)cfg->n_envs * out->n_entities >= (int64_t)1 << 31)
        return fail(nullptr, GSM_EINVAL, "n_envs too large for int32 edge ids/offsets; shard the envs");
    return GSM_OK;
}

int gsm_create(const gsm_config *cfg, gsm_handle **out) {
    if (!out) return fail(nullptr, GSM_EINVAL, "out is NULL");
    *out = nullptr;
    gsm_sizes sz;
    const int rc = gsm_query_sizes(cfg, &sz);
    if (rc) return rc;
    gsm_handle *h = new (std::nothrow) gsm_handle();
    if (!h) return fail(nullptr, GSM_EINVAL, "out of host memory");
    h->cfg = *cfg;
    h->sz = sz;
    derive(cfg, &h->dp);
    h->dp.edge_capacity = sz.edge_capacity;
    *out = h;
    return GSM_OK;
}

int gsm_bind(gsm_handle *h, const gsm_buffers *b) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!b) return fail(h, GSM_EINVAL, "buffers is NULL");
    const void *req[] = {b->pos, b->vel, b->step_count, b->episode, b->ep_acc, b->ep_last,
                         b->node_feat, b->reward, b->cost, b->done, b->edge_count,
                         b->block_edge_sum, b->edge_ptr, b->edge_index, b->edge_attr,
                         b->row_mask, b->contact_mask};
    for (const void *q : req)
        if (!q) return fail(h, GSM_EINVAL, "a required buffer pointer is NULL");
    const bool ragged = h->dp.path == gsm::kPathRagged;
    if (ragged && (!b->env_shape || !b->assign))
        return fail(h, GSM_EINVAL, "polygon/line/mixed need the env_shape and assign buffers");
    if (ragged) {
        const hipError_t e = gsm::upload_ragged_tables();
        if (e != hipSuccess) return hip_fail(h, e, "ragged constant tables");
        const int rc = update_block_order(h, nullptr);
        if (rc) return rc;
        const hipError_t es = hipStreamSynchronize(nullptr);   // bind is not stream-ordered
        if (es != hipSuccess) return hip_fail(h, es, "hipStreamSynchronize (block order)");
    }
    if (((uintptr_t)b->pos | (uintptr_t)b->vel | (uintptr_t)b->ep_acc | (uintptr_t)b->ep_last) & 7)
        return fail(h, GSM_EINVAL, "pos/vel/ep_acc/ep_last must be 8-byte aligned");
    gsm::DevParams &p = h->dp;
    p.pos = (float2 *)b->pos;
    p.vel = (float2 *)b->vel;
    p.step_count = b->step_count;
    p.episode = b->episode;
    p.ep_acc = (float2 *)b->ep_acc;
    p.ep_last = (float2 *)b->ep_last;
    p.node_feat = b->node_feat;
    p.reward = b->reward;
    p.cost = b->cost;
    p.done = b->done;
    p.edge_count = b->edge_count;
    p.block_edge_sum = b->block_edge_sum;
    p.edge_ptr = b->edge_ptr;
    p.edge_index = b->edge_index;
    p.edge_attr = b->edge_attr;
    p.row_mask = b->row_mask;
    p.contact_mask = b->contact_mask;
    p.env_shape = b->env_shape;
    p.assign = b->assign;
    p.degenerate = b->degenerate;
    p.lsa_v = (b->lsa_v && b->lsa_col) ? b->lsa_v : nullptr;
    p.lsa_col = p.lsa_v ? b->lsa_col : nullptr;
    p.lsa_stats = b->lsa_stats;
    h->bound = true;
    drop_graph(h);   // a captured graph holds the old pointers
    // (a failure here, e.g. no device yet, leaves the decision to the first
    // step, which reports it)
    if (h->eager_roll < 0 && eager_setup(h) != GSM_OK) h->eager_roll = -1;
    return GSM_OK;
}

int gsm_reset(gsm_handle *h, uint64_t seed, int reseed, const uint8_t *env_mask, void *stream) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (reseed && seed != h->cfg.seed) {
        h->cfg.seed = seed;
        h->dp.seed_lo = (uint32_t)(seed & 0xFFFFFFFFull);
        h->dp.seed_hi = (uint32_t)(seed >> 32);
        drop_graph(h);   // captured auto-resets would use the old key
        if (h->bound) {
            const int rc = update_block_order(h, as_stream(stream));   // mixed: the env shapes follow the seed
            if (rc) return rc;
        }
    }
    return launch(h, GSM_MODE_RESET, nullptr, 0, env_mask, reseed ? 1 : 0, as_stream(stream));
}

int gsm_step(gsm_handle *h, const void *actions, int action_fmt, void *stream) {
    return launch(h, GSM_MODE_STEP, actions, action_fmt, nullptr, 0, as_stream(stream));
}

int gsm_observe(gsm_handle *h, void *stream) {
    return launch(h, GSM_MODE_OBSERVE, nullptr, 0, nullptr, 0, as_stream(stream));
}

// state copies (gsm_state): direction 0 = bound -> caller, 1 = caller -> bound
static int copy_state(gsm_handle *h, const gsm_state *st, int dir, hipStream_t s) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!h->bound) return fail(h, GSM_ESTATE, "gsm_bind has not been called");
    if (!st) return fail(h, GSM_EINVAL, "state is NULL");
    const gsm::DevParams &p = h->dp;
    const size_t B = (size_t)p.B;
    struct F { void *caller, *bound; size_t bytes; } f[] = {
        {st->pos, p.pos, B * p.E * 8}, {st->vel, p.vel, B * p.N * 8},
        {st->step_count, p.step_count, B * 4}, {st->episode, p.episode, B * 4},
        {st->ep_acc, p.ep_acc, B * 8}, {st->ep_last, p.ep_last, B * 8},
        {st->env_shape, p.env_shape, B * 4},
    };
    for (const F &x : f) {
        if (!x.caller || !x.bound) continue;   // skipped (env_shape: navigation binds none)
        const hipError_t e = dir ? hipMemcpyAsync(x.bound, x.caller, x.bytes, hipMemcpyDeviceToDevice, s)
                                 : hipMemcpyAsync(x.caller, x.bound, x.bytes, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return hip_fail(h, e, "hipMemcpyAsync (state)");
    }
    return GSM_OK;
}

int gsm_get_state(gsm_handle *h, const gsm_state *out, void *stream) {
    return copy_state(h, out, 0, as_stream(stream));
}

int gsm_set_state(gsm_handle *h, const gsm_state *in, void *stream) {
    const int rc = copy_state(h, in, 1, as_stream(stream));
    if (rc) return rc;
    return launch(h, GSM_MODE_OBSERVE, nullptr, 0, nullptr, 0, as_stream(stream));
}

int gsm_step_into(gsm_handle *h, const void *actions, int action_fmt, const gsm_outputs *out, void *stream) {
    if (!out) return fail(h, GSM_EINVAL, "outputs is NULL");
    return launch(h, GSM_MODE_STEP, actions, action_fmt, nullptr, 0, as_stream(stream), out);
}

int gsm_observe_into(gsm_handle *h, const gsm_outputs *out, void *stream) {
    if (!out) return fail(h, GSM_EINVAL, "outputs is NULL");
    return launch(h, GSM_MODE_OBSERVE, nullptr, 0, nullptr, 0, as_stream(stream), out);
}

static int capture_impl(gsm_handle *h, int32_t slot, const void *actions, int64_t stride, int32_t n_actions,
                        int32_t n_steps, int action_fmt, int flags, const gsm_outputs *per_step);
static int capture_roll(gsm_handle *h, int32_t slot, const void *actions, int64_t stride, int32_t n_actions,
                        int32_t n_steps, int action_fmt, int flags, const gsm_outputs *per_step = nullptr,
                        bool fallback = false);
constexpr int kRollIneligible = 1;   // capture_roll(fallback = true): use the per-step chain instead

int gsm_graph_capture(gsm_handle *h, int32_t slot, const void *actions, int64_t stride,
                      int32_t n_actions, int32_t n_steps, int action_fmt, int flags) {
    return capture_impl(h, slot, actions, stride, n_actions, n_steps, action_fmt, flags, nullptr);
}

int gsm_graph_capture_into(gsm_handle *h, int32_t slot, const void *actions, int64_t stride,
                           int32_t n_actions, int32_t n_steps, int action_fmt, const gsm_outputs *per_step) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!h->bound) return fail(h, GSM_ESTATE, "gsm_bind has not been called");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    if (!per_step) return fail(h, GSM_EINVAL, "per_step outputs is NULL");
    // one rollout launch when the config has a rollout kernel and the slots
    // sit at constant strides (a rollout buffer), else the per-step chain
    const int rc = capture_roll(h, slot, actions, stride, n_actions, n_steps, action_fmt, 0, per_step, true);
    if (rc != kRollIneligible) return rc;
    return capture_impl(h, slot, actions, stride, n_actions, n_steps, action_fmt, 0, per_step);
}



// Fused rollout graph (GSM_GRAPH_ROLL): ONE gsm_roll_seg_kernel /
// gsm_roll_tile_kernel / gsm_roll_ragged_kernel launch for all n_steps steps
// and all their edges (a tail after the loop emits the last ones; that launch
// also advances the granule epoch). Every output equals the per-step chain's.
// The ragged rollout packs each step's edges `depth` steps late
// (GSM_ROLL_DEPTH, default 4, 2..kRaggedRollMaxDepth).
static int capture_roll(gsm_handle *h, int32_t slot, const void *actions, int64_t stride, int32_t n_actions,
                        int32_t n_steps, int action_fmt, int flags, const gsm_outputs *per_step, bool fallback) {
    // every caller checks these first; repeated so that no path reaches the
    // slot or the bound buffers without them
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!h->bound) return fail(h, GSM_ESTATE, "gsm_bind has not been called");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    if (flags & ~(GSM_GRAPH_ROLL | GSM_GRAPH_TIME_ENDS))
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL combines with GSM_GRAPH_TIME_ENDS only");
    if (!actions || n_actions < 1 || stride < 0) return fail(h, GSM_EINVAL, "bad capture arguments");
    // the rollout kernels address the action rows with 32-bit byte offsets
    if ((uint64_t)n_actions * (uint64_t)stride >= ((uint64_t)1 << 32)) {
        if (fallback) return kRollIneligible;
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: the action rows must span < 4 GiB");
    }
    if (n_steps < 1) return fail(h, GSM_EINVAL, "n_steps must be >= 1");
    if (action_fmt < GSM_ACT_ONEHOT || action_fmt > GSM_ACT_CONT) return fail(h, GSM_EINVAL, "bad action_fmt");
    gsm::DevParams p = h->dp;
    p.mode = GSM_MODE_STEP;
    p.action_fmt = action_fmt;
    p.env_mask = nullptr;
    p.reseed = 0;
    const bool tile = p.path == gsm::kPathTile, ragged = p.path == gsm::kPathRagged;
    const bool slots = per_step != nullptr;
    const void *roll_fn = tile ? gsm::roll_tile_kernel_fn(p, slots)
                               : ragged ? gsm::roll_ragged_kernel_fn(p, slots) : gsm::roll_seg_kernel_fn(p, slots);
    if (!roll_fn && fallback) return kRollIneligible;
    if (!roll_fn) return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: no fused rollout kernel for this config "
                                             "(segmented path with a compiled shape, tile path with the "
                                             "symmetric sweep, or a ragged batch)");
    // step k's outputs at base + k * stride (a rollout buffer's slots) or all
    // in the bound buffers
    gsm::DevParams::RollOut ro{p.node_feat, p.reward, p.cost, p.done, p.edge_count, p.edge_ptr, p.edge_index,
                               p.edge_attr, 0, 0, 0, 0, 0, 0, 0, p.edge_capacity, nullptr, nullptr, p.assign, 0};
    if (per_step) {
        int64_t cost_s = 0;
        bool ok = slot_field(per_step, n_steps, &gsm_outputs::node_feat, &ro.nf, &ro.nf_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::reward, &ro.rew, &ro.rc_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::cost, &ro.cost, &cost_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::done, &ro.done, &ro.done_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::edge_count, &ro.ecount, &ro.ec_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::edge_ptr, &ro.eptr, &ro.ep_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::edge_index, &ro.eidx, &ro.ei_s) &&
                  slot_field(per_step, n_steps, &gsm_outputs::edge_attr, &ro.eattr, &ro.ea_s) &&
                  cost_s == ro.rc_s && (ragged ? slot_field(per_step, n_steps, &gsm_outputs::assign, &ro.asg, &ro.as_s)
                                               : !per_step[0].assign);
        for (int j = 0; ok && j < n_steps; ++j) {
            const int rc = redirect(h, &p, &per_step[j]);   // validates the slot
            if (rc) return rc;
            ok = !per_step[0].edge_index || per_step[j].edge_capacity == per_step[0].edge_capacity;
        }
        if (!ok) {
            if (fallback) return kRollIneligible;
            return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: per-step outputs must sit at constant strides");
        }
        if (per_step[0].edge_index) ro.cap = per_step[0].edge_capacity;
        // p now describes the last slot: the final emit launch writes it
    }
    // segmented / ragged rollout: one env per wave whatever the config's G (4 per workgroup), or four
    // small envs per wave (16 per workgroup)
    const int per_blk = tile ? 1 : ragged ? gsm::kWavesPerBlock : gsm::roll_seg_envs_per_block(p);
    const int nb = tile ? gsm::step_grid_blocks(p) : (p.B + per_blk - 1) / per_blk;
    const size_t roll_lds = tile ? gsm::roll_tile_kernel_lds(p)
                                 : ragged ? gsm::roll_ragged_kernel_lds(p) : gsm::roll_kernel_lds(p);
    // every workgroup resident at once (one residency round; a workgroup only
    // waits on lower-numbered ones, so this is for speed, not for progress)
    int dev = 0, per_cu = 0, n_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, roll_fn, gsm::roll_block_threads(p), roll_lds);
    if (e != hipSuccess) return hip_fail(h, e, "occupancy query");
    if ((int64_t)per_cu * n_cu < nb) {
        if (fallback) return kRollIneligible;
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: the batch exceeds one residency round of the rollout kernel");
    }
    const int K = n_steps;
    // granule tags carry the step in 12 bits; checked before the slot's
    // graph is dropped
    if (K > gsm::kRollMaxSteps) {
        if (fallback) return kRollIneligible;
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: n_steps must be <= 4094");
    }
    // ragged and packed small envs: per-wave granules, groups of 64 waves (at
    // most 128 groups: one residency round holds <= 8192 waves); ragged: edges
    // packed `depth` steps late
    const int xW = nb * gsm::kWavesPerBlock, xNG = (xW + gsm::kWave - 1) / gsm::kWave;
    // per-wave granules (Xfer): ragged and packed small envs; the other
    // segmented shapes and the tile path look back per workgroup
    const bool per_wave = ragged || (!tile && gsm::roll_packed(p));
    if (per_wave && xNG > 2 * gsm::kWave) {
        if (fallback) return kRollIneligible;
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: more than 8192 envs in one rollout launch");
    }
    int depth = 0;
    if (ragged) {
        depth = 4;
        if (const char *ev = getenv("GSM_ROLL_DEPTH")) depth = atoi(ev);
        depth = std::min(std::max(depth, 2), gsm::kRaggedRollMaxDepth);
        // the env slabs of depth + 1 steps (each env's edges at a fixed stride:
        // max_edges_per_env + 1 words, then as many distances)
        const size_t need = (size_t)(depth + 1) * p.B * 8 * ((size_t)h->sz.max_edges_per_env + 1);
        if (h->slab_bytes < need) {
            // a deeper ring than before: the slabs are re-allocated, and every
            // earlier ragged rollout slot is re-pointed at them (a slab holds
            // only the edges in flight within one launch, so nothing in the
            // old one outlives its launches: drained first)
            void *fresh = nullptr;
            e = hipMalloc(&fresh, need);
            if (e != hipSuccess) {
                if (fallback) return kRollIneligible;
                return hip_fail(h, e, "hipMalloc (rollout edge slabs)");
            }
            if (h->slab) {
                e = hipDeviceSynchronize();
                if (e != hipSuccess) { (void)hipFree(fresh); return hip_fail(h, e, "hipDeviceSynchronize (slabs)"); }
                (void)hipFree(h->slab);
            }
            for (auto &o : h->slots)
                if (o.roll && o.args.path == gsm::kPathRagged) {
                    o.args.roll.slab = (int32_t *)fresh;
                    o.args.roll.slab_end = (int32_t *)((char *)fresh + need);
                }
            h->slab = fresh;
            h->slab_bytes = need;
        }
    }
    if (!h->roll_status) {
        e = hipMalloc(&h->roll_status, 16);
        if (e == hipSuccess) e = clear_status(h);
        if (e != hipSuccess) { h->roll_status = nullptr; return hip_fail(h, e, "hipMalloc (rollout status)"); }
    }
    if (!h->cap_stream) {
        e = hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_fail(h, e, "hipStreamCreate");
    }
    // in the bound buffers, the edges of every step but the last go to a
    // scratch of the bound capacity (DevParams::RollOut); allocated once
    if (!per_step && !h->edge_scratch) {
        e = hipMalloc(&h->edge_scratch, 12 * (size_t)h->sz.edge_capacity);
        if (e != hipSuccess) {
            h->edge_scratch = nullptr;
            if (fallback) return kRollIneligible;
            return hip_fail(h, e, "hipMalloc (rollout edge scratch)");
        }
    }
    gsm_handle::Slot &sl = h->slots[slot];
    drop_slot(sl);
    // a 16-byte header (unused), then 8-byte granules. Ragged and packed
    // small envs: per-wave counts [K][xW] and group sums [K][xNG]; the tile
    // path and the other segmented shapes (one env per workgroup or per
    // wave): aggregates [K][nb], two halves of chunk sums [K][nc] kCsumStride
    // apart (gsm_device.h roll_prefix) and two halves of pace counters
    // (gsm_device.h pace_level). Zeroed once here — granules are tagged with the launch
    // epoch, so replays never clear them; the untagged chunk sums and counters
    // are zeroed by the launch before the one that uses them
    // (ragged: then the placement words, gsm::PlaceArea)
    const bool one_hop = !per_wave;   // one-hop prefix and pacing: the one-env-per-wave and tile rollouts
    const size_t nc = ((size_t)nb + gsm::kPrefixChunk - 1) / gsm::kPrefixChunk;
    if (one_hop && nc > (size_t)gsm::kWave) {   // roll_prefix: one chunk sum per lane
        if (fallback) return kRollIneligible;
        return fail(h, GSM_EINVAL, "GSM_GRAPH_ROLL: more than 4096 workgroups in one rollout launch");
    }
    const size_t csum_half = one_hop ? (size_t)K * nc * kCsumStride : 0;   // u64
    const size_t pace_words = one_hop ? (size_t)gsm::kPaceKeys * gsm::kPaceStride : 0;   // u32, per half
    const size_t gran_alloc = 16 + ((size_t)K * (per_wave ? (size_t)(xW + xNG) : (size_t)nb) +
                                    2 * csum_half) * sizeof(uint64_t) +
                              2 * pace_words * sizeof(uint32_t) +
                              (ragged ? gsm::PlaceArea::words(xW) * sizeof(uint64_t) : 0);
    e = gran_malloc(&sl.gran_base, &sl.gran, gran_alloc);
    if (e != hipSuccess) {
        sl.gran = nullptr;
        if (fallback) return kRollIneligible;   // the per-step chain needs no granules
        return hip_fail(h, e, "hipMalloc (rollout granules)");
    }
    // Zeroed once (tag 0 never matches). Every launch then takes its own
    // epoch (next_launch_epoch, set in gsm_graph_launch): a memset or
    // store-zeroed allocation was seen to still show an agent-scope load
    // granules left at that address by a freed graph's last replay, and with
    // per-capture epochs those could carry this graph's tags.
    e = gsm::launch_granule_init(sl.gran, gran_alloc, 0u, h->cap_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->cap_stream);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "rollout granule init"); }
    // pacing: the rank offset in quarter steps (GSM_ROLL_PACE, default 2;
    // 0 = no pacing: an A/B knob, outputs are the same either way)
    int pace_q = 0;
    bool pace_on = true;
    if (const char *ev = getenv("GSM_ROLL_PACE")) {
        if (!strcmp(ev, "off"))
            pace_on = false;
        else
            pace_q = std::max(0, atoi(ev));
    }
    if (one_hop) {
        uint64_t *const after = sl.gran + 2 + (size_t)K * nb;
        sl.csum = after;
        sl.csum_half = (int64_t)csum_half;
        sl.pace = pace_on ? (uint32_t *)(after + 2 * csum_half) : nullptr;
    }
    const bool ends = (flags & GSM_GRAPH_TIME_ENDS) != 0;
    sl.events.resize(ends ? 2 : 0, nullptr);
    for (auto &ev : sl.events) {
        e = hipEventCreate(&ev);
        if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipEventCreate"); }
    }
    e = hipGraphCreate(&sl.graph, 0);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphCreate"); }
    hipGraphNode_t prev = nullptr;
    const char *what = "event node";
    auto add_event = [&](hipEvent_t ev) -> hipError_t {
        hipGraphNode_t n;
        const hipError_t r = hipGraphAddEventRecordNode(&n, sl.graph, prev ? &prev : nullptr, prev ? 1 : 0, ev);
        if (r == hipSuccess) prev = n;
        return r;
    };
    if (e == hipSuccess && ends) { what = "event node"; e = add_event(sl.events[0]); }
    // all steps and their edges in one launch; the last step's sums go to the
    // bound edge-sum buffer (later eager emits read it)
    if (!per_step) {
        ro.eidx_mid = (int32_t *)h->edge_scratch;
        ro.eattr_mid = (float *)(ro.eidx_mid + 2 * h->sz.edge_capacity);
    }
    p.actions = actions;
    p.ro = ro;
    // ragged mixed: envs dealt to the SIMDs by cost when the grid fills every
    // SIMD with the same number of waves (GSM_ROLL_PLACE=0: env = wave index)
    const int place_S = 4 * n_cu;
    int place_R = 0;
    if (ragged && h->place_order && xW % place_S == 0) place_R = xW / place_S;
    // (GSM_ROLL_PLACE=2, a test knob: every wave registers, then the launch
    // decides identity, the partial-residency fallback)
    int place_force = 0;
    if (const char *ev = getenv("GSM_ROLL_PLACE")) {
        if (atoi(ev) == 0) place_R = 0;
        if (atoi(ev) == 2) place_force = 1;
    }
    p.roll = gsm::DevParams::Roll{(const char *)actions, stride, n_actions, 0, K, xW, xNG, depth,
                                  h->sz.max_edges_per_env, place_R, sl.gran + 2, h->roll_status, 0u, place_force,
                                  (int32_t *)h->slab, place_R ? h->place_order : nullptr, place_S, pace_q};
    p.roll.csum_stride = kCsumStride;   // (csum, pace: set per launch, gsm_graph_launch)
    p.roll.gran_end = (uint64_t *)((char *)sl.gran + gran_alloc);
    p.roll.slab_end = h->slab ? (int32_t *)((char *)h->slab + h->slab_bytes) : nullptr;
    if (e == hipSuccess) {
        what = "rollout kernel node";
        hipKernelNodeParams kp = {};
        void *args[] = {&p};
        kp.func = const_cast<void *>(roll_fn);
        kp.gridDim = dim3(nb);
        kp.blockDim = dim3(gsm::roll_block_threads(p));
        kp.sharedMemBytes = (unsigned)roll_lds;
        kp.kernelParams = args;
        kp.extra = nullptr;
        hipGraphNode_t n;
        e = hipGraphAddKernelNode(&n, sl.graph, prev ? &prev : nullptr, prev ? 1 : 0, &kp);
        if (e == hipSuccess) prev = n;
        sl.direct = true;
        sl.fn = roll_fn;
        sl.grid = kp.gridDim;
        sl.block = kp.blockDim;
        sl.lds = kp.sharedMemBytes;
        sl.args = p;
    }
    if (e == hipSuccess && ends) { what = "event node"; e = add_event(sl.events[1]); }
    if (e != hipSuccess) {
        drop_slot(sl);
        char where[96];
        snprintf(where, sizeof where, "rollout graph build (%s)", what);
        return hip_fail(h, e, where);
    }
    e = hipGraphInstantiate(&sl.exec, sl.graph, nullptr, nullptr, 0);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphInstantiate"); }
    e = hipGraphUpload(sl.exec, h->cap_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->cap_stream);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphUpload"); }
    // timing (TIME_ENDS): the events bracket the rollout launch alone, so
    // gsm_graph_kernel_ms reports its time per step
    sl.each = false;
    sl.kern = GSM_GRAPH_STEP;
    sl.steps = n_steps;
    sl.roll = true;
    return GSM_OK;
}

int gsm_graph_info(gsm_handle *h, int32_t slot, int32_t *steps, int32_t *fused) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    const gsm_handle::Slot &sl = h->slots[slot];
    if (steps) *steps = sl.exec ? sl.steps : 0;
    if (fused) *fused = sl.exec && sl.roll ? 1 : 0;
    return GSM_OK;
}

int gsm_graph_roll_status(gsm_handle *h, int32_t *gave_up) {
    if (!h || !gave_up) return fail(h, GSM_EINVAL, "NULL argument");
    *gave_up = 0;
    if (!h->roll_status) return GSM_OK;
    uint32_t v = 0;
    hipError_t e = hipMemcpy(&v, h->roll_status, sizeof v, hipMemcpyDeviceToHost);
    if (e == hipSuccess && v) {   // word 0 only (words 1-2: the placement counts)
        e = gsm::launch_granule_init(h->roll_status, sizeof(uint32_t), 0u, nullptr);
        if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    }
    if (e != hipSuccess) return hip_fail(h, e, "rollout status read");
    *gave_up = (int32_t)v;   // the reason code (gsm.h), 0 if none
    return GSM_OK;
}

int gsm_graph_roll_placement(gsm_handle *h, int64_t *dealt, int64_t *fallback) {
    if (!h || !dealt || !fallback) return fail(h, GSM_EINVAL, "NULL argument");
    *dealt = *fallback = 0;
    if (!h->roll_status) return GSM_OK;
    uint32_t v[2] = {0, 0};
    hipError_t e = hipMemcpy(v, h->roll_status + 1, sizeof v, hipMemcpyDeviceToHost);
    if (e == hipSuccess && (v[0] || v[1])) {
        e = gsm::launch_granule_init(h->roll_status + 1, sizeof v, 0u, nullptr);
        if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    }
    if (e != hipSuccess) return hip_fail(h, e, "rollout placement read");
    *fallback = v[0];
    *dealt = v[1];
    return GSM_OK;
}

static int capture_impl(gsm_handle *h, int32_t slot, const void *actions, int64_t stride, int32_t n_actions,
                        int32_t n_steps, int action_fmt, int flags, const gsm_outputs *per_step) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (!h->bound) return fail(h, GSM_ESTATE, "gsm_bind has not been called");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    if (flags & GSM_GRAPH_ROLL) return capture_roll(h, slot, actions, stride, n_actions, n_steps, action_fmt, flags);
    int kern = flags & (GSM_GRAPH_STEP | GSM_GRAPH_EMIT);
    if (!kern) kern = GSM_GRAPH_STEP | GSM_GRAPH_EMIT;
    const bool each = (flags & GSM_GRAPH_TIME_EACH) != 0, ends = (flags & GSM_GRAPH_TIME_ENDS) != 0;
    const bool lag_only = (flags & GSM_GRAPH_LAG_ONLY) != 0;
    const bool can_lag = gsm::lag_step_kernel_fn(h->dp) != nullptr;
    if (lag_only && (!can_lag || each || (flags & (GSM_GRAPH_STEP | GSM_GRAPH_EMIT | GSM_GRAPH_UNFUSED))))
        return fail(h, GSM_EINVAL, "GSM_GRAPH_LAG_ONLY: segmented / ragged configs only, no other kernel/timing-each flags");
    if (lag_only) kern = GSM_GRAPH_STEP;
    // lagged emission: step_0, lag_step_1 .. lag_step_{T-1}, emit_{T-1}
    const bool lag = lag_only || (can_lag && !each && kern == (GSM_GRAPH_STEP | GSM_GRAPH_EMIT) &&
                                  !(flags & GSM_GRAPH_UNFUSED));
    if ((kern & GSM_GRAPH_STEP) && (!actions || n_actions < 1 || stride < 0))
        return fail(h, GSM_EINVAL, "bad capture arguments");
    if (n_steps < 1) return fail(h, GSM_EINVAL, "n_steps must be >= 1");
    if (action_fmt < GSM_ACT_ONEHOT || action_fmt > GSM_ACT_CONT) return fail(h, GSM_EINVAL, "bad action_fmt");
    gsm_handle::Slot &sl = h->slots[slot];
    drop_slot(sl);
    hipError_t e;
    if (lag && !h->bsum_alt) {
        e = hipMalloc(&h->bsum_alt, (size_t)h->sz.n_blocks * sizeof(int32_t) + 16);
        if (e != hipSuccess) { h->bsum_alt = nullptr; return hip_fail(h, e, "hipMalloc (edge-sum buffer)"); }
    }
    if (!h->cap_stream) {
        e = hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_fail(h, e, "hipStreamCreate");
    }
    // The graph is built node by node (a linear chain) rather than by stream
    // capture: event-record nodes for timing are then explicit (the capture
    // path of the HIP runtime bundled with PyTorch rejects
    // hipEventRecordWithFlags(..., hipEventRecordExternal)).
    //   TIME_EACH:  [E0] step_0 [E1] emit_0 [E2] step_1 ...   (events: 2 per step + 1)
    //   TIME_ENDS:  [E0] step_0 emit_0 step_1 ... [E1]
    const size_t n_ev = each ? 2 * (size_t)n_steps + 1 : (ends ? 2 : 0);
    sl.events.resize(n_ev, nullptr);
    for (auto &ev : sl.events) {
        e = hipEventCreate(&ev);
        if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipEventCreate"); }
    }
    sl.each = each;
    sl.kern = kern;
    e = hipGraphCreate(&sl.graph, 0);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphCreate"); }
    if (lag && !h->roll_status) {   // the ragged lagged step's bounded wait reports through it
        e = hipMalloc(&h->roll_status, 16);
        if (e == hipSuccess) e = clear_status(h);
        if (e != hipSuccess) { h->roll_status = nullptr; drop_slot(sl); return hip_fail(h, e, "hipMalloc (status)"); }
    }
    gsm::DevParams p = h->dp;
    p.mode = GSM_MODE_STEP;
    p.action_fmt = action_fmt;
    p.env_mask = nullptr;
    p.reseed = 0;
    if (lag) p.roll.status = h->roll_status;
    hipGraphNode_t prev = nullptr;
    const char *what = "";
    int at = 0;
    auto add_event = [&](hipEvent_t ev) -> hipError_t {
        hipGraphNode_t n;
        const hipError_t r = hipGraphAddEventRecordNode(&n, sl.graph, prev ? &prev : nullptr, prev ? 1 : 0, ev);
        if (r == hipSuccess) prev = n;
        return r;
    };
    auto add_kernel = [&](const void *fn, size_t lds) -> hipError_t {
        hipKernelNodeParams kp = {};
        void *args[] = {&p};
        kp.func = const_cast<void *>(fn);
        kp.gridDim = dim3(fn == gsm::emit_kernel_fn(p) ? gsm::grid_blocks(p) : gsm::step_grid_blocks(p));
        kp.blockDim = dim3(gsm::block_threads(p));
        kp.sharedMemBytes = (unsigned)lds;
        kp.kernelParams = args;
        kp.extra = nullptr;
        hipGraphNode_t n;
        const hipError_t r = hipGraphAddKernelNode(&n, sl.graph, prev ? &prev : nullptr, prev ? 1 : 0, &kp);
        if (r == hipSuccess) prev = n;
        return r;
    };
    what = "event node";
    e = n_ev ? add_event(sl.events[0]) : hipSuccess;
    const gsm::DevParams p_bound = p;
    // edge-sum halves: the bound buffer holds the sums of the current state
    // before and after every graph (eager emits read it); a lagged chain
    // alternates so that its last step writes the bound half.
    int32_t *half[2] = {p_bound.block_edge_sum, h->bsum_alt};
    gsm::DevParams last = p_bound;   // outputs of the previous step
    for (int t = 0; t < n_steps && e == hipSuccess; ++t) {
        at = t;
        if (per_step) {
            p = p_bound;
            const int rc = redirect(h, &p, &per_step[t]);
            if (rc) {
                drop_slot(sl);
                return rc;
            }
        }
        const bool lag_node = lag && (lag_only || t > 0);
        if (lag) {
            // lag-only: node t reads half t%2; chain: node t writes half (T-1-t)%2
            const int w = lag_only ? (t + 1) % 2 : (n_steps - 1 - t) % 2;
            p.block_edge_sum = half[w];
            p.lag = gsm::DevParams::Lag{half[1 - w], last.edge_count, last.edge_ptr, last.edge_index,
                                        last.edge_attr, last.edge_capacity};
        }
        if (kern & GSM_GRAPH_STEP) {
            p.actions = (const char *)actions + (int64_t)(t % n_actions) * stride;
            what = lag_node ? "lagged step kernel node" : "step kernel node";
            e = add_kernel(lag_node ? gsm::lag_step_kernel_fn(p) : gsm::step_kernel_fn(p), gsm::step_kernel_lds(p));
            if (e == hipSuccess && each) { what = "event node"; e = add_event(sl.events[2 * t + 1]); }
        }
        // the two-kernel chain emits every step; a lagged chain only the last
        if (e == hipSuccess && (kern & GSM_GRAPH_EMIT) && (!lag || t == n_steps - 1)) {
            what = "emit kernel node";
            e = add_kernel(gsm::emit_kernel_fn(p), gsm::emit_kernel_lds(p));
        }
        if (e == hipSuccess && each) { what = "event node"; e = add_event(sl.events[2 * t + 2]); }
        last = p;
    }
    if (e == hipSuccess && ends && !each) { what = "event node"; e = add_event(sl.events[1]); }
    if (e != hipSuccess) {
        drop_slot(sl);
        char where[96];
        snprintf(where, sizeof where, "graph build (step %d, %s)", at, what);
        return hip_fail(h, e, where);
    }
    e = hipGraphInstantiate(&sl.exec, sl.graph, nullptr, nullptr, 0);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphInstantiate"); }
    e = hipGraphUpload(sl.exec, h->cap_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->cap_stream);
    if (e != hipSuccess) { drop_slot(sl); return hip_fail(h, e, "hipGraphUpload"); }
    sl.steps = n_steps;
    return GSM_OK;
}

int gsm_graph_launch(gsm_handle *h, int32_t slot, void *stream) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    gsm_handle::Slot &sl = h->slots[slot];
    if (!sl.exec) return fail(h, GSM_ESTATE, "no graph captured in this slot");
    if (sl.direct) {   // a rollout graph: its one kernel, launched directly
        // (GSM_GRAPH_TIME_ENDS: events recorded on the stream around it — as
        // graph event nodes they added ≈7% to the launch they bracketed)
        hipStream_t st = as_stream(stream);
        // Every launch takes its own epoch and its half of the slot's double
        // buffers, set in the arguments here: a launch captured into the
        // caller's graph would replay one of each every time (stale granules
        // matching its tags, unzeroed chunk sums)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        hipError_t e = hipStreamIsCapturing(st, &cs);
        if (e != hipSuccess) return hip_fail(h, e, "hipStreamIsCapturing");
        if (cs != hipStreamCaptureStatusNone)
            return fail(h, GSM_ESTATE, "a rollout graph cannot be launched into a stream capture (every launch "
                                       "takes its own hand-off epoch); capture the per-step chain instead");
        if (!h->roll_done) {
            e = hipEventCreateWithFlags(&h->roll_done, hipEventDisableTiming);
            if (e != hipSuccess) { h->roll_done = nullptr; return hip_fail(h, e, "hipEventCreate (rollout)"); }
        }
        // rollout launches of one handle never overlap: they share its
        // scratch and state, so a launch on another stream than the previous
        // one waits for it, asynchronously (an event recorded behind every
        // launch: nothing here depends on the previous stream still existing)
        if (h->roll_launched && h->roll_stream != st) {
            e = hipStreamWaitEvent(st, h->roll_done, 0);
            if (e != hipSuccess) return hip_fail(h, e, "hipStreamWaitEvent (previous rollout launch)");
        }
        sl.args.roll.epoch = fresh_epoch(sl.last_epoch);   // copied with the arguments at the launch
        const int par = (int)(sl.launches & 1u);
        if (sl.csum) {
            sl.args.roll.csum = sl.csum + par * sl.csum_half;
            sl.args.roll.csum_next = sl.csum + (1 - par) * sl.csum_half;
        }
        if (sl.pace) {
            const size_t half = (size_t)gsm::kPaceKeys * gsm::kPaceStride;
            sl.args.roll.pace = sl.pace + par * half;
            sl.args.roll.pace_next = sl.pace + (1 - par) * half;
        }
        void *args[] = {&sl.args};
        e = sl.events.empty() ? hipSuccess : hipEventRecord(sl.events.front(), st);
        if (e == hipSuccess) e = hipLaunchKernel(sl.fn, sl.grid, sl.block, args, sl.lds, st);
        if (e != hipSuccess) return hip_fail(h, e, "hipLaunchKernel (rollout)");
        sl.launches++;
        h->roll_stream = st;
        h->roll_launched = true;
        e = sl.events.empty() ? hipSuccess : hipEventRecord(sl.events.back(), st);
        if (e == hipSuccess) e = hipEventRecord(h->roll_done, st);
        if (e != hipSuccess) return hip_fail(h, e, "hipEventRecord (rollout)");
        return GSM_OK;
    }
    const hipError_t e = hipGraphLaunch(sl.exec, as_stream(stream));
    if (e != hipSuccess) return hip_fail(h, e, "hipGraphLaunch");
    return GSM_OK;
}

int gsm_graph_kernel_ms(gsm_handle *h, int32_t slot, float *step_ms, float *emit_ms, float *total_ms) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    if (bad_slot(slot)) return fail(h, GSM_EINVAL, "bad graph slot");
    const gsm_handle::Slot &sl = h->slots[slot];
    if (!sl.exec || sl.events.empty()) return fail(h, GSM_ESTATE, "no timed graph in this slot");
    float total = 0;
    hipError_t e = hipEventElapsedTime(&total, sl.events.front(), sl.events.back());
    if (e != hipSuccess) return hip_fail(h, e, "hipEventElapsedTime");
    double a = 0, b = 0;
    if (sl.each) {
        for (int t = 0; t < sl.steps; ++t) {
            float x = 0, y = 0;
            if (sl.kern & GSM_GRAPH_STEP) e = hipEventElapsedTime(&x, sl.events[2 * t], sl.events[2 * t + 1]);
            if (e == hipSuccess && (sl.kern & GSM_GRAPH_EMIT))
                e = hipEventElapsedTime(&y, sl.events[2 * t + ((sl.kern & GSM_GRAPH_STEP) ? 1 : 0)],
                                        sl.events[2 * t + 2]);
            if (e != hipSuccess) return hip_fail(h, e, "hipEventElapsedTime");
            a += x;
            b += y;
        }
        a /= sl.steps;
        b /= sl.steps;
    } else {
        // back-to-back launches of one kind: the mean per launch
        if (sl.kern == GSM_GRAPH_STEP) a = total / sl.steps;
        else if (sl.kern == GSM_GRAPH_EMIT) b = total / sl.steps;
    }
    if (step_ms) *step_ms = (float)a;
    if (emit_ms) *emit_ms = (float)b;
    if (total_ms) *total_ms = total;
    return GSM_OK;
}

int gsm_attn_aggregate(const float *q, const float *k, const float *v, const float *edge_w, const float *w_e,
                       const int64_t *row_ptr, const int32_t *col, const float *skip, int64_t n_nodes,
                       int32_t heads, int32_t channels, float scale, float *out, void *stream) {
    if (n_nodes < 0 || n_nodes >= ((int64_t)1 << 40)) return fail(nullptr, GSM_EINVAL, "bad n_nodes");
    if (heads < 1 || channels < 1 || (channels & (channels - 1)) || heads * channels > 64)
        return fail(nullptr, GSM_EINVAL, "need channels a power of two and heads*channels <= 64");
    if (n_nodes == 0) return GSM_OK;
    if (!q || !k || !v || !row_ptr || !col || !out) return fail(nullptr, GSM_EINVAL, "a required pointer is NULL");
    if (!!edge_w != !!w_e) return fail(nullptr, GSM_EINVAL, "edge_w and w_e go together");
    const hipError_t e = gsm::launch_attn_aggregate(q, k, v, edge_w, w_e, row_ptr, col, skip, n_nodes,
                                                    heads * channels, channels, scale, out, as_stream(stream));
    if (e != hipSuccess) return hip_fail(nullptr, e, "gsm_attn_aggregate launch");
    return GSM_OK;
}

int gsm_render(const float *node_feat, int64_t n_envs, int32_t n_entities, const int64_t *edge_ptr,
               const int32_t *edge_index, int64_t edge_capacity, const int32_t *env_ids, int32_t n_frames,
               float half_width, float agent_size, float target_size, float obstacle_size, int32_t width,
               int32_t height, int32_t flags, uint8_t *rgba, void *stream) {
    if (n_frames < 0 || n_frames > 65535) return fail(nullptr, GSM_EINVAL, "n_frames must be in [0, 65535]");
    if (width < 1 || height < 1 || width > 8192 || height > 8192)
        return fail(nullptr, GSM_EINVAL, "width and height must be in [1, 8192]");
    if (n_entities < 1 || n_entities > 4096) return fail(nullptr, GSM_EINVAL, "n_entities must be in [1, 4096]");
    if (n_envs < 1) return fail(nullptr, GSM_EINVAL, "n_envs must be >= 1");
    if (!(agent_size >= 0.0f && target_size >= 0.0f && obstacle_size >= 0.0f))
        return fail(nullptr, GSM_EINVAL, "sizes must be >= 0");
    if (n_frames == 0) return GSM_OK;
    const bool edges = (flags & GSM_RENDER_EDGES) != 0;
    if (!node_feat || !env_ids || !rgba || (edges && (!edge_ptr || !edge_index || edge_capacity < 1)))
        return fail(nullptr, GSM_EINVAL, "a required pointer is NULL");
    if ((uintptr_t)rgba & 3) return fail(nullptr, GSM_EINVAL, "rgba must be 4-byte aligned");
    const hipError_t e = gsm::launch_render(node_feat, n_envs, n_entities, edge_ptr, edge_index, edge_capacity,
                                            env_ids, n_frames, half_width, agent_size, target_size,
                                            obstacle_size, width, height, edges ? 1 : 0, rgba,
                                            as_stream(stream));
    if (e != hipSuccess) return hip_fail(nullptr, e, "gsm_render launch");
    return GSM_OK;
}

int gsm_debug_set_stamps(gsm_handle *h, void *stamps) {
    if (!h) return fail(nullptr, GSM_EINVAL, "handle is NULL");
    h->dp.stamps = (uint64_t *)stamps;
    drop_graph(h);
    return GSM_OK;
}

int gsm_destroy(gsm_handle *h) {
    if (!h) return GSM_OK;
    drop_graph(h);
    if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
    if (h->bsum_alt) (void)hipFree(h->bsum_alt);
    if (h->roll_status) (void)hipFree(h->roll_status);
    if (h->edge_scratch) (void)hipFree(h->edge_scratch);
    if (h->slab) (void)hipFree(h->slab);
    if (h->eager_base) (void)hipFree(h->eager_base);
    if (h->order_copied) (void)hipEventSynchronize(h->order_copied);
    if (h->block_order) (void)hipFree(h->block_order);
    if (h->order_host) (void)hipHostFree(h->order_host);
    if (h->order_copied) (void)hipEventDestroy(h->order_copied);
    if (h->roll_done) (void)hipEventDestroy(h->roll_done);
    delete h;
    return GSM_OK;
}

int gsm_last_error(const gsm_handle *h, char *buf, size_t len) {
    const std::string &m = h ? h->err : g_err;
    if (buf && len) {
        const size_t n = m.size() < len - 1 ? m.size() : len - 1;
        memcpy(buf, m.data(), n);
        buf[n] = 0;
    }
    return (int)m.size();
}

}  // extern "C"
