// Internal (non-ABI) declarations shared by gsm_kernels.hip and gsm_abi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsm {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;              // one env per wave
constexpr int kBlock = kWave * kWavesPerBlock;
enum : int32_t { kPathSeg = 1, kPathRagged = 2, kPathTile = 3 };
constexpr int kTileBlock = 512;                // tile path: one workgroup per env
enum : int32_t { kScnNav = 0, kScnPolygon = 1, kScnLine = 2, kScnMixed = 3 };
constexpr int kTileEmitScr = 6144;   // tile emitter: staged edge words per env (24 KB of LDS)
constexpr int kRaggedMaxAgents = 32;                                  // = GSM_RAGGED_MAX_AGENTS
constexpr int kRaggedTable = kRaggedMaxAgents * (kRaggedMaxAgents + 1) / 2;   // rows n = 1..32
// ragged assignment scratch per wave (gsm_ragged_kernels.hip LsaLds): cost
// matrix rows (a multiple of 8) at an odd stride of at least that many
// columns (the row passes read whole chunks of 8: the columns past N hold
// +inf), column and row duals, column -> row
__host__ __device__ constexpr int lsa_stride(int nmax) { return ((nmax + 7) & ~7) | 1; }
__host__ __device__ constexpr int lsa_cost_bytes(int nmax) { return 4 * ((nmax + 7) & ~7) * lsa_stride(nmax); }
__host__ __device__ constexpr int lsa_lds_bytes(int nmax) {
    return ((lsa_cost_bytes(nmax) + 15) & ~15) + 16 * kRaggedMaxAgents + 4 * kRaggedMaxAgents;
}
// cap on envs per wave, keeping a block's envs (4G) within one wave's lanes
// (C2, 3 x 4096: G = 4 runs 6.0 us per step against 6.9 at G = 10)
constexpr int kMaxSegEnvsPerWave = 4;
// steps of one rollout launch (the step field of the 32-bit granule tags,
// gsm_device.h roll_epoch_tag)
// (step field 4095 tags the ragged rollout's placement words, PlaceArea)
constexpr int kRollMaxSteps = 4094;
// pacing counters of the segmented rollout: one per CU, keyed by 11 bits of
// XCC_ID / HW_ID (XCC, shader engine, shader array, CU), one per 64 bytes
constexpr int kPaceKeys = 2048, kPaceStride = 16;   // counters, u32 words between them
// workgroups per chunk sum of the segmented rollout's one-hop CSR prefix
// (gsm_device.h roll_prefix)
constexpr int kPrefixChunk = 64;
// the one-launch eager step's device-side epoch: replicas one per 64 bytes,
// workgroup w reading replica w % kEpochReps (no single word read by the whole
// grid at entry)
constexpr int kEpochReps = 64, kEpochStride = 16;

// Everything a launch needs, passed by value (kernarg segment, < 4 KB).
// fp32 constants are formed on the host exactly as oracle/batch_ref.py:Spec
// forms them in fp32 mode (gsm_abi.hip: derive()).
struct DevParams {
    int32_t B, N, No, E, M, EL, auto_reset, shared_reward;
    int32_t mode, action_fmt, reseed;
    int32_t path;          // kPathSeg (navigation, M <= 64), kPathTile (M > 64) or kPathRagged
    int32_t scenario;      // ragged: kScnPolygon / kScnLine / kScnMixed
    int32_t T;             // ragged: target rows per env (T_max); N, No, E, M are the padded maxima
    int32_t n_min;         // ragged mixed: smallest N_env
    int32_t W;             // uint64 words per mask row (tile path: ceil(M/64))
    int32_t nf_full;       // write every node-feature row (redirected outputs)
    int32_t G;             // envs per wave (segmented path), 1 otherwise
    int32_t tile_sym;      // tile path: symmetric sweep (its LDS fits), gsm_tile_kernels.hip
    int32_t strict;        // App. A S16 strict mode: coincident-pair / NaN forces as in MPE
    uint32_t seed_lo, seed_hi;
    int64_t env_base;
    int32_t wave_lds_step, wave_lds_emit;      // bytes of LDS per wave
    float dt, omd, mass, inv_mass, cf, k, inv_k, sens, max_speed, L, twoL, R2;
    float dmin_aa, dmin_ao, dmin2_aa, dmin2_ao, cut2_aa, cut2_ao;
    float form_r;          // polygon radius
    float fixed_L;         // ragged: world_half > 0 -> every env's half-width, else 0 (per-N table)
    // caller-owned device buffers (see gsm.h gsm_buffers)
    float2 *pos, *vel;
    int32_t *step_count, *episode;
    float2 *ep_acc, *ep_last;
    float *node_feat, *reward, *cost;
    uint8_t *done;
    int32_t *edge_count, *block_edge_sum;
    int64_t *edge_ptr;
    int32_t *edge_index;
    float *edge_attr;
    uint64_t *row_mask;       // [B][M] radius row masks (segmented path)
    uint64_t *contact_mask;   // [B][N] contact candidates (segmented path)
    int32_t *env_shape;       // [B] ragged: N_env | scenario << 8
    int32_t *assign;          // [B][N] ragged: LSA slot per agent
    uint8_t *degenerate;      // [B] optional: GSM_DEGENERATE_* bits of the launch's final state
    double *lsa_v;            // [B][N] optional: ragged assignment warm start (column duals)
    int32_t *lsa_col;         // [B][N] with lsa_v: the last matching (row -> column)
    int32_t *lsa_stats;       // [B][2] optional: certified warm starts, assignments solved
    const int32_t *block_order;   // ragged mixed: workgroup -> env block, heaviest first (nullptr: identity)
    int64_t edge_capacity;
    const void *actions;
    const uint8_t *env_mask;
    uint64_t *stamps;         // diagnostic builds only (GSM_STAMPS): [waves][8] s_memtime
    // Lagged emission (segmented path, graph chains): a fused step kernel
    // first emits the edges of the PREVIOUS step (its positions and row masks
    // are this launch's inputs) into these outputs, using the per-workgroup
    // edge sums the previous launch wrote to `block_sum`; this launch writes
    // its own sums to block_edge_sum (the other half of a double buffer).
    struct Lag {
        const int32_t *block_sum, *edge_count;
        int64_t *edge_ptr;
        int32_t *edge_index;
        float *edge_attr;
        int64_t cap;
    } lag;
    // Fused rollout (one env per wave or per workgroup, graph chains): K
    // consecutive steps in one launch (gsm_roll_seg_kernel,
    // gsm_roll_tile_kernel). Iteration k runs step t_first + k with the
    // actions at actions + ((t_first + k) % n_actions) * stride and emits the
    // edges of an earlier step (ro); the tail after the loop emits the last.
    // The CSR prefix of step t crosses waves / workgroups through `gran`.
    // Granules are 8-byte {tag32, value32} (gsm_device.h roll_epoch_tag:
    // 20-bit launch epoch, 12-bit step): the ragged rollout's per-wave counts
    // and group sums (Xfer, packing `depth` steps behind), the seg / tile
    // rollouts' workgroup aggregates [K][grid] then inclusive prefixes
    // [K][grid] (decoupled look-back). `epoch` is assigned by the host to
    // every launch from one process-wide counter (gsm_abi.hip
    // next_launch_epoch), so no granule is ever cleared between launches and
    // no granule left by another launch — of this graph or of any graph whose
    // allocation this one reuses — carries this launch's tag. `status` is set
    // when a bounded wait gave up.
    struct Roll {
        const char *actions;
        int64_t stride;
        int32_t n_actions, t_first, K;
        int32_t xW, xNG;      // per-wave hand-off (ragged and packed rollouts): waves of the grid, groups of 64 (gsm_device.h Xfer)
        int32_t depth;        // ragged rollout: steps between an env's step and the packing of its edges
        int32_t slab_e;       // ragged rollout: edges per env slab (the config's max_edges_per_env)
        int32_t place_R;      // ragged rollout placement: waves per SIMD when the grid fills every SIMD
        uint64_t *gran;
        uint32_t *status;
        uint32_t epoch;       // this launch's epoch (20 bits), set per launch by gsm_graph_launch
        int32_t place_force;  // test knob (GSM_ROLL_PLACE=2): register, then decide identity
        int32_t *slab;        // ragged rollout: [depth + 1][B] slabs of [slab_e + 1] u32 row-pair words + [slab_e + 1] f32
        const int32_t *place; // ragged rollout: [W] envs by descending cost (nullptr: env = wave index)
        int32_t place_S;      // SIMDs the grid fills (place_R * place_S = W)
        // pacing of the one-env-per-wave segmented rollout (gsm_seg_kernels.hip
        // pace_level): the rank offset between a CU's workgroups in quarter
        // steps, and per-CU {workgroups arrived, steps finished} counters
        // [kPaceKeys] of this launch and of the slot's next (zeroed by this
        // one); pace nullptr: off
        int32_t pace_q;
        uint32_t *pace, *pace_next;
        // the one-hop CSR prefix of that rollout (gsm_device.h roll_prefix):
        // this launch's chunk sums [K][nc] at csum_stride u64 apart, and the
        // other half of the slot's double buffer (zeroed by this launch)
        uint64_t *csum, *csum_next;
        int32_t csum_stride, pad2;
        // one past the slot's granule words and the ragged slabs (bounds of
        // the checked build's address tests, gsm_device.h gran_chk)
        uint64_t *gran_end;
        int32_t *slab_end;
        // the one-launch eager step's epoch in device memory (kEpochReps
        // replicas kEpochStride u32 apart; gsm_roll_seg_kernel kEager)
        uint32_t *dev_epoch;
    } roll;
    // A rollout's per-step outputs: step k's at base + k * stride (elements;
    // stride 0 = every step into the bound buffers, > 0 = a rollout buffer's
    // slots, gsm_graph_capture_into). Edges of step k at index / attr + k *
    // e_s, edge_ptr + k * ep_s, capacity cap. In the bound buffers (stride 0)
    // only the last step's edges go to eidx / eattr; the earlier steps' go to
    // the library's scratch eidx_mid / eattr_mid (same capacity): workgroups
    // emit at different paces, and an earlier step's edges written late must
    // not land on the last step's (roll_edge_sink).
    struct RollOut {
        float *nf, *rew, *cost;
        uint8_t *done;
        int32_t *ecount;
        int64_t *eptr;
        int32_t *eidx;
        float *eattr;
        int64_t nf_s, rc_s, done_s, ec_s, ep_s, ei_s, ea_s, cap;
        int32_t *eidx_mid;
        float *eattr_mid;
        int32_t *asg;         // ragged: assignment [B][N] of step k at asg + k * as_s
        int64_t as_s;
    } ro;
};

// where an emission writes its edges
struct EdgeSink {
    int32_t *index;   // [2][cap]: sources, then destinations
    float *attr;
    int64_t cap;
};

// Where a rollout launch of K steps emits step j's edges (DevParams::RollOut):
// a rollout buffer's slot j, else the bound buffers for the last step and the
// library's scratch for the others.
template <bool kSlots, typename Params>
__device__ __forceinline__ EdgeSink roll_edge_sink(const Params &q, int j, int K) {
    if (kSlots) return EdgeSink{q.ro.eidx + j * q.ro.ei_s, q.ro.eattr + j * q.ro.ea_s, q.ro.cap};
    if (j == K - 1) return EdgeSink{q.ro.eidx, q.ro.eattr, q.ro.cap};
    return EdgeSink{q.ro.eidx_mid, q.ro.eattr_mid, q.ro.cap};
}

// Launch the step kernel (physics / reset / observe by p.mode) and the edge
// emitter for all B envs on `s`. Returns the first hipError_t.
hipError_t launch_step(const DevParams &p, hipStream_t s);
// for explicit graph construction (kernel nodes)
int grid_blocks(const DevParams &p);        // emit kernel (and tile/ragged step) workgroups
int step_grid_blocks(const DevParams &p);   // step kernel workgroups
const void *step_kernel_fn(const DevParams &p);
const void *emit_kernel_fn(const DevParams &p);
const void *step_seg_kernel_fn(const DevParams &p);
// step kernel that emits the previous step's edges first (p.lag); nullptr
// where the path has none (tile: measured no faster than its own emit
// launch)
const void *lag_step_kernel_fn(const DevParams &p);
const void *lag_step_seg_kernel_fn(const DevParams &p);
const void *emit_seg_kernel_fn(const DevParams &p);
// fused K-step rollout kernel (nullptr where the config has none: G > 1,
// runtime shapes, other families) and its LDS bytes
const void *roll_seg_kernel_fn(const DevParams &p, bool slots);   // slots: a rollout buffer's outputs
// the one-launch eager step (K = 1, device-side epoch; one env per wave shapes)
const void *roll_seg_eager_kernel_fn(const DevParams &p);
int roll_seg_envs_per_block(const DevParams &p);
// the segmented rollout packs four small envs per wave (gsm_roll_pack_kernel):
// per-wave CSR hand-off granules, as the ragged rollout (Roll::xW / xNG)
bool roll_packed(const DevParams &p);   // 4 (one env per wave) or 16 (small envs, four per wave)
size_t roll_kernel_lds(const DevParams &p);
const void *roll_tile_kernel_fn(const DevParams &p, bool slots);   // nullptr unless p.tile_sym
size_t roll_tile_kernel_lds(const DevParams &p);
const void *step_ragged_kernel_fn();
// fused K-step rollout of a ragged batch (one env per wave, edges packed
// `depth` steps behind through per-env slabs) and its LDS bytes
const void *roll_ragged_kernel_fn(const DevParams &p, bool slots);
size_t roll_ragged_kernel_lds(const DevParams &p);
constexpr int kRaggedRollMaxDepth = 8;
// The ragged rollout's SIMD-balanced placement (gsm_ragged_kernels.hip
// roll_place): u64 words after its per-wave granules. SIMD keys are 13 bits
// of HW_ID / XCC_ID.
struct PlaceArea {
    static constexpr int kKeys = 8192;
    static constexpr int kMask = 0;                 // [kKeys] {tag, wave-slot bits}
    static constexpr int kRank = kKeys;             // [kKeys] {tag, SIMD index within its XCC}
    static constexpr int kBad = 2 * kKeys;          // {tag, 0}: a SIMD holds more than place_R waves
    static constexpr int kGroups = 64;              // counter groups: XCC x shader engine
    static constexpr int kArrive = 2 * kKeys + 8;   // [kGroups] workgroups arrived, one per 64 bytes
    static constexpr int kNsimd = kArrive + 8 * kGroups;   // [kGroups] SIMDs seen, one per 64 bytes
    static constexpr int kMode = kNsimd + 8 * kGroups;     // [kGroups] {tag, decision} replicas, one per 64 bytes
    static constexpr int kClaim = kMode + 8 * kGroups;     // [W] u32 tags: the env claimed this launch
    static constexpr size_t words(int W) { return (size_t)kClaim + ((size_t)W + 1) / 2; }
};
const void *lag_step_ragged_kernel_fn();   // kLag: the previous step's emission first
const void *step_tile_kernel_fn();
const void *emit_tile_kernel_fn();
int block_threads(const DevParams &p);
// threads per workgroup of the config's rollout kernel (the split packed
// small-env rollout runs 512: four stepping and four emitting waves)
int roll_block_threads(const DevParams &p);
bool roll_pack_split(const DevParams &p);
const void *emit_ragged_kernel_fn();
// ragged path: per-device constant tables (unit circle, line fractions,
// half-widths) computed on the host with libm; uploaded once per device.
hipError_t upload_ragged_tables();
size_t step_kernel_lds(const DevParams &p);
size_t emit_kernel_lds(const DevParams &p);
hipError_t launch_step_kernel(const DevParams &p, hipStream_t s);
// rollout granules: word 0 = epoch0, the rest 0, by agent-scope atomic stores
hipError_t launch_granule_init(void *g, size_t bytes, uint32_t epoch0, hipStream_t s);
hipError_t launch_emit_kernel(const DevParams &p, hipStream_t s);
hipError_t launch_attn_aggregate(const float *q, const float *k, const float *v, const float *edge_w,
                                 const float *w_e, const int64_t *row_ptr, const int32_t *col,
                                 const float *skip, int64_t n_nodes, int HC, int C, float scale, float *out,
                                 hipStream_t s);
hipError_t launch_render(const float *node_feat, int64_t n_envs, int32_t n_entities, const int64_t *edge_ptr,
                         const int32_t *edge_index, int64_t edge_capacity, const int32_t *env_ids,
                         int32_t n_frames, float half_width, float r_agent, float r_target, float r_obst,
                         int32_t width, int32_t height, int32_t draw_edges, uint8_t *rgba_out, hipStream_t s);

}  // namespace gsm
