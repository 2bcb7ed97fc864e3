/*
 * gsm.h — C ABI of libgsm.so, the MI355X (gfx950) batched step path of
 * GS-MARL's MultiAgentGraphConstrainEnv.
 *
 * Drop-in boundary. The reference has no FFI: its boundary is the Python
 * env classes in gsmarl/envs/mpe_env/multiagent/environment.py
 * (/root/reference/GSMARL.egg-info/SOURCES.txt:15; contracts at
 * /root/reference/readme.md:29-41), constructed by make_env.py
 * (SOURCES.txt:12) and called from the vec-env workers (SOURCES.txt:11).
 * The reference sources are absent (readme.md:1), so each entry point below
 * cites the reference interface it replaces at the granularity available.
 * The binding a maintainer adds on the reference side (ctypes) is shown in
 * INTEGRATION.md; the in-tree binding is gs-marl_amd/gsmarl_amd/_lib.py.
 *
 * Rules of the ABI:
 *  - plain C types only; pointers to device memory are owned by the caller
 *    (PyTorch allocates them) and merely borrowed by the library;
 *  - nothing is allocated and nothing synchronises inside gsm_step /
 *    gsm_reset / gsm_observe, so they can be captured into a HIP graph;
 *  - every call returns GSM_OK (0) or a negative gsm_status; no C++
 *    exception crosses the boundary; gsm_last_error() has the message;
 *  - a handle is used from one host thread at a time (the GIL serialises);
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default).
 */
#ifndef GSM_H_
#define GSM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 4: lagged-emission graph chains (GSM_GRAPH_UNFUSED / _LAG_ONLY), gsm_render
 * 5: degenerate-state handling: gsm_config.strict_degenerate,
 *    gsm_buffers.degenerate */
/* 6: fused rollout graphs (GSM_GRAPH_ROLL, gsm_graph_roll_status, gsm_graph_info)
 * 7: gsm_get_state / gsm_set_state; rollout graphs emit every step's edges in
 *    their one launch (no separate emit launch)
 * 8: ragged rollouts (n_steps <= 4094), gsm_graph_roll_placement */
#define GSM_ABI_VERSION 8

typedef enum gsm_status {
    GSM_OK = 0,
    GSM_EINVAL = -1,   /* bad argument / config                        */
    GSM_EHIP = -2,     /* HIP runtime error (message has hipError_t)    */
    GSM_ESTATE = -3,   /* call out of order (e.g. step before bind)     */
} gsm_status;

typedef enum gsm_scenario {
    GSM_SCEN_NAVIGATION = 0,   /* scenarios/exp1.py|exp2.py (SOURCES.txt:21-22)          */
    GSM_SCEN_POLYGON = 1,      /* scenarios/simple_formation.py (SOURCES.txt:24; readme.md:89) */
    GSM_SCEN_LINE = 2,         /* scenarios/simple_line.py (SOURCES.txt:25; readme.md:90)      */
    GSM_SCEN_MIXED = 3,        /* env id mod 3 -> navigation/polygon/line, N per env drawn   */
} gsm_scenario;

/* Ragged batches (polygon, line, mixed): every env has its own agent count
 * N_env <= n_agents (= N_max <= GSM_RAGGED_MAX_AGENTS) and its own scenario,
 * stored padded: entity rows agents [0, N_max), targets [N_max, N_max+T_max),
 * obstacles [N_max+T_max, E). env_shape[b] = N_env | scenario << 8. */
#define GSM_RAGGED_MAX_AGENTS 32

typedef enum gsm_action_fmt {
    GSM_ACT_ONEHOT = 0,   /* float32 [B][N][5]; u = [a1-a2, a3-a4] (MPE discrete_action_space) */
    GSM_ACT_INDEX = 1,    /* int32   [B][N];    same mapping as the one-hot of the index        */
    GSM_ACT_CONT = 2,     /* float32 [B][N][2]; u = a (continuous)                              */
} gsm_action_fmt;

/* Launch modes of the step kernel (gsm_observe / gsm_reset reuse it). */
typedef enum gsm_mode {
    GSM_MODE_STEP = 0,
    GSM_MODE_RESET = 1,
    GSM_MODE_OBSERVE = 2,
} gsm_mode;

/* Environment configuration; mirrors gsmarl_amd.config.EnvConfig 1:1.
 * Replaces the env part of gsmarl/config.py (SOURCES.txt:7, readme.md:47)
 * and the constants of core.py / the scenario files. */
typedef struct gsm_config {
    int32_t abi_version;      /* = GSM_ABI_VERSION                           */
    int32_t scenario;         /* gsm_scenario                                */
    int32_t n_envs;           /* B: env instances held by this handle        */
    int32_t n_agents;         /* N (goals = N)                               */
    int32_t n_obstacles;      /* No                                          */
    int32_t episode_length;   /* readme.md:101 -> 100                        */
    int32_t auto_reset;       /* reset an env in-kernel when its episode ends */
    int32_t shared_reward;    /* every agent gets the sum of rewards         */
    int64_t env_base;         /* global id of env 0 (sharding; Philox key)   */
    uint64_t seed;
    float dt, damping, mass, contact_force, contact_margin, sensitivity;
    float max_speed;          /* <= 0: no clamp (MPE max_speed = None)       */
    float world_half;         /* L: layout box is [-L, L]^2                  */
    float agent_size, goal_size, obstacle_size;
    float sense_radius;       /* R: graph edge radius                        */
    float contact_cutoff;     /* skip pair force when d - dmin > cutoff*k     */
    /* ragged scenarios (ignored by navigation) */
    int32_t n_agents_min;     /* mixed: N_env drawn from [n_agents_min, n_agents] */
    float formation_radius;   /* polygon: N-gon radius (readme.md:89 -> 0.5)  */
    /* App. A S16. A coincident collider pair (d = 0, at least one agent) has
     * no direction: by default its contact force is guarded to zero; with
     * strict_degenerate != 0 it is NaN as in MPE's get_collision_force
     * (delta / dist with dist = 0), and, as MPE evaluates every pair, an
     * agent whose position is NaN makes the force of every agent of its env
     * NaN. Either way the env is flagged in gsm_buffers.degenerate. */
    int32_t strict_degenerate;
} gsm_config;

/* Sizes the caller must allocate (gsm_query_sizes). */
typedef struct gsm_sizes {
    int32_t n_entities;       /* E = 2N + No                                 */
    int32_t node_feat_dim;    /* 7                                           */
    int32_t obs_dim;          /* 6                                           */
    int32_t envs_per_block;   /* envs handled by one step-kernel workgroup   */
    int32_t n_blocks;         /* length of block_edge_sum                    */
    int32_t max_edges_per_env;
    int64_t edge_capacity;    /* length of edge_attr and of each edge_index row */
    int32_t n_colliders;      /* M: collider rows per env (agents + obstacles)  */
    int32_t n_targets;        /* T_max: goal/landmark rows per env            */
    int32_t mask_words;       /* W: uint64 words per mask row, ceil(M / 64)   */
} gsm_sizes;

/* Caller-owned device buffers (all contiguous, row-major). */
typedef struct gsm_buffers {
    /* state */
    float *pos;               /* [B][E][2]   agents, goals/landmarks, obstacles */
    float *vel;               /* [B][N][2]   agents only (landmarks immovable) */
    int32_t *step_count;      /* [B]         steps since reset                */
    int32_t *episode;         /* [B]         episode index (-1 before reset)  */
    float *ep_acc;            /* [B][2]      running (sum reward, sum cost)   */
    float *ep_last;           /* [B][2]      totals of the last finished episode */
    /* outputs of the last reset/step/observe */
    float *node_feat;         /* [B][E][7]   vx vy px py gx-px gy-py type     */
    float *reward;            /* [B][N]                                       */
    float *cost;              /* [B][N]      collision counts (exact ints)    */
    uint8_t *done;            /* [B]                                          */
    int32_t *edge_count;      /* [B]                                          */
    int32_t *block_edge_sum;  /* [n_blocks]  scratch                          */
    int64_t *edge_ptr;        /* [B+1]       CSR offsets into edge arrays     */
    int32_t *edge_index;      /* [2][edge_capacity] global node ids (b*E+e)   */
    float *edge_attr;         /* [edge_capacity]    distance                  */
    /* derived state, valid for the positions in `pos` after any reset/step/
     * observe; a caller that rewrites `pos`/`vel` must call gsm_observe      */
    uint64_t *row_mask;       /* [B][M][W] radius adjacency rows (bit = collider) */
    uint64_t *contact_mask;   /* [B][N][W] contact candidates of each agent        */
    /* ragged scenarios only (may be NULL for navigation) */
    int32_t *env_shape;       /* [B]    N_env | scenario << 8 (set at every layout) */
    int32_t *assign;          /* [B][N] polygon/line slot of each agent (LSA), -1 else */
    /* optional (NULL: not written): per env, after every reset/step/observe,
     * GSM_DEGENERATE_COINCIDENT if two colliders (at least one an agent) sit
     * at the same position — the next step meets d = 0 — and
     * GSM_DEGENERATE_NONFINITE if an agent position is not finite (strict
     * mode, or a caller-written state) */
    uint8_t *degenerate;      /* [B] */
    /* optional, polygon/line assignment warm start (NULL: every per-step
     * assignment is solved from scratch): the column duals and the matching
     * of each env's last assignment, kept by the library between launches.
     * A warm-started assignment is used only when certified to be the unique
     * optimum — then it IS scipy's result; otherwise the scipy recurrence runs
     * from scratch. Initialise lsa_col to -1 (lsa_v to 0). */
    double *lsa_v;            /* [B][N] */
    int32_t *lsa_col;         /* [B][N] */
    int32_t *lsa_stats;       /* [B][2] optional counters: certified warm starts, assignments solved */
} gsm_buffers;

#define GSM_DEGENERATE_COINCIDENT 1
#define GSM_DEGENERATE_NONFINITE 2

/* Output redirection (an on-device rollout buffer
 * filled without copies). Where one step / observe writes its outputs; NULL
 * members keep the bound buffers. edge_index is [2][edge_capacity] when
 * redirected; edges past edge_capacity are not written, while edge_ptr keeps
 * the true offsets (edge_ptr[B] > edge_capacity flags the overflow). A
 * redirected launch writes full node-feature rows (goal / obstacle rows are
 * otherwise rewritten only when a layout changes). */
typedef struct gsm_outputs {
    float *node_feat;         /* [B][E][7] */
    float *reward;            /* [B][N]    */
    float *cost;              /* [B][N]    */
    uint8_t *done;            /* [B]       */
    int32_t *edge_count;      /* [B]       */
    int64_t *edge_ptr;        /* [B+1]     */
    int32_t *edge_index;      /* [2][edge_capacity] */
    float *edge_attr;         /* [edge_capacity]    */
    int32_t *assign;          /* [B][N]  (ragged scenarios) */
    int64_t edge_capacity;
} gsm_outputs;

typedef struct gsm_handle gsm_handle;

int gsm_abi_version(void);

/* Validates cfg and fills sizes. Host-only, no HIP call. */
int gsm_query_sizes(const gsm_config *cfg, gsm_sizes *out);

/* Replaces make_env(scenario) -> MultiAgentGraphConstrainEnv(world, ...)
 * (make_env.py, SOURCES.txt:12; environment.py, SOURCES.txt:15). Host-only. */
int gsm_create(const gsm_config *cfg, gsm_handle **out);

/* Borrow caller-allocated device buffers (sizes from gsm_query_sizes). */
int gsm_bind(gsm_handle *h, const gsm_buffers *bufs);

/* Replaces env.reset() -> scenario.reset_world(world) (environment.py /
 * scenario.py, SOURCES.txt:15,19). reseed != 0: episode counters restart
 * and `seed` becomes the layout key. env_mask: device uint8 [B] or NULL
 * (= all envs). Outputs are recomputed for every env. */
int gsm_reset(gsm_handle *h, uint64_t seed, int reseed, const uint8_t *env_mask, void *stream);

/* Replaces env.step(action_n) (environment.py, SOURCES.txt:15): _set_action,
 * world.step() (core.py, SOURCES.txt:14), reward/cost/done callbacks and the
 * graph observation, for all B envs. actions: device pointer in action_fmt.
 * One kernel launch (the config's rollout kernel with one step) at 6-24
 * navigation agents, else a step kernel + an emit kernel; GSM_EAGER_ONE_LAUNCH
 * (read at gsm_bind) forces either. Same outputs either way. */
int gsm_step(gsm_handle *h, const void *actions, int action_fmt, void *stream);

/* Recompute every output for the current state (after the caller rewrote
 * state buffers, e.g. set_state). */
int gsm_observe(gsm_handle *h, void *stream);

/* The simulator state (SURVEY.md §8(b) gsm_get_state / gsm_set_state):
 * device pointers of the caller; NULL members are skipped. Everything else
 * the library keeps (the row / contact masks, node features, edges) is
 * derived from it. */
typedef struct gsm_state {
    float *pos;               /* [B][E][2] */
    float *vel;               /* [B][N][2] */
    int32_t *step_count;      /* [B]       */
    int32_t *episode;         /* [B]       */
    float *ep_acc;            /* [B][2]    */
    float *ep_last;           /* [B][2]    */
    int32_t *env_shape;       /* [B]       ragged scenarios: N_env | scenario << 8 */
} gsm_state;

/* Checkpoint / injection of env state (what a reference caller does by
 * reading or writing the world's entity states directly, core.py
 * EntityState, SOURCES.txt:14). gsm_get_state copies the bound state into
 * `out`. gsm_set_state copies `in` into the bound state and then runs
 * gsm_observe, which re-derives every output and the derived per-position
 * state (row masks, contact candidates) the next step relies on — the one
 * call a non-Python caller needs after writing positions or velocities.
 * Stream-ordered device-to-device copies; no synchronisation. */
int gsm_get_state(gsm_handle *h, const gsm_state *out, void *stream);
int gsm_set_state(gsm_handle *h, const gsm_state *in, void *stream);

/* gsm_step / gsm_observe with their outputs redirected (gsm_outputs). */
int gsm_step_into(gsm_handle *h, const void *actions, int action_fmt, const gsm_outputs *out, void *stream);
int gsm_observe_into(gsm_handle *h, const gsm_outputs *out, void *stream);

/* Build HIP graph `slot` (0..GSM_GRAPH_SLOTS-1) of n_steps steps; the j-th
 * step reads its actions at actions + (j % n_actions) * action_stride_bytes.
 * flags: which kernels each step runs (GSM_GRAPH_STEP | GSM_GRAPH_EMIT; 0 =
 * both) and optional HIP event-record nodes: GSM_GRAPH_TIME_EACH brackets
 * every kernel, GSM_GRAPH_TIME_ENDS brackets the whole graph (per-kernel
 * means over back-to-back launches, no event nodes between kernels).
 * A graph running only GSM_GRAPH_EMIT re-emits the current step's edges.
 * Segmented (navigation, N + No <= 64) and ragged (polygon / line / mixed)
 * configs chain the two kernels with lagged emission: step j+1's kernel first emits step j's edges (they depend
 * only on its input positions and row masks), so a step is one launch and a
 * final emit launch ends the graph; every step's outputs are complete when
 * the graph has run, exactly as with the two-kernel chain (the library
 * allocates one n_blocks int32 buffer for this on first use).
 * GSM_GRAPH_UNFUSED forces the two-kernel chain (TIME_EACH implies it);
 * GSM_GRAPH_LAG_ONLY builds n_steps lagged step kernels and nothing else
 * (a timing tool: the last step's edges are left unemitted; segmented / ragged only).
 * Graphs are dropped by gsm_bind and by a reseed to a different seed. */
#define GSM_GRAPH_SLOTS 4
#define GSM_GRAPH_STEP 1
#define GSM_GRAPH_EMIT 2
#define GSM_GRAPH_TIME_EACH 4
#define GSM_GRAPH_TIME_ENDS 8
#define GSM_GRAPH_UNFUSED 16
#define GSM_GRAPH_LAG_ONLY 32
/* GSM_GRAPH_ROLL: all n_steps (<= 4094) steps and their edges run in ONE
 * launch (navigation configs with a compiled rollout shape — 3, 6, 12 or 24
 * agents with as many obstacles, one env per wave — the tile path, one env
 * per workgroup, and ragged batches, one env per wave; the whole batch in one
 * residency round). Each wave keeps its
 * env's state on chip across the steps; workgroups hand the CSR edge-count
 * prefix to each other through tagged granules (bounded waits), and a tail
 * iteration emits the last step's edges. Outputs after the graph are
 * identical to the lagged chain's (every step's edges are emitted; in the
 * bound buffers the earlier steps' go to a library scratch of the bound edge
 * capacity, allocated on first use, since a workgroup may trail its
 * successors by steps). Combines with GSM_GRAPH_TIME_ENDS only (the events
 * then bracket the launch: gsm_graph_kernel_ms gives its time per step);
 * GSM_EINVAL where the config has no rollout kernel, where the action rows
 * span 4 GiB or more (n_actions * action_stride_bytes >= 2^32: the rollout
 * kernels address them with 32-bit offsets), where n_steps > 4094, or where
 * the batch exceeds one residency round of the rollout kernel (occupancy x
 * CUs; on an MI355X 8192 envs of the one-env-per-wave and ragged rollouts —
 * 2048 workgroups, also the bound of the one-hop CSR prefix's 64 chunk sums of
 * 64 workgroups — 16384 of the packed small-env rollout, 1024 of the tile
 * rollout; shard larger batches across handles or GPUs, env_base). Without
 * GSM_GRAPH_ROLL such a capture takes the per-step chain instead. */
#define GSM_GRAPH_ROLL 64
int gsm_graph_capture(gsm_handle *h, int32_t slot, const void *actions, int64_t action_stride_bytes,
                      int32_t n_actions, int32_t n_steps, int action_fmt, int flags);
/* As gsm_graph_capture (both kernels, no timing events), with the j-th
 * step's outputs redirected to per_step[j] (n_steps entries). Where the config
 * has a rollout kernel (GSM_GRAPH_ROLL) and every redirected field of the
 * slots sits at a constant stride (a rollout buffer), the graph is one rollout
 * launch writing step j's outputs into slot j; else the per-step chain. */
int gsm_graph_capture_into(gsm_handle *h, int32_t slot, const void *actions, int64_t action_stride_bytes,
                           int32_t n_actions, int32_t n_steps, int action_fmt, const gsm_outputs *per_step);
/* Launch the graph in `slot` on `stream` (stream-ordered, asynchronous). A
 * rollout slot (GSM_GRAPH_ROLL, or a rollout buffer's single launch) is its one
 * kernel launched directly, with a fresh launch epoch for its hand-off tags and
 * its half of the slot's pacing counters; so it cannot be recorded into a
 * stream capture (GSM_ESTATE on a capturing stream: capture the per-step chain
 * instead). The rollout slots of a handle share its state and scratch, so their
 * launches never overlap: a launch on a different stream than the handle's
 * previous rollout launch first waits, on the device, for an event the library
 * records behind every rollout launch (no host synchronisation; the previous
 * stream may have been destroyed since). */
int gsm_graph_launch(gsm_handle *h, int32_t slot, void *stream);
/* The graph in `slot`: its step count (0 if none) and whether it is one
 * fused rollout launch (GSM_GRAPH_ROLL, or gsm_graph_capture_into on a
 * rollout buffer) rather than a per-step chain. */
int gsm_graph_info(gsm_handle *h, int32_t slot, int32_t *steps, int32_t *fused);
/* After graph launches have completed: *gave_up = a non-zero reason code if
 * any bounded in-launch wait timed out (1: a rollout launch's CSR hand-off, or
 * the ragged lagged chain's staging wait) or an in-launch check failed (2: an
 * out-of-range CSR offset, 4: a doubly claimed env, 5: a placement slot
 * outside its table; 6, in a checked build (-DGSM_CHECKED): a hand-off granule
 * or slab address outside its allocation) since the last call (that launch's
 * outputs are then invalid), else 0. Clears the flag. Synchronises (reads a
 * device word). */
int gsm_graph_roll_status(gsm_handle *h, int32_t *gave_up);
/* Ragged mixed rollouts deal their envs to the SIMDs by estimated cost when
 * every wave of the launch is resident (else env = wave index; same outputs
 * either way). After launches have completed: how many dealt their envs and
 * how many fell back since the last call. Clears the counts; synchronises. */
int gsm_graph_roll_placement(gsm_handle *h, int64_t *dealt, int64_t *fallback);
/* After a timed launch of `slot` has completed: mean duration (ms) of the
 * step and emit kernels (TIME_EACH), and the whole graph (both flags). */
int gsm_graph_kernel_ms(gsm_handle *h, int32_t slot, float *step_mean_ms, float *emit_mean_ms,
                        float *total_ms);

/* Graph-attention message passing over a CSR graph (SURVEY.md §8(f) next #3:
 * the GNN encoder after the observation; replaces the edge-softmax /
 * aggregation of torch-geometric's TransformerConv, requirements.txt:119, as
 * used by the reference's GNN in gsmarl/algorithms, SOURCES.txt:8). For each
 * target i with sources j = col[row_ptr[i] .. row_ptr[i+1]), per head h:
 *   e_ij = edge_w[ij] * w_e[h*C + c]           (edge_w, w_e may be NULL: e = 0)
 *   a_ij = softmax_j(scale * <q_i[h], k_j[h] + e_ij>)
 *   out_i[h] = sum_j a_ij (v_j[h] + e_ij) + skip_i[h]      (skip may be NULL)
 * q, k, v, skip, out: device f32 [n_nodes][heads*channels]; row_ptr: int64
 * [n_nodes+1]; col: int32 source ids; channels a power of two and
 * heads*channels <= 64. Stateless; asynchronous on `stream`. */
int gsm_attn_aggregate(const float *q, const float *k, const float *v, const float *edge_w, const float *w_e,
                       const int64_t *row_ptr, const int32_t *col, const float *skip, int64_t n_nodes,
                       int32_t heads, int32_t channels, float scale, float *out, void *stream);

/* Episode frames (replaces the pyglet viewer of
 * multiagent/rendering.py, SOURCES.txt:18, used by scripts/render_mpe.py,
 * SOURCES.txt:30, for the demo/ GIFs, readme.md:64). Draws env env_ids[f]
 * of a batch into frame f of rgba (uint8 [n_frames][height][width][4]) from
 * its node-feature rows (node_feat: f32 [n_envs][n_entities][7], position in
 * columns 2-3, type 0 agent / 1 goal-target / 2 obstacle / -1 padding in
 * column 6) and, with GSM_RENDER_EDGES, its packed CSR edges (edge_ptr int64
 * [n_envs+1], edge_index int32 [2][edge_capacity], global ids b*n_entities+e)
 * as black lines. Camera [-L, L]^2 with L = half_width, or sqrt(n_agents/3)
 * of the env when half_width <= 0; disc radii = the three sizes. Any rollout
 * slot can be rendered. Out-of-range env ids give white frames. Stateless;
 * asynchronous on `stream`. */
#define GSM_RENDER_EDGES 1
int gsm_render(const float *node_feat, int64_t n_envs, int32_t n_entities, const int64_t *edge_ptr,
               const int32_t *edge_index, int64_t edge_capacity, const int32_t *env_ids, int32_t n_frames,
               float half_width, float agent_size, float target_size, float obstacle_size, int32_t width,
               int32_t height, int32_t flags, uint8_t *rgba, void *stream);

/* Diagnostics: device buffer (uint64 [2 * n_blocks * 4][16]) that libraries
 * built with -DGSM_STAMPS fill with per-wave phase timestamps; ignored by the
 * product build. NULL disables. */
int gsm_debug_set_stamps(gsm_handle *h, void *stamps);

int gsm_destroy(gsm_handle *h);

/* Copies the last error message of h (or of the library when h == NULL). */
int gsm_last_error(const gsm_handle *h, char *buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* GSM_H_ */
