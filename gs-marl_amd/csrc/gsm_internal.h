// Internal (non-ABI) declarations shared by gsm_kernels.hip and gsm_abi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsm {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;              // one env per wave
constexpr int kBlock = kWave * kWavesPerBlock;
enum : int32_t { kPathGeneric = 0, kPathSeg = 1 };
constexpr int kMaxSegEnvsPerWave = 16;   // keeps a block's envs (4G) within one wave's lanes

// Everything a launch needs, passed by value (kernarg segment, < 4 KB).
// fp32 constants are formed on the host exactly as oracle/batch_ref.py:Spec
// forms them in fp32 mode (gsm_abi.hip: derive()).
struct DevParams {
    int32_t B, N, No, E, M, S, EL, auto_reset, shared_reward;
    int32_t mode, action_fmt, reseed;
    int32_t path;          // kPathSeg (M <= 64) or kPathGeneric
    int32_t G;             // envs per wave (segmented path), 1 otherwise
    uint32_t seed_lo, seed_hi;
    int64_t env_base;
    int32_t wave_lds_step, wave_lds_emit;      // bytes of LDS per wave
    float dt, omd, mass, inv_mass, cf, k, inv_k, sens, max_speed, L, twoL, R2;
    float dmin_aa, dmin_ao, dmin2_aa, dmin2_ao, cut2_aa, cut2_ao;
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
    int64_t edge_capacity;
    const void *actions;
    const uint8_t *env_mask;
    uint64_t *stamps;         // diagnostic builds only (GSM_STAMPS): [waves][8] s_memtime
};

// Launch the step kernel (physics / reset / observe by p.mode) and the edge
// emitter for all B envs on `s`. Returns the first hipError_t.
hipError_t launch_step(const DevParams &p, hipStream_t s);
// for explicit graph construction (kernel nodes)
int grid_blocks(const DevParams &p);
const void *step_kernel_fn(const DevParams &p);
const void *emit_kernel_fn(const DevParams &p);
const void *step_seg_kernel_fn(const DevParams &p);
const void *emit_seg_kernel_fn(const DevParams &p);
size_t step_kernel_lds(const DevParams &p);
size_t emit_kernel_lds(const DevParams &p);
hipError_t launch_step_kernel(const DevParams &p, hipStream_t s);
hipError_t launch_emit_kernel(const DevParams &p, hipStream_t s);

}  // namespace gsm
