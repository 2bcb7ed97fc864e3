// gsm_kernels.hip — kernel dispatch for the three kernel families.
//
// Each env.step is two launches: a step kernel (physics,
// reward/cost, done/auto-reset, node features, adjacency masks, edge count)
// and an edge emitter (global offsets from the step kernel's edge counts,
// then the row-major COO edges). The family follows the config:
//
//   segmented  navigation, M = N + No <= 64 colliders: G = 64/M envs per
//              wave, 4 waves per workgroup (gsm_seg_kernels.hip);
//   tile       navigation, M > 64: one 512-thread workgroup per env
//              (gsm_tile_kernels.hip);
//   ragged     polygon / line / mixed: one wave per env, per-env shape,
//              per-step assignment (gsm_ragged_kernels.hip).
//
// Inside a graph chain the segmented and ragged families fuse the emitter of
// step t into the step kernel of step t+1 ("lagged emission"):
// the edges of step t are functions of the positions and row masks that step
// t+1 loads anyway, so the chain is step_0, lag_step_1, ..., lag_step_{T-1},
// emit_{T-1}: one launch per step instead of two.
//
// Launches go through hipLaunchKernel with the family's kernel pointers; the
// HIP-graph builder (gsm_abi.hip) uses the same pointers, grid and LDS sizes.
#include "gsm_device.h"

namespace gsm {

int block_threads(const DevParams &p) { return p.path == kPathTile ? kTileBlock : kBlock; }

int grid_blocks(const DevParams &p) {
    if (p.path == kPathTile) return p.B;
    const int per_block = kWavesPerBlock * p.G;
    return (p.B + per_block - 1) / per_block;
}
int step_grid_blocks(const DevParams &p) { return grid_blocks(p); }
const void *step_kernel_fn(const DevParams &p) {
    if (p.path == kPathRagged) return step_ragged_kernel_fn();
    if (p.path == kPathTile) return step_tile_kernel_fn();
    return step_seg_kernel_fn(p);
}
const void *lag_step_kernel_fn(const DevParams &p) {
    if (p.path == kPathRagged) return lag_step_ragged_kernel_fn();
    return p.path == kPathSeg ? lag_step_seg_kernel_fn(p) : nullptr;
}
const void *emit_kernel_fn(const DevParams &p) {
    if (p.path == kPathRagged) return emit_ragged_kernel_fn();
    if (p.path == kPathTile) return emit_tile_kernel_fn();
    return emit_seg_kernel_fn(p);
}
size_t step_kernel_lds(const DevParams &p) {
    // segmented / ragged: + per-wave edge sums and (lagged emission) per-wave prefix words;
    // ragged: + the lagged emission's staged inputs (gsm_ragged_kernels.hip RaggedLagLds:
    // counters, 4 x 64 row masks, 4 x E_max positions)
    if (p.path == kPathTile) return (size_t)p.wave_lds_step;
    const size_t lag = p.path == kPathRagged ? 64 + 8 * kWave * kWavesPerBlock + 8 * (size_t)kWavesPerBlock * p.E : 0;
    return (size_t)kWavesPerBlock * p.wave_lds_step + 32 + lag;
}
size_t emit_kernel_lds(const DevParams &p) {
    return p.path == kPathTile ? (size_t)p.wave_lds_emit : (size_t)kWavesPerBlock * p.wave_lds_emit + 16;
}

static hipError_t launch_fn(const void *fn, const DevParams &p, int grid, size_t lds, hipStream_t s) {
    (void)hipGetLastError();   // report this launch's error only
    void *args[] = {const_cast<DevParams *>(&p)};
    const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(block_threads(p)), args, lds, s);
    return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_step_kernel(const DevParams &p, hipStream_t s) {
    return launch_fn(step_kernel_fn(p), p, step_grid_blocks(p), step_kernel_lds(p), s);
}

hipError_t launch_emit_kernel(const DevParams &p, hipStream_t s) {
    return launch_fn(emit_kernel_fn(p), p, grid_blocks(p), emit_kernel_lds(p), s);
}

hipError_t launch_step(const DevParams &p, hipStream_t s) {
    hipError_t e = launch_step_kernel(p, s);
    if (e != hipSuccess) return e;
    return launch_emit_kernel(p, s);
}

// Rollout granules are initialised by the same agent-scope stores the
// rollouts publish with: a recycled allocation can otherwise show an agent-scope
// load the previous allocation's granules (observed: a memset's zeros did not
// supersede them), and a stale granule whose tag happens to match would be
// taken for this launch's. Word 0 is the launch epoch, the rest zero.
__global__ __launch_bounds__(256) void gsm_granule_init_kernel(uint32_t *g, int64_t words, uint32_t epoch0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
        __hip_atomic_store((gu32 *)(g + i), i == 0 ? epoch0 : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t launch_granule_init(void *g, size_t bytes, uint32_t epoch0, hipStream_t s) {
    const int64_t words = (int64_t)(bytes / 4);
    const int64_t need = (words + 255) / 256;
    const int blocks = (int)(need < 1024 ? need : 1024);
    uint32_t *gp = (uint32_t *)g;
    int64_t n = words;
    void *args[] = {&gp, &n, &epoch0};
    return hipLaunchKernel(reinterpret_cast<const void *>(&gsm_granule_init_kernel), dim3(blocks), dim3(256), args, 0,
                           s);
}

}  // namespace gsm
