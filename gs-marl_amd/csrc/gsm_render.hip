// gsm_render.hip — episode frames from the env's own outputs (SURVEY.md
// §8(f) next #4; the reference renders with the MPE pyglet viewer,
// multiagent/rendering.py, SOURCES.txt:18, and ships GIFs under demo/,
// readme.md:64). The drawing convention (camera over [-L, L]^2, disc colours,
// outline width, black edge lines) is the one pinned to the demo GIFs in
// oracle/render_ref.py; this kernel makes the same float32 operations in the
// same order (built with -ffp-contract=off), so frames are bit-identical to it.
//
// Input is what a step already wrote — node_feat rows (position in columns
// 2-3, type in column 6, -1 = padding) and the packed CSR edge list — so any
// rollout slot can be rendered after the fact. One workgroup = 256 pixels of
// one frame; the frame's entities and, in chunks, its edges are staged in
// LDS; each pixel walks the discs in entity order, then the edges.
#include "gsm_device.h"

namespace gsm {

namespace {

constexpr int kRenderBlock = 256;
constexpr int kEdgeChunk = 256;

struct RenderArgs {
    const float *node_feat;
    const int64_t *edge_ptr;
    const int32_t *edge_index;
    int64_t edge_cap, n_envs;
    const int32_t *env_ids;
    int32_t E, W, H, draw_edges;
    float half_width, r_agent, r_target, r_obst;
    uint32_t *out;
};

__device__ __forceinline__ uint32_t rgba(uint32_t r, uint32_t g, uint32_t b) {
    return r | (g << 8) | (b << 16) | (255u << 24);
}

__global__ __launch_bounds__(kRenderBlock) void gsm_render_kernel(RenderArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *s_x = (float *)smem;                 // [E]
    float *s_y = s_x + a.E;                     // [E]
    int *s_t = (int *)(s_y + a.E);              // [E]
    int2 *s_e = (int2 *)(s_t + a.E + (a.E & 1)); // [kEdgeChunk] (8-byte aligned)
    __shared__ int s_nagents;
    const int f = blockIdx.y;
    const int64_t b = a.env_ids[f];
    const int64_t npix = (int64_t)a.W * a.H;
    const int64_t pix = (int64_t)blockIdx.x * kRenderBlock + threadIdx.x;
    const bool env_ok = b >= 0 && b < a.n_envs;
    if (threadIdx.x == 0) s_nagents = 0;
    __syncthreads();
    int my_agents = 0;
    if (env_ok) {
        const float *rows = a.node_feat + b * a.E * 7;
        for (int e = threadIdx.x; e < a.E; e += kRenderBlock) {
            s_x[e] = rows[e * 7 + 2];
            s_y[e] = rows[e * 7 + 3];
            const int t = (int)rows[e * 7 + 6];
            s_t[e] = t;
            my_agents += t == 0 ? 1 : 0;
        }
    }
    if (my_agents) atomicAdd(&s_nagents, my_agents);
    __syncthreads();
    // camera: [-L, L]^2, L = half_width or sqrt(n_agents / 3)
    const float L = a.half_width > 0.0f ? a.half_width : sqrtf((float)s_nagents / 3.0f);
    const float sx = (2.0f * L) / (float)a.W, sy = (2.0f * L) / (float)a.H;
    const int px = (int)(pix % a.W), py = (int)(pix / a.W);
    const float x = ((float)px + 0.5f) * sx - L;
    const float y = L - ((float)py + 0.5f) * sy;
    uint32_t color = rgba(255, 255, 255);
    if (env_ok) {
        const float rad[3] = {a.r_agent, a.r_target, a.r_obst};
        const uint32_t fill[3] = {rgba(159, 159, 223), rgba(64, 64, 64), rgba(128, 128, 128)};
        const uint32_t ring[3] = {rgba(127, 127, 191), rgba(48, 48, 48), rgba(96, 96, 96)};
        float r2[3], ri2[3];
        for (int k = 0; k < 3; ++k) {
            const float ri = fmaxf(rad[k] - 1.5f * sx, 0.0f);
            r2[k] = rad[k] * rad[k];
            ri2[k] = ri * ri;
        }
        for (int e = 0; e < a.E; ++e) {
            const int k = s_t[e];
            if (k < 0 || k > 2) continue;
            const float dx = x - s_x[e], dy = y - s_y[e];
            const float d2 = dx * dx + dy * dy;
            if (d2 <= r2[k]) color = d2 > ri2[k] ? ring[k] : fill[k];
        }
    }
    if (env_ok && a.draw_edges) {
        const int64_t lo = a.edge_ptr[b], hi = min(a.edge_ptr[b + 1], a.edge_cap);
        const int32_t g0 = (int32_t)(b * a.E);
        const float w = 0.5f * sx;
        const float w2 = w * w;
        bool on = false;
        for (int64_t c0 = lo; c0 < hi; c0 += kEdgeChunk) {
            const int n = (int)min((int64_t)kEdgeChunk, hi - c0);
            __syncthreads();
            if ((int)threadIdx.x < n) {
                s_e[threadIdx.x] = make_int2(a.edge_index[c0 + threadIdx.x] - g0,
                                             a.edge_index[a.edge_cap + c0 + threadIdx.x] - g0);
            }
            __syncthreads();
            for (int i = 0; i < n; ++i) {
                const int2 ed = s_e[i];
                if (ed.x >= ed.y || ed.x < 0 || ed.y >= a.E) continue;   // each undirected edge once
                const float ax = s_x[ed.x], ay = s_y[ed.x], bx = s_x[ed.y], by = s_y[ed.y];
                const float abx = bx - ax, aby = by - ay;
                const float apx = x - ax, apy = y - ay;
                const float t = apx * abx + apy * aby;
                const float l2 = abx * abx + aby * aby;
                bool hit;
                if (t <= 0.0f) {
                    hit = apx * apx + apy * apy <= w2;
                } else if (t >= l2) {
                    const float bpx = x - bx, bpy = y - by;
                    hit = bpx * bpx + bpy * bpy <= w2;
                } else {
                    const float cr = apx * aby - apy * abx;
                    hit = cr * cr <= w2 * l2;
                }
                on = on || hit;
            }
        }
        if (on) color = rgba(0, 0, 0);
    }
    if (pix < npix) a.out[(int64_t)f * npix + pix] = color;
}

}  // namespace

hipError_t launch_render(const float *node_feat, int64_t n_envs, int32_t n_entities, const int64_t *edge_ptr,
                         const int32_t *edge_index, int64_t edge_capacity, const int32_t *env_ids,
                         int32_t n_frames, float half_width, float r_agent, float r_target, float r_obst,
                         int32_t width, int32_t height, int32_t draw_edges, uint8_t *rgba_out, hipStream_t s) {
    RenderArgs a;
    a.node_feat = node_feat;
    a.edge_ptr = edge_ptr;
    a.edge_index = edge_index;
    a.edge_cap = edge_capacity;
    a.n_envs = n_envs;
    a.env_ids = env_ids;
    a.E = n_entities;
    a.W = width;
    a.H = height;
    a.draw_edges = draw_edges;
    a.half_width = half_width;
    a.r_agent = r_agent;
    a.r_target = r_target;
    a.r_obst = r_obst;
    a.out = (uint32_t *)rgba_out;
    const int64_t npix = (int64_t)width * height;
    const dim3 grid((unsigned)((npix + kRenderBlock - 1) / kRenderBlock), (unsigned)n_frames);
    const size_t lds = (size_t)(3 * n_entities + 1) * 4 + 8 + kEdgeChunk * sizeof(int2);
    (void)hipGetLastError();
    gsm_render_kernel<<<grid, kRenderBlock, lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace gsm
