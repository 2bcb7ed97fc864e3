// gsm_gnn.hip — graph-attention message passing over the env graph
// (the GNN encoder that consumes node_feat /
// edge_index; reference: gsmarl/algorithms, SOURCES.txt:8, torch-geometric
// 2.3.1 requirements.txt:119 — the InforMARL lineage uses PyG TransformerConv).
//
// The dense projections (q = W_q x, k = W_k x, v = W_v x, skip = W_r x) are
// GEMMs and stay on hipBLASLt (torch.matmul). This kernel is the part that is
// a gather / segmented softmax / scatter over the graph, for target node i with
// source neighbours j (CSR rows: row_ptr / col), per head h:
//
//   e_ij   = w_ij * w_e[h]                    (edge feature, edge_dim = 1)
//   s_ij   = scale * <q_i[h], k_j[h] + e_ij>
//   a_ij   = softmax_j(s_ij)                  (over the row; empty row -> 0)
//   out_i[h] = sum_j a_ij (v_j[h] + e_ij)  (+ skip_i[h])
//
// Layout: q, k, v, skip, out are [n_nodes][H*C] f32 (head-major channels).
// Mapping: four channels per lane (16-byte gathers of the k_j / v_j rows)
// when the heads allow, so a node takes pow2 >= H*C/4 lanes and a wave works
// on 64/that nodes at once (memory-level parallelism for the dependent
// row_ptr -> col -> k/v loads); a head's lanes reduce the score with xor
// shuffles; an online softmax keeps (max, denominator, accumulator) in
// registers while the row's edges stream through (the next edge's index one
// iteration ahead), so every k_j / v_j row is read once per edge.
#include "gsm_device.h"

namespace gsm {

template <int kVec>
struct VecT;
template <>
struct VecT<1> {
    using T = float;
    static __device__ __forceinline__ float get(const T &x, int) { return x; }
    static __device__ __forceinline__ void set(T &x, int, float v) { x = v; }
};
template <>
struct VecT<4> {
    using T = float4;
    static __device__ __forceinline__ float get(const T &x, int i) {
        return i == 0 ? x.x : (i == 1 ? x.y : (i == 2 ? x.z : x.w));
    }
    static __device__ __forceinline__ void set(T &x, int i, float v) {
        if (i == 0) x.x = v;
        else if (i == 1) x.y = v;
        else if (i == 2) x.z = v;
        else x.w = v;
    }
};

// kLP lanes per node, kVec consecutive channels per lane (a lane's channels
// belong to one head: C % kVec == 0); 64 / kLP nodes per wave.
template <int kLP, int kVec>
__global__ __launch_bounds__(256) void gsm_attn_aggregate_kernel(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ edge_w, const float *__restrict__ w_e, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const float *__restrict__ skip, int64_t n_nodes, int HC, int C,
    float scale, float *__restrict__ out) {
    using V = VecT<kVec>;
    using T = typename V::T;
    constexpr int kNPW = kWave / kLP;                       // nodes per wave
    const int lane = threadIdx.x & 63;
    const int sub = lane / kLP, ch = (lane % kLP) * kVec;
    const int64_t node = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kNPW + sub;
    const bool live = node < n_nodes && ch < HC;
    const int64_t nd = node < n_nodes ? node : 0;
    const int lanes_per_head = C / kVec;                    // power of two
    T qi, we, acc;
    for (int i = 0; i < kVec; ++i) {
        V::set(qi, i, 0.0f);
        V::set(we, i, 0.0f);
        V::set(acc, i, 0.0f);
    }
    if (live) {
        qi = *(const T *)(q + nd * HC + ch);
        if (w_e) we = *(const T *)(w_e + ch);
    }
    const int64_t r0 = node < n_nodes ? row_ptr[nd] : 0, r1 = node < n_nodes ? row_ptr[nd + 1] : 0;
    const int deg = (int)(r1 - r0);
    int wdeg = deg;                                          // the wave runs its longest row
#pragma unroll
    for (int o = kLP; o < kWave; o <<= 1) wdeg = max(wdeg, __shfl_xor(wdeg, o));
    float mx = -__builtin_inff(), den = 0.0f;
    // next edge's source and weight fetched one iteration ahead
    int64_t jn = (live && deg > 0) ? col[r0] : 0;
    float wn = (live && deg > 0 && edge_w) ? edge_w[r0] : 0.0f;
    for (int t = 0; t < wdeg; ++t) {
        const bool on = live && t < deg;
        const int64_t j = jn;
        const float w = wn;
        if (live && t + 1 < deg) {
            jn = col[r0 + t + 1];
            if (edge_w) wn = edge_w[r0 + t + 1];
        }
        T kj, vj;
        for (int i = 0; i < kVec; ++i) {
            V::set(kj, i, 0.0f);
            V::set(vj, i, 0.0f);
        }
        if (on) {
            kj = *(const T *)(k + j * HC + ch);
            vj = *(const T *)(v + j * HC + ch);
        }
        float sc = 0.0f;
#pragma unroll
        for (int i = 0; i < kVec; ++i) sc += V::get(qi, i) * (V::get(kj, i) + w * V::get(we, i));
#pragma unroll
        for (int o = 1; o < kLP; o <<= 1)
            if (o < lanes_per_head) sc += __shfl_xor(sc, o);   // sum over the head's lanes
        sc *= scale;
        if (on) {
            const float m2 = fmaxf(mx, sc);
            const float a = __expf(mx - m2), b = __expf(sc - m2);
            den = den * a + b;
#pragma unroll
            for (int i = 0; i < kVec; ++i)
                V::set(acc, i, V::get(acc, i) * a + b * (V::get(vj, i) + w * V::get(we, i)));
            mx = m2;
        }
    }
    if (live) {
        const float inv = den > 0.0f ? 1.0f / den : 0.0f;
        T r;
        T sk;
        if (skip) sk = *(const T *)(skip + nd * HC + ch);
#pragma unroll
        for (int i = 0; i < kVec; ++i)
            V::set(r, i, V::get(acc, i) * inv + (skip ? V::get(sk, i) : 0.0f));
        *(T *)(out + nd * HC + ch) = r;
    }
}

hipError_t launch_attn_aggregate(const float *q, const float *k, const float *v, const float *edge_w,
                                 const float *w_e, const int64_t *row_ptr, const int32_t *col,
                                 const float *skip, int64_t n_nodes, int HC, int C, float scale, float *out,
                                 hipStream_t s) {
    // four channels per lane (16-byte gathers) when every head spans whole
    // lanes and the rows are 16-byte aligned; one channel per lane otherwise
    const bool vec4 = C % 4 == 0 && HC % 4 == 0 && ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v |
                                                     (uintptr_t)out | (uintptr_t)(skip ? skip : out) |
                                                     (uintptr_t)(w_e ? w_e : out)) % 16 == 0;
    const int vec = vec4 ? 4 : 1;
    int lp = 1;
    while (lp * vec < HC) lp <<= 1;
    if (lp > kWave) return hipErrorInvalidValue;
    const int npw = kWave / lp;
    const int64_t waves = (n_nodes + npw - 1) / npw;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    (void)hipGetLastError();
#define GSM_ATTN(LP, VEC)                                                                                \
    gsm_attn_aggregate_kernel<LP, VEC><<<blocks, 256, 0, s>>>(q, k, v, edge_w, w_e, row_ptr, col, skip, \
                                                              n_nodes, HC, C, scale, out)
    if (vec4) {
        switch (lp) {
            case 1: GSM_ATTN(1, 4); break;
            case 2: GSM_ATTN(2, 4); break;
            case 4: GSM_ATTN(4, 4); break;
            case 8: GSM_ATTN(8, 4); break;
            case 16: GSM_ATTN(16, 4); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (lp) {
            case 1: GSM_ATTN(1, 1); break;
            case 2: GSM_ATTN(2, 1); break;
            case 4: GSM_ATTN(4, 1); break;
            case 8: GSM_ATTN(8, 1); break;
            case 16: GSM_ATTN(16, 1); break;
            case 32: GSM_ATTN(32, 1); break;
            case 64: GSM_ATTN(64, 1); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef GSM_ATTN
    return hipGetLastError();
}

}  // namespace gsm
