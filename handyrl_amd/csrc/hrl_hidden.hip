// hrl_hidden.hip — the recurrent state plumbing of forward_prediction (handyrl/train.py:155-174).
//
// For a recurrent net the learner unrolls T steps; every step it masks the
// state by the observation mask, sums it over players (turn-based training
// without opponent observation) and, after the net's step, mixes the new
// state in:
//
//   h_in  = sum_p h[:, p] * m[:, p]            (or h * m, one row per player)
//   h'    = h * (1 - m) + nh * m               (nh broadcast over players if it has one)
//
// GeisterNet carries 6 state tensors, so in torch that is ~36 elementwise
// launches forward and more backward per step.  Here the state of all
// tensors lives in ONE leaf-major buffer (leaf l: (B, P, F_l) contiguous at
// offset off_l) and each operation and its adjoint is one launch over all
// leaves.  Arithmetic is torch's: (1 - m) first, products, then the sum
// (p ascending; P = 2 in every turn-based env, where it matches torch.sum).
// Elementwise, HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kMaxLeaves = 16;
constexpr int kThreads = 256;

// Leaf table.  Launch geometry: blockIdx.z = leaf, blockIdx.y strides over the
// row index (b, or (b, p)), threads run along the leaf's contiguous features in
// float4 (all F % 4 == 0, the usual board-state case) or floats -- no integer
// division anywhere.
struct Leaves {
    int n;
    int F[kMaxLeaves];          // floats per (b, p) of each leaf
    int64_t off[kMaxLeaves];    // offset of leaf l in the leaf-major (B, P, F_l) state buffer
    const float *src[kMaxLeaves];
    float *dst[kMaxLeaves];
};

template <int VW>
struct V;
template <>
struct V<4> {
    using T = float4;
    static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
    static __device__ __forceinline__ T mul(T a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }
    static __device__ __forceinline__ T add(T a, T b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
};
template <>
struct V<1> {
    using T = float;
    static __device__ __forceinline__ T zero() { return 0.f; }
    static __device__ __forceinline__ T mul(T a, float s) { return a * s; }
    static __device__ __forceinline__ T add(T a, T b) { return a + b; }
};

#define HRL_LEAF_LOOP                                                                     \
    const int l = blockIdx.z;                                                             \
    const int nv = L.F[l] / VW;                                                           \
    const int v = blockIdx.x * kThreads + threadIdx.x;                                    \
    if (v >= nv) return;

// gather, summed over players: out_l[b, v] = sum_p H_l[b, p, v] * m[b, p]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_sum_kernel(const float *__restrict__ H,
                                                                     const float *__restrict__ m, int B, int P,
                                                                     Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(H + L.off[l]);
    T *out = reinterpret_cast<T *>(L.dst[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        T acc = W::mul(h[(int64_t)(b * P) * nv + v], m[b * P]);
        for (int p = 1; p < P; ++p) acc = W::add(acc, W::mul(h[(int64_t)(b * P + p) * nv + v], m[b * P + p]));
        out[(int64_t)b * nv + v] = acc;
    }
}

// gather, one row per player: out_l[bp, v] = H_l[bp, v] * m[bp]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_keep_kernel(const float *__restrict__ H,
                                                                      const float *__restrict__ m, int BP, Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(H + L.off[l]);
    T *out = reinterpret_cast<T *>(L.dst[l]);
    for (int r = blockIdx.y; r < BP; r += gridDim.y) out[(int64_t)r * nv + v] = W::mul(h[(int64_t)r * nv + v], m[r]);
}

// adjoint of the gather: dH_l[b, p, v] = g_l[b or bp, v] * m[b, p]; a NULL g_l is a zero gradient
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_bwd_kernel(const float *__restrict__ m, int B, int P,
                                                                     int summed, Leaves L, float *__restrict__ dH) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *g = reinterpret_cast<const T *>(L.src[l]);
    T *d = reinterpret_cast<T *>(dH + L.off[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            T val = W::zero();
            if (g) val = W::mul(g[(int64_t)(summed ? b : bp) * nv + v], m[bp]);
            d[(int64_t)bp * nv + v] = val;
        }
    }
}

// update: out_l[b, p, v] = H_l[b, p, v] * (1 - m[b, p]) + nh_l[b, p or 0, v] * m[b, p]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_update_kernel(const float *__restrict__ H,
                                                                 const float *__restrict__ m, int B, int P, int Pn,
                                                                 Leaves L, float *__restrict__ out) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(H + L.off[l]);
    const T *nh = reinterpret_cast<const T *>(L.src[l]);
    T *o = reinterpret_cast<T *>(out + L.off[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            const float mv = m[bp];
            o[(int64_t)bp * nv + v] = W::add(W::mul(h[(int64_t)bp * nv + v], 1.0f - mv),
                                             W::mul(nh[(int64_t)(b * Pn + (Pn == 1 ? 0 : p)) * nv + v], mv));
        }
    }
}

// adjoint of the update: dH = dout * (1 - m); dnh = sum_p dout * m (Pn = 1) or dout * m
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_update_bwd_kernel(const float *__restrict__ dout,
                                                                     const float *__restrict__ m, int B, int P,
                                                                     int Pn, Leaves L, float *__restrict__ dH) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *g = reinterpret_cast<const T *>(dout + L.off[l]);
    T *d = reinterpret_cast<T *>(dH + L.off[l]);
    T *dn = reinterpret_cast<T *>(L.dst[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        if (Pn == 1) {
            T acc = W::mul(g[(int64_t)(b * P) * nv + v], m[b * P]);
            for (int p = 1; p < P; ++p) acc = W::add(acc, W::mul(g[(int64_t)(b * P + p) * nv + v], m[b * P + p]));
            dn[(int64_t)b * nv + v] = acc;
        }
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            const T gv = g[(int64_t)bp * nv + v];
            d[(int64_t)bp * nv + v] = W::mul(gv, 1.0f - m[bp]);
            if (Pn != 1) dn[(int64_t)bp * nv + v] = W::mul(gv, m[bp]);
        }
    }
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// leaf table; vw = 4 when every leaf allows float4 access
bool build(int n, const int64_t *F, int64_t B, int64_t P, const float *const *src, float *const *dst,
           const float *a, const float *b, Leaves &L, int &vw, int &fmax) {
    if (n < 1 || n > kMaxLeaves || B < 0 || P < 1 || B * P > (int64_t)1 << 30) return false;
    L.n = n;
    vw = aligned16(a) && aligned16(b) ? 4 : 1;
    fmax = 0;
    int64_t off = 0;
    for (int l = 0; l < n; ++l) {
        if (F[l] < 1 || F[l] > (1 << 30)) return false;
        L.F[l] = (int)F[l];
        L.off[l] = off;
        L.src[l] = src ? src[l] : nullptr;
        L.dst[l] = dst ? dst[l] : nullptr;
        if (F[l] % 4 || (off * 4) % 16 || !aligned16(L.src[l]) || !aligned16(L.dst[l])) vw = 1;
        if (F[l] > fmax) fmax = (int)F[l];
        off += B * P * F[l];
    }
    return true;
}

dim3 grid_of(int fmax, int vw, int64_t rows, int n) {
    const int nv = fmax / vw;
    const int gx = (nv + kThreads - 1) / kThreads;
    const int64_t gy = rows < 1 ? 1 : (rows > 4096 ? 4096 : rows);
    return dim3((unsigned)gx, (unsigned)gy, (unsigned)n);
}

}  // namespace

extern "C" {

int hrl_hidden_gather(const float *H, const float *mask, int64_t B, int64_t P, int nleaves, const int64_t *F,
                      int sum, float *const *out, void *stream) {
    if (!H || !mask || !F || !out) return HRL_EINVAL;
    Leaves L;
    int vw, fmax;
    if (!build(nleaves, F, B, P, nullptr, out, H, nullptr, L, vw, fmax)) return HRL_EINVAL;
    for (int l = 0; l < nleaves; ++l)
        if (!out[l]) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, sum ? B : B * P, nleaves);
    if (sum) {
        if (vw == 4) hipLaunchKernelGGL(hidden_gather_sum_kernel<4>, grid, dim3(kThreads), 0, s, H, mask, (int)B, (int)P, L);
        else hipLaunchKernelGGL(hidden_gather_sum_kernel<1>, grid, dim3(kThreads), 0, s, H, mask, (int)B, (int)P, L);
    } else {
        if (vw == 4) hipLaunchKernelGGL(hidden_gather_keep_kernel<4>, grid, dim3(kThreads), 0, s, H, mask, (int)(B * P), L);
        else hipLaunchKernelGGL(hidden_gather_keep_kernel<1>, grid, dim3(kThreads), 0, s, H, mask, (int)(B * P), L);
    }
    return status();
}

int hrl_hidden_gather_backward(const float *const *dout, const float *mask, int64_t B, int64_t P, int nleaves,
                               const int64_t *F, int sum, float *dH, void *stream) {
    if (!dout || !mask || !F || !dH) return HRL_EINVAL;
    Leaves L;
    int vw, fmax;
    if (!build(nleaves, F, B, P, dout, nullptr, dH, nullptr, L, vw, fmax)) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_gather_bwd_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, sum, L, dH);
    else hipLaunchKernelGGL(hidden_gather_bwd_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, sum, L, dH);
    return status();
}

int hrl_hidden_update(const float *H, const float *const *nh, int64_t Pn, const float *mask, int64_t B, int64_t P,
                      int nleaves, const int64_t *F, float *out, void *stream) {
    if (!H || !nh || !mask || !F || !out || (Pn != 1 && Pn != P)) return HRL_EINVAL;
    Leaves L;
    int vw, fmax;
    if (!build(nleaves, F, B, P, nh, nullptr, H, out, L, vw, fmax)) return HRL_EINVAL;
    for (int l = 0; l < nleaves; ++l)
        if (!nh[l]) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_update_kernel<4>, grid, dim3(kThreads), 0, s, H, mask, (int)B, (int)P, (int)Pn, L, out);
    else hipLaunchKernelGGL(hidden_update_kernel<1>, grid, dim3(kThreads), 0, s, H, mask, (int)B, (int)P, (int)Pn, L, out);
    return status();
}

int hrl_hidden_update_backward(const float *dout, const float *mask, int64_t B, int64_t P, int64_t Pn, int nleaves,
                               const int64_t *F, float *dH, float *const *dnh, void *stream) {
    if (!dout || !mask || !F || !dH || !dnh || (Pn != 1 && Pn != P)) return HRL_EINVAL;
    Leaves L;
    int vw, fmax;
    if (!build(nleaves, F, B, P, nullptr, dnh, dout, dH, L, vw, fmax)) return HRL_EINVAL;
    for (int l = 0; l < nleaves; ++l)
        if (!dnh[l]) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_update_bwd_kernel<4>, grid, dim3(kThreads), 0, s, dout, mask, (int)B, (int)P, (int)Pn, L, dH);
    else hipLaunchKernelGGL(hidden_update_bwd_kernel<1>, grid, dim3(kThreads), 0, s, dout, mask, (int)B, (int)P, (int)Pn, L, dH);
    return status();
}

}  // extern "C"
