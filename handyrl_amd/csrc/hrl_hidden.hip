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
// launches forward and more backward per step.  Here each operation and its
// adjoint is ONE launch over all state tensors (a table of per-tensor
// pointers).  The tensors stay separate: a state tensor whose gradient is
// None (it never reaches an output) is simply left out of the backward
// launch, preserving autograd's pruning.  Arithmetic is torch's: (1 - m) first, products, then the sum
// (p ascending; P = 2 in every turn-based env, where it matches torch.sum).
// Elementwise, HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kMaxLeaves = 16;
constexpr int kThreads = 256;

// Per-leaf table.  Launch geometry: blockIdx.z = leaf, blockIdx.y strides over
// rows (b), threads run along the leaf's contiguous features in float4 (every
// F % 4 == 0 and 16-byte aligned pointers) or floats -- no integer division.
struct Leaves {
    int n;
    int F[kMaxLeaves];
    const float *a[kMaxLeaves];   // gather: H; gather bwd: g; update: H; update bwd: dout
    const float *b[kMaxLeaves];   // update: nh
    float *c[kMaxLeaves];         // gather: out; gather bwd: dH; update: out; update bwd: dH
    float *d[kMaxLeaves];         // update bwd: dnh
    const float *e[kMaxLeaves];   // gather bwd: addend of dH; update bwd: addend of dnh (NULL: none)
    int64_t es[kMaxLeaves];       // the addend's row stride in floats (a channel slice of a wider tensor)
    const float *f[kMaxLeaves];   // update-gather bwd: addend of dnh (e: of the new state's gradient)
    int64_t fs[kMaxLeaves];
};

template <int VW>
struct V;
template <>
struct V<4> {
    using T = float4;
    static __device__ __forceinline__ T mul(T a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }
    static __device__ __forceinline__ T add(T a, T b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
};
template <>
struct V<1> {
    using T = float;
    static __device__ __forceinline__ T mul(T a, float s) { return a * s; }
    static __device__ __forceinline__ T add(T a, T b) { return a + b; }
};

#define HRL_LEAF_LOOP                                                                     \
    const int l = blockIdx.z;                                                             \
    const int nv = L.F[l] / VW;                                                           \
    const int v = blockIdx.x * kThreads + threadIdx.x;                                    \
    if (v >= nv) return;

// gather, summed over players: out[b, v] = sum_p H[b, p, v] * m[b, p]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_sum_kernel(const float *__restrict__ m, int B, int P,
                                                                     Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(L.a[l]);
    T *out = reinterpret_cast<T *>(L.c[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        T acc = W::mul(h[(int64_t)(b * P) * nv + v], m[b * P]);
        for (int p = 1; p < P; ++p) acc = W::add(acc, W::mul(h[(int64_t)(b * P + p) * nv + v], m[b * P + p]));
        out[(int64_t)b * nv + v] = acc;
    }
}

// gather, one row per player: out[bp, v] = H[bp, v] * m[bp]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_keep_kernel(const float *__restrict__ m, int BP, Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(L.a[l]);
    T *out = reinterpret_cast<T *>(L.c[l]);
    for (int r = blockIdx.y; r < BP; r += gridDim.y) out[(int64_t)r * nv + v] = W::mul(h[(int64_t)r * nv + v], m[r]);
}

// adjoint of the gather: dH[b, p, v] = g[b or bp, v] * m[b, p]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_gather_bwd_kernel(const float *__restrict__ m, int B, int P,
                                                                     int summed, Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *g = reinterpret_cast<const T *>(L.a[l]);
    const T *e = reinterpret_cast<const T *>(L.e[l]);
    T *d = reinterpret_cast<T *>(L.c[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            const T t = W::mul(g[(int64_t)(summed ? b : bp) * nv + v], m[bp]);
            // the state's other consumer's gradient (the update's keep path), summed here instead of by autograd
            d[(int64_t)bp * nv + v] = e ? W::add(e[(int64_t)bp * (L.es[l] / VW) + v], t) : t;
        }
    }
}

// update: out[b, p, v] = H[b, p, v] * (1 - m[b, p]) + nh[b, p or 0, v] * m[b, p]
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_update_kernel(const float *__restrict__ m, int B, int P, int Pn,
                                                                 Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(L.a[l]);
    const T *nh = reinterpret_cast<const T *>(L.b[l]);
    T *o = reinterpret_cast<T *>(L.c[l]);
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
__global__ __launch_bounds__(kThreads) void hidden_update_bwd_kernel(const float *__restrict__ m, int B, int P, int Pn,
                                                                     Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *g = reinterpret_cast<const T *>(L.a[l]);
    const T *e = reinterpret_cast<const T *>(L.e[l]);
    T *d = reinterpret_cast<T *>(L.c[l]);
    T *dn = reinterpret_cast<T *>(L.d[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        if (Pn == 1) {
            T acc = W::mul(g[(int64_t)(b * P) * nv + v], m[b * P]);
            for (int p = 1; p < P; ++p) acc = W::add(acc, W::mul(g[(int64_t)(b * P + p) * nv + v], m[b * P + p]));
            // the new state's other consumer's gradient (e.g. the step's output to the heads), summed here
            dn[(int64_t)b * nv + v] = e ? W::add(e[(int64_t)b * (L.es[l] / VW) + v], acc) : acc;
        }
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            const T gv = g[(int64_t)bp * nv + v];
            d[(int64_t)bp * nv + v] = W::mul(gv, 1.0f - m[bp]);
            if (Pn != 1) {
                const T t = W::mul(gv, m[bp]);
                dn[(int64_t)bp * nv + v] = e ? W::add(e[(int64_t)bp * (L.es[l] / VW) + v], t) : t;
            }
        }
    }
}

// step t's update fused with step t+1's gather (round 5): out = H (1 - m) + nh m as hidden_update_kernel, then
// the next step's input from out with mask mn as hidden_gather_sum/keep_kernel (the same float operations in the
// same order: the two launches' results bit for bit).  a = H, b = nh, c = out, d = the gathered input.
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_update_gather_kernel(const float *__restrict__ m,
                                                                        const float *__restrict__ mn, int B, int P,
                                                                        int Pn, int summed, Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *h = reinterpret_cast<const T *>(L.a[l]);
    const T *nh = reinterpret_cast<const T *>(L.b[l]);
    T *o = reinterpret_cast<T *>(L.c[l]);
    T *go = reinterpret_cast<T *>(L.d[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        T acc;
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            const float mv = m[bp];
            const T ov = W::add(W::mul(h[(int64_t)bp * nv + v], 1.0f - mv),
                                W::mul(nh[(int64_t)(b * Pn + (Pn == 1 ? 0 : p)) * nv + v], mv));
            o[(int64_t)bp * nv + v] = ov;
            const T t = W::mul(ov, mn[bp]);
            if (summed) acc = p == 0 ? t : W::add(acc, t);
            else go[(int64_t)bp * nv + v] = t;
        }
        if (summed) go[(int64_t)b * nv + v] = acc;
    }
}

// its adjoint: the gather's (dout = g m_next [+ e, the new state's other gradient]) then the update's (dH = dout
// (1 - m); dnh = sum_p dout m (Pn = 1) or dout m [+ f, the step output's gradient]) -- the two adjoint launches'
// operations in their order.  a = the gathered input's gradient (NULL: zero), c = dH, d = dnh.
template <int VW>
__global__ __launch_bounds__(kThreads) void hidden_update_gather_bwd_kernel(const float *__restrict__ m,
                                                                            const float *__restrict__ mn, int B,
                                                                            int P, int Pn, int summed, Leaves L) {
    using W = V<VW>;
    using T = typename W::T;
    HRL_LEAF_LOOP
    const T *g = reinterpret_cast<const T *>(L.a[l]);
    const T *e = reinterpret_cast<const T *>(L.e[l]);
    const T *fa = reinterpret_cast<const T *>(L.f[l]);
    T *d = reinterpret_cast<T *>(L.c[l]);
    T *dn = reinterpret_cast<T *>(L.d[l]);
    for (int b = blockIdx.y; b < B; b += gridDim.y) {
        T acc;
        for (int p = 0; p < P; ++p) {
            const int bp = b * P + p;
            T go;
            if (g) {
                const T t = W::mul(g[(int64_t)(summed ? b : bp) * nv + v], mn[bp]);
                go = e ? W::add(e[(int64_t)bp * (L.es[l] / VW) + v], t) : t;
            } else {
                go = e[(int64_t)bp * (L.es[l] / VW) + v];
            }
            d[(int64_t)bp * nv + v] = W::mul(go, 1.0f - m[bp]);
            const T t = W::mul(go, m[bp]);
            if (Pn == 1) {
                acc = p == 0 ? t : W::add(acc, t);
            } else {
                dn[(int64_t)bp * nv + v] = fa ? W::add(fa[(int64_t)bp * (L.fs[l] / VW) + v], t) : t;
            }
        }
        if (Pn == 1) dn[(int64_t)b * nv + v] = fa ? W::add(fa[(int64_t)b * (L.fs[l] / VW) + v], acc) : acc;
    }
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// fill the table from up to four pointer arrays (NULL arrays are skipped); false on a bad argument
bool build(int n, const int64_t *F, int64_t B, int64_t P, const float *const *a, const float *const *b,
           float *const *c, float *const *d, Leaves &L, int &vw, int &fmax) {
    if (n < 1 || n > kMaxLeaves || B < 0 || P < 1 || B * P > ((int64_t)1 << 30) || !F || !a || !c) return false;
    L.n = n;
    vw = 4;
    fmax = 0;
    for (int l = 0; l < n; ++l) {
        if (F[l] < 1 || F[l] > (1 << 28) || !a[l] || !c[l] || (b && !b[l]) || (d && !d[l])) return false;
        L.F[l] = (int)F[l];
        L.a[l] = a[l];
        L.b[l] = b ? b[l] : nullptr;
        L.c[l] = c[l];
        L.d[l] = d ? d[l] : nullptr;
        L.e[l] = nullptr;
        L.es[l] = F[l];
        L.f[l] = nullptr;
        L.fs[l] = F[l];
        if (F[l] % 4 || !aligned16(L.a[l]) || !aligned16(L.b[l]) || !aligned16(L.c[l]) || !aligned16(L.d[l])) vw = 1;
        if (F[l] > fmax) fmax = (int)F[l];
    }
    return true;
}

dim3 grid_of(int fmax, int vw, int64_t rows, int n) {
    const int nv = fmax / vw;
    const int gx = (nv + kThreads - 1) / kThreads;
    const int64_t gy = rows < 1 ? 1 : (rows > 4096 ? 4096 : rows);
    return dim3((unsigned)gx, (unsigned)gy, (unsigned)n);
}

// the addend table (NULL, or per leaf NULL / rows of the output's row length F, `strides` floats apart (NULL:
// F)): false on a stride shorter than the row
bool set_addend(Leaves &L, const float *const *add, const int64_t *strides, int &vw) {
    if (!add) return true;
    for (int l = 0; l < L.n; ++l) {
        L.e[l] = add[l];
        const int64_t st = strides ? strides[l] : L.F[l];
        if (add[l] && (st < L.F[l] || st > ((int64_t)1 << 31))) return false;
        L.es[l] = st;
        if (!aligned16(add[l]) || st % 4) vw = 1;
    }
    return true;
}

}  // namespace

extern "C" {

int hrl_hidden_gather(const float *const *H, const float *mask, int64_t B, int64_t P, int nleaves, const int64_t *F,
                      int sum, float *const *out, void *stream) {
    Leaves L;
    int vw, fmax;
    if (!mask || !build(nleaves, F, B, P, H, nullptr, out, nullptr, L, vw, fmax)) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, sum ? B : B * P, nleaves);
    if (sum) {
        if (vw == 4) hipLaunchKernelGGL(hidden_gather_sum_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, L);
        else hipLaunchKernelGGL(hidden_gather_sum_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, L);
    } else {
        if (vw == 4) hipLaunchKernelGGL(hidden_gather_keep_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)(B * P), L);
        else hipLaunchKernelGGL(hidden_gather_keep_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)(B * P), L);
    }
    return status();
}

int hrl_hidden_gather_backward(const float *const *dout, const float *mask, int64_t B, int64_t P, int nleaves,
                               const int64_t *F, int sum, float *const *dH, void *stream) {
    return hrl_hidden_gather_backward_add(dout, mask, B, P, nleaves, F, sum, nullptr, nullptr, dH, stream);
}

int hrl_hidden_gather_backward_add(const float *const *dout, const float *mask, int64_t B, int64_t P, int nleaves,
                                   const int64_t *F, int sum, const float *const *addend,
                                   const int64_t *addend_strides, float *const *dH, void *stream) {
    Leaves L;
    int vw, fmax;
    if (!mask || !build(nleaves, F, B, P, dout, nullptr, dH, nullptr, L, vw, fmax) || !set_addend(L, addend, addend_strides, vw))
        return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_gather_bwd_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, sum, L);
    else hipLaunchKernelGGL(hidden_gather_bwd_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, sum, L);
    return status();
}

int hrl_hidden_update(const float *const *H, const float *const *nh, int64_t Pn, const float *mask, int64_t B,
                      int64_t P, int nleaves, const int64_t *F, float *const *out, void *stream) {
    Leaves L;
    int vw, fmax;
    if (!mask || !nh || (Pn != 1 && Pn != P)) return HRL_EINVAL;
    if (!build(nleaves, F, B, P, H, nh, out, nullptr, L, vw, fmax)) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_update_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, (int)Pn, L);
    else hipLaunchKernelGGL(hidden_update_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, (int)Pn, L);
    return status();
}

int hrl_hidden_update_backward(const float *const *dout, const float *mask, int64_t B, int64_t P, int64_t Pn,
                               int nleaves, const int64_t *F, float *const *dH, float *const *dnh, void *stream) {
    return hrl_hidden_update_backward_add(dout, mask, B, P, Pn, nleaves, F, nullptr, nullptr, dH, dnh, stream);
}

int hrl_hidden_update_backward_add(const float *const *dout, const float *mask, int64_t B, int64_t P, int64_t Pn,
                                   int nleaves, const int64_t *F, const float *const *addend,
                                   const int64_t *addend_strides, float *const *dH, float *const *dnh,
                                   void *stream) {
    Leaves L;
    int vw, fmax;
    if (!mask || !dnh || (Pn != 1 && Pn != P)) return HRL_EINVAL;
    if (!build(nleaves, F, B, P, dout, nullptr, dH, dnh, L, vw, fmax) || !set_addend(L, addend, addend_strides, vw))
        return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4) hipLaunchKernelGGL(hidden_update_bwd_kernel<4>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, (int)Pn, L);
    else hipLaunchKernelGGL(hidden_update_bwd_kernel<1>, grid, dim3(kThreads), 0, s, mask, (int)B, (int)P, (int)Pn, L);
    return status();
}

int hrl_hidden_update_gather(const float *const *H, const float *const *nh, int64_t Pn, const float *mask,
                             const float *mask_next, int64_t B, int64_t P, int nleaves, const int64_t *F, int sum,
                             float *const *out, float *const *gathered, void *stream) {
    Leaves L;
    int vw, fmax;
    if (!mask || !mask_next || !nh || !gathered || (Pn != 1 && Pn != P)) return HRL_EINVAL;
    if (!build(nleaves, F, B, P, H, nh, out, gathered, L, vw, fmax)) return HRL_EINVAL;
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4)
        hipLaunchKernelGGL(hidden_update_gather_kernel<4>, grid, dim3(kThreads), 0, s, mask, mask_next, (int)B, (int)P,
                           (int)Pn, sum, L);
    else
        hipLaunchKernelGGL(hidden_update_gather_kernel<1>, grid, dim3(kThreads), 0, s, mask, mask_next, (int)B, (int)P,
                           (int)Pn, sum, L);
    return status();
}

int hrl_hidden_update_gather_backward(const float *const *dgathered, const float *mask, const float *mask_next,
                                      int64_t B, int64_t P, int64_t Pn, int nleaves, const int64_t *F, int sum,
                                      const float *const *dstate, const int64_t *dstate_strides,
                                      const float *const *dout_add, const int64_t *dout_add_strides,
                                      float *const *dH, float *const *dnh, void *stream) {
    if (!mask || !mask_next || !dgathered || !dnh || (Pn != 1 && Pn != P) || nleaves < 1 || nleaves > kMaxLeaves)
        return HRL_EINVAL;
    // a leaf's gathered-input gradient may be NULL (zero) when its new-state gradient is given
    const float *a[kMaxLeaves];
    for (int l = 0; l < nleaves; ++l) {
        if (!dgathered[l] && !(dstate && dstate[l])) return HRL_EINVAL;
        a[l] = dgathered[l] ? dgathered[l] : dnh[l];   // placeholder for build's check; reset below
    }
    Leaves L;
    int vw, fmax;
    if (!build(nleaves, F, B, P, a, nullptr, dH, dnh, L, vw, fmax) || !set_addend(L, dstate, dstate_strides, vw))
        return HRL_EINVAL;
    for (int l = 0; l < nleaves; ++l) {
        L.a[l] = dgathered[l];
        if (dout_add) {
            const int64_t st = dout_add_strides ? dout_add_strides[l] : L.F[l];
            if (dout_add[l] && (st < L.F[l] || st > ((int64_t)1 << 31))) return HRL_EINVAL;
            L.f[l] = dout_add[l];
            L.fs[l] = st;
            if (!aligned16(dout_add[l]) || st % 4) vw = 1;
        }
    }
    if (B == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid = grid_of(fmax, vw, B, nleaves);
    if (vw == 4)
        hipLaunchKernelGGL(hidden_update_gather_bwd_kernel<4>, grid, dim3(kThreads), 0, s, mask, mask_next, (int)B,
                           (int)P, (int)Pn, sum, L);
    else
        hipLaunchKernelGGL(hidden_update_gather_bwd_kernel<1>, grid, dim3(kThreads), 0, s, mask, mask_next, (int)B,
                           (int)P, (int)Pn, sum, L);
    return status();
}

}  // extern "C"
