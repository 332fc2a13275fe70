// hrl_lstm.hip — fused ConvLSTM cell gates (GeisterNet DRC, handyrl/envs/geister.py:48-63).
//
// The cell's convolution produces the 4*H gate pre-activations per board cell
// in the channel order i, f, o, g.  Torch runs the rest as ~9 elementwise
// launches forward and ~15 backward per cell, and GeisterNet applies 9 cells
// per time step (3 layers x 3 repeats), so a T=16 learner step spends most of
// its time in launch-bound elementwise kernels.  Here each direction is ONE
// pass over the cell's tensors:
//
//   forward   z = zx + zh                      (x half and h half of the conv)
//             i, f, o = sigmoid(z_i, z_f, z_o); g = tanh(z_g)
//             c' = f*c + i*g;  h' = o*tanh(c')  -> h', c', saved gates (i,f,o,g)
//   backward  tc = tanh(c');  dct = dc' + dh*o*(1-tc^2)
//             dz = (dct*g*i(1-i), dct*c*f(1-f), dh*tc*o(1-o), dct*i*(1-g^2)); dc = dct*f
//
// zx may be a channel slice of a wider tensor (the x halves of all layers are
// computed by one convolution): its per-sample stride is a parameter.  HBM
// traffic per cell and sample: forward reads 8H+H and writes 2H+4H board
// planes, backward reads 4H+3H (+dh, dc') and writes 4H+H.  Bandwidth-bound
// elementwise work, float4 along the board cells when HW % 4 == 0.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

template <int VW>
struct Vec;
template <>
struct Vec<4> {
    using T = float4;
};
template <>
struct Vec<1> {
    using T = float;
};

template <int VW>
__device__ __forceinline__ typename Vec<VW>::T ld(const float *p) {
    return *reinterpret_cast<const typename Vec<VW>::T *>(p);
}
template <int VW>
__device__ __forceinline__ void st(float *p, const typename Vec<VW>::T &v) {
    *reinterpret_cast<typename Vec<VW>::T *>(p) = v;
}
template <int VW>
__device__ __forceinline__ float get(const typename Vec<VW>::T &v, int j);
template <>
__device__ __forceinline__ float get<4>(const float4 &v, int j) {
    return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
template <>
__device__ __forceinline__ float get<1>(const float &v, int) { return v; }
template <int VW>
__device__ __forceinline__ void put(typename Vec<VW>::T &v, int j, float x);
template <>
__device__ __forceinline__ void put<4>(float4 &v, int j, float x) {
    if (j == 0) v.x = x;
    else if (j == 1) v.y = x;
    else if (j == 2) v.z = x;
    else v.w = x;
}
template <>
__device__ __forceinline__ void put<1>(float &v, int, float x) { v = x; }

struct Geo {
    int64_t N;
    int H, HW, nq;          // nq = HW / VW vectors per channel plane
    int64_t zx_stride;      // floats between samples of zx
    const float *bias;      // (bias_rows, 4H) added to zx before zh, or NULL
    int bias_rows;          // sample n uses bias row n % bias_rows (stacked layers)
};

template <int VW>
__global__ void lstm_fwd_kernel(const float *__restrict__ zx, const float *__restrict__ zh,
                                const float *__restrict__ c, Geo g, float *__restrict__ h_out,
                                float *__restrict__ c_out, float *__restrict__ gates) {
    using V = typename Vec<VW>::T;
    const int64_t total = g.N * g.H * g.nq;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(e % g.nq);
        const int64_t nc = e / g.nq;
        const int ch = (int)(nc % g.H);
        const int64_t n = nc / g.H;
        const int64_t plane = (int64_t)g.HW;
        const int64_t zoff = n * 4 * g.H * plane + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t xoff = n * g.zx_stride + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t soff = nc * plane + (int64_t)q * VW;
        const int64_t gstep = (int64_t)g.H * plane;
        V zi = ld<VW>(zh + zoff), zf = ld<VW>(zh + zoff + gstep), zo = ld<VW>(zh + zoff + 2 * gstep),
          zg = ld<VW>(zh + zoff + 3 * gstep);
        V xi = zi, xf = zf, xo = zo, xg = zg;
        if (zx) {
            xi = ld<VW>(zx + xoff);
            xf = ld<VW>(zx + xoff + gstep);
            xo = ld<VW>(zx + xoff + 2 * gstep);
            xg = ld<VW>(zx + xoff + 3 * gstep);
        }
        float bi = 0.f, bf = 0.f, bo = 0.f, bg = 0.f;
        if (g.bias) {   // the x half's conv bias, added as the biased convolution would: (zx + b) + zh
            const float *b = g.bias + (n % g.bias_rows) * 4 * g.H + ch;
            bi = b[0];
            bf = b[g.H];
            bo = b[2 * g.H];
            bg = b[3 * g.H];
        }
        const V cv = ld<VW>(c + soff);
        V gi, gf, go, gg, cn, hn;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            float a_i = get<VW>(zi, j), a_f = get<VW>(zf, j), a_o = get<VW>(zo, j), a_g = get<VW>(zg, j);
            if (zx && g.bias) {
                a_i = (get<VW>(xi, j) + bi) + a_i;
                a_f = (get<VW>(xf, j) + bf) + a_f;
                a_o = (get<VW>(xo, j) + bo) + a_o;
                a_g = (get<VW>(xg, j) + bg) + a_g;
            } else if (zx) {
                a_i = get<VW>(xi, j) + a_i;
                a_f = get<VW>(xf, j) + a_f;
                a_o = get<VW>(xo, j) + a_o;
                a_g = get<VW>(xg, j) + a_g;
            }
            const float si = sigm(a_i), sf = sigm(a_f), so = sigm(a_o), tg = tanhf(a_g);
            const float fc = sf * get<VW>(cv, j);
            const float ig = si * tg;
            const float cc = fc + ig;
            put<VW>(gi, j, si);
            put<VW>(gf, j, sf);
            put<VW>(go, j, so);
            put<VW>(gg, j, tg);
            put<VW>(cn, j, cc);
            put<VW>(hn, j, so * tanhf(cc));
        }
        if (gates) {   // NULL in inference: nothing to save for a backward
            st<VW>(gates + zoff, gi);
            st<VW>(gates + zoff + gstep, gf);
            st<VW>(gates + zoff + 2 * gstep, go);
            st<VW>(gates + zoff + 3 * gstep, gg);
        }
        st<VW>(c_out + soff, cn);
        st<VW>(h_out + soff, hn);
    }
}

// The layers of one DRC repeat in one launch (hrl_lstm_gates_forward_grouped): layer l's zh is a channel slice of
// one grouped convolution's output (per-sample stride zhs), its zx, c and outputs have their own pointers.  Each
// element runs lstm_fwd_kernel's float operations (z = zx + zh), so the outputs equal L separate launches.
constexpr int kMaxLayers = 4;
struct LayerTable {
    const float *zx[kMaxLayers];
    int64_t zxs[kMaxLayers];
    const float *c[kMaxLayers];
    float *h_out[kMaxLayers], *c_out[kMaxLayers], *gates[kMaxLayers];
};

template <int VW>
__global__ void lstm_fwd_grouped_kernel(const float *__restrict__ zh, int64_t zhs, LayerTable t, int L, Geo g) {
    using V = typename Vec<VW>::T;
    const int64_t per = g.N * g.H * g.nq;
    const int64_t total = per * L;
    for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e0 < total;
         e0 += (int64_t)gridDim.x * blockDim.x) {
        const int l = (int)(e0 / per);
        const int64_t e = e0 - (int64_t)l * per;
        const int q = (int)(e % g.nq);
        const int64_t nc = e / g.nq;
        const int ch = (int)(nc % g.H);
        const int64_t n = nc / g.H;
        const int64_t plane = (int64_t)g.HW;
        const int64_t gstep = (int64_t)g.H * plane;
        const int64_t hoff = n * zhs + (int64_t)l * 4 * gstep + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t zoff = n * 4 * gstep + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t xoff = n * t.zxs[l] + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t soff = nc * plane + (int64_t)q * VW;
        const V zi = ld<VW>(zh + hoff), zf = ld<VW>(zh + hoff + gstep), zo = ld<VW>(zh + hoff + 2 * gstep),
                zg = ld<VW>(zh + hoff + 3 * gstep);
        const float *zx = t.zx[l];
        const V xi = ld<VW>(zx + xoff), xf = ld<VW>(zx + xoff + gstep), xo = ld<VW>(zx + xoff + 2 * gstep),
                xg = ld<VW>(zx + xoff + 3 * gstep);
        const V cv = ld<VW>(t.c[l] + soff);
        V gi, gf, go, gg, cn, hn;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const float a_i = get<VW>(xi, j) + get<VW>(zi, j), a_f = get<VW>(xf, j) + get<VW>(zf, j),
                        a_o = get<VW>(xo, j) + get<VW>(zo, j), a_g = get<VW>(xg, j) + get<VW>(zg, j);
            const float si = sigm(a_i), sf = sigm(a_f), so = sigm(a_o), tg = tanhf(a_g);
            const float fc = sf * get<VW>(cv, j);
            const float ig = si * tg;
            const float cc = fc + ig;
            put<VW>(gi, j, si);
            put<VW>(gf, j, sf);
            put<VW>(go, j, so);
            put<VW>(gg, j, tg);
            put<VW>(cn, j, cc);
            put<VW>(hn, j, so * tanhf(cc));
        }
        if (float *gates = t.gates[l]) {
            st<VW>(gates + zoff, gi);
            st<VW>(gates + zoff + gstep, gf);
            st<VW>(gates + zoff + 2 * gstep, go);
            st<VW>(gates + zoff + 3 * gstep, gg);
        }
        st<VW>(t.c_out[l] + soff, cn);
        st<VW>(t.h_out[l] + soff, hn);
    }
}

template <int VW>
__global__ void lstm_bwd_kernel(const float *__restrict__ gates, const float *__restrict__ c,
                                const float *__restrict__ c_out, const float *__restrict__ dh,
                                const float *__restrict__ dc_out, Geo g, float *__restrict__ dz,
                                float *__restrict__ dc) {
    using V = typename Vec<VW>::T;
    const int64_t total = g.N * g.H * g.nq;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(e % g.nq);
        const int64_t nc = e / g.nq;
        const int ch = (int)(nc % g.H);
        const int64_t n = nc / g.H;
        const int64_t plane = (int64_t)g.HW;
        const int64_t zoff = n * 4 * g.H * plane + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t soff = nc * plane + (int64_t)q * VW;
        const int64_t gstep = (int64_t)g.H * plane;
        const V gi = ld<VW>(gates + zoff), gf = ld<VW>(gates + zoff + gstep), go = ld<VW>(gates + zoff + 2 * gstep),
                gg = ld<VW>(gates + zoff + 3 * gstep);
        const V cv = ld<VW>(c + soff), cn = ld<VW>(c_out + soff);
        V dhv = {}, dcv = {};
        if (dh) dhv = ld<VW>(dh + soff);
        if (dc_out) dcv = ld<VW>(dc_out + soff);
        V di, df, dout, dg, dprev;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const float si = get<VW>(gi, j), sf = get<VW>(gf, j), so = get<VW>(go, j), tg = get<VW>(gg, j);
            const float tc = tanhf(get<VW>(cn, j));
            const float d_h = dh ? get<VW>(dhv, j) : 0.f;
            const float d_c = dc_out ? get<VW>(dcv, j) : 0.f;
            const float dct = d_c + d_h * so * (1.f - tc * tc);
            put<VW>(di, j, dct * tg * (si * (1.f - si)));
            put<VW>(df, j, dct * get<VW>(cv, j) * (sf * (1.f - sf)));
            put<VW>(dout, j, d_h * tc * (so * (1.f - so)));
            put<VW>(dg, j, dct * si * (1.f - tg * tg));
            put<VW>(dprev, j, dct * sf);
        }
        st<VW>(dz + zoff, di);
        st<VW>(dz + zoff + gstep, df);
        st<VW>(dz + zoff + 2 * gstep, dout);
        st<VW>(dz + zoff + 3 * gstep, dg);
        st<VW>(dc + soff, dprev);
    }
}

// lstm_bwd_kernel for a recurrent unroll step's repeats (hrl_lstm_gates_backward_ex): dh may be the sum of S
// partial input gradients (the K-split adjoint conv's groups, summed here in s order instead of by a separate
// pass), and the x half's gradient dzx accumulates over the repeats (dzx = dz on the first, dzx += dz after)
struct BwdEx {
    const float *dh;
    int64_t dhs, dps;   // floats from one game to the next in dh / from one partial to the next
    int S;
    float *dzx;
    int dzx_init;
};

template <int VW>
__global__ void lstm_bwd_ex_kernel(const float *__restrict__ gates, const float *__restrict__ c,
                                   const float *__restrict__ c_out, BwdEx x, const float *__restrict__ dc_out, Geo g,
                                   float *__restrict__ dz, float *__restrict__ dc) {
    using V = typename Vec<VW>::T;
    const int64_t total = g.N * g.H * g.nq;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(e % g.nq);
        const int64_t nc = e / g.nq;
        const int ch = (int)(nc % g.H);
        const int64_t n = nc / g.H;
        const int64_t plane = (int64_t)g.HW;
        const int64_t zoff = n * 4 * g.H * plane + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t soff = nc * plane + (int64_t)q * VW;
        const int64_t hoff = n * x.dhs + (int64_t)ch * plane + (int64_t)q * VW;
        const int64_t gstep = (int64_t)g.H * plane;
        const V gi = ld<VW>(gates + zoff), gf = ld<VW>(gates + zoff + gstep), go = ld<VW>(gates + zoff + 2 * gstep),
                gg = ld<VW>(gates + zoff + 3 * gstep);
        const V cv = ld<VW>(c + soff), cn = ld<VW>(c_out + soff);
        V dhv = {}, dcv = {};
        if (x.dh) {
            dhv = ld<VW>(x.dh + hoff);
            for (int sp = 1; sp < x.S; ++sp) {
                const V p = ld<VW>(x.dh + hoff + sp * x.dps);
#pragma unroll
                for (int j = 0; j < VW; ++j) put<VW>(dhv, j, get<VW>(dhv, j) + get<VW>(p, j));
            }
        }
        if (dc_out) dcv = ld<VW>(dc_out + soff);
        V di, df, dout, dg, dprev;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const float si = get<VW>(gi, j), sf = get<VW>(gf, j), so = get<VW>(go, j), tg = get<VW>(gg, j);
            const float tc = tanhf(get<VW>(cn, j));
            const float d_h = x.dh ? get<VW>(dhv, j) : 0.f;
            const float d_c = dc_out ? get<VW>(dcv, j) : 0.f;
            const float dct = d_c + d_h * so * (1.f - tc * tc);
            put<VW>(di, j, dct * tg * (si * (1.f - si)));
            put<VW>(df, j, dct * get<VW>(cv, j) * (sf * (1.f - sf)));
            put<VW>(dout, j, d_h * tc * (so * (1.f - so)));
            put<VW>(dg, j, dct * si * (1.f - tg * tg));
            put<VW>(dprev, j, dct * sf);
        }
        st<VW>(dz + zoff, di);
        st<VW>(dz + zoff + gstep, df);
        st<VW>(dz + zoff + 2 * gstep, dout);
        st<VW>(dz + zoff + 3 * gstep, dg);
        st<VW>(dc + soff, dprev);
        if (x.dzx) {
            const V d4[4] = {di, df, dout, dg};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float *p = x.dzx + zoff + k * gstep;
                if (x.dzx_init) {
                    st<VW>(p, d4[k]);
                } else {
                    V a = ld<VW>(p);
#pragma unroll
                    for (int j = 0; j < VW; ++j) put<VW>(a, j, get<VW>(a, j) + get<VW>(d4[k], j));
                    st<VW>(p, a);
                }
            }
        }
    }
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned(const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

unsigned grid_for(int64_t total) {
    int64_t b = (total + 255) / 256;
    return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

extern "C" {

int hrl_lstm_gates_forward(const float *zx, int64_t zx_stride, const float *zh, const float *c, int64_t N, int64_t H,
                           int64_t HW, const float *bias, int64_t bias_rows, float *h_out, float *c_out, float *gates,
                           void *stream) {
    if (N == 0) return HRL_OK;
    if (!zh || !c || !h_out || !c_out || N < 0 || H < 1 || HW < 1) return HRL_EINVAL;
    if (bias && (!zx || bias_rows < 1)) return HRL_EINVAL;
    if (zx && zx_stride < 4 * H * HW) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool vec = HW % 4 == 0 && (!zx || zx_stride % 4 == 0) && aligned(zx) && aligned(zh) && aligned(c) &&
                     aligned(h_out) && aligned(c_out) && aligned(gates);
    Geo g{N, (int)H, (int)HW, (int)(vec ? HW / 4 : HW), zx_stride, bias, (int)(bias ? bias_rows : 1)};
    const int64_t total = N * H * g.nq;
    if (vec)
        hipLaunchKernelGGL(lstm_fwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, s, zx, zh, c, g, h_out, c_out,
                           gates);
    else
        hipLaunchKernelGGL(lstm_fwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s, zx, zh, c, g, h_out, c_out,
                           gates);
    return status();
}

int hrl_lstm_gates_forward_grouped(int L, const float *zh, int64_t zh_stride, const float *const *zx,
                                   const int64_t *zx_strides, const float *const *c, int64_t N, int64_t H, int64_t HW,
                                   float *const *h_out, float *const *c_out, float *const *gates, void *stream) {
    if (N == 0) return HRL_OK;
    if (L < 1 || L > kMaxLayers || !zh || !zx || !zx_strides || !c || !h_out || !c_out || N < 0 || H < 1 || HW < 1)
        return HRL_EINVAL;
    if (zh_stride < L * 4 * H * HW) return HRL_EINVAL;
    LayerTable t{};
    bool vec = HW % 4 == 0 && zh_stride % 4 == 0 && aligned(zh);
    for (int l = 0; l < L; ++l) {
        if (!zx[l] || !c[l] || !h_out[l] || !c_out[l] || zx_strides[l] < 4 * H * HW) return HRL_EINVAL;
        t.zx[l] = zx[l]; t.zxs[l] = zx_strides[l]; t.c[l] = c[l];
        t.h_out[l] = h_out[l]; t.c_out[l] = c_out[l]; t.gates[l] = gates ? gates[l] : nullptr;
        vec = vec && zx_strides[l] % 4 == 0 && aligned(zx[l]) && aligned(c[l]) && aligned(h_out[l]) &&
              aligned(c_out[l]) && aligned(t.gates[l]);
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    Geo g{N, (int)H, (int)HW, (int)(vec ? HW / 4 : HW), 0, nullptr, 1};
    const int64_t total = N * H * g.nq * L;
    if (vec) hipLaunchKernelGGL(lstm_fwd_grouped_kernel<4>, dim3(grid_for(total)), dim3(256), 0, s, zh, zh_stride, t, L, g);
    else hipLaunchKernelGGL(lstm_fwd_grouped_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s, zh, zh_stride, t, L, g);
    return status();
}

int hrl_lstm_gates_backward(const float *gates, const float *c, const float *c_out, const float *dh,
                            const float *dc_out, int64_t N, int64_t H, int64_t HW, float *dz, float *dc,
                            void *stream) {
    if (N == 0) return HRL_OK;
    if (!gates || !c || !c_out || !dz || !dc || N < 0 || H < 1 || HW < 1) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool vec = HW % 4 == 0 && aligned(gates) && aligned(c) && aligned(c_out) && aligned(dh) &&
                     aligned(dc_out) && aligned(dz) && aligned(dc);
    Geo g{N, (int)H, (int)HW, (int)(vec ? HW / 4 : HW), 0};
    const int64_t total = N * H * g.nq;
    if (vec)
        hipLaunchKernelGGL(lstm_bwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, s, gates, c, c_out, dh, dc_out,
                           g, dz, dc);
    else
        hipLaunchKernelGGL(lstm_bwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s, gates, c, c_out, dh, dc_out,
                           g, dz, dc);
    return status();
}

int hrl_lstm_gates_backward_ex(const float *gates, const float *c, const float *c_out, const float *dh,
                               int64_t dh_stride, int dh_parts, int64_t dh_part_stride, const float *dc_out,
                               int64_t N, int64_t H, int64_t HW, float *dz, float *dc, float *dzx, int dzx_init,
                               void *stream) {
    if (N == 0) return HRL_OK;
    if (!gates || !c || !c_out || !dz || !dc || N < 0 || H < 1 || HW < 1 || dh_parts < 1) return HRL_EINVAL;
    if (dh && (dh_stride < H * HW || (dh_parts > 1 && dh_part_stride < H * HW))) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool vec = HW % 4 == 0 && aligned(gates) && aligned(c) && aligned(c_out) && aligned(dh) &&
                     aligned(dc_out) && aligned(dz) && aligned(dc) && aligned(dzx) && dh_stride % 4 == 0 &&
                     dh_part_stride % 4 == 0;
    Geo g{N, (int)H, (int)HW, (int)(vec ? HW / 4 : HW), 0};
    BwdEx x{dh, dh_stride, dh_part_stride, dh ? dh_parts : 1, dzx, dzx_init};
    const int64_t total = N * H * g.nq;
    if (vec)
        hipLaunchKernelGGL(lstm_bwd_ex_kernel<4>, dim3(grid_for(total)), dim3(256), 0, s, gates, c, c_out, x, dc_out,
                           g, dz, dc);
    else
        hipLaunchKernelGGL(lstm_bwd_ex_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s, gates, c, c_out, x, dc_out,
                           g, dz, dc);
    return status();
}

}  // extern "C"
