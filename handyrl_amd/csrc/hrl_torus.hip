// hrl_torus.hip — 3x3 convolution on a torus board with fp32 MFMA (gfx950).
//
// GeeseNet (handyrl/envs/kaggle/hungry_geese.py:23-57, config C4) is 13
// TorusConv2d layers on the 7x11 Hungry Geese board: the reference wraps the
// board with two torch.cat copies and runs a 'valid' 3x3 conv
// (hungry_geese.py:30-35).  Here the wrap is addressing:
//
//   y[n, co, q] = b[co] + sum_{ci, tap} W[co, ci, tap] * x[n, ci, nbr(q, tap)]
//   nbr(q, tap) = ((r + ky - 1) mod H) * W + (c + kx - 1) mod W,  q = r*W + c, tap = ky*3 + kx
//
// torus_conv_kernel<KS, VEC, STATS> (forward; also the input gradient, run on
// dy with the weights transposed and the taps mirrored -- on a torus the
// adjoint of the conv is again a conv):
//   * one wave computes one sample at a time as the GEMM
//       Y^T (cells x 32) = Im2col^T (cells x 9*Cin) . W^T (9*Cin x 32)
//     with v_mfma_f32_16x16x4_f32 (exact fp32 products): 5 cell tiles x 2
//     channel tiles = 10 accumulators, 9 * KS k-steps of 4 input channels;
//   * the sample (Cin x HW floats) is staged in LDS as [ci][cell] rows of
//     stride 81; the A fragment of lane l is the gather
//     tile[ci][nbr(cell, tap)] with the 45 neighbour offsets of the lane's
//     cells precomputed in registers;
//   * the packed weights [tap][k-step][co-tile][64] sit in LDS once per
//     workgroup (B fragments are consecutive, conflict-free ds_read_b32);
//   * the next sample's global loads are in flight during the MFMAs; the
//     output goes through the (dead) input tile to coalesced stores;
//   * STATS: the epilogue also sums y and y^2 per output channel (fp32 per
//     sample, fp64 across samples, fixed-order folds) for the BatchNorm
//     that follows every GeeseNet conv -> hrl_bn_finalize_stats.
// torus_wgrad_kernel<KS>: dW[co, ci, tap] = sum_{n, q} dy[n, co, q] x[n, ci, nbr(q, tap)]
//   and db[co] = sum dy, per wave as C (co x ci) += dY (co x cells) . X_tap (cells x ci)
//   over 20 k-steps of 4 cells per sample (36 accumulators: 9 taps x 2 x 2
//   tiles); the neighbour of the k-step's cell comes from an LDS table.
//   Waves fold through LDS and workgroups through a fixed-order reduce
//   (deterministic).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"
#include "hrl_split.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCo = 32;                  // output channels (2 MFMA column tiles)
constexpr int kMT = 5;                   // 16-cell tiles: boards of at most 80 cells
constexpr int kMaxCells = kMT * 16;
constexpr int kS = 81;                   // LDS row stride: odd, 16 consecutive rows -> 16 banks
constexpr int kTaps = 9;
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = kCo * kS;          // floats of one wave's sample tile (>= KS*4 rows)
constexpr int kKCells = kMaxCells / 4;   // wgrad k-steps per sample (20)

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The split path's helpers (exact three-way bf16 split, six partial products): hrl_split.h.
using hrl_split::split8;
using hrl_split::mfma_split;

__device__ __forceinline__ int torus_nbr(int q, int H, int W, int tap) {
    const int r = q / W, c = q - r * W;
    int rr = r + tap / 3 - 1, cc = c + tap % 3 - 1;
    rr = rr < 0 ? rr + H : (rr >= H ? rr - H : rr);
    cc = cc < 0 ? cc + W : (cc >= W ? cc - W : cc);
    return rr * W + cc;
}

// floor(e / d) for 0 <= e < 2^20 given inv = 1/d (exact: see hrl_targets.hip fdiv)
__device__ __forceinline__ int fdiv(int e, float inv) { return (int)(((float)e + 0.5f) * inv); }

// An index the compiler cannot see through: the per-element tile / coefficient addresses of the staging
// loops are sample-invariant, and hoisting all of them out of the sample loop spills (40-80 registers).
__device__ __forceinline__ int opaque(int i) {
    asm volatile("" : "+v"(i));
    return i;
}

// The LDS tile slots of the float4 at element 4i of a [c][cell] sample: channel c0 = floor(4i / HW) (one
// division per float4) and cell r0; element 4i+j is in channel c0 + wrap_j, wrap_j = [r0 + j >= HW].
struct Quad {
    int c0, base, r0;
    __device__ __forceinline__ Quad(int i, int HW, float inv_hw) {
        c0 = fdiv(4 * i, inv_hw);
        r0 = 4 * i - c0 * HW;
        base = c0 * kS + r0;
    }
    __device__ __forceinline__ bool wrap(int j, int HW) const { return r0 + j >= HW; }
    __device__ __forceinline__ int slot(int j, int HW) const { return base + j + (wrap(j, HW) ? kS - HW : 0); }
};

// ------------------------------------------------------------------ sample staging
// One sample's n_elem = C*HW floats: global (contiguous) -> registers -> LDS [c][cell] rows.
template <bool VEC, int NLD, bool OPQ = false>
struct Stage {
    float4 v[VEC ? NLD : 1];
    float s[VEC ? 1 : NLD];

    __device__ __forceinline__ void load(const float *src, int n_elem, int lane) {
        if constexpr (VEC) {
            const int nv = n_elem >> 2;
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = min(k * 64 + lane, nv - 1);   // clamp: loads issue back to back
                v[k] = reinterpret_cast<const float4 *>(src)[i];
            }
        } else {
#pragma unroll
            for (int k = 0; k < NLD; ++k) s[k] = src[min(k * 64 + lane, n_elem - 1)];
        }
    }
    __device__ __forceinline__ void to_lds(float *tile, int n_elem, int HW, float inv_hw, int lane) const {
        if constexpr (VEC) {
            const int nv = n_elem >> 2;
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = OPQ ? opaque(k * 64 + lane) : k * 64 + lane;
                if (i < nv) {
                    const float x4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
                    const Quad q(i, HW, inv_hw);
#pragma unroll
                    for (int j = 0; j < 4; ++j) tile[q.slot(j, HW)] = x4[j];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int e = OPQ ? opaque(k * 64 + lane) : k * 64 + lane;
                if (e < n_elem) {
                    const int c = fdiv(e, inv_hw);
                    tile[c * kS + (e - c * HW)] = s[k];
                }
            }
        }
    }
};

// LDS tile [c][cell] -> one sample's output (n_elem = channels*HW floats, contiguous);
// with `add`: out = tile + add * [mask > 0] elementwise (add, mask shaped like the output)
__device__ __forceinline__ void store_sample(const float *tile, float *dst, int n_elem, bool vec, int HW,
                                             float inv_hw, int lane, const float *add, const float *mask) {
    if (vec) {
        const int nv = n_elem >> 2;
        for (int i = lane; i < nv; i += 64) {
            float x4[4];
            const Quad q(i, HW, inv_hw);
#pragma unroll
            for (int j = 0; j < 4; ++j) x4[j] = tile[q.slot(j, HW)];
            if (add) {
                const float4 a = reinterpret_cast<const float4 *>(add)[i];
                const float4 m = reinterpret_cast<const float4 *>(mask)[i];
                x4[0] += m.x > 0.f ? a.x : 0.f;
                x4[1] += m.y > 0.f ? a.y : 0.f;
                x4[2] += m.z > 0.f ? a.z : 0.f;
                x4[3] += m.w > 0.f ? a.w : 0.f;
            }
            reinterpret_cast<float4 *>(dst)[i] = make_float4(x4[0], x4[1], x4[2], x4[3]);
        }
    } else {
        for (int e = lane; e < n_elem; e += 64) {
            const int c = fdiv(e, inv_hw);
            float v = tile[c * kS + (e - c * HW)];
            if (add) v += mask[e] > 0.f ? add[e] : 0.f;
            dst[e] = v;
        }
    }
}

__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS operations done
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ forward / input gradient
// x: (N, Cin, HW); wpk: [tap][KS][2][64]; y: (N, out_c, HW), out_c <= 32 (the first out_c channels of
// the 32 computed); part: [grid][32][2] (STATS, SUMS)
struct ConvArgs {
    const float *x;
    int64_t N;
    int Cin, H, W;
    const float *wpk, *bias;
    int out_c;
    bool vec_out;
    float *y;
    double *part;
    const float *add, *add_mask;   // out = conv + add * [add_mask > 0]
    // PRO: x is the previous unit's conv output; the conv input is h = relu([res +] x*alpha[c] + beta[c])
    // (bn_apply_kernel / bn_res_apply_kernel arithmetic), also written to hout
    const float *res, *alpha, *beta;
    float *hout;
    // SUMS: with v the stored output and m = [hmask > 0], per channel sum(v m) and sum(v m (yprev - mean))
    // (bn_bwd_reduce_kernel<MASK = 2> of the previous unit)
    const float *hmask, *yprev, *mean;
    int co_total;   // output channels of y per sample; workgroup column blockIdx.y computes 32 of them
};

__device__ __forceinline__ float relu(float v) { return v < 0.f ? 0.f : v; }   // NaN stays NaN

// PRO prologue: the staged previous conv output (and residual) -> h in the LDS tile and in global memory
template <int PRO, int NLD>
__device__ __forceinline__ void pro_to_lds(const Stage<true, NLD, true> &sx, const Stage<true, NLD, true> &sr, float *tile,
                                           float *hout, int n_elem, int HW, float inv_hw, int lane,
                                           const float *al, const float *be) {
    const int nv = n_elem >> 2;
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
        const int i = opaque(k * 64 + lane);
        if (i < nv) {
            const float x4[4] = {sx.v[k].x, sx.v[k].y, sx.v[k].z, sx.v[k].w};
            const float r4[4] = {sr.v[k].x, sr.v[k].y, sr.v[k].z, sr.v[k].w};
            float o[4];
            const Quad q(i, HW, inv_hw);
            const float a0 = al[q.c0], a1 = al[q.c0 + 1], b0 = be[q.c0], b1 = be[q.c0 + 1];   // coef_s has 33+ rows
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool w = q.wrap(j, HW);
                float v = x4[j] * (w ? a1 : a0) + (w ? b1 : b0);
                if constexpr (PRO == 2) v = r4[j] + v;
                v = relu(v);
                tile[q.slot(j, HW)] = v;
                o[j] = v;
            }
            reinterpret_cast<float4 *>(hout)[i] = make_float4(o[0], o[1], o[2], o[3]);
        }
        __builtin_amdgcn_sched_barrier(0);   // one float4 at a time: hoisting every coefficient read spills
    }
}

// SUMS epilogue, after the output tile is complete (vec layout only): store out = tile + add*[mask > 0],
// then the per-channel sums of out*[hmask > 0] (s1) and out*[hmask > 0]*(yprev - mean) (s2) in fp64.
// Lane l owns channel l & 31 and half (l >> 5) of the cells: it reads its 40 yprev values straight from the
// channel row (issued after the store pass, in flight during the first sums: issued earlier they spill) and the
// masked values from the tile twice.
// Every global load of a pass is issued before its first use: the per-float4 loop this replaces waited for each
// iteration's loads in turn, ten round trips per sample.
__device__ __forceinline__ void store_sample_sums(float *tile, float *dst, int n_elem, int HW, float inv_hw,
                                                  int lane, const float *__restrict__ add,
                                                  const float *__restrict__ mask, const float *__restrict__ hmask,
                                                  const float *__restrict__ yprev, const float *mean_s,
                                                  double &s1, double &s2) {
    constexpr int kNV = kCo * kMaxCells / 4 / 64;   // float4 per lane of an 80-cell sample
    constexpr int kH = kNV / 2;                     // the store pass in two halves: 15 float4 in flight
    constexpr int kHalf = kMaxCells / 2;
    const int nv = n_elem >> 2;
    const int c = lane & 31, c0 = (lane >> 5) * kHalf;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        asm volatile("" ::: "memory");
        float4 a[kH], m[kH], hm[kH];
#pragma unroll
        for (int k = 0; k < kH; ++k) {
            const int i = min((h * kH + k) * 64 + lane, nv - 1);
            a[k] = reinterpret_cast<const float4 *>(add)[i];
            m[k] = reinterpret_cast<const float4 *>(mask)[i];
            hm[k] = reinterpret_cast<const float4 *>(hmask)[i];
        }
#pragma unroll
        for (int k = 0; k < kH; ++k) {
            const int i = (h * kH + k) * 64 + lane;
            if (i < nv) {
                const float a4[4] = {a[k].x, a[k].y, a[k].z, a[k].w}, m4[4] = {m[k].x, m[k].y, m[k].z, m[k].w};
                const float h4[4] = {hm[k].x, hm[k].y, hm[k].z, hm[k].w};
                float x4[4];
                const Quad q(i, HW, inv_hw);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float *slot = tile + q.slot(j, HW);
                    x4[j] = *slot + (m4[j] > 0.f ? a4[j] : 0.f);
                    *slot = h4[j] > 0.f ? x4[j] : 0.f;
                }
                reinterpret_cast<float4 *>(dst)[i] = make_float4(x4[0], x4[1], x4[2], x4[3]);
            }
        }
    }
    // the lane's channel row segment through a buffer descriptor over the sample: one address register, the cell as
    // the immediate offset; cells past the row read the next channel's (unused), past the sample 0
    float yv[kHalf];
    {
        const uint64_t p = reinterpret_cast<uint64_t>(yprev);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, n_elem * 4, 0x00020000);
        const int vo = (c * HW + c0) * 4;
#pragma unroll
        for (int j = 0; j < kHalf; ++j)
            yv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, vo, j * 4, 0));
    }
    lds_fence();
    float t1 = 0.f, t2 = 0.f;   // fp32 within the sample, fp64 across samples (as the STATS epilogue)
#pragma unroll
    for (int j = 0; j < kHalf; ++j) t1 += c0 + j < HW ? tile[c * kS + c0 + j] : 0.f;
    s1 += (double)t1;
    const float mu = mean_s[c];
#pragma unroll
    for (int j = 0; j < kHalf; ++j)
        if (c0 + j < HW) t2 += tile[c * kS + c0 + j] * (yv[j] - mu);
    s2 += (double)t2;
}

// MT: 16-cell tiles (boards of at most 16*MT cells).  ZPAD: zero padding instead of the torus wrap (a 'same'
// 3x3 nn.Conv2d, e.g. GeisterNet's 6x6 board): taps off the board read a slot that is never written.
// blockIdx.y: the 32-channel output chunk (weights packed per chunk).
template <int KS, bool VEC, bool STATS, bool SPLIT, int PRO = 0, bool SUMS = false, int MT = kMT, bool ZPAD = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void torus_conv_kernel(ConvArgs a) {
    static_assert(VEC || (PRO == 0 && !SUMS), "the prologue / sums forms need the float4 layout");
    const float *__restrict__ x = a.x;
    const int64_t N = a.N;
    const int Cin = a.Cin, H = a.H, W = a.W, out_c = a.out_c;
    const float *__restrict__ wpk = a.wpk;
    const float *__restrict__ bias = a.bias;
    float *__restrict__ y = a.y;
    const bool vec_out = a.vec_out;
    double *__restrict__ part = a.part;
    const float *__restrict__ add = a.add;
    const float *__restrict__ add_mask = a.add_mask;
    constexpr int kNW = kTaps * KS * 2 * 64;
    constexpr int kCells = MT * 16;
    constexpr int kNLd = VEC ? (KS * 4 * kCells / 4 + 63) / 64 : (KS * 4 * kCells + 63) / 64;
    __shared__ float w_lds[kNW];
    __shared__ float tiles[kWaves * kTile];
    __shared__ float coef_s[2 * kCo + 2];   // PRO: alpha[32], beta[32]; SUMS: mean[32]; +1 read past the last channel
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int HW = H * W;
    const float inv_hw = 1.0f / (float)HW;
    const int in_elem = Cin * HW;
    float *tile = tiles + wave * kTile;

    const int chunk = (int)blockIdx.y;
    for (int i = threadIdx.x; i < kNW; i += kThreads) w_lds[i] = wpk[(int64_t)chunk * kNW + i];
    if constexpr (PRO != 0) {
        if (threadIdx.x < 2 * kCo) coef_s[threadIdx.x] = threadIdx.x < kCo ? a.alpha[threadIdx.x] : a.beta[threadIdx.x - kCo];
    }
    if constexpr (SUMS) {
        if (threadIdx.x < kCo) coef_s[threadIdx.x] = a.mean[threadIdx.x];
    }
    // channel rows Cin .. 4*KS-1 stay zero (their packed weights are zero too; no NaN * 0)
    for (int i = lane; i < kTile; i += 64) tile[i] = 0.f;

    // the lane's A-fragment cells: q = mt*16 + (lane & 15); cells past the board read cell q - HW.
    // nbr(q, tap) = row part (ky) + column part (kx), packed as row | column << 16: 15 registers instead
    // of 45 (the kernel sits at the 256-register limit of 2 waves per SIMD)
    uint32_t nbp[MT][ZPAD ? 9 : 3];   // ZPAD: the offset per tap (taps off the board -> the zero slot kS-1)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        int q = mt * 16 + (lane & 15);
        while (q >= HW) q -= HW;
        const int r = q / W, c = q - r * W;
        if constexpr (ZPAD) {
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int rr = r + t / 3 - 1, cc = c + t % 3 - 1;
                const bool in = rr >= 0 && rr < H && cc >= 0 && cc < W;
                nbp[mt][t] = (uint32_t)((in ? rr * W + cc : kS - 1) + (lane >> 4) * kS);
            }
        } else {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                int rr = r + d - 1, cc = c + d - 1;
                rr = rr < 0 ? rr + H : (rr >= H ? rr - H : rr);
                cc = cc < 0 ? cc + W : (cc >= W ? cc - W : cc);
                nbp[mt][d] = (uint32_t)(rr * W + (lane >> 4) * kS) | ((uint32_t)cc << 16);
            }
        }
    }
    auto nbr_ofs = [&](int mt, int t) -> int {
        if constexpr (ZPAD) return (int)nbp[mt][t];
        else return (int)(nbp[mt][t / 3] & 0xffffu) + (int)(nbp[mt][t % 3] >> 16);
    };
    float bias_v[2] = {0.f, 0.f};
    if (bias) {
        bias_v[0] = bias[chunk * kCo + (lane & 15)];
        bias_v[1] = bias[chunk * kCo + 16 + (lane & 15)];
    }
    double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};

    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t n = (int64_t)blockIdx.x * kWaves + wave;
    Stage<VEC, kNLd, true> st;
    Stage<VEC, kNLd, true> sr;   // PRO == 2: the residual input
    if (n < N) {
        st.load(x + n * in_elem, in_elem, lane);
        if constexpr (PRO == 2) sr.load(a.res + n * in_elem, in_elem, lane);
    }
    __syncthreads();   // weights (and coefficients) in LDS, tiles zeroed

    for (; n < N; n += stride) {
        if constexpr (PRO != 0)
            pro_to_lds<PRO>(st, sr, tile, a.hout + n * in_elem, in_elem, HW, inv_hw, lane, coef_s, coef_s + kCo);
        else
            st.to_lds(tile, in_elem, HW, inv_hw, lane);
        lds_fence();
        const int64_t next = n + stride;
        if (next < N) st.load(x + next * in_elem, in_elem, lane);   // in flight during the MFMAs

        f32x4 acc[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt][0] = acc[mt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const float *wl = w_lds + lane;
        if constexpr (SPLIT) {
            // one k-step of 32 input channels per tap: lane l's A/B k are channels 8(l>>4) + e.
            // nrow carries the fp32 mapping's channel offset (l>>4)*kS; move it to 8(l>>4)*kS.
            const int cofs = 7 * (lane >> 4) * kS;
#pragma unroll
            for (int t = 0; t < kTaps; ++t) {
                // B: W^T[ci][co = 16ct + (l&15)] from the packed [tap][s][ct][64] (ci = 4s + (l'>>4)),
                // zero past the KS*4 packed channels
                uint4 Bh[2], Bm[2], Bl[2];
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    float bv[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int ci = 8 * (lane >> 4) + e;
                        const int sk = ci >> 2;
                        const float w = w_lds[((t * KS + min(sk, KS - 1)) * 2 + ct) * 64 + (ci & 3) * 16 + (lane & 15)];
                        bv[e] = sk < KS ? w : 0.f;
                    }
                    split8(bv, Bh[ct], Bm[ct], Bl[ct]);
                }
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const float *ap = tile + nbr_ofs(mt, t) + cofs;
                    float av[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) av[e] = ap[e * kS];
                    uint4 Ah, Am, Al;
                    split8(av, Ah, Am, Al);
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct)
                        acc[mt][ct] = mfma_split(Ah, Am, Al, Bh[ct], Bm[ct], Bl[ct], acc[mt][ct]);
                }
            }
        } else {
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const float b0 = wl[((t * KS + s) * 2 + 0) * 64];
                const float b1 = wl[((t * KS + s) * 2 + 1) * 64];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const float a = tile[nbr_ofs(mt, t) + s * 4 * kS];
                    acc[mt][0] = mfma(a, b0, acc[mt][0]);
                    acc[mt][1] = mfma(a, b1, acc[mt][1]);
                }
            }
        }
        }
        lds_fence();   // every lane's A reads done before the tile is overwritten
        if constexpr (PRO == 2) {
            if (next < N) sr.load(a.res + next * in_elem, in_elem, lane);   // in flight during the epilogue
        }

        // accumulators (cell = mt*16 + (lane>>4)*4 + r, co = ct*16 + (lane&15)) -> tile [co][cell]
        float t1[2] = {0.f, 0.f}, t2[2] = {0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int cell = mt * 16 + (lane >> 4) * 4 + r;
                    const int co = ct * 16 + (lane & 15);
                    if (cell < HW) {
                        const float v = acc[mt][ct][r] + bias_v[ct];
                        tile[co * kS + cell] = v;
                        if constexpr (STATS) {
                            t1[ct] += v;
                            t2[ct] += v * v;
                        }
                    }
                }
        if constexpr (STATS) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                s1[ct] += (double)t1[ct];
                s2[ct] += (double)t2[ct];
            }
        }
        lds_fence();
        const int64_t ob = n * ((int64_t)a.co_total * HW) + (int64_t)chunk * kCo * HW;
        if constexpr (SUMS)
            store_sample_sums(tile, y + ob, out_c * HW, HW, inv_hw, lane, add + ob, add_mask + ob, a.hmask + ob,
                              a.yprev + ob, coef_s, s1[0], s2[0]);
        else
            store_sample(tile, y + ob, out_c * HW, vec_out, HW, inv_hw, lane, add ? add + ob : nullptr,
                         add ? add_mask + ob : nullptr);
        lds_fence();
        // padding rows must read as zero again for the next sample (the output tile used them)
        for (int i = in_elem / HW * kS + lane; i < (SPLIT ? kCo : KS * 4) * kS; i += 64) tile[i] = 0.f;
    }
    if constexpr (STATS) {
        // fold the 4 lanes sharing a channel and the 4 waves in a fixed order
        __syncthreads();
        double *red = reinterpret_cast<double *>(tiles);   // [wave][group][32][2]
        const int grp = lane >> 4;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const int co = ct * 16 + (lane & 15);
            red[((wave * 4 + grp) * kCo + co) * 2 + 0] = s1[ct];
            red[((wave * 4 + grp) * kCo + co) * 2 + 1] = s2[ct];
        }
        __syncthreads();
        if (threadIdx.x < 2 * kCo) {
            const int co = threadIdx.x >> 1, k = threadIdx.x & 1;
            double t = 0.0;
            for (int i = 0; i < kWaves * 4; ++i) t += red[(i * kCo + co) * 2 + k];
            part[((int64_t)blockIdx.x * kCo + co) * 2 + k] = t;
        }
    }
    if constexpr (SUMS) {
        // lane l holds channel l & 31 over half l >> 5 of the cells: fold halves and waves in a fixed order
        __syncthreads();
        double *red = reinterpret_cast<double *>(tiles);   // [wave][half][32][2]
        red[((wave * 2 + (lane >> 5)) * kCo + (lane & 31)) * 2 + 0] = s1[0];
        red[((wave * 2 + (lane >> 5)) * kCo + (lane & 31)) * 2 + 1] = s2[0];
        __syncthreads();
        if (threadIdx.x < 2 * kCo) {
            const int co = threadIdx.x >> 1, k = threadIdx.x & 1;
            double t = 0.0;
            for (int i = 0; i < kWaves * 2; ++i) t += red[(i * kCo + co) * 2 + k];
            part[((int64_t)blockIdx.x * kCo + co) * 2 + k] = t;
        }
    }
}

// ------------------------------------------------------------------ pre-split forward / input gradient (round 5)
// torus_conv_ps_kernel<PRO, STATS, SUMS>: the split torus_conv_kernel for 32 input channels with each input value
// split ONCE per sample instead of once per tap that gathers it (9x).  The kernel above spends ≈27k SIMD cycles
// per sample, ≈60% of them in the A splits' vector instructions, against 8.6k of MFMA.
//   * the sample's image is kept in LDS already split: a cell row of 192 bytes = [part h/m/l][channels 0-31] as
//     bf16, so an A fragment (8 consecutive channels at one cell) is one ds_read_b128 per part.  The 16-byte
//     channel chunk g of cell c sits at chunk g ^ ((c >> 2) & 3) of its part: 16 lanes reading 16 consecutive
//     cells hit 16 distinct bank quads (the row stride is 48 dwords);
//   * staging: lane unit u = (channel group g, cell c) loads its 8 channels at cell c with dword loads (lanes of
//     a load instruction read consecutive cells: coalesced), optionally applies the BatchNorm prologue, splits the
//     8 values and writes the three 16-byte fragments;
//   * 8 waves per workgroup, one workgroup per CU (8 x 15 KB images + the 37 KB packed weights = 156 KB of LDS):
//     the same two waves per SIMD as the 4-wave kernel at two workgroups per CU.  A wave walks the samples
//     n = 8 b + w (mod 2048) that wave w & 3 of the 4-wave kernel's block 2b + (w >> 2) walks, and its
//     statistics / sums fold into that block's partial row in the same order: results are bit-identical to
//     torus_conv_kernel<8, *, *, true, PRO, SUMS> (tests/test_geese.py::test_presplit_form_is_bit_identical).
// The B fragments are split per tap from the fp32 packed weights as before (pre-split weights would not fit).
constexpr int kPW = 8;
constexpr int kPThreads = 64 * kPW;
constexpr int kRowDw = 48;                    // dwords per cell row of the split image
constexpr int kImgDw = kMaxCells * kRowDw;    // dwords per wave image (15 KB)
constexpr int kPU = 4 * kMaxCells / 64;       // staging units per lane (4 channel groups x 80 cells / 64 lanes)
static_assert(kImgDw >= kTile, "the fp32 output tile lives in the image region");

__device__ __forceinline__ int ps_row(int cell, int g) { return cell * kRowDw + 4 * (g ^ ((cell >> 2) & 3)); }

template <int PRO, bool STATS, bool SUMS>
__global__ __launch_bounds__(kPThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void torus_conv_ps_kernel(
    ConvArgs a, int nvb) {
    const int64_t N = a.N;
    const int H = a.H, W = a.W, out_c = a.out_c, Cin = a.Cin;
    constexpr int kNW = kTaps * 8 * 2 * 64;
    __shared__ float w_lds[kNW];
    __shared__ __attribute__((aligned(16))) uint32_t imgs[kPW * kImgDw];
    __shared__ __attribute__((aligned(16))) float coef_s[2 * kCo + 2];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int HW = H * W;
    const float inv_hw = 1.0f / (float)HW;
    const int in_elem = Cin * HW;
    uint32_t *img = imgs + wave * kImgDw;
    float *tile = reinterpret_cast<float *>(img);

    for (int i = threadIdx.x; i < kNW; i += kPThreads) w_lds[i] = a.wpk[i];
    if constexpr (PRO != 0) {
        if (threadIdx.x < 2 * kCo) coef_s[threadIdx.x] = threadIdx.x < kCo ? a.alpha[threadIdx.x] : a.beta[threadIdx.x - kCo];
    }
    if constexpr (SUMS) {
        if (threadIdx.x < kCo) coef_s[threadIdx.x] = a.mean[threadIdx.x];
    }

    uint32_t nbp[kMT][3];   // (row (r + d - 1) * W) | (column (c + d - 1)) << 16 of the lane's A cells
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt) {
        int q = mt * 16 + (lane & 15);
        while (q >= HW) q -= HW;
        const int r = q / W, c = q - r * W;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            int rr = r + d - 1, cc = c + d - 1;
            rr = rr < 0 ? rr + H : (rr >= H ? rr - H : rr);
            cc = cc < 0 ? cc + W : (cc >= W ? cc - W : cc);
            nbp[mt][d] = (uint32_t)(rr * W) | ((uint32_t)cc << 16);
        }
    }
    const int g = lane >> 4;
    float bias_v[2] = {0.f, 0.f};
    if (a.bias) {
        bias_v[0] = a.bias[lane & 15];
        bias_v[1] = a.bias[16 + (lane & 15)];
    }
    double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};

    // staging unit u = k * 64 + lane (valid below 4 HW): channels 8 gu .. 8 gu + 7 at cell cu
    float sv[kPU][8], sr[PRO == 2 ? kPU : 1][8];
    auto unit = [&](int k, int &gu, int &cu) {
        const int u = opaque(k * 64 + lane);
        gu = fdiv(u, inv_hw);
        cu = u - gu * HW;
        return u < 4 * HW;
    };
    auto load = [&](float (&v)[kPU][8], const float *src) {
#pragma unroll
        for (int k = 0; k < kPU; ++k) {
            int gu, cu;
            const bool ok = unit(k, gu, cu);
            const float *p = src + (ok ? 8 * gu * HW + cu : 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[k][e] = (!ok || 8 * gu + e < Cin) ? p[e * HW] : 0.f;   // rows >= Cin: 0
        }
    };

    const int64_t stride = (int64_t)gridDim.x * kPW;
    int64_t n = (int64_t)blockIdx.x * kPW + wave;
    if (n < N) {
        load(sv, a.x + n * in_elem);
        if constexpr (PRO == 2) load(sr, a.res + n * in_elem);
    }
    __syncthreads();   // weights (and coefficients) in LDS

    for (; n < N; n += stride) {
        // the staged sample -> (prologue) -> split image
#pragma unroll
        for (int k = 0; k < kPU; ++k) {
            int gu, cu;
            if (unit(k, gu, cu)) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = sv[k][e];
                if constexpr (PRO != 0) {
                    const float4 *al = reinterpret_cast<const float4 *>(coef_s + 8 * gu);
                    const float4 *be = reinterpret_cast<const float4 *>(coef_s + kCo + 8 * gu);
                    const float4 a0 = al[0], a1 = al[1], b0 = be[0], b1 = be[1];
                    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                    float *ho = a.hout + n * in_elem + 8 * gu * HW + cu;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float t = v[e] * av[e] + bv[e];
                        if constexpr (PRO == 2) t = sr[k][e] + t;
                        v[e] = relu(t);
                        ho[e * HW] = v[e];
                    }
                }
                uint4 Ah, Am, Al;
                split8(v, Ah, Am, Al);
                uint4 *row = reinterpret_cast<uint4 *>(img + ps_row(cu, gu));
                row[0] = Ah;
                row[4] = Am;
                row[8] = Al;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_fence();
        const int64_t next = n + stride;
        if (next < N) {
            load(sv, a.x + next * in_elem);   // in flight during the MFMAs
            if constexpr (PRO == 2) load(sr, a.res + next * in_elem);
        }

        f32x4 acc[kMT][2];
#pragma unroll
        for (int mt = 0; mt < kMT; ++mt) acc[mt][0] = acc[mt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            uint4 Bh[2], Bm[2], Bl[2];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                float bv[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int ci = 8 * g + e;
                    bv[e] = w_lds[((t * 8 + (ci >> 2)) * 2 + ct) * 64 + (ci & 3) * 16 + (lane & 15)];
                }
                split8(bv, Bh[ct], Bm[ct], Bl[ct]);
            }
#pragma unroll
            for (int mt = 0; mt < kMT; ++mt) {
                const int cell = (int)(nbp[mt][t / 3] & 0xffffu) + (int)(nbp[mt][t % 3] >> 16);
                const uint4 *row = reinterpret_cast<const uint4 *>(img + ps_row(cell, g));
                const uint4 Ah = row[0], Am = row[4], Al = row[8];
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
                    acc[mt][ct] = mfma_split(Ah, Am, Al, Bh[ct], Bm[ct], Bl[ct], acc[mt][ct]);
            }
        }
        lds_fence();   // every lane's A reads done before the image becomes the output tile

        float t1[2] = {0.f, 0.f}, t2[2] = {0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int cell = mt * 16 + (lane >> 4) * 4 + r;
                    const int co = ct * 16 + (lane & 15);
                    if (cell < HW) {
                        const float v = acc[mt][ct][r] + bias_v[ct];
                        tile[co * kS + cell] = v;
                        if constexpr (STATS) {
                            t1[ct] += v;
                            t2[ct] += v * v;
                        }
                    }
                }
        if constexpr (STATS) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                s1[ct] += (double)t1[ct];
                s2[ct] += (double)t2[ct];
            }
        }
        lds_fence();
        const int64_t ob = n * ((int64_t)out_c * HW);
        if constexpr (SUMS)
            store_sample_sums(tile, a.y + ob, out_c * HW, HW, inv_hw, lane, a.add + ob, a.add_mask + ob, a.hmask + ob,
                              a.yprev + ob, coef_s, s1[0], s2[0]);
        else
            store_sample(tile, a.y + ob, out_c * HW, a.vec_out, HW, inv_hw, lane, a.add ? a.add + ob : nullptr,
                         a.add ? a.add_mask + ob : nullptr);
        lds_fence();   // the tile's reads done before the next image is written
    }
    if constexpr (STATS || SUMS) {
        // the 4-wave kernel's fold per virtual block vb = 2 b + (w >> 2): its waves w & 3 (and their lane
        // groups / halves) in the same fixed order
        constexpr int kG = STATS ? 4 : 2;   // lane groups (STATS: l >> 4 of a column tile) or halves (SUMS)
        __syncthreads();
        double *red = reinterpret_cast<double *>(imgs);   // [wave][group][32][2]
        if constexpr (STATS) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int co = ct * 16 + (lane & 15);
                red[((wave * kG + g) * kCo + co) * 2 + 0] = s1[ct];
                red[((wave * kG + g) * kCo + co) * 2 + 1] = s2[ct];
            }
        } else {
            red[((wave * kG + (lane >> 5)) * kCo + (lane & 31)) * 2 + 0] = s1[0];
            red[((wave * kG + (lane >> 5)) * kCo + (lane & 31)) * 2 + 1] = s2[0];
        }
        __syncthreads();
        if (threadIdx.x < 4 * kCo) {
            const int hb = threadIdx.x >> 6, co = (threadIdx.x & 63) >> 1, k = threadIdx.x & 1;
            const int vb = 2 * (int)blockIdx.x + hb;
            double t = 0.0;
            for (int i = 0; i < 4 * kG; ++i) t += red[((hb * 4 * kG + i) * kCo + co) * 2 + k];
            if (vb < nvb) a.part[((int64_t)vb * kCo + co) * 2 + k] = t;
        }
    }
}

// W (32, Cin, 3, 3) -> packed [tap][KS][ct][64]: lane l of k-step s holds W^T[ci = 4s + (l>>4)][co = 16ct + (l&15)].
// flip = 1 (KS = 8): the input gradient's weights, W'[co' = ci][ci' = co][tap] = W[co][ci][8 - tap],
// output channels ci >= Cin zero.
__global__ void torus_pack_kernel(const float *__restrict__ w, int Cin, int KS, int flip, float *__restrict__ wpk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kTaps * KS * 2 * 64) return;
    const int l = i & 63, ct = (i >> 6) & 1, s = (i >> 7) % KS, tap = i / (128 * KS);
    const int oc = ct * 16 + (l & 15);   // output channel of this conv
    const int ic = s * 4 + (l >> 4);     // input channel of this conv
    float v = 0.f;
    if (!flip) {
        if (ic < Cin) v = w[(oc * Cin + ic) * kTaps + tap];
    } else {
        if (oc < Cin) v = w[(ic * Cin + oc) * kTaps + (kTaps - 1 - tap)];
    }
    wpk[i] = v;
}

// Zero-padded board conv weights: W (Cout, cin_total, 3, 3) restricted to input channels [ci0, ci0 + 32) ->
// per 32-channel output chunk the packed [tap][8][ct][64] layout of torus_pack_kernel.
__global__ void board_pack_kernel(const float *__restrict__ w, int nchunks, int cin_total, int ci0,
                                  float *__restrict__ wpk) {
    constexpr int kNW = kTaps * 8 * 2 * 64;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nchunks * kNW) return;
    const int chunk = i / kNW, j = i - chunk * kNW;
    const int l = j & 63, ct = (j >> 6) & 1, s = (j >> 7) % 8, tap = j / (128 * 8);
    const int oc = chunk * kCo + ct * 16 + (l & 15);
    const int ic = s * 4 + (l >> 4);
    wpk[i] = w[((int64_t)oc * cin_total + ci0 + ic) * kTaps + tap];
}

// ------------------------------------------------------------------ weight gradient
// partial[block]: [tap][ci 32][co 32] then db [32]
template <int KS, bool VEC>
__global__ __launch_bounds__(kThreads) void torus_wgrad_kernel(const float *__restrict__ x,
                                                               const float *__restrict__ dy, int64_t N, int Cin,
                                                               int H, int W, float *__restrict__ partial) {
    constexpr int kNLdX = VEC ? (KS * 4 * kMaxCells / 4 + 63) / 64 : (KS * 4 * kMaxCells + 63) / 64;
    constexpr int kNLdG = (kCo * kMaxCells / 4 + 63) / 64;   // dy samples: 32*HW floats
    constexpr int kJT = (KS * 4 + 15) / 16;                   // ci tiles
    constexpr int kPart = kTaps * kCo * kCo + kCo;
    __shared__ float lds[2 * kWaves * kTile];                 // per wave: x tile, dy tile
    __shared__ int nbr_tab[kMaxCells * kTaps];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int HW = H * W;
    const float inv_hw = 1.0f / (float)HW;
    const int in_elem = Cin * HW, g_elem = kCo * HW;
    float *xs = lds + wave * kTile;
    float *gs = lds + (kWaves + wave) * kTile;
    for (int i = threadIdx.x; i < kMaxCells * kTaps; i += kThreads) {
        const int q = i / kTaps, t = i - q * kTaps;
        nbr_tab[i] = q < HW ? torus_nbr(q, H, W, t) : 0;   // cells past the board: dy is zero there
    }
    for (int i = lane; i < kTile; i += 64) { xs[i] = 0.f; gs[i] = 0.f; }
    __syncthreads();

    f32x4 acc[kTaps][2][kJT];
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int jt = 0; jt < kJT; ++jt) acc[t][it][jt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float bsum[2] = {0.f, 0.f};

    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t n = (int64_t)blockIdx.x * kWaves + wave;
    Stage<VEC, kNLdX> sx;
    Stage<VEC, VEC ? kNLdG : (kCo * kMaxCells + 63) / 64> sg;
    if (n < N) {
        sx.load(x + n * in_elem, in_elem, lane);
        sg.load(dy + n * g_elem, g_elem, lane);
    }
    const int i16 = lane & 15, kk = lane >> 4;
    for (; n < N; n += stride) {
        sx.to_lds(xs, in_elem, HW, inv_hw, lane);
        sg.to_lds(gs, g_elem, HW, inv_hw, lane);
        lds_fence();
        const int64_t next = n + stride;
        if (next < N) {
            sx.load(x + next * in_elem, in_elem, lane);
            sg.load(dy + next * g_elem, g_elem, lane);
        }
#pragma unroll 2
        for (int ks = 0; ks < kKCells; ++ks) {
            const int cell = ks * 4 + kk;
            const float a0 = gs[i16 * kS + cell];
            const float a1 = gs[(16 + i16) * kS + cell];
            bsum[0] += a0;
            bsum[1] += a1;
            const int *nb = nbr_tab + cell * kTaps;
#pragma unroll
            for (int t = 0; t < kTaps; ++t) {
                const int p = nb[t];
#pragma unroll
                for (int jt = 0; jt < kJT; ++jt) {
                    const float b = xs[(jt * 16 + i16) * kS + p];
                    acc[t][0][jt] = mfma(a0, b, acc[t][0][jt]);
                    acc[t][1][jt] = mfma(a1, b, acc[t][1][jt]);
                }
            }
        }
        lds_fence();
    }
    // fold the 4 waves in a fixed order ((w0 + w1) + w2) + w3 through the (now free) tile LDS;
    // one partial per workgroup
    float *red = lds;
    float *bred = lds + kPart;   // [wave][k group][32]
    static_assert(2 * kWaves * kTile >= kPart + kWaves * 4 * kCo, "fold buffer");
    __syncthreads();
#pragma unroll 1
    for (int w = 0; w < kWaves; ++w) {
        if (wave == w) {
#pragma unroll
            for (int t = 0; t < kTaps; ++t)
#pragma unroll
                for (int it = 0; it < 2; ++it)
#pragma unroll
                    for (int jt = 0; jt < kJT; ++jt)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            // C[i = co][j = ci]: row = (lane>>4)*4 + r, col = lane & 15
                            const int co = it * 16 + (lane >> 4) * 4 + r;
                            const int ci = jt * 16 + (lane & 15);
                            float *d = red + (t * kCo + ci) * kCo + co;
                            *d = w == 0 ? acc[t][it][jt][r] : *d + acc[t][it][jt][r];
                        }
#pragma unroll
            for (int it = 0; it < 2; ++it) bred[(wave * 4 + kk) * kCo + it * 16 + i16] = bsum[it];
        }
        __syncthreads();
    }
    float *out = partial + (int64_t)blockIdx.x * kPart;
    for (int i = threadIdx.x; i < kTaps * kCo * kCo; i += kThreads) out[i] = red[i];
    if (threadIdx.x < kCo) {
        float b = 0.f;
        for (int i = 0; i < kWaves * 4; ++i) b += bred[i * kCo + threadIdx.x];
        out[kTaps * kCo * kCo + threadIdx.x] = b;
    }
}

// Weight gradient on the exact bf16 split (default with hrl_torus_set_split; Cin = 32, float4 layout).
// Per tap dW[tap] (co x ci) is one v_mfma_f32_32x32x16_bf16 tile: dW[tap] += dY (co x 16 cells) .
// X_tap (16 cells x ci) over the 5 k-steps of a sample (80 cells, dY zero past the board), six partial
// products per k-step (hrl_split.h), 270 MFMAs of 32 cycles per sample against the fp32 kernel's 720
// 16x16x4 MFMAs of 32 cycles.  Lane l = (r = l & 31, h = l >> 5) holds cells 8h..8h+7 of the k-step:
// A[co = r][cell] from the fp32 dY tile (two ds_read_b128: rows of kSG = 84 floats), split once per k-step
// and reused by the 9 taps; B[cell][ci = r] = X[r][nbr(cell, tap)] gathered from X split ONCE per sample
// into LDS as 64-bit slots (hi | mid << 16, lo): a gather is one ds_read_b64 (row stride 162 dwords: a
// half-wave's 32 rows cover the 64 banks once), three permutes build the fragments.  A cell's
// neighbours come from three packed (row part | column part << 16) words.  The bias gradient sums the
// A values.  Waves fold in a fixed order: deterministic.
constexpr int kSG = 84;   // dY tile row stride: 16-byte aligned rows, conflict-free ds_read_b128
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma32(const uint4 &a, const uint4 &b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

// APPLY (round 5): dY is not read but formed in the staging from the BatchNorm that follows the conv,
// dY = (((g [out > 0] - gmean) - (y - mean) k) invstd) gamma per channel (bn_bwd_apply_kernel<4, false, 2>'s
// operations, hrl_bn_backward_apply_masked), and written to dy_out for the input gradient: the separate masked
// apply pass (3 reads + 1 write of the activation) becomes 2 extra reads here.  The block output's mask
// [out > 0] is recomputed as [([x +] (y alpha + beta)) > 0] (residual: the block's input x is its residual),
// the forward's own operations (bn_res_apply_kernel, torus_conv_ps_kernel's prologue), so out is not read.
// X32 = false: x has Cin < 32 channels (GeeseNet's 17-channel stem, dword loads); rows Cin..31 stay zero.
struct WgArgs {
    const float *x, *dy;
    int64_t N;
    int Cin, H, W;
    float *partial;
    const float *yb, *gb, *mean, *invstd, *gamma, *kcoef, *gmean, *alpha, *beta;   // APPLY
    float *dy_out;
    bool residual;
};

template <bool APPLY, bool X32>
__global__ __launch_bounds__(kThreads) void torus_wgrad_split_kernel(WgArgs args) {
    const float *__restrict__ x = args.x;
    const float *__restrict__ dy = args.dy;
    const int64_t N = args.N;
    const int H = args.H, W = args.W, Cin = X32 ? kCo : args.Cin;
    float *__restrict__ partial = args.partial;
    constexpr int kNLd = (kCo * kMaxCells / 4 + 63) / 64;   // float4 per lane per sample tensor
    constexpr int kStemCin = 17;                             // !X32: the only narrower input (shape_ok)
    constexpr int kNLdS = (kStemCin * kMaxCells + 63) / 64; // !X32: x floats per lane
    constexpr int kPart = kTaps * kCo * kCo + kCo;
    constexpr int kHalf = kMaxCells / 2;
    __shared__ __attribute__((aligned(16))) float gs_all[kWaves][kCo * kSG];   // dY [co][cell]
    __shared__ uint2 xs_all[kWaves][kCo * kS];                                  // X (hi | mid << 16, lo) [ci][cell]
    __shared__ uint32_t nbp_tab[kMaxCells * 3];   // per cell and d: (row (r + d - 1) * W) | (column (c + d - 1)) << 16
    __shared__ float bnc[APPLY ? 7 * kCo + 1 : 1];   // APPLY: mean, k, gmean, invstd, gamma, alpha, beta (+1 pad)
    static_assert(sizeof(gs_all) + sizeof(xs_all) >= (kPart + kWaves * 2 * kCo) * sizeof(float), "fold buffer");
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int HW = H * W;
    const float inv_hw = 1.0f / (float)HW;
    const int n_elem = kCo * HW, nv = n_elem / 4, x_elem = Cin * HW;
    float *gs = gs_all[wave];
    uint2 *xs = xs_all[wave];
    if constexpr (APPLY) {
        if (threadIdx.x < kCo) {
            const int c = threadIdx.x;
            bnc[c] = args.mean[c];
            bnc[kCo + c] = args.kcoef[c];
            bnc[2 * kCo + c] = args.gmean[c];
            bnc[3 * kCo + c] = args.invstd[c];
            bnc[4 * kCo + c] = args.gamma ? args.gamma[c] : 1.0f;
            bnc[5 * kCo + c] = args.alpha[c];
            bnc[6 * kCo + c] = args.beta[c];
        }
        if (threadIdx.x == kCo) bnc[7 * kCo] = 0.f;
    }
    for (int i = threadIdx.x; i < kMaxCells * 3; i += kThreads) {
        const int q = i / 3, d = i - q * 3;
        uint32_t v = 0u;   // cells past the board: dY is zero there, any cell will do
        if (q < HW) {
            const int r = q / W, c = q - r * W;
            int rr = r + d - 1, cc = c + d - 1;
            rr = rr < 0 ? rr + H : (rr >= H ? rr - H : rr);
            cc = cc < 0 ? cc + W : (cc >= W ? cc - W : cc);
            v = (uint32_t)(rr * W) | ((uint32_t)cc << 16);
        }
        nbp_tab[i] = v;
    }
    for (int i = lane; i < kCo * kSG; i += 64) gs[i] = 0.f;
    for (int i = lane; i < kCo * kS; i += 64) xs[i] = make_uint2(0u, 0u);
    __syncthreads();

    f32x16 acc[kTaps];
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    float bsum = 0.f;
    const int r = lane & 31, h = lane >> 5;

    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t n = (int64_t)blockIdx.x * kWaves + wave;
    float4 sx[X32 ? kNLd : 1], sg[kNLd], sy[APPLY ? kNLd : 1];
    float sxs[X32 ? 1 : kNLdS];
    auto load = [&](int64_t m) {
        if constexpr (X32) {
            const float4 *xp = reinterpret_cast<const float4 *>(x + m * n_elem);
#pragma unroll
            for (int k = 0; k < kNLd; ++k) sx[k] = xp[min(k * 64 + lane, nv - 1)];
        } else {
            const float *xp = x + m * x_elem;
#pragma unroll
            for (int k = 0; k < kNLdS; ++k) sxs[k] = xp[min(k * 64 + lane, x_elem - 1)];
        }
        const float4 *gp = reinterpret_cast<const float4 *>((APPLY ? args.gb : dy) + m * n_elem);
#pragma unroll
        for (int k = 0; k < kNLd; ++k) sg[k] = gp[min(k * 64 + lane, nv - 1)];
        if constexpr (APPLY) {
            const float4 *yp = reinterpret_cast<const float4 *>(args.yb + m * n_elem);
#pragma unroll
            for (int k = 0; k < kNLd; ++k) sy[k] = yp[min(k * 64 + lane, nv - 1)];
        }
    };
    if (n < N) load(n);
    for (; n < N; n += stride) {
        if constexpr (!X32) {
#pragma unroll
            for (int k = 0; k < kNLdS; ++k) {
                const int e = opaque(k * 64 + lane);
                if (e < x_elem) {
                    const int c = fdiv(e, inv_hw);
                    uint32_t hb, mb, lb;
                    hrl_split::split3(sxs[k], hb, mb, lb);
                    xs[c * kS + (e - c * HW)] = make_uint2(hb | (mb << 16), lb);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kNLd; ++k) {
            const int i = k * 64 + lane;
            if (i < nv) {
                const Quad q(i, HW, inv_hw);
                float g4[4] = {sg[k].x, sg[k].y, sg[k].z, sg[k].w};
                const float x4[4] = {sx[X32 ? k : 0].x, sx[X32 ? k : 0].y, sx[X32 ? k : 0].z, sx[X32 ? k : 0].w};
                if constexpr (APPLY) {
                    const float y4[4] = {sy[k].x, sy[k].y, sy[k].z, sy[k].w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int c = q.c0 + (q.wrap(j, HW) ? 1 : 0);
                        const float z = y4[j] * bnc[5 * kCo + c] + bnc[6 * kCo + c];
                        const float o = (X32 && args.residual) ? x4[j] + z : z;   // relu(o) > 0 <=> o > 0
                        const float gv = o > 0.f ? g4[j] : 0.f;
                        const float t = (y4[j] - bnc[c]) * bnc[kCo + c];
                        g4[j] = (((gv - bnc[2 * kCo + c]) - t) * bnc[3 * kCo + c]) * bnc[4 * kCo + c];
                    }
                    reinterpret_cast<float4 *>(args.dy_out + n * n_elem)[i] = make_float4(g4[0], g4[1], g4[2], g4[3]);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool w = q.wrap(j, HW);
                    const int c = q.c0 + (w ? 1 : 0), cell = q.r0 + j - (w ? HW : 0);
                    if constexpr (X32) {
                        uint32_t hb, mb, lb;
                        hrl_split::split3(x4[j], hb, mb, lb);
                        xs[c * kS + cell] = make_uint2(hb | (mb << 16), lb);
                    }
                    gs[c * kSG + cell] = g4[j];
                }
            }
            if constexpr (APPLY) __builtin_amdgcn_sched_barrier(0);
        }
        lds_fence();
        if (n + stride < N) load(n + stride);   // in flight during the MFMAs

#pragma unroll 1
        for (int ks = 0; ks < kMaxCells / 16; ++ks) {
            const int cell0 = ks * 16 + 8 * h;
            const float4 g0 = *reinterpret_cast<const float4 *>(gs + r * kSG + cell0);
            const float4 g1 = *reinterpret_cast<const float4 *>(gs + r * kSG + cell0 + 4);
            const float av[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum += av[j];
            uint4 Ah, Am, Al;
            hrl_split::split8(av, Ah, Am, Al);
            uint32_t nbp[8][3];
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int d = 0; d < 3; ++d) nbp[j][d] = nbp_tab[(cell0 + j) * 3 + d];
            const uint2 *xrow = xs + r * kS;
#pragma unroll
            for (int t = 0; t < kTaps; ++t) {
                uint32_t hm[8], lo[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint2 v = xrow[(nbp[j][t / 3] & 0xffffu) + (nbp[j][t % 3] >> 16)];
                    hm[j] = v.x;
                    lo[j] = v.y;
                }
                uint32_t bh[4], bm[4], bl[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    bh[d] = __builtin_amdgcn_perm(hm[2 * d + 1], hm[2 * d], 0x05040100u);   // hi(e0) | hi(e1) << 16
                    bm[d] = __builtin_amdgcn_perm(hm[2 * d + 1], hm[2 * d], 0x07060302u);   // mid(e0) | mid(e1) << 16
                    bl[d] = lo[2 * d] | (lo[2 * d + 1] << 16);
                }
                const uint4 Bh = make_uint4(bh[0], bh[1], bh[2], bh[3]);
                const uint4 Bm = make_uint4(bm[0], bm[1], bm[2], bm[3]);
                const uint4 Bl = make_uint4(bl[0], bl[1], bl[2], bl[3]);
                f32x16 c = acc[t];
                c = mfma32(Al, Bh, c);   // smallest terms first
                c = mfma32(Am, Bm, c);
                c = mfma32(Ah, Bl, c);
                c = mfma32(Am, Bh, c);
                c = mfma32(Ah, Bm, c);
                c = mfma32(Ah, Bh, c);
                acc[t] = c;
            }
        }
        lds_fence();   // the tiles are rewritten for the next sample
    }
    (void)kHalf;
    // fold the 4 waves in a fixed order ((w0 + w1) + w2) + w3: red[tap][ci][co], then db per (wave, half)
    float *red = reinterpret_cast<float *>(gs_all);
    float *bred = red + kPart;
    __syncthreads();
#pragma unroll 1
    for (int w = 0; w < kWaves; ++w) {
        if (wave == w) {
#pragma unroll
            for (int t = 0; t < kTaps; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    // C/D: col = lane & 31 (ci), row = (reg & 3) + 8 (reg >> 2) + 4h (co)
                    const int co = (i & 3) + 8 * (i >> 2) + 4 * h;
                    float *d = red + (t * kCo + r) * kCo + co;
                    *d = w == 0 ? acc[t][i] : *d + acc[t][i];
                }
            bred[(wave * 2 + h) * kCo + r] = bsum;
        }
        __syncthreads();
    }
    float *out = partial + (int64_t)blockIdx.x * kPart;
    for (int i = threadIdx.x; i < kTaps * kCo * kCo; i += kThreads) out[i] = red[i];
    if (threadIdx.x < kCo) {
        float b = 0.f;
        for (int i = 0; i < kWaves * 2; ++i) b += bred[i * kCo + threadIdx.x];
        out[kTaps * kCo * kCo + threadIdx.x] = b;
    }
}

// fold per-workgroup partials (fixed order, fp64) into dW (32, Cin, 3, 3) and db (32)
__global__ __launch_bounds__(256) void torus_wgrad_reduce_kernel(const float *__restrict__ partial, int nparts,
                                                                 int Cin, float *__restrict__ dw,
                                                                 float *__restrict__ db) {
    constexpr int kPart = kTaps * kCo * kCo + kCo;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // partial index
    if (i >= kPart) return;
    double s = 0.0;
    for (int w = 0; w < nparts; ++w) s += (double)partial[(int64_t)w * kPart + i];
    if (i < kTaps * kCo * kCo) {
        const int co = i % kCo, ci = (i / kCo) % kCo, tap = i / (kCo * kCo);
        if (ci < Cin) dw[(co * Cin + ci) * kTaps + tap] = (float)s;
    } else if (db) {
        db[i - kTaps * kCo * kCo] = (float)s;
    }
}

// ------------------------------------------------------------------ GeeseNet head pooling
// hungry_geese.py:52-53: head[n, c] = sum_q h[n, c, q] * x[n, 0, q], avg[n, c] = mean_q h[n, c, q].
// One wave per sample: the sample is staged [c][cell] in LDS (coalesced float4 loads), then lane l sums
// channel l & 31 over the cells, lanes 0-31 the x-weighted sum and 32-63 the mean (sum / HW, as the
// reference's CPU mean: sum then divide).
// (round 5: each sample's loads are issued together and the next sample's are in flight during this one's sums;
// the per-float4 loops waited for every iteration's loads in turn)
__global__ __launch_bounds__(kThreads) void torus_head_pool_kernel(const float *__restrict__ h,
                                                                   const float *__restrict__ x, int64_t N, int HW,
                                                                   int64_t x_stride, float *__restrict__ head,
                                                                   float *__restrict__ avg) {
    constexpr int kNV = kCo * kMaxCells / 4 / 64;   // float4 per lane of an 80-cell sample
    constexpr int kNX = kMaxCells / 64 + 1;         // x0 cells per lane
    __shared__ float tiles[kWaves * kTile];
    __shared__ float x0s[kWaves][kMaxCells];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float *tile = tiles + wave * kTile;
    float *x0 = x0s[wave];
    const float inv_hw = 1.0f / (float)HW;
    const int nv = kCo * HW / 4;
    const int c = lane & 31;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    float4 v[kNV];
    float xv[kNX];
    auto load = [&](int64_t m) __attribute__((always_inline)) {
        const float4 *src = reinterpret_cast<const float4 *>(h + m * (kCo * HW));
#pragma unroll
        for (int k = 0; k < kNV; ++k) v[k] = src[min(k * 64 + lane, nv - 1)];
#pragma unroll
        for (int k = 0; k < kNX; ++k) xv[k] = x[m * x_stride + min(k * 64 + lane, HW - 1)];
    };
    int64_t n = (int64_t)blockIdx.x * kWaves + wave;
    if (n < N) load(n);
    for (; n < N; n += stride) {
#pragma unroll
        for (int k = 0; k < kNV; ++k) {
            const int i = k * 64 + lane;
            if (i < nv) {
                const float v4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
                const Quad q(i, HW, inv_hw);
#pragma unroll
                for (int j = 0; j < 4; ++j) tile[q.slot(j, HW)] = v4[j];
            }
        }
#pragma unroll
        for (int k = 0; k < kNX; ++k)
            if (k * 64 + lane < HW) x0[k * 64 + lane] = xv[k];
        lds_fence();
        if (n + stride < N) load(n + stride);   // in flight during the sums
        float acc = 0.f;
        if (lane < 32) {
            for (int q = 0; q < HW; ++q) acc += tile[c * kS + q] * x0[q];
            head[n * kCo + c] = acc;
        } else {
            for (int q = 0; q < HW; ++q) acc += tile[c * kS + q];
            avg[n * kCo + c] = acc / (float)HW;
        }
        lds_fence();
    }
}

// the backward of both poolings as CPU autograd computes it (mul backward dhead*x0, mean backward davg / HW,
// summed):
// g[n, c, q] = dhead[n, c] * x[n, 0, q] + davg[n, c] / HW; one wave per sample, float4 stores.  The sample's
// dhead / davg / x0 go through LDS, the next sample's loads in flight during this one's stores.
__global__ __launch_bounds__(kThreads) void torus_head_unpool_kernel(const float *__restrict__ dhead,
                                                                     const float *__restrict__ davg,
                                                                     const float *__restrict__ x, int64_t N, int HW,
                                                                     int64_t x_stride, float *__restrict__ g) {
    constexpr int kNX = kMaxCells / 64 + 1;
    __shared__ float sds[kWaves][2 * kCo + kMaxCells];   // dhead [32] | davg [32] | x0 [80]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float *sd = sds[wave];
    const float inv_hw = 1.0f / (float)HW;
    const float fhw = (float)HW;
    const int nv = kCo * HW / 4;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    float dv, xv[kNX];
    auto load = [&](int64_t m) __attribute__((always_inline)) {
        dv = lane < kCo ? dhead[m * kCo + lane] : davg[m * kCo + lane - kCo];
#pragma unroll
        for (int k = 0; k < kNX; ++k) xv[k] = x[m * x_stride + min(k * 64 + lane, HW - 1)];
    };
    int64_t n = (int64_t)blockIdx.x * kWaves + wave;
    if (n < N) load(n);
    for (; n < N; n += stride) {
        sd[lane] = dv;
#pragma unroll
        for (int k = 0; k < kNX; ++k)
            if (k * 64 + lane < HW) sd[2 * kCo + k * 64 + lane] = xv[k];
        lds_fence();
        if (n + stride < N) load(n + stride);
        float4 *dst = reinterpret_cast<float4 *>(g + n * (kCo * HW));
        for (int i = lane; i < nv; i += 64) {
            const Quad q(i, HW, inv_hw);
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool w = q.wrap(j, HW);
                const int c = q.c0 + (w ? 1 : 0);
                const int cell = q.r0 + j - (w ? HW : 0);
                o[j] = sd[c] * sd[2 * kCo + cell] + sd[kCo + c] / fhw;
            }
            dst[i] = make_float4(o[0], o[1], o[2], o[3]);
        }
        lds_fence();
    }
}

constexpr int kGridConv = 512;    // 2 workgroups per CU (78 KB LDS each)
constexpr int kGridWgrad = 256;   // 1 workgroup per CU (83 KB of tiles + the neighbour table)

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int grid_for(int64_t N, int cap) {
    const int64_t blocks = (N + kWaves - 1) / kWaves;
    return (int)(blocks < cap ? blocks : cap);
}

bool shape_ok(int64_t N, int64_t Cin, int64_t Cout, int64_t H, int64_t W) {
    return N >= 1 && Cout == kCo && (Cin == 17 || Cin == 32) && H >= 1 && W >= 1 && H * W <= kMaxCells &&
           N * Cin * H * W < ((int64_t)1 << 40);
}

constexpr int64_t kPackFloats = kTaps * 8 * 2 * 64;
constexpr int64_t kPartFloats = kTaps * kCo * kCo + kCo;

// Forward / input-gradient arithmetic: exact-split bf16 MFMA (1, default) or fp32 MFMA (0).
int g_split = 1;
// The split 32-channel torus forward / input gradient: 2 = pre-split images (torus_conv_ps_kernel, default),
// 1 = per-tap splits (torus_conv_kernel).  Bit-identical results.
int g_form = 2;

// torus_conv_ps_kernel launch: the 4-wave kernel's blocks pairwise (its partial rows: grid_for(N, kGridConv))
template <int PRO, bool STATS, bool SUMS>
void launch_ps(const ConvArgs &a, hipStream_t s) {
    const int nvb = grid_for(a.N, kGridConv);
    hipLaunchKernelGGL((torus_conv_ps_kernel<PRO, STATS, SUMS>), dim3((nvb + 1) / 2), dim3(kPThreads), 0, s, a, nvb);
}

}  // namespace

extern "C" {

int hrl_torus_set_split(int on) {
    const int prev = g_split;
    g_split = on ? 1 : 0;
    return prev;
}

int hrl_torus_set_form(int form) {
    const int prev = g_form;
    if (form == 1 || form == 2) g_form = form;
    return prev;
}

int64_t hrl_torus_workspace_bytes(int64_t N) {
    if (N < 1) return -1;
    return (kPackFloats + (int64_t)grid_for(N, kGridWgrad) * kPartFloats) * 4;
}

int64_t hrl_torus_stats_blocks(int64_t N) { return N < 1 ? -1 : grid_for(N, kGridConv); }

int hrl_torus_conv_forward(const float *x, int64_t N, int64_t Cin, int64_t Cout, int64_t H, int64_t W,
                           const float *weight, const float *bias, int flip, float *y, double *part,
                           const float *add, const float *add_mask, void *workspace, int64_t workspace_bytes,
                           void *stream) {
    if (!shape_ok(N, Cin, Cout, H, W) || !x || !weight || !y || !workspace) return HRL_EINVAL;
    if (flip && bias) return HRL_EINVAL;
    if ((add == nullptr) != (add_mask == nullptr)) return HRL_EINVAL;
    if (workspace_bytes < hrl_torus_workspace_bytes(N)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the conv this launch computes: forward Cin -> 32; flip: 32 -> Cin (the forward's adjoint)
    const int in_c = flip ? (int)kCo : (int)Cin;
    const int out_c = flip ? (int)Cin : (int)kCo;
    const bool ps = g_split && g_form == 2;   // the pre-split kernel (32 or 17 input channels, KS = 8 packing)
    const int KS = in_c == 17 && !ps ? 5 : 8;
    float *wpk = static_cast<float *>(workspace);
    hipLaunchKernelGGL(torus_pack_kernel, dim3((kTaps * KS * 128 + 255) / 256), dim3(256), 0, s, weight, (int)Cin, KS,
                       flip, wpk);
    int rc = status();
    if (rc) return rc;
    const int HW = (int)(H * W);
    // float4 staging: a float4 spans at most two channels, so boards of at least 4 cells
    const bool vec = HW >= 4 && (in_c * HW) % 4 == 0 && aligned16(x);
    const bool vec_out = HW >= 4 && (out_c * HW) % 4 == 0 && aligned16(y) &&
                         (!add || (aligned16(add) && aligned16(add_mask)));
    ConvArgs a{};
    a.x = x; a.N = N; a.Cin = in_c; a.H = (int)H; a.W = (int)W; a.wpk = wpk; a.bias = bias; a.out_c = out_c;
    a.vec_out = vec_out; a.y = y; a.part = part; a.add = add; a.add_mask = add_mask; a.co_total = out_c;
    const dim3 grid(grid_for(N, kGridConv)), block(kThreads);
#define HRL_TORUS_LAUNCH(KS_, VEC_, ST_)                                                                           \
    do {                                                                                                         \
        if (g_split) hipLaunchKernelGGL((torus_conv_kernel<KS_, VEC_, ST_, true>), grid, block, 0, s, a);        \
        else hipLaunchKernelGGL((torus_conv_kernel<KS_, VEC_, ST_, false>), grid, block, 0, s, a);               \
    } while (0)
    const bool st = part != nullptr;
    if (ps) {
        if (st) launch_ps<0, true, false>(a, s); else launch_ps<0, false, false>(a, s);
        return status();
    }
    if (KS == 8) {
        if (vec) { if (st) HRL_TORUS_LAUNCH(8, true, true); else HRL_TORUS_LAUNCH(8, true, false); }
        else { if (st) HRL_TORUS_LAUNCH(8, false, true); else HRL_TORUS_LAUNCH(8, false, false); }
    } else {
        if (st) HRL_TORUS_LAUNCH(5, false, true); else HRL_TORUS_LAUNCH(5, false, false);
    }
#undef HRL_TORUS_LAUNCH
    return status();
}

int64_t hrl_board_conv_workspace_bytes(int64_t Cout) {
    return (Cout < kCo || Cout % kCo) ? -1 : (Cout / kCo) * kTaps * 8 * 2 * 64 * 4;
}

int hrl_board_conv_pack(const float *weight, int64_t w_cin_total, int64_t w_ci0, int64_t Cout, void *packed,
                        int64_t packed_bytes, void *stream) {
    if (!weight || !packed || w_ci0 < 0 || w_ci0 + kCo > w_cin_total || hrl_board_conv_workspace_bytes(Cout) < 0 ||
        packed_bytes < hrl_board_conv_workspace_bytes(Cout))
        return HRL_EINVAL;
    const int nchunks = (int)(Cout / kCo);
    const int npk = nchunks * kTaps * 8 * 2 * 64;
    hipLaunchKernelGGL(board_pack_kernel, dim3((npk + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                       weight, nchunks, (int)w_cin_total, (int)w_ci0, static_cast<float *>(packed));
    return status();
}

int hrl_board_conv_forward_packed(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const void *packed,
                                  int64_t Cout, const float *bias, float *y, void *stream) {
    const int64_t HW = H * W;
    if (N < 1 || Cin != kCo || H < 1 || W < 1 || HW < 4 || HW > kMaxCells || !x || !packed || !y) return HRL_EINVAL;
    if (hrl_board_conv_workspace_bytes(Cout) < 0 || N * Cout * HW >= ((int64_t)1 << 40)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nchunks = (int)(Cout / kCo);
    const float *wpk = static_cast<const float *>(packed);
    ConvArgs a{};
    a.x = x; a.N = N; a.Cin = kCo; a.H = (int)H; a.W = (int)W; a.wpk = wpk; a.bias = bias; a.out_c = kCo;
    a.vec_out = (kCo * HW) % 4 == 0 && aligned16(y); a.y = y; a.co_total = (int)Cout;
    const bool vec = (kCo * HW) % 4 == 0 && aligned16(x);
    // ~kGridConv workgroups in all: each loads its chunk's 37 KB of packed weights once, so at large N it
    // must walk many samples (one sample per wave per chunk reloaded the weights every 4 samples)
    const int cap = kGridConv / nchunks > 0 ? kGridConv / nchunks : 1;
    const dim3 grid(grid_for(N, cap), nchunks), block(kThreads);
#define HRL_BOARD_LAUNCH(VEC_, MT_)                                                                                 \
    do {                                                                                                          \
        if (g_split) hipLaunchKernelGGL((torus_conv_kernel<8, VEC_, false, true, 0, false, MT_, true>), grid, block, 0, \
                                        s, a);                                                                    \
        else hipLaunchKernelGGL((torus_conv_kernel<8, VEC_, false, false, 0, false, MT_, true>), grid, block, 0, s, a); \
    } while (0)
    if (HW <= 48) { if (vec) HRL_BOARD_LAUNCH(true, 3); else HRL_BOARD_LAUNCH(false, 3); }
    else { if (vec) HRL_BOARD_LAUNCH(true, 5); else HRL_BOARD_LAUNCH(false, 5); }
#undef HRL_BOARD_LAUNCH
    return status();
}

int hrl_board_conv_forward(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const float *weight,
                           int64_t w_cin_total, int64_t w_ci0, int64_t Cout, const float *bias, float *y,
                           void *workspace, int64_t workspace_bytes, void *stream) {
    const int rc = hrl_board_conv_pack(weight, w_cin_total, w_ci0, Cout, workspace, workspace_bytes, stream);
    if (rc) return rc;
    return hrl_board_conv_forward_packed(x, N, Cin, H, W, workspace, Cout, bias, y, stream);
}

int hrl_torus_unit_forward(const float *y_prev, const float *res, const float *alpha, const float *beta, float *h,
                           int64_t N, int64_t H, int64_t W, const float *weight, const float *bias, float *y,
                           double *part, void *workspace, int64_t workspace_bytes, void *stream) {
    if (!shape_ok(N, kCo, kCo, H, W) || !y_prev || !alpha || !beta || !h || !weight || !y || !part || !workspace)
        return HRL_EINVAL;
    if (workspace_bytes < hrl_torus_workspace_bytes(N)) return HRL_EINVAL;
    if (H * W < 4 || (kCo * H * W) % 4 != 0 || !aligned16(y_prev) || !aligned16(h) || !aligned16(y) || (res && !aligned16(res)))
        return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    float *wpk = static_cast<float *>(workspace);
    hipLaunchKernelGGL(torus_pack_kernel, dim3((kTaps * 8 * 128 + 255) / 256), dim3(256), 0, s, weight, (int)kCo, 8, 0,
                       wpk);
    int rc = status();
    if (rc) return rc;
    ConvArgs a{};
    a.x = y_prev; a.N = N; a.Cin = kCo; a.H = (int)H; a.W = (int)W; a.wpk = wpk; a.bias = bias; a.out_c = kCo;
    a.vec_out = true; a.y = y; a.part = part; a.res = res; a.alpha = alpha; a.beta = beta; a.hout = h;
    a.co_total = kCo;
    if (g_split && g_form == 2) {
        if (res) launch_ps<2, true, false>(a, s); else launch_ps<1, true, false>(a, s);
        return status();
    }
    const dim3 grid(grid_for(N, kGridConv)), block(kThreads);
    if (res) {
        if (g_split) hipLaunchKernelGGL((torus_conv_kernel<8, true, true, true, 2>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((torus_conv_kernel<8, true, true, false, 2>), grid, block, 0, s, a);
    } else {
        if (g_split) hipLaunchKernelGGL((torus_conv_kernel<8, true, true, true, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((torus_conv_kernel<8, true, true, false, 1>), grid, block, 0, s, a);
    }
    return status();
}

int hrl_torus_unit_input_grad(const float *dy, int64_t N, int64_t H, int64_t W, const float *weight, const float *g,
                              const float *out, float *dh, const float *h_mask, const float *y_prev,
                              const float *mean_prev, double *part, void *workspace, int64_t workspace_bytes,
                              void *stream) {
    if (!shape_ok(N, kCo, kCo, H, W) || !dy || !weight || !g || !out || !dh || !h_mask || !y_prev || !mean_prev ||
        !part || !workspace)
        return HRL_EINVAL;
    if (workspace_bytes < hrl_torus_workspace_bytes(N)) return HRL_EINVAL;
    if (H * W < 4 || (kCo * H * W) % 4 != 0) return HRL_EINVAL;
    for (const void *p : {(const void *)dy, (const void *)g, (const void *)out, (const void *)dh, (const void *)h_mask,
                          (const void *)y_prev})
        if (!aligned16(p)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    float *wpk = static_cast<float *>(workspace);
    hipLaunchKernelGGL(torus_pack_kernel, dim3((kTaps * 8 * 128 + 255) / 256), dim3(256), 0, s, weight, (int)kCo, 8, 1,
                       wpk);
    int rc = status();
    if (rc) return rc;
    ConvArgs a{};
    a.x = dy; a.N = N; a.Cin = kCo; a.H = (int)H; a.W = (int)W; a.wpk = wpk; a.out_c = kCo; a.vec_out = true;
    a.y = dh; a.part = part; a.add = g; a.add_mask = out; a.hmask = h_mask; a.yprev = y_prev; a.mean = mean_prev;
    a.co_total = kCo;
    if (g_split && g_form == 2) {
        launch_ps<0, false, true>(a, s);
        return status();
    }
    const dim3 grid(grid_for(N, kGridConv)), block(kThreads);
    if (g_split) hipLaunchKernelGGL((torus_conv_kernel<8, true, false, true, 0, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((torus_conv_kernel<8, true, false, false, 0, true>), grid, block, 0, s, a);
    return status();
}

int hrl_torus_conv_wgrad(const float *x, const float *dy, int64_t N, int64_t Cin, int64_t Cout, int64_t H, int64_t W,
                         float *dweight, float *dbias, void *workspace, int64_t workspace_bytes, void *stream) {
    if (!shape_ok(N, Cin, Cout, H, W) || !x || !dy || !dweight || !workspace) return HRL_EINVAL;
    if (workspace_bytes < hrl_torus_workspace_bytes(N)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int HW = (int)(H * W);
    const bool vec = HW >= 4 && (Cin * HW) % 4 == 0 && (kCo * HW) % 4 == 0 && aligned16(x) && aligned16(dy);
    const int grid = grid_for(N, kGridWgrad);
    float *partial = static_cast<float *>(workspace) + kPackFloats;
    const bool dy_vec = HW >= 4 && aligned16(dy);   // 32 * HW is a multiple of 4
    WgArgs wa{};
    wa.x = x; wa.dy = dy; wa.N = N; wa.Cin = (int)Cin; wa.H = (int)H; wa.W = (int)W; wa.partial = partial;
    if (Cin == kCo && vec && g_split) {
        hipLaunchKernelGGL((torus_wgrad_split_kernel<false, true>), dim3(grid), dim3(kThreads), 0, s, wa);
    } else if (Cin != kCo && dy_vec && g_split) {
        hipLaunchKernelGGL((torus_wgrad_split_kernel<false, false>), dim3(grid), dim3(kThreads), 0, s, wa);
    } else if (Cin == kCo) {
        if (vec)
            hipLaunchKernelGGL((torus_wgrad_kernel<8, true>), dim3(grid), dim3(kThreads), 0, s, x, dy, N, (int)Cin,
                               (int)H, (int)W, partial);
        else
            hipLaunchKernelGGL((torus_wgrad_kernel<8, false>), dim3(grid), dim3(kThreads), 0, s, x, dy, N, (int)Cin,
                               (int)H, (int)W, partial);
    } else {
        hipLaunchKernelGGL((torus_wgrad_kernel<5, false>), dim3(grid), dim3(kThreads), 0, s, x, dy, N, (int)Cin,
                           (int)H, (int)W, partial);
    }
    int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(torus_wgrad_reduce_kernel, dim3((int)((kPartFloats + 255) / 256)), dim3(256), 0, s, partial,
                       grid, (int)Cin, dweight, dbias);
    return status();
}

int hrl_torus_conv_wgrad_bn(const float *x, int64_t N, int64_t Cin, int64_t H, int64_t W, const float *y,
                            const float *g, const float *alpha, const float *beta, int residual, const float *gamma,
                            const float *save_mean, const float *save_invstd, const float *kcoef, const float *gmean,
                            float *dy, float *dweight, float *dbias, void *workspace, int64_t workspace_bytes,
                            void *stream) {
    if (!shape_ok(N, Cin, kCo, H, W) || !x || !y || !g || !alpha || !beta || !save_mean || !save_invstd || !kcoef ||
        !gmean || !dy || !dweight || !workspace)
        return HRL_EINVAL;
    if (residual && Cin != kCo) return HRL_EINVAL;
    if (workspace_bytes < hrl_torus_workspace_bytes(N) || !g_split) return HRL_EINVAL;
    const int64_t HW = H * W;
    if (HW < 4) return HRL_EINVAL;
    for (const void *p : {(const void *)y, (const void *)g, (const void *)dy})
        if (!aligned16(p)) return HRL_EINVAL;
    const bool x32 = Cin == kCo;
    if (x32 && !aligned16(x)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = grid_for(N, kGridWgrad);
    float *partial = static_cast<float *>(workspace) + kPackFloats;
    WgArgs wa{};
    wa.x = x; wa.N = N; wa.Cin = (int)Cin; wa.H = (int)H; wa.W = (int)W; wa.partial = partial;
    wa.yb = y; wa.gb = g; wa.mean = save_mean; wa.invstd = save_invstd; wa.gamma = gamma;
    wa.kcoef = kcoef; wa.gmean = gmean; wa.alpha = alpha; wa.beta = beta; wa.dy_out = dy; wa.residual = residual != 0;
    if (x32) hipLaunchKernelGGL((torus_wgrad_split_kernel<true, true>), dim3(grid), dim3(kThreads), 0, s, wa);
    else hipLaunchKernelGGL((torus_wgrad_split_kernel<true, false>), dim3(grid), dim3(kThreads), 0, s, wa);
    int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(torus_wgrad_reduce_kernel, dim3((int)((kPartFloats + 255) / 256)), dim3(256), 0, s, partial,
                       grid, (int)Cin, dweight, dbias);
    return status();
}

int hrl_torus_head_pool(const float *h, const float *x, int64_t N, int64_t H, int64_t W, int64_t x_stride,
                        float *head, float *avg, void *stream) {
    const int64_t HW = H * W;
    if (N < 1 || HW < 4 || HW > kMaxCells || !h || !x || !head || !avg || x_stride < HW || !aligned16(h)) return HRL_EINVAL;
    hipLaunchKernelGGL(torus_head_pool_kernel, dim3(grid_for(N, 2048)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), h, x, N, (int)HW, x_stride, head, avg);
    return status();
}

int hrl_torus_head_unpool(const float *dhead, const float *davg, const float *x, int64_t N, int64_t H, int64_t W,
                          int64_t x_stride, float *g, void *stream) {
    const int64_t HW = H * W;
    if (N < 1 || HW < 4 || HW > kMaxCells || !dhead || !davg || !x || !g || x_stride < HW || !aligned16(g))
        return HRL_EINVAL;
    hipLaunchKernelGGL(torus_head_unpool_kernel, dim3(grid_for(N, 2048)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), dhead, davg, x, N, (int)HW, x_stride, g);
    return status();
}

}  // extern "C"
