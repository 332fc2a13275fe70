// hrl_heads.hip — the TicTacToe net's two output heads as one fused pass (gfx950).
//
// SimpleConv2dModel (handyrl/envs/tictactoe.py:35-49, 59-60) ends with two
// Heads on the body output h (N, 32, 3, 3):
//   conv1x1 32 -> Cm (+bias) -> LeakyReLU(0.1) -> flatten -> Linear(9*Cm -> out, no bias)
// with (Cm, out) = (2, 9) for the policy and (1, 1) for the value (the model
// applies tanh).  As library GEMMs this is ~10 launches forward and backward
// on skinny shapes ([N,288]x[288,27], [N,18]x[18,9], ...) that hipBLASLt runs
// at a fraction of HBM bandwidth, plus the board-weight expansions and the
// activation kernels.  Here:
//
// heads_fwd_kernel: one wave owns 64 rows (samples) at a time; h streams in
//   slices of 4 channels (36 floats per row) with coalesced float4 loads into
//   an LDS tile [row][36] (stride 37: one row per lane, conflict-free), the
//   next slice in flight while this one is consumed; each lane accumulates
//   its row's 27 conv outputs in registers (bias first, channels in order),
//   applies the LeakyReLU and the two fc heads.  Writes the activations a
//   (N x 18 policy, N x 9 value: the backward's only saved state) and the
//   outputs (N x 9, N x 1).  151 MB read at N = 131072 (HBM-bound).
// heads_bwd_kernel: per row, dz = (dp . Wp | dv . Wv) * leaky'(a); the input
//   gradient dh[c, q] = sum_m W1[m, c] dz[m, q] leaves through the same LDS
//   tile with coalesced stores while h streams in again for the conv weight
//   gradient; the conv weight/bias gradients accumulate per lane in
//   registers, are folded across the wave with a fixed butterfly, and per
//   wave into partials; fc_grad_kernel forms the fc weight gradients
//   dp^T a_p and dv^T a_v (one thread per weight, rows in a fixed order) into
//   the same partial rows; heads_reduce_kernel folds every column with a
//   fixed-shape tree (deterministic).  151 MB read + 151 MB written.
// With the body's last BatchNorm fused in front (BnIn; nn._ChainHeadsFn) both
// kernels read that BN's raw input y and apply relu(y*alpha + beta) per slice,
// and the backward also emits the BN's backward sums, so the body's output
// never reaches HBM and its last BN needs no separate reduce pass.
// Numerics: fp32 throughout (-ffp-contract=off; the forward's conv and fc sums are explicit fused multiply-adds,
// packed on cell pairs, and the fused BN apply keeps bn_apply_kernel's separate multiply and add); sums in a fixed
// order; the LeakyReLU and its gradient follow torch (x > 0 ? x : x * 0.1f).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kC = 32;                 // body channels
constexpr int kHW = 9;                 // 3x3 board
constexpr int kRow = kC * kHW;         // 288 floats per sample
constexpr int kMP = 2, kMV = 1;        // conv channels of the policy / value head
constexpr int kM = kMP + kMV;          // 3
constexpr int kZ = kM * kHW;           // 27 activations per sample
constexpr int kZP = kMP * kHW;         // 18 (policy fc inputs)
constexpr int kOP = 9;                 // policy outputs
constexpr int kSC = 4;                 // channels per slice
constexpr int kNS = kC / kSC;          // 8 slices
constexpr int kSF = kSC * kHW;         // 36 floats per row slice
constexpr int kSV = kSF / 4;           // 9 float4 per row slice
constexpr int kTS = kSF + 1;           // LDS row stride (odd)
constexpr float kSlope = 0.1f;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int hu32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int hu32x4 __attribute__((ext_vector_type(4)));

// parameter-gradient partial layout (per workgroup): dW1 [3][32] | db1 [3] | dWp [9][18] | dWv [9]
constexpr int kGW1 = 0;
constexpr int kGB1 = kGW1 + kM * kC;
constexpr int kGWP = kGB1 + kM;
constexpr int kGWV = kGWP + kOP * kZP;
constexpr int kGN = kGWV + kHW;        // 270

struct Weights {
    const float *w1p, *w1v, *b1p, *b1v, *wp, *wv;
};

// Optional BatchNorm + ReLU in front of the heads (the body's last BN, fused_chain_heads): h = relu(y*alpha + beta)
// computed as each slice is read; the backward also forms that BN's backward sums (sum g*m, sum g*m*(y - mean),
// m = [y*alpha + beta > 0]) per channel, fp64 per workgroup -> part[block][32][2] (hrl_bn_finalize_backward).
struct BnIn {
    const float *alpha, *beta, *mean;
    double *part;
};

__device__ __forceinline__ float bn_relu(float y, float a, float b) {
    const float t = y * a + b;   // bn_apply_kernel's float operations
    return t < 0.f ? 0.f : t;
}

__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float w1_at(const Weights &w, int m, int c) {
    return m < kMP ? w.w1p[m * kC + c] : w.w1v[(m - kMP) * kC + c];
}

// the 64 rows [base, base+nrows) x slice s (channels 4s..4s+3): 576 float4, 9 per lane
__device__ __forceinline__ void load_slice(const float *__restrict__ h, int64_t base, int nrows, int s, int lane,
                                           float4 (&st)[kSV]) {
#pragma unroll
    for (int k = 0; k < kSV; ++k) {
        const int i = k * 64 + lane;
        const int r = i / kSV, c4 = i - r * kSV;
        const int rr = r < nrows ? r : nrows - 1;
        st[k] = *reinterpret_cast<const float4 *>(h + (base + rr) * kRow + s * kSF + c4 * 4);
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t heads_rsrc(const void *base, uint32_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                             0x00020000);
}

// load_slice through a buffer descriptor over the 64-row block (rows past N read 0): lane offsets vo[k] are
// slice-invariant, the slice's 144-byte step is the scalar offset -- 9 VGPRs of addressing instead of 9 pointers
__device__ __forceinline__ void slice_offsets(int lane, uint32_t (&vo)[kSV]) {
#pragma unroll
    for (int k = 0; k < kSV; ++k) {
        const int i = k * 64 + lane;
        const int r = i / kSV, c4 = i - r * kSV;
        vo[k] = (uint32_t)((r * kRow + c4 * 4) * 4);
    }
}

__device__ __forceinline__ void load_slice_buf(__amdgpu_buffer_rsrc_t rs, const uint32_t (&vo)[kSV], int s,
                                               float4 (&st)[kSV]) {
#pragma unroll
    for (int k = 0; k < kSV; ++k) {
        const hu32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo[k], s * kSF * 4, 0);
        st[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
    }
}

__device__ __forceinline__ void slice_to_lds(const float4 (&st)[kSV], float *tile, int lane) {
#pragma unroll
    for (int k = 0; k < kSV; ++k) {
        const int i = k * 64 + lane;
        const int r = i / kSV, c4 = i - r * kSV;
        float *d = tile + r * kTS + c4 * 4;
        d[0] = st[k].x; d[1] = st[k].y; d[2] = st[k].z; d[3] = st[k].w;
    }
}

// ------------------------------------------------------------------ forward
// nf contiguous floats from LDS to global: float4 per lane where whole (dst 16-byte aligned: a 64-row block's
// run), the tail one float at a time
__device__ __forceinline__ void store_rows(const float *src, float *dst, int nf, int lane) {
    if (reinterpret_cast<uintptr_t>(dst) & 15) {   // an unaligned caller buffer: one float per lane
        for (int e = lane; e < nf; e += 64) dst[e] = src[e];
        return;
    }
    for (int i = lane; 4 * i < nf; i += 64) {
        if (4 * i + 4 <= nf) {
            reinterpret_cast<float4 *>(dst)[i] = *reinterpret_cast<const float4 *>(src + 4 * i);
        } else {
            for (int e = 4 * i; e < nf; ++e) dst[e] = src[e];
        }
    }
}

__global__ __launch_bounds__(64, 2) void heads_fwd_kernel(const float *__restrict__ h, int64_t N, Weights w, BnIn bn,
                                                       float *__restrict__ a_p, float *__restrict__ a_v,
                                                       float *__restrict__ p_out, float *__restrict__ v_out,
                                                       bool tanh_v) {
    __shared__ __attribute__((aligned(16))) float tile[64 * kTS];
    __shared__ float sw1[kM * kC], sb1[kM], swp[kOP * kZP], swv[kHW], sal[kC], sbe[kC];
    const int lane = threadIdx.x;
    if (bn.alpha && lane < kC) {
        sal[lane] = bn.alpha[lane];
        sbe[lane] = bn.beta[lane];
    }
    for (int i = lane; i < kM * kC; i += 64) sw1[i] = w1_at(w, i / kC, i % kC);
    if (lane < kM) sb1[lane] = lane < kMP ? w.b1p[lane] : w.b1v[lane - kMP];
    for (int i = lane; i < kOP * kZP; i += 64) swp[i] = w.wp[i];
    if (lane < kHW) swv[lane] = w.wv[lane];
    __syncthreads();
    uint32_t vo[kSV];
    slice_offsets(lane, vo);

    for (int64_t base = (int64_t)blockIdx.x * 64; base < N; base += (int64_t)gridDim.x * 64) {
        // Wp / W1 / the BN constants are re-read from LDS per block: hoisted out of the loop they held ~170 VGPRs
        // (2 waves per SIMD, one 2.3 KB slice in flight per wave)
        asm volatile("" ::: "memory");
        const int nrows = (int)min<int64_t>(64, N - base);
        // z[m][q] = b1[m] + sum_c W1[m][c] h[c][q] (fused multiply-adds, channels in order): cells 0..7 as 4 pairs
        f32x2 zp[kM][4];
        float z8[kM];
#pragma unroll
        for (int m = 0; m < kM; ++m) {
#pragma unroll
            for (int k = 0; k < 4; ++k) zp[m][k] = (f32x2){sb1[m], sb1[m]};
            z8[m] = sb1[m];
        }
        // two slices in flight: st0 holds the even slices, st1 the odd ones; slice s + 2 is issued into the
        // registers slice s just left for LDS
        float4 st0[kSV], st1[kSV];
        const __amdgpu_buffer_rsrc_t rh = heads_rsrc(h + base * kRow, (uint32_t)(nrows * kRow * 4));
        load_slice_buf(rh, vo, 0, st0);
        load_slice_buf(rh, vo, 1, st1);
        auto slice = [&](float4 (&st)[kSV], int s) __attribute__((always_inline)) {
            slice_to_lds(st, tile, lane);
            lds_fence();
            if (s + 2 < kNS) load_slice_buf(rh, vo, s + 2, st);   // in flight during the FMAs
#pragma unroll
            for (int cc = 0; cc < kSC; ++cc) {
                // channel c's 9 cells as 4 pairs + 1: packed fp32 (v_pk_mul / v_pk_add / v_pk_fma) on cell pairs;
                // one channel's LDS reads at a time (hoisted, the slice's 36 + its weights crowd the registers)
                asm volatile("" ::: "memory");
                const int c = s * kSC + cc;
                const float *tr = tile + lane * kTS + cc * kHW;
                f32x2 xp[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) xp[k] = (f32x2){tr[2 * k], tr[2 * k + 1]};
                float x8 = tr[8];
                if (bn.alpha) {   // bn_apply_kernel's float operations (a multiply, then an add), then the ReLU
                    const float al = sal[c], be = sbe[c];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const f32x2 t = xp[k] * (f32x2){al, al} + (f32x2){be, be};
                        xp[k] = (f32x2){t.x < 0.f ? 0.f : t.x, t.y < 0.f ? 0.f : t.y};
                    }
                    x8 = bn_relu(x8, al, be);
                }
#pragma unroll
                for (int m = 0; m < kM; ++m) {
                    const float wv1 = sw1[m * kC + c];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        zp[m][k] = __builtin_elementwise_fma((f32x2){wv1, wv1}, xp[k], zp[m][k]);
                    z8[m] = __builtin_fmaf(wv1, x8, z8[m]);
                }
            }
            lds_fence();   // every lane's reads done before the next slice overwrites the tile
        };
#pragma unroll 1
        for (int s = 0; s < kNS; s += 2) {
            slice(st0, s);
            slice(st1, s + 1);
        }
        float a[kZ];
#pragma unroll
        for (int m = 0; m < kM; ++m) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[m * kHW + 2 * k] = zp[m][k].x;
                a[m * kHW + 2 * k + 1] = zp[m][k].y;
            }
            a[m * kHW + 8] = z8[m];
        }
#pragma unroll
        for (int j = 0; j < kZ; ++j) a[j] = a[j] > 0.f ? a[j] : a[j] * kSlope;
        float p[kOP];
#pragma unroll
        for (int k = 0; k < kOP; ++k) {
            asm volatile("" ::: "memory");   // one output's 18 weights in flight at a time, not all 162
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < kZP; ++j) t = __builtin_fmaf(swp[k * kZP + j], a[j], t);
            p[k] = t;
        }
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < kHW; ++q) v = __builtin_fmaf(swv[q], a[kZP + q], v);
        v = tanh_v ? tanhf(v) : v;   // the model's torch.tanh on the value head, folded
        // the block's outputs leave through the (dead) tile as contiguous runs: one row per lane straight from
        // registers is a 36- or 72-byte stride across the wave's 64 rows, many partial lines per store
        // (tile = [a_p 64 x 18 | a_v 64 x 9 | p 64 x 9 | v 64] = 64 x 37 floats)
        float *to_ap = tile, *to_av = tile + 64 * kZP, *to_p = to_av + 64 * kHW, *to_v = to_p + 64 * kOP;
#pragma unroll
        for (int j = 0; j < kZP; ++j) to_ap[lane * kZP + j] = a[j];
#pragma unroll
        for (int q = 0; q < kHW; ++q) to_av[lane * kHW + q] = a[kZP + q];
#pragma unroll
        for (int k = 0; k < kOP; ++k) to_p[lane * kOP + k] = p[k];
        to_v[lane] = v;
        lds_fence();
        store_rows(to_p, p_out + base * kOP, nrows * kOP, lane);
        store_rows(to_v, v_out + base, nrows, lane);
        if (a_p) {
            store_rows(to_ap, a_p + base * kZP, nrows * kZP, lane);
            store_rows(to_av, a_v + base * kHW, nrows * kHW, lane);
        }
        lds_fence();   // the stores' LDS reads are done before the next block's slices land in the tile
    }
}

// ------------------------------------------------------------------ backward
__device__ __forceinline__ float wave_sum(float v) {
    // fixed butterfly over the 64 lanes: every lane ends with the same, order-fixed total
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(64) void heads_bwd_kernel(const float *__restrict__ h, int64_t N, Weights w, BnIn bn,
                                                       const float *__restrict__ a_p, const float *__restrict__ a_v,
                                                       const float *__restrict__ dp, const float *__restrict__ dv,
                                                       const float *__restrict__ vt, float *__restrict__ dv_raw,
                                                       float *__restrict__ dh, float *__restrict__ part) {
    __shared__ float tile[64 * kTS];
    __shared__ float sw1[kM * kC], swp[kOP * kZP], swv[kHW], sal[kC], sbe[kC], smu[kC];
    __shared__ float gw1[kM * kC * 64];   // per-lane conv weight-gradient accumulators [m*32 + c][lane]
    __shared__ float gbn[kC * 2 * 64];    // per-lane BN backward sums [c][2][lane] (bn.part)
    const int lane = threadIdx.x;
    for (int i = lane; i < kM * kC; i += 64) sw1[i] = w1_at(w, i / kC, i % kC);
    for (int i = lane; i < kOP * kZP; i += 64) swp[i] = w.wp[i];
    if (lane < kHW) swv[lane] = w.wv[lane];
    for (int i = lane; i < kM * kC * 64; i += 64) gw1[i] = 0.f;
    if (bn.alpha && lane < kC) {
        sal[lane] = bn.alpha[lane];
        sbe[lane] = bn.beta[lane];
        smu[lane] = bn.part ? bn.mean[lane] : 0.f;
    }
    if (bn.part)
        for (int i = lane; i < kC * 2 * 64; i += 64) gbn[i] = 0.f;
    __syncthreads();

    float gb1[kM];
#pragma unroll
    for (int i = 0; i < kM; ++i) gb1[i] = 0.f;

    for (int64_t base = (int64_t)blockIdx.x * 64; base < N; base += (int64_t)gridDim.x * 64) {
        const int nrows = (int)min<int64_t>(64, N - base);
        const bool valid = lane < nrows;
        const int64_t n = base + (valid ? lane : 0);
        float4 st[kSV];
        load_slice(h, base, nrows, 0, lane, st);   // in flight while dz is formed
        float a[kZ], g[kOP], gv;
#pragma unroll
        for (int j = 0; j < kZP; ++j) a[j] = a_p[n * kZP + j];
#pragma unroll
        for (int q = 0; q < kHW; ++q) a[kZP + q] = a_v[n * kHW + q];
#pragma unroll
        for (int k = 0; k < kOP; ++k) g[k] = valid ? dp[n * kOP + k] : 0.f;
        gv = valid ? dv[n] : 0.f;
        if (vt) {   // tanh backward (grad * (1 - y*y), as torch's CPU kernel), kept for fc_grad_kernel
            gv = gv * (1.f - vt[n] * vt[n]);
            if (valid) dv_raw[n] = gv;
        }
        // the activation gradient (the fc weight gradients are dp^T a_p, dv^T a_v: host side)
        float dz[kZ];
#pragma unroll
        for (int j = 0; j < kZP; ++j) {
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < kOP; ++k) t += g[k] * swp[k * kZP + j];
            dz[j] = a[j] > 0.f ? t : t * kSlope;
        }
#pragma unroll
        for (int q = 0; q < kHW; ++q) {
            const float t = gv * swv[q];
            dz[kZP + q] = a[kZP + q] > 0.f ? t : t * kSlope;
        }
#pragma unroll
        for (int m = 0; m < kM; ++m) {
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < kHW; ++q) t += dz[m * kHW + q];
            gb1[m] += t;
        }
#pragma unroll 1
        for (int s = 0; s < kNS; ++s) {
            slice_to_lds(st, tile, lane);
            lds_fence();
            if (s + 1 < kNS) load_slice(h, base, nrows, s + 1, lane, st);
            float x[kSF], yraw[kSF];
#pragma unroll
            for (int j = 0; j < kSF; ++j) x[j] = yraw[j] = tile[lane * kTS + j];
            if (bn.alpha) {
#pragma unroll
                for (int j = 0; j < kSF; ++j) x[j] = bn_relu(x[j], sal[s * kSC + j / kHW], sbe[s * kSC + j / kHW]);
            }
            // conv weight gradient: dW1[m, c] += sum_q dz[m, q] * h[c, q]
#pragma unroll
            for (int m = 0; m < kM; ++m)
#pragma unroll
                for (int cc = 0; cc < kSC; ++cc) {
                    float t = 0.f;
#pragma unroll
                    for (int q = 0; q < kHW; ++q) t += dz[m * kHW + q] * x[cc * kHW + q];
                    gw1[(m * kC + s * kSC + cc) * 64 + lane] += t;   // this lane's own slot
                }
            // input gradient of this slice: dh[c, q] = sum_m W1[m, c] * dz[m, q] -> the lane's LDS row
            lds_fence();
#pragma unroll
            for (int cc = 0; cc < kSC; ++cc) {
                const int c = s * kSC + cc;
                float t1 = 0.f, t2 = 0.f;   // this row's BN backward sums of channel c
#pragma unroll
                for (int q = 0; q < kHW; ++q) {
                    float t = 0.f;
#pragma unroll
                    for (int m = 0; m < kM; ++m) t += sw1[m * kC + c] * dz[m * kHW + q];
                    tile[lane * kTS + cc * kHW + q] = t;
                    if (bn.part) {   // bn_bwd_reduce_kernel's mask and products
                        const float y = yraw[cc * kHW + q];
                        const float gm = (y * sal[c] + sbe[c] > 0.f) ? t : 0.f;
                        t1 += gm;
                        t2 += gm * (y - smu[c]);
                    }
                }
                if (bn.part) {
                    gbn[(c * 2 + 0) * 64 + lane] += t1;
                    gbn[(c * 2 + 1) * 64 + lane] += t2;
                }
            }
            lds_fence();
            // coalesced float4 stores of the 64 x 36 slice
#pragma unroll
            for (int k = 0; k < kSV; ++k) {
                const int i = k * 64 + lane;
                const int r = i / kSV, c4 = i - r * kSV;
                if (r < nrows) {
                    const float *sp = tile + r * kTS + c4 * 4;
                    *reinterpret_cast<float4 *>(dh + (base + r) * kRow + s * kSF + c4 * 4) =
                        make_float4(sp[0], sp[1], sp[2], sp[3]);
                }
            }
            lds_fence();
        }
    }
    // fold the lanes in a fixed order, one partial row per wave
    float *out = part + (int64_t)blockIdx.x * kGN;
    lds_fence();
    for (int i = lane; i < kM * kC; i += 64) {
        float t = 0.f;
        for (int l = 0; l < 64; ++l) t += gw1[i * 64 + l];
        out[kGW1 + i] = t;
    }
#pragma unroll
    for (int i = 0; i < kM; ++i) {
        const float t = wave_sum(gb1[i]);
        if (lane == 0) out[kGB1 + i] = t;
    }
    if (bn.part) {   // lanes in order, fp64: part[block][c][2]
        const int c = lane >> 1, k = lane & 1;
        double t = 0.0;
        for (int l = 0; l < 64; ++l) t += (double)gbn[(c * 2 + k) * 64 + l];
        bn.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = t;
    }
}

// ------------------------------------------------------------------ backward, lane-per-channel form
// heads_bwd_kernel keeps a row per lane, so its 3 x 32 conv weight-gradient and 32 x 2 BN-sum accumulators live in
// LDS (52 KB per one-wave workgroup: 3 waves per CU, <= 27 KB of loads in flight per CU; 107 us in the step, 3 TB/s).
// Here a lane owns (row half r = lane >> 5, channel c = lane & 31): per row pair it reads its channel's 9 cells, so
// its weight-gradient and BN-sum accumulators are 5 registers, W1[:, c] and the BN constants of c are 6 more.  h
// arrives in 8-row groups as contiguous float4s (9 per lane, one group ahead) through the wave's LDS tile, the lanes
// read their cells there and write dh in their place, and the group leaves as contiguous float4 stores (36-byte
// per-lane runs straight to and from HBM ran at half the rate); with the row block's small inputs and dz, 72 KB of
// LDS per 4-wave workgroup, 2 per CU.
//  * stage (lanes 0..31, one row each): dz[m][q] = leaky'(a) * (dp . Wp | dv' . Wv) and db1's per-row sums, dz and
//    the row's dp / dv' / a_p / a_v into LDS;
//  * fc weight gradients: lane l owns weights l, l + 64, l + 128 of [dWp (9 x 18) | dWv (9)] and adds the block's
//    rows in order (the products of fc_grad_kernel, dv' = the tanh backward's output);
//  * main loop over the block's groups and their row pairs: x (BN + ReLU applied when fused), dW1[m][c] +=
//    sum_q dz[m][q] x[q], dh[q] = sum_m W1[m][c] dz[m][q] (the old kernel's operation order per element), the BN
//    sums, dh through the tile;
//  * the accumulators fold over the two row halves and the four waves in a fixed order into this workgroup's
//    partial row (heads_reduce_kernel folds the workgroups) -- deterministic.
constexpr int kBR = 32;                // rows per block (one wave)
constexpr int kDZS = 28;               // LDS stride of a row's dz (27 + pad: 7 x ds_read_b128)
constexpr int kSMS = 40;               // LDS stride of a row's small inputs: g[9] gv a_p[18] a_v[9] pad
constexpr int kSmG = 0, kSmGV = 9, kSmAP = 10, kSmAV = 28;
constexpr int kFcN = kOP * kZP + kHW;  // 171 fc weights
constexpr int kWaves2 = 4;
constexpr int kGR = 8;                 // rows per contiguous load / store group
constexpr int kGV = kGR * kRow / 4 / 64;   // 9 float4 per lane per group

// rows [row0, row0 + 8) of h as 9 contiguous float4 per lane (rows past N read 0)
__device__ __forceinline__ void load_group(__amdgpu_buffer_rsrc_t rh, int64_t row0, int lane, hu32x4 (&st)[kGV]) {
    const uint32_t ob = (uint32_t)(row0 * kRow * 4);
#pragma unroll
    for (int k = 0; k < kGV; ++k) st[k] = __builtin_amdgcn_raw_buffer_load_b128(rh, ob + (k * 64 + lane) * 16, 0, 0);
}

template <bool BN>
__global__ __launch_bounds__(256, 2) void heads_bwd2_kernel(const float *__restrict__ h, int64_t N, Weights w, BnIn bn,
                                                         const float *__restrict__ a_p, const float *__restrict__ a_v,
                                                         const float *__restrict__ dp, const float *__restrict__ dv,
                                                         const float *__restrict__ vt, float *__restrict__ dh,
                                                         float *__restrict__ part) {
    // the row blocks' dz and small inputs; after the loop the same bytes hold the folds
    __shared__ __attribute__((aligned(16))) float sdz[kWaves2][kBR * kDZS];
    __shared__ __attribute__((aligned(16))) float ssm[kWaves2][kBR * kSMS];
    __shared__ float swp[kOP * kZP], swv[kHW];
    __shared__ __attribute__((aligned(16))) float sx[kWaves2][kGR * kRow];   // a wave's 8-row group: x, then dh
    static_assert(sizeof(float) * kWaves2 * 64 * 8 <= sizeof(float) * kWaves2 * kBR * kSMS, "fold");
    static_assert(sizeof(double) * kWaves2 * 64 * 2 <= sizeof(float) * kWaves2 * kBR * kDZS, "foldd");
    float(*fold)[64 * 8] = reinterpret_cast<float(*)[64 * 8]>(&ssm[0][0]);
    double(*foldd)[64 * 2] = reinterpret_cast<double(*)[64 * 2]>(&sdz[0][0]);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 31, r = lane >> 5;
    for (int i = threadIdx.x; i < kOP * kZP; i += 256) swp[i] = w.wp[i];
    if (threadIdx.x < kHW) swv[threadIdx.x] = w.wv[threadIdx.x];
    float w1[kM];
#pragma unroll
    for (int m = 0; m < kM; ++m) w1[m] = w1_at(w, m, c);
    float al = 1.f, be = 0.f, mu = 0.f;
    if constexpr (BN) {
        al = bn.alpha[c];
        be = bn.beta[c];
        mu = bn.part ? bn.mean[c] : 0.f;
    }
    __syncthreads();
    float *dzs = sdz[wave];
    float *sm = ssm[wave];
    // per-lane accumulators: dW1[:, c] over this lane's rows, db1 (lanes < 32, per staged row), the fc weights the
    // lane owns, the BN sums of channel c
    float gw[kM] = {0.f, 0.f, 0.f}, gb[kM] = {0.f, 0.f, 0.f}, fc[3] = {0.f, 0.f, 0.f};
    double t1d = 0.0, t2d = 0.0;
    // fc weight i = lane + 64 s: (k, j) of dWp or q of dWv, as LDS offsets into a staged row
    int fo_g[3], fo_a[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int i = lane + 64 * s;
        const bool pol = i < kOP * kZP;
        fo_g[s] = pol ? kSmG + i / kZP : kSmGV;
        fo_a[s] = pol ? kSmAP + i % kZP : kSmAV + (i - kOP * kZP < kHW ? i - kOP * kZP : 0);
    }
    const __amdgpu_buffer_rsrc_t rh = heads_rsrc(h, (uint32_t)(N * kRow * 4));
    const __amdgpu_buffer_rsrc_t rd = heads_rsrc(dh, (uint32_t)(N * kRow * 4));
    const int64_t nblocks = (N + kBR - 1) / kBR;
    const int64_t wstep = (int64_t)gridDim.x * kWaves2;
    float *sxw = sx[wave];
    hu32x4 st[kGV];
    if ((int64_t)blockIdx.x * kWaves2 + wave < nblocks)
        load_group(rh, ((int64_t)blockIdx.x * kWaves2 + wave) * kBR, lane, st);
    for (int64_t blk = (int64_t)blockIdx.x * kWaves2 + wave; blk < nblocks; blk += wstep) {
        const int64_t base = blk * kBR;
        asm volatile("" ::: "memory");   // Wp / Wv are re-read from LDS per block, not held in 171 registers
        {
            // row lane & 31; the half-waves split its dz: r = 0 the policy cells j = 0..8 and the value head,
            // r = 1 the policy cells j = 9..17 (each dz the same 9-term sum in the same order as one lane alone)
            const int row = lane & (kBR - 1);
            const int64_t n = base + row;
            const bool valid = n < N;
            const int64_t nn = valid ? n : 0;
            const int j0 = r * kHW;          // this half's policy cells
            float ap[kHW], g[kOP];
#pragma unroll
            for (int j = 0; j < kHW; ++j) ap[j] = a_p[nn * kZP + j0 + j];
#pragma unroll
            for (int k = 0; k < kOP; ++k) g[k] = valid ? dp[nn * kOP + k] : 0.f;
            float dzp[kHW];
#pragma unroll
            for (int j = 0; j < kHW; ++j) {
                // one dz at a time: the compiler would otherwise issue all the products (packed) before any sum
                asm volatile("" ::: "memory");
                float t = 0.f;
#pragma unroll
                for (int k = 0; k < kOP; ++k) t += g[k] * swp[k * kZP + j0 + j];
                dzp[j] = ap[j] > 0.f ? t : t * kSlope;
            }
            {
                float t = 0.f;
#pragma unroll
                for (int q = 0; q < kHW; ++q) t += dzp[q];
                gb[r] += t;                  // db1[m = r]: lanes < 32 hold m = 0, lanes >= 32 m = 1
            }
            float *dzr = dzs + row * kDZS;
            float *smr = sm + row * kSMS;
#pragma unroll
            for (int j = 0; j < kHW; ++j) {
                dzr[j0 + j] = dzp[j];
                smr[kSmAP + j0 + j] = valid ? ap[j] : 0.f;
            }
            if (r == 0) {
                float av[kHW];
#pragma unroll
                for (int q = 0; q < kHW; ++q) av[q] = a_v[nn * kHW + q];
                float gv = valid ? dv[nn] : 0.f;
                if (vt) gv = gv * (1.f - vt[nn] * vt[nn]);   // tanh backward, torch's CPU operations
                float t2 = 0.f;
#pragma unroll
                for (int q = 0; q < kHW; ++q) {
                    const float t = gv * swv[q];
                    const float d = av[q] > 0.f ? t : t * kSlope;
                    dzr[kZP + q] = d;
                    t2 += d;
                    smr[kSmAV + q] = valid ? av[q] : 0.f;
                }
                gb[2] += t2;
                dzr[kZ] = 0.f;
#pragma unroll
                for (int k = 0; k < kOP; ++k) smr[kSmG + k] = g[k];
                smr[kSmGV] = gv;
            }
        }
        lds_fence();
        // fc weight gradients over the block's rows, in order
#pragma unroll 4
        for (int row = 0; row < kBR; ++row) {
            const float *smr = sm + row * kSMS;
#pragma unroll
            for (int s = 0; s < 3; ++s) fc[s] += smr[fo_g[s]] * smr[fo_a[s]];
        }
        // the block's four 8-row groups: x arrives as contiguous float4s (st, one group ahead) through this wave's
        // LDS tile; lane (r, c) reads its channel's 9 cells of rows 2j + r, writes dh in their place, and the group
        // leaves as contiguous float4 stores (36-byte per-lane runs straight from registers ran at half the rate)
#pragma unroll 1
        for (int g = 0; g < kBR / kGR; ++g) {
#pragma unroll
            for (int k = 0; k < kGV; ++k) *reinterpret_cast<hu32x4 *>(sxw + 4 * (k * 64 + lane)) = st[k];
            lds_fence();
            {   // the next group: this block's, or the wave's next block's first
                const int64_t nb = g + 1 < kBR / kGR ? base + kGR * (g + 1) : base + wstep * kBR;
                if (nb < N) {
                    load_group(rh, nb, lane, st);
                } else {   // past the batch: zeros (no stale rows, no offset past 32 bits)
#pragma unroll
                    for (int k = 0; k < kGV; ++k) st[k] = (hu32x4){0u, 0u, 0u, 0u};
                }
            }
#pragma unroll 1
            for (int jj = 0; jj < kGR / 2; ++jj) {
                const int lr = 2 * jj + r;             // row within the group
                float *xr = sxw + lr * kRow + c * kHW;
                float x[kHW];
#pragma unroll
                for (int q = 0; q < kHW; ++q) x[q] = xr[q];
                float dz[kZ + 1];
                const float4 *dzr = reinterpret_cast<const float4 *>(dzs + (kGR * g + lr) * kDZS);
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const float4 v = dzr[t];
                    dz[4 * t] = v.x; dz[4 * t + 1] = v.y; dz[4 * t + 2] = v.z; dz[4 * t + 3] = v.w;
                }
                float hx[kHW];
#pragma unroll
                for (int q = 0; q < kHW; ++q) hx[q] = BN ? bn_relu(x[q], al, be) : x[q];
                // conv weight gradient: dW1[m, c] += sum_q dz[m, q] * h[c, q]
#pragma unroll
                for (int m = 0; m < kM; ++m) {
                    float t = 0.f;
#pragma unroll
                    for (int q = 0; q < kHW; ++q) t += dz[m * kHW + q] * hx[q];
                    gw[m] += t;
                }
                // input gradient dh[c, q] = sum_m W1[m, c] dz[m, q], the BN sums of channel c
                float t1 = 0.f, t2 = 0.f;
#pragma unroll
                for (int q = 0; q < kHW; ++q) {
                    float t = 0.f;
#pragma unroll
                    for (int m = 0; m < kM; ++m) t += w1[m] * dz[m * kHW + q];
                    if constexpr (BN) {
                        if (bn.part) {   // bn_bwd_reduce_kernel's mask and products
                            const float gm = (x[q] * al + be > 0.f) ? t : 0.f;
                            t1 += gm;
                            t2 += gm * (x[q] - mu);
                        }
                    }
                    xr[q] = t;
                }
                t1d += (double)t1;
                t2d += (double)t2;
            }
            lds_fence();
            const uint32_t ob = (uint32_t)((base + kGR * g) * kRow * 4);
#pragma unroll
            for (int k = 0; k < kGV; ++k)   // rows past N: dropped (the descriptor's range)
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const hu32x4 *>(sxw + 4 * (k * 64 + lane)),
                                                       rd, ob + (k * 64 + lane) * 16, 0, 0);
            lds_fence();   // the tile's reads are done before the next group overwrites it
        }
        lds_fence();   // the block's LDS rows are read before the next block overwrites them
    }
    // fixed-order folds: lanes (r, c) of the 4 waves -> channel c; the wave's lanes < 32 -> db1; fc per lane
    __syncthreads();   // every wave is out of its loop: the staging LDS is free
    float *fw = fold[wave];
#pragma unroll
    for (int m = 0; m < kM; ++m) fw[m * 64 + lane] = gw[m];
#pragma unroll
    for (int m = 0; m < kM; ++m) fw[(3 + m) * 64 + lane] = gb[m];
    fw[6 * 64 + lane] = 0.f;
    foldd[wave][lane * 2] = t1d;
    foldd[wave][lane * 2 + 1] = t2d;
    __syncthreads();
    float *out = part + (int64_t)blockIdx.x * kGN;
    if (wave == 0) {
        // dW1[m][c]: lanes c and c + 32 of waves 0..3, in order
        for (int i = lane; i < kM * kC; i += 64) {
            const int m = i / kC, cc = i % kC;
            float t = 0.f;
            for (int wv = 0; wv < kWaves2; ++wv) t += fold[wv][m * 64 + cc] + fold[wv][m * 64 + cc + 32];
            out[kGW1 + i] = t;
        }
        if (lane < kM) {
            // db1[m]: the rows' lanes in order -- m = 0, 2 on lanes 0..31, m = 1 on lanes 32..63
            const int l0 = lane == 1 ? kBR : 0;
            float t = 0.f;
            for (int wv = 0; wv < kWaves2; ++wv)
                for (int l = 0; l < kBR; ++l) t += fold[wv][(3 + lane) * 64 + l0 + l];
            out[kGB1 + lane] = t;
        }
        if (BN && bn.part) {   // part[block][c][2], fp64: halves and waves in order
            const int cc = lane >> 1, k = lane & 1;
            double t = 0.0;
            for (int wv = 0; wv < kWaves2; ++wv) t += foldd[wv][cc * 2 + k] + foldd[wv][(cc + 32) * 2 + k];
            bn.part[((int64_t)blockIdx.x * kC + cc) * 2 + k] = t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 3; ++s) fw[s * 64 + lane] = fc[s];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            const int i = lane + 64 * s;
            if (i < kFcN) {
                float t = 0.f;
                for (int wv = 0; wv < kWaves2; ++wv) t += fold[wv][s * 64 + lane];
                out[kGWP + i] = t;
            }
        }
    }
}

// fc weight gradients: dWp[k][j] = sum_n dp[n,k] a_p[n,j], dWv[q] = sum_n dv[n] a_v[n,q]; workgroup b sums
// its row range (rows in order) into partial row b, columns kGWP.. (one thread per weight)
__global__ __launch_bounds__(256) void fc_grad_kernel(const float *__restrict__ a_p, const float *__restrict__ a_v,
                                                      const float *__restrict__ dp, const float *__restrict__ dv,
                                                      int64_t N, int64_t rows_per_block, float *__restrict__ part) {
    const int t = threadIdx.x;
    if (t >= kOP * kZP + kHW) return;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(N, r0 + rows_per_block);
    const bool pol = t < kOP * kZP;
    const int k = pol ? t / kZP : 0, j = pol ? t % kZP : t - kOP * kZP;
    // rows in order into one accumulator; the loads of 8 rows are issued ahead of their FMAs
    float acc = 0.f;
    int64_t n = r0;
    for (; n + 8 <= r1; n += 8) {
        float x[8], y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            x[u] = pol ? dp[(n + u) * kOP + k] : dv[n + u];
            y[u] = pol ? a_p[(n + u) * kZP + j] : a_v[(n + u) * kHW + j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += x[u] * y[u];
    }
    for (; n < r1; ++n) acc += pol ? dp[n * kOP + k] * a_p[n * kZP + j] : dv[n] * a_v[n * kHW + j];
    part[(int64_t)blockIdx.x * kGN + kGWP + t] = acc;
}

// fixed-order fold of the per-workgroup partials: one workgroup per column, a strided fp64 sum per
// thread, then a fixed-shape LDS tree (deterministic)
__global__ __launch_bounds__(256) void heads_reduce_kernel(const float *__restrict__ part, int nparts,
                                                           float *__restrict__ dw1p, float *__restrict__ dw1v,
                                                           float *__restrict__ db1p, float *__restrict__ db1v,
                                                           float *__restrict__ dwp, float *__restrict__ dwv) {
    __shared__ double red[256];
    const int i = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nparts; b += 256) s += (double)part[(int64_t)b * kGN + i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const float v = (float)red[0];
    if (i < kGB1) {
        const int m = i / kC, c = i % kC;
        if (m < kMP) dw1p[m * kC + c] = v;
        else dw1v[(m - kMP) * kC + c] = v;
    } else if (i < kGWP) {
        const int m = i - kGB1;
        if (m < kMP) db1p[m] = v;
        else db1v[m - kMP] = v;
    } else if (i < kGWV) {
        dwp[i - kGWP] = v;
    } else {
        dwv[i - kGWV] = v;
    }
}

// Workgroups (one wave each).  The backward's 51.9 KB of LDS lets 3 reside per CU, so 768 on the
// 256 CUs run in one round: its former 1024 ran as 768 + a tail of 256 at a third of the
// occupancy.  The forward (10.8 KB LDS, 230 VGPRs) keeps all 1024 resident.
constexpr int kGridFwd = 4096;   // one-wave workgroups: 64-row blocks, up to 4 waves per SIMD
constexpr int kGridBwd = 768;
constexpr int kGridBwd2 = 512;    // heads_bwd2_kernel: 2 four-wave workgroups per CU (72 KB LDS each)
int g_heads_bwd_form = 2;         // hrl_heads_set_bwd_form

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int grid_for(int64_t N, int cap = kGridBwd) {
    const int64_t blocks = (N + 63) / 64;
    return (int)(blocks < cap ? blocks : cap);
}

// the backward's workgroups (its partial rows): form 2 runs 4-wave workgroups over 32-row blocks
int grid_bwd(int64_t N) {
    if (g_heads_bwd_form != 2) return grid_for(N);
    const int64_t wgs = ((N + kBR - 1) / kBR + kWaves2 - 1) / kWaves2;
    return (int)(wgs < kGridBwd2 ? wgs : kGridBwd2);
}

}  // namespace

extern "C" {

// workspace: the per-workgroup partials, then dv through the folded tanh's backward (N floats)
int64_t hrl_heads_workspace_bytes(int64_t N) {
    return N < 1 ? -1 : ((int64_t)std::max(grid_for(N), grid_bwd(N)) * kGN + N) * 4;
}

int64_t hrl_heads_bn_parts(int64_t N) { return N < 1 ? -1 : grid_bwd(N); }

int hrl_heads_set_bwd_form(int form) {
    const int prev = g_heads_bwd_form;
    if (form == 1 || form == 2) g_heads_bwd_form = form;   // any other value only queries
    return prev;
}

int hrl_heads_forward(const float *h, int64_t N, const float *w1p, const float *b1p, const float *w1v,
                      const float *b1v, const float *wp, const float *wv, const float *bn_alpha, const float *bn_beta,
                      float *a_p, float *a_v, float *p_out, float *v_out, int tanh_v, void *stream) {
    if (N < 1 || !h || !w1p || !b1p || !w1v || !b1v || !wp || !wv || !p_out || !v_out) return HRL_EINVAL;
    if ((a_p == nullptr) != (a_v == nullptr) || (bn_alpha == nullptr) != (bn_beta == nullptr) || !aligned16(h))
        return HRL_EINVAL;
    const Weights w{w1p, w1v, b1p, b1v, wp, wv};
    const BnIn bn{bn_alpha, bn_beta, nullptr, nullptr};
    hipLaunchKernelGGL(heads_fwd_kernel, dim3(grid_for(N, kGridFwd)), dim3(64), 0, static_cast<hipStream_t>(stream), h, N, w,
                       bn, a_p, a_v, p_out, v_out, tanh_v != 0);
    return status();
}

int hrl_heads_backward(const float *h, int64_t N, const float *w1p, const float *w1v, const float *wp,
                       const float *wv, const float *bn_alpha, const float *bn_beta, const float *bn_mean,
                       double *bn_part, const float *a_p, const float *a_v, const float *dp, const float *dv,
                       const float *v_tanh, float *dh, float *dw1p, float *db1p, float *dw1v, float *db1v, float *dwp, float *dwv,
                       void *workspace, int64_t workspace_bytes, void *stream) {
    if (N < 1 || !h || !w1p || !w1v || !wp || !wv || !a_p || !a_v || !dp || !dv || !dh || !workspace)
        return HRL_EINVAL;
    const bool defer = !dw1p && !db1p && !dw1v && !db1v && !dwp && !dwv;   // partials left for a later fold
    if (!defer && (!dw1p || !db1p || !dw1v || !db1v || !dwp || !dwv)) return HRL_EINVAL;
    if (defer && g_heads_bwd_form != 2) return HRL_EINVAL;
    if ((bn_alpha == nullptr) != (bn_beta == nullptr) || (bn_part && (!bn_alpha || !bn_mean))) return HRL_EINVAL;
    if (!aligned16(h) || !aligned16(dh) || workspace_bytes < hrl_heads_workspace_bytes(N)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const Weights w{w1p, w1v, nullptr, nullptr, wp, wv};
    const BnIn bn{bn_alpha, bn_beta, bn_mean, bn_part};
    float *part = static_cast<float *>(workspace);
    if (g_heads_bwd_form == 2) {
        if ((N + kBR) * kRow * 4 >= (int64_t)1 << 32) return HRL_EINVAL;   // 32-bit buffer offsets (+ a block)
        const int grid = grid_bwd(N);
        if (bn_alpha)
            hipLaunchKernelGGL(heads_bwd2_kernel<true>, dim3(grid), dim3(256), 0, s, h, N, w, bn, a_p, a_v, dp, dv,
                               v_tanh, dh, part);
        else
            hipLaunchKernelGGL(heads_bwd2_kernel<false>, dim3(grid), dim3(256), 0, s, h, N, w, bn, a_p, a_v, dp, dv,
                               v_tanh, dh, part);
        const int rc = status();
        if (rc || defer) return rc;
        hipLaunchKernelGGL(heads_reduce_kernel, dim3(kGN), dim3(256), 0, s, part, grid, dw1p, dw1v, db1p, db1v, dwp,
                           dwv);
        return status();
    }
    const int grid = grid_for(N);
    float *dv_raw = part + (int64_t)grid * kGN;
    hipLaunchKernelGGL(heads_bwd_kernel, dim3(grid), dim3(64), 0, s, h, N, w, bn, a_p, a_v, dp, dv, v_tanh, dv_raw, dh,
                       part);
    int rc = status();
    if (rc) return rc;
    const int64_t rows = (N + grid - 1) / grid;
    hipLaunchKernelGGL(fc_grad_kernel, dim3(grid), dim3(256), 0, s, a_p, a_v, dp, v_tanh ? dv_raw : dv, N, rows, part);
    rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(heads_reduce_kernel, dim3(kGN), dim3(256), 0, s, part, grid, dw1p, dw1v, db1p, db1v, dwp,
                       dwv);
    return status();
}

}  // extern "C"
