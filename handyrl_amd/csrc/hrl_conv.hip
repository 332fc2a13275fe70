// hrl_conv.hip — 3x3 'same' convolution on a 3x3 board with fp32 MFMA (gfx950).
//
// The TicTacToe body (tictactoe.py:52-69) is three 32->32 3x3 convs on a 3x3
// board over N = B*T*P samples.  As a dense matrix the layer is the GEMM
// Y[N, 288] = X[N, 288] @ W_board[288, 288], but only 49 of the 81
// (input cell p, output cell q) 32x32 blocks of W_board are real taps: the
// others fall off the board.  These kernels skip them:
//
//   out[n, co, q] = sum_{p in nbhd(q)} sum_ci in[n, ci, p] * W[co, ci, tap(p, q)]
//
// with v_mfma_f32_16x16x4_f32 (exact fp32 products, k-ordered accumulation).
//
// conv3x3_kernel<PRO, STATS> (forward; also the input gradient, run on dY
// with the kernel flipped and transposed — a 'same' conv's adjoint):
//   * a workgroup = 4 waves; each wave owns a 16-row tile of the (N, C*9)
//     NCHW rows per iteration and walks row tiles grid-stride;
//   * the packed weights [tap][co-tile][ci][16] (36 KB) sit in LDS;
//   * each wave's A tile is 16 rows x 288 floats in LDS with a row stride of
//     290 (== 2 mod 32), conflict-free for the A fragment reads;
//   * the next row tile's global loads are issued before the MFMA loop and
//     land in registers while the MFMAs run;
//   * 9 output cells x 2 column tiles = 18 accumulators; the epilogue stages
//     the 16x288 output tile through LDS and leaves with coalesced 16-byte
//     stores;
//   * optional fusions with the BatchNorm+ReLU around it (PRO / STATS below)
//     so a conv -> BN -> ReLU chain writes each activation once.
//   Measured (tools/conv_bench.py, M = 131072): 125-138 us per launch, the
//   784 MFMAs per tile at ~1.7 GHz, the clock the chip holds under this
//   MFMA+LDS load on random data (MI355X_MICROARCH.md, DVFS give-back).
// conv3x3_wgrad_kernel (weight gradient): dW[tap][ci][co] accumulates
//   X^T dY over (row, (p,q) pairs with that tap) per wave (36 accumulators);
//   the 4 waves fold through LDS, and a wide reduce folds the per-workgroup
//   partials, both in a fixed order (deterministic).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"
#include "hrl_split.h"
#include "hrl_stamps.h"

namespace {

HRL_STAMP_DECL

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBoard = 3;                 // 3x3 board
constexpr int kCells = kBoard * kBoard;   // 9
constexpr int kTaps = 9;                  // 3x3 kernel
constexpr int kC = 32;                    // channels (in and out) per launch
constexpr int kRow = kC * kCells;         // 288 floats per sample
constexpr int kStride = kRow + 2;         // LDS row stride, == 2 (mod 32)
constexpr int kTile = 16;                 // rows per wave tile
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kVec = kTile * kRow / 4 / 64;   // float4 per lane per tile (18)

// tap index of input cell p feeding output cell q (dy, dx in 0..2), or -1
__host__ __device__ constexpr int tap_of(int p, int q) {
    const int dy = p / kBoard - q / kBoard + 1;
    const int dx = p % kBoard - q % kBoard + 1;
    return (dy < 0 || dy > 2 || dx < 0 || dx > 2) ? -1 : dy * 3 + dx;
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The SPLIT path: exact three-way bf16 split of both fp32 operands, six partial products on
// v_mfma_f32_16x16x32_bf16 (hrl_split.h: error analysis and helpers).
using hrl_split::split3;
using hrl_split::split_part;
using hrl_split::mfma_bf16;

// The split (exact bf16, six partial products) MFMA loop of conv3x3_kernel over one wave's 16-row A tile
// in LDS (rows of stride kStride): acc[q][ct] += sum_p A_p . W'[tap(p, q)][ct] on v_mfma_f32_16x16x32_bf16.
//  * the B fragments (split weights) are [tap][ct][part h/m/l][lane] x 4 dwords in LDS;
//  * A fragment of cell p: row lane & 15, input channels 8*(lane >> 4) + e (e = 0..7), read as
//    relu(a*pa[e] + pb[e]) when PRO; the next cell's A reads are issued before this cell's MFMAs;
//  * ROWLOOP: the board rows stay a loop (a row's three cells unrolled), for callers whose live
//    registers leave no room for the fully unrolled form (every cell's fragments and B reads hoisted).
template <bool PRO, bool ROWLOOP>
__device__ __forceinline__ void split_tile_mfma(const float *as, const uint32_t *w_lds_u, int lane, const float *pa,
                                                const float *pb, f32x4 (&acc)[kCells][2]) {
    const int ar = lane & 15;          // A row (sample within the tile)
    const int ak = lane >> 4;          // A k group
    const float *arow = as + ar * kStride;
    const uint4 *wb = reinterpret_cast<const uint4 *>(w_lds_u) + lane;
    // A fragment of cell p: row ar, input channels 8*ak + e (e = 0..7); the next cell's
    // A reads are issued before this cell's MFMAs.
    const float *acol = arow + 8 * ak * kCells;
    float an[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) an[e] = acol[e * kCells];
    auto cell = [&](int p) __attribute__((always_inline)) {
        float av[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = an[e];
        if (p + 1 < kCells) {
#pragma unroll
            for (int e = 0; e < 8; ++e) an[e] = acol[e * kCells + p + 1];
        }
        uint32_t ah[4], am[4], al[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            float v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = 2 * d + u;
                float a = av[e];
                if constexpr (PRO) {   // input channel 8ak+e: the previous block's BN+ReLU
                    const float t = a * pa[e] + pb[e];
                    a = t < 0.f ? 0.f : t;
                }
                v[u] = a;
            }
            uint32_t h0, m0, l0, h1, m1, l1;
            split3(v[0], h0, m0, l0);
            split3(v[1], h1, m1, l1);
            ah[d] = h0 | (h1 << 16);
            am[d] = m0 | (m1 << 16);
            al[d] = l0 | (l1 << 16);
        }
        const uint4 Ah = make_uint4(ah[0], ah[1], ah[2], ah[3]);
        const uint4 Am = make_uint4(am[0], am[1], am[2], am[3]);
        const uint4 Al = make_uint4(al[0], al[1], al[2], al[3]);
        const int py = p / kBoard, px = p - py * kBoard;
#pragma unroll
        for (int q = 0; q < kCells; ++q) {
            // tap_of(p, q) with p uniform at run time: a scalar branch
            const int dy = py - q / kBoard + 1, dx = px - q % kBoard + 1;
            if (dy < 0 || dy > 2 || dx < 0 || dx > 2) continue;
            const int tap = dy * 3 + dx;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const uint4 *wf = wb + (tap * 2 + ct) * 3 * 64;
                const uint4 Bh = wf[0], Bm = wf[64], Bl = wf[128];
                f32x4 c = acc[q][ct];
                c = mfma_bf16(Al, Bh, c);   // smallest terms first
                c = mfma_bf16(Am, Bm, c);
                c = mfma_bf16(Ah, Bl, c);
                c = mfma_bf16(Am, Bh, c);
                c = mfma_bf16(Ah, Bm, c);
                c = mfma_bf16(Ah, Bh, c);
                acc[q][ct] = c;
            }
        }
    };
    if constexpr (ROWLOOP) {
#pragma unroll 1
        for (int py = 0; py < kBoard; ++py) {
#pragma unroll
            for (int px = 0; px < kBoard; ++px) cell(py * kBoard + px);
        }
    } else {
#pragma unroll
        for (int p = 0; p < kCells; ++p) cell(p);
    }
}

// ------------------------------------------------------------------ forward / input gradient
// x: (M, 288) rows; wpk: packed [tap][ct][ci][16] = W'[tap][ci][ct*16+j]; y: (M, 288)
// Forward / input gradient.
//  * the packed weights [tap][co-tile][ci][16] (36 KB) are staged in LDS once
//    per workgroup; the B fragment of lane l (k = l>>4, j = l&15) is a
//    bank-conflict-free ds_read_b32;
//  * p-major MFMA order: one A fragment feeds every output cell q it reaches
//    (up to 18 independent accumulators), hiding the 40-cycle dependent-MFMA
//    latency; each accumulator sums in (p, s) order;
//  PRO:   the input is the previous block's raw conv output and the kernel
//         applies that block's BatchNorm+ReLU, relu(x*alpha[c] + beta[c]),
//         to each A fragment as it is read (a lane's channels are fixed, so
//         alpha/beta are 16 registers); the activation never reaches HBM;
//  EPI (what the epilogue does besides storing y):
//   1 STATS: per output channel sum and sum of squares of y, fp32 per tile
//            (36 values per lane) folded into fp64;
//   2 BNRED: y is the gradient w.r.t. relu(ref*alpha + beta) of the block
//            before (input gradient of a chain); sums g = [ref*alpha+beta > 0] y
//            and g*(ref - mean) per channel -- bn_bwd_reduce_kernel's sums,
//            without re-reading y;
//   3 MASK:  y *= [ref > 0] before the store (the backward of a ReLU on the
//            chain's input, threshold_backward);
//   partials go to part[block][c][2] (fp64), the layout bn_finalize_kernel folds.
//   ref tiles (EPI 2, 3) are loaded with the next input tile and transposed
//   to the accumulator layout through the tile's LDS buffer.
template <bool PRO, int EPI, bool SPLIT>
__global__ __launch_bounds__(kThreads) void conv3x3_kernel(const float *__restrict__ x, int64_t M,
                                                           const float *__restrict__ wpk,
                                                           const float *__restrict__ bias,
                                                           const float *__restrict__ in_alpha,
                                                           const float *__restrict__ in_beta,
                                                           const float *__restrict__ ref,
                                                           const float *__restrict__ ep_mean,
                                                           const float *__restrict__ ep_alpha,
                                                           const float *__restrict__ ep_beta,
                                                           float *__restrict__ y, double *__restrict__ part) {
    constexpr bool kRef = EPI == 2 || EPI == 3;
    constexpr bool kSums = EPI == 1 || EPI == 2;
    // fp32: packed [tap][ct][ci][16] (36 KB).  SPLIT: the B fragments of
    // v_mfma_f32_16x16x32_bf16, [tap][ct][part h/m/l][lane] x 4 dwords (54 KB): lane l's
    // 8 bf16 are W'[tap][ci = 8(l>>4) + e][co = 16ct + (l&15)], e = 0..7, one
    // conflict-free ds_read_b128 per fragment.
    constexpr int kWWords = SPLIT ? kTaps * 2 * 3 * 64 * 4 : kTaps * 2 * kC * 16;
    __shared__ __attribute__((aligned(16))) uint32_t w_lds_u[kWWords];
    __shared__ float a_lds[kWaves][kTile * kStride];       // 4 x 18.1 KB
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if constexpr (SPLIT) {
        for (int i = threadIdx.x; i < kWWords; i += kThreads) {
            const int d = i & 3, l = (i >> 2) & 63, f = i >> 8;      // f = (tap*2 + ct)*3 + part
            const int part = f % 3, tc = f / 3;                      // tc = tap*2 + ct
            const int ci = 8 * (l >> 4) + 2 * d, j = l & 15;
            const float w0 = wpk[(tc * kC + ci) * 16 + j];
            const float w1 = wpk[(tc * kC + ci + 1) * 16 + j];
            w_lds_u[i] = split_part(w0, part) | (split_part(w1, part) << 16);
        }
    } else {
        for (int i = threadIdx.x; i < kWWords; i += kThreads) w_lds_u[i] = __float_as_uint(wpk[i]);
    }
    const float *w_lds = reinterpret_cast<const float *>(w_lds_u);
    // PRO: a lane's A fragments are input channels 4s + (lane>>4), s = 0..7 (fp32 path)
    // or 8(lane>>4) + e, e = 0..7 (SPLIT)
    float pa[PRO ? kC / 4 : 1], pb[PRO ? kC / 4 : 1];
    if constexpr (PRO) {
#pragma unroll
        for (int s = 0; s < kC / 4; ++s) {
            const int ci = SPLIT ? 8 * (lane >> 4) + s : 4 * s + (lane >> 4);
            pa[s] = in_alpha[ci];
            pb[s] = in_beta[ci];
        }
    }
    // epilogue: a lane's outputs are channels (lane & 15) and 16 + (lane & 15)
    float em[2] = {0.f, 0.f}, ea[2] = {1.f, 1.f}, eb[2] = {0.f, 0.f};
    if constexpr (EPI == 2) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            em[ct] = ep_mean[ct * 16 + (lane & 15)];
            ea[ct] = ep_alpha[ct * 16 + (lane & 15)];
            eb[ct] = ep_beta[ct * 16 + (lane & 15)];
        }
    }
    double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};   // EPI 1, 2: this lane's two channels

    const int64_t ntiles = (M + kTile - 1) / kTile;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
    float *as = a_lds[wave];
    const int64_t lim = M * kRow;
    float bias_v[2] = {0.f, 0.f};
    if (bias) {
        bias_v[0] = bias[lane & 15];
        bias_v[1] = bias[16 + (lane & 15)];
    }
    float4 stage[kVec];
    float4 rstage[kRef ? kVec : 1];
    auto load_tile = [&](const float *src, int64_t t, float4 *dst) {
        // rows t*16 .. t*16+15 are contiguous: 16*288 floats = 1152 float4
        const int64_t base = t * kTile * kRow;
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int64_t e = base + (int64_t)(k * 64 + lane) * 4;
            const int64_t ec = e < lim ? e : lim - 4;          // clamp (ragged last tile), no branch
            dst[k] = *reinterpret_cast<const float4 *>(src + ec);
        }
    };
    auto to_lds = [&](const float4 *src) {
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int e = (k * 64 + lane) * 4;                 // element within the tile
            const int r = e / kRow, c = e - r * kRow;          // kRow % 4 == 0: one row per float4
            float *d = as + r * kStride + c;
            d[0] = src[k].x; d[1] = src[k].y; d[2] = src[k].z; d[3] = src[k].w;
        }
    };
    if (tile < ntiles) load_tile(x, tile, stage);
    __syncthreads();   // weights in LDS

    for (; tile < ntiles; tile += stride) {
        to_lds(stage);                        // staged tile -> LDS (padded rows)
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();
        if constexpr (kRef) load_tile(ref, tile, rstage);   // this tile's reference, for the epilogue
        const int64_t next = tile + stride;
        if (next < ntiles) load_tile(x, next, stage);        // in flight during the MFMAs

        f32x4 acc[kCells][2];
#pragma unroll
        for (int q = 0; q < kCells; ++q) acc[q][0] = acc[q][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const int ar = lane & 15;          // A row (sample within the tile)
        const int ak = lane >> 4;          // A/B k within the 4-wide step
        const float *arow = as + ar * kStride;
        const float *wl = w_lds + ak * 16 + (lane & 15);
        if constexpr (SPLIT) {
            // kRef: the reference tile's 72 staging registers leave no room for the unrolled form
            split_tile_mfma<PRO, kRef>(as, w_lds_u, lane, pa, pb, acc);
        } else {
#pragma unroll
        for (int p = 0; p < kCells; ++p) {
#pragma unroll
            for (int s = 0; s < kC / 4; ++s) {
                float a = arow[(4 * s + ak) * kCells + p];
                if constexpr (PRO) {   // input channel 4s+ak: the previous block's BN+ReLU (bn_apply_kernel's ops)
                    const float t = a * pa[s] + pb[s];
                    a = t < 0.f ? 0.f : t;
                }
#pragma unroll
                for (int q = 0; q < kCells; ++q) {
                    const int tap = tap_of(p, q);
                    if (tap < 0) continue;
                    acc[q][0] = mfma(a, wl[((tap * 2 + 0) * kC) * 16 + s * 64], acc[q][0]);
                    acc[q][1] = mfma(a, wl[((tap * 2 + 1) * kC) * 16 + s * 64], acc[q][1]);
                }
            }
        }
        }

        const int64_t valid = M - tile * kTile;          // rows of this tile inside the batch
        __builtin_amdgcn_wave_barrier();
        if constexpr (kRef) {
            // reference tile -> LDS, read back in the accumulator layout
            to_lds(rstage);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            float t1[2] = {0.f, 0.f}, t2[2] = {0.f, 0.f};
#pragma unroll
            for (int q = 0; q < kCells; ++q)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = (lane >> 4) * 4 + r;
                        const int co = ct * 16 + (lane & 15);
                        const float rv = as[row * kStride + co * kCells + q];
                        if constexpr (EPI == 3) {
                            if (!(rv > 0.f)) acc[q][ct][r] = 0.f;
                        } else {
                            // bn_bwd_reduce_kernel's mask and sums (float products, fp32 per tile here)
                            const float gm = (rv * ea[ct] + eb[ct] > 0.f && row < valid) ? acc[q][ct][r] : 0.f;
                            t1[ct] += gm;
                            t2[ct] += gm * (rv - em[ct]);
                        }
                    }
            if constexpr (EPI == 2) {
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    s1[ct] += (double)t1[ct];
                    s2[ct] += (double)t2[ct];
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
        }

        // accumulators -> LDS tile [row][co*9 + q] -> coalesced stores
        float t1[2] = {0.f, 0.f}, t2[2] = {0.f, 0.f};   // EPI 1: this tile's fp32 partials
#pragma unroll
        for (int q = 0; q < kCells; ++q)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = (lane >> 4) * 4 + r;       // C/D: row = (lane>>4)*4 + reg
                    const int co = ct * 16 + (lane & 15);      //      col = lane & 15
                    const float v = acc[q][ct][r] + bias_v[ct];
                    as[row * kStride + co * kCells + q] = v;
                    if constexpr (EPI == 1) {
                        const float u = row < valid ? v : 0.f;
                        t1[ct] += u;
                        t2[ct] += u * u;
                    }
                }
        if constexpr (EPI == 1) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                s1[ct] += (double)t1[ct];
                s2[ct] += (double)t2[ct];
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int64_t obase = tile * kTile * kRow;
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int e = (k * 64 + lane) * 4;
            const int r = e / kRow, c = e - r * kRow;
            const float *sp = as + r * kStride + c;
            if (obase + e < lim) *reinterpret_cast<float4 *>(y + obase + e) = make_float4(sp[0], sp[1], sp[2], sp[3]);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (kSums) {
        // fold the lanes sharing a channel (4 row groups) and the 4 waves in a fixed order
        __syncthreads();
        double *red = reinterpret_cast<double *>(&a_lds[0][0]);   // [wave][group][32][2]
        const int grp = lane >> 4;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const int co = ct * 16 + (lane & 15);
            red[((wave * 4 + grp) * kC + co) * 2 + 0] = s1[ct];
            red[((wave * 4 + grp) * kC + co) * 2 + 1] = s2[ct];
        }
        __syncthreads();
        if (threadIdx.x < 2 * kC) {
            const int co = threadIdx.x >> 1, k = threadIdx.x & 1;
            double t = 0.0;
            for (int i = 0; i < kWaves * 4; ++i) t += red[(i * kC + co) * 2 + k];
            part[((int64_t)blockIdx.x * kC + co) * 2 + k] = t;
        }
    }
}

// ------------------------------------------------------------------ weight gradient
// dW[tap][ci][co] = sum_rows sum_{(p,q): tap(p,q) = tap} x[row, ci, p] * dy[row, co, q]
// MFMA C tile = 16 ci x 16 co; A[i = ci][k = row], B[k = row][j = co]
// fp32 MFMA form (hrl_conv3x3_set_split(0)); the default is conv3x3_wgrad_split_kernel below.
template <bool PRO>
__global__ __launch_bounds__(kThreads) void conv3x3_wgrad_kernel(const float *__restrict__ x,
                                                                 const float *__restrict__ in_alpha,
                                                                 const float *__restrict__ in_beta,
                                                                 const float *__restrict__ dy, int64_t M,
                                                                 float *__restrict__ partial) {
    // one LDS array: per-wave x and dy tiles during the loop, the 4 wave partials after it
    __shared__ float lds[2 * kWaves * kTile * kStride];    // 148 KB >= 4 x 9216 floats
    static_assert(2 * kWaves * kTile * kStride >= kWaves * kTaps * kC * kC, "fold buffer");
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float *xs = lds + wave * kTile * kStride;
    float *gs = lds + (kWaves + wave) * kTile * kStride;
    // PRO: x is a raw conv output read as relu(x*alpha + beta); a lane's A
    // fragments are channels (lane & 15) and 16 + (lane & 15)
    float pa0 = 1.f, pb0 = 0.f, pa1 = 1.f, pb1 = 0.f;
    if constexpr (PRO) {
        pa0 = in_alpha[lane & 15];
        pb0 = in_beta[lane & 15];
        pa1 = in_alpha[16 + (lane & 15)];
        pb1 = in_beta[16 + (lane & 15)];
    }
    const int64_t ntiles = (M + kTile - 1) / kTile;
    const int64_t stride = (int64_t)gridDim.x * kWaves;

    f32x4 acc[kTaps][2][2];
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles; tile += stride) {
        const int64_t base = tile * kTile * kRow;
        const int64_t lim = M * kRow;
        float4 sx[kVec], sg[kVec];
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int64_t e = base + (int64_t)(k * 64 + lane) * 4;
            const bool ok = e < lim;
            const int64_t ec = ok ? e : lim - 4;
            sx[k] = *reinterpret_cast<const float4 *>(x + ec);
            sg[k] = *reinterpret_cast<const float4 *>(dy + ec);
            if (!ok) sg[k] = make_float4(0.f, 0.f, 0.f, 0.f);   // ragged tile: zero gradient rows
        }
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int e = (k * 64 + lane) * 4;
            const int r = e / kRow, c = e - r * kRow;
            float *d = xs + r * kStride + c;
            d[0] = sx[k].x; d[1] = sx[k].y; d[2] = sx[k].z; d[3] = sx[k].w;
            float *h = gs + r * kStride + c;
            h[0] = sg[k].x; h[1] = sg[k].y; h[2] = sg[k].z; h[3] = sg[k].w;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int i16 = lane & 15;   // A row = ci within the tile / B col = co within the tile
        const int kk = lane >> 4;    // k = row within the 4-row step
#pragma unroll
        for (int q = 0; q < kCells; ++q) {
#pragma unroll
            for (int p = 0; p < kCells; ++p) {
                const int tap = tap_of(p, q);
                if (tap < 0) continue;
#pragma unroll
                for (int s = 0; s < kTile / 4; ++s) {
                    const int row = 4 * s + kk;
                    float a0 = xs[row * kStride + (0 * 16 + i16) * kCells + p];
                    float a1 = xs[row * kStride + (1 * 16 + i16) * kCells + p];
                    if constexpr (PRO) {
                        const float t0 = a0 * pa0 + pb0, t1 = a1 * pa1 + pb1;
                        a0 = t0 < 0.f ? 0.f : t0;
                        a1 = t1 < 0.f ? 0.f : t1;
                    }
                    const float b0 = gs[row * kStride + (0 * 16 + i16) * kCells + q];
                    const float b1 = gs[row * kStride + (1 * 16 + i16) * kCells + q];
                    acc[tap][0][0] = mfma(a0, b0, acc[tap][0][0]);
                    acc[tap][0][1] = mfma(a0, b1, acc[tap][0][1]);
                    acc[tap][1][0] = mfma(a1, b0, acc[tap][1][0]);
                    acc[tap][1][1] = mfma(a1, b1, acc[tap][1][1]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // fold the block's 4 wave partials in a fixed order through the (now free) tile LDS,
    // then write one partial per workgroup: partial[block][tap][ci][co]
    __syncthreads();
    float *red = lds;
    constexpr int kW = kTaps * kC * kC;
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ci = it * 16 + (lane >> 4) * 4 + r;
                    const int co = jt * 16 + (lane & 15);
                    red[wave * kW + (t * kC + ci) * kC + co] = acc[t][it][jt][r];
                }
    __syncthreads();
    float *out = partial + (int64_t)blockIdx.x * kW;
    for (int i = threadIdx.x; i < kW; i += kThreads)
        out[i] = ((red[i] + red[kW + i]) + red[2 * kW + i]) + red[3 * kW + i];
}

// Weight gradient on the exact bf16 split (default; hrl_conv3x3_set_split).  One tap's dW is a 32x32
// (ci, co) matrix, i.e. exactly one v_mfma_f32_32x32x16_bf16 tile, and a 16-row tile is one K=16 step:
//   dW[tap] += X_p^T (32 ci x 16 rows) . dY_q (16 rows x 32 co)   for every (p, q) with tap(p, q) = tap,
// six partial products per pair (hrl_split.h), 49 pairs x 6 = 294 MFMAs of 32 cycles per tile against
// 784 fp32 16x16x4 MFMAs of 32 cycles.  Both operands are split ONCE per tile: the nine dY_q fragments
// are split up front and held in registers, X_p is split as the p loop reaches it (a former split form
// re-split every operand per (p, q) pair and ran at 274 us).  Lane l = (r = l & 31, h = l >> 5) holds
// rows 8h..8h+7 of channel r of a cell: A[i = ci = r][k = row], B[k = row][j = co = r].  The tiles sit in
// LDS with a row stride of 292 floats (16-byte aligned rows, so tiles are written with ds_write_b128;
// 8 x 292 == 32 (mod 64), so the two lane halves' column reads do not collide).  Waves fold in a fixed
// order: deterministic.
constexpr int kStrideW = kRow + 4;   // 292
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma32(const uint4 &a, const uint4 &b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

template <bool PRO>
__global__ __launch_bounds__(kThreads) void conv3x3_wgrad_split_kernel(const float *__restrict__ x,
                                                                       const float *__restrict__ in_alpha,
                                                                       const float *__restrict__ in_beta,
                                                                       const float *__restrict__ dy, int64_t M,
                                                                       float *__restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float lds[2 * kWaves * kTile * kStrideW];   // 149.5 KB
    static_assert(2 * kWaves * kTile * kStrideW >= kWaves * kTaps * kC * kC, "fold buffer");
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float *xs = lds + wave * kTile * kStrideW;
    float *gs = lds + (kWaves + wave) * kTile * kStrideW;
    const int r = lane & 31, h = lane >> 5;
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {   // x is a raw conv output read as relu(x*alpha + beta); A rows are channel r
        pa = in_alpha[r];
        pb = in_beta[r];
    }
    const int64_t ntiles = (M + kTile - 1) / kTile;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    const int64_t lim = M * kRow;

    f32x16 acc[kTaps];
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles; tile += stride) {
        {
            const int64_t base = tile * kTile * kRow;
            float4 sx[kVec], sg[kVec];
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int64_t e = base + (int64_t)(k * 64 + lane) * 4;
                const int64_t ec = e < lim ? e : lim - 4;
                sx[k] = *reinterpret_cast<const float4 *>(x + ec);
                sg[k] = *reinterpret_cast<const float4 *>(dy + ec);
            }
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int e = (k * 64 + lane) * 4;
                const int row = e / kRow, c = e - row * kRow;
                const bool ok = base + e < lim;   // ragged tile: zero gradient rows
                *reinterpret_cast<float4 *>(xs + row * kStrideW + c) = sx[k];
                *reinterpret_cast<float4 *>(gs + row * kStrideW + c) = ok ? sg[k] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();

        // the nine dY_q fragments, split once
        uint4 Bh[kCells], Bm[kCells], Bl[kCells];
        const float *gcol = gs + (8 * h) * kStrideW + r * kCells;
#pragma unroll
        for (int q = 0; q < kCells; ++q) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = gcol[j * kStrideW + q];
            hrl_split::split8(v, Bh[q], Bm[q], Bl[q]);
        }
        const float *xcol = xs + (8 * h) * kStrideW + r * kCells;
#pragma unroll
        for (int p = 0; p < kCells; ++p) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float a = xcol[j * kStrideW + p];
                if constexpr (PRO) {   // bn_apply_kernel's float operations
                    const float t = a * pa + pb;
                    a = t < 0.f ? 0.f : t;
                }
                v[j] = a;
            }
            uint4 Ah, Am, Al;
            hrl_split::split8(v, Ah, Am, Al);
#pragma unroll
            for (int q = 0; q < kCells; ++q) {
                const int tap = tap_of(p, q);
                if (tap < 0) continue;
                f32x16 c = acc[tap];
                c = mfma32(Al, Bh[q], c);   // smallest terms first
                c = mfma32(Am, Bm[q], c);
                c = mfma32(Ah, Bl[q], c);
                c = mfma32(Am, Bh[q], c);
                c = mfma32(Ah, Bm[q], c);
                c = mfma32(Ah, Bh[q], c);
                acc[tap] = c;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // fold the block's 4 wave partials in a fixed order: partial[block][tap][ci][co]
    __syncthreads();
    float *red = lds;
    constexpr int kW = kTaps * kC * kC;
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int ci = (i & 3) + 8 * (i >> 2) + 4 * h;   // C/D: col = lane & 31, row = (reg&3) + 8(reg>>2) + 4h
            red[wave * kW + (t * kC + ci) * kC + r] = acc[t][i];
        }
    __syncthreads();
    float *out = partial + (int64_t)blockIdx.x * kW;
    for (int i = threadIdx.x; i < kW; i += kThreads)
        out[i] = ((red[i] + red[kW + i]) + red[2 * kW + i]) + red[3 * kW + i];
}

// ------------------------------------------------------------------ one chain block's backward, fused
// For a chain block y_i = conv_i(x'), out_i = relu(BN_i(y_i)) with x' = relu(x*in_alpha + in_beta) (or x), from
// g = dL/d out_i in ONE launch:
//   dY   = BN_i's input gradient, bn_bwd_apply_kernel's float operations (hrl_bn.hip), in registers;
//   dW  += x'^T dY, the weight gradient of conv3x3_wgrad_split_kernel (32x32x16 bf16, exact split);
//   gin  = conv_i^T(dY), conv3x3_kernel's split input-gradient loop on dY staged in LDS, with the
//          epilogue of hrl_conv3x3_forward_ex: 2 = BN_{i-1}'s backward sums (ref = x), 3 = x > 0 mask.
// It replaces bn_bwd_apply (reads g, y; writes dY), the weight gradient (reads x, dY) and the input gradient
// (reads dY, x): 1.2 GB of a B=4096 T=32 step's block traffic becomes 604 MB (reads g, y, x; writes gin; the
// epilogue's second read of x hits L2), and neither dY nor x' reaches HBM.
// Data layout: lane l = (r = l & 31, h = l >> 5) owns channel r of rows 8h..8h+7 of a 16-row tile, i.e. the
// wgrad operand layout, so BN_i's, the prologue's and the epilogue's per-channel constants are registers and
// the loads are 36-byte runs (three buffer_load_dwordx3 per row; the descriptor's range check zeroes rows past
// the batch and drops their stores).
struct BlockBwdArgs {
    const float *g, *y;                                          // dL/d out_i, y_i: (M, 288)
    const float *bn_w, *bn_b, *bn_mean, *bn_invstd, *bn_k, *bn_gm;   // BN_i (hrl_bn_backward_apply's arguments)
    const float *x, *in_alpha, *in_beta;                         // conv_i's input (raw), its prologue
    const float *wpk;                                            // packed input-gradient weights (flip layout)
    const float *ep_mean, *ep_alpha, *ep_beta;                   // epilogue 2: BN_{i-1}
    float *gin;                                                  // dL/dx' masked per the epilogue (DG)
    double *part;                                                // epilogue 2 sums [block][32][2]
    float *wpart;                                                // weight-gradient partials [block][tap][ci][co]
    int64_t M;
    unsigned *tickets;                                           // block form 2: per-CU arrival tickets
    int stagger;                                                 // block form 2: s_sleep(32)s of the later arrival
    // a BatchNorm finalize folded into the prologue (fold_part nullptr: none; bnfold below): mode 0 = the input BN's
    // forward statistics -> its alpha / beta (the conv's prologue), mode 1 = BN_i's backward sums -> k / mean(dy)
    const double *fold_part;                                     // partial rows [fold_nblocks][32][2]
    int fold_nblocks, fold_mode;
    double fold_count, fold_eps;
    float fold_momentum;
    const float *fold_w, *fold_b;                                // mode 0: the BN's weight / bias
    float *fold_rm, *fold_rv;                                    // mode 0: running statistics (workgroup 0)
    float *fold_o0, *fold_o1, *fold_o2, *fold_o3;                // mode 0: mean invstd alpha beta; 1: dw db k gm
};

// ------------------------------------------------------------------ BatchNorm finalize in a consumer's prologue
// hrl_bn_finalize_stats / _backward (bn_finalize_kernel, one group) as the first step of the kernel that consumes
// its coefficients, instead of a launch of its own: every 512-thread workgroup folds the fold_nblocks partial rows
// of all 32 channels in bn_finalize_kernel's exact order -- thread i of its 256 sums rows i, i + 256 (0.0 first),
// then the fixed tree (i, i + 128), (i, i + 64), (i, i + 32) ... (i, i + 1) -- and computes the channel's
// coefficients with its float operations; workgroup 0 writes the outputs the separate launch wrote (the running
// statistics advance once).  Bit-identical to the two launches (tests/test_bn_gpu.py).  Here lane (c, k) of wave j
// holds leaves j + 8 m (m < 32; one contiguous 512-byte row per wave load): the levels 128 .. 8 are its register
// tree, 4, 2, 1 run over the eight waves' nodes through LDS.
namespace bnfold {

constexpr int kThreadsFold = 512;

__device__ __forceinline__ void fold(const BlockBwdArgs &a, unsigned char *lds, float &c0, float &c1) {
    double *sums = reinterpret_cast<double *>(lds);                 // [32][2]
    double *part8 = reinterpret_cast<double *>(lds + 64 * 8 + 64 * 4);   // [8][64]: the tree's level-8 nodes
    float *coef = reinterpret_cast<float *>(lds + 64 * 8);          // [2][32]
    const int tid = threadIdx.x;
    // lane (c, k) = tid & 63 reads one double of every row its wave j = tid >> 6 owns: rows j + 8 m, 512 contiguous
    // bytes per wave instruction
    const int ck = tid & 63, j = tid >> 6;
    const int nb = a.fold_nblocks;
    const double *pc = a.fold_part + ck;
    double v[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
        const int i = j + 8 * m;
        const double lo = i < nb ? pc[(int64_t)i * kC * 2] : 0.0;
        const double hi = i + 256 < nb ? pc[(int64_t)(i + 256) * kC * 2] : 0.0;
        v[m] = (0.0 + lo) + hi;      // bn_finalize_kernel's s = 0.0; s += part[i]; s += part[i + 256] (+0.0 exact)
    }
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1)
#pragma unroll
        for (int m = 0; m < w; ++m) v[m] += v[m + w];
    part8[j * 64 + ck] = v[0];
    __syncthreads();
    if (tid < 64) {   // the levels 4, 2, 1 over the eight waves' nodes
        double e[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) e[q] = part8[q * 64 + ck];
#pragma unroll
        for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
            for (int q = 0; q < w; ++q) e[q] += e[q + w];
        sums[ck] = e[0];
    }
    __syncthreads();
    if (tid < kC) {
        const int ch = tid;
        const double S0 = sums[ch * 2], S1 = sums[ch * 2 + 1];
        const double M = a.fold_count;
        const bool out = blockIdx.x == 0;
        if (a.fold_mode == 0) {   // bn_finalize_kernel mode 0's float operations
            const float w = a.fold_w ? a.fold_w[ch] : 1.0f;
            const double mean = S0 / M;
            double var = S1 / M - mean * mean;
            if (var < 0.0) var = 0.0;
            const float meanf = (float)mean;
            const float invstd = (float)(1.0 / sqrt(var + a.fold_eps));
            const float alpha = invstd * w;
            const float beta = (a.fold_b ? a.fold_b[ch] : 0.0f) - meanf * alpha;
            coef[ch] = alpha;
            coef[kC + ch] = beta;
            if (out) {
                const float momentum = a.fold_momentum;
                a.fold_o0[ch] = meanf;
                a.fold_o1[ch] = invstd;
                a.fold_o2[ch] = alpha;
                a.fold_o3[ch] = beta;
                if (a.fold_rm) a.fold_rm[ch] = momentum * meanf + (1.0f - momentum) * a.fold_rm[ch];
                if (a.fold_rv) {
                    const float unbiased = (float)(M > 1.0 ? var * M / (M - 1.0) : var);
                    a.fold_rv[ch] = momentum * unbiased + (1.0f - momentum) * a.fold_rv[ch];
                }
            }
        } else {                  // mode 1: the BN's saved invstd is bn_invstd
            const float invstd = a.bn_invstd[ch];
            const float sum_dy = (float)S0, dot = (float)S1;
            const float kc = dot * invstd * invstd / (float)M;
            const float gm = sum_dy / (float)M;
            coef[ch] = kc;
            coef[kC + ch] = gm;
            if (out) {
                if (a.fold_o0) a.fold_o0[ch] = dot * invstd;
                if (a.fold_o1) a.fold_o1[ch] = sum_dy;
                a.fold_o2[ch] = kc;
                a.fold_o3[ch] = gm;
            }
        }
    }
    __syncthreads();
    const int ch = threadIdx.x & 31;
    c0 = coef[ch];
    c1 = coef[kC + ch];
    __syncthreads();   // every lane has its coefficients before the caller's staging reuses these bytes
}

}  // namespace bnfold

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// buffer descriptor over `bytes` bytes at `base`; the inputs are made provably wave-uniform so the compiler
// keeps the descriptor in SGPRs (no waterfall loops around the buffer ops)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void *base, uint32_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                             0x00020000);
}

// the 9 cells of one channel of one row (36 bytes at byte offset off)
__device__ __forceinline__ void load_cells(__amdgpu_buffer_rsrc_t rs, int off, float (&d)[kCells]) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, off + 12 * m, 0, 0);
        d[3 * m + 0] = __uint_as_float(v.x);
        d[3 * m + 1] = __uint_as_float(v.y);
        d[3 * m + 2] = __uint_as_float(v.z);
    }
}

__device__ __forceinline__ void store_cells(__amdgpu_buffer_rsrc_t rs, int off, const float (&d)[kCells]) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        u32x3 v;
        v.x = __float_as_uint(d[3 * m + 0]);
        v.y = __float_as_uint(d[3 * m + 1]);
        v.z = __float_as_uint(d[3 * m + 2]);
        __builtin_amdgcn_raw_buffer_store_b96(v, rs, off + 12 * m, 0, 0);
    }
}

template <bool PRO, int EPI, bool DG>
__global__ __launch_bounds__(kThreads) void conv3x3_block_bwd_kernel(BlockBwdArgs a) {
    constexpr int kWWords = kTaps * 2 * 3 * 64 * 4;            // split input-gradient weights (54 KB)
    constexpr int kTileF = kTile * kStride;                    // one wave's dY / output tile (18.1 KB)
    constexpr int kW = kTaps * kC * kC;
    constexpr int kFoldF = (kWaves - 1) * kW;                  // waves 1..3's weight-gradient partials
    constexpr int kUseF = DG ? kWWords + kWaves * kTileF : 0;
    constexpr int kSmemF = kUseF > kFoldF ? kUseF : kFoldF;
    __shared__ __attribute__((aligned(16))) float smem[kSmemF];
    uint32_t *w_lds_u = reinterpret_cast<uint32_t *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float *as = smem + kWWords + wave * kTileF;
    if constexpr (DG) {
        for (int i = threadIdx.x; i < kWWords; i += kThreads) {
            const int d = i & 3, l = (i >> 2) & 63, f = i >> 8;      // f = (tap*2 + ct)*3 + part
            const int part = f % 3, tc = f / 3;
            const int ci = 8 * (l >> 4) + 2 * d, j = l & 15;
            const float w0 = a.wpk[(tc * kC + ci) * 16 + j];
            const float w1 = a.wpk[(tc * kC + ci + 1) * 16 + j];
            w_lds_u[i] = split_part(w0, part) | (split_part(w1, part) << 16);
        }
    }
    const int r = lane & 31, h = lane >> 5;
    // BN_i's backward apply for channel r (bn_bwd_apply_kernel's per-channel values)
    const float mu = a.bn_mean[r], kk = a.bn_k[r], gmn = a.bn_gm[r], is = a.bn_invstd[r];
    const float ww = a.bn_w ? a.bn_w[r] : 1.0f;
    const float al = is * ww;
    const float be = (a.bn_b ? a.bn_b[r] : 0.0f) - mu * al;
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {
        pa = a.in_alpha[r];
        pb = a.in_beta[r];
    }
    float em = 0.f, ea = 1.f, eb = 0.f;
    if constexpr (DG && EPI == 2) {
        em = a.ep_mean[r];
        ea = a.ep_alpha[r];
        eb = a.ep_beta[r];
    }
    double s1 = 0.0, s2 = 0.0;
    f32x16 wacc[kTaps];
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) wacc[t][i] = 0.f;
    if constexpr (DG) __syncthreads();   // weights in LDS

    const int64_t ntiles = (a.M + kTile - 1) / kTile;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    const int off0 = ((8 * h) * kRow + r * kCells) * 4;         // byte offset of this lane's first run
    HRL_STAMP_WALL(14);
    int st_it = 0;   // stamps: the first two tiles of wave 0, slots 0..11
    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles; tile += stride, ++st_it) {
        if (st_it < 2) HRL_STAMP(6 * st_it + 0);
        const int64_t row0 = tile * kTile;
        const int rows = (int)min<int64_t>(kTile, a.M - row0);
        const uint32_t bytes = (uint32_t)rows * kRow * 4;
        const int64_t eofs = row0 * kRow;
        const __amdgpu_buffer_rsrc_t rg = wave_rsrc(a.g + eofs, bytes);
        const __amdgpu_buffer_rsrc_t ry = wave_rsrc(a.y + eofs, bytes);
        const __amdgpu_buffer_rsrc_t rx = wave_rsrc(a.x + eofs, bytes);
        float G[8][kCells], X[8][kCells];
        {
            float Y[8][kCells];
            // dY = BN_i backward apply; rows past the batch are zero (their zero inputs would not give 0)
            auto bn_apply = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool valid = 8 * h + j < rows;
#pragma unroll
                    for (int c = 0; c < kCells; ++c) {
                        const float yv = Y[j][c];
                        float gv = G[j][c];
                        if (!(yv * al + be > 0.f)) gv = 0.f;
                        const float t = (yv - mu) * kk;
                        const float d = (((gv - gmn) - t) * is) * ww;
                        G[j][c] = valid ? d : 0.f;
                    }
                }
            };
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                load_cells(rg, off0 + j * kRow * 4, G[j]);
                load_cells(ry, off0 + j * kRow * 4, Y[j]);
                load_cells(rx, off0 + j * kRow * 4, X[j]);
            }
            bn_apply();
        }
        if (st_it < 2) HRL_STAMP(6 * st_it + 1);
        if constexpr (DG) {   // dY -> this wave's LDS tile, the input gradient's A operand
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int c = 0; c < kCells; ++c) as[(8 * h + j) * kStride + r * kCells + c] = G[j][c];
        }
        // weight gradient: the nine dY_q fragments split once, x'_p split as the p loop reaches it
        {
            uint4 Bh[kCells], Bm[kCells], Bl[kCells];
#pragma unroll
            for (int q = 0; q < kCells; ++q) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = G[j][q];
                hrl_split::split8(v, Bh[q], Bm[q], Bl[q]);
            }
#pragma unroll
            for (int p = 0; p < kCells; ++p) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float xv = X[j][p];
                    if constexpr (PRO) {   // bn_apply_kernel's float operations
                        const float t = xv * pa + pb;
                        xv = t < 0.f ? 0.f : t;
                    }
                    v[j] = xv;
                }
                uint4 Ah, Am, Al;
                hrl_split::split8(v, Ah, Am, Al);
#pragma unroll
                for (int q = 0; q < kCells; ++q) {
                    const int tap = tap_of(p, q);
                    if (tap < 0) continue;
                    f32x16 c = wacc[tap];
                    c = mfma32(Al, Bh[q], c);   // smallest terms first
                    c = mfma32(Am, Bm[q], c);
                    c = mfma32(Ah, Bl[q], c);
                    c = mfma32(Am, Bh[q], c);
                    c = mfma32(Ah, Bm[q], c);
                    c = mfma32(Ah, Bh[q], c);
                    wacc[tap] = c;
                }
            }
        }
        if (st_it < 2) HRL_STAMP(6 * st_it + 2);
        if constexpr (DG) {
            // the epilogue's reference (x itself) is read again rather than held through the weight gradient
            // (registers); the tile was read a few microseconds ago, so these loads hit L2.  Issued before the
            // MFMAs, they land during them.
            float R[8][kCells];
            if constexpr (EPI == 2 || EPI == 3) {
#pragma unroll
                for (int j = 0; j < 8; ++j) load_cells(rx, off0 + j * kRow * 4, R[j]);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the dY tile is in LDS
            __builtin_amdgcn_wave_barrier();
            f32x4 acc[kCells][2];
#pragma unroll
            for (int q = 0; q < kCells; ++q) acc[q][0] = acc[q][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
            split_tile_mfma<false, true>(as, w_lds_u, lane, nullptr, nullptr, acc);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            if (st_it < 2) HRL_STAMP(6 * st_it + 3);
            // accumulators -> the tile [row][c*9 + q] -> this lane's channel-r runs, epilogue, stores
#pragma unroll
            for (int q = 0; q < kCells; ++q)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = (lane >> 4) * 4 + rr;   // C/D: row = (lane>>4)*4 + reg, col = lane & 15
                        const int co = ct * 16 + (lane & 15);
                        as[row * kStride + co * kCells + q] = acc[q][ct][rr];
                    }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const __amdgpu_buffer_rsrc_t ro = wave_rsrc(a.gin + eofs, bytes);
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool valid = 8 * h + j < rows;
                float o[kCells];
#pragma unroll
                for (int c = 0; c < kCells; ++c) {
                    float v = as[(8 * h + j) * kStride + r * kCells + c];
                    const float rv = (EPI == 2 || EPI == 3) ? R[j][c] : 0.f;
                    if constexpr (EPI == 3) {
                        if (!(rv > 0.f)) v = 0.f;
                    } else if constexpr (EPI == 2) {   // bn_bwd_reduce_kernel's mask and sums
                        const float gm = (rv * ea + eb > 0.f && valid) ? v : 0.f;
                        t1 += gm;
                        t2 += gm * (rv - em);
                    }
                    o[c] = v;
                }
                store_cells(ro, off0 + j * kRow * 4, o);
            }
            if constexpr (EPI == 2) {
                s1 += (double)t1;
                s2 += (double)t2;
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);   // this tile's LDS reads are done before the next tile's writes
            __builtin_amdgcn_wave_barrier();
        }
        if (st_it < 2) HRL_STAMP(6 * st_it + 4);
    }
    HRL_STAMP(12);
    // weight-gradient partials: waves 1..3 through LDS, wave 0 folds ((w0 + w1) + w2) + w3 and writes
    // partial[block][tap][ci][co] (C/D layout of 32x32x16: col = co = r, row = ci = (i&3) + 8(i>>2) + 4h)
    __syncthreads();
    float *red = smem;
    if (wave > 0) {
#pragma unroll
        for (int t = 0; t < kTaps; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int ci = (i & 3) + 8 * (i >> 2) + 4 * h;
                red[(wave - 1) * kW + (t * kC + ci) * kC + r] = wacc[t][i];
            }
    }
    __syncthreads();
    if (wave == 0) {
        float *out = a.wpart + (int64_t)blockIdx.x * kW;
#pragma unroll
        for (int t = 0; t < kTaps; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int idx = (t * kC + (i & 3) + 8 * (i >> 2) + 4 * h) * kC + r;
                out[idx] = ((wacc[t][i] + red[idx]) + red[kW + idx]) + red[2 * kW + idx];
            }
    }
    if constexpr (DG && EPI == 2) {   // BN_{i-1}'s sums: lanes (h, r) of the 4 waves, fixed order
        __syncthreads();
        double *dred = reinterpret_cast<double *>(smem);
        dred[((wave * 2 + h) * kC + r) * 2 + 0] = s1;
        dred[((wave * 2 + h) * kC + r) * 2 + 1] = s2;
        __syncthreads();
        if (threadIdx.x < 2 * kC) {
            const int c = threadIdx.x >> 1, k = threadIdx.x & 1;
            double t = 0.0;
            for (int i = 0; i < 2 * kWaves; ++i) t += dred[(i * kC + c) * 2 + k];
            a.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = t;
        }
    }
    HRL_STAMP(13);
    HRL_STAMP_WALL(15);
}

// ------------------------------------------------------------------ one chain block's backward, tile-shared
// conv3x3_block_bwd_kernel gives every wave a 16-row tile of its own and runs load + BN apply, the weight
// gradient and the input gradient back to back with one wave per SIMD: HBM is busy in the load phase only and
// idles through both MFMA phases (no registers left for a prefetch; profiles/r02_stamps_block_bwd.txt).  This
// form shares each tile among a workgroup of 8 waves (2 per SIMD) and pipelines the tiles:
//  * every wave stages 1/8 of tile k+1 -- BN_i's backward apply gives dY, the prologue gives x' = relu(x*a + b),
//    both split exactly into bf16 h/m/l parts -- into a second LDS buffer while the tile-k MFMAs run, and its
//    loads of tile k+2 are in flight behind that (30 registers per lane);
//  * LDS per buffer: dY and x' as part images [part][cell][channel][row] (27 KB each), so no MFMA operand is
//    split twice and none needs VALU: the weight gradient reads x'_p and dY_q (channel per lane, 8 rows) with
//    ds_read_b128, the input gradient reads dY_p (row per lane, 8 channels) with ds_read_b64_tr_b16 (T10);
//    the 16-byte chunks are XOR-swizzled so these reads are conflict-free, and a wave stages a diagonal of
//    (channel, row pair)s so the stage's 4-byte writes are too;
//  * waves 4-7 own the weight gradient (taps {0,1}, {2,5}, {3,4}, {6,7,8}), waves 0-3 the input gradient
//    (column tile ct = wave & 1, output cells {4..8} or {0..3}) with the h and m parts of their weights in
//    registers (the l parts in LDS); the MFMA cycles of each SIMD's two waves (w, w+4) are balanced to 2 %;
//  * the two waves of a SIMD order their phases oppositely (the heavier one computes first), so one wave's
//    staging VALU and LDS writes run beside its partner's MFMAs;
//  * the epilogue re-reads the raw x it needs (its loads are issued before the tile's MFMAs) and each input-
//    gradient wave stores its gin block straight from the accumulators right after its MFMAs (per row one run of
//    4-5 floats), so one barrier per tile remains and no wave waits for a staged gin tile.
// The input gradient runs split_tile_mfma's arithmetic in its order (bit-identical gin); the weight gradient sums
// each tap over the workgroup's tiles in one accumulator: the same pairs in the same per-tile order, a different
// association across tiles than the per-wave kernel.
namespace bb2 {

// diagnostic variants (tools/bb2_variants.sh builds them; the product is 0): bit 1 = no stage VALU (raw bits
// packed into the images), bit 2 = no MFMA phase, bit 4 = no epilogue / gin store, bit 8 = every wave computes
// first, bit 16 = no gin store (epilogue kept), bit 32 = raised wave priority (s_setprio 2) through the MFMA phase
#ifndef BB2_VARIANT
#define BB2_VARIANT 0
#endif
constexpr int kVariant = BB2_VARIANT;

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kPartBytes = kCells * kC * kTile * 2;        // one bf16 part image (9 KB)
constexpr int kImgBytes = 3 * kPartBytes;                  // h, m, l (27 KB)
constexpr int kDy0 = 0;                                    // dY images, buffers 0/1
constexpr int kX0 = 2 * kImgBytes;                         // x' images, buffers 0/1
// the epilogue's raw x (fp32, [row][channel][cell], rows kXrStride floats apart), buffers 0/1: staged with the
// images instead of re-read from HBM (the re-read cost more than the MFMAs: tools/bb2_variants.sh)
constexpr int kXrStride = kRow + 4;                        // 292: the 4 row groups of a read 16 banks apart
constexpr int kXrBytes = kTile * kXrStride * 4;            // 18,688 B
constexpr int kXr0 = 4 * kImgBytes;
constexpr int kLdsBytes = kXr0 + 2 * kXrBytes;             // 147,968 B
static_assert(kLdsBytes <= 160 * 1024, "LDS");

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// byte offset of the 16-byte chunk holding rows 8*half .. 8*half+7 of (cell c, channel ch) in a part image:
// chunk (2*(ch&7) + half) ^ 9*((ch>>3)&1) of the cell's 256-byte row ch>>3
__device__ __forceinline__ int img_off(int c, int ch, int half) {
    const int R = ch >> 3, j = ch & 7;
    return c * 1024 + R * 256 + 16 * ((2 * j + half) ^ (9 * (R & 1)));
}

__device__ __forceinline__ void bar_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// wave roles: input-gradient waves 0-3 (column tile kCt, output cells kQ[0..kNq)), weight-gradient waves 4-7
// (taps kTap[0..kNt)); kCFirst: compute before staging
template <int W> struct Role;
template <> struct Role<0> { static constexpr bool kIg = true, kCFirst = true; static constexpr int kCt = 0, kNq = 5, kNt = 0;
                             static constexpr int kQ[5] = {4, 5, 6, 7, 8}; static constexpr int kTap[1] = {0}; };
template <> struct Role<1> { static constexpr bool kIg = true, kCFirst = true; static constexpr int kCt = 1, kNq = 5, kNt = 0;
                             static constexpr int kQ[5] = {4, 5, 6, 7, 8}; static constexpr int kTap[1] = {0}; };
template <> struct Role<2> { static constexpr bool kIg = true, kCFirst = false; static constexpr int kCt = 0, kNq = 4, kNt = 0;
                             static constexpr int kQ[4] = {0, 1, 2, 3}; static constexpr int kTap[1] = {0}; };
template <> struct Role<3> { static constexpr bool kIg = true, kCFirst = false; static constexpr int kCt = 1, kNq = 4, kNt = 0;
                             static constexpr int kQ[4] = {0, 1, 2, 3}; static constexpr int kTap[1] = {0}; };
template <> struct Role<4> { static constexpr bool kIg = false, kCFirst = false; static constexpr int kCt = 0, kNq = 0, kNt = 2;
                             static constexpr int kQ[1] = {0}; static constexpr int kTap[2] = {0, 1}; };
template <> struct Role<5> { static constexpr bool kIg = false, kCFirst = false; static constexpr int kCt = 0, kNq = 0, kNt = 2;
                             static constexpr int kQ[1] = {0}; static constexpr int kTap[2] = {2, 5}; };
template <> struct Role<6> { static constexpr bool kIg = false, kCFirst = true; static constexpr int kCt = 0, kNq = 0, kNt = 2;
                             static constexpr int kQ[1] = {0}; static constexpr int kTap[2] = {3, 4}; };
template <> struct Role<7> { static constexpr bool kIg = false, kCFirst = true; static constexpr int kCt = 0, kNq = 0, kNt = 3;
                             static constexpr int kQ[1] = {0}; static constexpr int kTap[3] = {6, 7, 8}; };

// does the wave's work involve input cell p (weight gradient: x'_p; input gradient: dY_p)?
template <int W> __device__ constexpr bool uses_p(int p) {
    using R = Role<W>;
    if constexpr (R::kIg) {
        for (int s = 0; s < R::kNq; ++s)
            if (tap_of(p, R::kQ[s]) >= 0) return true;
    } else {
        for (int s = 0; s < R::kNt; ++s) {
            const int dy = R::kTap[s] / 3, dx = R::kTap[s] % 3;
            const int qy = p / 3 - dy + 1, qx = p % 3 - dx + 1;
            if (qy >= 0 && qy < 3 && qx >= 0 && qx < 3) return true;
        }
    }
    return false;
}
// does the input-gradient wave use tap t?
template <int W> __device__ constexpr bool uses_tap(int t) {
    using R = Role<W>;
    for (int s = 0; s < R::kNq; ++s)
        for (int p = 0; p < kCells; ++p)
            if (tap_of(p, R::kQ[s]) == t) return true;
    return false;
}

// diagnostic build (-DHRL_STAMPS, tools/bb2_stamps.py): lane 0 of every wave writes the shader clock at the
// phase boundaries of iterations 2 and 3, WITHOUT draining (the wave's issue timeline; the compiler's own waits
// for loaded registers stay where they are): slot = ((block * 8 + wave) * 2 + iteration - 2) * 8 + point
#ifdef HRL_STAMPS
#define BB2_STAMP(it, k)                                                                                        \
    do {                                                                                                       \
        if ((it) == 2 || (it) == 3) {                                                                          \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
            if (lane == 0 && g_hrl_stamps)                                                                     \
                g_hrl_stamps[(((size_t)blockIdx.x * 8 + W) * 2 + (it) - 2) * 8 + (k)] = t_;                    \
        }                                                                                                      \
    } while (0)
#else
#define BB2_STAMP(it, k) do { } while (0)
#endif

template <bool PRO, int EPI, int W>
__device__ __forceinline__ void run(const BlockBwdArgs &a, unsigned char *smem, int lane) {
    using R = Role<W>;
    constexpr bool kIg = R::kIg;
    constexpr int kNq = R::kNq > 0 ? R::kNq : 1;
    constexpr int kNt = R::kNt > 0 ? R::kNt : 1;
    constexpr int kCt = R::kCt;
    const int ch = lane & 31, hh = lane >> 5;
    // EPI 1 (kFwd): the forward conv in this form -- the staged image is x' = relu(x a + b) instead of dY, the
    // input-gradient waves compute the conv with the forward weights, the weight-gradient waves only stage, and the
    // epilogue emits the BN statistics of the output (conv3x3_kernel<PRO, 1>'s sums)
    constexpr bool kFwd = EPI == 1;
    // BN_i's backward apply for channel ch (bn_bwd_apply_kernel's per-channel values), the prologue's BN_{i-1}
    float mu = 0.f, kk = 0.f, gmn = 0.f, is = 1.f, ww = 1.f, al = 1.f, be = 0.f;
    if constexpr (!kFwd) {
        // BN_i's backward finalize (bnfold) first, while the registers are free (beside tile 0's loads it spilled)
        if (a.fold_part) bnfold::fold(a, smem, kk, gmn);
        else { kk = a.bn_k[ch]; gmn = a.bn_gm[ch]; }
        mu = a.bn_mean[ch]; is = a.bn_invstd[ch];
        ww = a.bn_w ? a.bn_w[ch] : 1.0f;
        al = is * ww;
        be = (a.bn_b ? a.bn_b[ch] : 0.0f) - mu * al;
    }
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {
        pa = a.in_alpha[ch];
        pb = a.in_beta[ch];
    }
    // the input gradient's weights: all three parts of its taps in registers ([tap][ct][part][lane] layout of
    // conv3x3_block_bwd_kernel's LDS fragments: lane l holds W'[tap][ci = 8(l>>4) + e][co = 16ct + (l&15)])
    uint4 wh[kTaps], wm[kTaps], wl[kTaps];
    if constexpr (kIg) {
        const int ci0 = 8 * (lane >> 4), j = lane & 15;
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            if (!uses_tap<W>(t)) continue;
            uint32_t hv[4], mv[4], lv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int tc = t * 2 + kCt;
                const float w0 = a.wpk[(tc * kC + ci0 + 2 * d) * 16 + j];
                const float w1 = a.wpk[(tc * kC + ci0 + 2 * d + 1) * 16 + j];
                uint32_t h0, m0, l0, h1, m1, l1;
                hrl_split::split3(w0, h0, m0, l0);
                hrl_split::split3(w1, h1, m1, l1);
                hv[d] = h0 | (h1 << 16);
                mv[d] = m0 | (m1 << 16);
                lv[d] = l0 | (l1 << 16);
            }
            wh[t] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            wm[t] = make_uint4(mv[0], mv[1], mv[2], mv[3]);
            wl[t] = make_uint4(lv[0], lv[1], lv[2], lv[3]);
        }
    }
    float em = 0.f, ea = 1.f, eb = 0.f;     // epilogue 2: BN_{i-1} of this lane's output channel
    if constexpr (EPI == 2 && kIg) {
        em = a.ep_mean[kCt * 16 + (lane & 15)];
        ea = a.ep_alpha[kCt * 16 + (lane & 15)];
        eb = a.ep_beta[kCt * 16 + (lane & 15)];
    }
    double s1 = 0.0, s2 = 0.0;
    f32x16 wacc[kNt];
#pragma unroll
    for (int t = 0; t < kNt; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) wacc[t][i] = 0.f;

    const int64_t ntiles = (a.M + kTile - 1) / kTile;
    const int64_t t0 = blockIdx.x;
    const int64_t step = gridDim.x;
    const int n_iter = t0 < ntiles ? (int)((ntiles - 1 - t0) / step + 1) : 0;
    // this lane stages rows rho0, rho0 + 1 (a diagonal over the waves: conflict-free image writes) and cells
    // c0 .. c0+4 of channel ch (lanes hh = 1 take cells 4..8)
    const int rho0 = 2 * ((W + (ch >> 2)) & 7);
    const int c0 = hh ? 4 : 0;
    const int ldoff = (rho0 * kRow + ch * kCells + c0) * 4;
    float G[2][5], Y[2][5], X[2][5];
    auto rsrc_of = [&](const float *base, int it, int &rows) __attribute__((always_inline)) {
        const int64_t t = t0 + (int64_t)it * step;
        const bool ok = it < n_iter;
        rows = ok ? (int)min<int64_t>(kTile, a.M - t * kTile) : 0;
        return wave_rsrc(base + (ok ? t * kTile * kRow : 0), (uint32_t)rows * kRow * 4);
    };
    auto issue = [&](int it) __attribute__((always_inline)) {   // loads of iteration it's tile (zeros past the end)
        int rows;
        const __amdgpu_buffer_rsrc_t rg = rsrc_of(a.g, it, rows), ry = rsrc_of(a.y, it, rows),
                                     rx = rsrc_of(a.x, it, rows);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int off = ldoff + r * kRow * 4;
#pragma unroll
            for (int k = kFwd ? 2 : 0; k < 3; ++k) {
                const __amdgpu_buffer_rsrc_t rs = k == 0 ? rg : (k == 1 ? ry : rx);
                float(&d)[5] = k == 0 ? G[r] : (k == 1 ? Y[r] : X[r]);
                const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
                const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 12, 0, 0);
                d[0] = __uint_as_float(v.x);
                d[1] = __uint_as_float(v.y);
                d[2] = __uint_as_float(v.z);
                d[3] = __uint_as_float(u.x);
                d[4] = __uint_as_float(u.y);
            }
        }
    };
    auto stage = [&](int it) __attribute__((always_inline)) {   // registers -> the images of buffer it & 1
        const int64_t t = t0 + (int64_t)it * step;
        const int rows = (int)max<int64_t>(0, min<int64_t>(kTile, a.M - t * kTile));
        unsigned char *dyi = smem + kDy0 + (it & 1) * kImgBytes;
        unsigned char *xi = smem + kX0 + (it & 1) * kImgBytes;
        uint32_t dp[3][5], xp[3][5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            float dv[2], xv2[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                // dY = BN_i backward apply (bn_bwd_apply_kernel's float operations); rows past the batch are 0
                const bool valid = rho0 + r < rows;
                const float yv = Y[r][i];
                float gv = G[r][i];
                if (!(yv * al + be > 0.f)) gv = 0.f;
                const float tt = (yv - mu) * kk;
                float d = (((gv - gmn) - tt) * is) * ww;
                d = valid ? d : 0.f;
                float xv = X[r][i];
                if constexpr (PRO) {   // bn_apply_kernel's float operations
                    const float u = xv * pa + pb;
                    xv = u < 0.f ? 0.f : u;
                }
                if constexpr (kFwd) d = xv;   // the forward's A operand: x' in the input-gradient waves' image
                dv[r] = d;
                xv2[r] = xv;
            }
            if constexpr (kVariant & 1) {
                dp[0][i] = dp[1][i] = dp[2][i] = __builtin_amdgcn_perm(__float_as_uint(G[1][i]), __float_as_uint(G[0][i]), 0x07060302u);
                xp[0][i] = xp[1][i] = __builtin_amdgcn_perm(__float_as_uint(X[1][i]), __float_as_uint(X[0][i]), 0x07060302u);
                xp[2][i] = __builtin_amdgcn_perm(__float_as_uint(Y[1][i]), __float_as_uint(Y[0][i]), 0x07060302u);
            } else {
                hrl_split::split_pair(dv[0], dv[1], dp[0][i], dp[1][i], dp[2][i]);
                if constexpr (!kFwd) hrl_split::split_pair(xv2[0], xv2[1], xp[0][i], xp[1][i], xp[2][i]);
            }
        }
        const int half = rho0 >> 3, sub = 2 * (rho0 & 7);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = img_off(c0 + i, ch, half) + sub;
#pragma unroll
            for (int part = 0; part < 3; ++part) {
                *reinterpret_cast<uint32_t *>(dyi + part * kPartBytes + o) = dp[part][i];
                if constexpr (!kFwd) *reinterpret_cast<uint32_t *>(xi + part * kPartBytes + o) = xp[part][i];
            }
        }
        if constexpr (EPI == 2 || EPI == 3) {   // the epilogue's raw x (rows past the batch are loaded as 0)
            float *xr = reinterpret_cast<float *>(smem + kXr0 + (it & 1) * kXrBytes);
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int i = 0; i < 5; ++i) xr[(rho0 + r) * kXrStride + ch * kCells + c0 + i] = X[r][i];
        }
    };
    f32x4 acc[kNq];
    auto compute = [&](int it) __attribute__((always_inline)) {
        const unsigned char *dyi = smem + kDy0 + (it & 1) * kImgBytes;
        if constexpr (kVariant & 2) {
            if constexpr (kIg) {
#pragma unroll
                for (int s = 0; s < kNq; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
            }
        } else if constexpr (!kIg && kFwd) {
            // the forward has no weight gradient: these waves only stage
        } else if constexpr (!kIg) {
            // weight gradient: dW[tap] += x'_p^T (32 ci x 16 rows) . dY_q (16 rows x 32 co), p ascending
            const unsigned char *xi = smem + kX0 + (it & 1) * kImgBytes;
            const int kg = lane >> 5;
#pragma unroll
            for (int p = 0; p < kCells; ++p) {
                if (!uses_p<W>(p)) continue;
                const int o = img_off(p, ch, kg);
                const uint4 Ah = *reinterpret_cast<const uint4 *>(xi + o);
                const uint4 Am = *reinterpret_cast<const uint4 *>(xi + kPartBytes + o);
                const uint4 Al = *reinterpret_cast<const uint4 *>(xi + 2 * kPartBytes + o);
#pragma unroll
                for (int s = 0; s < R::kNt; ++s) {
                    const int dy = R::kTap[s] / 3, dx = R::kTap[s] % 3;
                    const int qy = p / 3 - dy + 1, qx = p % 3 - dx + 1;
                    if (qy < 0 || qy > 2 || qx < 0 || qx > 2) continue;
                    const int ob = img_off(qy * 3 + qx, ch, kg);
                    const uint4 Bh = *reinterpret_cast<const uint4 *>(dyi + ob);
                    const uint4 Bm = *reinterpret_cast<const uint4 *>(dyi + kPartBytes + ob);
                    const uint4 Bl = *reinterpret_cast<const uint4 *>(dyi + 2 * kPartBytes + ob);
                    f32x16 c = wacc[s];
                    c = mfma32(Al, Bh, c);   // smallest terms first
                    c = mfma32(Am, Bm, c);
                    c = mfma32(Ah, Bl, c);
                    c = mfma32(Am, Bh, c);
                    c = mfma32(Ah, Bm, c);
                    c = mfma32(Ah, Bh, c);
                    wacc[s] = c;
                }
            }
        } else {
            // input gradient blocks (q, kCt): acc += sum_p dY_p (16 rows x 32 co) . W'[tap(p, q)][kCt], p ascending
#pragma unroll
            for (int s = 0; s < kNq; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
            const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
            const int tr_sub = 8 * (pp & 1);
#pragma unroll
            for (int p = 0; p < kCells; ++p) {
                if (!uses_p<W>(p)) continue;
                uint32_t A[3][4];
#pragma unroll
                for (int part = 0; part < 3; ++part) {
#pragma unroll
                    for (int hlf = 0; hlf < 2; ++hlf) {
                        const int o = part * kPartBytes + img_off(p, 8 * g + 4 * hlf + qq, pp >> 1) + tr_sub;
                        const v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_v4s *)((__attribute__((address_space(3))) unsigned char *)(dyi + o)));
                        const uint2 u = __builtin_bit_cast(uint2, r);
                        A[part][2 * hlf] = u.x;
                        A[part][2 * hlf + 1] = u.y;
                    }
                }
                const uint4 Ah = make_uint4(A[0][0], A[0][1], A[0][2], A[0][3]);
                const uint4 Am = make_uint4(A[1][0], A[1][1], A[1][2], A[1][3]);
                const uint4 Al = make_uint4(A[2][0], A[2][1], A[2][2], A[2][3]);
#pragma unroll
                for (int s = 0; s < R::kNq; ++s) {
                    const int tap = tap_of(p, R::kQ[s]);
                    if (tap < 0) continue;
                    const uint4 Bl = wl[tap];
                    f32x4 c = acc[s];
                    c = mfma_bf16(Al, wh[tap], c);   // smallest terms first
                    c = mfma_bf16(Am, wm[tap], c);
                    c = mfma_bf16(Ah, Bl, c);
                    c = mfma_bf16(Am, wh[tap], c);
                    c = mfma_bf16(Ah, wm[tap], c);
                    c = mfma_bf16(Ah, wh[tap], c);
                    acc[s] = c;
                }
            }
        }
    };
    auto epilogue = [&](int it) __attribute__((always_inline)) {   // accumulators -> gin, straight from registers
        if constexpr (kIg && !(kVariant & 4)) {
            int rows;
            const __amdgpu_buffer_rsrc_t ro = rsrc_of(a.gin, it, rows);
            const int co = kCt * 16 + (lane & 15);
            // the raw x of the wave's output cells, staged in LDS with the tile's images
            float rv[kNq < 4 ? 4 : kNq][4];
            if constexpr (EPI == 2 || EPI == 3) {
                const float *xr = reinterpret_cast<const float *>(smem + kXr0 + (it & 1) * kXrBytes);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = (lane >> 4) * 4 + rr;
#pragma unroll
                    for (int s = 0; s < R::kNq; ++s) rv[s][rr] = xr[row * kXrStride + co * kCells + R::kQ[s]];
                }
            }
            if constexpr (EPI == 1) {   // the output's BN statistics (conv3x3_kernel<PRO, 1>'s sums)
                float t1 = 0.f, t2 = 0.f;
#pragma unroll
                for (int s = 0; s < R::kNq; ++s) {
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = (lane >> 4) * 4 + rr;
                        const float u = row < rows ? acc[s][rr] : 0.f;
                        t1 += u;
                        t2 += u * u;
                    }
                }
                s1 += (double)t1;
                s2 += (double)t2;
            }
            if constexpr (EPI == 2) {   // bn_bwd_reduce_kernel's mask and sums
                float t1 = 0.f, t2 = 0.f;
#pragma unroll
                for (int s = 0; s < R::kNq; ++s) {
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = (lane >> 4) * 4 + rr;     // C/D: row = (lane>>4)*4 + reg, col = lane & 15
                        const float x0 = rv[s][rr];
                        const float gm = (x0 * ea + eb > 0.f && row < rows) ? acc[s][rr] : 0.f;
                        t1 += gm;
                        t2 += gm * (x0 - em);
                    }
                }
                s1 += (double)t1;
                s2 += (double)t2;
            }
            // per row the wave's output cells are one run of kNq floats (rows past the batch: dropped)
            if constexpr (!(kVariant & 16)) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = (lane >> 4) * 4 + rr;
                    const int off = (row * kRow + co * kCells + R::kQ[0]) * 4;
                    float v[kNq];
#pragma unroll
                    for (int s = 0; s < R::kNq; ++s) {
                        v[s] = acc[s][rr];
                        if constexpr (EPI == 3)
                            if (!(rv[s][rr] > 0.f)) v[s] = 0.f;
                    }
                    u32x4 w;
                    w.x = __float_as_uint(v[0]);
                    w.y = __float_as_uint(v[1]);
                    w.z = __float_as_uint(v[2]);
                    w.w = __float_as_uint(v[3]);
                    __builtin_amdgcn_raw_buffer_store_b128(w, ro, off, 0, 0);
                    if constexpr (R::kNq > 4)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[4 % kNq]), ro, off + 16, 0, 0);
                }
            }
        }
    };

    if (n_iter > 0) {
        issue(0);
        stage(0);
        issue(1);
    }
    bar_lds();                                      // tile 0 in LDS
    for (int it = 0; it < n_iter; ++it) {
        BB2_STAMP(it, 0);
        // stage / issue run unconditionally (past the last tile they stage and load zeros that nothing reads):
        // a branch around them makes the compiler's wait for the loaded registers vmcnt(0) at the loop head,
        // which then also waits for the previous iteration's gin stores
        if constexpr (R::kCFirst || (kVariant & 8)) {
            if constexpr (kVariant & 32) __builtin_amdgcn_s_setprio(2);
            compute(it);
            if constexpr (kVariant & 32) __builtin_amdgcn_s_setprio(0);
            epilogue(it);
            BB2_STAMP(it, 1);
            stage(it + 1);
            issue(it + 2);
            BB2_STAMP(it, 2);
        } else {
            stage(it + 1);
            issue(it + 2);
            BB2_STAMP(it, 1);
            if constexpr (kVariant & 32) __builtin_amdgcn_s_setprio(2);
            compute(it);
            if constexpr (kVariant & 32) __builtin_amdgcn_s_setprio(0);
            epilogue(it);
            BB2_STAMP(it, 2);
        }
        bar_lds();                                  // tile it+1 staged, tile it's images free
        BB2_STAMP(it, 3);
    }
    // weight-gradient partials partial[block][tap][ci][co] (C/D layout of 32x32x16: col = co = lane & 31,
    // row = ci = (i&3) + 8(i>>2) + 4h); each tap has one owner wave: no fold inside the workgroup
    if constexpr (!kIg && !kFwd) {
        constexpr int kW = kTaps * kC * kC;
        float *outp = a.wpart + (int64_t)blockIdx.x * kW;
        const int h = lane >> 5;
#pragma unroll
        for (int s = 0; s < R::kNt; ++s)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int ci = (i & 3) + 8 * (i >> 2) + 4 * h;
                outp[(R::kTap[s] * kC + ci) * kC + ch] = wacc[s][i];
            }
    }
    if constexpr (EPI == 1 || EPI == 2) {   // the sums: waves 0-3 [wave][lane] -> channel (wave&1)*16 + (lane&15)
        __syncthreads();
        double *dred = reinterpret_cast<double *>(smem);
        if (kIg) {
            dred[(W * 64 + lane) * 2 + 0] = s1;
            dred[(W * 64 + lane) * 2 + 1] = s2;
        }
        __syncthreads();
        if (W == 0) {
            const int c = lane >> 1, k = lane & 1, ct = c >> 4, l16 = c & 15;
            double tot = 0.0;
            for (int w = ct; w < 4; w += 2)
                for (int lg = 0; lg < 4; ++lg) tot += dred[(w * 64 + lg * 16 + l16) * 2 + k];
            a.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = tot;
        }
    }
}

}  // namespace bb2

// ------------------------------------------------------------------ one chain block's backward, two workgroups per CU
// conv3x3_block_bwd4_kernel<PRO, EPI, DG> (block form 2): bb2's arithmetic with the CU shared by TWO independent
// 4-wave workgroups instead of one 8-wave workgroup.  bb2 double-buffered its images in 148 KB of LDS, so one
// workgroup filled the CU and all 8 waves met at every tile's barrier: a wave whose loads came late held the other
// seven (18-28 % of every tile at the barrier, MFMA busy 0.39 of the SIMD cycles: profiles/r05_bb2_stamps.txt).
// Here a workgroup's images are single-buffered (dY and x' part images 2 x 27 KB + the epilogue's raw x 18.3 KB =
// 72.3 KB), so two workgroups reside on every CU, one wave of each on every SIMD, and each runs
//     MFMAs of tile k + epilogue | barrier | stage tile k+1 (registers -> images) | issue the loads of tile k+2 | barrier
// -- while one workgroup waits at a barrier or stages, the other's MFMAs run on the same SIMDs: the tile skew is
// absorbed by the other workgroup instead of costing all eight waves.  Per workgroup:
//  * waves 0, 1: the input gradient of column tile ct = wave for ALL nine output cells (49 (p, q) pairs, 294
//    v_mfma_f32_16x16x32_bf16), the three split parts of their weights in registers; a row's nine cells leave in
//    one 36-byte run per lane (two dwordx4 + one dword);
//  * waves 2, 3: the weight gradient of taps {0, 2, 4, 6, 8} (25 pairs) and {1, 3, 5, 7} (24 pairs), 32x32x16;
//  * the waves stage the tile as bb2's eight (row pair, channel) diagonals: one each for the input-gradient waves
//    (30 registers of loads in flight per lane beside their 144 of weights and accumulators), three each for the
//    weight-gradient waves (90).
// Same operands, same images and the same per-accumulator MFMA order as bb2: the input gradient is bit-identical;
// the weight gradient sums 16 instead of 32 tiles per partial row (512 rows per launch: a different association
// across tiles); the epilogue-2 sums are per workgroup (hrl_conv3x3_block_sum_blocks rows).
namespace bb4 {

// diagnostic variants (tools/bb4_variants.sh; the product is 0): bit 1 = loads of the first tile only, bit 2 = no
// MFMA phase, bit 4 = no epilogue / gin store
#ifndef BB4_VARIANT
#define BB4_VARIANT 0
#endif
constexpr int kVariant = BB4_VARIANT;

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kPartBytes = bb2::kPartBytes;
constexpr int kImgBytes = bb2::kImgBytes;
constexpr int kDy0 = 0;
constexpr int kX0 = kImgBytes;
constexpr int kXrStride = bb2::kXrStride;                  // 292
constexpr int kXrBytes = bb2::kXrBytes;
constexpr int kXr0 = 2 * kImgBytes;
constexpr int kLdsBytes = kXr0 + kXrBytes;                 // 73,984 B
static_assert(2 * kLdsBytes <= 160 * 1024, "two workgroups per CU");
constexpr int kPerCu = 2;                                  // resident workgroups per CU
constexpr int kGrid = 256 * kPerCu;

// the weight-gradient waves' taps: corners + centre (4 x 4 + 9 = 25 pairs) and edges (4 x 6 = 24)
template <int W> struct Taps;
template <> struct Taps<2> { static constexpr int kN = 5; static constexpr int kT[5] = {0, 2, 4, 6, 8}; };
template <> struct Taps<3> { static constexpr int kN = 4; static constexpr int kT[4] = {1, 3, 5, 7}; };
template <> struct Taps<0> { static constexpr int kN = 1; static constexpr int kT[1] = {0}; };
template <> struct Taps<1> { static constexpr int kN = 1; static constexpr int kT[1] = {0}; };

// the (row pair, channel) diagonals a wave stages (bb2's diagonal of wave D: rows 2 ((D + ch/4) & 7) + {0, 1}), 30
// registers of loads each: one for each input-gradient wave (108 registers of weights, 20 of accumulators, the
// epilogue), three for each weight-gradient wave (80 / 64 accumulators) -- no wave spills (a spill reload is a
// vector-memory operation: its wait would also wait for the next tile's loads)
template <int W> struct Diags;
template <> struct Diags<0> { static constexpr int kN = 1; static constexpr int kD[1] = {0}; };
template <> struct Diags<1> { static constexpr int kN = 1; static constexpr int kD[1] = {1}; };
template <> struct Diags<2> { static constexpr int kN = 3; static constexpr int kD[3] = {2, 4, 6}; };
template <> struct Diags<3> { static constexpr int kN = 3; static constexpr int kD[3] = {3, 5, 7}; };

// the lane id from an instruction the compiler may not hoist: the staging addresses derived from it are recomputed
// where they are used (a few VALU) instead of held across the loop in registers the input-gradient waves lack
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <bool PRO, int EPI, bool DG, int W>
__device__ __forceinline__ void run(const BlockBwdArgs &a, unsigned char *smem, int lane, int delay) {
    constexpr bool kIg = W < 2;
    constexpr int kCt = W & 1;
    constexpr int kNt = Taps<W>::kN;
    const int ch = lane & 31, hh = lane >> 5;
    // BN_i's backward apply for channel ch (bn_bwd_apply_kernel's per-channel values), the prologue's BN_{i-1}
    const float mu = a.bn_mean[ch], kk = a.bn_k[ch], gmn = a.bn_gm[ch], is = a.bn_invstd[ch];
    const float ww = a.bn_w ? a.bn_w[ch] : 1.0f;
    const float al = is * ww;
    const float be = (a.bn_b ? a.bn_b[ch] : 0.0f) - mu * al;
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {
        pa = a.in_alpha[ch];
        pb = a.in_beta[ch];
    }
    // the input gradient's weights, all three parts of all nine taps in registers (bb2's fragment layout)
    uint4 wh[kTaps], wm[kTaps], wl[kTaps];
    if constexpr (kIg && DG) {
        const int ci0 = 8 * (lane >> 4), j = lane & 15;
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            uint32_t hv[4], mv[4], lv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int tc = t * 2 + kCt;
                const float w0 = a.wpk[(tc * kC + ci0 + 2 * d) * 16 + j];
                const float w1 = a.wpk[(tc * kC + ci0 + 2 * d + 1) * 16 + j];
                uint32_t h0, m0, l0, h1, m1, l1;
                hrl_split::split3(w0, h0, m0, l0);
                hrl_split::split3(w1, h1, m1, l1);
                hv[d] = h0 | (h1 << 16);
                mv[d] = m0 | (m1 << 16);
                lv[d] = l0 | (l1 << 16);
            }
            wh[t] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            wm[t] = make_uint4(mv[0], mv[1], mv[2], mv[3]);
            wl[t] = make_uint4(lv[0], lv[1], lv[2], lv[3]);
        }
    }
    float em = 0.f, ea = 1.f, eb = 0.f;     // epilogue 2: BN_{i-1} of this lane's output channel
    if constexpr (EPI == 2 && kIg && DG) {
        em = a.ep_mean[kCt * 16 + (lane & 15)];
        ea = a.ep_alpha[kCt * 16 + (lane & 15)];
        eb = a.ep_beta[kCt * 16 + (lane & 15)];
    }
    double s1 = 0.0, s2 = 0.0;
    f32x16 wacc[kNt];
#pragma unroll
    for (int t = 0; t < kNt; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) wacc[t][i] = 0.f;

    const int64_t ntiles = (a.M + kTile - 1) / kTile;
    const int64_t t0 = blockIdx.x;
    const int64_t step = gridDim.x;
    const int n_iter = t0 < ntiles ? (int)((ntiles - 1 - t0) / step + 1) : 0;
    // this lane stages rows rho_of(j), rho_of(j) + 1 (bb2's diagonals Diags<W>::kD) and cells c0 .. c0+4 of channel
    // ch (lanes hh = 1 take cells 4..8)
    constexpr int kNd = Diags<W>::kN;
    auto rho_of = [](int j, int c) __attribute__((always_inline)) { return 2 * ((Diags<W>::kD[j] + (c >> 2)) & 7); };
    float G[kNd][2][5], Y[kNd][2][5], X[kNd][2][5];
    auto rsrc_of = [&](const float *base, int it, int &rows) __attribute__((always_inline)) {
        const int64_t t = t0 + (int64_t)it * step;
        const bool ok = it < n_iter;
        rows = ok ? (int)min<int64_t>(kTile, a.M - t * kTile) : 0;
        return wave_rsrc(base + (ok ? t * kTile * kRow : 0), (uint32_t)rows * kRow * 4);
    };
    auto issue = [&](int it) __attribute__((always_inline)) {   // loads of iteration it's tile (zeros past the end)
        if constexpr (kVariant & 1) {
            if (it > 0) return;
        }
        int rows;
        const __amdgpu_buffer_rsrc_t rg = rsrc_of(a.g, it, rows), ry = rsrc_of(a.y, it, rows),
                                     rx = rsrc_of(a.x, it, rows);
        const int ln = fresh_lane(), cl = ln & 31, c0 = (ln >> 5) ? 4 : 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int j = 0; j < kNd; ++j) {
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int off = ((rho_of(j, cl) + r) * kRow + cl * kCells + c0) * 4;
                    const __amdgpu_buffer_rsrc_t rs = k == 0 ? rg : (k == 1 ? ry : rx);
                    float(&d)[5] = k == 0 ? G[j][r] : (k == 1 ? Y[j][r] : X[j][r]);
                    const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
                    const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 12, 0, 0);
                    d[0] = __uint_as_float(v.x);
                    d[1] = __uint_as_float(v.y);
                    d[2] = __uint_as_float(v.z);
                    d[3] = __uint_as_float(u.x);
                    d[4] = __uint_as_float(u.y);
                }
            }
        }
    };
    unsigned char *dyi = smem + kDy0;
    unsigned char *xi = smem + kX0;
    float *xr = reinterpret_cast<float *>(smem + kXr0);
    auto stage = [&](int it) __attribute__((always_inline)) {   // registers -> the images
        const int64_t t = t0 + (int64_t)it * step;
        const int rows = (int)max<int64_t>(0, min<int64_t>(kTile, a.M - t * kTile));
        const int ln = fresh_lane(), cl = ln & 31, c0 = (ln >> 5) ? 4 : 0;
#pragma unroll
        for (int j = 0; j < kNd; ++j) {
            const int rj = rho_of(j, cl);
            uint32_t dp[3][5], xp[3][5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                float dv[2], xv2[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    // dY = BN_i backward apply (bn_bwd_apply_kernel's float operations); rows past the batch are 0
                    const bool valid = rj + r < rows;
                    const float yv = Y[j][r][i];
                    float gv = G[j][r][i];
                    if (!(yv * al + be > 0.f)) gv = 0.f;
                    const float tt = (yv - mu) * kk;
                    float d = (((gv - gmn) - tt) * is) * ww;
                    dv[r] = valid ? d : 0.f;
                    float xv = X[j][r][i];
                    if constexpr (PRO) {   // bn_apply_kernel's float operations
                        const float u = xv * pa + pb;
                        xv = u < 0.f ? 0.f : u;
                    }
                    xv2[r] = xv;
                }
                hrl_split::split_pair(dv[0], dv[1], dp[0][i], dp[1][i], dp[2][i]);
                hrl_split::split_pair(xv2[0], xv2[1], xp[0][i], xp[1][i], xp[2][i]);
            }
            const int half = rj >> 3, sub = 2 * (rj & 7);
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const int o = bb2::img_off(c0 + i, cl, half) + sub;
#pragma unroll
                for (int part = 0; part < 3; ++part) {
                    *reinterpret_cast<uint32_t *>(dyi + part * kPartBytes + o) = dp[part][i];
                    *reinterpret_cast<uint32_t *>(xi + part * kPartBytes + o) = xp[part][i];
                }
            }
            if constexpr (DG && (EPI == 2 || EPI == 3)) {   // the epilogue's raw x (rows past the batch: 0)
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int i = 0; i < 5; ++i) xr[(rj + r) * kXrStride + cl * kCells + c0 + i] = X[j][r][i];
            }
        }
    };
    auto wgrad = [&]() __attribute__((always_inline)) {
        // weight gradient: dW[tap] += x'_p^T (32 ci x 16 rows) . dY_q (16 rows x 32 co), p ascending
        const int kg = lane >> 5;
#pragma unroll
        for (int p = 0; p < kCells; ++p) {
            // one input cell's operands at a time: hoisting the next cells' LDS reads spilled (see Diags)
            __builtin_amdgcn_sched_barrier(0);
            const int o = bb2::img_off(p, ch, kg);
            const uint4 Ah = *reinterpret_cast<const uint4 *>(xi + o);
            const uint4 Am = *reinterpret_cast<const uint4 *>(xi + kPartBytes + o);
            const uint4 Al = *reinterpret_cast<const uint4 *>(xi + 2 * kPartBytes + o);
#pragma unroll
            for (int s = 0; s < kNt; ++s) {
                const int dy = Taps<W>::kT[s] / 3, dx = Taps<W>::kT[s] % 3;
                const int qy = p / 3 - dy + 1, qx = p % 3 - dx + 1;
                if (qy < 0 || qy > 2 || qx < 0 || qx > 2) continue;
                const int ob = bb2::img_off(qy * 3 + qx, ch, kg);
                const uint4 Bh = *reinterpret_cast<const uint4 *>(dyi + ob);
                const uint4 Bm = *reinterpret_cast<const uint4 *>(dyi + kPartBytes + ob);
                const uint4 Bl = *reinterpret_cast<const uint4 *>(dyi + 2 * kPartBytes + ob);
                f32x16 c = wacc[s];
                c = mfma32(Al, Bh, c);   // smallest terms first
                c = mfma32(Am, Bm, c);
                c = mfma32(Ah, Bl, c);
                c = mfma32(Am, Bh, c);
                c = mfma32(Ah, Bm, c);
                c = mfma32(Ah, Bh, c);
                wacc[s] = c;
            }
        }
    };
    // input gradient blocks (q, kCt) of output cells Q0 .. Q0+NQ-1: acc[s] += sum_p dY_p (16 rows x 32 co) .
    // W'[tap(p, Q0+s)][kCt], p ascending, then their epilogue; the input-gradient waves run two such passes (cells
    // 0-4 and 5-8), so their accumulators take 20 registers instead of 36 (the spill reloads a 36-accumulator form
    // needed were vector-memory operations: each one's wait also waited for the next tile's loads)
    float t1 = 0.f, t2 = 0.f;
    auto ig_pass = [&](int it, auto q0c, auto nqc) __attribute__((always_inline)) {
        constexpr int Q0 = decltype(q0c)::value, NQ = decltype(nqc)::value;
        f32x4 acc[NQ];
#pragma unroll
        for (int s = 0; s < NQ; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (!(kVariant & 2)) {
            const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
            const int tr_sub = 8 * (pp & 1);
#pragma unroll
            for (int p = 0; p < kCells; ++p) {
                uint32_t A[3][4];
#pragma unroll
                for (int part = 0; part < 3; ++part) {
#pragma unroll
                    for (int hlf = 0; hlf < 2; ++hlf) {
                        const int o = part * kPartBytes + bb2::img_off(p, 8 * g + 4 * hlf + qq, pp >> 1) + tr_sub;
                        const bb2::v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (bb2::lds_v4s *)((__attribute__((address_space(3))) unsigned char *)(dyi + o)));
                        const uint2 u = __builtin_bit_cast(uint2, r);
                        A[part][2 * hlf] = u.x;
                        A[part][2 * hlf + 1] = u.y;
                    }
                }
                const uint4 Ah = make_uint4(A[0][0], A[0][1], A[0][2], A[0][3]);
                const uint4 Am = make_uint4(A[1][0], A[1][1], A[1][2], A[1][3]);
                const uint4 Al = make_uint4(A[2][0], A[2][1], A[2][2], A[2][3]);
#pragma unroll
                for (int s = 0; s < NQ; ++s) {
                    const int tap = tap_of(p, Q0 + s);
                    if (tap < 0) continue;
                    f32x4 c = acc[s];
                    c = mfma_bf16(Al, wh[tap], c);   // smallest terms first
                    c = mfma_bf16(Am, wm[tap], c);
                    c = mfma_bf16(Ah, wl[tap], c);
                    c = mfma_bf16(Am, wh[tap], c);
                    c = mfma_bf16(Ah, wm[tap], c);
                    c = mfma_bf16(Ah, wh[tap], c);
                    acc[s] = c;
                }
            }
        }
        if constexpr (kVariant & 4) return;
        __builtin_amdgcn_sched_barrier(0);
        // epilogue: accumulators -> gin straight from registers, per row one run of the pass's NQ cells
        int rows;
        const __amdgpu_buffer_rsrc_t ro = rsrc_of(a.gin, it, rows);
        const int co = kCt * 16 + (lane & 15);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int row = (lane >> 4) * 4 + rr;     // C/D: row = (lane>>4)*4 + reg, col = lane & 15
            float v[NQ];
#pragma unroll
            for (int s = 0; s < NQ; ++s) {
                v[s] = acc[s][rr];
                if constexpr (EPI == 2 || EPI == 3) {
                    const float x0 = xr[row * kXrStride + co * kCells + Q0 + s];
                    if constexpr (EPI == 2) {   // bn_bwd_reduce_kernel's mask and sums
                        const float gm = (x0 * ea + eb > 0.f && row < rows) ? v[s] : 0.f;
                        t1 += gm;
                        t2 += gm * (x0 - em);
                    } else {
                        if (!(x0 > 0.f)) v[s] = 0.f;
                    }
                }
            }
            const int off = (row * kRow + co * kCells + Q0) * 4;
            u32x4 w0;
            w0.x = __float_as_uint(v[0]);
            w0.y = __float_as_uint(v[1]);
            w0.z = __float_as_uint(v[2]);
            w0.w = __float_as_uint(v[3]);
            __builtin_amdgcn_raw_buffer_store_b128(w0, ro, off, 0, 0);
            if constexpr (NQ > 4) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[4 % NQ]), ro, off + 16, 0, 0);
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;

    // stage(it + 1) follows the tile-it gin stores in every iteration, the first included (its loads were issued
    // before them, in the prologue or the previous iteration), so the compiler's wait for the staged registers counts
    // the stores as younger and never waits for them; stage / issue also run past the last tile (zeros nothing
    // reads): a branch around them would make that wait a vmcnt(0)
    if (n_iter > 0) {
        issue(0);
        stage(0);
        issue(1);
    }
    for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(32);
    bb2::bar_lds();                                  // tile 0 staged
    for (int it = 0; it < n_iter; ++it) {
        if constexpr (!kIg) {
            if constexpr (!(kVariant & 2)) wgrad();
        } else if constexpr (DG) {
            t1 = 0.f;
            t2 = 0.f;
            ig_pass(it, I0{}, I5{});                 // output cells 0-4
            ig_pass(it, I5{}, I4{});                 // output cells 5-8
            if constexpr (EPI == 2) {
                s1 += (double)t1;
                s2 += (double)t2;
            }
        }
        bb2::bar_lds();                              // tile it's images read: the next stage may overwrite them
        stage(it + 1);
        issue(it + 2);
        bb2::bar_lds();                              // tile it+1 staged
    }
    // weight-gradient partials partial[block][tap][ci][co] (C/D layout of 32x32x16: col = co = lane & 31,
    // row = ci = (i&3) + 8(i>>2) + 4h); each tap has one owner wave
    if constexpr (!kIg) {
        constexpr int kW = kTaps * kC * kC;
        float *outp = a.wpart + (int64_t)blockIdx.x * kW;
        const int h = lane >> 5;
#pragma unroll
        for (int s = 0; s < kNt; ++s)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int ci = (i & 3) + 8 * (i >> 2) + 4 * h;
                outp[(Taps<W>::kT[s] * kC + ci) * kC + ch] = wacc[s][i];
            }
    }
    if constexpr (DG && EPI == 2) {   // the sums: waves 0-1 [wave][lane] -> channel wave*16 + (lane&15)
        double *dred = reinterpret_cast<double *>(smem);     // the loop's last barrier freed the images
        if (kIg) {
            dred[(W * 64 + lane) * 2 + 0] = s1;
            dred[(W * 64 + lane) * 2 + 1] = s2;
        }
        __syncthreads();
        if (W == 0) {
            const int c = lane >> 1, k = lane & 1, ct = c >> 4, l16 = c & 15;
            double tot = 0.0;
            for (int lg = 0; lg < 4; ++lg) tot += dred[(ct * 64 + lg * 16 + l16) * 2 + k];
            a.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = tot;
        }
    }
}

}  // namespace bb4

// ------------------------------------------------------------------ the chain's forward conv, LDS-DMA ring
// conv3x3_fwd_dma_kernel<PRO>: y = conv(x') with x' = relu(x*in_alpha + in_beta) (PRO) or x, and the output's BN
// statistics (sum y, sum y^2 per channel): every output block is the same split MFMA sequence as bb2's forward (EPI 1)
// on the same x' (bit-identical y); the statistics are fp32 per tile and wave, folded in fp64 in a fixed order.
// bb2 loaded each 16-row tile into registers one tile ahead (≈18 KB in flight per CU, one burst per tile) and gave
// four waves all the MFMAs and four waves only staging: the forward ran at 0.42 of HBM, and stamps of a first
// LDS-DMA form showed the staging waves beside the heaviest MFMA waves as the critical path.  Here
//  * every wave computes: wave W owns column tile W & 1 and the output cells {0,1,2} | {3,4} | {5,6} | {7,8} (W >> 1)
//    -- 14, 15, 10 and 10 (input cell, output cell) pairs, so each SIMD's two waves (w, w+4) carry 24-25 pairs,
//    and a row's cells leave as one store;
//  * x streams into a kSlots-deep LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction,
//    no VGPRs), issued by every wave as inline asm (hipcc would drain a visible LDS-DMA at every ds_read) with its
//    vmcnt counted by hand, kSlots-1 tiles ahead;
//  * every wave stages 1/8 of the next tile's x' part images (prologue + exact split, bb2's image layout and
//    diagonal write order) from the ring, then its MFMAs run on the current tile: one raw s_barrier per tile.
// Rows past the batch: their LDS-DMA is dropped by the descriptor's range check, so the ring holds stale rows
// there; every output row depends on its own input row only, its store is dropped and its statistics masked.
namespace fw3 {

// diagnostic variants (FW3_VARIANT; the product is 0): bit 1 = the y stores by lane 0 only (same instruction count,
// so the counted vmcnt waits stay right; ~no write traffic), bit 2 = no MFMAs
#ifndef FW3_VARIANT
#define FW3_VARIANT 0
#endif
constexpr int kVariant = FW3_VARIANT;

constexpr int kSlots = 5;                                   // raw-x ring depth
constexpr int kRawBytes = kTile * kRow * 4;                 // one tile of x (18,432 B, rows contiguous)
constexpr int kPieces = kRawBytes / 1024;                   // 18 LDS-DMA wave-instructions per tile
constexpr int kImg0 = 0;                                    // x' part images, buffers 0/1 (bb2's layout)
constexpr int kRaw0 = 2 * bb2::kImgBytes;                   // the ring
constexpr int kLdsBytes = kRaw0 + kSlots * kRawBytes;       // 147,456 B
static_assert(kLdsBytes <= 160 * 1024, "LDS");
static_assert(kRawBytes % 1024 == 0, "whole LDS-DMA pieces per tile");

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// one LDS-DMA piece (16 B per lane to M0 + 16 * lane); M0 saved and restored inside the statement
__device__ __forceinline__ void dma16(u32x4 desc, uint32_t voff, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(desc), "s"(lds_byte)
                 : "memory");
}

// wave_rsrc's buffer descriptor as four wave-uniform dwords (for the inline-asm buffer ops)
__device__ __forceinline__ u32x4 wave_desc(const void *base, uint32_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    u32x4 d;
    d.x = __builtin_amdgcn_readfirstlane((uint32_t)p);
    d.y = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32)) & 0xffffu;
    d.z = __builtin_amdgcn_readfirstlane(bytes);
    d.w = 0x00020000u;
    return d;
}

// the output cells of cell group G (W >> 1): runs of consecutive cells, so a row's cells leave in one store
// (14, 15, 10 and 10 (input, output) cell pairs: the SIMD pairs (w, w+4) carry 24 and 25)
template <int G> struct Cells;
template <> struct Cells<0> { static constexpr int kN = 3; static constexpr int kQ[3] = {0, 1, 2}; };
template <> struct Cells<1> { static constexpr int kN = 2; static constexpr int kQ[2] = {3, 4}; };
template <> struct Cells<2> { static constexpr int kN = 2; static constexpr int kQ[2] = {5, 6}; };
template <> struct Cells<3> { static constexpr int kN = 2; static constexpr int kQ[2] = {7, 8}; };

template <int G> __device__ constexpr bool g_uses_p(int p) {
    for (int s = 0; s < Cells<G>::kN; ++s)
        if (tap_of(p, Cells<G>::kQ[s]) >= 0) return true;
    return false;
}
template <int G> __device__ constexpr bool g_uses_tap(int t) {
    for (int s = 0; s < Cells<G>::kN; ++s)
        for (int p = 0; p < kCells; ++p)
            if (tap_of(p, Cells<G>::kQ[s]) == t) return true;
    return false;
}

template <int W> __device__ constexpr int pieces_of() {     // pieces p = W, W+8, W+16 < 18 of every tile
    int n = 0;
    for (int p = W; p < kPieces; p += 8) ++n;
    return n;
}

// the counted wait at the end of iteration it for the ring's tile it+2: the younger vector-memory operations of
// this wave are its later LDS-DMA groups (NP each) and output stores (NS per tile)
template <int NP, int NS>
__device__ __forceinline__ void wait_tile_after(int it) {
    static_assert((kSlots - 2) * (NP + NS) + NS <= 63, "vmcnt");
    // tile it+2 came with the prologue while it + 2 < kSlots: younger are the prologue's later groups and every
    // iteration's group and stores so far, (kSlots - 2) NP + (it + 1) NS; later it came with iteration
    // it + 2 - kSlots, and (kSlots - 2) (NP + NS) + NS are younger
    if (it == 0) vm_wait<(kSlots - 2) * NP + NS>();
    else if (it == 1) vm_wait<(kSlots - 2) * NP + 2 * NS>();
    else if (it == 2) vm_wait<(kSlots - 2) * NP + 3 * NS>();
    else vm_wait<(kSlots - 2) * (NP + NS) + NS>();
    static_assert(kSlots == 5, "the early-iteration counts above are written for kSlots = 5");
}

template <bool PRO, int W>
__device__ __forceinline__ void run(const BlockBwdArgs &a, unsigned char *smem, int lane) {
    constexpr int kCt = W & 1, G = W >> 1;
    using C = Cells<G>;
    constexpr int kNq = C::kN;
    constexpr int NP = pieces_of<W>();
    constexpr int NS = 4;                               // one store per row: the group's run of cells
    const int64_t ntiles = (a.M + kTile - 1) / kTile;
    const int64_t t0 = blockIdx.x;
    const int64_t step = gridDim.x;
    const int n_iter = t0 < ntiles ? (int)((ntiles - 1 - t0) / step + 1) : 0;
    const int ch = lane & 31, hh = lane >> 5;
    // the forward weights of the wave's taps: all three split parts in registers (bb2's fragment layout)
    uint4 wh[kTaps], wm[kTaps], wl[kTaps];
    {
        const int ci0 = 8 * (lane >> 4), j = lane & 15;
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            if (!g_uses_tap<G>(t)) continue;
            uint32_t hv[4], mv[4], lv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int tc = t * 2 + kCt;
                const float w0 = a.wpk[(tc * kC + ci0 + 2 * d) * 16 + j];
                const float w1 = a.wpk[(tc * kC + ci0 + 2 * d + 1) * 16 + j];
                uint32_t h0, m0, l0, h1, m1, l1;
                hrl_split::split3(w0, h0, m0, l0);
                hrl_split::split3(w1, h1, m1, l1);
                hv[d] = h0 | (h1 << 16);
                mv[d] = m0 | (m1 << 16);
                lv[d] = l0 | (l1 << 16);
            }
            wh[t] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            wm[t] = make_uint4(mv[0], mv[1], mv[2], mv[3]);
            wl[t] = make_uint4(lv[0], lv[1], lv[2], lv[3]);
        }
    }
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {
        if (!a.fold_part) {
            pa = a.in_alpha[ch];
            pb = a.in_beta[ch];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the weight and prologue loads, before any DMA is counted
    const uint32_t smem_base = (uint32_t)(uintptr_t)smem;
    auto dma = [&](int it, int slot) __attribute__((always_inline)) {
        const int64_t t = t0 + (int64_t)it * step;
        const bool ok = it < n_iter;
        const int rows = ok ? (int)min<int64_t>(kTile, a.M - t * kTile) : 0;
        const u32x4 desc = wave_desc(a.x + (ok ? t * kTile * kRow : 0), (uint32_t)rows * kRow * 4);
        const uint32_t raw = smem_base + kRaw0 + (uint32_t)slot * kRawBytes;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int p = W + 8 * j;
            dma16(desc, p * 1024 + lane * 16, raw + p * 1024);
        }
    };
    const int c0 = hh ? 4 : 0;
    const int rho0 = 2 * ((W + (ch >> 2)) & 7);              // bb2 staging wave W's row pair (its diagonal)
    auto stage = [&](int it, int slot) __attribute__((always_inline)) {
        const float *raw = reinterpret_cast<const float *>(smem + kRaw0 + slot * kRawBytes);
        unsigned char *xi = smem + kImg0 + (it & 1) * bb2::kImgBytes;
        uint32_t xp[3][5];
        float xv[2][5];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const float *src = raw + (rho0 + r) * kRow + ch * kCells + c0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                float v = src[i];
                if constexpr (PRO) {   // bn_apply_kernel's float operations
                    const float u = v * pa + pb;
                    v = u < 0.f ? 0.f : u;
                }
                xv[r][i] = v;
            }
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) hrl_split::split_pair(xv[0][i], xv[1][i], xp[0][i], xp[1][i], xp[2][i]);
        const int half = rho0 >> 3, sub = 2 * (rho0 & 7);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = bb2::img_off(c0 + i, ch, half) + sub;
#pragma unroll
            for (int part = 0; part < 3; ++part)
                *reinterpret_cast<uint32_t *>(xi + part * bb2::kPartBytes + o) = xp[part][i];
        }
    };
    const int co = kCt * 16 + (lane & 15);
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int tr_sub = 8 * (pp & 1);
    double s1 = 0.0, s2 = 0.0;
    // prologue: tiles 0 .. kSlots-1 in flight; tile 0 staged
#pragma unroll
    for (int j = 0; j < kSlots; ++j) dma(j, j);
    if constexpr (PRO) {
        // the input BN's finalize (bnfold) while the ring fills; its loads' wait also covers the DMAs issued
        // before them (the counted waits below then pass at once)
        if (a.fold_part) bnfold::fold(a, smem, pa, pb);
    }
    vm_wait<(kSlots - 1) * NP>();                            // tile 0 landed
    bb2::bar_lds();
    stage(0, 0);
    vm_wait<(kSlots - 2) * NP>();                            // tile 1 landed
    bb2::bar_lds();
    int slot = 0;                                            // ring slot of tile it (= it % kSlots)
    for (int it = 0; it < n_iter; ++it) {
        BB2_STAMP(it, 0);
        // tile it's slot was read by stage(it) before the last barrier: tile it + kSlots goes there
        dma(it + kSlots, slot);
        const int next = slot + 1 == kSlots ? 0 : slot + 1;
        stage(it + 1, next);                                 // runs past the last tile too (stale rows, unread)
        BB2_STAMP(it, 1);
        // the MFMAs of tile it: acc[s] += sum_p x'_p (16 rows x 32 ci) . W[tap(p, q_s)][kCt], p ascending
        const unsigned char *img = smem + kImg0 + (it & 1) * bb2::kImgBytes;
        f32x4 acc[kNq];
#pragma unroll
        for (int s = 0; s < kNq; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < kCells; ++p) {
            if (!g_uses_p<G>(p) || (kVariant & 2)) continue;
            uint32_t A[3][4];
#pragma unroll
            for (int part = 0; part < 3; ++part) {
#pragma unroll
                for (int hlf = 0; hlf < 2; ++hlf) {
                    const int o = part * bb2::kPartBytes + bb2::img_off(p, 8 * g + 4 * hlf + qq, pp >> 1) + tr_sub;
                    const bb2::v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (bb2::lds_v4s *)((__attribute__((address_space(3))) unsigned char *)(img + o)));
                    const uint2 u = __builtin_bit_cast(uint2, r);
                    A[part][2 * hlf] = u.x;
                    A[part][2 * hlf + 1] = u.y;
                }
            }
            const uint4 Ah = make_uint4(A[0][0], A[0][1], A[0][2], A[0][3]);
            const uint4 Am = make_uint4(A[1][0], A[1][1], A[1][2], A[1][3]);
            const uint4 Al = make_uint4(A[2][0], A[2][1], A[2][2], A[2][3]);
#pragma unroll
            for (int s = 0; s < kNq; ++s) {
                const int tap = tap_of(p, C::kQ[s]);
                if (tap < 0) continue;
                f32x4 c = acc[s];
                c = mfma_bf16(Al, wh[tap], c);   // smallest terms first (bb2's order)
                c = mfma_bf16(Am, wm[tap], c);
                c = mfma_bf16(Ah, wl[tap], c);
                c = mfma_bf16(Am, wh[tap], c);
                c = mfma_bf16(Ah, wm[tap], c);
                c = mfma_bf16(Ah, wh[tap], c);
                acc[s] = c;
            }
        }
        BB2_STAMP(it, 2);
        // epilogue: the output's BN statistics (fp32 per tile, fp64 across tiles), y straight from the accumulators
        const int64_t t = t0 + (int64_t)it * step;
        const int rows = (int)min<int64_t>(kTile, a.M - t * kTile);
        const __amdgpu_buffer_rsrc_t od = wave_rsrc(a.gin + t * kTile * kRow, (uint32_t)rows * kRow * 4);
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int s = 0; s < kNq; ++s) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = (lane >> 4) * 4 + rr;
                const float u = row < rows ? acc[s][rr] : 0.f;
                t1 += u;
                t2 += u * u;
            }
        }
        s1 += (double)t1;
        s2 += (double)t2;
        // compiler-visible stores: hipcc then keeps the MFMA -> store-data wait states (inline-asm stores read some
        // accumulators before their MFMA had written them); vmcnt is still counted by hand
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int row = (lane >> 4) * 4 + rr;
            const int off = (row * kRow + co * kCells + C::kQ[0]) * 4;
            if constexpr (kVariant & 1) {
                if (lane != 0) continue;
            }
            if constexpr (kNq == 3) {
                u32x3 v;
                v.x = __float_as_uint(acc[0][rr]);
                v.y = __float_as_uint(acc[1][rr]);
                v.z = __float_as_uint(acc[2 % kNq][rr]);
                __builtin_amdgcn_raw_buffer_store_b96(v, od, off, 0, 0);
            } else {
                u32x2 v;
                v.x = __float_as_uint(acc[0][rr]);
                v.y = __float_as_uint(acc[1][rr]);
                __builtin_amdgcn_raw_buffer_store_b64(v, od, off, 0, 0);
            }
        }
        wait_tile_after<NP, NS>(it);                         // tile it+2 landed (it+3 .. it+kSlots in flight)
        BB2_STAMP(it, 3);
        bb2::bar_lds();                                      // tile it+1's image staged, tile it's image free
        slot = next;
    }
    vm_wait<0>();
    // the sums: [wave][lane] -> channel (wave & 1) * 16 + (lane & 15), waves and lane groups in a fixed order
    __syncthreads();
    double *dred = reinterpret_cast<double *>(smem);
    dred[(W * 64 + lane) * 2 + 0] = s1;
    dred[(W * 64 + lane) * 2 + 1] = s2;
    __syncthreads();
    if (W == 0) {
        const int c = lane >> 1, k = lane & 1, ct = c >> 4, l16 = c & 15;
        double tot = 0.0;
        for (int w = ct; w < 8; w += 2)
            for (int lg = 0; lg < 4; ++lg) tot += dred[(w * 64 + lg * 16 + l16) * 2 + k];
        a.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = tot;
    }
}

}  // namespace fw3

// ------------------------------------------------------------------ the chain's forward conv, y staged in the ring
// conv3x3_fwd_ls_kernel<PRO> (fwd form 3): fw3's ring, staging and split MFMA sequence (bit-identical y and sums),
// with y leaving through LDS.  fw3 stores y straight from the accumulators: 8- and 12-byte runs 36 bytes apart per
// lane, which cost more than the ring's reads (a ping-pong form measured them: profiles/r06_fw4_pingpong.txt).  A
// tile of y is 18,432 contiguous bytes of HBM and exactly one ring slot, and tile it's slot is free once its x' is
// staged, so:
//  * iteration it: the MFMAs of tile it, then y(it) into ring slot it % kSlots as [row][288] fp32 (the HBM image);
//  * iteration it + 1, after the barrier: wave W reads back its LDS-DMA pieces p = W, W + 8, W + 16 of that slot,
//    stores them as 1 KiB contiguous buffer stores, then issues tile it + kSlots's LDS-DMA into the same pieces
//    (only this wave reads or writes them, so no barrier between);
//  * tile X's LDS-DMA is issued in iteration X - 4 (fw3: X - 5): one ring slot holds the drained tile.
namespace fw5 {

// diagnostic variants (FW5_VARIANT; the product is 0): bit 1 = the y stores by lane 0 only (same instruction
// count), bit 2 = y written to LDS with the row groups 16 banks apart (wrong y: the bank-conflict-free write cost)
#ifndef FW5_VARIANT
#define FW5_VARIANT 0
#endif
constexpr int kVariant = FW5_VARIANT;

constexpr int kSlots = fw3::kSlots;
constexpr int kRawBytes = fw3::kRawBytes;
constexpr int kImg0 = fw3::kImg0;
constexpr int kRaw0 = fw3::kRaw0;
constexpr int kLdsBytes = fw3::kLdsBytes;
static_assert(kSlots == 5 && kRawBytes == kTile * kRow * 4, "one ring slot = one tile of y");

template <bool PRO, int W>
__device__ __forceinline__ void run(const BlockBwdArgs &a, unsigned char *smem, int lane) {
    constexpr int kCt = W & 1, G = W >> 1;
    using C = fw3::Cells<G>;
    constexpr int kNq = C::kN;
    constexpr int NP = fw3::pieces_of<W>();
    const int64_t ntiles = (a.M + kTile - 1) / kTile;
    const int64_t t0 = blockIdx.x;
    const int64_t step = gridDim.x;
    const int n_iter = t0 < ntiles ? (int)((ntiles - 1 - t0) / step + 1) : 0;
    const int ch = lane & 31, hh = lane >> 5;
    uint4 wh[kTaps], wm[kTaps], wl[kTaps];
    {
        const int ci0 = 8 * (lane >> 4), j = lane & 15;
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            if (!fw3::g_uses_tap<G>(t)) continue;
            uint32_t hv[4], mv[4], lv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int tc = t * 2 + kCt;
                const float w0 = a.wpk[(tc * kC + ci0 + 2 * d) * 16 + j];
                const float w1 = a.wpk[(tc * kC + ci0 + 2 * d + 1) * 16 + j];
                uint32_t h0, m0, l0, h1, m1, l1;
                hrl_split::split3(w0, h0, m0, l0);
                hrl_split::split3(w1, h1, m1, l1);
                hv[d] = h0 | (h1 << 16);
                mv[d] = m0 | (m1 << 16);
                lv[d] = l0 | (l1 << 16);
            }
            wh[t] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            wm[t] = make_uint4(mv[0], mv[1], mv[2], mv[3]);
            wl[t] = make_uint4(lv[0], lv[1], lv[2], lv[3]);
        }
    }
    float pa = 1.f, pb = 0.f;
    if constexpr (PRO) {
        pa = a.in_alpha[ch];
        pb = a.in_beta[ch];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the weight and prologue loads, before any DMA is counted
    const uint32_t smem_base = (uint32_t)(uintptr_t)smem;
    auto rows_of = [&](int it) __attribute__((always_inline)) {
        const int64_t t = t0 + (int64_t)it * step;
        return it < n_iter ? (int)min<int64_t>(kTile, a.M - t * kTile) : 0;
    };
    auto dma = [&](int it) __attribute__((always_inline)) {   // tile it -> ring slot it % kSlots (this wave's pieces)
        const int64_t t = t0 + (int64_t)it * step;
        const int rows = rows_of(it);
        const u32x4 desc = fw3::wave_desc(a.x + (rows > 0 ? t * kTile * kRow : 0), (uint32_t)rows * kRow * 4);
        const uint32_t raw = smem_base + kRaw0 + (uint32_t)(it % kSlots) * kRawBytes;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int p = W + 8 * j;
            fw3::dma16(desc, p * 1024 + lane * 16, raw + p * 1024);
        }
    };
    const int c0 = hh ? 4 : 0;
    const int rho0 = 2 * ((W + (ch >> 2)) & 7);              // bb2 staging wave W's row pair (its diagonal)
    auto stage = [&](int it) __attribute__((always_inline)) {
        const float *raw = reinterpret_cast<const float *>(smem + kRaw0 + (it % kSlots) * kRawBytes);
        unsigned char *xi = smem + kImg0 + (it & 1) * bb2::kImgBytes;
        uint32_t xp[3][5];
        float xv[2][5];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const float *src = raw + (rho0 + r) * kRow + ch * kCells + c0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                float v = src[i];
                if constexpr (PRO) {   // bn_apply_kernel's float operations
                    const float u = v * pa + pb;
                    v = u < 0.f ? 0.f : u;
                }
                xv[r][i] = v;
            }
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) hrl_split::split_pair(xv[0][i], xv[1][i], xp[0][i], xp[1][i], xp[2][i]);
        const int half = rho0 >> 3, sub = 2 * (rho0 & 7);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = bb2::img_off(c0 + i, ch, half) + sub;
#pragma unroll
            for (int part = 0; part < 3; ++part)
                *reinterpret_cast<uint32_t *>(xi + part * bb2::kPartBytes + o) = xp[part][i];
        }
    };
    // tile it's y: this wave's pieces of its ring slot -> HBM (1 KiB contiguous per store), then tile it + kSlots's
    // LDS-DMA into the same pieces (the stores have consumed the reads)
    auto drain = [&](int it, bool refill) __attribute__((always_inline)) {
        const int64_t t = t0 + (int64_t)it * step;
        const int rows = rows_of(it);
        const __amdgpu_buffer_rsrc_t od = wave_rsrc(a.gin + (rows > 0 ? t * kTile * kRow : 0), (uint32_t)rows * kRow * 4);
        const unsigned char *raw = smem + kRaw0 + (it % kSlots) * kRawBytes;
        u32x4 v[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) v[j] = *reinterpret_cast<const u32x4 *>(raw + (W + 8 * j) * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if constexpr (kVariant & 1) {
                if (lane != 0) continue;
            }
            __builtin_amdgcn_raw_buffer_store_b128(v[j], od, (W + 8 * j) * 1024 + lane * 16, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the pieces are read before the DMA rewrites them
        if (refill) dma(it + kSlots);
    };
    const int co = kCt * 16 + (lane & 15);
    const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int tr_sub = 8 * (pp & 1);
    double s1 = 0.0, s2 = 0.0;
    // prologue: tiles 0 .. kSlots-2 in flight; tile 0 staged
#pragma unroll
    for (int j = 0; j < kSlots - 1; ++j) dma(j);
    fw3::vm_wait<(kSlots - 2) * NP>();                       // tile 0 landed
    bb2::bar_lds();
    stage(0);
    fw3::vm_wait<(kSlots - 3) * NP>();                       // tile 1 landed
    bb2::bar_lds();
    for (int it = 0; it < n_iter; ++it) {
        BB2_STAMP(it, 0);
        if (it == 0) dma(kSlots - 1);                        // ring slot kSlots-1 is still empty
        else drain(it - 1, true);                            // y(it-1) out, tile it-1+kSlots in
        stage(it + 1);                                       // runs past the last tile too (stale rows, unread)
        BB2_STAMP(it, 1);
        const unsigned char *img = smem + kImg0 + (it & 1) * bb2::kImgBytes;
        f32x4 acc[kNq];
#pragma unroll
        for (int s = 0; s < kNq; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < kCells; ++p) {
            if (!fw3::g_uses_p<G>(p)) continue;
            uint32_t A[3][4];
#pragma unroll
            for (int part = 0; part < 3; ++part) {
#pragma unroll
                for (int hlf = 0; hlf < 2; ++hlf) {
                    const int o = part * bb2::kPartBytes + bb2::img_off(p, 8 * g + 4 * hlf + qq, pp >> 1) + tr_sub;
                    const bb2::v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (bb2::lds_v4s *)((__attribute__((address_space(3))) unsigned char *)(img + o)));
                    const uint2 u = __builtin_bit_cast(uint2, r);
                    A[part][2 * hlf] = u.x;
                    A[part][2 * hlf + 1] = u.y;
                }
            }
            const uint4 Ah = make_uint4(A[0][0], A[0][1], A[0][2], A[0][3]);
            const uint4 Am = make_uint4(A[1][0], A[1][1], A[1][2], A[1][3]);
            const uint4 Al = make_uint4(A[2][0], A[2][1], A[2][2], A[2][3]);
#pragma unroll
            for (int s = 0; s < kNq; ++s) {
                const int tap = tap_of(p, C::kQ[s]);
                if (tap < 0) continue;
                f32x4 c = acc[s];
                c = mfma_bf16(Al, wh[tap], c);   // smallest terms first (bb2's order)
                c = mfma_bf16(Am, wm[tap], c);
                c = mfma_bf16(Ah, wl[tap], c);
                c = mfma_bf16(Am, wh[tap], c);
                c = mfma_bf16(Ah, wm[tap], c);
                c = mfma_bf16(Ah, wh[tap], c);
                acc[s] = c;
            }
        }
        BB2_STAMP(it, 2);
        // the output's BN statistics (fp32 per tile, fp64 across tiles), then y into tile it's ring slot
        const int rows = rows_of(it);
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int s = 0; s < kNq; ++s) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = g * 4 + rr;
                const float u = row < rows ? acc[s][rr] : 0.f;
                t1 += u;
                t2 += u * u;
            }
        }
        s1 += (double)t1;
        s2 += (double)t2;
        {
            float *yo = reinterpret_cast<float *>(smem + kRaw0 + (it % kSlots) * kRawBytes);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                for (int s = 0; s < kNq; ++s) {
                    int o = (g * 4 + rr) * kRow + co * kCells + C::kQ[s];
                    if constexpr (kVariant & 2) o = (o + 16 * g) % (kTile * kRow);
                    yo[o] = acc[s][rr];
                }
        }
        // tile it+2 landed: younger are this wave's later LDS-DMA pieces and y stores (tile X's DMA is issued in
        // iteration X-4, after that iteration's stores; the prologue issued tiles 0..3, iteration 0 tile 4)
        if (it == 0) fw3::vm_wait<2 * NP>();
        else if (it == 1) fw3::vm_wait<3 * NP>();
        else fw3::vm_wait<4 * NP>();
        BB2_STAMP(it, 3);
        bb2::bar_lds();                                      // y(it) and tile it+1's image staged
    }
    if (n_iter > 0) drain(n_iter - 1, false);
    fw3::vm_wait<0>();
    // the sums: [wave][lane] -> channel (wave & 1) * 16 + (lane & 15), waves and lane groups in a fixed order
    __syncthreads();
    double *dred = reinterpret_cast<double *>(smem);
    dred[(W * 64 + lane) * 2 + 0] = s1;
    dred[(W * 64 + lane) * 2 + 1] = s2;
    __syncthreads();
    if (W == 0) {
        const int c = lane >> 1, k = lane & 1, ct = c >> 4, l16 = c & 15;
        double tot = 0.0;
        for (int w = ct; w < 8; w += 2)
            for (int lg = 0; lg < 4; ++lg) tot += dred[(w * 64 + lg * 16 + l16) * 2 + k];
        a.part[((int64_t)blockIdx.x * kC + c) * 2 + k] = tot;
    }
}

}  // namespace fw5


template <bool PRO>
__global__ __launch_bounds__(bb2::kThreads) void conv3x3_fwd_dma_kernel(BlockBwdArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[fw3::kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (wave) {
    case 0: fw3::run<PRO, 0>(a, smem, lane); break;
    case 1: fw3::run<PRO, 1>(a, smem, lane); break;
    case 2: fw3::run<PRO, 2>(a, smem, lane); break;
    case 3: fw3::run<PRO, 3>(a, smem, lane); break;
    case 4: fw3::run<PRO, 4>(a, smem, lane); break;
    case 5: fw3::run<PRO, 5>(a, smem, lane); break;
    case 6: fw3::run<PRO, 6>(a, smem, lane); break;
    default: fw3::run<PRO, 7>(a, smem, lane); break;
    }
}

template <bool PRO>
__global__ __launch_bounds__(bb2::kThreads) void conv3x3_fwd_ls_kernel(BlockBwdArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[fw5::kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (wave) {
    case 0: fw5::run<PRO, 0>(a, smem, lane); break;
    case 1: fw5::run<PRO, 1>(a, smem, lane); break;
    case 2: fw5::run<PRO, 2>(a, smem, lane); break;
    case 3: fw5::run<PRO, 3>(a, smem, lane); break;
    case 4: fw5::run<PRO, 4>(a, smem, lane); break;
    case 5: fw5::run<PRO, 5>(a, smem, lane); break;
    case 6: fw5::run<PRO, 6>(a, smem, lane); break;
    default: fw5::run<PRO, 7>(a, smem, lane); break;
    }
}

template <bool PRO, int EPI>
__global__ __launch_bounds__(bb2::kThreads) void conv3x3_block_bwd2_kernel(BlockBwdArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[bb2::kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (wave) {
    case 0: bb2::run<PRO, EPI, 0>(a, smem, lane); break;
    case 1: bb2::run<PRO, EPI, 1>(a, smem, lane); break;
    case 2: bb2::run<PRO, EPI, 2>(a, smem, lane); break;
    case 3: bb2::run<PRO, EPI, 3>(a, smem, lane); break;
    case 4: bb2::run<PRO, EPI, 4>(a, smem, lane); break;
    case 5: bb2::run<PRO, EPI, 5>(a, smem, lane); break;
    case 6: bb2::run<PRO, EPI, 6>(a, smem, lane); break;
    default: bb2::run<PRO, EPI, 7>(a, smem, lane); break;
    }
}

// two 4-wave workgroups per CU: at most 256 registers per lane (two waves per SIMD), 72.3 KB of LDS each
template <bool PRO, int EPI, bool DG>
__global__ __launch_bounds__(bb4::kThreads, 2) void conv3x3_block_bwd4_kernel(BlockBwdArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[bb4::kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the two workgroups of a CU run the same program with a barrier per phase and fall into lockstep (both
    // staging, then both issuing MFMAs; MI355X_MICROARCH.md "Two waves per SIMD" item 9): the later arrival on its
    // CU (a per-CU ticket: HW_ID's CU/SH/SE fields and XCC_ID) starts `stagger` s_sleep(32)s behind
    int delay = 0;
    if (a.stagger > 0) {
        if (threadIdx.x == 0) {      // one lane: a vector atomic
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            const unsigned key = ((xcc & 7u) << 8) | ((hw >> 8) & 0xffu);
            *reinterpret_cast<volatile unsigned *>(smem) = atomicAdd(a.tickets + key, 1u) & 1u;
        }
        __syncthreads();
        delay = *reinterpret_cast<volatile unsigned *>(smem) ? a.stagger : 0;
        delay = __builtin_amdgcn_readfirstlane(delay);
        __syncthreads();
    }
#ifdef BB4_ONLY_W
    bb4::run<PRO, EPI, DG, BB4_ONLY_W>(a, smem, lane, delay);
#else
    switch (wave) {
    case 0: bb4::run<PRO, EPI, DG, 0>(a, smem, lane, delay); break;
    case 1: bb4::run<PRO, EPI, DG, 1>(a, smem, lane, delay); break;
    case 2: bb4::run<PRO, EPI, DG, 2>(a, smem, lane, delay); break;
    default: bb4::run<PRO, EPI, DG, 3>(a, smem, lane, delay); break;
    }
#endif
}

// fold per-workgroup partials into dW[co][ci][3][3]: a workgroup owns 64 consecutive
// outputs; its 4 waves take every 4th partial (4 independent sums in flight per
// thread) and combine in a fixed order -> deterministic.
__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce_kernel(const float *__restrict__ partial, int nparts,
                                                                   float *__restrict__ dw) {
    __shared__ float red[4][64];
    constexpr int kW = kTaps * kC * kC;
    const int col = threadIdx.x & 63, sub = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + col;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int w = sub;
    for (; w + 12 < nparts; w += 16) {
        s0 += partial[(int64_t)w * kW + i];
        s1 += partial[(int64_t)(w + 4) * kW + i];
        s2 += partial[(int64_t)(w + 8) * kW + i];
        s3 += partial[(int64_t)(w + 12) * kW + i];
    }
    for (; w < nparts; w += 4) s0 += partial[(int64_t)w * kW + i];
    red[sub][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (sub == 0) {
        const float s = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
        const int co = i % kC, ci = (i / kC) % kC, tap = i / (kC * kC);
        dw[(co * kC + ci) * kTaps + tap] = s;
    }
}

// W[co][ci][tap] -> packed [tap][ct][ci'][16] for the conv kernel.
// flip = 0: forward (ci' = ci, output co);  flip = 1: input gradient (ci' = co, output ci, tap mirrored)
__global__ void conv3x3_pack_kernel(const float *__restrict__ w, int flip, float *__restrict__ wpk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // packed index
    if (i >= kTaps * 2 * kC * 16) return;
    const int j = i % 16, k = (i / 16) % kC, ct = (i / (16 * kC)) % 2, tap = i / (16 * kC * 2);
    const int out_c = ct * 16 + j;   // output channel of this conv
    const int in_c = k;              // input channel of this conv (the MFMA k)
    float v;
    if (!flip) v = w[(out_c * kC + in_c) * kTaps + tap];
    else v = w[(in_c * kC + out_c) * kTaps + (kTaps - 1 - tap)];
    wpk[i] = v;
}

// Both layouts of up to 8 weights in one launch: packed[(l*2 + flip) * kPack + i] (hrl_conv3x3_pack_n)
constexpr int kPack = kTaps * 2 * kC * 16;
struct WeightList {
    const float *w[8];
};
__global__ void conv3x3_pack_n_kernel(WeightList wl, int n, float *__restrict__ packed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * 2 * kPack) return;
    const int l = i / (2 * kPack), flip = (i / kPack) & 1, e = i % kPack;
    const int j = e % 16, k = (e / 16) % kC, ct = (e / (16 * kC)) % 2, tap = e / (16 * kC * 2);
    const int out_c = ct * 16 + j, in_c = k;
    const float *w = wl.w[l];
    packed[i] = !flip ? w[(out_c * kC + in_c) * kTaps + tap] : w[(in_c * kC + out_c) * kTaps + (kTaps - 1 - tap)];
}

// Forward / input-gradient arithmetic: exact-split bf16 MFMA (1, default) or fp32 MFMA (0).
int g_split = 1;
// Chain block backward: 1 = the 8-wave tile-shared conv3x3_block_bwd2_kernel (default); 2 = two 4-wave workgroups
// per CU, conv3x3_block_bwd4_kernel (round 6: bit-identical, slower -- DESIGN §4.3); 0 = the per-wave
// conv3x3_block_bwd_kernel (the tests' reference form).  Forms 0 and 1 run the per-wave kernel when there is no
// input gradient.
int g_block_form = 1;
// block form 2: the later-arriving workgroup of each CU starts this many s_sleep(32) behind (0: no stagger);
// HRL_BB4_STAGGER overrides (tools)
int g_bb4_stagger = [] {
    const char *e = getenv("HRL_BB4_STAGGER");
    return e ? atoi(e) : 0;
}();
// The chain's forward conv (epilogue 1, packed weights, no bias): 3 = the ring form with y staged through LDS (fw5),
// 2 = the LDS-DMA ring form (fw3, default), 1 = the tile-shared form (bb2, EPI 1), 0 = conv3x3_kernel<PRO, 1>.
int g_fwd_form = 2;

// One 4-wave workgroup per CU (LDS: 109 KB forward, 145 KB weight gradient);
// the waves walk row tiles grid-stride so the next tile's loads overlap MFMAs.
constexpr int kGrid = 256;

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int grid_for(int64_t M) {
    const int64_t tiles = (M + kTile - 1) / kTile;
    const int64_t blocks = (tiles + kWaves - 1) / kWaves;
    return (int)(blocks < kGrid ? blocks : kGrid);
}

// block form 2: one 16-row tile per workgroup and iteration, two workgroups per CU
int grid4_for(int64_t M) {
    const int64_t tiles = (M + kTile - 1) / kTile;
    return (int)(tiles < bb4::kGrid ? tiles : bb4::kGrid);
}

// workgroups (= weight-gradient partial rows and epilogue-2 sum rows) of hrl_conv3x3_block_backward
int block_grid_for(int64_t M) { return g_block_form == 2 ? grid4_for(M) : grid_for(M); }

}  // namespace

extern "C" {

#ifdef HRL_STAMPS
int hrl_debug_set_stamps_conv(void *buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hrl_stamps), &buf, sizeof(buf)); }
#endif

constexpr int64_t kTicketBytes = 2048 * 4;   // block form 2's per-CU tickets (any contents: only parity is used)

int64_t hrl_conv3x3_workspace_bytes(int64_t M) {
    if (M < 1) return -1;
    const int64_t rows = grid4_for(M) > grid_for(M) ? grid4_for(M) : grid_for(M);   // every block form's partials
    return rows * kTaps * kC * kC * 4 + (int64_t)kTaps * 2 * kC * 16 * 4 * 2 + kTicketBytes;
}

int64_t hrl_conv3x3_stats_blocks(int64_t M) { return M < 1 ? -1 : grid_for(M); }

int64_t hrl_conv3x3_block_sum_blocks(int64_t M) { return M < 1 ? -1 : block_grid_for(M); }

int hrl_conv3x3_set_block_form(int form) {
    const int prev = g_block_form;
    g_block_form = form < 0 ? 0 : (form > 2 ? 2 : form);
    return prev;
}

int hrl_conv3x3_set_fwd_form(int form) {
    const int prev = g_fwd_form;
    g_fwd_form = form < 0 ? 0 : (form > 3 ? 3 : form);
    return prev;
}

int hrl_conv3x3_set_split(int on) {
    const int prev = g_split;
    g_split = on ? 1 : 0;
    return prev;
}

int hrl_conv3x3_forward_ex(const float *x, int64_t M, const float *in_alpha, const float *in_beta,
                           const float *weight, const float *bias, int flip, float *y, int epilogue,
                           const float *ref, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                           double *part, void *workspace, int64_t workspace_bytes, void *stream) {
    if (M < 1 || !x || !weight || !y || !workspace) return HRL_EINVAL;
    if (!aligned16(x) || !aligned16(y) || workspace_bytes < hrl_conv3x3_workspace_bytes(M)) return HRL_EINVAL;
    if ((in_alpha == nullptr) != (in_beta == nullptr)) return HRL_EINVAL;
    if (epilogue < 0 || epilogue > 3) return HRL_EINVAL;
    if ((epilogue == 1 || epilogue == 2) && !part) return HRL_EINVAL;
    if ((epilogue == 2 || epilogue == 3) && (!ref || !aligned16(ref))) return HRL_EINVAL;
    if (epilogue == 2 && (!ep_mean || !ep_alpha || !ep_beta)) return HRL_EINVAL;
    if (epilogue >= 2 && bias) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const float *wpk = weight;   // flip & 2: `weight` is already in the packed layout (hrl_conv3x3_pack_n)
    if (!(flip & 2)) {
        float *dst = static_cast<float *>(workspace);
        hipLaunchKernelGGL(conv3x3_pack_kernel, dim3((kPack + 255) / 256), dim3(256), 0, s, weight, flip & 1, dst);
        const int rc = status();
        if (rc) return rc;
        wpk = dst;
    }
    if (epilogue == 1 && (flip & 2) && !bias && g_split && g_fwd_form >= 1 && M * kRow * 4 <= 0xffffffffLL) {
        // the chain's forward: 2 = the LDS-DMA ring form (fw3), 1 = the block backward's tile-shared form (bb2, EPI 1)
        BlockBwdArgs a{};
        a.x = x; a.in_alpha = in_alpha; a.in_beta = in_beta; a.wpk = wpk; a.gin = y; a.part = part; a.M = M;
        const dim3 grid(grid_for(M)), block(bb2::kThreads);
        if (g_fwd_form == 3) {
            if (in_alpha) hipLaunchKernelGGL((conv3x3_fwd_ls_kernel<true>), grid, block, 0, s, a);
            else hipLaunchKernelGGL((conv3x3_fwd_ls_kernel<false>), grid, block, 0, s, a);
        } else if (g_fwd_form == 2) {
            if (in_alpha) hipLaunchKernelGGL((conv3x3_fwd_dma_kernel<true>), grid, block, 0, s, a);
            else hipLaunchKernelGGL((conv3x3_fwd_dma_kernel<false>), grid, block, 0, s, a);
        } else if (in_alpha) {
            hipLaunchKernelGGL((conv3x3_block_bwd2_kernel<true, 1>), grid, block, 0, s, a);
        } else {
            hipLaunchKernelGGL((conv3x3_block_bwd2_kernel<false, 1>), grid, block, 0, s, a);
        }
        return status();
    }
    const dim3 grid(grid_for(M)), block(kThreads);
#define HRL_CONV_LAUNCH(PRO, EPI)                                                                             \
    do {                                                                                                      \
        if (g_split)                                                                                          \
            hipLaunchKernelGGL((conv3x3_kernel<PRO, EPI, true>), grid, block, 0, s, x, M, wpk, bias, in_alpha, \
                               in_beta, ref, ep_mean, ep_alpha, ep_beta, y, part);                            \
        else                                                                                                  \
            hipLaunchKernelGGL((conv3x3_kernel<PRO, EPI, false>), grid, block, 0, s, x, M, wpk, bias, in_alpha, \
                               in_beta, ref, ep_mean, ep_alpha, ep_beta, y, part);                            \
    } while (0)
    const bool pro = in_alpha != nullptr;
    switch (epilogue) {
    case 0: if (pro) HRL_CONV_LAUNCH(true, 0); else HRL_CONV_LAUNCH(false, 0); break;
    case 1: if (pro) HRL_CONV_LAUNCH(true, 1); else HRL_CONV_LAUNCH(false, 1); break;
    case 2: if (pro) HRL_CONV_LAUNCH(true, 2); else HRL_CONV_LAUNCH(false, 2); break;
    default: if (pro) HRL_CONV_LAUNCH(true, 3); else HRL_CONV_LAUNCH(false, 3); break;
    }
#undef HRL_CONV_LAUNCH
    return status();
}

int hrl_conv3x3_pack_n(const float *const *weights, int n, float *packed, void *stream) {
    if (n < 1 || n > 8 || !weights || !packed) return HRL_EINVAL;
    WeightList wl{};
    for (int i = 0; i < n; ++i) {
        if (!weights[i]) return HRL_EINVAL;
        wl.w[i] = weights[i];
    }
    hipLaunchKernelGGL(conv3x3_pack_n_kernel, dim3((n * 2 * kPack + 255) / 256), dim3(256), 0,
                       static_cast<hipStream_t>(stream), wl, n, packed);
    return status();
}

int hrl_conv3x3_forward(const float *x, int64_t M, int64_t C_in, int64_t C_out, const float *weight,
                        const float *bias, int flip, float *y, void *workspace, int64_t workspace_bytes,
                        void *stream) {
    if (C_in != kC || C_out != kC) return HRL_EINVAL;
    return hrl_conv3x3_forward_ex(x, M, nullptr, nullptr, weight, bias, flip, y, 0, nullptr, nullptr, nullptr,
                                  nullptr, nullptr, workspace, workspace_bytes, stream);
}

int hrl_conv3x3_wgrad_ex(const float *x, const float *in_alpha, const float *in_beta, const float *dy, int64_t M,
                         float *dweight, void *workspace, int64_t workspace_bytes, void *stream) {
    if (M < 1 || !x || !dy || !dweight || !workspace) return HRL_EINVAL;
    if ((in_alpha == nullptr) != (in_beta == nullptr)) return HRL_EINVAL;
    if (!aligned16(x) || !aligned16(dy) || workspace_bytes < hrl_conv3x3_workspace_bytes(M)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = grid_for(M);
    float *partial = static_cast<float *>(workspace) + kTaps * 2 * kC * 16 * 2;
    if (g_split) {
        if (in_alpha)
            hipLaunchKernelGGL((conv3x3_wgrad_split_kernel<true>), dim3(grid), dim3(kThreads), 0, s, x, in_alpha,
                               in_beta, dy, M, partial);
        else
            hipLaunchKernelGGL((conv3x3_wgrad_split_kernel<false>), dim3(grid), dim3(kThreads), 0, s, x, in_alpha,
                               in_beta, dy, M, partial);
    } else if (in_alpha) {
        hipLaunchKernelGGL((conv3x3_wgrad_kernel<true>), dim3(grid), dim3(kThreads), 0, s, x, in_alpha, in_beta, dy,
                           M, partial);
    } else {
        hipLaunchKernelGGL((conv3x3_wgrad_kernel<false>), dim3(grid), dim3(kThreads), 0, s, x, in_alpha, in_beta,
                           dy, M, partial);
    }
    int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3(kTaps * kC * kC / 64), dim3(256), 0, s, partial, grid,
                       dweight);
    return status();
}

int hrl_conv3x3_block_backward(const float *g, const float *y, int64_t M, const float *bn_weight,
                               const float *bn_bias, const float *save_mean, const float *save_invstd,
                               const float *kcoef, const float *gmean, const float *x, const float *in_alpha,
                               const float *in_beta, const float *packed_flip, float *dweight, float *gin,
                               int epilogue, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                               double *part, void *workspace, int64_t workspace_bytes, void *stream) {
    if (M < 1 || !g || !y || !save_mean || !save_invstd || !kcoef || !gmean || !x || !workspace)
        return HRL_EINVAL;
    if ((in_alpha == nullptr) != (in_beta == nullptr)) return HRL_EINVAL;
    if (workspace_bytes < hrl_conv3x3_workspace_bytes(M) || M * kRow * 4 > 0xffffffffLL) return HRL_EINVAL;
    if (gin && (!packed_flip || epilogue < 0 || epilogue == 1 || epilogue > 3)) return HRL_EINVAL;
    if (gin && epilogue == 2 && (!ep_mean || !ep_alpha || !ep_beta || !part)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = block_grid_for(M);
    float *wpart = static_cast<float *>(workspace) + kTaps * 2 * kC * 16 * 2;
    BlockBwdArgs a{g, y, bn_weight, bn_bias, save_mean, save_invstd, kcoef, gmean, x, in_alpha, in_beta, packed_flip,
                   ep_mean, ep_alpha, ep_beta, gin, part, wpart, M};
    a.tickets = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + workspace_bytes - kTicketBytes);
    a.stagger = g_bb4_stagger;
    const bool pro = in_alpha != nullptr;
#define HRL_BLOCK_LAUNCH(PRO, EPI, DG) \
    hipLaunchKernelGGL((conv3x3_block_bwd_kernel<PRO, EPI, DG>), dim3(grid), dim3(kThreads), 0, s, a)
#define HRL_BLOCK2_LAUNCH(PRO, EPI) \
    hipLaunchKernelGGL((conv3x3_block_bwd2_kernel<PRO, EPI>), dim3(grid), dim3(bb2::kThreads), 0, s, a)
#define HRL_BLOCK4_LAUNCH(PRO, EPI, DG) \
    hipLaunchKernelGGL((conv3x3_block_bwd4_kernel<PRO, EPI, DG>), dim3(grid), dim3(bb4::kThreads), 0, s, a)
    if (g_block_form == 2) {
        if (!gin) {
            if (pro) HRL_BLOCK4_LAUNCH(true, 0, false); else HRL_BLOCK4_LAUNCH(false, 0, false);
        } else if (epilogue == 2) {
            if (pro) HRL_BLOCK4_LAUNCH(true, 2, true); else HRL_BLOCK4_LAUNCH(false, 2, true);
        } else if (epilogue == 3) {
            if (pro) HRL_BLOCK4_LAUNCH(true, 3, true); else HRL_BLOCK4_LAUNCH(false, 3, true);
        } else {
            if (pro) HRL_BLOCK4_LAUNCH(true, 0, true); else HRL_BLOCK4_LAUNCH(false, 0, true);
        }
    } else if (!gin) {
        if (pro) HRL_BLOCK_LAUNCH(true, 0, false); else HRL_BLOCK_LAUNCH(false, 0, false);
    } else if (g_block_form == 0) {   // the per-wave form (kept for comparison)
        if (epilogue == 2) {
            if (pro) HRL_BLOCK_LAUNCH(true, 2, true); else HRL_BLOCK_LAUNCH(false, 2, true);
        } else if (epilogue == 3) {
            if (pro) HRL_BLOCK_LAUNCH(true, 3, true); else HRL_BLOCK_LAUNCH(false, 3, true);
        } else {
            if (pro) HRL_BLOCK_LAUNCH(true, 0, true); else HRL_BLOCK_LAUNCH(false, 0, true);
        }
    } else if (epilogue == 2) {
        if (pro) HRL_BLOCK2_LAUNCH(true, 2); else HRL_BLOCK2_LAUNCH(false, 2);
    } else if (epilogue == 3) {
        if (pro) HRL_BLOCK2_LAUNCH(true, 3); else HRL_BLOCK2_LAUNCH(false, 3);
    } else {
        if (pro) HRL_BLOCK2_LAUNCH(true, 0); else HRL_BLOCK2_LAUNCH(false, 0);
    }
#undef HRL_BLOCK_LAUNCH
#undef HRL_BLOCK2_LAUNCH
#undef HRL_BLOCK4_LAUNCH
    int rc = status();
    if (rc || !dweight) return rc;   // no dweight: the partials stay for a later fold (hrl_grad_fold_norm)
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3(kTaps * kC * kC / 64), dim3(256), 0, s, wpart, grid,
                       dweight);
    return status();
}

int hrl_conv3x3_forward_bnfold(const float *x, int64_t M, const double *prev_part, int64_t prev_nblocks,
                               const float *gamma, const float *beta, float *running_mean, float *running_var,
                               double momentum, double eps, float *save_mean, float *save_invstd, float *alpha,
                               float *beta_out, const float *packed, float *y, double *part, void *workspace,
                               int64_t workspace_bytes, void *stream) {
    if (M < 1 || !x || !prev_part || prev_nblocks < 1 || !save_mean || !save_invstd || !alpha || !beta_out ||
        !packed || !y || !part || !workspace)
        return HRL_EINVAL;
    if (!aligned16(x) || !aligned16(y) || workspace_bytes < hrl_conv3x3_workspace_bytes(M)) return HRL_EINVAL;
    if (prev_part == part) return HRL_EINVAL;   // the prologue reads every row the epilogue rewrites
    if (g_fwd_form != 2 || !g_split || prev_nblocks > 512 || M * kRow * 4 > 0xffffffffLL) {
        // the other forms: the two launches
        const int rc = hrl_bn_finalize_stats(prev_part, prev_nblocks, kC, M * kCells, gamma, beta, running_mean,
                                             running_var, momentum, eps, save_mean, save_invstd, alpha, beta_out,
                                             stream);
        if (rc) return rc;
        return hrl_conv3x3_forward_ex(x, M, alpha, beta_out, packed, nullptr, 2, y, 1, nullptr, nullptr, nullptr,
                                      nullptr, part, workspace, workspace_bytes, stream);
    }
    BlockBwdArgs a{};
    a.x = x; a.wpk = packed; a.gin = y; a.part = part; a.M = M;
    a.fold_part = prev_part; a.fold_nblocks = (int)prev_nblocks; a.fold_mode = 0;
    a.fold_count = (double)(M * kCells); a.fold_eps = eps; a.fold_momentum = (float)momentum;
    a.fold_w = gamma; a.fold_b = beta; a.fold_rm = running_mean; a.fold_rv = running_var;
    a.fold_o0 = save_mean; a.fold_o1 = save_invstd; a.fold_o2 = alpha; a.fold_o3 = beta_out;
    hipLaunchKernelGGL((conv3x3_fwd_dma_kernel<true>), dim3(grid_for(M)), dim3(bb2::kThreads), 0,
                       static_cast<hipStream_t>(stream), a);
    return status();
}

int hrl_conv3x3_block_backward_bnfold(const float *g, const float *y, int64_t M, const float *bn_weight,
                                      const float *bn_bias, const float *save_mean, const float *save_invstd,
                                      const double *sums, int64_t sums_nblocks, float *dgamma, float *dbeta,
                                      float *kcoef, float *gmean, const float *x, const float *in_alpha,
                                      const float *in_beta, const float *packed_flip, float *dweight, float *gin,
                                      int epilogue, const float *ep_mean, const float *ep_alpha, const float *ep_beta,
                                      double *part, void *workspace, int64_t workspace_bytes, void *stream) {
    if (!sums || sums_nblocks < 1 || !save_invstd || !kcoef || !gmean) return HRL_EINVAL;
    if (part && sums == part) return HRL_EINVAL;   // the prologue reads every row the epilogue rewrites
    const bool fused = g_block_form == 1 && gin && sums_nblocks <= 512;
    if (!fused) {   // the other forms: the two launches
        const int rc = hrl_bn_finalize_backward(sums, sums_nblocks, kC, M * kCells, bn_weight, save_invstd, dgamma,
                                                dbeta, kcoef, gmean, stream);
        if (rc) return rc;
        return hrl_conv3x3_block_backward(g, y, M, bn_weight, bn_bias, save_mean, save_invstd, kcoef, gmean, x,
                                          in_alpha, in_beta, packed_flip, dweight, gin, epilogue, ep_mean, ep_alpha,
                                          ep_beta, part, workspace, workspace_bytes, stream);
    }
    if (M < 1 || !g || !y || !save_mean || !x || !workspace) return HRL_EINVAL;
    if ((in_alpha == nullptr) != (in_beta == nullptr)) return HRL_EINVAL;
    if (workspace_bytes < hrl_conv3x3_workspace_bytes(M) || M * kRow * 4 > 0xffffffffLL) return HRL_EINVAL;
    if (!packed_flip || epilogue < 0 || epilogue == 1 || epilogue > 3) return HRL_EINVAL;
    if (epilogue == 2 && (!ep_mean || !ep_alpha || !ep_beta || !part)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = block_grid_for(M);
    float *wpart = static_cast<float *>(workspace) + kTaps * 2 * kC * 16 * 2;
    BlockBwdArgs a{g, y, bn_weight, bn_bias, save_mean, save_invstd, kcoef, gmean, x, in_alpha, in_beta, packed_flip,
                   ep_mean, ep_alpha, ep_beta, gin, part, wpart, M};
    a.fold_part = sums; a.fold_nblocks = (int)sums_nblocks; a.fold_mode = 1; a.fold_count = (double)(M * kCells);
    a.fold_o0 = dgamma; a.fold_o1 = dbeta; a.fold_o2 = kcoef; a.fold_o3 = gmean;
    const bool pro = in_alpha != nullptr;
#define HRL_BLOCK2_LAUNCH(PRO, EPI) \
    hipLaunchKernelGGL((conv3x3_block_bwd2_kernel<PRO, EPI>), dim3(grid), dim3(bb2::kThreads), 0, s, a)
    if (epilogue == 2) {
        if (pro) HRL_BLOCK2_LAUNCH(true, 2); else HRL_BLOCK2_LAUNCH(false, 2);
    } else if (epilogue == 3) {
        if (pro) HRL_BLOCK2_LAUNCH(true, 3); else HRL_BLOCK2_LAUNCH(false, 3);
    } else {
        if (pro) HRL_BLOCK2_LAUNCH(true, 0); else HRL_BLOCK2_LAUNCH(false, 0);
    }
#undef HRL_BLOCK2_LAUNCH
    int rc = status();
    if (rc || !dweight) return rc;
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3(kTaps * kC * kC / 64), dim3(256), 0, s, wpart, grid,
                       dweight);
    return status();
}

int64_t hrl_conv3x3_wgrad_partials(int64_t M, int64_t *offset_bytes) {
    if (M < 1) return -1;
    if (offset_bytes) *offset_bytes = (int64_t)kTaps * 2 * kC * 16 * 2 * 4;
    return block_grid_for(M);
}

int hrl_conv3x3_wgrad(const float *x, const float *dy, int64_t M, int64_t C_in, int64_t C_out, float *dweight,
                      void *workspace, int64_t workspace_bytes, void *stream) {
    if (C_in != kC || C_out != kC) return HRL_EINVAL;
    return hrl_conv3x3_wgrad_ex(x, nullptr, nullptr, dy, M, dweight, workspace, workspace_bytes, stream);
}

}  // extern "C"
