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
};

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

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

}  // namespace

extern "C" {

#ifdef HRL_STAMPS
int hrl_debug_set_stamps_conv(void *buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hrl_stamps), &buf, sizeof(buf)); }
#endif

int64_t hrl_conv3x3_workspace_bytes(int64_t M) {
    if (M < 1) return -1;
    return (int64_t)grid_for(M) * kTaps * kC * kC * 4 + (int64_t)kTaps * 2 * kC * 16 * 4 * 2;
}

int64_t hrl_conv3x3_stats_blocks(int64_t M) { return M < 1 ? -1 : grid_for(M); }

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
    if (M < 1 || !g || !y || !save_mean || !save_invstd || !kcoef || !gmean || !x || !dweight || !workspace)
        return HRL_EINVAL;
    if ((in_alpha == nullptr) != (in_beta == nullptr)) return HRL_EINVAL;
    if (workspace_bytes < hrl_conv3x3_workspace_bytes(M) || M * kRow * 4 > 0xffffffffLL) return HRL_EINVAL;
    if (gin && (!packed_flip || epilogue < 0 || epilogue == 1 || epilogue > 3)) return HRL_EINVAL;
    if (gin && epilogue == 2 && (!ep_mean || !ep_alpha || !ep_beta || !part)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = grid_for(M);
    float *wpart = static_cast<float *>(workspace) + kTaps * 2 * kC * 16 * 2;
    BlockBwdArgs a{g, y, bn_weight, bn_bias, save_mean, save_invstd, kcoef, gmean, x, in_alpha, in_beta, packed_flip,
                   ep_mean, ep_alpha, ep_beta, gin, part, wpart, M};
    const bool pro = in_alpha != nullptr;
#define HRL_BLOCK_LAUNCH(PRO, EPI, DG) \
    hipLaunchKernelGGL((conv3x3_block_bwd_kernel<PRO, EPI, DG>), dim3(grid), dim3(kThreads), 0, s, a)
    if (!gin) {
        if (pro) HRL_BLOCK_LAUNCH(true, 0, false); else HRL_BLOCK_LAUNCH(false, 0, false);
    } else if (epilogue == 2) {
        if (pro) HRL_BLOCK_LAUNCH(true, 2, true); else HRL_BLOCK_LAUNCH(false, 2, true);
    } else if (epilogue == 3) {
        if (pro) HRL_BLOCK_LAUNCH(true, 3, true); else HRL_BLOCK_LAUNCH(false, 3, true);
    } else {
        if (pro) HRL_BLOCK_LAUNCH(true, 0, true); else HRL_BLOCK_LAUNCH(false, 0, true);
    }
#undef HRL_BLOCK_LAUNCH
    int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3(kTaps * kC * kC / 64), dim3(256), 0, s, wpart, grid,
                       dweight);
    return status();
}

int hrl_conv3x3_wgrad(const float *x, const float *dy, int64_t M, int64_t C_in, int64_t C_out, float *dweight,
                      void *workspace, int64_t workspace_bytes, void *stream) {
    if (C_in != kC || C_out != kC) return HRL_EINVAL;
    return hrl_conv3x3_wgrad_ex(x, nullptr, nullptr, dy, M, dweight, workspace, workspace_bytes, stream);
}

}  // extern "C"
