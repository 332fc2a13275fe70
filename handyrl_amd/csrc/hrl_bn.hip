// hrl_bn.hip — training-mode BatchNorm2d forward/backward for board-game nets on MI355X.
//
// The learner's env nets (tictactoe.py:17-69, geister.py:100-167,
// hungry_geese.py:23-57) put BatchNorm2d on activations of N = B*T*P samples
// x C = 32 channels x a tiny board (HW = 9 / 36 / 77).  The vendor spatial
// BatchNorm runs that shape at ~3% of HBM bandwidth (1.3 ms forward, 1.7 ms
// backward for 151 MB at N = 131072, HW = 9: profiles/r01_*).  Here every pass
// is a coalesced streaming pass:
//
//   forward : stats (1 read)  -> finalize (C blocks) -> apply (1 read + 1 write)
//   backward: reduce (2 reads) -> finalize            -> apply (2 reads + 1 write)
//
// Mapping: an (N, C*HW) row-major view; a workgroup owns a contiguous range
// of rows, each thread owns FIXED columns (a float4 of a row, or one float),
// so the channel of every element a thread touches is computed once, never
// per element.  Per-thread partials accumulate in fp64; the block folds them
// per column through LDS in a fixed order and then per channel; the finalize
// kernel folds the per-block partials with a fixed-shape tree.  Results are
// deterministic run to run.
// Formulas mirror PyTorch's CPU batch_norm (the reference learner runs on
// the CPU): y = x*alpha + beta with alpha = invstd*w, beta = b - mean*alpha;
// dx = ((dy - mean(dy)) - (x-mean)*k) * invstd * w with k = dot*invstd^2/M.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxSlots = 4;        // column slots per thread
constexpr int kMaxBlocks = 2048;
constexpr int kMaxRowFloats = 3072; // S = C*HW limit (LDS column accumulators: 2*S doubles)

struct Geo {
    int64_t N;
    int C, HW, S;      // S = C*HW floats per row (sample)
    int ncol;          // S / VW
    int rp;            // rows per iteration (ncol <= 256)
    int kc;            // column slots per thread (ncol > 256)
    int rows_per_block;
    int nblocks;
    // groups (a recurrent net's time steps run as one launch): rows [g*Ng, (g+1)*Ng) are group g, whose
    // statistics and coefficients are its own; nbg blocks per group, a block never straddles two
    int64_t Ng;
    int G, nbg;
};

// This block's rows [r0, r1) and group.
__device__ __forceinline__ void block_rows(const Geo &g, int64_t &r0, int64_t &r1, int &grp) {
    grp = (int)(blockIdx.x / (unsigned)g.nbg);
    const int lb = (int)blockIdx.x - grp * g.nbg;
    const int64_t gb = (int64_t)grp * g.Ng;
    r0 = gb + (int64_t)lb * g.rows_per_block;
    r1 = min(gb + g.Ng, r0 + g.rows_per_block);
}

template <int VW>
struct VecT;
template <>
struct VecT<4> { using T = float4; };
template <>
struct VecT<1> { using T = float; };

template <int VW>
__device__ __forceinline__ void load_vec(const float *p, float (&v)[VW]) {
    if constexpr (VW == 4) {
        const float4 q = *reinterpret_cast<const float4 *>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
        v[0] = *p;
    }
}

template <int VW>
__device__ __forceinline__ void store_vec(float *p, const float (&v)[VW]) {
    if constexpr (VW == 4) {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        *p = v[0];
    }
}

// This thread's place in the block: row offset `ro` (rows ro, ro+rp, ...) and column slots.
struct Lane {
    int ro;
    int col[kMaxSlots];   // vector column, -1 when unused
    __device__ __forceinline__ void init(const Geo &g) {
        const int t = threadIdx.x;
        if (g.ncol <= kThreads) {
            ro = t / g.ncol;
            col[0] = (ro < g.rp) ? t - ro * g.ncol : -1;
#pragma unroll
            for (int k = 1; k < kMaxSlots; ++k) col[k] = -1;
        } else {
            ro = 0;
#pragma unroll
            for (int k = 0; k < kMaxSlots; ++k) {
                const int cidx = t + k * kThreads;
                col[k] = (k < g.kc && cidx < g.ncol) ? cidx : -1;
            }
        }
    }
};

// Fold per-thread column partials (a, b) into LDS colsum[2][S] in a fixed
// order, then per channel into part[block][c][2].
template <int VW>
__device__ __forceinline__ void block_fold(const Geo &g, const Lane &ln, const double (&a)[kMaxSlots][VW],
                                           const double (&b)[kMaxSlots][VW], double *sh, double *part) {
    for (int i = threadIdx.x; i < 2 * g.S; i += kThreads) sh[i] = 0.0;
    __syncthreads();
    const int phases = (g.ncol <= kThreads) ? g.rp : 1;
    for (int p = 0; p < phases; ++p) {
        if (ln.ro == p) {
#pragma unroll
            for (int k = 0; k < kMaxSlots; ++k) {
                if (ln.col[k] >= 0) {
#pragma unroll
                    for (int j = 0; j < VW; ++j) {
                        sh[ln.col[k] * VW + j] += a[k][j];
                        sh[g.S + ln.col[k] * VW + j] += b[k][j];
                    }
                }
            }
        }
        __syncthreads();
    }
    for (int c = threadIdx.x; c < g.C; c += kThreads) {
        double sa = 0.0, sb = 0.0;
        for (int p = 0; p < g.HW; ++p) {
            sa += sh[c * g.HW + p];
            sb += sh[g.S + c * g.HW + p];
        }
        part[((int64_t)blockIdx.x * g.C + c) * 2 + 0] = sa;
        part[((int64_t)blockIdx.x * g.C + c) * 2 + 1] = sb;
    }
}

// ---- forward statistics: per-block sum and sum of squares per channel ----
template <int VW>
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const float *__restrict__ x, Geo g,
                                                            double *__restrict__ part) {
    extern __shared__ double sh[];
    Lane ln;
    ln.init(g);
    double a[kMaxSlots][VW], b[kMaxSlots][VW];
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
#pragma unroll
        for (int j = 0; j < VW; ++j) a[k][j] = b[k][j] = 0.0;

    int64_t r0, r1;
    int grp;
    block_rows(g, r0, r1, grp);
    const int step = (g.ncol <= kThreads) ? g.rp : 1;
    for (int64_t r = r0 + ln.ro; r < r1; r += step) {
        const float *row = x + r * g.S;
#pragma unroll
        for (int k = 0; k < kMaxSlots; ++k) {
            if (ln.col[k] >= 0) {
                float v[VW];
                load_vec<VW>(row + ln.col[k] * VW, v);
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    const double d = v[j];
                    a[k][j] += d;
                    b[k][j] += d * d;
                }
            }
        }
    }
    block_fold<VW>(g, ln, a, b, sh, part);
}

// ---- fold the per-block partials of each channel (one workgroup per channel) ----
// mode 0 (forward):  (sum x, sum x^2) -> mean, invstd, running stats, alpha/beta
// mode 1 (backward): (sum dy, sum dy*(x-mean)) -> dweight, dbias, k, mean(dy)
// With G groups the blocks [g*nbg, (g+1)*nbg) are group g: its statistics and coefficients land at
// [g*C + c]; the groups are visited in order, so the running statistics advance exactly as G sequential
// calls would, and dweight / dbias are the groups' sums.
__global__ __launch_bounds__(kThreads) void bn_finalize_kernel(
    int mode, const double *__restrict__ part, int nblocks, int C, double M, const float *__restrict__ weight,
    const float *__restrict__ bias, float *running_mean, float *running_var, float momentum, double eps,
    float *save_mean, float *save_invstd, float *coef_a, float *coef_b, float *dweight, float *dbias, int G) {
    __shared__ double red[2][kThreads];
    const int c = blockIdx.x;
    const int nbg = nblocks / G;
    const float w = weight ? weight[c] : 1.0f;
    float dw = 0.f, db = 0.f;
    // group grp's statistics -> its outputs (one thread; groups in order: the running statistics advance as G
    // sequential calls would)
    auto fin = [&](int grp, double S0, double S1) {
        const int gc = grp * C + c;
        if (mode == 0) {
            const double mean = S0 / M;
            double var = S1 / M - mean * mean;
            if (var < 0.0) var = 0.0;
            const float meanf = (float)mean;
            const float invstd = (float)(1.0 / sqrt(var + eps));
            save_mean[gc] = meanf;
            save_invstd[gc] = invstd;
            const float alpha = invstd * w;
            coef_a[gc] = alpha;
            coef_b[gc] = (bias ? bias[c] : 0.0f) - meanf * alpha;
            if (running_mean) running_mean[c] = momentum * meanf + (1.0f - momentum) * running_mean[c];
            if (running_var) {
                const float unbiased = (float)(M > 1.0 ? var * M / (M - 1.0) : var);
                running_var[c] = momentum * unbiased + (1.0f - momentum) * running_var[c];
            }
        } else {
            const float invstd = save_invstd[gc];
            const float sum_dy = (float)S0, dot = (float)S1;
            dw = grp == 0 ? dot * invstd : dw + dot * invstd;
            db = grp == 0 ? sum_dy : db + sum_dy;
            coef_a[gc] = dot * invstd * invstd / (float)M;   // k
            coef_b[gc] = sum_dy / (float)M;                   // mean(dy)
        }
    };
    if (G > 1 && G <= kThreads / 2) {
        // the groups' partial sums fold in parallel (tpg threads per group, a power of two, fixed tree order),
        // then one thread finalizes the groups in order: one reduction round instead of G
        int tpg = 1;
        while (tpg * 2 * G <= kThreads) tpg *= 2;
        const int grp = threadIdx.x / tpg, sub = threadIdx.x % tpg;
        double s0 = 0.0, s1 = 0.0;
        if (grp < G) {
            for (int i = sub; i < nbg; i += tpg) {
                const int64_t b = (int64_t)grp * nbg + i;
                s0 += part[(b * C + c) * 2 + 0];
                s1 += part[(b * C + c) * 2 + 1];
            }
        }
        red[0][threadIdx.x] = s0;
        red[1][threadIdx.x] = s1;
        __syncthreads();
        for (int wd = tpg / 2; wd > 0; wd >>= 1) {
            if (grp < G && sub < wd) {
                red[0][threadIdx.x] += red[0][threadIdx.x + wd];
                red[1][threadIdx.x] += red[1][threadIdx.x + wd];
            }
            __syncthreads();
        }
        // each group's outputs by a thread of its own (the fp64 divisions and square roots in parallel), then the
        // order-dependent parts -- the running statistics' G updates, the weight / bias gradient sums -- by one
        // thread in group order, as fin would run them (bit-identical)
        __shared__ float gv[2][kThreads / 2];
        if ((int)threadIdx.x < G) {
            const int grp = threadIdx.x, gc = grp * C + c;
            const double S0 = red[0][grp * tpg], S1 = red[1][grp * tpg];
            if (mode == 0) {
                const double mean = S0 / M;
                double var = S1 / M - mean * mean;
                if (var < 0.0) var = 0.0;
                const float meanf = (float)mean;
                const float invstd = (float)(1.0 / sqrt(var + eps));
                save_mean[gc] = meanf;
                save_invstd[gc] = invstd;
                const float alpha = invstd * w;
                coef_a[gc] = alpha;
                coef_b[gc] = (bias ? bias[c] : 0.0f) - meanf * alpha;
                gv[0][grp] = meanf;
                gv[1][grp] = (float)(M > 1.0 ? var * M / (M - 1.0) : var);
            } else {
                const float invstd = save_invstd[gc];
                const float sum_dy = (float)S0, dot = (float)S1;
                coef_a[gc] = dot * invstd * invstd / (float)M;   // k
                coef_b[gc] = sum_dy / (float)M;                   // mean(dy)
                gv[0][grp] = dot * invstd;
                gv[1][grp] = sum_dy;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int g2 = 0; g2 < G; ++g2) {
                if (mode == 0) {
                    if (running_mean) running_mean[c] = momentum * gv[0][g2] + (1.0f - momentum) * running_mean[c];
                    if (running_var) running_var[c] = momentum * gv[1][g2] + (1.0f - momentum) * running_var[c];
                } else {
                    dw = g2 == 0 ? gv[0][g2] : dw + gv[0][g2];
                    db = g2 == 0 ? gv[1][g2] : db + gv[1][g2];
                }
            }
            if (mode == 1) {
                if (dweight) dweight[c] = dw;
                if (dbias) dbias[c] = db;
            }
        }
        return;
    }
    for (int grp = 0; grp < G; ++grp) {
        double s0 = 0.0, s1 = 0.0;
        for (int i = threadIdx.x; i < nbg; i += kThreads) {
            const int64_t b = (int64_t)grp * nbg + i;
            s0 += part[(b * C + c) * 2 + 0];
            s1 += part[(b * C + c) * 2 + 1];
        }
        red[0][threadIdx.x] = s0;
        red[1][threadIdx.x] = s1;
        __syncthreads();
        // the fixed tree t += t + wd: the levels above one wave through LDS, the last six in wave 0's registers
        // (the same pairs and order, without a barrier per level)
        for (int wd = kThreads / 2; wd >= 64; wd >>= 1) {
            if ((int)threadIdx.x < wd) {
                red[0][threadIdx.x] += red[0][threadIdx.x + wd];
                red[1][threadIdx.x] += red[1][threadIdx.x + wd];
            }
            __syncthreads();
        }
        if (threadIdx.x < 64) {
            double v0 = red[0][threadIdx.x], v1 = red[1][threadIdx.x];
#pragma unroll
            for (int wd = 32; wd > 0; wd >>= 1) {
                v0 += __shfl_down(v0, wd, 64);
                v1 += __shfl_down(v1, wd, 64);
            }
            if (threadIdx.x == 0) fin(grp, v0, v1);
        }
        __syncthreads();   // red is reused by the next group
    }
    if (mode == 1 && threadIdx.x == 0) {
        if (dweight) dweight[c] = dw;
        if (dbias) dbias[c] = db;
    }
}

// ---- eval-mode coefficients from the running statistics ----
__global__ void bn_eval_coef_kernel(int C, const float *__restrict__ weight, const float *__restrict__ bias,
                                    const float *__restrict__ running_mean, const float *__restrict__ running_var,
                                    double eps, float *__restrict__ alpha, float *__restrict__ beta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float invstd = (float)(1.0 / sqrt((double)running_var[c] + eps));
    const float a = invstd * (weight ? weight[c] : 1.0f);
    alpha[c] = a;
    beta[c] = (bias ? bias[c] : 0.0f) - running_mean[c] * a;
}

// ---- forward apply: y = x*alpha[c] + beta[c] ----
// relu(v) as torch.relu: negatives to 0, NaN stays NaN
__device__ __forceinline__ float relu(float v) { return v < 0.f ? 0.f : v; }

template <int VW, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const float *__restrict__ x, Geo g,
                                                            const float *__restrict__ alpha,
                                                            const float *__restrict__ beta, float *__restrict__ y) {
    Lane ln;
    ln.init(g);
    int64_t r0, r1;
    int grp;
    block_rows(g, r0, r1, grp);
    alpha += grp * g.C;   // this block's group's coefficients
    beta += grp * g.C;
    float al[kMaxSlots][VW], be[kMaxSlots][VW];
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const int ch = ln.col[k] >= 0 ? (ln.col[k] * VW + j) / g.HW : 0;
            al[k][j] = alpha[ch];
            be[k][j] = beta[ch];
        }
    const int step = (g.ncol <= kThreads) ? g.rp : 1;
    for (int64_t r = r0 + ln.ro; r < r1; r += step) {
#pragma unroll
        for (int k = 0; k < kMaxSlots; ++k) {
            if (ln.col[k] >= 0) {
                const int64_t off = r * g.S + ln.col[k] * VW;
                float v[VW];
                load_vec<VW>(x + off, v);
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    v[j] = v[j] * al[k][j] + be[k][j];
                    if constexpr (RELU) v[j] = relu(v[j]);
                }
                store_vec<VW>(y + off, v);
            }
        }
    }
}

// ---- residual apply: y = relu(res + (x*alpha[c] + beta[c])) (GeeseNet block, hungry_geese.py:50-51) ----
template <int VW>
__global__ __launch_bounds__(kThreads) void bn_res_apply_kernel(const float *__restrict__ x,
                                                                const float *__restrict__ res, Geo g,
                                                                const float *__restrict__ alpha,
                                                                const float *__restrict__ beta,
                                                                float *__restrict__ y) {
    Lane ln;
    ln.init(g);
    int64_t r0, r1;
    int grp;
    block_rows(g, r0, r1, grp);
    alpha += grp * g.C;
    beta += grp * g.C;
    float al[kMaxSlots][VW], be[kMaxSlots][VW];
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const int ch = ln.col[k] >= 0 ? (ln.col[k] * VW + j) / g.HW : 0;
            al[k][j] = alpha[ch];
            be[k][j] = beta[ch];
        }
    const int step = (g.ncol <= kThreads) ? g.rp : 1;
    for (int64_t r = r0 + ln.ro; r < r1; r += step) {
#pragma unroll
        for (int k = 0; k < kMaxSlots; ++k) {
            if (ln.col[k] >= 0) {
                const int64_t off = r * g.S + ln.col[k] * VW;
                float v[VW], rv[VW];
                load_vec<VW>(x + off, v);
                load_vec<VW>(res + off, rv);
#pragma unroll
                for (int j = 0; j < VW; ++j) v[j] = relu(rv[j] + (v[j] * al[k][j] + be[k][j]));
                store_vec<VW>(y + off, v);
            }
        }
    }
}

// ---- backward reduce: per-block sum(dy) and sum(dy*(x-mean)) per channel ----
// With RELU the forward output was relu(x*alpha + beta): the incoming gradient
// is masked where that pre-activation is <= 0 (threshold_backward), recomputed
// here from x with the forward's own per-channel alpha/beta.
// MASK = 2: the gradient is masked where an external tensor `mo` (the forward's output after a
// ReLU, e.g. relu(h + bn(x)) of a residual block) is <= 0.
template <int VW, bool RELU, int MASK>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_kernel(const float *__restrict__ x,
                                                                 const float *__restrict__ dy, Geo g,
                                                                 const float *__restrict__ mean,
                                                                 const float *__restrict__ invstd,
                                                                 const float *__restrict__ weight,
                                                                 const float *__restrict__ bias,
                                                                 double *__restrict__ part,
                                                                 const float *__restrict__ mo) {
    extern __shared__ double sh[];
    Lane ln;
    ln.init(g);
    int64_t r0, r1;
    int grp;
    block_rows(g, r0, r1, grp);
    mean += grp * g.C;     // this block's group's statistics
    invstd += grp * g.C;
    float mu[kMaxSlots][VW], al[kMaxSlots][VW], be[kMaxSlots][VW];
    double a[kMaxSlots][VW], b[kMaxSlots][VW];
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            a[k][j] = b[k][j] = 0.0;
            const int ch = ln.col[k] >= 0 ? (ln.col[k] * VW + j) / g.HW : 0;
            mu[k][j] = mean[ch];
            // the forward's alpha/beta, recomputed with the same float operations (bn_finalize_kernel)
            al[k][j] = RELU ? invstd[ch] * (weight ? weight[ch] : 1.0f) : 0.f;
            be[k][j] = RELU ? (bias ? bias[ch] : 0.0f) - mean[ch] * al[k][j] : 0.f;
        }
    const int step = (g.ncol <= kThreads) ? g.rp : 1;
    for (int64_t r = r0 + ln.ro; r < r1; r += step) {
#pragma unroll
        for (int k = 0; k < kMaxSlots; ++k) {
            if (ln.col[k] >= 0) {
                const int64_t off = r * g.S + ln.col[k] * VW;
                float xv[VW], gv[VW], mv[VW];
                load_vec<VW>(x + off, xv);
                load_vec<VW>(dy + off, gv);
                if constexpr (MASK == 2) load_vec<VW>(mo + off, mv);
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    if constexpr (RELU) {
                        if (!(xv[j] * al[k][j] + be[k][j] > 0.f)) gv[j] = 0.f;
                    }
                    if constexpr (MASK == 2) {
                        if (!(mv[j] > 0.f)) gv[j] = 0.f;
                    }
                    a[k][j] += (double)gv[j];
                    b[k][j] += (double)gv[j] * (double)(xv[j] - mu[k][j]);
                }
            }
        }
    }
    block_fold<VW>(g, ln, a, b, sh, part);
}

// ---- backward apply: dx = ((dy - mean(dy)) - (x-mean)*k) * invstd * w ----
template <int VW, bool RELU, int MASK>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const float *__restrict__ x,
                                                                const float *__restrict__ dy, Geo g,
                                                                const float *__restrict__ mean,
                                                                const float *__restrict__ invstd,
                                                                const float *__restrict__ weight,
                                                                const float *__restrict__ kcoef,
                                                                const float *__restrict__ gmean,
                                                                const float *__restrict__ bias,
                                                                float *__restrict__ dx,
                                                                const float *__restrict__ mo) {
    Lane ln;
    ln.init(g);
    int64_t r0, r1;
    int grp;
    block_rows(g, r0, r1, grp);
    mean += grp * g.C;     // this block's group's statistics and backward coefficients
    invstd += grp * g.C;
    kcoef += grp * g.C;
    gmean += grp * g.C;
    float mu[kMaxSlots][VW], kk[kMaxSlots][VW], gm[kMaxSlots][VW], is[kMaxSlots][VW], ww[kMaxSlots][VW];
    float al[kMaxSlots][VW], be[kMaxSlots][VW];
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const int ch = ln.col[k] >= 0 ? (ln.col[k] * VW + j) / g.HW : 0;
            mu[k][j] = mean[ch];
            kk[k][j] = kcoef[ch];
            gm[k][j] = gmean[ch];
            is[k][j] = invstd[ch];
            ww[k][j] = weight ? weight[ch] : 1.0f;
            al[k][j] = RELU ? is[k][j] * ww[k][j] : 0.f;
            be[k][j] = RELU ? (bias ? bias[ch] : 0.0f) - mu[k][j] * al[k][j] : 0.f;
        }
    const int step = (g.ncol <= kThreads) ? g.rp : 1;
    for (int64_t r = r0 + ln.ro; r < r1; r += step) {
#pragma unroll
        for (int k = 0; k < kMaxSlots; ++k) {
            if (ln.col[k] >= 0) {
                const int64_t off = r * g.S + ln.col[k] * VW;
                float xv[VW], gv[VW], mv[VW];
                load_vec<VW>(x + off, xv);
                load_vec<VW>(dy + off, gv);
                if constexpr (MASK == 2) load_vec<VW>(mo + off, mv);
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    if constexpr (RELU) {
                        if (!(xv[j] * al[k][j] + be[k][j] > 0.f)) gv[j] = 0.f;
                    }
                    if constexpr (MASK == 2) {
                        if (!(mv[j] > 0.f)) gv[j] = 0.f;
                    }
                    const float t = (xv[j] - mu[k][j]) * kk[k][j];
                    xv[j] = (((gv[j] - gm[k][j]) - t) * is[k][j]) * ww[k][j];
                }
                store_vec<VW>(dx + off, xv);
            }
        }
    }
}

// ---------------------------------------------------------------- host side

bool make_geo(int64_t N, int64_t C, int64_t HW, int VW, Geo &g, int64_t G = 1) {
    if (N < 1 || C < 1 || HW < 1 || G < 1 || N % G != 0 || G > kMaxBlocks) return false;
    const int64_t S = C * HW;
    if (S > kMaxRowFloats || S % VW != 0) return false;
    g.N = N; g.C = (int)C; g.HW = (int)HW; g.S = (int)S;
    g.ncol = (int)(S / VW);
    if (g.ncol <= kThreads) {
        g.rp = kThreads / g.ncol;
        g.kc = 1;
    } else {
        g.rp = 1;
        g.kc = (g.ncol + kThreads - 1) / kThreads;
        if (g.kc > kMaxSlots) return false;
    }
    // ~16K floats per workgroup, at most kMaxBlocks workgroups; small tensors (a recurrent learner's
    // per-step BatchNorm, 256 x 1152 floats) get down to ~2K floats per workgroup instead of a handful of
    // workgroups each walking its rows serially (18 workgroups: 20 us for a 1.2 MB reduce)
    const int64_t total = N * S;
    int64_t nb = (total + 16383) / 16384;
    if (nb < 256) nb = std::min<int64_t>(256, (total + 2047) / 2048);
    nb = nb < 1 ? 1 : (nb > kMaxBlocks ? kMaxBlocks : nb);
    // per group: a share of the blocks, whole rows, never straddling groups
    const int64_t Ng = N / G;
    int64_t nbg = (nb + G - 1) / G;
    if (nbg > Ng) nbg = Ng;
    if (nbg * G > kMaxBlocks) nbg = kMaxBlocks / G;
    if (nbg < 1) nbg = 1;
    g.rows_per_block = (int)((Ng + nbg - 1) / nbg);
    g.nbg = (int)((Ng + g.rows_per_block - 1) / g.rows_per_block);
    g.Ng = Ng;
    g.G = (int)G;
    g.nblocks = g.nbg * g.G;
    return true;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// workspace layout: part[nblocks][C][2] doubles | coef_a[G*C] | coef_b[G*C] floats
int64_t ws_bytes(const Geo &g) { return (int64_t)g.nblocks * g.C * 16 + 2 * (int64_t)g.G * g.C * 4 + 64; }

int launch_status() {
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err;
}

}  // namespace

namespace {

template <int VW, bool RELU>
void launch_apply(const Geo &g, hipStream_t s, const float *x, const float *ca, const float *cb, float *y) {
    hipLaunchKernelGGL((bn_apply_kernel<VW, RELU>), dim3(g.nblocks), dim3(kThreads), 0, s, x, g, ca, cb, y);
}

template <int VW, bool RELU>
void launch_bwd(const Geo &g, hipStream_t s, size_t lds, const float *x, const float *dy, const float *mean,
                const float *invstd, const float *weight, const float *bias, double *part) {
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<VW, RELU, 0>), dim3(g.nblocks), dim3(kThreads), lds, s, x, dy, g, mean,
                       invstd, weight, bias, part, (const float *)nullptr);
}

template <int VW, bool RELU>
void launch_bwd_apply(const Geo &g, hipStream_t s, const float *x, const float *dy, const float *mean,
                      const float *invstd, const float *weight, const float *kcoef, const float *gmean,
                      const float *bias, float *dx) {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<VW, RELU, 0>), dim3(g.nblocks), dim3(kThreads), 0, s, x, dy, g, mean,
                       invstd, weight, kcoef, gmean, bias, dx, (const float *)nullptr);
}

}  // namespace

extern "C" {

int64_t hrl_bn_workspace_bytes(int64_t N, int64_t C, int64_t HW) {
    // the block partition depends on N and C*HW only, not on the vector width
    Geo g;
    if (make_geo(N, C, HW, 4, g) || make_geo(N, C, HW, 1, g)) return ws_bytes(g);
    return -1;
}

int64_t hrl_bn_workspace_bytes_grouped(int64_t N, int64_t C, int64_t HW, int64_t G) {
    Geo g;
    if (make_geo(N, C, HW, 4, g, G) || make_geo(N, C, HW, 1, g, G)) return ws_bytes(g);
    return -1;
}

int hrl_bn_forward_train_grouped(const float *x, int64_t N, int64_t C, int64_t HW, int64_t G, const float *weight,
                                 const float *bias, float *running_mean, float *running_var, double momentum,
                                 double eps, int relu, float *y, float *save_mean, float *save_invstd,
                                 void *workspace, int64_t workspace_bytes, void *stream) {
    if (!x || !y || !save_mean || !save_invstd || !workspace) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(y);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g, G)) return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    float *coef_a = reinterpret_cast<float *>(part + (int64_t)g.nblocks * g.C * 2);
    float *coef_b = coef_a + g.G * g.C;
    const size_t lds = sizeof(double) * 2 * g.S;
    if (vec) hipLaunchKernelGGL(bn_stats_kernel<4>, dim3(g.nblocks), dim3(kThreads), lds, s, x, g, part);
    else hipLaunchKernelGGL(bn_stats_kernel<1>, dim3(g.nblocks), dim3(kThreads), lds, s, x, g, part);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(g.C), dim3(kThreads), 0, s, 0, part, g.nblocks, g.C,
                       (double)g.Ng * (double)HW, weight, bias, running_mean, running_var, (float)momentum, eps,
                       save_mean, save_invstd, coef_a, coef_b, (float *)nullptr, (float *)nullptr, g.G);
    rc = launch_status();
    if (rc) return rc;
    if (vec) relu ? launch_apply<4, true>(g, s, x, coef_a, coef_b, y) : launch_apply<4, false>(g, s, x, coef_a, coef_b, y);
    else relu ? launch_apply<1, true>(g, s, x, coef_a, coef_b, y) : launch_apply<1, false>(g, s, x, coef_a, coef_b, y);
    return launch_status();
}

int hrl_bn_forward_train(const float *x, int64_t N, int64_t C, int64_t HW, const float *weight, const float *bias,
                         float *running_mean, float *running_var, double momentum, double eps, int relu, float *y,
                         float *save_mean, float *save_invstd, void *workspace, int64_t workspace_bytes,
                         void *stream) {
    return hrl_bn_forward_train_grouped(x, N, C, HW, 1, weight, bias, running_mean, running_var, momentum, eps, relu,
                                        y, save_mean, save_invstd, workspace, workspace_bytes, stream);
}

int hrl_bn_finalize_stats(const double *part, int64_t nparts, int64_t C, int64_t count, const float *weight,
                          const float *bias, float *running_mean, float *running_var, double momentum, double eps,
                          float *save_mean, float *save_invstd, float *alpha, float *beta, void *stream) {
    if (!part || !save_mean || !save_invstd || !alpha || !beta || nparts < 1 || C < 1 || count < 1)
        return HRL_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)C), dim3(kThreads), 0, static_cast<hipStream_t>(stream), 0,
                       part, (int)nparts, (int)C, (double)count, weight, bias, running_mean, running_var,
                       (float)momentum, eps, save_mean, save_invstd, alpha, beta, (float *)nullptr, (float *)nullptr,
                       1);
    return launch_status();
}

int hrl_bn_apply(const float *x, int64_t N, int64_t C, int64_t HW, const float *alpha, const float *beta, int relu,
                 float *y, void *stream) {
    if (!x || !y || !alpha || !beta) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(y);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (vec) relu ? launch_apply<4, true>(g, s, x, alpha, beta, y) : launch_apply<4, false>(g, s, x, alpha, beta, y);
    else relu ? launch_apply<1, true>(g, s, x, alpha, beta, y) : launch_apply<1, false>(g, s, x, alpha, beta, y);
    return launch_status();
}

int hrl_bn_forward_eval(const float *x, int64_t N, int64_t C, int64_t HW, const float *weight, const float *bias,
                        const float *running_mean, const float *running_var, double eps, int relu, float *y,
                        float *coef, void *stream) {
    if (!x || !y || !running_mean || !running_var || !coef) return HRL_EINVAL;
    if (N == 0) return HRL_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, (int)C, weight, bias,
                       running_mean, running_var, eps, coef, coef + C);
    const int rc = launch_status();
    if (rc) return rc;
    return hrl_bn_apply(x, N, C, HW, coef, coef + C, relu, y, stream);
}

int hrl_bn_finalize_backward(const double *part, int64_t nparts, int64_t C, int64_t count, const float *weight,
                             const float *save_invstd, float *dweight, float *dbias, float *kcoef, float *gmean,
                             void *stream) {
    if (!part || !save_invstd || !kcoef || !gmean || nparts < 1 || C < 1 || count < 1) return HRL_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)C), dim3(kThreads), 0, static_cast<hipStream_t>(stream), 1,
                       part, (int)nparts, (int)C, (double)count, weight, (const float *)nullptr, (float *)nullptr,
                       (float *)nullptr, 0.f, 0.0, (float *)nullptr, const_cast<float *>(save_invstd), kcoef, gmean,
                       dweight, dbias, 1);
    return launch_status();
}

int hrl_bn_backward_apply(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW, const float *weight,
                          const float *bias, const float *save_mean, const float *save_invstd, int relu,
                          const float *kcoef, const float *gmean, float *dx, void *stream) {
    if (!x || !dy || !dx || !save_mean || !save_invstd || !kcoef || !gmean || dx == dy) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(dy) && aligned16(dx);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (vec) {
        if (relu) launch_bwd_apply<4, true>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
        else launch_bwd_apply<4, false>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
    } else {
        if (relu) launch_bwd_apply<1, true>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
        else launch_bwd_apply<1, false>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
    }
    return launch_status();
}

int hrl_bn_backward_grouped(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW, int64_t G,
                            const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                            int relu, float *dx, float *dweight, float *dbias, void *workspace,
                            int64_t workspace_bytes, void *stream) {
    if (!x || !dy || !dx || !save_mean || !save_invstd || !workspace || dx == dy) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(dy) && aligned16(dx);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g, G)) return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    float *kcoef = reinterpret_cast<float *>(part + (int64_t)g.nblocks * g.C * 2);
    float *gmean = kcoef + g.G * g.C;
    const size_t lds = sizeof(double) * 2 * g.S;
    if (vec) relu ? launch_bwd<4, true>(g, s, lds, x, dy, save_mean, save_invstd, weight, bias, part)
                  : launch_bwd<4, false>(g, s, lds, x, dy, save_mean, save_invstd, weight, bias, part);
    else relu ? launch_bwd<1, true>(g, s, lds, x, dy, save_mean, save_invstd, weight, bias, part)
              : launch_bwd<1, false>(g, s, lds, x, dy, save_mean, save_invstd, weight, bias, part);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(g.C), dim3(kThreads), 0, s, 1, part, g.nblocks, g.C,
                       (double)g.Ng * (double)HW, weight, (const float *)nullptr, (float *)nullptr, (float *)nullptr,
                       0.0f, 0.0, (float *)nullptr, const_cast<float *>(save_invstd), kcoef, gmean, dweight, dbias,
                       g.G);
    rc = launch_status();
    if (rc) return rc;
    if (vec) relu ? launch_bwd_apply<4, true>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx)
                  : launch_bwd_apply<4, false>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
    else relu ? launch_bwd_apply<1, true>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx)
              : launch_bwd_apply<1, false>(g, s, x, dy, save_mean, save_invstd, weight, kcoef, gmean, bias, dx);
    return launch_status();
}

int hrl_bn_backward(const float *x, const float *dy, int64_t N, int64_t C, int64_t HW, const float *weight,
                    const float *bias, const float *save_mean, const float *save_invstd, int relu, float *dx,
                    float *dweight, float *dbias, void *workspace, int64_t workspace_bytes, void *stream) {
    return hrl_bn_backward_grouped(x, dy, N, C, HW, 1, weight, bias, save_mean, save_invstd, relu, dx, dweight, dbias,
                                   workspace, workspace_bytes, stream);
}

int hrl_bn_apply_residual(const float *x, const float *res, int64_t N, int64_t C, int64_t HW, const float *alpha,
                          const float *beta, float *y, void *stream) {
    if (!res) return hrl_bn_apply(x, N, C, HW, alpha, beta, 1, y, stream);
    if (!x || !y || !alpha || !beta) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(res) && aligned16(y);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (vec) hipLaunchKernelGGL(bn_res_apply_kernel<4>, dim3(g.nblocks), dim3(kThreads), 0, s, x, res, g, alpha, beta, y);
    else hipLaunchKernelGGL(bn_res_apply_kernel<1>, dim3(g.nblocks), dim3(kThreads), 0, s, x, res, g, alpha, beta, y);
    return launch_status();
}

int hrl_bn_backward_apply_masked(const float *x, const float *dy, const float *out, int64_t N, int64_t C, int64_t HW,
                                 const float *weight, const float *save_mean, const float *save_invstd,
                                 const float *kcoef, const float *gmean, float *dx, void *stream) {
    if (!x || !dy || !out || !dx || !save_mean || !save_invstd || !kcoef || !gmean || dx == dy) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(dy) && aligned16(dx) && aligned16(out);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(g.nblocks), block(kThreads);
    const float *nul = nullptr;
    if (vec) hipLaunchKernelGGL((bn_bwd_apply_kernel<4, false, 2>), grid, block, 0, s, x, dy, g, save_mean, save_invstd,
                                weight, kcoef, gmean, nul, dx, out);
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<1, false, 2>), grid, block, 0, s, x, dy, g, save_mean, save_invstd,
                            weight, kcoef, gmean, nul, dx, out);
    return launch_status();
}

int hrl_bn_backward_masked_coefs(const float *x, const float *dy, const float *out, int64_t N, int64_t C,
                                 int64_t HW, const float *weight, const float *save_mean, const float *save_invstd,
                                 float *kcoef, float *gmean, float *dweight, float *dbias, void *workspace,
                                 int64_t workspace_bytes, void *stream) {
    if (!x || !dy || !out || !save_mean || !save_invstd || !kcoef || !gmean || !workspace) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(dy) && aligned16(out);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    const size_t lds = sizeof(double) * 2 * g.S;
    const dim3 grid(g.nblocks), block(kThreads);
    const float *nul = nullptr;
    if (vec) hipLaunchKernelGGL((bn_bwd_reduce_kernel<4, false, 2>), grid, block, lds, s, x, dy, g, save_mean,
                                save_invstd, weight, nul, part, out);
    else hipLaunchKernelGGL((bn_bwd_reduce_kernel<1, false, 2>), grid, block, lds, s, x, dy, g, save_mean,
                            save_invstd, weight, nul, part, out);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(g.C), dim3(kThreads), 0, s, 1, part, g.nblocks, g.C,
                       (double)N * (double)HW, weight, (const float *)nullptr, (float *)nullptr, (float *)nullptr,
                       0.0f, 0.0, (float *)nullptr, const_cast<float *>(save_invstd), kcoef, gmean, dweight, dbias,
                       1);
    return launch_status();
}

int hrl_bn_backward_masked(const float *x, const float *dy, const float *out, int64_t N, int64_t C, int64_t HW,
                           const float *weight, const float *save_mean, const float *save_invstd, float *dx,
                           float *dweight, float *dbias, void *workspace, int64_t workspace_bytes, void *stream) {
    if (!x || !dy || !out || !dx || !save_mean || !save_invstd || !workspace || dx == dy) return HRL_EINVAL;
    const bool vec = (C * HW) % 4 == 0 && aligned16(x) && aligned16(dy) && aligned16(dx) && aligned16(out);
    Geo g;
    if (!make_geo(N, C, HW, vec ? 4 : 1, g)) return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(g)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    float *kcoef = reinterpret_cast<float *>(part + (int64_t)g.nblocks * g.C * 2);
    float *gmean = kcoef + g.C;
    const size_t lds = sizeof(double) * 2 * g.S;
    const dim3 grid(g.nblocks), block(kThreads);
    const float *nul = nullptr;
    if (vec) hipLaunchKernelGGL((bn_bwd_reduce_kernel<4, false, 2>), grid, block, lds, s, x, dy, g, save_mean,
                                save_invstd, weight, nul, part, out);
    else hipLaunchKernelGGL((bn_bwd_reduce_kernel<1, false, 2>), grid, block, lds, s, x, dy, g, save_mean,
                            save_invstd, weight, nul, part, out);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(g.C), dim3(kThreads), 0, s, 1, part, g.nblocks, g.C,
                       (double)N * (double)HW, weight, (const float *)nullptr, (float *)nullptr, (float *)nullptr,
                       0.0f, 0.0, (float *)nullptr, const_cast<float *>(save_invstd), kcoef, gmean, dweight, dbias,
                       1);
    rc = launch_status();
    if (rc) return rc;
    if (vec) hipLaunchKernelGGL((bn_bwd_apply_kernel<4, false, 2>), grid, block, 0, s, x, dy, g, save_mean, save_invstd,
                                weight, kcoef, gmean, nul, dx, out);
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<1, false, 2>), grid, block, 0, s, x, dy, g, save_mean, save_invstd,
                            weight, kcoef, gmean, nul, dx, out);
    return launch_status();
}

}  // extern "C"
