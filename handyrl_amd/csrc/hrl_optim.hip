// hrl_optim.hip — the learner step's tail on the flat gradient buffer (gfx950): gradient clipping, the deferred
// weight-gradient folds and Adam.
//
// The reference clips with nn.utils.clip_grad_norm_(params, 4.0) before Adam
// (handyrl/train.py:384): total = ||g||_2 over all parameters,
// coef = max_norm / (total + 1e-6), g *= min(coef, 1).  As torch ops on the
// flat buffer that is six launches (norm, add, reciprocal, mul, clamp, mul);
// the buffer is small (29 k floats for the TicTacToe net, 234 k for
// GeisterNet), so one workgroup reads it, folds the squares (fp64, fixed
// order), forms the coefficient and scales it in place: one launch.
//
// The step tail (hrl_grad_fold_norm + hrl_adam_clip) replaces what followed the backward as separate launches:
// the weight-gradient folds of the HIP Functions (per-workgroup partial rows -> the parameter gradients: the
// chain blocks' conv3x3_wgrad_reduce, heads_reduce, stem_reduce), the clip, torch's capturable step-count
// increment, the BatchNorm batch counters and torch's fused Adam -- two launches:
//  * step_fold_norm_kernel: 64-position blocks of the flat buffer; a position that a fold covers takes the
//    fixed-order fp64 sum of the partial column at that position (16 waves over interleaved partial rows,
//    combined in wave order) and adds it into its element (for a transposed fold, another position of the same fold), the
//    rest are read; each block writes the fp64 sum of squares of its final values; block 0 also
//    advances the step count and the batch counters;
//  * adam_clip_kernel: every workgroup folds the block sums in one fixed order (so all agree on the norm bit for
//    bit), forms clip_grad_norm_'s coefficient, scales its chunk of the gradient in place (p.grad is the clipped
//    gradient afterwards, as in the reference) and applies torch's fused Adam arithmetic (ATen
//    fused_adam_utils.cuh adam_math, ADAM_MODE::ORIGINAL, the same double / float promotions) to the parameters
//    of the live tensors.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kThreads = 1024;

__global__ __launch_bounds__(kThreads) void clip_kernel(float *__restrict__ g, int64_t n, float max_norm,
                                                        float *__restrict__ total_out) {
    __shared__ double red[kThreads];
    __shared__ float coef_s;
    const int t = threadIdx.x;
    double s = 0.0;
    const int64_t nv = n / 4;
    float4 *g4 = reinterpret_cast<float4 *>(g);
    for (int64_t i = t; i < nv; i += kThreads) {
        const float4 v = g4[i];
        s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    for (int64_t i = nv * 4 + t; i < n; i += kThreads) s += (double)g[i] * g[i];
    red[t] = s;
    __syncthreads();
    for (int w = kThreads / 2; w > 0; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    if (t == 0) {
        const float total = (float)sqrt(red[0]);
        total_out[0] = total;
        const float c = max_norm / (total + 1e-6f);
        // torch.clamp(c, max=1) propagates NaN: a NaN norm turns every gradient into NaN, as the
        // reference's clip_grad_norm_ does (an inf norm gives c = 0: finite gradients become 0)
        coef_s = (c < 1.0f || c != c) ? c : 1.0f;
    }
    __syncthreads();
    const float c = coef_s;
    for (int64_t i = t; i < nv; i += kThreads) {
        float4 v = g4[i];
        v.x *= c; v.y *= c; v.z *= c; v.w *= c;
        g4[i] = v;
    }
    for (int64_t i = nv * 4 + t; i < n; i += kThreads) g[i] *= c;
}

// Large buffers (GeisterNet: 234 k floats, 47 us in one workgroup): two launches over kParts workgroups.
// clip_partial_kernel: workgroup b folds the squares of its fixed chunk (fp64, fixed order) into part[b];
// clip_apply_kernel: every workgroup folds part[0 .. kParts) in the same fixed order (so all agree on the norm
// bit for bit), workgroup 0 writes it, and each scales its own chunk.  Deterministic; no inter-workgroup sync.
constexpr int kParts = 64;
constexpr int kThreads2 = 256;
constexpr int64_t kSplitAbove = 65536;   // floats; below it the one-launch kernel is faster

__device__ __forceinline__ void chunk_of(int64_t nv, int b, int64_t &lo, int64_t &hi) {
    const int64_t per = (nv + kParts - 1) / kParts;
    lo = min(nv, (int64_t)b * per);
    hi = min(nv, lo + per);
}

__global__ __launch_bounds__(kThreads2) void clip_partial_kernel(const float *__restrict__ g, int64_t n,
                                                                  double *__restrict__ part) {
    __shared__ double red[kThreads2];
    const int t = threadIdx.x, b = blockIdx.x;
    const int64_t nv = n / 4;
    int64_t lo, hi;
    chunk_of(nv, b, lo, hi);
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    double s = 0.0;
    for (int64_t i = lo + t; i < hi; i += kThreads2) {
        const float4 v = g4[i];
        s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    if (b == kParts - 1)   // the tail past the last float4
        for (int64_t i = nv * 4 + t; i < n; i += kThreads2) s += (double)g[i] * g[i];
    red[t] = s;
    __syncthreads();
    for (int w = kThreads2 / 2; w > 0; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    if (t == 0) part[b] = red[0];
}

__global__ __launch_bounds__(kThreads2) void clip_apply_kernel(float *__restrict__ g, int64_t n, float max_norm,
                                                                const double *__restrict__ part,
                                                                float *__restrict__ total_out) {
    __shared__ float coef_s;
    const int t = threadIdx.x, b = blockIdx.x;
    if (t == 0) {
        double s = 0.0;
        for (int i = 0; i < kParts; ++i) s += part[i];   // the same order in every workgroup
        const float total = (float)sqrt(s);
        if (b == 0) total_out[0] = total;
        const float c = max_norm / (total + 1e-6f);
        coef_s = (c < 1.0f || c != c) ? c : 1.0f;          // clip_kernel's clamp (NaN propagates)
    }
    __syncthreads();
    const float c = coef_s;
    const int64_t nv = n / 4;
    int64_t lo, hi;
    chunk_of(nv, b, lo, hi);
    float4 *g4 = reinterpret_cast<float4 *>(g);
    for (int64_t i = lo + t; i < hi; i += kThreads2) {
        float4 v = g4[i];
        v.x *= c; v.y *= c; v.z *= c; v.w *= c;
        g4[i] = v;
    }
    if (b == kParts - 1)
        for (int64_t i = nv * 4 + t; i < n; i += kThreads2) g[i] *= c;
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

// ------------------------------------------------------------------ the step tail
constexpr int kMaxFolds = 16;
constexpr int kMaxTensors = 64;
constexpr int kMaxCounters = 8;
constexpr int kBlk = 64;    // elements per fold/norm block

struct FoldTable {
    const float *part[kMaxFolds];
    int64_t stride[kMaxFolds], col0[kMaxFolds], nparts[kMaxFolds], dst[kMaxFolds], count[kMaxFolds];
    int mode[kMaxFolds];
    int nfolds;
};

struct StepCounters {
    float *step;                       // the optimizer's step count (float, as torch's capturable state)
    int64_t *ctr[kMaxCounters];        // BatchNorm num_batches_tracked
    int64_t inc[kMaxCounters];         // their increments (a recurrent unroll's per-step BatchNorm: T)
    int nctr;
};

// destination element of a fold's source column j: mode 0 identity; mode 1 a (Cout = 32, Cin = 32, 3, 3) conv
// weight from the chain blocks' [tap][ci][co] partial layout (conv3x3_wgrad_reduce_kernel's transposition).  A
// lane takes the source column at its own position, so a wave's 64 loads of a partial row are one contiguous
// 256-byte run; the transposition moves to the (once per element) store
__device__ __forceinline__ int64_t fold_dst(int mode, int64_t j) {
    if (mode == 1) {
        const int tap = (int)(j >> 10), ci = (int)((j >> 5) & 31), co = (int)(j & 31);
        return co * 288 + ci * 9 + tap;
    }
    return j;
}

constexpr int kFoldWaves = 16;   // waves per fold block: 16 x 8 row loads of 256 B in flight per workgroup

__global__ __launch_bounds__(64 * kFoldWaves) void step_fold_norm_kernel(float *__restrict__ g, int64_t n,
                                                                        FoldTable ft, StepCounters sc,
                                                                        double *__restrict__ norm_part) {
    __shared__ double red[kFoldWaves][kBlk];
    __shared__ double sq[kBlk];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * kBlk + lane;
    int f = -1;
    if (i < n)
        for (int k = 0; k < ft.nfolds; ++k)
            if (i >= ft.dst[k] && i < ft.dst[k] + ft.count[k]) f = k;
    double s = 0.0;
    if (f >= 0) {
        const float *src = ft.part[f] + ft.col0[f] + (i - ft.dst[f]);
        const int64_t np = ft.nparts[f], st = ft.stride[f];
        // wave w takes rows w, w+16, w+32, ...: eight independent chains (rows w + 16k + 128r, k < 8) with all
        // eight loads of a round issued before their adds, combined in chain order -- a fixed order
        double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        int64_t b = w;
        for (; b + 7 * kFoldWaves < np; b += 8 * kFoldWaves) {
            float t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = src[(b + kFoldWaves * k) * st];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += (double)t[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (b + kFoldWaves * k < np) acc[k] += (double)src[(b + kFoldWaves * k) * st];
        s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0) {
        double v;
        if (f >= 0) {
            v = 0.0;
            for (int k = 0; k < kFoldWaves; ++k) v += red[k][lane];   // wave order
            // accumulated, not assigned: a parameter reached again later in the backward has had that use's
            // gradient added into its p.grad by autograd already (the buffer is zeroed at step start, so a
            // single-use parameter gets 0 + fold = the fold exactly)
            const int64_t d = ft.dst[f] + fold_dst(ft.mode[f], i - ft.dst[f]);
            const float fv = g[d] + (float)v;
            g[d] = fv;
            v = (double)fv;
        } else {
            v = i < n ? (double)g[i] : 0.0;
        }
        sq[lane] = v * v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < kBlk; ++k) t += sq[k];
        norm_part[blockIdx.x] = t;
        if (blockIdx.x == 0) {
            if (sc.step) sc.step[0] += 1.0f;
            for (int k = 0; k < sc.nctr; ++k) sc.ctr[k][0] += sc.inc[k];
        }
    }
}

struct AdamTable {
    float *p[kMaxTensors];
    int64_t off[kMaxTensors + 1];      // flat offsets; off[nt] = n
    uint64_t live;                     // bit t: tensor t is updated (a parameter with no gradient is skipped)
    int nt;
};

struct AdamArgs {
    float *g, *m, *v;
    int64_t n;
    const double *norm_part;
    int64_t nblocks;
    float max_norm;
    float *total_out;
    const float *lr, *step;
    double beta1, beta2, eps, wd;
    // the learner's running statistics: acc_dst[k] += *acc_src[k] (NULL: the norm), once per step
    const float *acc_src[kMaxCounters];
    float *acc_dst;
    int nacc;
};

__global__ __launch_bounds__(256) void adam_clip_kernel(AdamArgs a, AdamTable tab) {
    __shared__ double red[256];
    __shared__ float coef_s;
    const int t = threadIdx.x;
    double s = 0.0;
    for (int64_t k = t; k < a.nblocks; k += 256) s += a.norm_part[k];
    red[t] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    if (t == 0) {
        const float total = (float)sqrt(red[0]);
        if (blockIdx.x == 0) {
            a.total_out[0] = total;
            for (int k = 0; k < a.nacc; ++k) a.acc_dst[k] += a.acc_src[k] ? a.acc_src[k][0] : total;
        }
        const float c = a.max_norm / (total + 1e-6f);
        coef_s = (c < 1.0f || c != c) ? c : 1.0f;      // clip_kernel's clamp (NaN propagates)
    }
    __syncthreads();
    const float c = coef_s;
    // fused_adam_utils.cuh: bias corrections in double, handed to adam_math as opmath_t (float)
    const double stepd = (double)a.step[0];
    const float bc1 = (float)(1.0 - pow(a.beta1, stepd));
    const float bc2s = (float)sqrt(1.0 - pow(a.beta2, stepd));
    const double lr = (double)a.lr[0];
    const float step_size = (float)(lr / bc1);
    const int64_t per = (a.n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = min(a.n, lo + per);
    int tt = 0;
    while (tt + 1 < tab.nt && lo >= tab.off[tt + 1]) ++tt;     // the chunk's first tensor (uniform)
    for (int64_t i = lo + t; i < hi; i += 256) {
        float gr = a.g[i] * c;
        a.g[i] = gr;
        while (tt + 1 < tab.nt && i >= tab.off[tt + 1]) ++tt;   // i ascends per thread: the tensor only advances
        if (!((tab.live >> tt) & 1)) continue;
        float *pp = tab.p[tt] + (i - tab.off[tt]);
        float param = *pp;
        float exp_avg = a.m[i], exp_avg_sq = a.v[i];
        if (a.wd != 0) gr = (float)((double)gr + (double)param * a.wd);
        exp_avg = (float)(a.beta1 * (double)exp_avg + (1 - a.beta1) * (double)gr);
        exp_avg_sq = (float)(a.beta2 * (double)exp_avg_sq + (1 - a.beta2) * (double)gr * (double)gr);
        const float denom = (float)((double)(sqrtf(exp_avg_sq) / bc2s) + a.eps);
        param -= step_size * exp_avg / denom;
        *pp = param;
        a.m[i] = exp_avg;
        a.v[i] = exp_avg_sq;
    }
}

}  // namespace

extern "C" {

int hrl_clip_grad_norm(float *grads, int64_t n, double max_norm, float *total_norm, void *stream) {
    if (!grads || !total_norm || n < 0 || (reinterpret_cast<uintptr_t>(grads) & 15) != 0) return HRL_EINVAL;
    hipLaunchKernelGGL(clip_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), grads, n,
                       (float)max_norm, total_norm);
    return status();
}

int64_t hrl_grad_fold_norm_blocks(int64_t n) { return n < 1 ? -1 : (n + kBlk - 1) / kBlk; }

int hrl_grad_fold_norm(float *grads, int64_t n, const float *const *parts, const int64_t *strides,
                       const int64_t *col0, const int64_t *nparts, const int64_t *dst, const int64_t *count,
                       const int *modes, int nfolds, float *step, int64_t *const *counters,
                       const int64_t *increments, int ncounters, double *norm_part, int64_t norm_part_bytes,
                       void *stream) {
    if (!grads || n < 1 || nfolds < 0 || nfolds > kMaxFolds || ncounters < 0 || ncounters > kMaxCounters ||
        !norm_part || norm_part_bytes < hrl_grad_fold_norm_blocks(n) * 8)
        return HRL_EINVAL;
    FoldTable ft{};
    for (int k = 0; k < nfolds; ++k) {
        if (!parts[k] || nparts[k] < 1 || count[k] < 1 || dst[k] < 0 || dst[k] + count[k] > n || col0[k] < 0 ||
            (modes[k] != 0 && modes[k] != 1) || (modes[k] == 1 && count[k] != 9216))
            return HRL_EINVAL;
        const int64_t span = modes[k] == 1 ? 9216 : count[k];
        if (strides[k] < col0[k] + span) return HRL_EINVAL;
        ft.part[k] = parts[k]; ft.stride[k] = strides[k]; ft.col0[k] = col0[k]; ft.nparts[k] = nparts[k];
        ft.dst[k] = dst[k]; ft.count[k] = count[k]; ft.mode[k] = modes[k];
    }
    ft.nfolds = nfolds;
    StepCounters sc{};
    sc.step = step;
    for (int k = 0; k < ncounters; ++k) {
        if (!counters[k] || (increments && increments[k] < 0)) return HRL_EINVAL;
        sc.ctr[k] = counters[k];
        sc.inc[k] = increments ? increments[k] : 1;
    }
    sc.nctr = ncounters;
    hipLaunchKernelGGL(step_fold_norm_kernel, dim3((unsigned)hrl_grad_fold_norm_blocks(n)), dim3(64 * kFoldWaves), 0,
                       static_cast<hipStream_t>(stream), grads, n, ft, sc, norm_part);
    return status();
}

int hrl_adam_clip(float *grads, int64_t n, const double *norm_part, double max_norm, float *total_norm,
                  float *const *params, const int64_t *offsets, const int *live, int ntensors, float *exp_avg,
                  float *exp_avg_sq, const float *lr, const float *step, double beta1, double beta2, double eps,
                  double weight_decay, const float *const *acc_src, int nacc, float *acc_dst, void *stream) {
    if (!grads || n < 1 || !norm_part || !total_norm || !params || !offsets || !live || ntensors < 1 ||
        ntensors > kMaxTensors || !exp_avg || !exp_avg_sq || !lr || !step || nacc < 0 || nacc > kMaxCounters ||
        (nacc > 0 && (!acc_src || !acc_dst)))
        return HRL_EINVAL;
    AdamTable tab{};
    for (int k = 0; k < ntensors; ++k) {
        if (!params[k] || offsets[k] < 0 || offsets[k + 1] < offsets[k]) return HRL_EINVAL;
        tab.p[k] = params[k];
        tab.off[k] = offsets[k];
        if (live[k]) tab.live |= (uint64_t)1 << k;
    }
    if (offsets[0] != 0 || offsets[ntensors] != n) return HRL_EINVAL;
    tab.off[ntensors] = n;
    tab.nt = ntensors;
    AdamArgs a{grads, exp_avg, exp_avg_sq, n, norm_part, hrl_grad_fold_norm_blocks(n), (float)max_norm, total_norm,
               lr, step, beta1, beta2, eps, weight_decay, {}, acc_dst, nacc};
    for (int k = 0; k < nacc; ++k) a.acc_src[k] = acc_src[k];
    // one element per thread up to 256 workgroups (each folds the block sums itself: a few KB from L2)
    const int64_t grid = (n + 255) / 256 < 256 ? (n + 255) / 256 : 256;
    hipLaunchKernelGGL(adam_clip_kernel, dim3((unsigned)grid), dim3(256), 0, static_cast<hipStream_t>(stream), a,
                       tab);
    return status();
}

int64_t hrl_clip_workspace_bytes(int64_t n) { return n < 0 ? -1 : (int64_t)kParts * 8; }

int hrl_clip_grad_norm_ws(float *grads, int64_t n, double max_norm, float *total_norm, void *workspace,
                          int64_t workspace_bytes, void *stream) {
    if (!grads || !total_norm || n < 0 || (reinterpret_cast<uintptr_t>(grads) & 15) != 0) return HRL_EINVAL;
    if (n <= kSplitAbove) return hrl_clip_grad_norm(grads, n, max_norm, total_norm, stream);
    if (!workspace || workspace_bytes < hrl_clip_workspace_bytes(n) || (reinterpret_cast<uintptr_t>(workspace) & 7))
        return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    hipLaunchKernelGGL(clip_partial_kernel, dim3(kParts), dim3(kThreads2), 0, s, grads, n, part);
    const int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(clip_apply_kernel, dim3(kParts), dim3(kThreads2), 0, s, grads, n, (float)max_norm, part,
                       total_norm);
    return status();
}

}  // extern "C"
