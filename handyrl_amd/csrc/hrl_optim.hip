// hrl_optim.hip — gradient clipping of the learner's flat gradient buffer in one launch (gfx950).
//
// The reference clips with nn.utils.clip_grad_norm_(params, 4.0) before Adam
// (handyrl/train.py:384): total = ||g||_2 over all parameters,
// coef = max_norm / (total + 1e-6), g *= min(coef, 1).  As torch ops on the
// flat buffer that is six launches (norm, add, reciprocal, mul, clamp, mul);
// the buffer is small (29 k floats for the TicTacToe net, 234 k for
// GeisterNet), so one workgroup reads it, folds the squares (fp64, fixed
// order), forms the coefficient and scales it in place: one launch.

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

}  // namespace

extern "C" {

int hrl_clip_grad_norm(float *grads, int64_t n, double max_norm, float *total_norm, void *stream) {
    if (!grads || !total_norm || n < 0 || (reinterpret_cast<uintptr_t>(grads) & 15) != 0) return HRL_EINVAL;
    hipLaunchKernelGGL(clip_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), grads, n,
                       (float)max_norm, total_norm);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

}  // extern "C"
