// hrl_selfplay.hip — the sampling and recording tail of a self-play ply (handyrl/generation.py:43-62).
//
// Per ply the reference masks the illegal actions' logits (-1e32, generation.py:50-51), samples an action
// from softmax over the legal ones (random.choices, :53) and appends the moment (observation, policy,
// action_mask, action, value, reward, turn) to the episode (:55-62).  DeviceGenerator does that for E games
// at once with Gumbel-max over uniforms drawn up front; as torch ops it is ~25 launches per ply (mask,
// subtract, two logs, argmax, a where + index_copy per record), here ONE launch:
//   one wave per game, lanes over the A action labels:
//     m = legal ? 0 : 1e32;  p = logit - m;  g = p - log(-log(u))      (the torch formulation's fp32 ops)
//     action = argmax g, ties to the lowest label, NaN first (torch.argmax's order), shuffle reduction
//   slot t of each record gets the game's value when it is active and the reset value otherwise
//   (policy 0, action mask 1e32, action / value / turn / reward 0).
// The ply index t is read from device memory, so the launch is replayed unchanged by the ply's HIP graph.
// HBM-light (E*A*(4+1+4 in, 4+4 out) bytes, ~18 MB per ply at E=2048, A=214): latency bound.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/hrl_env.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kWave = 64;
constexpr int kGamesPerBlock = 4;

// torch.argmax's order: NaN beats everything, then larger values, ties to the lower index
__device__ __forceinline__ bool better(float a, int ia, float b, int ib) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return na && (!nb || ia < ib);
    return a > b || (a == b && ia < ib);
}

__global__ __launch_bounds__(kWave *kGamesPerBlock) void sample_record_kernel(
    const float *__restrict__ logits, int64_t lstride, const uint8_t *__restrict__ legal,
    const float *__restrict__ U, const int64_t *__restrict__ tptr, const float *__restrict__ value,
    const uint8_t *__restrict__ active, const int64_t *__restrict__ player, const double *__restrict__ reward,
    int64_t E, int A, int64_t Tm, int P, int64_t *__restrict__ action, float *__restrict__ policy_buf,
    float *__restrict__ amask_buf, int64_t *__restrict__ action_buf, float *__restrict__ value_buf,
    int64_t *__restrict__ turn_buf, double *__restrict__ reward_buf) {
    const int lane = threadIdx.x % kWave;
    const int64_t e = (int64_t)blockIdx.x * kGamesPerBlock + threadIdx.x / kWave;
    if (e >= E) return;
    const int64_t t = *tptr;
    const bool live = active[e] != 0;
    const float *lg = logits + e * lstride;
    const uint8_t *lm = legal + e * A;
    const float *u = U + (t * E + e) * A;
    float *pol = policy_buf + (e * Tm + t) * A;
    float *am = amask_buf + (e * Tm + t) * A;
    float best = 0.0f;
    int ib = A;   // no label yet
    for (int j = lane; j < A; j += kWave) {
        const float m = lm[j] ? 0.0f : 1e32f;
        const float p = lg[j] - m;
        const float g = p - logf(-logf(u[j]));
        if (ib == A || better(g, j, best, ib)) {
            best = g;
            ib = j;
        }
        pol[j] = live ? p : 0.0f;
        am[j] = live ? m : 1e32f;
    }
    for (int off = kWave / 2; off > 0; off >>= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(ib, off);
        if (oi != A && (ib == A || better(ob, oi, best, ib))) {
            best = ob;
            ib = oi;
        }
    }
    if (lane == 0) {
        action[e] = ib;
        const int64_t s = e * Tm + t;
        action_buf[s] = live ? ib : 0;
        value_buf[s] = live ? value[e] : 0.0f;
        turn_buf[s] = live ? player[e] : 0;
        if (reward && reward_buf)
            for (int q = 0; q < P; ++q) reward_buf[s * P + q] = live ? reward[e * P + q] : 0.0;
    }
}

// ---- the movers' recurrent state advance (generation.py:38-41): dst[l] row e <- src[l] row e where mask[e] ----
constexpr int kMaxRowLeaves = 16;
struct RowLeaves {
    float *dst[kMaxRowLeaves];
    const float *src[kMaxRowLeaves];
    int64_t dst_stride[kMaxRowLeaves], src_stride[kMaxRowLeaves], F[kMaxRowLeaves];
};

__global__ __launch_bounds__(256) void masked_rows_kernel(const uint8_t *__restrict__ mask, RowLeaves L) {
    const int64_t e = blockIdx.x;
    const int l = blockIdx.y;
    if (!mask[e]) return;
    const float *s = L.src[l] + e * L.src_stride[l];
    float *d = L.dst[l] + e * L.dst_stride[l];
    for (int64_t f = threadIdx.x; f < L.F[l]; f += blockDim.x) d[f] = s[f];
}

}  // namespace

extern "C" {

int hrl_masked_rows_copy(int nleaves, float *const *dst, const int64_t *dst_stride, const float *const *src,
                         const int64_t *src_stride, const int64_t *F, const uint8_t *mask, int64_t E, void *stream) {
    if (nleaves < 1 || nleaves > kMaxRowLeaves || !dst || !dst_stride || !src || !src_stride || !F || !mask || E < 0 ||
        E > 0x7fffffff)
        return HRL_EINVAL;
    RowLeaves L{};
    for (int l = 0; l < nleaves; ++l) {
        if (!dst[l] || !src[l] || F[l] < 1 || dst_stride[l] < F[l] || src_stride[l] < F[l]) return HRL_EINVAL;
        L.dst[l] = dst[l];
        L.src[l] = src[l];
        L.dst_stride[l] = dst_stride[l];
        L.src_stride[l] = src_stride[l];
        L.F[l] = F[l];
    }
    if (E == 0) return HRL_OK;
    hipLaunchKernelGGL(masked_rows_kernel, dim3((unsigned)E, nleaves), dim3(256), 0, static_cast<hipStream_t>(stream),
                       mask, L);
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err;
}


int hrl_selfplay_sample_record(const float *logits, int64_t logit_stride, const uint8_t *legal, const float *U,
                               const int64_t *t, const float *value, const uint8_t *active, const int64_t *player,
                               const double *reward, int64_t E, int64_t A, int64_t Tm, int64_t P, int64_t *action,
                               float *policy_buf, float *amask_buf, int64_t *action_buf, float *value_buf,
                               int64_t *turn_buf, double *reward_buf, void *stream) {
    if (E == 0) return HRL_OK;
    if (!logits || !legal || !U || !t || !value || !active || !player || !action || !policy_buf || !amask_buf ||
        !action_buf || !value_buf || !turn_buf || E < 0 || A < 1 || A > (1 << 20) || Tm < 1 || P < 1 ||
        logit_stride < A || ((reward == nullptr) != (reward_buf == nullptr)))
        return HRL_EINVAL;
    const int blocks = (int)((E + kGamesPerBlock - 1) / kGamesPerBlock);
    hipLaunchKernelGGL(sample_record_kernel, dim3(blocks), dim3(kWave * kGamesPerBlock), 0,
                       static_cast<hipStream_t>(stream), logits, logit_stride, legal, U, t, value, active, player,
                       reward, E, (int)A, Tm, (int)P, action, policy_buf, amask_buf, action_buf, value_buf, turn_buf,
                       reward_buf);
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err;
}

}  // extern "C"
