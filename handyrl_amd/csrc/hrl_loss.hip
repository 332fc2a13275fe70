// hrl_loss.hip — fused learner loss for HandyRL on MI355X (gfx950).
//
// One learner step's loss after the network forward, train.py:220-258 and
// compose_losses train.py:188-215, as five launches instead of ~60 small
// PyTorch kernels (log_softmax x2, gather x2, exp, clamp x2, stack/neg/div
// for the zero-sum symmetrisation, 2-4 target scans, the advantage
// composition, five masked reductions, Categorical entropy, ...):
//
//   prep   (one thread per (b,t)): log-softmax + gather of the behaviour and
//          target policies, rho = exp(lt - lb), clipped rho, entropy of the
//          target policy, zero-sum value symmetrisation and outcome padding
//   scan x2 (hrl_targets.hip): value head (value_target targets +
//          policy_target advantages) and return head, one launch each
//   terms  (one thread per (b,t)): turn advantages, the five loss sums and
//          dcnt as fp64 per-block partials
//   reduce (one workgroup): fixed-order fold of the partials -> 6 floats
//
// and the backward as ONE launch of closed-form gradients w.r.t. the target
// policy logits, the value head and the return head (targets and advantages
// are detached in the reference, train.py:228-232), scaled by the upstream
// gradients of the five losses read from device memory (graph-capturable).
// Sums are fp64 and fold in a fixed order: deterministic run to run.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/hrl_loss.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTerms = 6;   // p, v (before /2), r, ent, ent weighted by progress, dcnt

struct LossDims {
    int64_t B, T, BT;
    int P, Pp, A;
};

// workspace layout (floats, BT = B*T), then fp64 partials
struct Ws {
    float *lt, *crho, *ent, *vprep, *tv, *advv, *tr, *advr, *turn;
    double *part;
    int nblocks;
};

__host__ __device__ inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

__host__ __device__ inline Ws carve(void *base, const LossDims &d) {
    Ws w;
    float *f = static_cast<float *>(base);
    const int64_t np = d.BT * d.Pp, nv = d.BT * d.P;
    w.lt = f; f += np;
    w.crho = f; f += np;
    w.ent = f; f += np;
    w.vprep = f; f += nv;
    w.tv = f; f += nv;
    w.advv = f; f += nv;
    w.tr = f; f += nv;
    w.advr = f; f += nv;
    w.turn = f; f += d.BT;
    const int64_t off = align16((int64_t)((char *)f - (char *)base));
    w.part = reinterpret_cast<double *>((char *)base + off);
    w.nblocks = (int)((d.BT + kThreads - 1) / kThreads);
    return w;
}

int64_t ws_bytes(const LossDims &d) {
    const int64_t floats = 3 * d.BT * d.Pp + 5 * d.BT * d.P + d.BT;
    const int64_t nblocks = (d.BT + kThreads - 1) / kThreads;
    return align16(floats * 4) + nblocks * kTerms * 8 + 64;
}

struct FwdArgs {
    const float *tpol, *bpol;
    const int64_t *action;
    const float *emask, *tmask, *omask, *progress, *value, *outcome, *ret_out, *ret, *reward;
    int value_mc, symmetrize;
    float ent_coef, ent_decay;
};

// log-softmax pieces of one row of A logits: max m and s = sum exp(z - m)
__device__ __forceinline__ void row_stats(const float *z, int A, float &m, float &s) {
    m = z[0];
    for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
    s = 0.f;
    for (int a = 0; a < A; ++a) s += expf(z[a] - m);
}

// ---- prep: IS ratios, entropy, value preparation -----------------------------------------------
__global__ __launch_bounds__(kThreads) void loss_prep_kernel(FwdArgs a, LossDims d, Ws w) {
    const int64_t bt = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (bt >= d.BT) return;
    const int64_t b = bt / d.T;
    const float em = a.emask[bt];
    for (int pp = 0; pp < d.Pp; ++pp) {
        const int64_t row = bt * d.Pp + pp;
        const float *zt = a.tpol + row * d.A;
        const float *zb = a.bpol + row * d.A;
        const int64_t act = a.action[row];
        float mt, st, mb, sb;
        row_stats(zt, d.A, mt, st);
        row_stats(zb, d.A, mb, sb);
        // F.log_softmax(x)[act] = (x - max) - log(sum exp(x - max))      (train.py:224-225)
        const float lt = ((zt[act] - mt) - logf(st)) * em;
        const float lb = ((zb[act] - mb) - logf(sb)) * em;
        const float rho = expf(lt - lb);                                    // train.py:228-229
        w.lt[row] = lt;
        w.crho[row] = fminf(fmaxf(rho, 0.f), 1.f);                          // train.py:230-231
        // Categorical(logits).entropy(): logits normalised by logsumexp = m + log(s)
        const float lse = mt + logf(st);
        float h = 0.f;
        for (int q = 0; q < d.A; ++q) {
            const float la = zt[q] - lse;
            h += la * (expf(zt[q] - mt) / st);
        }
        w.ent[row] = -h;
    }
    if (a.value) {                                                          // train.py:234-239
        const float *v = a.value + bt * d.P;
        const float *om = a.omask + bt * d.P;
        for (int p = 0; p < d.P; ++p) {
            float vp = v[p];
            if (a.symmetrize) {   // two-player zero-sum: (v - swap(v)) / (sum omask + 1e-8)
                vp = (v[p] + (-v[1 - p])) / ((om[0] + om[1]) + 1e-8f);
            }
            const float oc = a.outcome[b * d.P + p];
            w.vprep[bt * d.P + p] = vp * em + oc * (1.f - em);
            if (a.value_mc) w.tv[bt * d.P + p] = oc;     // MC value target = outcome (losses.py:17)
        }
    }
    if (a.ret_out && a.value_mc) {                       // MC return target = batch['return']
        for (int p = 0; p < d.P; ++p) w.tr[bt * d.P + p] = a.ret[bt * d.P + p];
    }
}

// ---- terms: advantages, loss partial sums --------------------------------------------------------
__global__ __launch_bounds__(kThreads) void loss_terms_kernel(FwdArgs a, LossDims d, Ws w, int has_ret) {
    __shared__ double red[kTerms][kThreads];
    const int64_t bt = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    double acc[kTerms] = {0, 0, 0, 0, 0, 0};
    if (bt < d.BT) {
        const float *tm = a.tmask + bt * d.P;
        const float *om = a.omask + bt * d.P;
        // total_advantages = clipped_rhos * (adv_value + adv_return); turn sum under turn_mask
        float turn = 0.f;
        for (int p = 0; p < d.P; ++p) {
            const int pp = d.Pp == 1 ? 0 : p;
            float s = 0.f;
            if (a.value) s = s + w.advv[bt * d.P + p];
            if (has_ret) s = s + w.advr[bt * d.P + p];
            turn += (w.crho[bt * d.Pp + pp] * s) * tm[p];
        }
        w.turn[bt] = turn;
        for (int pp = 0; pp < d.Pp; ++pp) acc[0] += (double)(-w.lt[bt * d.Pp + pp] * turn);
        const float prog = 1.f - a.progress[bt] * (1.f - a.ent_decay);
        for (int p = 0; p < d.P; ++p) {
            const int pp = d.Pp == 1 ? 0 : p;
            if (a.value) {
                const float e = a.value[bt * d.P + p] - w.tv[bt * d.P + p];
                acc[1] += (double)((e * e) * om[p]);
            }
            if (has_ret) {
                const float x = a.ret_out[bt * d.P + p] - w.tr[bt * d.P + p];
                const float ax = fabsf(x);
                const float l = ax < 1.f ? 0.5f * x * x : ax - 0.5f;
                acc[2] += (double)(l * om[p]);
            }
            const float ent = w.ent[bt * d.Pp + pp] * tm[p];
            acc[3] += (double)ent;
            acc[4] += (double)(ent * prog);
            acc[5] += (double)tm[p];
        }
    }
#pragma unroll
    for (int k = 0; k < kTerms; ++k) red[k][threadIdx.x] = acc[k];
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
#pragma unroll
            for (int k = 0; k < kTerms; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x < kTerms) w.part[(int64_t)blockIdx.x * kTerms + threadIdx.x] = red[threadIdx.x][0];
}

// ---- reduce: fixed-order fold of the block partials -> p, v, r, ent, total, dcnt ---------------
__global__ __launch_bounds__(kThreads) void loss_reduce_kernel(Ws w, float ent_coef, float *losses) {
    __shared__ double red[kTerms][kThreads];
    double acc[kTerms] = {0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < w.nblocks; i += kThreads) {
#pragma unroll
        for (int k = 0; k < kTerms; ++k) acc[k] += w.part[(int64_t)i * kTerms + k];
    }
#pragma unroll
    for (int k = 0; k < kTerms; ++k) red[k][threadIdx.x] = acc[k];
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
#pragma unroll
            for (int k = 0; k < kTerms; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float lp = (float)red[0][0];
        const float lv = (float)(red[1][0] / 2.0);
        const float lr = (float)red[2][0];
        const float le = (float)red[3][0];
        const float lew = (float)red[4][0];
        losses[0] = lp;
        losses[1] = lv;
        losses[2] = lr;
        losses[3] = le;
        losses[4] = ((lp + lv) + lr) + lew * -ent_coef;   // train.py:211-213
        losses[5] = (float)red[5][0];
    }
}

// ---- backward: closed-form gradients ------------------------------------------------------------
struct BwdArgs {
    const float *tpol;
    const int64_t *action;
    const float *emask, *tmask, *omask, *progress, *value, *ret_out;
    const float *dl;   // upstream gradients of p, v, r, ent, total
    float *g_tpol, *g_value, *g_ret;
    float ent_coef, ent_decay;
};

__global__ __launch_bounds__(kThreads) void loss_backward_kernel(BwdArgs a, LossDims d, Ws w) {
    const int64_t bt = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (bt >= d.BT) return;
    const float dp = a.dl[0], dv = a.dl[1], dr = a.dl[2], de = a.dl[3], dt = a.dl[4];
    const float *tm = a.tmask + bt * d.P;
    const float *om = a.omask + bt * d.P;
    const float em = a.emask[bt];
    const float prog = 1.f - a.progress[bt] * (1.f - a.ent_decay);
    const float cp = -(dp + dt) * w.turn[bt] * em;           // d(-lt*turn)/d(lt) * d(lt)/d(log_softmax)
    for (int pp = 0; pp < d.Pp; ++pp) {
        const int64_t row = bt * d.Pp + pp;
        const float *z = a.tpol + row * d.A;
        float *g = a.g_tpol + row * d.A;
        // entropy weights of this policy row: players p that read it (all when Pp == 1)
        float wsum = 0.f, wdec = 0.f;
        for (int p = 0; p < d.P; ++p) {
            if (d.Pp == 1 || p == pp) {
                wsum += tm[p];
                wdec += tm[p] * prog;
            }
        }
        const float ce = de * wsum + dt * (-a.ent_coef) * wdec;
        float m, s;
        row_stats(z, d.A, m, s);
        const float lse = m + logf(s);
        const float h = w.ent[row];
        const int64_t act = a.action[row];
        for (int q = 0; q < d.A; ++q) {
            const float pq = expf(z[q] - m) / s;
            const float la = z[q] - lse;
            const float onehot = (q == act) ? 1.f : 0.f;
            g[q] = cp * (onehot - pq) + ce * (-pq * (la + h));    // dH/dz = -p (log p + H)
        }
    }
    for (int p = 0; p < d.P; ++p) {
        const int64_t i = bt * d.P + p;
        if (a.g_value) a.g_value[i] = (dv + dt) * (a.value[i] - w.tv[i]) * om[p];
        if (a.g_ret) {
            const float x = a.ret_out[i] - w.tr[i];
            const float sl = fminf(fmaxf(x, -1.f), 1.f);              // smooth_l1' (beta = 1)
            a.g_ret[i] = (dr + dt) * sl * om[p];
        }
    }
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool dims_ok(int64_t B, int64_t T, int64_t P, int64_t Pp, int64_t A, LossDims &d) {
    if (B < 1 || T < 1 || P < 1 || P > 64 || A < 1 || !(Pp == 1 || Pp == P)) return false;
    d.B = B; d.T = T; d.BT = B * T; d.P = (int)P; d.Pp = (int)Pp; d.A = (int)A;
    return d.BT < ((int64_t)1 << 40);
}

// ------------------------------------------------------------------ output masking
// forward_prediction's post-processing of a feed-forward net's outputs (train.py:176-183):
//   policy[bt, a] = sum_p o_pol[bt, p|0, a] * tmask[bt, p] - amask[bt, a]
//   value[bt, p]  = o_val[bt, p|0] * omask[bt, p]
// one launch each way instead of torch's mul / sum / sub / mul (and their backward mul / sum-to-size
// pairs).  The float operations and the p order are torch's: products rounded, summed from 0 in p order.
__global__ __launch_bounds__(kThreads) void out_mask_fwd_kernel(const float *__restrict__ opol,
                                                                const float *__restrict__ oval,
                                                                const float *__restrict__ tmask,
                                                                const float *__restrict__ omask,
                                                                const float *__restrict__ amask, int64_t BT, int P,
                                                                int Pq, int A, float *__restrict__ pol,
                                                                float *__restrict__ val) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t npol = BT * A;
    if (i < npol) {
        const int64_t bt = i / A;
        const int a = (int)(i - bt * A);
        float acc = 0.f;
        for (int p = 0; p < P; ++p) acc += opol[(bt * Pq + (Pq == 1 ? 0 : p)) * A + a] * tmask[bt * P + p];
        pol[i] = acc - amask[i];
    } else if (oval && i < npol + BT * P) {
        const int64_t j = i - npol;
        const int64_t bt = j / P;
        const int p = (int)(j - bt * P);
        val[j] = oval[bt * Pq + (Pq == 1 ? 0 : p)] * omask[j];
    }
}

__global__ __launch_bounds__(kThreads) void out_mask_bwd_kernel(const float *__restrict__ gpol,
                                                                const float *__restrict__ gval,
                                                                const float *__restrict__ tmask,
                                                                const float *__restrict__ omask, int64_t BT, int P,
                                                                int Pq, int A, float *__restrict__ gopol,
                                                                float *__restrict__ goval) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t npol = BT * Pq * A;
    if (i < npol) {
        const int64_t btq = i / A;
        const int a = (int)(i - btq * A);
        const int64_t bt = btq / Pq;
        const int q = (int)(btq - bt * Pq);
        const float g = gpol[bt * A + a];
        float acc;
        if (Pq == 1) {
            acc = 0.f;
            for (int p = 0; p < P; ++p) acc += g * tmask[bt * P + p];
        } else {
            acc = g * tmask[bt * P + q];
        }
        gopol[i] = acc;
    } else if (gval && i < npol + BT * Pq) {
        const int64_t btq = i - npol;
        const int64_t bt = btq / Pq;
        const int q = (int)(btq - bt * Pq);
        float acc;
        if (Pq == 1) {
            acc = 0.f;
            for (int p = 0; p < P; ++p) acc += gval[bt * P + p] * omask[bt * P + p];
        } else {
            acc = gval[bt * P + q] * omask[bt * P + q];
        }
        goval[btq] = acc;
    }
}

}  // namespace

extern "C" {

int64_t hrl_loss_workspace_bytes(int64_t B, int64_t T, int64_t P, int64_t Pp) {
    LossDims d;
    if (!dims_ok(B, T, P, Pp, 1, d)) return -1;
    return ws_bytes(d);
}

int hrl_loss_forward(const float *tpol, const float *bpol, const int64_t *action, int64_t B, int64_t T, int64_t P,
                     int64_t Pp, int64_t A, const float *emask, const float *tmask, const float *omask,
                     const float *progress, const float *value, const float *outcome, const float *ret_out,
                     const float *ret, const float *reward, int value_target, int policy_target, int symmetrize,
                     double lmb, double gamma, double ent_coef, double ent_decay, void *workspace,
                     int64_t workspace_bytes, float *losses, void *stream) {
    LossDims d;
    if (!dims_ok(B, T, P, Pp, A, d)) return HRL_EINVAL;
    if (!tpol || !bpol || !action || !emask || !tmask || !omask || !progress || !losses || !workspace)
        return HRL_EINVAL;
    if (value && !outcome) return HRL_EINVAL;
    if (ret_out && (!ret || !reward)) return HRL_EINVAL;
    if (symmetrize && P != 2) return HRL_EINVAL;
    if (value_target < HRL_ALG_MC || value_target > HRL_ALG_VTRACE || policy_target < HRL_ALG_MC ||
        policy_target > HRL_ALG_VTRACE)
        return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(d)) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Ws w = carve(workspace, d);
    FwdArgs a{tpol, bpol, action, emask, tmask, omask, progress, value, outcome, ret_out, ret, reward,
              value_target == HRL_ALG_MC, symmetrize, (float)ent_coef, (float)ent_decay};
    const dim3 grid(w.nblocks), block(kThreads);
    hipLaunchKernelGGL(loss_prep_kernel, grid, block, 0, s, a, d, w);
    int rc = status();
    if (rc) return rc;
    const int64_t rho_div = P / Pp;
    const bool mc = value_target == HRL_ALG_MC;
    if (value) {   // value head: returns = outcome (T-extent 1), no rewards, gamma = 1 (train.py:245)
        rc = hrl_compute_targets_fused(value_target, policy_target, w.vprep, outcome, nullptr, w.crho, w.crho, B, T,
                                       P, 1, Pp, rho_div, lmb, 1.0, mc ? nullptr : w.tv, w.advv, stream);
        if (rc) return rc;
    }
    if (ret_out) {  // return head: returns = batch['return'], rewards, gamma (train.py:246)
        rc = hrl_compute_targets_fused(value_target, policy_target, ret_out, ret, reward, w.crho, w.crho, B, T, P, T,
                                       Pp, rho_div, lmb, gamma, mc ? nullptr : w.tr, w.advr, stream);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(loss_terms_kernel, grid, block, 0, s, a, d, w, ret_out != nullptr ? 1 : 0);
    rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), block, 0, s, w, (float)ent_coef, losses);
    return status();
}

int hrl_loss_backward(const float *tpol, const int64_t *action, int64_t B, int64_t T, int64_t P, int64_t Pp,
                      int64_t A, const float *emask, const float *tmask, const float *omask, const float *progress,
                      const float *value, const float *ret_out, double ent_coef, double ent_decay,
                      const void *workspace, int64_t workspace_bytes, const float *dlosses, float *g_tpol,
                      float *g_value, float *g_ret, void *stream) {
    LossDims d;
    if (!dims_ok(B, T, P, Pp, A, d)) return HRL_EINVAL;
    if (!tpol || !action || !emask || !tmask || !omask || !progress || !dlosses || !g_tpol || !workspace)
        return HRL_EINVAL;
    if ((g_value && !value) || (g_ret && !ret_out)) return HRL_EINVAL;
    if (workspace_bytes < ws_bytes(d)) return HRL_EINVAL;
    Ws w = carve(const_cast<void *>(workspace), d);
    BwdArgs a{tpol, action, emask, tmask, omask, progress, value, ret_out, dlosses, g_tpol, g_value, g_ret,
              (float)ent_coef, (float)ent_decay};
    hipLaunchKernelGGL(loss_backward_kernel, dim3(w.nblocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream), a,
                       d, w);
    return status();
}

int hrl_output_mask_forward(const float *opol, const float *oval, const float *tmask, const float *omask,
                            const float *amask, int64_t BT, int64_t P, int64_t Pq, int64_t A, float *pol,
                            float *val, void *stream) {
    if (BT < 1 || P < 1 || P > 64 || A < 1 || A > (1 << 20) || (Pq != 1 && Pq != P)) return HRL_EINVAL;
    if (!opol || !tmask || !amask || !pol || (oval && (!omask || !val))) return HRL_EINVAL;
    const int64_t n = BT * A + (oval ? BT * P : 0);
    if (n > ((int64_t)1 << 40)) return HRL_EINVAL;
    hipLaunchKernelGGL(out_mask_fwd_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), opol, oval, tmask, omask, amask, BT, (int)P, (int)Pq,
                       (int)A, pol, val);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

int hrl_output_mask_backward(const float *gpol, const float *gval, const float *tmask, const float *omask,
                             int64_t BT, int64_t P, int64_t Pq, int64_t A, float *gopol, float *goval,
                             void *stream) {
    if (BT < 1 || P < 1 || P > 64 || A < 1 || A > (1 << 20) || (Pq != 1 && Pq != P)) return HRL_EINVAL;
    if (!gpol || !tmask || !gopol || (gval && (!omask || !goval))) return HRL_EINVAL;
    const int64_t n = BT * Pq * A + (gval ? BT * Pq : 0);
    if (n > ((int64_t)1 << 40)) return HRL_EINVAL;
    hipLaunchKernelGGL(out_mask_bwd_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), gpol, gval, tmask, omask, BT, (int)P, (int)Pq, (int)A,
                       gopol, goval);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

}  // extern "C"
