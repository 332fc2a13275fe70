// hrl_loss.hip — fused learner loss for HandyRL on MI355X (gfx950).
//
// One learner step's loss after the network forward, train.py:220-258 and
// compose_losses train.py:188-215, as two launches instead of ~60 small
// PyTorch kernels (log_softmax x2, gather x2, exp, clamp x2, stack/neg/div
// for the zero-sum symmetrisation, 2-4 target scans, the advantage
// composition, five masked reductions, Categorical entropy, ...):
//
//   fused  (one wave per G trajectories, LDS tiles of 32 time steps): the IS
//          ratios, the target policy's entropy, the value preparation, the
//          value- and return-head scans of hrl_scan.h (value_target targets +
//          policy_target advantages), the turn advantages and the five loss
//          sums and dcnt as fp64 per-wave partials
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

#include <type_traits>

#include "../../include/hrl_loss.h"
#include "../../include/hrl_targets.h"
#include "hrl_scan.h"

namespace {

using hrl_scan::Coef;

HRL_STAMP_DECL

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
    int nblocks;   // 256-thread blocks over B*T (backward)
    int nparts;    // waves of the fused forward, one fp64 partial set each
};

int fused_G(int64_t B, int P);

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
    const int G = fused_G(d.B, d.P);
    w.nparts = (int)((d.B + G - 1) / G);
    return w;
}

int64_t ws_bytes(const LossDims &d) {
    const int64_t floats = 3 * d.BT * d.Pp + 5 * d.BT * d.P + d.BT;
    const int G = fused_G(d.B, d.P);
    const int64_t nparts = (d.B + G - 1) / G;
    return align16(floats * 4) + nparts * kTerms * 8 + 64;
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
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

// One policy row (train.py:224-231): lt = log_softmax(target)[act] * emask, the clipped IS ratio
// clamp(exp(lt - lb), 0, 1) and the target policy's entropy.  AK > 0: the row has exactly AK actions
// (compile time) and sits in registers, so its loads issue at once and no per-action guard exists;
// AK = 0: any A, one action per loop trip.  Same float operations in the same order either way.
template <int AK>
__device__ __forceinline__ void policy_row(const float *zt, const float *zb, int A, int act, float em, float &lt,
                                           float &crho, float &ent) {
    float mt, st, mb, sb;
    float h = 0.f;
    if constexpr (AK > 0) {
        float xt[AK], xb[AK], et[AK];
#pragma unroll
        for (int q = 0; q < AK; ++q) {
            xt[q] = zt[q];
            xb[q] = zb[q];
        }
        mt = xt[0];
        mb = xb[0];
#pragma unroll
        for (int q = 1; q < AK; ++q) {
            mt = fmaxf(mt, xt[q]);
            mb = fmaxf(mb, xb[q]);
        }
        st = 0.f;
        sb = 0.f;
        float zta = xt[0], zba = xb[0];
#pragma unroll
        for (int q = 0; q < AK; ++q) {
            et[q] = expf(xt[q] - mt);
            st += et[q];
            sb += expf(xb[q] - mb);
            zta = q == act ? xt[q] : zta;
            zba = q == act ? xb[q] : zba;
        }
        lt = ((zta - mt) - logf(st)) * em;                                  // train.py:224-225
        const float lb = ((zba - mb) - logf(sb)) * em;
        const float lse = mt + logf(st);
#pragma unroll
        for (int q = 0; q < AK; ++q) h += (xt[q] - lse) * (et[q] / st);
        crho = fminf(fmaxf(expf(lt - lb), 0.f), 1.f);                        // train.py:228-231
    } else {
        row_stats(zt, A, mt, st);
        row_stats(zb, A, mb, sb);
        // F.log_softmax(x)[act] = (x - max) - log(sum exp(x - max))      (train.py:224-225)
        lt = ((zt[act] - mt) - logf(st)) * em;
        const float lb = ((zb[act] - mb) - logf(sb)) * em;
        // Categorical(logits).entropy(): logits normalised by logsumexp = m + log(s)
        const float lse = mt + logf(st);
        for (int q = 0; q < A; ++q) h += (zt[q] - lse) * (expf(zt[q] - mt) / st);
        crho = fminf(fmaxf(expf(lt - lb), 0.f), 1.f);                        // train.py:228-231
    }
    ent = -h;
}

// action counts with a register-resident specialisation of the fused loss (TicTacToe 9, Hungry Geese 4);
// any other A runs the wave form below

// fixed xor butterflies over the 64 lanes: every lane ends with the same, order-fixed result
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One policy row with the wave's lanes over its actions (A = 214 for Geister): coalesced loads and
// fixed-order butterfly reductions instead of one lane walking the row.  The same quantities as
// policy_row; the sums run in another (fixed) order.
__device__ __forceinline__ void policy_row_wave(const float *zt, const float *zb, int A, int act, float em, int lane,
                                                float &lt, float &crho, float &ent) {
    float mt = -INFINITY, mb = -INFINITY;
    for (int q = lane; q < A; q += 64) {
        mt = fmaxf(mt, zt[q]);
        mb = fmaxf(mb, zb[q]);
    }
    mt = wave_max(mt);
    mb = wave_max(mb);
    float st = 0.f, sb = 0.f;
    for (int q = lane; q < A; q += 64) {
        st += expf(zt[q] - mt);
        sb += expf(zb[q] - mb);
    }
    st = wave_sum(st);
    sb = wave_sum(sb);
    lt = ((zt[act] - mt) - logf(st)) * em;                                  // train.py:224-225
    const float lb = ((zb[act] - mb) - logf(sb)) * em;
    const float lse = mt + logf(st);
    float h = 0.f;
    for (int q = lane; q < A; q += 64) h += (zt[q] - lse) * (expf(zt[q] - mt) / st);
    ent = -wave_sum(h);
    crho = fminf(fmaxf(expf(lt - lb), 0.f), 1.f);                            // train.py:228-231
}

// ---- fused forward: prep + both target scans + loss terms, one wave per G trajectories ------------
//
// A wave owns G consecutive trajectories and walks them in LDS tiles of up to kLossTile time steps,
// top tile first (the scans run backwards in time).  Per tile:
//   1. prep (lanes over the tile's (g, t, pp) rows): log-softmax + gather of both policies, the IS
//      ratio and its clip, the target policy's entropy (train.py:224-231); the zero-sum value
//      preparation with outcome padding (train.py:234-239) and the return head's inputs, all into
//      LDS tiles laid out as the scans read them;
//   2. the value- and return-head recurrences (hrl_scan.h), lane (g, c) per column, straight from
//      and back into LDS: the 4-5 MB round trip of the former prep -> scan -> terms launches is gone;
//   3. terms (lanes over (g, t)): the turn advantages and the five loss sums and dcnt, accumulated
//      in fp64 per lane (train.py:202-213, 248-256); turn, the targets and the entropy go to the
//      workspace for the backward.
// The wave folds its partials in a fixed shuffle tree, so the sums are deterministic.
constexpr int kLossTile = 32;   // time steps per LDS tile (two register-resident recurrence chunks)

struct FusedArgs {
    FwdArgs a;
    LossDims d;
    Ws w;
    Coef kv;   // value head: gamma = 1 (train.py:245)
    Coef kr;   // return head: gamma (train.py:246)
    int G;     // trajectories per wave
};

// trajectories per wave: G*P <= 64 scan lanes, at most 8 (so a tile's prep/terms rows stay a few
// per lane), fewer at small B so the launch still has ~2048 waves: two per SIMD, so one wave's
// loads overlap the other's recurrence (B=4096: G=2, one prep row per lane at T=32)
int fused_G(int64_t B, int P) {
    const int gmax = min(8, hrl_scan::kWave / P);
    int g = 1;
    while (g * 2 <= gmax && B / (g * 2) >= 2048) g *= 2;
    return g;
}

size_t fused_lds_bytes(const LossDims &d, int G, bool hv, bool hr, bool vt_mc, bool pt_mc) {
    const int TT = d.T < kLossTile ? (int)d.T : kLossTile;
    const size_t vt = (size_t)G * hrl_scan::padded_row(TT * d.P, d.P);
    const size_t rt = (size_t)G * hrl_scan::padded_row(TT * d.Pp, 1);
    const int ntiles = (hv ? 2 + (vt_mc ? 0 : 1) : 0) + (hr ? 3 + (pt_mc ? 1 : 0) + (vt_mc ? 0 : 1) : 0);
    return sizeof(float) * (3 * rt + ntiles * vt);
}

template <int VT, int PT, bool HV, bool HR, int AK>
__global__ __launch_bounds__(hrl_scan::kWave) void loss_fused_kernel(FusedArgs f) {
    using namespace hrl_scan;
    constexpr int TGT = VT == HRL_ALG_MC ? kNone : VT;            // MC targets are the returns as given
    constexpr bool kRho = (TGT == HRL_ALG_VTRACE) || (PT == HRL_ALG_VTRACE);
    constexpr bool kRetT = PT == HRL_ALG_MC;                      // return-head MC reads ret at every t
    extern __shared__ float lds[];
    const FwdArgs &a = f.a;
    const LossDims &d = f.d;
    const Ws &w = f.w;
    const int lane = threadIdx.x;
    const int P = d.P, Pp = d.Pp, A = AK > 0 ? AK : d.A, T = (int)d.T;
    const int C = P, rhoC = Pp, rhoDiv = P / Pp;
    const int G = f.G;
    const int TT = T < kLossTile ? T : kLossTile;
    const int Lpv = padded_row(TT * C, C), Lpr = padded_row(TT * rhoC, 1);
    const int64_t b0 = (int64_t)blockIdx.x * G;
    const int ntraj = (int)min<int64_t>(G, d.B - b0);

    const int vt = G * Lpv, rt = G * Lpr;
    float *p = lds;
    float *t_rho = p; p += rt;
    float *t_lt = p; p += rt;
    float *t_ent = p; p += rt;
    float *t_v = p; p += HV ? vt : 0;
    float *t_tv = p; p += (HV && TGT != kNone) ? vt : 0;
    float *t_advv = p; p += HV ? vt : 0;
    float *t_rv = p; p += HR ? vt : 0;
    float *t_rr = p; p += HR ? vt : 0;
    float *t_rret = p; p += (HR && kRetT) ? vt : 0;
    float *t_tr = p; p += (HR && TGT != kNone) ? vt : 0;
    float *t_advr = p;

    const int g = lane / C;                 // scan lane (g, c)
    const int c = lane - g * C;
    const bool active = lane < G * C && g < ntraj;
    float boot_v = 0.f, boot_r = 0.f;
    if (active) {
        if constexpr (HV) boot_v = a.outcome[(b0 + g) * P + c];
        if constexpr (HR) boot_r = a.ret[((b0 + g) * d.T + (T - 1)) * P + c];
    }
    Carry sv{0.f, 0.f, 0.f, 0.f, 0.f}, sr{0.f, 0.f, 0.f, 0.f, 0.f};
    double acc[kTerms] = {0, 0, 0, 0, 0, 0};
    HRL_STAMP_WALL(14);
    HRL_STAMP(0);

    const int ntile = (T + kLossTile - 1) / kLossTile;
    for (int tile = ntile - 1; tile >= 0; --tile) {
        const int t0 = tile * kLossTile;
        const int tc = min(kLossTile, T - t0);

        // 1. prep: policy rows (g, t, pp)
        if constexpr (AK == 0) {   // the wave on one row at a time, lanes over its actions
            const int per = tc * Pp;
            for (int e = 0; e < ntraj * per; ++e) {
                const int gg = e / per;
                const int rem = e - gg * per;
                const int tt = rem / Pp;
                const int pp = rem - tt * Pp;
                const int64_t bt = (b0 + gg) * d.T + t0 + tt;
                const int64_t row = bt * Pp + pp;
                float lt, crho, ent;
                policy_row_wave(a.tpol + row * A, a.bpol + row * A, A, (int)a.action[row], a.emask[bt], lane, lt,
                                crho, ent);
                if (lane == 0) {
                    const int slot = gg * Lpr + tt * rhoC + pp;
                    t_rho[slot] = crho;
                    t_lt[slot] = lt;
                    t_ent[slot] = ent;
                }
            }
        } else {
            const int per = tc * Pp;
            const float inv_per = 1.0f / (float)per, inv_pp = 1.0f / (float)Pp;
            for (int e = lane; e < ntraj * per; e += kWave) {
                const int gg = fdiv(e, inv_per);
                const int rem = e - gg * per;
                const int tt = fdiv(rem, inv_pp);
                const int pp = rem - tt * Pp;
                const int64_t bt = (b0 + gg) * d.T + t0 + tt;
                const int64_t row = bt * Pp + pp;
                const float em = a.emask[bt];
                const int64_t act = a.action[row];
                float lt, crho, ent;
                policy_row<AK>(a.tpol + row * A, a.bpol + row * A, A, (int)act, em, lt, crho, ent);
                const int slot = gg * Lpr + tt * rhoC + pp;
                t_rho[slot] = crho;
                t_lt[slot] = lt;
                t_ent[slot] = ent;
            }
        }
        HRL_STAMP(1);
        // 1b. value-shaped inputs (g, t, p): prepared values (train.py:234-239), return-head inputs
        if constexpr (HV || HR) {
            const int per = tc * P;
            const float inv_per = 1.0f / (float)per, inv_p = 1.0f / (float)P;
            for (int e = lane; e < ntraj * per; e += kWave) {
                const int gg = fdiv(e, inv_per);
                const int rem = e - gg * per;
                const int tt = fdiv(rem, inv_p);
                const int q = rem - tt * P;
                const int64_t b = b0 + gg;
                const int64_t bt = b * d.T + t0 + tt;
                const int64_t i = bt * P + q;
                const int slot = gg * Lpv + tt * C + q;
                if constexpr (HV) {
                    const float em = a.emask[bt];
                    const float *v = a.value + bt * P;
                    float vp = v[q];
                    if (a.symmetrize) {   // two-player zero-sum: (v - swap(v)) / (sum omask + 1e-8)
                        const float *om = a.omask + bt * P;
                        vp = (v[q] + (-v[1 - q])) / ((om[0] + om[1]) + 1e-8f);
                    }
                    t_v[slot] = vp * em + a.outcome[b * P + q] * (1.f - em);
                }
                if constexpr (HR) {
                    t_rv[slot] = a.ret_out[i];
                    t_rr[slot] = a.reward[i];
                    if constexpr (kRetT) t_rret[slot] = a.ret[i];
                }
            }
        }
        __syncthreads();
        HRL_STAMP(2);

        // 2. the scans: value head (returns = outcome, no rewards, gamma 1) and return head
        if (active) {
            const int nsub = (tc + kTChunk - 1) / kTChunk;
            for (int sc = nsub - 1; sc >= 0; --sc) {
                const int tcs = min(kTChunk, tc - sc * kTChunk);
                const bool top = tile == ntile - 1 && sc == nsub - 1;
                const int vofs = g * Lpv + sc * kTChunk * C + c;
                const int rofs = g * Lpr + sc * kTChunk * rhoC + c / rhoDiv;
                auto run = [&](auto full, auto topc) __attribute__((always_inline)) {
                    constexpr bool F = decltype(full)::value, TOP = decltype(topc)::value;
                    if constexpr (HV)
                        recur_chunk<TGT, PT, false, kRho, false, F, TOP, true>(sv, boot_v, f.kv, tcs, C, rhoC, t_v,
                                                                         nullptr, nullptr, t_rho, t_rho, vofs,
                                                                         rofs, t_tv, t_advv);
                    if constexpr (HR)
                        recur_chunk<TGT, PT, true, kRho, kRetT, F, TOP>(sr, boot_r, f.kr, tcs, C, rhoC, t_rv,
                                                                        t_rr, t_rret, t_rho, t_rho, vofs, rofs,
                                                                        t_tr, t_advr);
                };
                // only the top chunk of the top tile can be partial (tiles and chunks are cut from t = 0)
                if (!top) run(std::true_type{}, std::false_type{});
                else if (tcs == kTChunk) run(std::true_type{}, std::true_type{});
                else run(std::false_type{}, std::true_type{});
            }
        }
        __syncthreads();
        HRL_STAMP(3);

        // 3. terms: turn advantages and the loss sums (train.py:202-213, 248-256)
        {
            const float inv_tc = 1.0f / (float)tc;
            for (int e = lane; e < ntraj * tc; e += kWave) {
                const int gg = fdiv(e, inv_tc);
                const int tt = e - gg * tc;
                const int64_t b = b0 + gg;
                const int64_t bt = b * d.T + t0 + tt;
                const float *tm = a.tmask + bt * P;
                const float *om = a.omask + bt * P;
                const int vrow = gg * Lpv + tt * C, rrow = gg * Lpr + tt * rhoC;
                // total_advantages = clipped_rhos * (adv_value + adv_return); turn sum under turn_mask
                float turn = 0.f;
                for (int q = 0; q < P; ++q) {
                    const int pp = Pp == 1 ? 0 : q;
                    float s = 0.f;
                    if constexpr (HV) s = s + t_advv[vrow + q];
                    if constexpr (HR) s = s + t_advr[vrow + q];
                    turn += (t_rho[rrow + pp] * s) * tm[q];
                }
                w.turn[bt] = turn;
                for (int pp = 0; pp < Pp; ++pp) {
                    acc[0] += (double)(-t_lt[rrow + pp] * turn);
                    w.ent[bt * Pp + pp] = t_ent[rrow + pp];
                }
                const float prog = 1.f - a.progress[bt] * (1.f - a.ent_decay);
                for (int q = 0; q < P; ++q) {
                    const int pp = Pp == 1 ? 0 : q;
                    const int64_t i = bt * P + q;
                    if constexpr (HV) {
                        const float tv = TGT == kNone ? a.outcome[b * P + q] : t_tv[vrow + q];
                        const float e2 = a.value[i] - tv;
                        acc[1] += (double)((e2 * e2) * om[q]);
                        w.tv[i] = tv;
                    }
                    if constexpr (HR) {
                        const float tr = TGT == kNone ? a.ret[i] : t_tr[vrow + q];
                        const float x = a.ret_out[i] - tr;
                        const float ax = fabsf(x);
                        const float l = ax < 1.f ? 0.5f * x * x : ax - 0.5f;
                        acc[2] += (double)(l * om[q]);
                        w.tr[i] = tr;
                    }
                    const float ent = t_ent[rrow + pp] * tm[q];
                    acc[3] += (double)ent;
                    acc[4] += (double)(ent * prog);
                    acc[5] += (double)tm[q];
                }
            }
        }
        __syncthreads();   // the next tile's prep rewrites the tiles
        HRL_STAMP(4);
    }

    // 4. fixed-order fold of the wave's partials (shuffle tree), lane 0 writes them
#pragma unroll
    for (int k = 0; k < kTerms; ++k) {
        double v = acc[k];
        for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_down(v, off, kWave);
        acc[k] = v;
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kTerms; ++k) w.part[(int64_t)blockIdx.x * kTerms + k] = acc[k];
    }
    HRL_STAMP(5);
    HRL_STAMP_WALL(15);
}

template <int VT, int PT, bool HV, bool HR>
int launch_fused(const FusedArgs &f, hipStream_t s) {
    const size_t lds = fused_lds_bytes(f.d, f.G, HV, HR, VT == HRL_ALG_MC, PT == HRL_ALG_MC);
    const dim3 grid((unsigned)f.w.nparts), block(hrl_scan::kWave);
    if (f.d.A == 9) hipLaunchKernelGGL((loss_fused_kernel<VT, PT, HV, HR, 9>), grid, block, lds, s, f);
    else if (f.d.A == 4) hipLaunchKernelGGL((loss_fused_kernel<VT, PT, HV, HR, 4>), grid, block, lds, s, f);
    else hipLaunchKernelGGL((loss_fused_kernel<VT, PT, HV, HR, 0>), grid, block, lds, s, f);
    return status();
}

template <int VT, int PT>
int launch_fused_heads(const FusedArgs &f, bool hv, bool hr, hipStream_t s) {
    if (hv) return hr ? launch_fused<VT, PT, true, true>(f, s) : launch_fused<VT, PT, true, false>(f, s);
    return hr ? launch_fused<VT, PT, false, true>(f, s) : launch_fused<VT, PT, false, false>(f, s);
}

template <int VT>
int launch_fused_pt(int pt, const FusedArgs &f, bool hv, bool hr, hipStream_t s) {
    switch (pt) {
        case HRL_ALG_MC: return launch_fused_heads<VT, HRL_ALG_MC>(f, hv, hr, s);
        case HRL_ALG_TD: return launch_fused_heads<VT, HRL_ALG_TD>(f, hv, hr, s);
        case HRL_ALG_UPGO: return launch_fused_heads<VT, HRL_ALG_UPGO>(f, hv, hr, s);
        default: return launch_fused_heads<VT, HRL_ALG_VTRACE>(f, hv, hr, s);
    }
}

int launch_fused_all(int vt, int pt, const FusedArgs &f, bool hv, bool hr, hipStream_t s) {
    switch (vt) {
        case HRL_ALG_MC: return launch_fused_pt<HRL_ALG_MC>(pt, f, hv, hr, s);
        case HRL_ALG_TD: return launch_fused_pt<HRL_ALG_TD>(pt, f, hv, hr, s);
        case HRL_ALG_UPGO: return launch_fused_pt<HRL_ALG_UPGO>(pt, f, hv, hr, s);
        default: return launch_fused_pt<HRL_ALG_VTRACE>(pt, f, hv, hr, s);
    }
}

// ---- reduce: fixed-order fold of the block partials -> p, v, r, ent, total, dcnt ---------------
__global__ __launch_bounds__(kThreads) void loss_reduce_kernel(Ws w, float ent_coef, float *losses) {
    __shared__ double red[kTerms][kThreads];
    double acc[kTerms] = {0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < w.nparts; i += kThreads) {
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

template <int AK>
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
        const float h = w.ent[row];
        const int64_t act = a.action[row];
        if constexpr (AK > 0) {   // the row in registers: its loads issue at once (same float operations)
            float x[AK];
#pragma unroll
            for (int q = 0; q < AK; ++q) x[q] = z[q];
            float m = x[0];
#pragma unroll
            for (int q = 1; q < AK; ++q) m = fmaxf(m, x[q]);
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < AK; ++q) s += expf(x[q] - m);
            const float lse = m + logf(s);
#pragma unroll
            for (int q = 0; q < AK; ++q) {
                const float pq = expf(x[q] - m) / s;
                const float la = x[q] - lse;
                const float onehot = (q == act) ? 1.f : 0.f;
                g[q] = cp * (onehot - pq) + ce * (-pq * (la + h));    // dH/dz = -p (log p + H)
            }
        } else {
            float m, s;
            row_stats(z, d.A, m, s);
            const float lse = m + logf(s);
            for (int q = 0; q < d.A; ++q) {
                const float pq = expf(z[q] - m) / s;
                const float la = z[q] - lse;
                const float onehot = (q == act) ? 1.f : 0.f;
                g[q] = cp * (onehot - pq) + ce * (-pq * (la + h));    // dH/dz = -p (log p + H)
            }
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

// any A (Geister's 214): a wave per (b, t), lanes over the actions of each policy row, then over the
// players for the value / return gradients; the same closed-form expressions as loss_backward_kernel
__global__ __launch_bounds__(kThreads) void loss_backward_wave_kernel(BwdArgs a, LossDims d, Ws w) {
    const int lane = threadIdx.x & 63;
    const int64_t bt = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (bt >= d.BT) return;
    const float dp = a.dl[0], dv = a.dl[1], dr = a.dl[2], de = a.dl[3], dt = a.dl[4];
    const float *tm = a.tmask + bt * d.P;
    const float *om = a.omask + bt * d.P;
    const float em = a.emask[bt];
    const float prog = 1.f - a.progress[bt] * (1.f - a.ent_decay);
    const float cp = -(dp + dt) * w.turn[bt] * em;
    for (int pp = 0; pp < d.Pp; ++pp) {
        const int64_t row = bt * d.Pp + pp;
        const float *z = a.tpol + row * d.A;
        float *g = a.g_tpol + row * d.A;
        float wsum = 0.f, wdec = 0.f;
        for (int p = 0; p < d.P; ++p) {
            if (d.Pp == 1 || p == pp) {
                wsum += tm[p];
                wdec += tm[p] * prog;
            }
        }
        const float ce = de * wsum + dt * (-a.ent_coef) * wdec;
        const float h = w.ent[row];
        const int64_t act = a.action[row];
        float m = -INFINITY;
        for (int q = lane; q < d.A; q += 64) m = fmaxf(m, z[q]);
        m = wave_max(m);
        float s = 0.f;
        for (int q = lane; q < d.A; q += 64) s += expf(z[q] - m);
        s = wave_sum(s);
        const float lse = m + logf(s);
        for (int q = lane; q < d.A; q += 64) {
            const float pq = expf(z[q] - m) / s;
            const float la = z[q] - lse;
            const float onehot = (q == act) ? 1.f : 0.f;
            g[q] = cp * (onehot - pq) + ce * (-pq * (la + h));    // dH/dz = -p (log p + H)
        }
    }
    for (int p = lane; p < d.P; p += 64) {
        const int64_t i = bt * d.P + p;
        if (a.g_value) a.g_value[i] = (dv + dt) * (a.value[i] - w.tv[i]) * om[p];
        if (a.g_ret) {
            const float x = a.ret_out[i] - w.tr[i];
            const float sl = fminf(fmaxf(x, -1.f), 1.f);              // smooth_l1' (beta = 1)
            a.g_ret[i] = (dr + dt) * sl * om[p];
        }
    }
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
// I: the index type -- 32-bit unsigned whenever every index fits (a 64-bit division by the runtime A / Pq is a
// long software sequence per element; the results are the same)
template <typename I>
__global__ __launch_bounds__(kThreads) void out_mask_fwd_kernel(const float *__restrict__ opol,
                                                                const float *__restrict__ oval,
                                                                const float *__restrict__ tmask,
                                                                const float *__restrict__ omask,
                                                                const float *__restrict__ amask, I BT, int P,
                                                                int Pq, int A, float *__restrict__ pol,
                                                                float *__restrict__ val) {
    const I i = (I)blockIdx.x * kThreads + threadIdx.x;
    const I npol = BT * (I)A;
    if (i < npol) {
        const I bt = i / (I)A;
        const int a = (int)(i - bt * (I)A);
        float acc = 0.f;
        for (int p = 0; p < P; ++p)
            acc += opol[(bt * (I)Pq + (I)(Pq == 1 ? 0 : p)) * (I)A + (I)a] * tmask[bt * (I)P + (I)p];
        pol[i] = acc - amask[i];
    } else if (oval && i < npol + BT * (I)P) {
        const I j = i - npol;
        const I bt = j / (I)P;
        const int p = (int)(j - bt * (I)P);
        val[j] = oval[bt * (I)Pq + (I)(Pq == 1 ? 0 : p)] * omask[j];
    }
}

template <typename I>
__global__ __launch_bounds__(kThreads) void out_mask_bwd_kernel(const float *__restrict__ gpol,
                                                                const float *__restrict__ gval,
                                                                const float *__restrict__ tmask,
                                                                const float *__restrict__ omask, I BT, int P,
                                                                int Pq, int A, float *__restrict__ gopol,
                                                                float *__restrict__ goval) {
    const I i = (I)blockIdx.x * kThreads + threadIdx.x;
    const I npol = BT * (I)Pq * (I)A;
    if (i < npol) {
        const I btq = i / (I)A;
        const int a = (int)(i - btq * (I)A);
        const I bt = btq / (I)Pq;
        const int q = (int)(btq - bt * (I)Pq);
        const float g = gpol[bt * (I)A + (I)a];
        float acc;
        if (Pq == 1) {
            acc = 0.f;
            for (int p = 0; p < P; ++p) acc += g * tmask[bt * (I)P + (I)p];
        } else {
            acc = g * tmask[bt * (I)P + (I)q];
        }
        gopol[i] = acc;
    } else if (gval && i < npol + BT * (I)Pq) {
        const I btq = i - npol;
        const I bt = btq / (I)Pq;
        const int q = (int)(btq - bt * (I)Pq);
        float acc;
        if (Pq == 1) {
            acc = 0.f;
            for (int p = 0; p < P; ++p) acc += gval[bt * (I)P + (I)p] * omask[bt * (I)P + (I)p];
        } else {
            acc = gval[bt * (I)P + (I)q] * omask[bt * (I)P + (I)q];
        }
        goval[btq] = acc;
    }
}

}  // namespace

extern "C" {

#ifdef HRL_STAMPS
int hrl_debug_set_stamps_loss(void *buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hrl_stamps), &buf, sizeof(buf)); }
#endif

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
    FusedArgs f{a, d, w, hrl_scan::make_coef(lmb, 1.0), hrl_scan::make_coef(lmb, gamma), fused_G(B, (int)P)};
    int rc = launch_fused_all(value_target, policy_target, f, value != nullptr, ret_out != nullptr, s);
    if (rc) return rc;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(kThreads), 0, s, w, (float)ent_coef, losses);
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
    const dim3 grid(w.nblocks), block(kThreads);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (A == 9) hipLaunchKernelGGL(loss_backward_kernel<9>, grid, block, 0, s, a, d, w);
    else if (A == 4) hipLaunchKernelGGL(loss_backward_kernel<4>, grid, block, 0, s, a, d, w);
    else
        hipLaunchKernelGGL(loss_backward_wave_kernel, dim3((unsigned)((d.BT + kThreads / 64 - 1) / (kThreads / 64))),
                           block, 0, s, a, d, w);
    return status();
}

int hrl_output_mask_forward(const float *opol, const float *oval, const float *tmask, const float *omask,
                            const float *amask, int64_t BT, int64_t P, int64_t Pq, int64_t A, float *pol,
                            float *val, void *stream) {
    if (BT < 1 || P < 1 || P > 64 || A < 1 || A > (1 << 20) || (Pq != 1 && Pq != P)) return HRL_EINVAL;
    if (!opol || !tmask || !amask || !pol || (oval && (!omask || !val))) return HRL_EINVAL;
    const int64_t n = BT * A + (oval ? BT * P : 0);
    if (n > ((int64_t)1 << 40)) return HRL_EINVAL;
    const dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    if (n + kThreads < ((int64_t)1 << 31))
        hipLaunchKernelGGL(out_mask_fwd_kernel<uint32_t>, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                           opol, oval, tmask, omask, amask, (uint32_t)BT, (int)P, (int)Pq, (int)A, pol, val);
    else
        hipLaunchKernelGGL(out_mask_fwd_kernel<int64_t>, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                           opol, oval, tmask, omask, amask, BT, (int)P, (int)Pq, (int)A, pol, val);
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
    const dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    if (n + kThreads < ((int64_t)1 << 31))
        hipLaunchKernelGGL(out_mask_bwd_kernel<uint32_t>, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                           gpol, gval, tmask, omask, (uint32_t)BT, (int)P, (int)Pq, (int)A, gopol, goval);
    else
        hipLaunchKernelGGL(out_mask_bwd_kernel<int64_t>, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                           gpol, gval, tmask, omask, BT, (int)P, (int)Pq, (int)A, gopol, goval);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

}  // extern "C"
