// hrl_scan.h — the return-target recurrences of handyrl/losses.py:16-58, shared by the
// standalone scan kernels (hrl_targets.hip) and the fused learner loss (hrl_loss.hip).
//
// Each recurrence performs the reference's float32 operations in the reference's
// order with the same float32-rounded coefficients (sources are built with
// -ffp-contract=off), so results are bit-identical to the reference CPU learner.
#ifndef HRL_SCAN_H
#define HRL_SCAN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_targets.h"

#include "hrl_stamps.h"

namespace hrl_scan {

constexpr int kWave = 64;
constexpr int kTChunk = 16;   // time steps per register-resident recurrence pass
constexpr int kNone = -1;     // "no target output"

struct Coef {
    float a;   // (float)(1 - lmb)
    float l;   // (float)lmb
    float g;   // (float)gamma
    float gl;  // (float)(gamma * lmb)
};

inline Coef make_coef(double lmb, double gamma) {
    Coef k;
    k.a = (float)(1.0 - lmb);
    k.l = (float)lmb;
    k.g = (float)gamma;
    k.gl = (float)(gamma * lmb);
    return k;
}

// torch.max(a, b) on two tensors propagates NaN (losses.py:36).  Written as selects
// (v_cndmask), not early returns: the branches the early-return form compiled to
// (two exec-mask regions per time step) sat on the scan's serial chain.  x is the
// carried v[t+1], known a step ahead, so its NaN test is off the chain; a NaN y fails
// `x > y` and is selected as is.  Same result, payloads included, as testing both.
__device__ __forceinline__ float max_nan(float x, float y) {
    const float m = x > y ? x : y;
    return (x != x) ? x : m;
}

// floor(e / d) for 0 <= e < 2^20 and d >= 1, given inv = 1.0f / d: the exact
// quotient of (e + 0.5) / d sits at least 0.5/d away from an integer, far more
// than the float32 rounding error at these magnitudes, so no integer divide.
__device__ __forceinline__ int fdiv(int e, float inv) {
    return (int)(((float)e + 0.5f) * inv);
}

// LDS row stride for rows of L floats read column-wise by lanes (g, c), c < Cx:
// the smallest Lp >= L with Lp == Cx (mod 32) makes g*Lp + c distinct modulo
// 32 over each 32-lane half when Cx divides 32 (conflict-free ds_read_b32).
__host__ __device__ __forceinline__ int padded_row(int L, int Cx) {
    const int m = 32;
    const int want = Cx % m;
    return L + ((want - L % m) % m + m) % m;
}

// Carried state of every recurrence for one column, walking t = T-1 .. 0.
struct Carry {
    float v_next;    // values[t+1]
    float tv_td;     // TD target at t+1
    float tv_up;     // UPGO target at t+1
    float acc;       // V-trace (vs - v) at t+1
    float vs_next;   // V-trace vs at t+1
};

// One time step of algorithm ALG for one column: reads the carry `s` of step
// t+1, writes this algorithm's fields of the carry `nx` for step t, returns
// the target and writes the advantage.  G1: gamma is exactly 1 (the value head,
// train.py:245), so `gamma * x` is x itself and the multiply is dropped: x * 1.0f
// equals x for every x, and the `reward + ...` add that follows quiets a
// signalling NaN either way.
template <int ALG, bool G1>
__device__ __forceinline__ float step(const Carry &s, Carry &nx, bool last, float v, float r, float rho,
                                      float c, float ret_t, float boot, const Coef &k, float &adv) {
    auto gx = [&](float x) __attribute__((always_inline)) { return G1 ? x : k.g * x; };
    if constexpr (ALG == HRL_ALG_MC) {                       // losses.py:16-17
        adv = ret_t - v;
        return ret_t;
    } else if constexpr (ALG == HRL_ALG_TD) {                // losses.py:20-28
        const float tv = last ? boot : r + gx(k.a * s.v_next + k.l * s.tv_td);
        nx.tv_td = tv;
        adv = tv - v;
        return tv;
    } else if constexpr (ALG == HRL_ALG_UPGO) {              // losses.py:31-40
        const float tv = last ? boot : r + gx(max_nan(s.v_next, k.a * s.v_next + k.l * s.tv_up));
        nx.tv_up = tv;
        adv = tv - v;
        return tv;
    } else {                                                 // losses.py:43-58
        const float v1 = last ? boot : s.v_next;
        const float delta = rho * ((r + gx(v1)) - v);
        const float acc = last ? delta : delta + (k.gl * c) * s.acc;   // vs_minus_v_xs, carried as is
        const float vs = acc + v;
        const float vs1 = last ? boot : s.vs_next;
        nx.acc = acc;
        nx.vs_next = vs;
        adv = (r + gx(vs1)) - v;
        return vs;
    }
}

// One time step of the fused pair: the target of TGT (kNone: none) and the advantages
// of ADV, as compute_target(TGT) and compute_target(ADV) give them (train.py:248-253).
template <int TGT, int ADV, bool G1>
__device__ __forceinline__ void fused_step(Carry &s, bool last, float v, float r, float rho, float c,
                                           float ret_t, float boot, const Coef &k, float &tgt_out,
                                           float &adv_out) {
    float adv, adv_unused;
    Carry nx = s;
    if constexpr (TGT != kNone && TGT != ADV) {
        tgt_out = step<TGT, G1>(s, nx, last, v, r, rho, c, ret_t, boot, k, adv_unused);
        step<ADV, G1>(s, nx, last, v, r, rho, c, ret_t, boot, k, adv);
    } else {
        tgt_out = step<ADV, G1>(s, nx, last, v, r, rho, c, ret_t, boot, k, adv);
    }
    adv_out = adv;
    nx.v_next = v;
    s = nx;
}

// The recurrence over up to kTChunk steps of one column whose inputs sit in LDS rows:
// value-shaped data at vofs + tt*C, rho-shaped at rofs + tt*rhoC.  Every LDS read is
// issued ahead of the dependent chain; results stay in registers until it is done.
// F: a full chunk: no guards, and in a TOP chunk the bootstrap step is tt = kTChunk-1 at
// compile time.  TOP: the chunk holds t = T-1.  A partial chunk (!F, always TOP: chunks are
// cut from t = 0) runs in 4-step blocks: a block above the chunk is skipped by one scalar
// branch, and inside a block every step runs unguarded with a run-time bootstrap select;
// the steps above tc - 1 read the top step's inputs again and their carry is discarded by
// that select, so no per-step branch sits on the serial chain.
template <int TGT, int ADV, bool REW, bool RHO, bool RET, bool F, bool TOP, bool G1 = false>
__device__ __forceinline__ void recur_chunk(Carry &s, float boot, const Coef &k, int tc, int C, int rhoC,
                                            const float *tv, const float *tr, const float *tret,
                                            const float *trho, const float *tcs, int vofs, int rofs,
                                            float *ttgt, float *tadv) {
    float xv[kTChunk], xr[kTChunk], xrho[kTChunk], xc[kTChunk], xret[kTChunk];
#pragma unroll
    for (int tt = 0; tt < kTChunk; ++tt) {
        if (F || tt < ((tc + 3) & ~3)) {
            const int ts = F ? tt : min(tt, tc - 1);
            const int iv = vofs + ts * C;
            const int ir = rofs + ts * rhoC;
            xv[tt] = tv[iv];
            xr[tt] = REW ? tr[iv] : 0.f;
            xrho[tt] = RHO ? trho[ir] : 0.f;
            xc[tt] = RHO ? tcs[ir] : 0.f;
            xret[tt] = RET ? tret[iv] : boot;
        }
    }
    float ot[kTChunk], oa[kTChunk];
    if constexpr (F) {
#pragma unroll
        for (int tt = kTChunk - 1; tt >= 0; --tt) {
            const bool last = TOP && tt == kTChunk - 1;
            fused_step<TGT, ADV, G1>(s, last, xv[tt], xr[tt], xrho[tt], xc[tt], xret[tt], boot, k, ot[tt], oa[tt]);
        }
    } else {
#pragma unroll
        for (int blk = kTChunk / 4 - 1; blk >= 0; --blk) {
            if (blk * 4 < tc) {
#pragma unroll
                for (int j = 3; j >= 0; --j) {
                    const int tt = blk * 4 + j;
                    fused_step<TGT, ADV, G1>(s, tt == tc - 1, xv[tt], xr[tt], xrho[tt], xc[tt], xret[tt], boot, k,
                                             ot[tt], oa[tt]);
                }
            }
        }
    }
#pragma unroll
    for (int tt = 0; tt < kTChunk; ++tt) {
        if (F || tt < tc) {
            const int iv = vofs + tt * C;
            if constexpr (TGT != kNone) ttgt[iv] = ot[tt];
            tadv[iv] = oa[tt];
        }
    }
}

}  // namespace hrl_scan

#endif  // HRL_SCAN_H
