// hrl_targets.hip — return-target scans for the HandyRL learner on MI355X (gfx950).
//
// Replaces handyrl/losses.py:16-74 (monte_carlo / temporal_difference / upgo /
// vtrace / compute_target).  The reference runs each recurrence as a Python
// loop of T-1 iterations of whole-batch torch ops (~140-344 elementwise ops
// per call at T=32).  Here one launch does the whole backward scan of every
// trajectory, and the fused entry point produces the value-target of one
// algorithm and the advantages of another in the same pass
// (train.py:248-253 issue 2-4 separate compute_target calls).
//
// Work decomposition (one wave64 per workgroup):
//   * a wave owns G <= 64 / C consecutive trajectories; lane = g*C + c owns one
//     value column (trajectory g, column c) and walks it backwards in time.
//     G = 64 / C at large B; at small B fewer, so the launch still has ~1024
//     waves: a wave's latency is its serial chain plus its share of the
//     load/transpose instructions, which shrinks with G;
//   * time is processed in chunks of up to TCHUNK steps.  Each chunk of every
//     input is loaded with coalesced 16-byte loads (the wave's trajectories are
//     contiguous in the (B,T,C) layout), ALL inputs' loads are issued before
//     any is consumed, and the values are transposed into a time-major LDS
//     tile [t][column] whose row stride (columns+1) makes both the transposing
//     writes and the per-lane column reads bank-conflict free;
//   * outputs go to LDS tiles of the same shape and leave through the mirror
//     transposition with coalesced 16-byte stores.
// Numerics: built with -ffp-contract=off; every recurrence performs the
// reference's float32 operations in the reference's order with the same
// float32-rounded coefficients, so results are bit-identical to the
// reference CPU learner (tests/test_targets_gpu.py checks max |diff|).
// Roofline: pure HBM streaming, ~1 flop/byte, no MFMA.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/hrl_targets.h"
#include "hrl_scan.h"

namespace {

using namespace hrl_scan;

HRL_STAMP_DECL

constexpr int kMaxTile = kTChunk * kWave;            // floats of one tensor chunk
constexpr int kMaxVec = kMaxTile / 4 / kWave;        // float4 loads per lane (8)
constexpr int kMaxScalar = kMaxTile / kWave;         // scalar loads per lane (32)

// One chunk of one (B, T, Cx) tensor for the wave's trajectories.
//   global: trajectory b0+g, time t0+tt, column cx at (b0+g)*R + t0*Cx + tt*Cx + cx
//   LDS   : trajectory-major rows, [g][tt*Cx + cx], row stride Lp
struct Chunk {
    const float *base;  // element (g=0, tt=0, cx=0)
    int R;              // row length of one trajectory (T*Cx)
    int L;              // span length of one trajectory in this chunk (tc*Cx)
    int Lp;             // padded LDS row stride
    int n;              // valid elements (ntraj * L)
    float invL;
    bool shape_ok;      // spans are whole float4s (or one contiguous run)
    bool vec;           // 16-byte loads are legal for this tensor

    __device__ __forceinline__ void setup(const float *p, int64_t b0, int T, int Cx, int t0, int tc,
                                          int ntraj, int Lp_) {
        R = T * Cx;
        L = tc * Cx;
        Lp = Lp_;
        n = ntraj * L;
        invL = 1.0f / (float)L;
        base = p + b0 * (int64_t)R + (int64_t)t0 * Cx;
        // Contiguous spans (L == R) may straddle trajectories inside a float4;
        // otherwise every span must be whole float4s.
        shape_ok = (L == R) || ((L & 3) == 0 && (R & 3) == 0);
        vec = shape_ok && ((reinterpret_cast<uintptr_t>(base) & 15) == 0);
    }

    // global offset (from base; < 2^31 by the host's size check) and LDS slot of element e
    __device__ __forceinline__ void locate(int e, int &gofs, int &slot) const {
        const int g = fdiv(e, invL);
        const int rem = e - g * L;
        gofs = (L == R) ? e : g * R + rem;
        slot = g * Lp + rem;
    }
    // LDS slots of elements e..e+3 given element e's trajectory g and offset rem
    __device__ __forceinline__ int slot_after(int g, int rem, int j) const {
        const int r = rem + j;
        const bool wrap = r >= L;   // only when a float4 straddles two trajectories
        return (wrap ? g + 1 : g) * Lp + (wrap ? r - L : r);
    }
};

// Registers holding one chunk between its global loads and its LDS writes.
template <bool VEC>
struct Staged {
    float x[VEC ? 4 * kMaxVec : kMaxScalar];

    __device__ __forceinline__ void load(const Chunk &c) {
        if (c.n <= 0) return;
        const int lane = threadIdx.x;
        if constexpr (VEC) {
            const int nv = c.n >> 2;
            if (nv == 0) return;
#pragma unroll
            for (int k = 0; k < kMaxVec; ++k) {
                if (k * kWave >= nv) break;   // wave-uniform: small tiles issue fewer rounds
                // clamp instead of branching so every load issues back to back
                const int vi = min(k * kWave + lane, nv - 1);
                int go; int slot;
                c.locate(vi * 4, go, slot);
                const float4 q = *reinterpret_cast<const float4 *>(c.base + go);
                x[4 * k + 0] = q.x; x[4 * k + 1] = q.y; x[4 * k + 2] = q.z; x[4 * k + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kMaxScalar; ++k) {
                if (k * kWave >= c.n) break;
                const int e = min(k * kWave + lane, c.n - 1);
                int go; int slot;
                c.locate(e, go, slot);
                x[k] = c.base[go];
            }
        }
    }

    __device__ __forceinline__ void to_lds(const Chunk &c, float *tile) const {
        if (c.n <= 0) return;
        const int lane = threadIdx.x;
        if constexpr (VEC) {
            const int nv = c.n >> 2;
#pragma unroll
            for (int k = 0; k < kMaxVec; ++k) {
                if (k * kWave >= nv) break;
                const int e = (k * kWave + lane) * 4;
                if (e < 4 * nv) {
                    const int g = fdiv(e, c.invL);
                    const int rem = e - g * c.L;
#pragma unroll
                    for (int j = 0; j < 4; ++j) tile[c.slot_after(g, rem, j)] = x[4 * k + j];
                }
            }
            // ragged tail (< 4 elements) of a contiguous span
            const int e = nv * 4 + lane;
            if (e < c.n) {
                int go; int slot;
                c.locate(e, go, slot);
                tile[slot] = c.base[go];
            }
        } else {
#pragma unroll
            for (int k = 0; k < kMaxScalar; ++k) {
                if (k * kWave >= c.n) break;
                const int e = k * kWave + lane;
                if (e < c.n) {
                    int go; int slot;
                    c.locate(e, go, slot);
                    tile[slot] = x[k];
                }
            }
        }
    }
};

// LDS tile -> global, the mirror of Staged (stores need no batching).
template <bool VEC>
__device__ __forceinline__ void store_chunk(const Chunk &c, const float *tile, float *out_base) {
    if (c.n <= 0) return;
    const int lane = threadIdx.x;
    float *base = out_base;
    if constexpr (VEC) {
        const int nv = c.n >> 2;
        for (int vi = lane; vi < nv; vi += kWave) {
            const int e = vi * 4;
            const int g = fdiv(e, c.invL);
            const int rem = e - g * c.L;
            float4 q;
            q.x = tile[c.slot_after(g, rem, 0)];
            q.y = tile[c.slot_after(g, rem, 1)];
            q.z = tile[c.slot_after(g, rem, 2)];
            q.w = tile[c.slot_after(g, rem, 3)];
            const int go = (c.L == c.R) ? e : g * c.R + rem;
            *reinterpret_cast<float4 *>(base + go) = q;
        }
        const int e = nv * 4 + lane;
        if (e < c.n) {
            int go; int slot;
            c.locate(e, go, slot);
            base[go] = tile[slot];
        }
    } else {
        for (int e = lane; e < c.n; e += kWave) {
            int go; int slot;
            c.locate(e, go, slot);
            base[go] = tile[slot];
        }
    }
}

struct Args {
    const float *values, *returns, *rewards, *rhos, *cs;
    float *targets, *advantages;
    int64_t B;
    int T, C, retT, rhoC, rhoDiv;
    int G;      // trajectories per wave (<= 64 / C; fewer when B is small, to spread waves)
    Coef k;
};

// TGT: algorithm whose target is written (kNone: no target output).
// ADV: algorithm whose advantages are written.
// REW: rewards present.  RETT: MC reads returns at every t (ret_T == T).
// LDS row stride for a tile of Cx columns per step read column-wise by lanes (g, c): an odd multiple of Cx, so
// g*Lp + c are distinct modulo 32 over each 32-lane half when Cx divides 32 (conflict-free ds_read_b32) with no
// more padding than one step's columns (padded_row pads a T = 9, Cx = 1 row of 9 floats to 33).
__host__ __device__ __forceinline__ int odd_row(int tmax, int Cx) { return Cx * (tmax | 1); }

// ONE: T <= kTChunk, the whole trajectory is one chunk (no prefetch path: ~70 registers instead of 216).
template <int TGT, int ADV, bool REW, bool RETT, bool VEC, bool ONE>
__global__ __launch_bounds__(kWave) void targets_kernel(Args a) {
    constexpr bool kRho = (TGT == HRL_ALG_VTRACE) || (ADV == HRL_ALG_VTRACE);
    constexpr bool kRet = RETT && (ADV == HRL_ALG_MC);

    extern __shared__ float lds[];
    const int lane = threadIdx.x;
    const int C = a.C;
    const int G = a.G;
    const int J = G * C;                      // value columns per wave
    const int T = a.T;
    const int tmax = T < kTChunk ? T : kTChunk;
    const int Lpv = odd_row(tmax, C);                // value-shaped rows
    const int Lpr = odd_row(tmax, a.rhoC);           // rho rows (lanes of one g share a slot)

    const int64_t b0 = (int64_t)blockIdx.x * G;
    const int ntraj = (int)min<int64_t>(G, a.B - b0);

    // LDS carve-up (sizes fixed by tmax, see launch).  The targets overwrite the values in place: recur_chunk
    // reads a column's inputs before it writes that column's outputs, and no lane touches another's column.
    const int vt = G * Lpv, rt = G * Lpr;
    float *t_v = lds;
    float *t_r = t_v + vt;
    float *t_ret = t_r + (REW ? vt : 0);
    float *t_tgt = t_v;
    float *t_adv = t_ret + (kRet ? vt : 0);
    float *t_rho = t_adv + vt;
    float *t_cs = t_rho + (kRho ? rt : 0);

    const int g = lane / C;
    const int c = lane - g * C;
    const bool active = (lane < J) && (g < ntraj);
    const int vbase = g * Lpv + c;                     // + tt*C
    const int rbase = g * Lpr + c / a.rhoDiv;          // + tt*rhoC

    HRL_STAMP_WALL(14);
    HRL_STAMP(0);
    float boot = 0.f;
    if (active) {
        boot = a.returns[(b0 + g) * (int64_t)a.retT * C + (int64_t)(a.retT - 1) * C + c];
    }

    Carry s{0.f, 0.f, 0.f, 0.f, 0.f};
    const int nchunks = (T + kTChunk - 1) / kTChunk;

    // Software pipeline over chunks (walking time backwards): chunk ch's inputs
    // arrive in registers one iteration ahead, so the global-load latency of
    // chunk ch-1 overlaps chunk ch's LDS transpose and recurrence.
    Chunk cv, cr, cret, crho, ccs;
    Staged<VEC> sv, sr, sret, srho, scs;
    auto setup_and_load = [&](int ch) {
        const int t0 = ch * kTChunk;
        const int tc = min(kTChunk, T - t0);
        cv.setup(a.values, b0, T, C, t0, tc, ntraj, Lpv);
        if constexpr (REW) cr.setup(a.rewards, b0, T, C, t0, tc, ntraj, Lpv);
        if constexpr (kRet) cret.setup(a.returns, b0, T, C, t0, tc, ntraj, Lpv);
        if constexpr (kRho) {
            crho.setup(a.rhos, b0, T, a.rhoC, t0, tc, ntraj, Lpr);
            ccs.setup(a.cs, b0, T, a.rhoC, t0, tc, ntraj, Lpr);
        }
        // every input's loads are issued before the first is consumed
        sv.load(cv);
        if constexpr (REW) sr.load(cr);
        if constexpr (kRet) sret.load(cret);
        if constexpr (kRho) { srho.load(crho); scs.load(ccs); }
    };
    setup_and_load(nchunks - 1);
    // Consume the bootstrap load here (in straight-line code the wait covers only that
    // load); afterwards `boot` is a plain register, so the waitcnt pass does not put a
    // full vmcnt(0) -- draining the prefetched chunk -- in front of the recurrence.
    asm volatile("" : "+v"(boot));
    HRL_STAMP(1);

    // The recurrence over one chunk held in LDS.  TOP: the chunk holds t = T-1 (the bootstrap
    // step).  Chunks are cut from t = 0, so only the top chunk can be partial; a FULL chunk
    // has no per-step guards and a compile-time bootstrap test (tt == kTChunk-1 in a full top
    // chunk, never elsewhere), so its serial chain has no compares, branches or spilled step
    // indices.  Only a partial top chunk (T % kTChunk != 0) tests `last` at run time.
    auto recur = [&](int tc, auto full, auto top) __attribute__((always_inline)) {
        recur_chunk<TGT, ADV, REW, kRho, kRet, decltype(full)::value, decltype(top)::value>(
            s, boot, a.k, tc, C, a.rhoC, t_v, t_r, t_ret, t_rho, t_cs, vbase, rbase, t_tgt, t_adv);
    };

    auto process = [&](int ch, auto prefetch) {
        const int t0 = ch * kTChunk;
        const int tc = min(kTChunk, T - t0);

        sv.to_lds(cv, t_v);
        if constexpr (REW) sr.to_lds(cr, t_r);
        if constexpr (kRet) sret.to_lds(cret, t_ret);
        if constexpr (kRho) { srho.to_lds(crho, t_rho); scs.to_lds(ccs, t_cs); }
        const Chunk out = cv;          // this chunk's output geometry
        // the next chunk's loads stay in flight through this chunk (unconditional in this
        // instantiation, so no register phi forces an early wait on them)
        if constexpr (decltype(prefetch)::value) setup_and_load(ch - 1);
        __syncthreads();
        HRL_STAMP(2 + 3 * (nchunks - 1 - ch));

        if (active) {
            if (ch != nchunks - 1) recur(tc, std::true_type{}, std::false_type{});
            else if (tc == kTChunk) recur(tc, std::true_type{}, std::true_type{});
            else recur(tc, std::false_type{}, std::true_type{});
        }
        __syncthreads();
        HRL_STAMP(3 + 3 * (nchunks - 1 - ch));

        const int64_t off = b0 * (int64_t)T * C + (int64_t)t0 * C;
        if constexpr (TGT != kNone) store_chunk<VEC>(out, t_tgt, a.targets + off);
        store_chunk<VEC>(out, t_adv, a.advantages + off);
        HRL_STAMP(4 + 3 * (nchunks - 1 - ch));
    };
    if constexpr (!ONE)
        for (int ch = nchunks - 1; ch > 0; --ch) process(ch, std::true_type{});
    process(0, std::false_type{});
    HRL_STAMP_WALL(15);
}

// Short trajectories (T <= kTChunk): targets_kernel spends a group's life in serial phases -- load, LDS
// transpose, barrier, chain, barrier, transpose, store -- and its LDS tiles and 216 registers hold the chip to
// ~8 waves per CU, so at T = 9 it streams at a third of HBM.  Here a lane owns one (trajectory, column) and
// nothing else: its T inputs come straight from global memory into registers (4-byte loads; a wave's loads of
// one step touch the same lines as its other steps', which L1/L2 serve once), the chain runs, and each step's
// outputs are stored as they are produced.  No LDS, no barrier, ~70 registers: enough waves in flight to hide
// the HBM latency.  The per-column arithmetic is fused_step's, in recur_chunk's order: bit-identical results.
template <int TGT, int ADV, bool REW, bool RETT>
__global__ __launch_bounds__(256) void targets_lane_kernel(Args a) {
    constexpr bool kRho = (TGT == HRL_ALG_VTRACE) || (ADV == HRL_ALG_VTRACE);
    constexpr bool kRet = RETT && (ADV == HRL_ALG_MC);
    const int C = a.C, T = a.T, G = a.G;
    const int lane = threadIdx.x & 63;
    const int g = lane / C;
    const int c = lane - g * C;
    const int64_t b = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + g;
    if (g >= G || b >= a.B) return;            // no barrier below
    const int64_t row = b * (int64_t)T;
    const float *pv = a.values + row * C + c;
    const float *pr = REW ? a.rewards + row * C + c : nullptr;
    const float *pret = kRet ? a.returns + row * C + c : nullptr;
    const int rc = c / a.rhoDiv;
    const float *prho = kRho ? a.rhos + row * a.rhoC + rc : nullptr;
    const float *pcs = kRho ? a.cs + row * a.rhoC + rc : nullptr;
    float xv[kTChunk], xr[kTChunk], xrho[kTChunk], xc[kTChunk], xret[kTChunk];
    const float boot = a.returns[b * (int64_t)a.retT * C + (int64_t)(a.retT - 1) * C + c];
#pragma unroll
    for (int tt = 0; tt < kTChunk; ++tt) {
        if (tt < T) {
            xv[tt] = pv[tt * C];
            xr[tt] = REW ? pr[tt * C] : 0.f;
            xret[tt] = kRet ? pret[tt * C] : boot;
            xrho[tt] = kRho ? prho[tt * a.rhoC] : 0.f;
            xc[tt] = kRho ? pcs[tt * a.rhoC] : 0.f;
        }
    }
    float *ptg = TGT != kNone ? a.targets + row * C + c : nullptr;
    float *pad = a.advantages + row * C + c;
    Carry s{0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tt = kTChunk - 1; tt >= 0; --tt) {
        if (tt < T) {
            float tg, ad;
            fused_step<TGT, ADV, false>(s, tt == T - 1, xv[tt], xr[tt], xrho[tt], xc[tt], xret[tt], boot, a.k, tg,
                                        ad);
            if constexpr (TGT != kNone) ptg[tt * C] = tg;
            pad[tt * C] = ad;
        }
    }
}

// hrl_targets_set_short_form, for T <= kTChunk: 1 (default) targets_lane_kernel for small batches (B*C <= 32768,
// where it is 10% faster: fewer serial phases per wave) and targets_kernel otherwise (coalesced loads: 48.6% of HBM
// at B = 2^20, T = 9 cold against the lane kernel's 29.5%, whose 4-byte column loads touch ~18 lines each);
// 2 the lane kernel always, 0 targets_kernel always
int g_short_form = 1;

template <int TGT, int ADV, bool REW, bool RETT, bool VEC>
int launch_one(const Args &a, hipStream_t stream) {
    constexpr bool kRho = (TGT == HRL_ALG_VTRACE) || (ADV == HRL_ALG_VTRACE);
    constexpr bool kRet = RETT && (ADV == HRL_ALG_MC);
    const int G = a.G;
    const int tmax = a.T < kTChunk ? a.T : kTChunk;
    const int vtiles = 1 + (REW ? 1 : 0) + (kRet ? 1 : 0) + 1;    // values (then targets), rewards, returns, adv
    const size_t vt = (size_t)G * odd_row(tmax, a.C);
    const size_t rt = (size_t)G * odd_row(tmax, a.rhoC);
    const size_t lds = sizeof(float) * (vtiles * vt + (kRho ? 2 : 0) * rt);
    const int64_t blocks = (a.B + G - 1) / G;
    if (blocks > 0x7fffffff) return HRL_EINVAL;
    if (a.T <= kTChunk && (g_short_form == 2 || (g_short_form == 1 && a.B * a.C <= 32768))) {
        Args b = a;
        b.G = kWave / a.C;
        const int64_t waves = (a.B + b.G - 1) / b.G;
        const int64_t wgs = (waves + 3) / 4;
        if (wgs > 0x7fffffff) return HRL_EINVAL;
        hipLaunchKernelGGL((targets_lane_kernel<TGT, ADV, REW, RETT>), dim3((unsigned)wgs), dim3(4 * kWave), 0,
                           stream, b);
    } else {
        if (a.T <= kTChunk)
            hipLaunchKernelGGL((targets_kernel<TGT, ADV, REW, RETT, VEC, true>), dim3((unsigned)blocks), dim3(kWave),
                               lds, stream, a);
        else
            hipLaunchKernelGGL((targets_kernel<TGT, ADV, REW, RETT, VEC, false>), dim3((unsigned)blocks), dim3(kWave),
                               lds, stream, a);
    }
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err;
}

// 16-byte loads/stores need every tensor 16-byte aligned and every per-
// trajectory span a whole number of float4s (or one contiguous run, T <= chunk).
bool vector_ok(const Args &a) {
    auto aligned = [](const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!aligned(a.values) || !aligned(a.returns) || !aligned(a.rewards) || !aligned(a.rhos) || !aligned(a.cs) ||
        !aligned(a.targets) || !aligned(a.advantages))
        return false;
    if (a.T <= kTChunk) return true;
    // full chunks are kTChunk*Cx floats (a multiple of 4); rows and the tail chunk must be too
    return ((a.T * a.C) & 3) == 0 && ((a.T * a.rhoC) & 3) == 0;
}

template <int TGT, int ADV, bool REW>
int launch_vec(const Args &a, hipStream_t s) {
    const bool rett = (ADV == HRL_ALG_MC) && a.retT == a.T && a.T > 1;
    if (vector_ok(a)) return rett ? launch_one<TGT, ADV, REW, true, true>(a, s) : launch_one<TGT, ADV, REW, false, true>(a, s);
    return rett ? launch_one<TGT, ADV, REW, true, false>(a, s) : launch_one<TGT, ADV, REW, false, false>(a, s);
}

template <int TGT, int ADV>
int launch_flags(const Args &a, hipStream_t s) {
    return a.rewards != nullptr ? launch_vec<TGT, ADV, true>(a, s) : launch_vec<TGT, ADV, false>(a, s);
}

template <int TGT>
int launch_adv(int adv, const Args &a, hipStream_t s) {
    switch (adv) {
        case HRL_ALG_MC: return launch_flags<TGT, HRL_ALG_MC>(a, s);
        case HRL_ALG_TD: return launch_flags<TGT, HRL_ALG_TD>(a, s);
        case HRL_ALG_UPGO: return launch_flags<TGT, HRL_ALG_UPGO>(a, s);
        case HRL_ALG_VTRACE: return launch_flags<TGT, HRL_ALG_VTRACE>(a, s);
        default: return HRL_EINVAL;
    }
}

int dispatch(int tgt, int adv, const Args &a, hipStream_t s) {
    switch (tgt) {
        case kNone: return launch_adv<kNone>(adv, a, s);
        case HRL_ALG_TD: return launch_adv<HRL_ALG_TD>(adv, a, s);
        case HRL_ALG_UPGO: return launch_adv<HRL_ALG_UPGO>(adv, a, s);
        case HRL_ALG_VTRACE: return launch_adv<HRL_ALG_VTRACE>(adv, a, s);
        default: return HRL_EINVAL;
    }
}

bool valid_alg(int alg) { return alg >= HRL_ALG_MC && alg <= HRL_ALG_VTRACE; }

int prepare(int target_alg, int adv_alg, const float *values, const float *returns, const float *rewards,
            const float *rhos, const float *cs, int64_t B, int64_t T, int64_t C, int64_t ret_T,
            int64_t rho_C, int64_t rho_div, double lmb, double gamma, float *targets, float *advantages,
            void *stream) {
    if (!valid_alg(target_alg) || !valid_alg(adv_alg)) return HRL_EINVAL;
    if (B < 0 || T < 1 || C < 1 || C > kWave || T > (1 << 24)) return HRL_EINVAL;
    if (ret_T != 1 && ret_T != T) return HRL_EINVAL;
    if (rho_C < 1 || rho_div < 1 || rho_C * rho_div != C) {
        // rho columns must tile the value columns: rho_C == 1 (rho_div == C) or rho_C == P (rho_div == K)
        return HRL_EINVAL;
    }
    if (target_alg == HRL_ALG_MC && targets != nullptr) return HRL_EINVAL;
    if (B == 0) return HRL_OK;  // empty batch: nothing to read or write (data pointers may be NULL)
    const bool need_rho = target_alg == HRL_ALG_VTRACE || adv_alg == HRL_ALG_VTRACE;
    if (!values || !returns || !advantages || (need_rho && (!rhos || !cs))) return HRL_EINVAL;
    if (B * T * C > (int64_t)1 << 40 || T * C * kWave >= ((int64_t)1 << 31)) return HRL_EINVAL;
    Args a;
    a.values = values; a.returns = returns; a.rewards = rewards; a.rhos = rhos; a.cs = cs;
    a.targets = targets; a.advantages = advantages;
    a.B = B; a.T = (int)T; a.C = (int)C; a.retT = (int)ret_T; a.rhoC = (int)rho_C; a.rhoDiv = (int)rho_div;
    a.k = make_coef(lmb, gamma);
    // Waves per launch: a wave's trajectories are walked by one serial chain, so at small B
    // spread them over at least ~1024 waves (one per SIMD) instead of filling every lane.
    {
        // G stays a multiple of 4 (or 64 / C itself), so every wave's first trajectory starts
        // 16-byte aligned whenever the tensors are (the float4 path's precondition).
        const int gmax = kWave / a.C;
        int g = gmax < 4 ? gmax : 4;
        while (g * 2 <= gmax && B / (g * 2) >= 1024) g *= 2;
        a.G = g;
    }
    const int tgt = (targets == nullptr || target_alg == HRL_ALG_MC) ? kNone : target_alg;
    return dispatch(tgt, adv_alg, a, static_cast<hipStream_t>(stream));
}

}  // namespace

extern "C" {

#ifdef HRL_STAMPS
int hrl_debug_set_stamps_targets(void *buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hrl_stamps), &buf, sizeof(buf));
}
#endif

int hrl_abi_version(void) { return 26; }

int hrl_targets_set_short_form(int form) {
    const int prev = g_short_form;
    g_short_form = form < 0 ? 0 : (form > 2 ? 2 : form);
    return prev;
}

const char *hrl_strerror(int code) {
    if (code == HRL_OK) return "success";
    if (code == HRL_EINVAL) return "invalid argument (algorithm, shape or pointer)";
    if (code <= HRL_ELAUNCH_BASE) return hipGetErrorString(static_cast<hipError_t>(HRL_ELAUNCH_BASE - code));
    return "unknown error";
}

int hrl_compute_target(int alg, const float *values, const float *returns, const float *rewards,
                       const float *rhos, const float *cs, int64_t B, int64_t T, int64_t C, int64_t ret_T,
                       int64_t rho_C, int64_t rho_div, double lmb, double gamma, float *targets,
                       float *advantages, void *stream) {
    return prepare(alg, alg, values, returns, rewards, rhos, cs, B, T, C, ret_T, rho_C, rho_div, lmb, gamma,
                   targets, advantages, stream);
}

int hrl_compute_targets_fused(int target_alg, int adv_alg, const float *values, const float *returns,
                              const float *rewards, const float *rhos, const float *cs, int64_t B, int64_t T,
                              int64_t C, int64_t ret_T, int64_t rho_C, int64_t rho_div, double lmb,
                              double gamma, float *targets, float *advantages, void *stream) {
    return prepare(target_alg, adv_alg, values, returns, rewards, rhos, cs, B, T, C, ret_T, rho_C, rho_div, lmb,
                   gamma, targets, advantages, stream);
}

}  // extern "C"
