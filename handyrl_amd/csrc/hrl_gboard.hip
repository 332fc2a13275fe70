// hrl_gboard.hip — 3x3 'same' (zero padding) convolution on the 6x6 Geister board, games as MFMA rows.
//
// GeisterNet's convolutions (handyrl/envs/geister.py:17-63 ConvLSTMCell, :99-167 GeisterNet: the stem
// 25 -> 32, the cells' x halves 32 -> 3*128, their h halves as one grouped 3 x (32 -> 128), the move head
// 64 -> 8) at self-play sizes (E = 2048 games per ply).  Per output cell q the convolution is the GEMM
//     Y_q (16 games x 16 co) += sum_{p in nbhd(q)} X_p (16 games x 32 ci) . W[tap(p, q)] (32 ci x 16 co)
// on v_mfma_f32_16x16x32_bf16 with the exact three-way split of hrl_split.h (fp32-accurate: six partial
// products).  Taps off the board are never computed: 256 of the 324 (cell, tap) pairs are real.
//  * one wave owns one 16-channel column tile ct for the whole launch: the split weight fragments
//    [kc][tap][part] of its tile (108 VGPRs per 32-channel k-step), pre-split by gboard_pack_kernel, are
//    loaded once (once per k-step for two-step convolutions);
//  * the wave walks 16-game tiles.  A tile's 36 cells of accumulators (144 AGPRs) stay in registers; the input
//    is read p-major four cells at a time (one float4 per (game, channel)), split once per cell and fed to
//    every output cell it reaches; three groups of loads rotate through registers, two in flight;
//  * the waves of one game tile (its column tiles) sit in one XCD, so the tile is read from HBM once;
//  * epilogue: + bias, BatchNorm apply (y*alpha + beta, hrl_bn_apply's float operations) and ReLU, each
//    optional; a lane's 36 cells of one (game, channel) are one contiguous 144-byte run (9 float4 stores).
// Bound: MFMA (6 bf16 MFMAs per fp32-accurate 16x16x32 product).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"
#include "hrl_split.h"

namespace {

using hrl_split::f32x4;
using hrl_split::mfma_split;
using hrl_split::split8;

constexpr int kBH = 6, kBW = 6, kHW = kBH * kBW;
constexpr int kQuads = kHW / 4;   // float4 groups of cells per channel row
constexpr int kTaps = 9;
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kCUs = 256;         // one 4-wave workgroup per CU (one wave per SIMD)

struct GbArgs {
    const float *x, *x2;   // x2 (optional): input channels 32.. (the move head's [h_e, h_last] without a copy)
    int64_t N, xs, xs2;    // games; floats from one game to the next in x / x2
    const float *xg[4];    // per-group inputs (hrl_gboard_forward_groups: the DRC layers' separate states), or NULL
    int64_t xgs[4];        // floats from one game to the next in xg[g]
    int cin_g, cout_g;     // input / output channels per group
    const uint4 *wpk;      // split weight fragments [ct][kc][tap][part][64]
    int nct, cout;         // 16-channel column tiles; output channels stored
    const float *bias, *alpha, *beta;
    int relu;
    float *y;
    int64_t ys;            // floats from one game to the next in y
};

// tap of input cell p for output cell q (-1 off the 3x3 neighbourhood)
__host__ __device__ constexpr int tap_pq(int p, int q) {
    const int dy = p / kBW - q / kBW + 1, dx = p % kBW - q % kBW + 1;
    return (dy < 0 || dy > 2 || dx < 0 || dx > 2) ? -1 : dy * 3 + dx;
}

template <int I> using IC = std::integral_constant<int, I>;

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(IC<I>{});
        static_for<I + 1, N>(f);
    }
}

__device__ __forceinline__ float relu_f(float v) { return v < 0.f ? 0.f : v; }   // NaN stays NaN

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma32(const uint4 &a, const uint4 &b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

__device__ __forceinline__ void bar_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// output-cell bands: NB waves share a column tile, wave band b owns the cells of quads [band_q0, band_q1)
__host__ __device__ constexpr int band_q0(int NB, int b) { return NB == 1 ? 0 : (NB == 2 ? 5 * b : 2 * b); }
__host__ __device__ constexpr int band_q1(int NB, int b) {
    return NB == 1 ? kQuads : (NB == 2 ? (b == 0 ? 5 : kQuads) : (b == 3 ? kQuads : 2 * b + 2));
}
// does output band b of NB use input cell p?
__host__ __device__ constexpr bool band_uses(int NB, int b, int p) {
    for (int q = 4 * band_q0(NB, b); q < 4 * band_q1(NB, b); ++q)
        if (tap_pq(p, q) >= 0) return true;
    return false;
}

constexpr int kPartBytes = 4 * 16 * 32 * 2;   // one split part of one quad's image: [cell][game][channel] bf16
constexpr int kSlotBytes = 3 * kPartBytes;     // 12 KB per quad
constexpr int kLdsBytes = 3 * kSlotBytes;      // ring of three quads

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }   // lstm_fwd_kernel's

// One wave of gboard_conv_kernel: column tile (task's tile group * NCTW + ctl), output band BAND of NB = 4 / NCTW.
template <int KC, bool PADC, int NCTW, int BAND, int R = 3>
__device__ __forceinline__ void gboard_run(const GbArgs &a, unsigned char *smem, int lane, int wave, int L) {
    constexpr int NB = 4 / NCTW;
    constexpr int Q0 = band_q0(NB, BAND), Q1 = band_q1(NB, BAND);
    constexpr int NCELL = 4 * (Q1 - Q0);
    const int ctl = wave % NCTW;
    const int n_ctg = a.nct / NCTW;
    const int64_t ntiles = (a.N + 15) >> 4;
    const int64_t ntasks = ntiles * n_ctg;
    const int r = lane & 15, g = lane >> 4;
    // staging role: game 4*wave + (lane >> 4) of the tile, channels 2cp, 2cp + 1 of the k-step
    const int sg = 4 * wave + (lane >> 4), cp = lane & 15;

    int64_t task = L;
    if (task >= ntasks) return;   // uniform over the workgroup: no barrier is left waiting
    auto tile_of = [&](int64_t t) { return t / n_ctg; };
    auto ct_of = [&](int64_t t) { return (int)(t % n_ctg) * NCTW + ctl; };
    // the staging lane's source row for (task, kc): channels 32kc + 2cp (+1) of game sg of the task's tile
    // (PADC: rows at or past cin_g read row cin_g - 1 and are zeroed)
    auto src = [&](int64_t t, int kc, int &c0, int &c1) -> const float * {
        const int64_t n = min(tile_of(t) * 16 + sg, a.N - 1);
        const int grp = ct_of(t) * 16 / a.cout_g;   // one group for all the workgroup's column tiles
        c0 = 32 * kc + 2 * cp;
        c1 = c0 + 1;
        if constexpr (PADC) {
            c0 = min(c0, a.cin_g - 1);
            c1 = min(c1, a.cin_g - 1);
        }
        if (KC > 1 && kc >= 1 && a.x2) return a.x2 + n * a.xs2 + (int64_t)(-32) * kHW;
        if (a.xg[0]) return a.xg[grp] + n * a.xgs[grp];
        return a.x + n * a.xs + (int64_t)(grp * a.cin_g) * kHW;
    };
    float4 raw[R][2];
    auto issue = [&](int64_t t, int kc, int quad, auto slot_c) __attribute__((always_inline)) {
        constexpr int slot = decltype(slot_c)::value;
        int c0, c1;
        const float *s = src(t, kc, c0, c1);
        raw[slot][0] = *reinterpret_cast<const float4 *>(s + c0 * kHW + 4 * quad);
        raw[slot][1] = *reinterpret_cast<const float4 *>(s + c1 * kHW + 4 * quad);
    };
    auto stage = [&](int kc, auto slot_c) __attribute__((always_inline)) {   // raw[slot] -> LDS slot
        constexpr int slot = decltype(slot_c)::value;
        const int c0 = 32 * kc + 2 * cp;
        unsigned char *dst = smem + slot * kSlotBytes + sg * 64 + cp * 4;
        static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
            constexpr int u = decltype(u_c)::value;
            const float4 &f0 = raw[slot][0], &f1 = raw[slot][1];
            float v0 = u == 0 ? f0.x : (u == 1 ? f0.y : (u == 2 ? f0.z : f0.w));
            float v1 = u == 0 ? f1.x : (u == 1 ? f1.y : (u == 2 ? f1.z : f1.w));
            if constexpr (PADC) {
                if (c0 >= a.cin_g) v0 = 0.f;
                if (c0 + 1 >= a.cin_g) v1 = 0.f;
            }
            uint32_t h0, m0, l0, h1, m1, l1;
            hrl_split::split3(v0, h0, m0, l0);
            hrl_split::split3(v1, h1, m1, l1);
            *reinterpret_cast<uint32_t *>(dst + (0 * 4 + u) * 1024) = h0 | (h1 << 16);
            *reinterpret_cast<uint32_t *>(dst + (1 * 4 + u) * 1024) = m0 | (m1 << 16);
            *reinterpret_cast<uint32_t *>(dst + (2 * 4 + u) * 1024) = l0 | (l1 << 16);
        });
    };
    uint4 Bw[kTaps][3];
    auto load_b = [&](int ct, int kc) __attribute__((always_inline)) {
        const uint4 *wp = a.wpk + (((int64_t)ct * KC + kc) * kTaps * 3) * 64 + lane;
        static_for<0, kTaps * 3>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int i = decltype(i_c)::value;
            Bw[i / 3][i % 3] = wp[i * 64];
        });
    };
    f32x4 acc[NCELL];
    static_for<0, NCELL>([&](auto q_c) __attribute__((always_inline)) {
        acc[decltype(q_c)::value] = (f32x4){0.f, 0.f, 0.f, 0.f};
    });

    const int64_t step = gridDim.x;
    // compute quad j of the current task from LDS slot `slot`
    auto compute = [&](auto j_c, auto slot_c) __attribute__((always_inline)) {
        constexpr int j = decltype(j_c)::value;
        const unsigned char *img = smem + decltype(slot_c)::value * kSlotBytes + r * 64 + g * 16;
        static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
            constexpr int u = decltype(u_c)::value;
            constexpr int p = 4 * j + u;
            if constexpr (band_uses(NB, BAND, p)) {
                const uint4 Ah = *reinterpret_cast<const uint4 *>(img + (0 * 4 + u) * 1024);
                const uint4 Am = *reinterpret_cast<const uint4 *>(img + (1 * 4 + u) * 1024);
                const uint4 Al = *reinterpret_cast<const uint4 *>(img + (2 * 4 + u) * 1024);
                static_for<4 * Q0, 4 * Q1>([&](auto q_c) __attribute__((always_inline)) {
                    constexpr int q = decltype(q_c)::value;
                    constexpr int t = tap_pq(p, q);
                    if constexpr (t >= 0)
                        acc[q - 4 * Q0] = mfma_split(Ah, Am, Al, Bw[t][0], Bw[t][1], Bw[t][2], acc[q - 4 * Q0]);
                });
            }
        });
    };
    // WHOLE (R = 9, one k-step, one task per workgroup): the tile's nine quads are loaded and staged at once
    // and the waves then compute without a barrier per quad -- the output bands need different input quads,
    // so a per-quad lockstep idles the waves of one band while the other's are busy
    constexpr bool WHOLE = R == kQuads && KC == 1;
    int ct_b = -1;
    if constexpr (WHOLE) {
        static_for<0, kQuads>([&](auto i_c) __attribute__((always_inline)) {
            issue(task, 0, decltype(i_c)::value, i_c);
        });
        static_for<0, kQuads>([&](auto i_c) __attribute__((always_inline)) { stage(0, i_c); });
        ct_b = ct_of(task);
        load_b(ct_b, 0);   // after the staging: the raw quads' registers are free again
    } else {
        // prologue: quad 0 staged, quads 1 .. R - 2 in flight
        static_assert((KC * kQuads) % R == 0 && R - 1 <= KC * kQuads, "the ring's slots repeat per task");
        static_for<0, R - 1>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int i = decltype(i_c)::value;
            issue(task, i / kQuads, i % kQuads, IC<i>{});
        });
        stage(0, IC<0>{});
    }
    bar_lds();
    for (; task < ntasks; task += step) {
        const int64_t nxt = task + step < ntasks ? task + step : task;   // loads past the end: re-read
        const int ct = ct_of(task);
        if (KC == 1 && ct != ct_b) load_b(ct, 0);
        ct_b = ct;
        if constexpr (WHOLE) {
            static_for<0, kQuads>([&](auto j_c) __attribute__((always_inline)) {
                compute(j_c, j_c);
                __builtin_amdgcn_sched_barrier(0);   // keeps the quads' LDS reads from being hoisted (spills)
            });
        } else
        static_for<0, KC>([&](auto kc_c) __attribute__((always_inline)) {
            constexpr int kc = decltype(kc_c)::value;
            if constexpr (KC > 1) load_b(ct, kc);
            static_for<0, kQuads>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int j = decltype(j_c)::value;
                constexpr int s = kc * kQuads + j;   // step within the task; slots are s % R
                // loads R - 1 quads ahead into the slot staged last step, then stage the next quad
                constexpr int s2 = s + R - 1, s1 = s + 1;
                if constexpr (s2 < KC * kQuads) issue(task, s2 / kQuads, s2 % kQuads, IC<s2 % R>{});
                else issue(nxt, (s2 - KC * kQuads) / kQuads, (s2 - KC * kQuads) % kQuads, IC<s2 % R>{});
                compute(j_c, IC<s % R>{});   // quad j from slot s % R
                if constexpr (s1 < KC * kQuads) stage(s1 / kQuads, IC<s1 % R>{});
                else stage(0, IC<s1 % R>{});   // the next task's quad 0
                bar_lds();
            });
        });
        const int64_t tile = tile_of(task);
        // epilogue: C/D row (game) = 4g + i, column (channel) = r
        const int co = ct * 16 + r;
        if (co < a.cout) {
            const float bv = a.bias ? a.bias[co] : 0.f;
            const float al = a.alpha ? a.alpha[co] : 1.f;
            const float be = a.alpha ? a.beta[co] : 0.f;
            static_for<0, 4>([&](auto i_c) __attribute__((always_inline)) {
                constexpr int i = decltype(i_c)::value;
                const int64_t n = tile * 16 + 4 * g + i;
                if (n < a.N) {
                    float *yo = a.y + n * a.ys + (int64_t)co * kHW;
                    static_for<Q0, Q1>([&](auto j_c) __attribute__((always_inline)) {
                        constexpr int j = decltype(j_c)::value;
                        float o[4];
                        static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
                            constexpr int u = decltype(u_c)::value;
                            float v = acc[4 * (j - Q0) + u][i];
                            if (a.bias) v = v + bv;
                            if (a.alpha) v = v * al + be;
                            if (a.relu) v = relu_f(v);
                            o[u] = v;
                        });
                        *reinterpret_cast<float4 *>(yo + 4 * j) = make_float4(o[0], o[1], o[2], o[3]);
                    });
                }
            });
        }
        static_for<0, NCELL>([&](auto q_c) __attribute__((always_inline)) {
            acc[decltype(q_c)::value] = (f32x4){0.f, 0.f, 0.f, 0.f};
        });
    }
}

// A workgroup's 4 waves share one 16-game tile per task: each stages a quarter of every quad (16 games x 32
// channels x 4 cells, split once into the LDS ring) and computes NCTW column tiles x (4 / NCTW) output bands.
// R: the ring's quads (loads R - 1 quads ahead).  3 when workgroups walk several tasks (the next task's loads
// overlap this one's MFMAs); 9 -- a whole 32-channel k-step (108 KB) -- when every workgroup has one task (few
// games: the learner's per-step 256), so all of it is in flight at once instead of one HBM latency per quad.
template <int KC, bool PADC, int NCTW, int R>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void gboard_conv_kernel(GbArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[R * kSlotBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwg = gridDim.x, b = blockIdx.x;
    // consecutive logical workgroups (which share game tiles) on one XCD (hardware deals b round robin)
    const int L = (nwg % 8 == 0) ? (b & 7) * (nwg >> 3) + (b >> 3) : b;
    constexpr int NB = 4 / NCTW;
    const int band = wave / NCTW;
    if constexpr (NB == 1) {
        gboard_run<KC, PADC, NCTW, 0, R>(a, smem, lane, wave, L);
    } else if constexpr (NB == 2) {
        if (band == 0) gboard_run<KC, PADC, NCTW, 0, R>(a, smem, lane, wave, L);
        else gboard_run<KC, PADC, NCTW, 1, R>(a, smem, lane, wave, L);
    } else {
        switch (band) {
        case 0: gboard_run<KC, PADC, NCTW, 0, R>(a, smem, lane, wave, L); break;
        case 1: gboard_run<KC, PADC, NCTW, 1, R>(a, smem, lane, wave, L); break;
        case 2: gboard_run<KC, PADC, NCTW, 2, R>(a, smem, lane, wave, L); break;
        default: gboard_run<KC, PADC, NCTW, 3, R>(a, smem, lane, wave, L); break;
        }
    }
}

// W (Cout, w_cin_total, 3, 3), input channels [w_ci0, w_ci0 + cin_g) -> split fragments [ct][kc][tap][part][64]
// x 4 words: lane l of (ct, kc) holds W^T[ci = 32kc + 8(l>>4) + e][co = 16ct + (l&15)], e = 2d, 2d+1 in word d
// flip: the adjoint (input-gradient) conv of W's input slice, W'[co'][ci'][tap] = W[ci'][w_ci0 + co'][8 - tap]
// (cout = the slice width, cin_g = W's output channels)
__global__ void gboard_pack_kernel(const float *__restrict__ w, int cout, int cin_g, int w_cin_total, int w_ci0,
                                   int KC, int total, int flip, uint32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int d = i & 3, l = (i >> 2) & 63;
    int rest = i >> 8;
    const int part = rest % 3;
    rest /= 3;
    const int tap = rest % kTaps;
    rest /= kTaps;
    const int kc = rest % KC, ct = rest / KC;
    const int co = 16 * ct + (l & 15);
    const int ci = 32 * kc + 8 * (l >> 4) + 2 * d;
    auto wv = [&](int c) -> float {
        if (!(co < cout && c < cin_g)) return 0.f;
        return flip ? w[((int64_t)c * w_cin_total + w_ci0 + co) * kTaps + (kTaps - 1 - tap)]
                    : w[((int64_t)co * w_cin_total + w_ci0 + c) * kTaps + tap];
    };
    out[i] = hrl_split::split_part(wv(ci), part) | (hrl_split::split_part(wv(ci + 1), part) << 16);
}

// 1x1 convolution over the 6x6 board's channels (GeisterNet's move head conv2 8 -> 4 and the value / return heads'
// conv 64 -> 1 each, geister.py:238-264): y[n, o, q] = sum_c w[o, c] x[n, c, q] over x1's C1 channels then x2's
// C2 (the heads' [h_e, h_last] read in place), then the optional BatchNorm apply (y*alpha + beta) and ReLU.
// HBM-bound: a thread per (game, cell) walks the channels (consecutive threads read consecutive cells) with
// its O sums in registers, channels in order.
template <int O>
__global__ __launch_bounds__(256) void pointwise_kernel(const float *__restrict__ x1, int64_t s1, int C1,
                                                        const float *__restrict__ x2, int64_t s2, int C2,
                                                        const float *__restrict__ w, const float *__restrict__ alpha,
                                                        const float *__restrict__ beta, int relu,
                                                        float *__restrict__ y, int64_t ys, int64_t N) {
    __shared__ float ws[O * 128];
    const int C = C1 + C2;
    for (int i = threadIdx.x; i < O * C; i += blockDim.x) ws[i] = w[i];
    __syncthreads();
    const int64_t total = N * kHW;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = e / kHW;
        const int q = (int)(e - n * kHW);
        float acc[O];
#pragma unroll
        for (int o = 0; o < O; ++o) acc[o] = 0.f;
        const float *xp = x1 + n * s1 + q;
        for (int c = 0; c < C1; ++c) {
            const float v = xp[c * kHW];
#pragma unroll
            for (int o = 0; o < O; ++o) acc[o] = acc[o] + ws[o * C + c] * v;
        }
        if (x2) {
            const float *xq = x2 + n * s2 + q;
            for (int c = 0; c < C2; ++c) {
                const float v = xq[c * kHW];
#pragma unroll
                for (int o = 0; o < O; ++o) acc[o] = acc[o] + ws[o * C + C1 + c] * v;
            }
        }
#pragma unroll
        for (int o = 0; o < O; ++o) {
            float v = acc[o];
            if (alpha) v = v * alpha[o] + beta[o];
            if (relu) v = relu_f(v);
            y[n * ys + o * kHW + q] = v;
        }
    }
}

// ------------------------------------------------------------------ weight gradient, games as the MFMA K
// gboard_wgrad_kernel: the batched weight (and bias) gradient of a 3x3 'same' conv on the 6x6 board over every use
// recorded in a recurrent unroll (nn.DeferredGrads.flush; handyrl/train.py:155-174 runs the net T times):
//     dW[co][ci][tap] = sum_n sum_q dY[n][co][q] X[n][ci][p(q, tap)],   db[co] = sum_n sum_q dY[n][co][q]
// For a 16-game tile and one (output cell q, tap) pair the sum over the tile's games is one 32x32x16 MFMA block:
// A = dY_q (32 co x 16 games), B = X_p (16 games x 32 ci), both as the exact bf16 split (six products,
// fp32-accurate).  A workgroup (4 waves) owns up to four (32-co, 32-ci) units: with 4 units each wave takes one
// unit and all 9 taps (144 accumulators), with fewer the waves of a unit split its taps.  It walks 16-game tiles
// (grid-stride over every recorded segment, no concatenation) one board row of output cells at a time: the
// row's dY cells and the next input row are staged into LDS as part images [cell][part][half][channel][8 games]
// (a lane's 8 games of one channel are one conflict-free ds_read_b128), input rows in a ring of three.  Each
// workgroup writes its partial dW / db; gboard_wgrad_reduce_kernel folds them in a fixed order (deterministic)
// and ADDS the result into the gradient tensor's input-channel slice.
constexpr int kWgSegs = 64;
struct WgArgs {
    const float *x[kWgSegs];
    const float *dy[kWgSegs];
    int64_t xs[kWgSegs], dys[kWgSegs];   // floats from one game to the next
    int64_t n[kWgSegs];
    int64_t tile0[kWgSegs + 1];          // first global 16-game tile of each segment
    int nseg;
    int cout, cin;                       // output channels, input channels of the slice (x holds them contiguous)
    int cto, cti;                        // 32-channel tiles
    float *part;                         // [block][cto*cti][9][32][32] then [block][cto*32] bias sums
    int bias;
};
constexpr int kWgCellPart = 1024;                       // one part of one cell: [half][32 ch][8 games] bf16
constexpr int kWgCell = 3 * kWgCellPart;                // h, m, l
constexpr int kWgRow = 6 * kWgCell;                     // one board row of one 32-channel tile (18 KB)

template <int CTO, int CTI, int TPH>
__device__ __forceinline__ void gboard_wgrad_run(const WgArgs &a, unsigned char *smem, int lane, int wave) {
    // LDS: dY row [cto][6 cells] then the input-row ring [3][cti][6 cells]
    constexpr int U = CTO * CTI;
    constexpr int WPU = 4 / U;                            // waves per unit: they split the unit's taps (TPH)
    const int unit = wave % U;
    const int uco = unit / CTI, uci = unit % CTI;         // the unit's 32-channel tiles
    unsigned char *dy_img = smem;
    unsigned char *x_img = smem + CTO * kWgRow;
    const int64_t ntiles = a.tile0[a.nseg];
    f32x16 acc[9];
    static_for<0, 9>([&](auto t_c) __attribute__((always_inline)) {
        constexpr int t = decltype(t_c)::value;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    });
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};                 // bias partials of the staging items' channels
    // staging item k of this thread: (channel c, game pair jp) over nch channels x 8 pairs
    auto stage_rows = [&](const float *base, int64_t gs, int64_t n_in_tile, int nch_valid, auto ntile_c,
                          int cell0, unsigned char *img, auto is_dy_c) __attribute__((always_inline)) {
        // base: game 0 of the tile, channel 0, cell cell0 (6 cells of one board row)
        constexpr int ntile_ch = decltype(ntile_c)::value, nitems = ntile_ch;
        constexpr bool is_dy = decltype(is_dy_c)::value;
#pragma unroll
        for (int k = 0; k < nitems; ++k) {
            const int item = (int)threadIdx.x + 256 * k;
            const int c = item % (32 * ntile_ch), jp = item / (32 * ntile_ch);
            float v[2][6];
#pragma unroll
            for (int gi = 0; gi < 2; ++gi) {
                const int g = 2 * jp + gi;
                if (g < n_in_tile && c < nch_valid) {
                    const float *p = base + g * gs + (int64_t)c * kHW + cell0;
                    const float2 a0 = *reinterpret_cast<const float2 *>(p);
                    const float2 a1 = *reinterpret_cast<const float2 *>(p + 2);
                    const float2 a2 = *reinterpret_cast<const float2 *>(p + 4);
                    v[gi][0] = a0.x; v[gi][1] = a0.y; v[gi][2] = a1.x; v[gi][3] = a1.y; v[gi][4] = a2.x; v[gi][5] = a2.y;
                } else {
#pragma unroll
                    for (int e = 0; e < 6; ++e) v[gi][e] = 0.f;
                }
            }
            if constexpr (is_dy) {
#pragma unroll
                for (int e = 0; e < 6; ++e) bsum[k] += v[0][e] + v[1][e];
            }
            const int tile_ch = c >> 5, ch = c & 31, half = jp >> 2, sub = jp & 3;
            unsigned char *dst = img + tile_ch * kWgRow + ((half * 32 + ch) * 16 + 4 * sub);
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                uint32_t h0, m0, l0, h1, m1, l1;
                hrl_split::split3(v[0][e], h0, m0, l0);
                hrl_split::split3(v[1][e], h1, m1, l1);
                *reinterpret_cast<uint32_t *>(dst + e * kWgCell + 0 * kWgCellPart) = h0 | (h1 << 16);
                *reinterpret_cast<uint32_t *>(dst + e * kWgCell + 1 * kWgCellPart) = m0 | (m1 << 16);
                *reinterpret_cast<uint32_t *>(dst + e * kWgCell + 2 * kWgCellPart) = l0 | (l1 << 16);
            }
        }
    };
    constexpr int nitems_dy = CTO, nitems_x = CTI;       // items per thread (32 channels x 8 pairs per 256)
    const int h = lane >> 5, cl = lane & 31;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        int sg = 0;
        while (sg + 1 < a.nseg && a.tile0[sg + 1] <= tile) ++sg;
        const int64_t n0 = (tile - a.tile0[sg]) * 16;
        const int64_t nin = min<int64_t>(16, a.n[sg] - n0);
        const float *xb = a.x[sg] + n0 * a.xs[sg];
        const float *db = a.dy[sg] + n0 * a.dys[sg];
        // input rows 0 and 1 into ring slots 0 and 1
        stage_rows(xb, a.xs[sg], nin, a.cin, IC<CTI>{}, 0, x_img + 0 * CTI * kWgRow, std::false_type{});
        stage_rows(xb, a.xs[sg], nin, a.cin, IC<CTI>{}, 6, x_img + 1 * CTI * kWgRow, std::false_type{});
        for (int r = 0; r < 6; ++r) {
            stage_rows(db, a.dys[sg], nin, a.cout, IC<CTO>{}, 6 * r, dy_img, std::true_type{});
            if (r + 1 < 6)
                stage_rows(xb, a.xs[sg], nin, a.cin, IC<CTI>{}, 6 * (r + 1), x_img + ((r + 1) % 3) * CTI * kWgRow,
                           std::false_type{});
            __syncthreads();
            // the row's (q, tap) pairs: A = dY_q (co = lane & 31, games 8h..8h+7), B = X_p (ci = lane & 31)
            const unsigned char *arow = dy_img + uco * kWgRow + (h * 32 + cl) * 16;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const uint4 Ah = *reinterpret_cast<const uint4 *>(arow + c * kWgCell + 0 * kWgCellPart);
                const uint4 Am = *reinterpret_cast<const uint4 *>(arow + c * kWgCell + 1 * kWgCellPart);
                const uint4 Al = *reinterpret_cast<const uint4 *>(arow + c * kWgCell + 2 * kWgCellPart);
                static_for<0, 9>([&](auto t_c) __attribute__((always_inline)) {
                    constexpr int t = decltype(t_c)::value;
                    if constexpr (t % WPU != TPH) return;
                    const int pr = r + t / 3 - 1, pc = c + t % 3 - 1;
                    if (pr < 0 || pr > 5 || pc < 0 || pc > 5) return;
                    const unsigned char *b = x_img + (pr % 3) * CTI * kWgRow + uci * kWgRow + pc * kWgCell +
                                             (h * 32 + cl) * 16;
                    const uint4 Bh = *reinterpret_cast<const uint4 *>(b + 0 * kWgCellPart);
                    const uint4 Bm = *reinterpret_cast<const uint4 *>(b + 1 * kWgCellPart);
                    const uint4 Bl = *reinterpret_cast<const uint4 *>(b + 2 * kWgCellPart);
                    f32x16 cc = acc[t];
                    cc = mfma32(Al, Bh, cc);   // smallest terms first
                    cc = mfma32(Am, Bm, cc);
                    cc = mfma32(Ah, Bl, cc);
                    cc = mfma32(Am, Bh, cc);
                    cc = mfma32(Ah, Bm, cc);
                    cc = mfma32(Ah, Bh, cc);
                    acc[t] = cc;
                });
            }
            __syncthreads();
        }
    }
    // partials: [block][unit][tap][co 32][ci 32]; C/D of 32x32x16: row (co) = (i&3) + 8(i>>2) + 4h, col (ci) = lane&31
    constexpr int nunits = U;
    float *outp = a.part + (int64_t)blockIdx.x * nunits * 9 * 1024 + (int64_t)unit * 9 * 1024;
    static_for<0, 9>([&](auto t_c) __attribute__((always_inline)) {
        constexpr int t = decltype(t_c)::value;
        if constexpr (t % WPU != TPH) return;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int co = (i & 3) + 8 * (i >> 2) + 4 * h;
            outp[(t * 32 + co) * 32 + cl] = acc[t][i];
        }
    });
    if (a.bias) {   // bias partials per channel: the staging threads' sums, folded through LDS in a fixed order
        __syncthreads();
        float *red = reinterpret_cast<float *>(smem);
#pragma unroll
        for (int k = 0; k < nitems_dy; ++k) red[threadIdx.x + 256 * k] = bsum[k];
        __syncthreads();
        const int nch = 32 * CTO;
        float *bp = a.part + (int64_t)gridDim.x * nunits * 9 * 1024 + (int64_t)blockIdx.x * nch;
        for (int c = threadIdx.x; c < nch; c += 256) {
            float t = 0.f;
            for (int i = c; i < 256 * nitems_dy; i += nch) t += red[i];   // items with channel c, pair order
            bp[c] = t;
        }
    }
}

template <int CTO, int CTI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gboard_wgrad_kernel(WgArgs a) {
    static_assert((CTO + 3 * CTI) * kWgRow <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) unsigned char smem[(CTO + 3 * CTI) * kWgRow];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int U = CTO * CTI;
    const int tph = wave / U;
    if constexpr (U == 4) {
        gboard_wgrad_run<CTO, CTI, 0>(a, smem, lane, wave);
    } else if constexpr (U == 2) {
        if (tph == 0) gboard_wgrad_run<CTO, CTI, 0>(a, smem, lane, wave);
        else gboard_wgrad_run<CTO, CTI, 1>(a, smem, lane, wave);
    } else {
        switch (tph) {
        case 0: gboard_wgrad_run<CTO, CTI, 0>(a, smem, lane, wave); break;
        case 1: gboard_wgrad_run<CTO, CTI, 1>(a, smem, lane, wave); break;
        case 2: gboard_wgrad_run<CTO, CTI, 2>(a, smem, lane, wave); break;
        default: gboard_wgrad_run<CTO, CTI, 3>(a, smem, lane, wave); break;
        }
    }
}

// fold the per-workgroup partials in block order and add into dst (the gradient of weight (Cout, w_cin_total, 3,
// 3), input channels [ci0, ci0 + cin)) and, with a bias, into dbias.  Thread i reads element i of every
// workgroup's [unit][tap][32 co][32 ci] slab (consecutive threads, consecutive addresses), four workgroup ranges
// per element over the block's waves, folded in range order through LDS (deterministic).
__global__ __launch_bounds__(256) void gboard_wgrad_reduce_kernel(const float *__restrict__ part, int blocks, int cto,
                                                                  int cti, int cout, int cin, int w_cin_total,
                                                                  int ci0, float *__restrict__ dst,
                                                                  float *__restrict__ dbias) {
    __shared__ float red[4][64];
    const int nunits = cto * cti;
    const int64_t slab = (int64_t)nunits * 9 * 1024;
    const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;   // element of the slab
    const int per = (blocks + 3) / 4;
    const int b0 = r * per, b1 = min(blocks, b0 + per);
    float s0 = 0.f, s1 = 0.f;
    if (e < slab) {
        int b = b0;
        for (; b + 1 < b1; b += 2) {
            s0 += part[(int64_t)b * slab + e];
            s1 += part[(int64_t)(b + 1) * slab + e];
        }
        if (b < b1) s0 += part[(int64_t)b * slab + e];
    }
    red[r][lane] = s0 + s1;
    __syncthreads();
    if (r == 0 && e < slab) {
        const float v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        const int ci_l = (int)(e & 31), co_l = (int)((e >> 5) & 31);
        const int tap = (int)((e >> 10) % 9), unit = (int)(e / (9 * 1024));
        const int co = (unit / cti) * 32 + co_l, ci = (unit % cti) * 32 + ci_l;
        if (co < cout && ci < cin) {
            float *d = dst + ((int64_t)co * w_cin_total + ci0 + ci) * 9 + tap;
            *d = *d + v;
        }
    }
    if (dbias && blockIdx.x == 0) {
        const float *bp = part + (int64_t)blocks * slab;
        const int nch = 32 * cto;
        for (int i = threadIdx.x; i < cout; i += 256) {
            float t = 0.f;
            for (int b = 0; b < blocks; ++b) t += bp[(int64_t)b * nch + i];
            dbias[i] = dbias[i] + t;
        }
    }
}

// The weight gradient of a 1x1 conv on the board (the heads' pointwise convs in the learner):
//     dW[o][c] = sum over games n and cells q of dy[n][o][q] * x[n][c][q]
// HBM-bound (x is read once).  Thread (slot, c) of a workgroup walks games slot, slot + slots, ... of the
// workgroup's range, summing each game's 36-cell dot products in cell order; the slots are folded in LDS and each
// workgroup writes its O x C partial, which pw_wgrad_reduce_kernel folds in block order (deterministic).
constexpr int kPwMaxO = 8;
__global__ __launch_bounds__(256) void pw_wgrad_kernel(const float *__restrict__ x, int64_t xs,
                                                       const float *__restrict__ dy, int64_t dys, int64_t N, int C,
                                                       int O, int64_t games_per_block, float *__restrict__ part) {
    __shared__ float red[256 * kPwMaxO];
    const int t = threadIdx.x;
    const int slots = 256 / C;
    const int slot = t / C, c = t % C;
    float acc[kPwMaxO];
#pragma unroll
    for (int o = 0; o < kPwMaxO; ++o) acc[o] = 0.f;
    const int64_t n0 = (int64_t)blockIdx.x * games_per_block;
    const int64_t n1 = min(n0 + games_per_block, N);
    if (slot < slots) {
        for (int64_t n = n0 + slot; n < n1; n += slots) {
            const float4 *xr = reinterpret_cast<const float4 *>(x + n * xs + (int64_t)c * kHW);
            float4 xv[kQuads];
#pragma unroll
            for (int k = 0; k < kQuads; ++k) xv[k] = xr[k];
#pragma unroll
            for (int o = 0; o < kPwMaxO; ++o) {
                if (o < O) {
                    const float4 *dr = reinterpret_cast<const float4 *>(dy + n * dys + (int64_t)o * kHW);
                    float d = 0.f;
#pragma unroll
                    for (int k = 0; k < kQuads; ++k) {
                        const float4 g = dr[k];
                        d += g.x * xv[k].x;
                        d += g.y * xv[k].y;
                        d += g.z * xv[k].z;
                        d += g.w * xv[k].w;
                    }
                    acc[o] += d;
                }
            }
        }
    }
#pragma unroll
    for (int o = 0; o < kPwMaxO; ++o) red[o * 256 + t] = acc[o];
    __syncthreads();
    if (t < C) {
        for (int o = 0; o < O; ++o) {
            float v = 0.f;
            for (int sl = 0; sl < slots; ++sl) v += red[o * 256 + sl * C + t];
            part[((int64_t)blockIdx.x * O + o) * C + t] = v;
        }
    }
}

__global__ __launch_bounds__(256) void pw_wgrad_reduce_kernel(const float *__restrict__ part, int blocks, int OC,
                                                              float *__restrict__ dw) {
    // element i = blockIdx.x * 64 + lane; the block's four waves sum four workgroup ranges, folded in order
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const int per = (blocks + 3) / 4;
    const int b0 = r * per, b1 = min(blocks, b0 + per);
    float s0 = 0.f, s1 = 0.f;
    if (i < OC) {
        int b = b0;
        for (; b + 1 < b1; b += 2) {
            s0 += part[(int64_t)b * OC + i];
            s1 += part[(int64_t)(b + 1) * OC + i];
        }
        if (b < b1) s0 += part[(int64_t)b * OC + i];
    }
    red[r][lane] = s0 + s1;
    __syncthreads();
    if (r == 0 && i < OC) dw[i] = dw[i] + (((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
}

int g_gboard_whole = 1;   // hrl_gboard_set_whole_ring
int g_gboard_nctw = 0;    // hrl_gboard_set_nctw: 0 = the launcher's choice
// hrl_gboard_launch_stats: which forms the launchers chose since the last reset (host-side counters, one thread)
enum { kStConv, kStWhole, kStNctw1, kStNctw2, kStNctw4, kStGroups4, kStFwdGroups, kStWgrad, kStWgradMaxSegs,
       kStWgradMaxTiles, kStWgradMultiTile, kStCount };
int64_t g_gboard_stats[kStCount] = {};

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

// k-steps of 32 input channels: 1, 2 or 4 (Cin_g <= 64 or 97..128)
bool kc_ok(int64_t Cin_g) { return Cin_g >= 1 && (Cin_g <= 64 || (Cin_g > 96 && Cin_g <= 128)); }

int64_t hrl_gboard_pack_bytes(int64_t Cout, int64_t Cin_g) {
    if (Cout < 1 || !kc_ok(Cin_g)) return -1;
    return ((Cout + 15) / 16) * ((Cin_g + 31) / 32) * kTaps * 3 * 64 * 16;
}

int hrl_gboard_pack(const float *weight, int64_t Cout, int64_t Cin_g, int64_t w_cin_total, int64_t w_ci0,
                    void *packed, int64_t packed_bytes, void *stream) {
    const int64_t need = hrl_gboard_pack_bytes(Cout, Cin_g);
    if (!weight || !packed || need < 0 || packed_bytes < need || w_ci0 < 0 || w_ci0 + Cin_g > w_cin_total)
        return HRL_EINVAL;
    const int KC = (int)((Cin_g + 31) / 32);
    const int total = (int)(need / 4);
    hipLaunchKernelGGL(gboard_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                       weight, (int)Cout, (int)Cin_g, (int)w_cin_total, (int)w_ci0, KC, total, 0,
                       static_cast<uint32_t *>(packed));
    return status();
}

int hrl_gboard_pack_adjoint(const float *weight, int64_t Cout_fwd, int64_t w_cin_total, int64_t w_ci0,
                            int64_t Cin_slice, void *packed, int64_t packed_bytes, void *stream) {
    const int64_t need = hrl_gboard_pack_bytes(Cin_slice, Cout_fwd);
    if (!weight || !packed || need < 0 || packed_bytes < need || w_ci0 < 0 || Cin_slice < 1 ||
        w_ci0 + Cin_slice > w_cin_total)
        return HRL_EINVAL;
    const int KC = (int)((Cout_fwd + 31) / 32);
    const int total = (int)(need / 4);
    hipLaunchKernelGGL(gboard_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                       weight, (int)Cin_slice, (int)Cout_fwd, (int)w_cin_total, (int)w_ci0, KC, total, 1,
                       static_cast<uint32_t *>(packed));
    return status();
}

int gboard_launch(GbArgs a, int64_t Cin_g, int64_t groups, hipStream_t s);

int hrl_gboard_forward_groups(const float *const *xs, const int64_t *x_strides, int64_t N, int64_t Cin_g,
                              int64_t groups, const void *packed, int64_t packed_bytes, int64_t Cout, float *y,
                              int64_t y_stride, void *stream) {
    if (!xs || !x_strides || !packed || !y || N < 1 || Cin_g < 1 || Cin_g > 32 || groups < 1 || groups > 4 ||
        Cout < 1 || Cout % groups || (Cout / groups) % 16)
        return HRL_EINVAL;
    // the kernel reads hrl_gboard_pack_bytes(Cout, Cin_g) bytes of split fragments: refuse a smaller buffer
    const int64_t need = hrl_gboard_pack_bytes(Cout, Cin_g);
    if (need < 0 || packed_bytes < need) return HRL_EINVAL;
    if (!aligned16(y) || y_stride % 4 || y_stride < Cout * kHW) return HRL_EINVAL;
    GbArgs a{};
    for (int g = 0; g < groups; ++g) {
        if (!xs[g] || !aligned16(xs[g]) || x_strides[g] % 4 || x_strides[g] < Cin_g * kHW) return HRL_EINVAL;
        a.xg[g] = xs[g];
        a.xgs[g] = x_strides[g];
    }
    a.x = xs[0]; a.N = N; a.xs = x_strides[0];
    a.cin_g = (int)Cin_g; a.cout_g = (int)(Cout / groups);
    a.wpk = static_cast<const uint4 *>(packed);
    a.nct = (int)((Cout + 15) / 16); a.cout = (int)Cout;
    a.y = y; a.ys = y_stride;
    ++g_gboard_stats[kStFwdGroups];
    return gboard_launch(a, Cin_g, groups, static_cast<hipStream_t>(stream));
}

int hrl_gboard_forward(const float *x, int64_t x_stride, const float *x2, int64_t x2_stride, int64_t N, int64_t Cin_g,
                       int64_t groups, const void *packed, int64_t packed_bytes, int64_t Cout, const float *bias,
                       const float *alpha, const float *beta, int relu, float *y, int64_t y_stride, void *stream) {
    if (!x || !packed || !y || N < 1 || !kc_ok(Cin_g) || groups < 1 || Cout < 1 || Cout % groups)
        return HRL_EINVAL;
    const int64_t need = hrl_gboard_pack_bytes(Cout, Cin_g);   // the split fragments the kernel reads
    if (need < 0 || packed_bytes < need) return HRL_EINVAL;
    const int64_t cout_g = Cout / groups;
    if (groups > 1 && cout_g % 16) return HRL_EINVAL;        // a column tile never straddles two groups
    if (x2 && (Cin_g <= 32 || Cin_g > 64 || groups != 1)) return HRL_EINVAL;
    if ((alpha == nullptr) != (beta == nullptr)) return HRL_EINVAL;
    if (!aligned16(x) || (x2 && !aligned16(x2)) || !aligned16(y) || x_stride % 4 || x2_stride % 4 || y_stride % 4)
        return HRL_EINVAL;
    if (x_stride < (x2 ? 32 : Cin_g * groups) * kHW || y_stride < Cout * kHW || (x2 && x2_stride < (Cin_g - 32) * kHW))
        return HRL_EINVAL;
    GbArgs a{};
    a.x = x; a.x2 = x2; a.N = N; a.xs = x_stride; a.xs2 = x2_stride;
    a.cin_g = (int)Cin_g; a.cout_g = (int)cout_g;
    a.wpk = static_cast<const uint4 *>(packed);
    a.nct = (int)((Cout + 15) / 16); a.cout = (int)Cout;
    a.bias = bias; a.alpha = alpha; a.beta = beta; a.relu = relu; a.y = y; a.ys = y_stride;
    return gboard_launch(a, Cin_g, groups, static_cast<hipStream_t>(stream));
}

int gboard_launch(GbArgs a, int64_t Cin_g, int64_t groups, hipStream_t s) {
    const int64_t N = a.N, cout_g = a.cout_g;
    const int64_t ntiles = (N + 15) / 16;
    // column tiles per workgroup (NCTW = 4, 2, 1; the other waves split the output cells into 4 / NCTW bands):
    // the fewest task rounds per band over the chip's 256 CUs (one 4-wave workgroup each), ties to the wider
    // NCTW (fewer workgroups stage each tile)
    int nctw = 1;
    double best = 1e30;
    for (int c = 4; c >= 1; c >>= 1) {
        if (a.nct % c || (groups > 1 && (cout_g / 16) % c)) continue;   // a workgroup's tiles share one group
        const int64_t tasks = ntiles * (a.nct / c);
        const double rounds = (double)((tasks + kCUs - 1) / kCUs) * c / 4.0;
        if (rounds < best - 1e-9) { best = rounds; nctw = c; }
    }
    if (g_gboard_nctw > 0 && a.nct % g_gboard_nctw == 0 && !(groups > 1 && (cout_g / 16) % g_gboard_nctw))
        nctw = g_gboard_nctw;   // hrl_gboard_set_nctw (measurement)
    const int64_t tasks = ntiles * (a.nct / nctw);
    int grid = (int)(tasks < kCUs ? tasks : kCUs);
    const dim3 block(kThreads);
    const int KC = (int)((Cin_g + 31) / 32);
    const bool padc = Cin_g % 32 != 0;
#define HRL_GB_LAUNCH_R(KC_, PADC_, R_)                                                                          \
    do {                                                                                                         \
        if (nctw == 4) hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 4, R_>), dim3(grid), block, 0, s, a);  \
        else if (nctw == 2)                                                                                      \
            hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 2, R_>), dim3(grid), block, 0, s, a);             \
        else hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 1, R_>), dim3(grid), block, 0, s, a);            \
    } while (0)
#define HRL_GB_LAUNCH(KC_, PADC_)                                                                                \
    do {                                                                                                         \
        if (whole) HRL_GB_LAUNCH_R(KC_, PADC_, ((KC_) == 1 ? 9 : 3)); else HRL_GB_LAUNCH_R(KC_, PADC_, 3);      \
    } while (0)
    // one task per workgroup: the whole k-step ring (see gboard_conv_kernel)
    const bool whole = tasks <= kCUs && g_gboard_whole && KC == 1;
    ++g_gboard_stats[kStConv];
    g_gboard_stats[kStWhole] += whole;
    ++g_gboard_stats[nctw == 1 ? kStNctw1 : (nctw == 2 ? kStNctw2 : kStNctw4)];
    g_gboard_stats[kStGroups4] += groups == 4;
    if (KC == 1) {
        if (padc) HRL_GB_LAUNCH(1, true); else HRL_GB_LAUNCH(1, false);
    } else if (KC == 2) {
        if (padc) HRL_GB_LAUNCH(2, true); else HRL_GB_LAUNCH(2, false);
    } else {
        if (padc) HRL_GB_LAUNCH(4, true); else HRL_GB_LAUNCH(4, false);
    }
#undef HRL_GB_LAUNCH_R
#undef HRL_GB_LAUNCH
    return status();
}

int64_t hrl_gboard_wgrad_workspace_bytes(int64_t Cout, int64_t Cin, int64_t total_games) {
    if (Cout < 1 || Cin < 1 || total_games < 1) return -1;
    const int64_t cto = (Cout + 31) / 32, cti = (Cin + 31) / 32;
    // the instantiated (32-channel) tile shapes: (co, ci) tiles 4x1, 2x2, 2x1, 1x2, 1x1
    if (!((cto == 4 && cti == 1) || (cto <= 2 && cti <= 2))) return -1;
    const int64_t tiles = (total_games + 15) / 16;
    const int64_t blocks = tiles < kCUs ? tiles : kCUs;
    return blocks * (cto * cti * 9 * 1024 + 32 * cto) * 4;
}

int hrl_gboard_wgrad(const float *const *xs, const int64_t *x_strides, const float *const *dys,
                     const int64_t *dy_strides, const int64_t *ns, int nseg, int64_t Cout, int64_t Cin,
                     float *dweight, int64_t w_cin_total, int64_t w_ci0, float *dbias, void *workspace,
                     int64_t workspace_bytes, void *stream) {
    if (nseg < 1 || nseg > kWgSegs || !xs || !dys || !ns || !x_strides || !dy_strides || !dweight || !workspace)
        return HRL_EINVAL;
    if (w_ci0 < 0 || w_ci0 + Cin > w_cin_total) return HRL_EINVAL;
    WgArgs a{};
    int64_t tiles = 0, games = 0;
    for (int i = 0; i < nseg; ++i) {
        if (!xs[i] || !dys[i] || ns[i] < 1 || (reinterpret_cast<uintptr_t>(xs[i]) & 7) ||
            (reinterpret_cast<uintptr_t>(dys[i]) & 7) || x_strides[i] % 2 || dy_strides[i] % 2 ||
            x_strides[i] < Cin * kHW || dy_strides[i] < Cout * kHW)
            return HRL_EINVAL;
        a.x[i] = xs[i]; a.dy[i] = dys[i]; a.xs[i] = x_strides[i]; a.dys[i] = dy_strides[i]; a.n[i] = ns[i];
        a.tile0[i] = tiles;
        tiles += (ns[i] + 15) / 16;
        games += ns[i];
    }
    a.tile0[nseg] = tiles;
    // one partial per workgroup, one workgroup per 16-game tile of a segment (each segment rounds up on its own)
    (void)games;
    const int64_t need = hrl_gboard_wgrad_workspace_bytes(Cout, Cin, tiles * 16);
    if (need < 0 || workspace_bytes < need) return HRL_EINVAL;
    a.nseg = nseg; a.cout = (int)Cout; a.cin = (int)Cin;
    a.cto = (int)((Cout + 31) / 32); a.cti = (int)((Cin + 31) / 32);
    a.part = static_cast<float *>(workspace);
    a.bias = dbias != nullptr;
    const int blocks = (int)(tiles < kCUs ? tiles : kCUs);
    ++g_gboard_stats[kStWgrad];
    g_gboard_stats[kStWgradMaxSegs] = std::max<int64_t>(g_gboard_stats[kStWgradMaxSegs], nseg);
    g_gboard_stats[kStWgradMaxTiles] = std::max<int64_t>(g_gboard_stats[kStWgradMaxTiles], tiles);
    g_gboard_stats[kStWgradMultiTile] += tiles > blocks;   // workgroups carrying accumulators over several tiles
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (a.cto == 4 && a.cti == 1) hipLaunchKernelGGL((gboard_wgrad_kernel<4, 1>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.cto == 2 && a.cti == 2) hipLaunchKernelGGL((gboard_wgrad_kernel<2, 2>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.cto == 2 && a.cti == 1) hipLaunchKernelGGL((gboard_wgrad_kernel<2, 1>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.cto == 1 && a.cti == 2) hipLaunchKernelGGL((gboard_wgrad_kernel<1, 2>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((gboard_wgrad_kernel<1, 1>), dim3(blocks), dim3(256), 0, s, a);
    int rc = status();
    if (rc) return rc;
    const int64_t slab = (int64_t)a.cto * a.cti * 9 * 1024;
    hipLaunchKernelGGL(gboard_wgrad_reduce_kernel, dim3((unsigned)((slab + 63) / 64)), dim3(256), 0, s, a.part, blocks, a.cto,
                       a.cti, (int)Cout, (int)Cin, (int)w_cin_total, (int)w_ci0, dweight, dbias);
    return status();
}

int hrl_gboard_set_nctw(int nctw) {
    const int prev = g_gboard_nctw;
    g_gboard_nctw = (nctw == 1 || nctw == 2 || nctw == 4) ? nctw : 0;
    return prev;
}

int hrl_gboard_launch_stats(int64_t *counts, int n, int reset) {
    const int m = counts ? std::min(n, (int)kStCount) : 0;
    for (int i = 0; i < m; ++i) counts[i] = g_gboard_stats[i];
    if (reset)
        for (int i = 0; i < kStCount; ++i) g_gboard_stats[i] = 0;
    return kStCount;
}

int hrl_gboard_set_whole_ring(int on) {
    const int prev = g_gboard_whole;
    g_gboard_whole = on ? 1 : 0;
    return prev;
}

int64_t hrl_gboard_pointwise_wgrad_workspace_bytes(int64_t C, int64_t O, int64_t N) {
    if (C < 1 || C > 256 || O < 1 || O > kPwMaxO || N < 1) return -1;
    const int64_t blocks = N < 2 * kCUs ? N : 2 * kCUs;
    return blocks * O * C * 4;
}

int hrl_gboard_pointwise_wgrad(const float *x, int64_t x_stride, const float *dy, int64_t dy_stride, int64_t N,
                               int64_t C, int64_t O, float *dweight, void *workspace, int64_t workspace_bytes,
                               void *stream) {
    const int64_t need = hrl_gboard_pointwise_wgrad_workspace_bytes(C, O, N);
    if (!x || !dy || !dweight || !workspace || need < 0 || workspace_bytes < need) return HRL_EINVAL;
    if (!aligned16(x) || !aligned16(dy) || x_stride % 4 || dy_stride % 4 || x_stride < C * kHW ||
        dy_stride < O * kHW)
        return HRL_EINVAL;
    const int64_t blocks = N < 2 * kCUs ? N : 2 * kCUs;
    const int64_t per = (N + blocks - 1) / blocks;
    hipStream_t s = static_cast<hipStream_t>(stream);
    float *part = static_cast<float *>(workspace);
    hipLaunchKernelGGL(pw_wgrad_kernel, dim3((int)blocks), dim3(256), 0, s, x, x_stride, dy, dy_stride, N, (int)C,
                       (int)O, per, part);
    int rc = status();
    if (rc) return rc;
    const int OC = (int)(O * C);
    hipLaunchKernelGGL(pw_wgrad_reduce_kernel, dim3((OC + 63) / 64), dim3(256), 0, s, part, (int)blocks, OC,
                       dweight);
    return status();
}

int hrl_gboard_pointwise(const float *x1, int64_t x1_stride, int64_t C1, const float *x2, int64_t x2_stride,
                          int64_t C2, int64_t N, const float *weight, int64_t O, const float *alpha, const float *beta,
                          int relu, float *y, int64_t y_stride, void *stream) {
    if (!x1 || !weight || !y || N < 1 || C1 < 1 || C2 < 0 || (C2 > 0) != (x2 != nullptr) || C1 + C2 > 128 ||
        (O != 1 && O != 2 && O != 4 && O != 8) || (alpha == nullptr) != (beta == nullptr))
        return HRL_EINVAL;
    if (x1_stride < C1 * kHW || (x2 && x2_stride < C2 * kHW) || y_stride < O * kHW) return HRL_EINVAL;
    const int64_t total = N * kHW;
    const int grid = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define HRL_PW(O_)                                                                                                \
    hipLaunchKernelGGL(pointwise_kernel<O_>, dim3(grid), dim3(256), 0, s, x1, x1_stride, (int)C1, x2, x2_stride,  \
                       (int)C2, weight, alpha, beta, relu, y, y_stride, N)
    if (O == 1) HRL_PW(1); else if (O == 2) HRL_PW(2); else if (O == 4) HRL_PW(4); else HRL_PW(8);
#undef HRL_PW
    return status();
}

}  // extern "C"
