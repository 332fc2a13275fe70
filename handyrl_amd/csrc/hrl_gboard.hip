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
    int cin_g, cout_g;     // input / output channels per group
    const uint4 *wpk;      // split weight fragments [ct][kc][tap][part][64]
    int nct, cout;         // 16-channel column tiles; output channels stored
    const float *bias, *alpha, *beta;
    int relu;
    float *y;
    int64_t ys;            // floats from one game to the next in y
    // GATES (hrl_gboard_lstm_forward): the conv is the ConvLSTM cells' h halves (groups = layers, 4H outputs per
    // layer in i, f, o, g order); the epilogue forms the gates with the x halves zx (+ bias) and the cell state
    // instead of storing the conv: c' = sig(f) c + sig(i) tanh(g), h' = sig(o) tanh(c') (lstm_fwd_kernel's ops)
    const float *zx;       // (N, layers*4H, 36), games zxs floats apart
    int64_t zxs;
    const float *c_in;     // (N, layers*H, 36), games cs floats apart; c_out may be c_in (same element, same lane)
    float *c_out, *h_out;  // h_out never aliases x (other workgroups still read it)
    int64_t cs, hs;
    int nh;                // H / 16: column tiles per gate
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
// GATES: the four gate waves exchange a 12-cell chunk of their accumulators [gate][cell][row i][lane] (48 KB)
constexpr int kGateChunk = 12;
constexpr int kXchgBytes = 4 * kGateChunk * 4 * 64 * 4;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }   // lstm_fwd_kernel's

// One wave of gboard_conv_kernel: column tile (task's tile group * NCTW + ctl), output band BAND of NB = 4 / NCTW.
template <int KC, bool PADC, int NCTW, int BAND, bool GATES = false>
__device__ __forceinline__ void gboard_run(const GbArgs &a, unsigned char *smem, int lane, int wave, int L) {
    static_assert(!GATES || (NCTW == 4 && KC == 1 && !PADC), "the gate epilogue: one gate per wave");
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
    // GATES: task group ctg = (layer, hidden block hb); wave ctl takes gate ctl's column tile of that block
    auto ct_of = [&](int64_t t) {
        const int ctg = (int)(t % n_ctg);
        if constexpr (GATES) return (ctg / a.nh) * 4 * a.nh + ctl * a.nh + ctg % a.nh;
        return ctg * NCTW + ctl;
    };
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
        return a.x + n * a.xs + (int64_t)(grp * a.cin_g) * kHW;
    };
    float4 raw[3][2];
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
    // prologue: quad 0 staged, quad 1 in flight
    issue(task, 0, 0, IC<0>{});
    issue(task, 0, 1, IC<1>{});
    stage(0, IC<0>{});
    int ct_b = -1;
    bar_lds();
    for (; task < ntasks; task += step) {
        const int64_t nxt = task + step < ntasks ? task + step : task;   // loads past the end: re-read
        const int ct = ct_of(task);
        if (KC == 1 && ct != ct_b) load_b(ct, 0);
        ct_b = ct;
        static_for<0, KC>([&](auto kc_c) __attribute__((always_inline)) {
            constexpr int kc = decltype(kc_c)::value;
            if constexpr (KC > 1) load_b(ct, kc);
            static_for<0, kQuads>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int j = decltype(j_c)::value;
                constexpr int s = kc * kQuads + j;   // step within the task; slots are s % 3 (kQuads % 3 == 0)
                // loads two quads ahead into the slot staged last step, then stage the next quad
                constexpr int s2 = s + 2, s1 = s + 1;
                if constexpr (s2 < KC * kQuads) issue(task, s2 / kQuads, s2 % kQuads, IC<s2 % 3>{});
                else issue(nxt, (s2 - KC * kQuads) / kQuads, (s2 - KC * kQuads) % kQuads, IC<s2 % 3>{});
                // compute quad j from slot s % 3
                const unsigned char *img = smem + (s % 3) * kSlotBytes + r * 64 + g * 16;
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
                if constexpr (s1 < KC * kQuads) stage(s1 / kQuads, IC<s1 % 3>{});
                else stage(0, IC<s1 % 3>{});   // the next task's quad 0
                bar_lds();
            });
        });
        const int64_t tile = tile_of(task);
        if constexpr (GATES) {
            // wave k holds gate k of hidden channels hb*16 + r for games 4g + i; in chunks of 12 cells every wave
            // writes its accumulators to LDS, then wave k' forms the cell update of row i = k' from all four gates
            float *xchg = reinterpret_cast<float *>(smem + kLdsBytes);
            const int ctg = (int)(task % n_ctg);
            const int layer = ctg / a.nh, ch = (ctg % a.nh) * 16 + r;
            const int H = 16 * a.nh;
            const int64_t n = tile * 16 + 4 * g + wave;   // this wave's row i = wave
            const int64_t nc = min(n, a.N - 1);
            const float *zp = a.zx + nc * a.zxs + (int64_t)(layer * 4 * H + ch) * kHW;
            const float *cp = a.c_in + nc * a.cs + (int64_t)(layer * H + ch) * kHW;
            float bgate[4];
            static_for<0, 4>([&](auto k_c) __attribute__((always_inline)) {
                constexpr int k = decltype(k_c)::value;
                bgate[k] = a.bias ? a.bias[layer * 4 * H + k * H + ch] : 0.f;
            });
            static_for<0, kHW / kGateChunk>([&](auto c_c) __attribute__((always_inline)) {
                constexpr int C0 = decltype(c_c)::value * kGateChunk;
                float4 zq[4][kGateChunk / 4], cq[kGateChunk / 4];   // the chunk's x halves and cell state
                static_for<0, kGateChunk / 4>([&](auto j_c) __attribute__((always_inline)) {
                    constexpr int j = decltype(j_c)::value;
                    static_for<0, 4>([&](auto k_c) __attribute__((always_inline)) {
                        constexpr int k = decltype(k_c)::value;
                        zq[k][j] = *reinterpret_cast<const float4 *>(zp + (int64_t)k * H * kHW + C0 + 4 * j);
                    });
                    cq[j] = *reinterpret_cast<const float4 *>(cp + C0 + 4 * j);
                });
                if constexpr (C0 > 0) bar_lds();   // the previous chunk's reads are done
                static_for<0, kGateChunk>([&](auto q_c) __attribute__((always_inline)) {
                    constexpr int ql = decltype(q_c)::value;
                    static_for<0, 4>([&](auto i_c) __attribute__((always_inline)) {
                        constexpr int i = decltype(i_c)::value;
                        xchg[((wave * kGateChunk + ql) * 4 + i) * 64 + lane] = acc[C0 + ql][i];
                    });
                });
                bar_lds();
                if (n < a.N) {
                    float *ho = a.h_out + n * a.hs + (int64_t)(layer * H + ch) * kHW + C0;
                    float *co = a.c_out + n * a.cs + (int64_t)(layer * H + ch) * kHW + C0;
                    static_for<0, kGateChunk / 4>([&](auto j_c) __attribute__((always_inline)) {
                        constexpr int j = decltype(j_c)::value;
                        float hv[4], cv[4];
                        static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
                            constexpr int u = decltype(u_c)::value;
                            constexpr int ql = 4 * j + u;
                            float z[4];
                            static_for<0, 4>([&](auto k_c) __attribute__((always_inline)) {
                                constexpr int k = decltype(k_c)::value;
                                const float4 &f = zq[k][j];
                                const float xv = u == 0 ? f.x : (u == 1 ? f.y : (u == 2 ? f.z : f.w));
                                const float zh = xchg[((k * kGateChunk + ql) * 4 + wave) * 64 + lane];
                                z[k] = a.bias ? (xv + bgate[k]) + zh : xv + zh;   // (zx + b) + zh
                            });
                            const float c0 = u == 0 ? cq[j].x : (u == 1 ? cq[j].y : (u == 2 ? cq[j].z : cq[j].w));
                            const float si = sigm(z[0]), sf = sigm(z[1]), so = sigm(z[2]), tg = tanhf(z[3]);
                            const float fc = sf * c0;
                            const float ig = si * tg;
                            const float cc = fc + ig;
                            cv[u] = cc;
                            hv[u] = so * tanhf(cc);
                        });
                        *reinterpret_cast<float4 *>(co + 4 * j) = make_float4(cv[0], cv[1], cv[2], cv[3]);
                        *reinterpret_cast<float4 *>(ho + 4 * j) = make_float4(hv[0], hv[1], hv[2], hv[3]);
                    });
                }
            });
            static_for<0, NCELL>([&](auto q_c) __attribute__((always_inline)) {
                acc[decltype(q_c)::value] = (f32x4){0.f, 0.f, 0.f, 0.f};
            });
            continue;
        }
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

// The ConvLSTM cells' h halves with the gate update in the epilogue (hrl_gboard_lstm_forward)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void gboard_lstm_kernel(GbArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[kLdsBytes + kXchgBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwg = gridDim.x, b = blockIdx.x;
    const int L = (nwg % 8 == 0) ? (b & 7) * (nwg >> 3) + (b >> 3) : b;
    gboard_run<1, false, 4, 0, true>(a, smem, lane, wave, L);
}

// A workgroup's 4 waves share one 16-game tile per task: each stages a quarter of every quad (16 games x 32
// channels x 4 cells, split once into the LDS ring) and computes NCTW column tiles x (4 / NCTW) output bands.
template <int KC, bool PADC, int NCTW>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void gboard_conv_kernel(GbArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwg = gridDim.x, b = blockIdx.x;
    // consecutive logical workgroups (which share game tiles) on one XCD (hardware deals b round robin)
    const int L = (nwg % 8 == 0) ? (b & 7) * (nwg >> 3) + (b >> 3) : b;
    constexpr int NB = 4 / NCTW;
    const int band = wave / NCTW;
    if constexpr (NB == 1) {
        gboard_run<KC, PADC, NCTW, 0>(a, smem, lane, wave, L);
    } else if constexpr (NB == 2) {
        if (band == 0) gboard_run<KC, PADC, NCTW, 0>(a, smem, lane, wave, L);
        else gboard_run<KC, PADC, NCTW, 1>(a, smem, lane, wave, L);
    } else {
        switch (band) {
        case 0: gboard_run<KC, PADC, NCTW, 0>(a, smem, lane, wave, L); break;
        case 1: gboard_run<KC, PADC, NCTW, 1>(a, smem, lane, wave, L); break;
        case 2: gboard_run<KC, PADC, NCTW, 2>(a, smem, lane, wave, L); break;
        default: gboard_run<KC, PADC, NCTW, 3>(a, smem, lane, wave, L); break;
        }
    }
}

// W (Cout, w_cin_total, 3, 3), input channels [w_ci0, w_ci0 + cin_g) -> split fragments [ct][kc][tap][part][64]
// x 4 words: lane l of (ct, kc) holds W^T[ci = 32kc + 8(l>>4) + e][co = 16ct + (l&15)], e = 2d, 2d+1 in word d
__global__ void gboard_pack_kernel(const float *__restrict__ w, int cout, int cin_g, int w_cin_total, int w_ci0,
                                   int KC, int total, uint32_t *__restrict__ out) {
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
        return (co < cout && c < cin_g) ? w[((int64_t)co * w_cin_total + w_ci0 + c) * kTaps + tap] : 0.f;
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

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

int64_t hrl_gboard_pack_bytes(int64_t Cout, int64_t Cin_g) {
    if (Cout < 1 || Cin_g < 1 || Cin_g > 64) return -1;
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
                       weight, (int)Cout, (int)Cin_g, (int)w_cin_total, (int)w_ci0, KC, total,
                       static_cast<uint32_t *>(packed));
    return status();
}

int hrl_gboard_forward(const float *x, int64_t x_stride, const float *x2, int64_t x2_stride, int64_t N, int64_t Cin_g,
                       int64_t groups, const void *packed, int64_t Cout, const float *bias, const float *alpha,
                       const float *beta, int relu, float *y, int64_t y_stride, void *stream) {
    if (!x || !packed || !y || N < 1 || Cin_g < 1 || Cin_g > 64 || groups < 1 || Cout < 1 || Cout % groups)
        return HRL_EINVAL;
    const int64_t cout_g = Cout / groups;
    if (groups > 1 && cout_g % 16) return HRL_EINVAL;        // a column tile never straddles two groups
    if (x2 && (Cin_g <= 32 || groups != 1)) return HRL_EINVAL;
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
    const int64_t tasks = ntiles * (a.nct / nctw);
    int grid = (int)(tasks < kCUs ? tasks : kCUs);
    const dim3 block(kThreads);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int KC = (int)((Cin_g + 31) / 32);
    const bool padc = Cin_g % 32 != 0;
#define HRL_GB_LAUNCH(KC_, PADC_)                                                                                  \
    do {                                                                                                         \
        if (nctw == 4) hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 4>), dim3(grid), block, 0, s, a);      \
        else if (nctw == 2) hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 2>), dim3(grid), block, 0, s, a); \
        else hipLaunchKernelGGL((gboard_conv_kernel<KC_, PADC_, 1>), dim3(grid), block, 0, s, a);                \
    } while (0)
    if (KC == 1) {
        if (padc) HRL_GB_LAUNCH(1, true); else HRL_GB_LAUNCH(1, false);
    } else {
        if (padc) HRL_GB_LAUNCH(2, true); else HRL_GB_LAUNCH(2, false);
    }
#undef HRL_GB_LAUNCH
    return status();
}

int hrl_gboard_lstm_forward(const float *h, int64_t h_stride, int64_t N, int64_t layers, int64_t H, const void *packed,
                            const float *zx, int64_t zx_stride, const float *bias, const float *c_in, float *c_out,
                            int64_t c_stride, float *h_out, int64_t hout_stride, void *stream) {
    if (!h || !packed || !zx || !c_in || !c_out || !h_out || N < 1 || layers < 1 || H < 16 || H > 64 || H % 16)
        return HRL_EINVAL;
    if (h_out == h) return HRL_EINVAL;   // other workgroups still read h while this one writes h'
    if (!aligned16(h) || !aligned16(zx) || !aligned16(c_in) || !aligned16(c_out) || !aligned16(h_out) ||
        h_stride % 4 || zx_stride % 4 || c_stride % 4 || hout_stride % 4)
        return HRL_EINVAL;
    if (h_stride < layers * H * kHW || zx_stride < layers * 4 * H * kHW || c_stride < layers * H * kHW ||
        hout_stride < layers * H * kHW)
        return HRL_EINVAL;
    GbArgs a{};
    a.x = h; a.x2 = nullptr; a.N = N; a.xs = h_stride; a.xs2 = 0;
    a.cin_g = (int)H; a.cout_g = (int)(4 * H);
    a.wpk = static_cast<const uint4 *>(packed);
    a.nct = (int)(layers * 4 * H / 16); a.cout = (int)(layers * 4 * H);
    a.bias = bias; a.zx = zx; a.zxs = zx_stride; a.c_in = c_in; a.c_out = c_out; a.h_out = h_out;
    a.cs = c_stride; a.hs = hout_stride; a.nh = (int)(H / 16);
    const int64_t tasks = ((N + 15) / 16) * (a.nct / 4);
    const int grid = (int)(tasks < kCUs ? tasks : kCUs);
    hipLaunchKernelGGL(gboard_lstm_kernel, dim3(grid), dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
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
