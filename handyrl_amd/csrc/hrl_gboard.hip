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
constexpr int kSlots = 1024;      // waves the chip holds at one wave per SIMD

struct GbArgs {
    const float *x, *x2;   // x2 (optional): input channels 32.. (the move head's [h_e, h_last] without a copy)
    int64_t N, xs, xs2;    // games; floats from one game to the next in x / x2
    int cin_g, cout_g;     // input / output channels per group
    const uint4 *wpk;      // split weight fragments [ct][kc][tap][part][64]
    int nct, cout;         // 16-channel column tiles; output channels stored
    int tpw;               // waves per column tile (the game tiles are dealt round robin among them)
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

template <int KC, bool PADC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void gboard_conv_kernel(GbArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nwg = gridDim.x, b = blockIdx.x;
    // consecutive logical workgroups (which share game tiles) on one XCD (hardware deals b round robin)
    const int L = (nwg % 8 == 0) ? (b & 7) * (nwg >> 3) + (b >> 3) : b;
    const int w = L * kWaves + wave;
    if (w >= a.nct * a.tpw) return;
    const int ct = w % a.nct;
    const int64_t ntiles = (a.N + 15) >> 4;
    const int r = lane & 15, g = lane >> 4;
    const int grp = (ct * 16) / a.cout_g;
    const float *xb = a.x + (int64_t)(grp * a.cin_g + 8 * g) * kHW;

    // A rows: game n0 + r (clamped: rows past the batch compute values that are never stored)
    auto src = [&](int64_t tile, int kc) -> const float * {
        const int64_t n = min(tile * 16 + r, a.N - 1);
        if (KC > 1 && kc >= 1 && a.x2) return a.x2 + n * a.xs2 + (int64_t)((kc - 1) * 32 + 8 * g) * kHW;
        return xb + n * a.xs + (int64_t)(32 * kc) * kHW;
    };
    // PADC: channel rows at or past cin_g (only the last k-step is ragged) read row cin_g - 1 and are zeroed;
    // emax may be negative (the lane's whole octet is past cin_g: its offsets reach back into valid rows)
    int emax = 7;
    if constexpr (PADC) emax = min(7, a.cin_g - 1 - 8 * g - 32 * (KC - 1));
    // every register array below is indexed by compile-time constants only (static_for): a runtime index,
    // even one that unrolling later folds, keeps the array in scratch
    float4 raw[3][8];
    auto issue = [&](const float *s, int quad, auto slot_c, bool last_kc) __attribute__((always_inline)) {
        constexpr int slot = decltype(slot_c)::value;
        static_for<0, 8>([&](auto e_c) __attribute__((always_inline)) {
            constexpr int e = decltype(e_c)::value;
            int ee = e;
            if constexpr (PADC) ee = last_kc ? min(e, emax) : e;
            raw[slot][e] = *reinterpret_cast<const float4 *>(s + ee * kHW + 4 * quad);
        });
    };
    uint4 Bw[kTaps][3];
    auto load_b = [&](int kc) __attribute__((always_inline)) {
        const uint4 *wp = a.wpk + (((int64_t)ct * KC + kc) * kTaps * 3) * 64 + lane;
        static_for<0, kTaps * 3>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int i = decltype(i_c)::value;
            Bw[i / 3][i % 3] = wp[i * 64];
        });
    };
    f32x4 acc[kHW];
    static_for<0, kHW>([&](auto q_c) __attribute__((always_inline)) {
        acc[decltype(q_c)::value] = (f32x4){0.f, 0.f, 0.f, 0.f};
    });

    int64_t tile = w / a.nct;
    if (tile >= ntiles) return;
    if constexpr (KC == 1) load_b(0);
    // prologue: quads 0 and 1 of the first (tile, k-step)
    {
        const float *s0 = src(tile, 0);
        issue(s0, 0, IC<0>{}, KC == 1);
        issue(s0, 1, IC<1>{}, KC == 1);
    }
    for (; tile < ntiles; tile += a.tpw) {
        const int64_t next = tile + a.tpw < ntiles ? tile + a.tpw : tile;   // loads past the end: re-read
        static_for<0, KC>([&](auto kc_c) __attribute__((always_inline)) {
            constexpr int kc = decltype(kc_c)::value;
            if constexpr (KC > 1) load_b(kc);
            const float *s_cur = src(tile, kc);
            const float *s_nxt = kc + 1 < KC ? src(tile, kc + 1) : src(next, 0);
            constexpr bool cur_last = kc == KC - 1;
            constexpr bool nxt_last = kc + 1 < KC ? kc + 1 == KC - 1 : KC == 1;
            static_for<0, kQuads>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int j = decltype(j_c)::value;
                // two quads ahead (slot (j + 2) % 3: kQuads is a multiple of 3, so slots line up across k-steps)
                if constexpr (j + 2 < kQuads) issue(s_cur, j + 2, IC<(j + 2) % 3>{}, cur_last);
                else issue(s_nxt, j + 2 - kQuads, IC<(j + 2) % 3>{}, nxt_last);
                constexpr int slot = j % 3;
                static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
                    constexpr int u = decltype(u_c)::value;
                    constexpr int p = 4 * j + u;
                    float v[8];
                    static_for<0, 8>([&](auto e_c) __attribute__((always_inline)) {
                        constexpr int e = decltype(e_c)::value;
                        const float4 &f = raw[slot][e];
                        v[e] = u == 0 ? f.x : (u == 1 ? f.y : (u == 2 ? f.z : f.w));
                        if constexpr (PADC && cur_last)
                            if (e > emax) v[e] = 0.f;
                    });
                    uint4 Ah, Am, Al;
                    split8(v, Ah, Am, Al);
                    static_for<0, kHW>([&](auto q_c) __attribute__((always_inline)) {
                        constexpr int q = decltype(q_c)::value;
                        constexpr int t = tap_pq(p, q);
                        if constexpr (t >= 0) acc[q] = mfma_split(Ah, Am, Al, Bw[t][0], Bw[t][1], Bw[t][2], acc[q]);
                    });
                });
            });
        });
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
                    static_for<0, kQuads>([&](auto j_c) __attribute__((always_inline)) {
                        constexpr int j = decltype(j_c)::value;
                        float o[4];
                        static_for<0, 4>([&](auto u_c) __attribute__((always_inline)) {
                            constexpr int u = decltype(u_c)::value;
                            float v = acc[4 * j + u][i];
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
        static_for<0, kHW>([&](auto q_c) __attribute__((always_inline)) {
            acc[decltype(q_c)::value] = (f32x4){0.f, 0.f, 0.f, 0.f};
        });
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
    // waves per column tile: fill the chip's wave slots, a multiple of 4 when that keeps the workgroups a
    // multiple of 8 (the XCD mapping), never more than there are game tiles
    int tpw = (int)(kSlots / a.nct > 0 ? kSlots / a.nct : 1);
    if (tpw >= 8) tpw &= ~3;
    if (tpw > ntiles) tpw = (int)ntiles;
    a.tpw = tpw;
    const int waves = a.nct * tpw;
    const dim3 grid((waves + kWaves - 1) / kWaves), block(kThreads);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int KC = (int)((Cin_g + 31) / 32);
    const bool padc = Cin_g % 32 != 0;
    if (KC == 1) {
        if (padc) hipLaunchKernelGGL((gboard_conv_kernel<1, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((gboard_conv_kernel<1, false>), grid, block, 0, s, a);
    } else {
        if (padc) hipLaunchKernelGGL((gboard_conv_kernel<2, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((gboard_conv_kernel<2, false>), grid, block, 0, s, a);
    }
    return status();
}

}  // extern "C"
