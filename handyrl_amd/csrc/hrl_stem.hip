// hrl_stem.hip — the 3x3-board stem convolution (Cin <= 3 -> 32 channels) with fp32 MFMA (gfx950).
//
// SimpleConv2dModel's first layer (handyrl/envs/tictactoe.py:57) is a 3x3
// 'same' conv of the 3 observation planes into 32 channels, with bias, over
// N = B*T samples.  On a 3x3 board the layer is the dense matrix
//   Y[n, co*9 + q] = sum_k X_aug[n, k] * Wb[k, co*9 + q],
//   X_aug = [x (Cin*9 values) | 1],  Wb[ci*9 + p, co*9 + q] = W[co, ci, tap(p, q)] (0 off the board),
//   Wb[Cin*9, co*9 + q] = b[co]
// (K = Cin*9 + 1 <= 28).  As a library GEMM it needed the ones column
// concatenated onto x, the expanded weight built, and ran at ~2x its HBM
// bound; the weight gradient was a chunked batched GEMM plus folds.  Here:
//
// stem_fwd_kernel: each wave keeps its B fragments of Wb (7 k-steps x 18
//   column tiles = 126 floats per lane) in registers for the whole launch;
//   per 16-sample tile it reads the A fragments straight from x (the ones
//   column is synthesized), runs 126 v_mfma_f32_16x16x4_f32 and stores the
//   16 x 288 output from the accumulators (64-byte row segments).  Bound:
//   the 151 MB output write at N = 131072.
// stem_wgrad_kernel: dWb = X_aug^T dY as MFMA tiles (features x columns,
//   36 accumulators) over 4-sample k-steps, dy tiles staged through LDS with
//   coalesced float4 loads; the 4 waves fold through LDS in a fixed order and
//   the workgroup folds the (p, q) pairs of each tap, so a partial is dW
//   (32, Cin, 3, 3) | db (32); stem_reduce_kernel sums the partials with a
//   fixed-shape tree (fp64).  Deterministic.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCo = 32;
constexpr int kCells = 9;
constexpr int kCols = kCo * kCells;    // 288 outputs per sample
constexpr int kNT = kCols / 16;        // 18 column tiles
constexpr int kKMax = 28;              // Cin*9 + 1 <= 28 (Cin <= 3)
constexpr int kKS = kKMax / 4;         // 7 k-steps
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kWbStride = kCols + 16;  // LDS row stride of Wb

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// tap index of input cell p feeding output cell q on the 3x3 board, or -1
__device__ __forceinline__ int tap_of(int p, int q) {
    const int dy = p / 3 - q / 3 + 1, dx = p % 3 - q % 3 + 1;
    return (dy < 0 || dy > 2 || dx < 0 || dx > 2) ? -1 : dy * 3 + dx;
}

// Wb entry (k, col) for weights w (32, Cin, 3, 3) and bias b (may be NULL)
__device__ __forceinline__ float wb_at(const float *w, const float *b, int Cin, int k, int col) {
    const int co = col / kCells, q = col - co * kCells;
    if (k < Cin * kCells) {
        const int ci = k / kCells, p = k - ci * kCells;
        const int t = tap_of(p, q);
        return t < 0 ? 0.f : w[(co * Cin + ci) * 9 + t];
    }
    return (k == Cin * kCells && b) ? b[co] : 0.f;
}

// X_aug[n, k]: x value, the ones column (bias), or zero padding
__device__ __forceinline__ float xa_at(const float *x, int64_t n, int64_t N, int Cin, bool bias, int k) {
    if (n >= N) return 0.f;
    if (k < Cin * kCells) return x[n * (Cin * kCells) + k];
    return (k == Cin * kCells && bias) ? 1.f : 0.f;
}

// ------------------------------------------------------------------ forward
__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(const float *__restrict__ x, int64_t N, int Cin,
                                                            const float *__restrict__ w, const float *__restrict__ b,
                                                            float *__restrict__ y) {
    __shared__ float wb[kKMax * kWbStride];
    for (int i = threadIdx.x; i < kKMax * kCols; i += kThreads) {
        const int k = i / kCols, col = i - k * kCols;
        wb[k * kWbStride + col] = wb_at(w, b, Cin, k, col);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kk = lane >> 4;
    // this lane's B fragments: Wb[ks*4 + kk][nt*16 + i16]
    float bf[kKS][kNT];
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) bf[ks][nt] = wb[(ks * 4 + kk) * kWbStride + nt * 16 + i16];
    const bool bias = b != nullptr;
    const int64_t ntiles = (N + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t t = (int64_t)blockIdx.x * kWaves + wave;
    float af[kKS];
    auto load_a = [&](int64_t tt) {
#pragma unroll
        for (int ks = 0; ks < kKS; ++ks) af[ks] = xa_at(x, tt * 16 + i16, N, Cin, bias, ks * 4 + kk);
    };
    if (t < ntiles) load_a(t);
    for (; t < ntiles; t += stride) {
        f32x4 acc[kNT];
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kKS; ++ks)
#pragma unroll
            for (int nt = 0; nt < kNT; ++nt) acc[nt] = mfma(af[ks], bf[ks][nt], acc[nt]);
        const int64_t next = t + stride;
        if (next < ntiles) load_a(next);   // in flight during the stores
        // C/D layout: row = kk*4 + r (sample in the tile), col = nt*16 + i16
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t n = t * 16 + kk * 4 + r;
            if (n < N) {
                float *yr = y + n * kCols + i16;
#pragma unroll
                for (int nt = 0; nt < kNT; ++nt) yr[nt * 16] = acc[nt][r];
            }
        }
    }
}

// a buffer descriptor over [base, base + bytes) (loads past it read 0, stores past it are dropped).
// readfirstlane returns an int: each half of the address goes through a uint32_t, or a low half with bit 31 set
// would sign-extend over the high half
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base, int64_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                             0x00020000);
}

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int hu32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ forward, lane per channel (form 2)
// stem_fwd2_kernel<CIN>: a wave takes 8-row octets; lane (h, co) computes output channel co of rows 4j + 2h and
// 4j + 2h + 1 (j = 0, 1) as one float2 each (v_pk_fma_f32 on the two rows), with its Cin*9 weights and bias in
// registers:
//   y[n][co][q] = b[co] + sum_ci sum_{p: tap(p, q) on the board} w[co][ci][tap(p, q)] * x[n][ci][p]
// (fused multiply-adds, ci then p ascending).  The octet's observation rows (8 x Cin*9 floats, contiguous) come in
// as float4s through LDS and are read back as broadcasts; its outputs go through LDS too and leave as contiguous
// float4 stores (1 KiB per wave instruction): the 36-byte per-lane runs written straight from registers ran at
// 3.0 TB/s against 6.6 for a plain fill (tools/stem_bench.py).
constexpr int kOct = 8;                       // rows per wave step
constexpr int kYO = kOct * kCols;             // 2304 output floats per octet

template <int CIN>
__global__ __launch_bounds__(kThreads) void stem_fwd2_kernel(const float *__restrict__ x, int64_t N,
                                                             const float *__restrict__ w,
                                                             const float *__restrict__ b, float *__restrict__ y) {
    constexpr int kXF = CIN * kCells;
    constexpr int kXO = kOct * kXF;           // observation floats per octet (multiple of 4: kXF * 8)
    __shared__ __attribute__((aligned(16))) float ys[kWaves][kYO];
    __shared__ __attribute__((aligned(16))) float xs[kWaves][kXO];
    const int lane = threadIdx.x & 63, co = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *yw = ys[wave];
    float *xw = xs[wave];
    float wr[kXF];
#pragma unroll
    for (int k = 0; k < kXF; ++k) wr[k] = w[co * kXF + k];
    const float bias = b ? b[co] : 0.f;
    const int64_t noct = (N + kOct - 1) / kOct;
    const int64_t wstep = (int64_t)gridDim.x * kWaves;
    // the octet's observations: kXO / 4 float4s (rows past N read 0); the next octet's are in flight during this
    // one's FMAs and stores
    auto load_x = [&](int64_t t) __attribute__((always_inline)) {
        const int64_t rows = min<int64_t>(kOct, N - kOct * t);
        const __amdgpu_buffer_rsrc_t rx = rsrc_of(x + kOct * t * kXF, rows * kXF * 4);
        return lane < kXO / 4 ? __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16, 0, 0) : (hu32x4){0u, 0u, 0u, 0u};
    };
    int64_t t = (int64_t)blockIdx.x * kWaves + wave;
    hu32x4 xn = t < noct ? load_x(t) : (hu32x4){0u, 0u, 0u, 0u};
    for (; t < noct; t += wstep) {
        const int64_t rows = min<int64_t>(kOct, N - kOct * t);
        const __amdgpu_buffer_rsrc_t ry = rsrc_of(y + kOct * t * kCols, rows * kCols * 4);
        if (lane < kXO / 4) *reinterpret_cast<hu32x4 *>(xw + 4 * lane) = xn;
        if (t + wstep < noct) xn = load_x(t + wstep);
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r0 = 4 * j + 2 * h;     // rows r0, r0 + 1 of the octet
            f32x2 xv[kXF];
#pragma unroll
            for (int k = 0; k < kXF; ++k) xv[k] = (f32x2){xw[r0 * kXF + k], xw[(r0 + 1) * kXF + k]};
            f32x2 acc[kCells];
#pragma unroll
            for (int q = 0; q < kCells; ++q) {
                acc[q] = (f32x2){bias, bias};
#pragma unroll
                for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
                    for (int p = 0; p < kCells; ++p) {
                        const int tap = tap_of(p, q);
                        if (tap < 0) continue;
                        const float wv = wr[ci * kCells + tap];
                        acc[q] = __builtin_elementwise_fma((f32x2){wv, wv}, xv[ci * kCells + p], acc[q]);
                    }
            }
#pragma unroll
            for (int q = 0; q < kCells; ++q) {
                yw[r0 * kCols + co * kCells + q] = acc[q].x;
                yw[(r0 + 1) * kCols + co * kCells + q] = acc[q].y;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < kYO / 4 / 64; ++k) {   // 9 contiguous float4 per lane (rows past N: dropped)
            const int i = k * 64 + lane;
            const hu32x4 v = *reinterpret_cast<const hu32x4 *>(yw + 4 * i);
            __builtin_amdgcn_raw_buffer_store_b128(v, ry, i * 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);        // the LDS reads done before the next octet overwrites
        __builtin_amdgcn_wave_barrier();
    }
}

// ------------------------------------------------------------------ weight gradient
constexpr int kDyStride = kCols + 4;   // LDS row stride of a staged dy tile (16 B aligned rows)
constexpr int kNOut = kCo * 3 * 9 + kCo;   // folded outputs per partial (Cin <= 3): dW then db

// Per 16-sample tile: dy rows staged in LDS with coalesced float4 loads (the next tile's in flight during
// the MFMAs); dWb = X_aug^T dY accumulates in MFMA tiles (features x columns).  At the end the 4 waves
// fold in a fixed order and the workgroup folds the (p, q) pairs of each tap: one partial of
// 32*Cin*9 + 32 values per workgroup, [dW (co, ci, tap) | db (co)].
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(const float *__restrict__ x,
                                                              const float *__restrict__ dy, int64_t N, int Cin,
                                                              int bias, float *__restrict__ partial) {
    __shared__ float lds[kWaves * 16 * kDyStride > 32 * kCols ? kWaves * 16 * kDyStride : 32 * kCols];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kk = lane >> 4;
    float *tile = lds + wave * 16 * kDyStride;
    f32x4 acc[2][kNT];
#pragma unroll
    for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[it][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int64_t ntiles = (N + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    constexpr int kV = 16 * kCols / 4 / 64;   // 18 float4 per lane per tile
    float4 st[kV];
    float xa[4][2];   // the tile's A values (features i16 and 16 + i16 of sample ks*4 + kk)
    auto load = [&](int64_t tt) {
        const int64_t lim = N * kCols;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int64_t n = tt * 16 + ks * 4 + kk;
            xa[ks][0] = xa_at(x, n, N, Cin, bias != 0, i16);
            xa[ks][1] = xa_at(x, n, N, Cin, bias != 0, 16 + i16);
        }
#pragma unroll
        for (int k = 0; k < kV; ++k) {
            const int64_t e = tt * 16 * kCols + (int64_t)(k * 64 + lane) * 4;
            st[k] = e < lim ? *reinterpret_cast<const float4 *>(dy + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    int64_t t = (int64_t)blockIdx.x * kWaves + wave;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += stride) {
#pragma unroll
        for (int k = 0; k < kV; ++k) {
            const int e = (k * 64 + lane) * 4;
            const int r = e / kCols, c = e - r * kCols;
            *reinterpret_cast<float4 *>(tile + r * kDyStride + c) = st[k];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        float a[4][2];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) { a[ks][0] = xa[ks][0]; a[ks][1] = xa[ks][1]; }
        if (t + stride < ntiles) load(t + stride);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {   // the MFMA k = sample t*16 + ks*4 + kk
            const float a0 = a[ks][0], a1 = a[ks][1];
            const float *br = tile + (ks * 4 + kk) * kDyStride + i16;
#pragma unroll
            for (int nt = 0; nt < kNT; ++nt) {
                const float bv = br[nt * 16];
                acc[0][nt] = mfma(a0, bv, acc[0][nt]);
                acc[1][nt] = mfma(a1, bv, acc[1][nt]);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    // fold the 4 waves in a fixed order ((w0 + w1) + w2) + w3 into red[k][col]
    float *red = lds;
    __syncthreads();
#pragma unroll 1
    for (int w = 0; w < kWaves; ++w) {
        if (wave == w) {
#pragma unroll
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float *d = red + (it * 16 + kk * 4 + r) * kCols + nt * 16 + i16;
                        *d = w == 0 ? acc[it][nt][r] : *d + acc[it][nt][r];
                    }
        }
        __syncthreads();
    }
    // fold the cell pairs of each tap (q, then p, in order): dW[co][ci][tap], then db[co]
    float *out = partial + (int64_t)blockIdx.x * kNOut;
    const int nw = kCo * Cin * 9;
    for (int o = threadIdx.x; o < nw + kCo; o += kThreads) {
        float s = 0.f;
        if (o < nw) {
            const int co = o / (Cin * 9), ci = (o / 9) % Cin, tap = o % 9;
            const int ky = tap / 3, kx = tap % 3;
            for (int q = 0; q < kCells; ++q) {   // the input cell of output cell q under this tap
                const int py = q / 3 + ky - 1, px = q % 3 + kx - 1;
                if (py >= 0 && py < 3 && px >= 0 && px < 3)
                    s += red[(ci * kCells + py * 3 + px) * kCols + co * kCells + q];
            }
        } else if (bias) {
            const int co = o - nw;
            for (int q = 0; q < kCells; ++q) s += red[(Cin * kCells) * kCols + co * kCells + q];
        }
        out[o] = s;
    }
}

// ------------------------------------------------------------------ weight gradient, lane-per-channel form
// stem_wgrad_kernel holds a 16-sample dy tile per wave in registers (18 float4 per lane) and 144 accumulators of
// the dense 28 x 288 dWb, one wave per SIMD: one tile of loads in flight per wave, 63 us in the step (2.6 TB/s).
// Only 49 (p, q) pairs x Cin of dWb are weights, so here a lane owns (row half r = lane >> 5, output channel
// co = lane & 31) and accumulates dW[co][ci][tap] (Cin x 9) and db[co] in 28 registers:
//   dW[co][ci][tap] += sum_{q on the board} dy[n][co][q] * x[n][ci][p(q, tap)],  db[co] += sum_q dy[n][co][q]
// per sample n (fmaf, taps in order, q ascending).  A wave's 64 lanes read two whole dy rows per step (36
// contiguous bytes per lane); the block's 32 observation rows (Cin*9 floats each) are staged in LDS once and read
// back as broadcasts.  ~90 VGPRs: 4 workgroups of 4 waves per CU, the next row pair's dy in flight.
template <int CIN>
__global__ __launch_bounds__(kThreads, 4) void stem_wgrad2_kernel(const float *__restrict__ x,
                                                                  const float *__restrict__ dy, int64_t N, int bias,
                                                                  float *__restrict__ partial) {
    constexpr int kBR = 32;                       // rows per block (one wave)
    constexpr int kXF = CIN * kCells;             // observation floats per row
    constexpr int kXS = (kXF + 3) / 4 * 4;        // LDS row stride (float4 reads)
    constexpr int kNW = kCo * CIN * 9;
    __shared__ __attribute__((aligned(16))) float xs[kWaves][kBR * kXS];   // after the loop: the fold
    static_assert(64 * (CIN * 9 + 1) <= kWaves * kBR * kXS, "fold");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int co = lane & 31, r = lane >> 5;
    float acc[CIN * 9], accb = 0.f;
#pragma unroll
    for (int i = 0; i < CIN * 9; ++i) acc[i] = 0.f;
    const __amdgpu_buffer_rsrc_t rd = rsrc_of(dy, N * kCols * 4);   // rows past N read 0
    float *xw = xs[wave];
    const int64_t nblocks = (N + kBR - 1) / kBR;
    const int64_t wstep = (int64_t)gridDim.x * kWaves;
    auto load_dy = [&](int64_t row, float (&d)[kCells]) __attribute__((always_inline)) {
        const uint32_t off = (uint32_t)((row * kCols + co * kCells) * 4);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rd, off + 12 * m, 0, 0);
            d[3 * m] = __uint_as_float(v.x);
            d[3 * m + 1] = __uint_as_float(v.y);
            d[3 * m + 2] = __uint_as_float(v.z);
        }
    };
    // the block's observation rows are one contiguous run of kBR * kXF floats: all of a lane's loads issue together
    // (a load-then-store loop over the padded LDS layout waited for each load in turn); the pad columns stay 0
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(x, N * kXF * 4);   // rows past N read 0
    constexpr int kXL = (kBR * kXF + 63) / 64;
    for (int i = lane; i < kBR * (kXS - kXF); i += 64) xw[(i / (kXS - kXF)) * kXS + kXF + i % (kXS - kXF)] = 0.f;
    // a lane takes two rows per step (4 it + 2 r and the next) as one packed f32x2 pair: v_pk_fma_f32 does both rows'
    // multiply-adds in one instruction (the kernel was VALU-bound at one FMA per MAC); per lane the rows still add
    // into its accumulators one after the other
    auto load_pair = [&](int64_t row, f32x2 (&d)[kCells]) __attribute__((always_inline)) {
        float a[kCells], b[kCells];
        load_dy(row, a);
        load_dy(row + 1, b);
#pragma unroll
        for (int q = 0; q < kCells; ++q) d[q] = (f32x2){a[q], b[q]};
    };
    for (int64_t blk = (int64_t)blockIdx.x * kWaves + wave; blk < nblocks; blk += wstep) {
        const int64_t base = blk * kBR;
        float xr[kXL];
        const uint32_t xb = (uint32_t)(base * kXF * 4);
#pragma unroll
        for (int k = 0; k < kXL; ++k) {
            const int e = k * 64 + lane;
            xr[k] = e < kBR * kXF ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xb + e * 4, 0, 0)) : 0.f;
        }
#pragma unroll
        for (int k = 0; k < kXL; ++k) {
            const int e = k * 64 + lane;
            if (e < kBR * kXF) {
                const int rr = e / kXF;
                xw[rr * kXS + e - rr * kXF] = xr[k];
            }
        }
        f32x2 dn[kCells];
        load_pair(base + 2 * r, dn);   // rows past N read 0 (the descriptor's range)
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int it = 0; it < kBR / 4; ++it) {
            f32x2 d[kCells];
#pragma unroll
            for (int q = 0; q < kCells; ++q) d[q] = dn[q];
            if (it + 1 < kBR / 4) load_pair(base + 4 * (it + 1) + 2 * r, dn);
            f32x2 tb = (f32x2){0.f, 0.f};
#pragma unroll
            for (int q = 0; q < kCells; ++q) tb += d[q];
            accb += tb.x;
            accb += tb.y;
            const float *xr0 = xw + (4 * it + 2 * r) * kXS;
#pragma unroll
            for (int ci = 0; ci < CIN; ++ci) {
                asm volatile("" ::: "memory");   // one input channel's observations at a time
                f32x2 xv[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) xv[k] = (f32x2){xr0[ci * 9 + k], xr0[kXS + ci * 9 + k]};
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    const int ky = tap / 3, kx = tap % 3;
                    f32x2 t = (f32x2){0.f, 0.f};
#pragma unroll
                    for (int q = 0; q < kCells; ++q) {
                        const int py = q / 3 + ky - 1, px = q % 3 + kx - 1;
                        if (py >= 0 && py < 3 && px >= 0 && px < 3)
                            t = __builtin_elementwise_fma(d[q], xv[py * 3 + px], t);
                    }
                    acc[ci * 9 + tap] += t.x;
                    acc[ci * 9 + tap] += t.y;
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // the block's LDS rows are read before the next block's overwrite
        __builtin_amdgcn_wave_barrier();
    }
    // fold: the 4 waves in order into red[i][lane], then lanes co and co + 32 -> partial [dW (co, ci, tap) | db (co)]
    float *red = &xs[0][0];
    __syncthreads();
#pragma unroll 1
    for (int wv = 0; wv < kWaves; ++wv) {
        if (wave == wv) {
#pragma unroll
            for (int i = 0; i < CIN * 9; ++i) red[i * 64 + lane] = wv == 0 ? acc[i] : red[i * 64 + lane] + acc[i];
            red[CIN * 9 * 64 + lane] = wv == 0 ? accb : red[CIN * 9 * 64 + lane] + accb;
        }
        __syncthreads();
    }
    float *out = partial + (int64_t)blockIdx.x * kNOut;
    for (int o = threadIdx.x; o < kNW + kCo; o += kThreads) {
        const int c = o < kNW ? o / (CIN * 9) : o - kNW;
        const int i = o < kNW ? o % (CIN * 9) : CIN * 9;
        const float t = red[i * 64 + c] + red[i * 64 + c + 32];
        out[o] = (o < kNW || bias) ? t : 0.f;
    }
}

int g_stem_wgrad_form = 2;   // hrl_stem_set_wgrad_form
int g_stem_fwd_form = 2;     // hrl_stem_set_fwd_form: 2 = stem_fwd2_kernel, 1 = the fp32 MFMA form

// fixed-order fold of the workgroup partials: one workgroup per output, strided fp64 sums, LDS tree
__global__ __launch_bounds__(256) void stem_reduce_kernel(const float *__restrict__ partial, int nparts, int nw,
                                                          float *__restrict__ dw, float *__restrict__ db) {
    __shared__ double red[256];
    const int o = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nparts; b += 256) s += (double)partial[(int64_t)b * kNOut + o];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (o < nw) dw[o] = (float)red[0];
        else if (db) db[o - nw] = (float)red[0];
    }
}

constexpr int kGrid = 256;

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

int grid_for(int64_t N, int cap) {
    const int64_t blocks = ((N + 15) / 16 + kWaves - 1) / kWaves;
    return (int)(blocks < cap ? blocks : cap);
}

constexpr int kGrid2 = 1024;   // stem_wgrad2_kernel: 4 workgroups per CU
constexpr int kGridF2 = 1024;  // stem_fwd2_kernel: 4 workgroups of 4 waves per CU (40 KB LDS each), over 8-row octets

// workgroups of the weight gradient's form: form 2 runs 4-wave workgroups over 32-row blocks
int grid_wgrad(int64_t N) {
    if (g_stem_wgrad_form != 2) return grid_for(N, kGrid);
    const int64_t wgs = ((N + 31) / 32 + kWaves - 1) / kWaves;
    return (int)(wgs < kGrid2 ? wgs : kGrid2);
}


}  // namespace

extern "C" {

int64_t hrl_stem_workspace_bytes(int64_t N) {
    if (N < 1) return -1;
    const int g1 = grid_for(N, kGrid), g2 = grid_wgrad(N);
    return (int64_t)(g1 > g2 ? g1 : g2) * kNOut * 4;
}

int64_t hrl_stem_wgrad_partials(int64_t N, int64_t *row_floats) {
    if (N < 1) return -1;
    if (row_floats) *row_floats = kNOut;
    return grid_wgrad(N);
}

int hrl_stem_set_wgrad_form(int form) {
    const int prev = g_stem_wgrad_form;
    if (form == 1 || form == 2) g_stem_wgrad_form = form;   // any other value only queries
    return prev;
}

int hrl_stem_set_fwd_form(int form) {
    const int prev = g_stem_fwd_form;
    if (form == 1 || form == 2) g_stem_fwd_form = form;   // any other value only queries
    return prev;
}

int hrl_stem_forward(const float *x, int64_t N, int64_t Cin, const float *weight, const float *bias, float *y,
                     void *stream) {
    if (N < 1 || Cin < 1 || Cin > 3 || !x || !weight || !y) return HRL_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (g_stem_fwd_form == 2) {
        const int64_t wgs = ((N + kOct - 1) / kOct + kWaves - 1) / kWaves;
        const dim3 grid((unsigned)(wgs < kGridF2 ? wgs : kGridF2));
        if (Cin == 3)
            hipLaunchKernelGGL(stem_fwd2_kernel<3>, grid, dim3(kThreads), 0, s, x, N, weight, bias, y);
        else if (Cin == 2)
            hipLaunchKernelGGL(stem_fwd2_kernel<2>, grid, dim3(kThreads), 0, s, x, N, weight, bias, y);
        else
            hipLaunchKernelGGL(stem_fwd2_kernel<1>, grid, dim3(kThreads), 0, s, x, N, weight, bias, y);
        return status();
    }
    hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid_for(N, 2 * kGrid)), dim3(kThreads), 0, s, x, N, (int)Cin, weight,
                       bias, y);
    return status();
}

int hrl_stem_wgrad(const float *x, const float *dy, int64_t N, int64_t Cin, float *dweight, float *dbias,
                   void *workspace, int64_t workspace_bytes, void *stream) {
    if (N < 1 || Cin < 1 || Cin > 3 || !x || !dy || !workspace) return HRL_EINVAL;
    if (workspace_bytes < hrl_stem_workspace_bytes(N)) return HRL_EINVAL;
    // no dweight (and no dbias): the partial rows [dW | db] stay in the workspace for a later fold
    const bool defer = !dweight;
    if (defer && (dbias || g_stem_wgrad_form != 2)) return HRL_EINVAL;
    const int want_bias = (dbias || defer) ? 1 : 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = grid_wgrad(N);
    float *partial = static_cast<float *>(workspace);
    if (g_stem_wgrad_form == 2) {
        if ((N + 32) * kCols * 4 >= (int64_t)1 << 32) return HRL_EINVAL;   // 32-bit buffer offsets (+ a block)
        if (Cin == 3)
            hipLaunchKernelGGL(stem_wgrad2_kernel<3>, dim3(grid), dim3(kThreads), 0, s, x, dy, N, want_bias, partial);
        else if (Cin == 2)
            hipLaunchKernelGGL(stem_wgrad2_kernel<2>, dim3(grid), dim3(kThreads), 0, s, x, dy, N, want_bias, partial);
        else
            hipLaunchKernelGGL(stem_wgrad2_kernel<1>, dim3(grid), dim3(kThreads), 0, s, x, dy, N, want_bias, partial);
    } else {
        hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(kThreads), 0, s, x, dy, N, (int)Cin, dbias ? 1 : 0,
                           partial);
    }
    int rc = status();
    if (rc || !dweight) return rc;   // no dweight: the partial rows stay for a later fold (hrl_grad_fold_norm)
    const int nw = kCo * (int)Cin * 9;
    hipLaunchKernelGGL(stem_reduce_kernel, dim3(nw + (dbias ? kCo : 0)), dim3(256), 0, s, partial, grid, nw, dweight,
                       dbias);
    return status();
}

}  // extern "C"
