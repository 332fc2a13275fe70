// hrl_board.hip — weight plumbing of the tiny-board convolution (handyrl_amd/nn.py BoardConv2d).
//
// On an HxW board with H*W <= 16 a 'same' convolution is the dense matrix
// W_board (Cin*HW x Cout*HW); the layer runs as one GEMM over the NCHW rows.
// These kernels build W_board from W (and the expanded bias) every step and
// fold the W_board gradient back onto W, one launch each instead of a
// cat/index/scatter chain of small framework kernels.  The fold gives each
// weight element to one thread, which sums its (at most H*W) board entries
// in a fixed order: deterministic.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_nn.h"
#include "../../include/hrl_targets.h"

namespace {

struct BoardGeo {
    int Cout, Cin, kh, kw, H, W, HW, ph, pw;
};

// W_board entry (row = ci*HW + p, col = co*HW + q)
__global__ void board_weight_kernel(const float *__restrict__ w, BoardGeo g, float *__restrict__ wb) {
    const int64_t n = (int64_t)g.Cin * g.HW * g.Cout * g.HW;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int col = (int)(i % (g.Cout * g.HW));
        const int row = (int)(i / (g.Cout * g.HW));
        const int ci = row / g.HW, p = row - ci * g.HW;
        const int co = col / g.HW, q = col - co * g.HW;
        const int dy = p / g.W - q / g.W + g.ph;
        const int dx = p % g.W - q % g.W + g.pw;
        float v = 0.f;
        if (dy >= 0 && dy < g.kh && dx >= 0 && dx < g.kw) v = w[((co * g.Cin + ci) * g.kh + dy) * g.kw + dx];
        wb[i] = v;
    }
}

// dW[co, ci, dy, dx] = sum over output cells q whose tap (dy, dx) lands on the board
__global__ void board_fold_kernel(const float *__restrict__ gb, BoardGeo g, float *__restrict__ gw) {
    const int n = g.Cout * g.Cin * g.kh * g.kw;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int dx = i % g.kw;
    const int dy = (i / g.kw) % g.kh;
    const int ci = (i / (g.kw * g.kh)) % g.Cin;
    const int co = i / (g.kw * g.kh * g.Cin);
    const int ncol = g.Cout * g.HW;
    float s = 0.f;
    for (int q = 0; q < g.HW; ++q) {
        const int py = q / g.W + dy - g.ph, px = q % g.W + dx - g.pw;
        if (py < 0 || py >= g.H || px < 0 || px >= g.W) continue;
        const int p = py * g.W + px;
        s += gb[(int64_t)(ci * g.HW + p) * ncol + co * g.HW + q];
    }
    gw[i] = s;
}

__global__ void board_bias_kernel(const float *__restrict__ b, int Cout, int HW, float *__restrict__ bb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Cout * HW) bb[i] = b[i / HW];
}

__global__ void board_bias_fold_kernel(const float *__restrict__ gb, int Cout, int HW, float *__restrict__ g) {
    const int co = blockIdx.x * blockDim.x + threadIdx.x;
    if (co >= Cout) return;
    float s = 0.f;
    for (int q = 0; q < HW; ++q) s += gb[co * HW + q];
    g[co] = s;
}

// ---- column sums of a row-major (M, N) matrix (bias gradients over M = B*T*P rows) ----
// stage 1: workgroup g folds rows [g*rpb, (g+1)*rpb) per column; each thread owns one
// column (N <= 256: 256/N rows at a time) and accumulates in fp64.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float *__restrict__ x, int64_t M, int N,
                                                             int64_t rows_per_block, double *__restrict__ part) {
    __shared__ double red[256];
    const int per = 256 / N;                  // rows handled side by side
    const int c = threadIdx.x % N, ro = threadIdx.x / N;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    double s = 0.0;
    if (ro < per)
        for (int64_t r = r0 + ro; r < r1; r += per) s += (double)x[r * N + c];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < N) {
        double t = 0.0;
        for (int k = 0; k < per; ++k) t += red[k * N + threadIdx.x];
        part[(int64_t)blockIdx.x * N + threadIdx.x] = t;
    }
}

// stage 2: one workgroup per column folds the block partials with a fixed-shape tree
__global__ __launch_bounds__(256) void colsum_final_kernel(const double *__restrict__ part, int nblocks, int N,
                                                           float *__restrict__ out) {
    __shared__ double red[256];
    const int c = blockIdx.x;
    double t = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += 256) t += part[(int64_t)b * N + c];
    red[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = (float)red[0];
}

bool geo(int64_t Cout, int64_t Cin, int64_t kh, int64_t kw, int64_t H, int64_t W, BoardGeo &g) {
    if (Cout < 1 || Cin < 1 || kh < 1 || kw < 1 || H < 1 || W < 1 || kh % 2 == 0 || kw % 2 == 0) return false;
    if (H * W > 64 || Cout * H * W > 65536 || Cin * H * W > 65536) return false;
    g.Cout = (int)Cout; g.Cin = (int)Cin; g.kh = (int)kh; g.kw = (int)kw; g.H = (int)H; g.W = (int)W;
    g.HW = (int)(H * W); g.ph = (int)(kh / 2); g.pw = (int)(kw / 2);
    return true;
}

int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)e;
}

}  // namespace

extern "C" {

int hrl_board_weight(const float *w, int64_t Cout, int64_t Cin, int64_t kh, int64_t kw, int64_t H, int64_t W,
                     float *w_board, void *stream) {
    BoardGeo g;
    if (!w || !w_board || !geo(Cout, Cin, kh, kw, H, W, g)) return HRL_EINVAL;
    const int64_t n = (int64_t)g.Cin * g.HW * g.Cout * g.HW;
    const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
    hipLaunchKernelGGL(board_weight_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), w, g,
                       w_board);
    return status();
}

int hrl_board_fold(const float *g_board, int64_t Cout, int64_t Cin, int64_t kh, int64_t kw, int64_t H, int64_t W,
                   float *g_w, void *stream) {
    BoardGeo g;
    if (!g_board || !g_w || !geo(Cout, Cin, kh, kw, H, W, g)) return HRL_EINVAL;
    const int n = g.Cout * g.Cin * g.kh * g.kw;
    hipLaunchKernelGGL(board_fold_kernel, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                       g_board, g, g_w);
    return status();
}

int hrl_board_bias(const float *b, int64_t Cout, int64_t HW, float *b_board, void *stream) {
    if (!b || !b_board || Cout < 1 || HW < 1 || Cout * HW > 65536) return HRL_EINVAL;
    const int n = (int)(Cout * HW);
    hipLaunchKernelGGL(board_bias_kernel, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), b,
                       (int)Cout, (int)HW, b_board);
    return status();
}

int hrl_board_bias_fold(const float *g_board, int64_t Cout, int64_t HW, float *g_b, void *stream) {
    if (!g_board || !g_b || Cout < 1 || HW < 1 || Cout * HW > 65536) return HRL_EINVAL;
    hipLaunchKernelGGL(board_bias_fold_kernel, dim3((int)((Cout + 63) / 64)), dim3(64), 0,
                       static_cast<hipStream_t>(stream), g_board, (int)Cout, (int)HW, g_b);
    return status();
}

int64_t hrl_colsum_workspace_bytes(int64_t M, int64_t N) {
    if (M < 1 || N < 1 || N > 256) return -1;
    return 1024 * N * 8;
}

int hrl_colsum(const float *x, int64_t M, int64_t N, float *out, void *workspace, int64_t workspace_bytes,
               void *stream) {
    if (!x || !out || !workspace || M < 1 || N < 1 || N > 256) return HRL_EINVAL;
    if (workspace_bytes < hrl_colsum_workspace_bytes(M, N)) return HRL_EINVAL;
    int64_t nb = (M + 127) / 128;
    nb = nb > 1024 ? 1024 : nb;
    const int64_t rpb = (M + nb - 1) / nb;
    nb = (M + rpb - 1) / rpb;
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *part = static_cast<double *>(workspace);
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)nb), dim3(256), 0, s, x, M, (int)N, rpb, part);
    int rc = status();
    if (rc) return rc;
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)N), dim3(256), 0, s, part, (int)nb, (int)N, out);
    return status();
}

}  // extern "C"
