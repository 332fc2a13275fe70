// Load-pattern microbenchmark for the chain block backward's staging (tools/micro, diagnostic only).
// 256 workgroups x 8 waves stream the (M, 288) fp32 tensors g, y, x (M = 131072) tile by tile, as
// conv3x3_block_bwd2_kernel's stage does, and fold every loaded float into one register (kept live).
//   mode 0: lane = (channel, half) holds 5 cells of 2 rows: b96 + b64 per row and tensor (12 loads per lane)
//   mode 1: lane = (channel, row) holds the 9 cells of 1 row: b128 + b128 + b32 per tensor (9 loads)
//   mode 2: row-major, coalesced: 2 rows per wave = 144 float4 per tensor, b128 (lanes 0..143) (9 loads)
//   mode 3: mode 0's cells with dwordx4+dword per row (b128 + b32)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(512) void k(const float *g, const float *y, const float *x, int64_t M, float *out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ch = lane & 31, hh = lane >> 5;
    const int64_t ntiles = M / 16;
    float acc = 0.f;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t e = t * 16 * 288;
        const __amdgpu_buffer_rsrc_t rs[3] = {rsrc(g + e, 16 * 288 * 4), rsrc(y + e, 16 * 288 * 4),
                                              rsrc(x + e, 16 * 288 * 4)};
#pragma unroll
        for (int k3 = 0; k3 < 3; ++k3) {
            if (MODE == 0 || MODE == 3) {
                const int rho0 = 2 * ((w + (ch >> 2)) & 7), c0 = hh ? 4 : 0;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int off = ((rho0 + r) * 288 + ch * 9 + c0) * 4;
                    if (MODE == 0) {
                        const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs[k3], off, 0, 0);
                        const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(rs[k3], off + 12, 0, 0);
                        acc += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) +
                               __uint_as_float(u.x) + __uint_as_float(u.y);
                    } else {
                        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs[k3], off, 0, 0);
                        const uint32_t u = __builtin_amdgcn_raw_buffer_load_b32(rs[k3], off + 16, 0, 0);
                        acc += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) +
                               __uint_as_float(v.w) + __uint_as_float(u);
                    }
                }
            } else if (MODE == 1) {
                const int rho = 2 * ((w + (ch >> 2)) & 7) + hh;
                const int off = (rho * 288 + ch * 9) * 4;
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs[k3], off, 0, 0);
                const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rs[k3], off + 16, 0, 0);
                const uint32_t u = __builtin_amdgcn_raw_buffer_load_b32(rs[k3], off + 32, 0, 0);
                acc += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w) +
                       __uint_as_float(v2.x) + __uint_as_float(v2.y) + __uint_as_float(v2.z) +
                       __uint_as_float(v2.w) + __uint_as_float(u);
            } else {
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    const int f = lane + 64 * m;
                    const int off = f < 144 ? (2 * w * 288 + 4 * f) * 4 : 16 * 288 * 4;
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs[k3], off, 0, 0);
                    acc += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) +
                           __uint_as_float(v.w);
                }
            }
        }
    }
    if (acc == 123.456f) out[threadIdx.x] = acc;
}

int main() {
    const int64_t M = 131072;
    const size_t n = M * 288;
    float *g, *y, *x, *o;
    hipMalloc(&g, n * 4); hipMalloc(&y, n * 4); hipMalloc(&x, n * 4); hipMalloc(&o, 4096);
    hipMemset(g, 0, n * 4); hipMemset(y, 0, n * 4); hipMemset(x, 0, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 4; ++mode) {
        auto run = [&]() {
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, g, y, x, M, o);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, g, y, x, M, o);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, g, y, x, M, o);
            if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, g, y, x, M, o);
        };
        for (int i = 0; i < 3; ++i) run();
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) run();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / 20;
        printf("mode %d: %.1f us per launch, %.2f TB/s (453 MB)\n", mode, us, 3.0 * n * 4 / us / 1e6);
    }
    return 0;
}
