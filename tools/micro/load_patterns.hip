// Streaming-read rate of the chain block backward's staging load pattern against contiguous loads (gfx950).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/load_patterns tools/micro/load_patterns.hip
//   tools/micro/load_patterns            (on the GPU box)
//
// Three 151 MB tensors (M = 131,072 rows of 288 floats, the bench size) read tile by tile (16 rows) by 256
// workgroups of 8 waves, one tile of loads in flight ahead in registers, values summed so nothing is dead:
//  A  conv3x3_block_bwd2_kernel's lanes: lane (ch, hh) of wave W takes rows rho0, rho0 + 1 with
//     rho0 = 2 ((W + ch / 4) & 7) and cells c0 .. c0 + 4 (c0 = 4 hh) of channel ch: buffer_load b96 + b64 per row
//  B  the same 20-byte runs with rho0 = 2 W (one row pair per wave instruction, no diagonal)
//  C  contiguous 16-byte loads: lane l of wave W takes float4s W * 64 + l + 512 k of the tile (all three tensors)
// and the matching store shapes for a 151 MB output (per-lane 20-byte runs vs contiguous float4).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kRow = 288, kTile = 16, kWaves = 8;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(512) void read3(const float *g, const float *y, const float *x, int64_t M, float *out) {
    const int lane = threadIdx.x & 63, W = threadIdx.x >> 6, ch = lane & 31, hh = lane >> 5;
    const int rho0 = MODE == 0 ? 2 * ((W + (ch >> 2)) & 7) : 2 * W;
    const int c0 = hh ? 4 : 0;
    const int ldoff = (rho0 * kRow + ch * 9 + c0) * 4;
    const int64_t ntiles = M / kTile;
    float acc = 0.f;
    const __amdgpu_buffer_rsrc_t rs[3] = {rsrc(g, M * kRow * 4), rsrc(y, M * kRow * 4), rsrc(x, M * kRow * 4)};
    if (MODE == 2) {
        u32x4 v[3][3];   // 3 tensors x 2.25 float4 per lane (1152 per tile / 512 lanes): 2 full + a partial third
        for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const uint32_t base = (uint32_t)(t * kTile * kRow * 4);
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int i = j * 512 + threadIdx.x;
                    v[k][j] = i < 1152 ? __builtin_amdgcn_raw_buffer_load_b128(rs[k], base + i * 16, 0, 0)
                                       : (u32x4){0u, 0u, 0u, 0u};
                }
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    acc += __uint_as_float(v[k][j].x) + __uint_as_float(v[k][j].y) + __uint_as_float(v[k][j].z) +
                           __uint_as_float(v[k][j].w);
        }
    } else {
        for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const uint32_t base = (uint32_t)(t * kTile * kRow * 4);
            float d[3][2][5];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t off = base + ldoff + r * kRow * 4;
                    const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(rs[k], off, 0, 0);
                    const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(rs[k], off + 12, 0, 0);
                    d[k][r][0] = __uint_as_float(a.x); d[k][r][1] = __uint_as_float(a.y);
                    d[k][r][2] = __uint_as_float(a.z); d[k][r][3] = __uint_as_float(b.x);
                    d[k][r][4] = __uint_as_float(b.y);
                }
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int i = 0; i < 5; ++i) acc += d[k][r][i];
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// stores: MODE 0 = per-lane 20-byte runs (b128 + b32 at row * 288 + co * 9 + q0, four rows per lane as the input-
// gradient waves' 16x16 accumulators give them), MODE 1 = contiguous float4
template <int MODE>
__global__ __launch_bounds__(512) void write1(float *o, int64_t M) {
    const int lane = threadIdx.x & 63, W = threadIdx.x >> 6;
    const int64_t ntiles = M / kTile;
    const __amdgpu_buffer_rsrc_t ro = rsrc(o, M * kRow * 4);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t base = (uint32_t)(t * kTile * kRow * 4);
        if (MODE == 0) {
            // wave W < 4: column tile W & 1, cells 4..8 (W < 2) or 0..3; waves 4-7 mirror them so all 8 store
            const int ct = W & 1, q0 = (W & 2) ? 0 : 4, nq = (W & 2) ? 4 : 5;
            const int co = ct * 16 + (lane & 15);
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const int row = (lane >> 4) * 4 + rr + 2 * (W >> 2);
                const uint32_t off = base + (row * kRow + co * 9 + q0) * 4;
                __builtin_amdgcn_raw_buffer_store_b128((u32x4){1u, 2u, 3u, 4u}, ro, off, 0, 0);
                if (nq > 4) __builtin_amdgcn_raw_buffer_store_b32(5u, ro, off + 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int i = j * 512 + threadIdx.x;
                if (i < 1152) __builtin_amdgcn_raw_buffer_store_b128((u32x4){1u, 2u, 3u, 4u}, ro, base + i * 16, 0, 0);
            }
        }
    }
}

int main() {
    const int64_t M = 131072;
    const size_t bytes = (size_t)M * kRow * 4;
    float *g, *y, *x, *o, *out;
    hipMalloc(&g, bytes); hipMalloc(&y, bytes); hipMalloc(&x, bytes); hipMalloc(&o, bytes);
    hipMalloc(&out, 256 * 512 * 4);
    hipMemset(g, 0, bytes); hipMemset(y, 0, bytes); hipMemset(x, 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 20;
    auto run = [&](const char *name, auto launch, double mb) {
        for (int i = 0; i < 3; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < iters; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / iters;
        printf("%-44s %8.2f us  %6.2f TB/s\n", name, us, mb / us / 1e6);
    };
    const double rd = 3.0 * bytes, wr = (double)bytes;
    for (int grid : {256, 512}) {
        printf("grid %d\n", grid);
        run("A bb2 lanes (diagonal rows, b96+b64)", [&] { read3<0><<<grid, 512>>>(g, y, x, M, out); }, rd);
        run("B 20-byte runs, one row pair per wave", [&] { read3<1><<<grid, 512>>>(g, y, x, M, out); }, rd);
        run("C contiguous float4", [&] { read3<2><<<grid, 512>>>(g, y, x, M, out); }, rd);
        run("store: 20-byte runs (b128 + b32)", [&] { write1<0><<<grid, 512>>>(o, M); }, wr);
        run("store: contiguous float4", [&] { write1<1><<<grid, 512>>>(o, M); }, wr);
    }
    return 0;
}
