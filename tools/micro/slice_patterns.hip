// Streaming-read rate of the heads forward's slice pattern (gfx950): one wave per 64-row block of 288-float rows,
// the row read slice by slice (one row per lane after the LDS transpose), two slices in flight.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/slice_patterns tools/micro/slice_patterns.hip
//   tools/micro/slice_patterns            (on the GPU box)
//
//  S144  heads_fwd_kernel's slices: 4 channels = 36 floats = 144 B of every row (runs straddle 128-B lines, and
//        the next slice re-touches the straddled lines)
//  S128  line-aligned slices: 32 floats = 128 B of every row, 9 per row
//  S384  3 lines = 96 floats per slice, 3 per row
//  CONT  the block's 73,728 bytes read contiguously (float4 per lane), 8 steps
// Values are summed so nothing is dead; 2048 blocks (N = 131,072 rows, 151 MB), grids of 1024 / 2048 / 4096 waves.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kRow = 288;

template <int SF, int DEPTH>   // SF floats per row slice (multiple of 4), DEPTH slices in flight
__global__ __launch_bounds__(64) void slices(const float *__restrict__ h, int64_t N, float *out) {
    constexpr int kNS = kRow / SF;
    constexpr int kV = SF * 64 / 4 / 64;   // float4 per lane per slice
    const int lane = threadIdx.x;
    float acc = 0.f;
    for (int64_t base = (int64_t)blockIdx.x * 64; base < N; base += (int64_t)gridDim.x * 64) {
        float4 st[DEPTH][kV];
        auto load = [&](float4 (&v)[kV], int s) {
#pragma unroll
            for (int k = 0; k < kV; ++k) {
                const int i = k * 64 + lane;
                const int r = i / (SF / 4), c4 = i - r * (SF / 4);
                v[k] = *reinterpret_cast<const float4 *>(h + (base + r) * kRow + s * SF + c4 * 4);
            }
        };
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) load(st[d], d);
#pragma unroll
        for (int s = 0; s < kNS; ++s) {
            float4 (&v)[kV] = st[s % DEPTH];
#pragma unroll
            for (int k = 0; k < kV; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
            if (s + DEPTH < kNS) load(v, s + DEPTH);
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

__global__ __launch_bounds__(64) void contiguous(const float *__restrict__ h, int64_t N, float *out) {
    const int lane = threadIdx.x;
    float acc = 0.f;
    constexpr int kV = 64 * kRow / 4 / 64 / 8;   // float4 per lane per step (36), 8 steps
    for (int64_t base = (int64_t)blockIdx.x * 64; base < N; base += (int64_t)gridDim.x * 64) {
        const float4 *p = reinterpret_cast<const float4 *>(h + base * kRow);
        float4 a[kV], b[kV];
#pragma unroll
        for (int k = 0; k < kV; ++k) a[k] = p[k * 64 + lane];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
            for (int k = 0; k < kV; ++k) {
                if (s + 1 < 8) b[k] = p[((s + 1) * kV + k) * 64 + lane];
                acc += a[k].x + a[k].y + a[k].z + a[k].w;
                a[k] = b[k];
            }
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

int main() {
    const int64_t N = 131072;
    const size_t bytes = (size_t)N * kRow * 4;
    // two buffers, alternated, so a launch does not find its input in the 256 MB Infinity Cache
    float *h[2], *out;
    hipMalloc(&h[0], bytes); hipMalloc(&h[1], bytes);
    hipMalloc(&out, 4096 * 64 * 4);
    hipMemset(h[0], 0, bytes); hipMemset(h[1], 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 20;
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 4; ++i) launch(h[i & 1]);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < iters; ++i) launch(h[i & 1]);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / iters;
        printf("%-40s %8.2f us  %6.2f TB/s\n", name, us, (double)bytes / us / 1e6);
    };
    for (int grid : {1024, 2048, 4096}) {
        printf("grid %d waves\n", grid);
        run("S144 depth 2 (heads_fwd)", [&](const float *p) { slices<36, 2><<<grid, 64>>>(p, N, out); });
        run("S144 depth 3", [&](const float *p) { slices<36, 3><<<grid, 64>>>(p, N, out); });
        run("S128 depth 2", [&](const float *p) { slices<32, 2><<<grid, 64>>>(p, N, out); });
        run("S128 depth 3", [&](const float *p) { slices<32, 3><<<grid, 64>>>(p, N, out); });
        run("S384 depth 2", [&](const float *p) { slices<96, 2><<<grid, 64>>>(p, N, out); });
        run("CONT", [&](const float *p) { contiguous<<<grid, 64>>>(p, N, out); });
    }
    return 0;
}
