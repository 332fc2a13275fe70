// Cycles per MFMA, back-to-back on one wave (4 independent accumulators): 16x16x16 vs 16x16x32 bf16, 16x16x4 f32.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int N = 4096;
__global__ void k16(float *out, long long *cyc) {
    s16x4 a = {(short)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (short)threadIdx.x};
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c3, 0, 0, 0);
    }
    long long t1 = clock64();
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k32(float *out, long long *cyc) {
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(float)(threadIdx.x + i); b[i] = (__bf16)(float)i; }
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
    }
    long long t1 = clock64();
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void kf32(float *out, long long *cyc) {
    float a = threadIdx.x, b = 1.f;
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    long long t1 = clock64();
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    float *out; long long *cyc, h;
    hipMalloc(&out, 64 * 4); hipMalloc(&cyc, 8);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k16, 1, 64, 0, 0, out, cyc); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("16x16x16 bf16: %.2f cycles/MFMA\n", (double)h / (4.0 * N));
        hipLaunchKernelGGL(k32, 1, 64, 0, 0, out, cyc); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("16x16x32 bf16: %.2f cycles/MFMA\n", (double)h / (4.0 * N));
        hipLaunchKernelGGL(kf32, 1, 64, 0, 0, out, cyc); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("16x16x4 f32:   %.2f cycles/MFMA\n", (double)h / (4.0 * N));
    }
    return 0;
}
