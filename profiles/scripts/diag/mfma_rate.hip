// Issue cost (cycles per MFMA per SIMD) of the MFMA forms the bf16x6 kernels mix -- 16x16x32 bf16, the legacy
// 16x16x16 bf16 (_1k) and 16x16x4 f32 -- with 1, 2 or 4 independent accumulator chains per wave (a chain = each
// MFMA's C operand is the previous one's result, as in bf16x6's six products), one wave per SIMD and four.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 2048;

template <int KIND>
__device__ __forceinline__ f32x4 op(f32x4 a, bf16x8 x8, s16x4 x4, float xf) {
    if (KIND == 0) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a, 0, 0, 0);
    if (KIND == 1) return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(xf, xf, a, 0, 0, 0);
}

template <int KIND, int NACC>
__global__ void k_rate(float* out, long long* cyc, float seed) {
    f32x4 a[4];
    for (int j = 0; j < 4; ++j) a[j] = f32x4{seed, 0, 0, 0};
    bf16x8 x8;
    s16x4 x4;
    for (int j = 0; j < 8; ++j) x8[j] = (__bf16)(seed * j);
    for (int j = 0; j < 4; ++j) x4[j] = (short)(threadIdx.x + j);
    const float xf = seed * threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j % NACC] = op<KIND>(a[j % NACC], x8, x4, xf);
    }
    const long long t1 = __builtin_readcyclecounter();
    f32x4 s = a[0];
    for (int j = 1; j < NACC; ++j) s += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int KIND, int NACC>
double run(float* out, long long* cyc, int threads) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((k_rate<KIND, NACC>), dim3(1), dim3(threads), 0, 0, out, cyc, 1.0f);
        hipDeviceSynchronize();
    }
    long long c = 0;
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    // cycles per MFMA per SIMD: waves per SIMD = threads / 256
    return (double)c / (4.0 * ITERS * (threads / 256.0 < 1 ? 1.0 : threads / 256.0));
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1024 * sizeof(float));
    hipMalloc(&cyc, sizeof(long long));
    const char* names[3] = {"16x16x32 bf16", "16x16x16 bf16 (_1k)", "16x16x4 f32"};
    for (int threads : {256, 1024}) {
        printf("%d waves per SIMD (cycles per MFMA per SIMD, readcyclecounter ticks)\n", threads / 256);
        printf("  %-22s %8.2f %8.2f %8.2f  (1 / 2 / 4 chains per wave)\n", names[0], run<0, 1>(out, cyc, threads),
               run<0, 2>(out, cyc, threads), run<0, 4>(out, cyc, threads));
        printf("  %-22s %8.2f %8.2f %8.2f\n", names[1], run<1, 1>(out, cyc, threads), run<1, 2>(out, cyc, threads),
               run<1, 4>(out, cyc, threads));
        printf("  %-22s %8.2f %8.2f %8.2f\n", names[2], run<2, 1>(out, cyc, threads), run<2, 2>(out, cyc, threads),
               run<2, 4>(out, cyc, threads));
    }
    return 0;
}
