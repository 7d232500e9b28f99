// Back-to-back issue cost (cycles per MFMA, one wave per SIMD, 4 independent accumulators) of the three
// MFMA forms the bf16x6 kernels mix: 16x16x32 bf16, the legacy 16x16x16 bf16 (_1k) and 16x16x4 f32.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

template <int KIND>
__global__ void k_rate(float* out, long long* cyc, float seed) {
    f32x4 a0 = {seed, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    bf16x8 x8;
    s16x4 x4;
    for (int j = 0; j < 8; ++j) x8[j] = (__bf16)(seed * j);
    for (int j = 0; j < 4; ++j) x4[j] = (short)(threadIdx.x + j);
    const float xf = seed * threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < ITERS; ++i) {
        if (KIND == 0) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x8, x8, a3, 0, 0, 0);
        } else if (KIND == 1) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x4, x4, a3, 0, 0, 0);
        } else {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xf, xf, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xf, xf, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(xf, xf, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(xf, xf, a3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    const f32x4 s = a0 + a1 + a2 + a3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 64 * sizeof(float));
    hipMalloc(&cyc, sizeof(long long));
    const char* names[3] = {"16x16x32 bf16", "16x16x16 bf16 (_1k)", "16x16x4 f32"};
    for (int k = 0; k < 3; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            if (k == 0) hipLaunchKernelGGL(k_rate<0>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0f);
            if (k == 1) hipLaunchKernelGGL(k_rate<1>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0f);
            if (k == 2) hipLaunchKernelGGL(k_rate<2>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0f);
            hipDeviceSynchronize();
        }
        long long c = 0;
        hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        printf("%-22s %.2f cycles per MFMA (s_memtime/readcyclecounter ticks)\n", names[k], (double)c / (4.0 * ITERS));
    }
    return 0;
}
