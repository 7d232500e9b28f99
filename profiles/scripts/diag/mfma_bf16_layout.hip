// Layout check of the gfx950 bf16 MFMAs used by the bf16x6 kernels, with exact small-integer data:
// C = A * B for one 16x16 tile, A/B filled per the assumed lane maps
//   16x16x32: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j < 8
//   16x16x16: lane l holds A[l&15][4(l>>4)+j], B[4(l>>4)+j][l&15], j < 4
// C[4(l>>4)+r][l&15] in register r. Prints max |C - C_ref| for both shapes (0 expected).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* A32, const float* B32, const float* A16, const float* B16, float* C32, float* C16) {
    const int l = threadIdx.x, lr = l & 15, lg = l >> 4;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)A32[lr * 32 + 8 * lg + j]; b[j] = (__bf16)B32[(8 * lg + j) * 16 + lr]; }
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C32[(4 * lg + r) * 16 + lr] = c[r];
    bf16x4 a4, b4;
    for (int j = 0; j < 4; ++j) { a4[j] = (__bf16)A16[lr * 16 + 4 * lg + j]; b4[j] = (__bf16)B16[(4 * lg + j) * 16 + lr]; }
    f32x4 d = {0, 0, 0, 0};
    d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a4), __builtin_bit_cast(s16x4, b4), d, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C16[(4 * lg + r) * 16 + lr] = d[r];
}

int main() {
    float hA32[16 * 32], hB32[32 * 16], hA16[16 * 16], hB16[16 * 16], hC32[256], hC16[256];
    for (int i = 0; i < 16 * 32; ++i) { hA32[i] = (float)((i * 7) % 11 - 5); hB32[i] = (float)((i * 5) % 13 - 6); }
    for (int i = 0; i < 256; ++i) { hA16[i] = (float)((i * 3) % 7 - 3); hB16[i] = (float)((i * 11) % 9 - 4); }
    float *dA32, *dB32, *dA16, *dB16, *dC32, *dC16;
    hipMalloc(&dA32, sizeof hA32); hipMalloc(&dB32, sizeof hB32); hipMalloc(&dA16, sizeof hA16);
    hipMalloc(&dB16, sizeof hB16); hipMalloc(&dC32, sizeof hC32); hipMalloc(&dC16, sizeof hC16);
    hipMemcpy(dA32, hA32, sizeof hA32, hipMemcpyHostToDevice); hipMemcpy(dB32, hB32, sizeof hB32, hipMemcpyHostToDevice);
    hipMemcpy(dA16, hA16, sizeof hA16, hipMemcpyHostToDevice); hipMemcpy(dB16, hB16, sizeof hB16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA32, dB32, dA16, dB16, dC32, dC16);
    hipMemcpy(hC32, dC32, sizeof hC32, hipMemcpyDeviceToHost); hipMemcpy(hC16, dC16, sizeof hC16, hipMemcpyDeviceToHost);
    double e32 = 0, e16 = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double r32 = 0, r16 = 0;
            for (int k2 = 0; k2 < 32; ++k2) r32 += hA32[i * 32 + k2] * hB32[k2 * 16 + j];
            for (int k2 = 0; k2 < 16; ++k2) r16 += hA16[i * 16 + k2] * hB16[k2 * 16 + j];
            e32 = fmax(e32, fabs(hC32[i * 16 + j] - r32));
            e16 = fmax(e16, fabs(hC16[i * 16 + j] - r16));
        }
    printf("16x16x32 bf16 max err %g   16x16x16 bf16 max err %g\n", e32, e16);
    return (e32 == 0 && e16 == 0) ? 0 : 1;
}
