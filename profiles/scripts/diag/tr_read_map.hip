// Exact-integer check of the side-A D-role operand maps (bf16x6 contraction):
//   A (16 o x 32 q): lane (lr, lg) element jj = G[q = 4lg + jj (jj<4) | 16 + 4lg + jj-4][o = lr]
//   B (32 q x 16 j): two ds_read_b64_tr_b16 of a row-major [32 q][112 j] bf16 image (224-B rows):
//     rows 4lg .. 4lg+3 and 16 + 4lg .. +3, columns 16t .. 16t+15; lane 4qq+pp supplies row r0+qq, cols +4pp
//   D[o][j] = sum_q G[q][o] Q[q][j]; lane holds D[o = 4lg + r][j = 16t + lr].
// Build: hipcc --offload-arch=gfx950 -O3 -o tr_read_map tr_read_map.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__global__ void k_map(const float* Q, const float* G, float* D) {
    __shared__ __attribute__((aligned(16))) __bf16 img[32 * 112];
    const int lane = threadIdx.x, lr = lane & 15, lg = lane >> 4;
    for (int i = lane; i < 32 * 112; i += 64) img[i] = (__bf16)Q[i];
    __syncthreads();
    bf16x8 a;
    for (int jj = 0; jj < 8; ++jj) {
        const int q = jj < 4 ? 4 * lg + jj : 16 + 4 * lg + jj - 4;
        a[jj] = (__bf16)G[q * 16 + lr];
    }
    for (int t = 0; t < 7; ++t) {
        typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
        const int qq = lr >> 2, pp = lr & 3;
        const __bf16* p0 = img + (4 * lg + qq) * 112 + 16 * t + 4 * pp;
        const __bf16* p1 = p0 + 16 * 112;
        const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p0));
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p1));
        bf16x8 b;
        for (int j = 0; j < 4; ++j) { b[j] = b0[j]; b[4 + j] = b1[j]; }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
        for (int r = 0; r < 4; ++r) D[(4 * lg + r) * 112 + 16 * t + lr] = acc[r];
    }
}

int main() {
    float hQ[32 * 112], hG[32 * 16], hD[16 * 112], ref[16 * 112];
    srand(7);
    for (int i = 0; i < 32 * 112; ++i) hQ[i] = (float)(rand() % 7 - 3);
    for (int i = 0; i < 32 * 16; ++i) hG[i] = (float)(rand() % 5 - 2);
    for (int o = 0; o < 16; ++o)
        for (int j = 0; j < 112; ++j) {
            float s = 0.f;
            for (int q = 0; q < 32; ++q) s += hG[q * 16 + o] * hQ[q * 112 + j];
            ref[o * 112 + j] = s;
        }
    float *Q, *G, *D;
    hipMalloc(&Q, sizeof(hQ)); hipMalloc(&G, sizeof(hG)); hipMalloc(&D, sizeof(hD));
    hipMemcpy(Q, hQ, sizeof(hQ), hipMemcpyHostToDevice);
    hipMemcpy(G, hG, sizeof(hG), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, Q, G, D);
    hipMemcpy(hD, D, sizeof(hD), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16 * 112; ++i) bad += hD[i] != ref[i];
    printf("tr_read_map: %d / %d mismatches\n", bad, 16 * 112);
    return bad != 0;
}
