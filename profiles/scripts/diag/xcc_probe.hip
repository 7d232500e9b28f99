// Which XCD runs workgroup b? (checks the b % 8 round-robin the XCD-aware launches assume). Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_xcc(int* out) {
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
        out[blockIdx.x] = (int)x;
    }
}
int main() {
    const int n = 1024;
    int* d;
    hipMalloc(&d, n * sizeof(int));
    hipLaunchKernelGGL(k_xcc, dim3(n), dim3(512), 0, 0, d);
    int h[n];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < n; ++b) bad += h[b] != b % 8;
    printf("blocks whose XCC != b %% 8: %d of %d; first 24:", bad, n);
    for (int b = 0; b < 24; ++b) printf(" %d", h[b]);
    printf("\n");
    return 0;
}
