// Rounding of the C-operand accumulation of v_mfma_f32_16x16x32_bf16 (diagnostic, round 5): one wave accumulates
// NSTEP MFMAs of random positive bf16 operands into one accumulator chain; the host compares every lane's result with
// the exact fp64 sum and with an fp32 round-to-nearest-even emulation of the same chain. A systematic shortfall (mean
// signed error well below zero) means the accumulation truncates. Build: hipcc --offload-arch=gfx950 -O3 -o _ab/mfma_acc_bias
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <random>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NSTEP = 512;

__global__ void k(const bf16x8* a, const bf16x8* b, float* out, int fresh) {
    const int l = threadIdx.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < NSTEP; ++s) {
        if (fresh) {   // block result from zero, added with an fp32 VALU add (round to nearest even)
            const f32x4 t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s * 64 + l], b[s * 64 + l], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            sum += t;
        } else {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s * 64 + l], b[s * 64 + l], acc, 0, 0, 0);
        }
    }
    const f32x4 r = fresh ? sum : acc;
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = r[i];
}

int main() {
    std::mt19937 g(1);
    std::uniform_real_distribution<float> U(0.5f, 1.0f);
    std::vector<__bf16> A(NSTEP * 64 * 8), B(NSTEP * 64 * 8);
    for (auto& x : A) x = (__bf16)U(g);
    for (auto& x : B) x = (__bf16)U(g);
    bf16x8 *da, *db;
    float* dout;
    hipMalloc(&da, A.size() * 2);
    hipMalloc(&db, B.size() * 2);
    hipMalloc(&dout, 256 * 4);
    hipMemcpy(da, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    // exact fp64 reference and fp32-RNE emulation per output (row i = 4(l>>4)+r, col j = l & 15), lane l holds
    // A[l & 15][8(l >> 4) + jj] and B[8(l >> 4) + jj][l & 15]
    std::vector<double> ex(256, 0.0);
    std::vector<float> rne(256, 0.f);
    for (int s = 0; s < NSTEP; ++s) {
        std::vector<double> blk(256, 0.0);
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double d = 0.0;
                for (int kk = 0; kk < 32; ++kk) {
                    const int la = i + 16 * (kk / 8), lb = j + 16 * (kk / 8);
                    d += (double)(float)A[(s * 64 + la) * 8 + kk % 8] * (double)(float)B[(s * 64 + lb) * 8 + kk % 8];
                }
                blk[i * 16 + j] = d;
            }
        for (int e = 0; e < 256; ++e) {
            ex[e] += blk[e];
            rne[e] = (float)((double)rne[e] + (double)(float)blk[e]);
        }
    }
    for (int fresh = 0; fresh < 2; ++fresh) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dout, fresh);
        std::vector<float> out(256);
        hipMemcpy(out.data(), dout, 256 * 4, hipMemcpyDeviceToHost);
        double me = 0, mr = 0, ms = 0;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
                const int i = 4 * (l >> 4) + r, j = l & 15, e = i * 16 + j;
                const double ulp = std::ldexp(1.0, std::ilogb(ex[e]) - 23);
                me += (out[l * 4 + r] - ex[e]) / ulp;
                ms += std::fabs(out[l * 4 + r] - ex[e]) / ulp;
                mr += (rne[e] - ex[e]) / ulp;
            }
        printf("%s: %d steps, mean signed error %+.2f ulp (mean |err| %.2f), fp32 RNE chain emulation %+.2f ulp\n",
               fresh ? "fresh blocks + VALU add" : "MFMA C-chain          ", NSTEP, me / 256, ms / 256, mr / 256);
    }
    return 0;
}
