// Standalone check of the bf16x6 fused forward against the fp32 fused forward (same source file, same
// random weights / inputs): prints the max |h_bf - h_fp32| / max|h_fp32| per layer. Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I vi-hmc_amd/csrc \
//         vi-hmc_amd/scripts/diag/fused_bf_vs_fp32.hip vi-hmc_amd/csrc/vihmc_fused.hip -o /tmp/fbchk
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include "vihmc_internal.h"

using namespace vihmc;

int main() {
    const int C = 16, NL = 8, rows[2] = {1000, 10201};
    const int64_t blk = 100 * 100 + 100, dp = NL * blk + 64;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> W(C * dp);
    for (auto& x : W) x = 0.1f * nd(rng);
    float *dW, *dIn[2], *dOa[2], *dOb[2];
    hipMalloc(&dW, W.size() * 4);
    hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice);
    FusedArgs a{};
    a.C = C; a.packed = dW; a.dp = dp;
    for (int net = 0; net < 2; ++net) {
        std::vector<float> in((size_t)C * rows[net] * 100);
        for (auto& x : in) x = std::tanh(nd(rng));
        hipMalloc(&dIn[net], in.size() * 4);
        hipMemcpy(dIn[net], in.data(), in.size() * 4, hipMemcpyHostToDevice);
        const int64_t ocs = (int64_t)NL * rows[net] * 100;
        hipMalloc(&dOa[net], C * ocs * 4);
        hipMalloc(&dOb[net], C * ocs * 4);
        FusedNet& f = a.net[net];
        f.in = dIn[net]; f.in_cs = (int64_t)rows[net] * 100; f.ldin = 100;
        f.out_cs = ocs; f.ldo = 100; f.nl = NL; f.rows = rows[net]; f.nblk = (rows[net] + 191) / 192;
        for (int j = 0; j < NL; ++j) {
            f.h_off[j] = (int64_t)j * rows[net] * 100;
            f.w_off[j] = 64 + j * blk;
            f.act[j] = j + 1 < NL ? ACT_TANH : ACT_ID;
        }
    }
    for (int net = 0; net < 2; ++net) a.net[net].out = dOa[net];
    if (launch_fwd_fused(a, 12, 0) != hipSuccess) { printf("launch fp32 failed\n"); return 1; }
    for (int net = 0; net < 2; ++net) a.net[net].out = dOb[net];
    if (launch_fwd_fused_bf(a, 0) != hipSuccess) { printf("launch bf failed\n"); return 1; }
    if (hipDeviceSynchronize() != hipSuccess) { printf("sync failed\n"); return 1; }
    for (int net = 0; net < 2; ++net) {
        const int64_t ocs = (int64_t)NL * rows[net] * 100;
        std::vector<float> A(C * ocs), B(C * ocs);
        hipMemcpy(A.data(), dOa[net], A.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(B.data(), dOb[net], B.size() * 4, hipMemcpyDeviceToHost);
        for (int j = 0; j < NL; ++j) {
            double e = 0, m = 0;
            int64_t worst = -1;
            for (int c = 0; c < C; ++c)
                for (int64_t i = 0; i < (int64_t)rows[net] * 100; ++i) {
                    const int64_t k = c * ocs + j * (int64_t)rows[net] * 100 + i;
                    m = std::fmax(m, std::fabs(A[k]));
                    const double d = std::fabs((double)A[k] - B[k]);
                    if (d > e) { e = d; worst = i; }
                }
            printf("net %d layer %d: max|h| %.4f  max|diff| %.3e  (row %lld col %lld)\n", net, j + 1, m, e,
                   (long long)(worst / 100), (long long)(worst % 100));
            if (j == 0) {
                printf("   per column tile:");
                for (int t = 0; t < 7; ++t) {
                    double et = 0;
                    for (int c = 0; c < C; ++c)
                        for (int r = 0; r < rows[net]; ++r)
                            for (int q = 16 * t; q < std::min(100, 16 * t + 16); ++q) {
                                const int64_t k = c * ocs + (int64_t)r * 100 + q;
                                et = std::fmax(et, std::fabs((double)A[k] - B[k]));
                            }
                    printf(" %.1e", et);
                }
                for (int ta = 0; ta < 7; ++ta) {
                    double ed = 0;
                    for (int r = 0; r < rows[net]; ++r)
                        for (int q = 0; q < 16 && 16 * ta + q < 100; ++q)
                            ed = std::fmax(ed, std::fabs((double)B[(int64_t)r * 100 + 80 + q] - A[(int64_t)r * 100 + 16 * ta + q]));
                    printf("\n   bf tile5 vs fp32 tile %d: %.1e", ta, ed);
                }
                printf("\n   per row mod 16 (tile 5):");
                for (int rr = 0; rr < 16; ++rr) {
                    double et = 0;
                    for (int r = rr; r < rows[net]; r += 16)
                        for (int q = 80; q < 96; ++q) et = std::fmax(et, std::fabs((double)A[(int64_t)r * 100 + q] - B[(int64_t)r * 100 + q]));
                    printf(" %.0e", et);
                }
                printf("\n");
            }
        }
    }
    return 0;
}
