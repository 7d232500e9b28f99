// HIP kernels for the VI-HMC log-posterior + gradient on MI355X (gfx950, CDNA4).
//
// All GEMM-shaped work runs on the fp32-input MFMA v_mfma_f32_16x16x4_f32 (exact fp32, the only
// fp32-parity matrix path on gfx950). Operand maps (cdna_hip_programming.md §3):
//   A (16x4): lane l holds A[l&15][l>>4]      B (4x16): lane l holds B[l>>4][l&15]
//   C (16x16): lane l, register r holds C[4*(l>>4)+r][l&15]
// Row-major operands whose contraction index is contiguous are loaded 16 k at a time as one
// float4 per lane: lane group g = l>>4 takes k = kb+4g..kb+4g+3 and MFMA step s uses component s,
// i.e. step s covers k = {kb+s, kb+4+s, kb+8+s, kb+12+s} on both operands (a k-permutation, exact).
//
// Reference math being replaced (file:line in /root/reference):
//   Functional_DeepONet.functional_model  Operator_network/VI_HMC/my_make_func.py:44-83
//   GaussianNLLLoss / regression ll        Operator_network/VI_HMC/main_VI_HMC_burgers.py:157-163
//   Normal prior                           Operator_network/VI_HMC/main_VI_HMC_burgers.py:74-102
//   Functional_Net.functional_model       Neural_network/VI_HMC/my_make_func.py:52-73
// and torch.autograd.grad through them (hamiltorch params_grad).
#include "vihmc_internal.h"
#include <algorithm>
#include <cstdlib>

namespace vihmc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float act_apply(int act, float z) {
    if (act == ACT_TANH) return tanhf(z);
    if (act == ACT_RELU) return fmaxf(z, 0.f);
    if (act == ACT_SINE) return sinf(z);
    return z;
}

// d act / d z expressed through the stored activation output (torch tanh_backward / threshold_backward)
__device__ __forceinline__ float act_grad_from_out(int act, float h) {
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// =============================================================================================
// Small kernels: packed-weight init / scatter, fixed-order partial reduction, likelihood
// finalisation, gradient gather + prior.
// =============================================================================================
__global__ void k_init_packed(float* packed, int64_t dp, const float* frozen, const int32_t* map_w,
                              const int32_t* map_wt, int64_t D) {
    const int c = blockIdx.y;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < D; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = frozen[i];
        packed[c * dp + map_w[i]] = v;
        const int32_t t = map_wt[i];
        if (t >= 0) packed[c * dp + t] = v;
    }
}

// sampled value k of chain c -> packed W, W^T and (when kept by the scatter) the forward's weight images. The
// destination offsets are read first (scatter_idx) so a caller can issue them beside its other loads: float
// stores may alias the float loads that follow them, so a load placed after a store waits for it
struct ScatterIdx {
    int32_t w, wt, iw, ifl, tw, tfl;
};
__device__ __forceinline__ ScatterIdx scatter_idx(const int32_t* smap_w, const int32_t* smap_wt, const ScatterImg& si,
                                                  int k) {
    ScatterIdx x;
    x.w = smap_w[k];
    x.wt = smap_wt[k];
    x.iw = si.img_w != nullptr ? si.img_w[k] : -1;
    x.ifl = si.img_w != nullptr ? si.img_f[k] : -1;
    x.tw = si.timg_w != nullptr ? si.timg_w[k] : -1;
    x.tfl = si.timg_w != nullptr ? si.timg_f[k] : -1;
    return x;
}

__device__ __forceinline__ void scatter_store(float* packed, int64_t dp, const ScatterImg& si, int c,
                                              const ScatterIdx& x, float v) {
    packed[c * dp + x.w] = v;
    if (x.wt >= 0) packed[c * dp + x.wt] = v;
    if (x.iw >= 0 || x.ifl >= 0) {
        unsigned char* img = si.img + c * si.img_cs;
        if (x.iw >= 0) {
            // the three planes exactly as k_split_wimg splits them
            const __bf16 a = (__bf16)v;
            const float r = v - (float)a;
            const __bf16 b = (__bf16)r;
            const __bf16 cc = (__bf16)(r - (float)b);
            *reinterpret_cast<__bf16*>(img + x.iw) = a;
            *reinterpret_cast<__bf16*>(img + x.iw + si.plane) = b;
            *reinterpret_cast<__bf16*>(img + x.iw + 2 * si.plane) = cc;
        }
        if (x.ifl >= 0) *reinterpret_cast<float*>(img + x.ifl) = v;
    }
    if (x.tw >= 0 || x.tfl >= 0) {
        unsigned char* img = si.timg + c * si.timg_cs;
        if (x.tw >= 0) {
            const __bf16 a = (__bf16)v;
            const float r = v - (float)a;
            const __bf16 b = (__bf16)r;
            const __bf16 cc = (__bf16)(r - (float)b);
            *reinterpret_cast<__bf16*>(img + x.tw) = a;
            *reinterpret_cast<__bf16*>(img + x.tw + si.tplane) = b;
            *reinterpret_cast<__bf16*>(img + x.tw + 2 * si.tplane) = cc;
        }
        if (x.tfl >= 0) *reinterpret_cast<float*>(img + x.tfl) = v;
    }
}

__device__ __forceinline__ void scatter_one(float* packed, int64_t dp, const int32_t* smap_w, const int32_t* smap_wt,
                                            const ScatterImg& si, int c, int k, float v) {
    scatter_store(packed, dp, si, c, scatter_idx(smap_w, smap_wt, si, k), v);
}

// one element per thread (a grid-stride loop left each thread's scattered stores' index loads serial: 10 us for
// config 4's 172,401 parameters)
__global__ __launch_bounds__(256) void k_scatter(float* packed, int64_t dp, const float* theta, int K,
                                                 const int32_t* smap_w, const int32_t* smap_wt, ScatterImg si) {
    const int c = blockIdx.y;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < K) scatter_one(packed, dp, smap_w, smap_wt, si, c, k, theta[(int64_t)c * K + k]);
}

__device__ double block_sum(double v, double* sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0) {
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    }
    __syncthreads();
    return t;   // valid in thread 0
}

__device__ void contract_stats_body(const StatsJob& J, int c) {
    __shared__ double sh[8];
    const bool alt = J.sel && chain_bit(J.bits, c);     // fit guard: this chain ran the other contraction form
    const double* st = alt ? J.stats2 + c * J.stats2_cs : J.stats + c * J.stats_cs;
    const int nw = alt ? J.n_waves2 : J.n_waves;
    double ssq = 0.0, gs = 0.0;
    for (int i = threadIdx.x; i < nw; i += blockDim.x) {
        ssq += st[2 * i];
        gs += st[2 * i + 1];
    }
    ssq = block_sum(ssq, sh);
    gs = block_sum(gs, sh);
    if (threadIdx.x == 0) {
        double ll;
        if (J.loss == 0) {
            const double v = fmax((double)J.tau_out, 1e-6);
            ll = -0.5 * (J.count * log(v) + ssq / v);
        } else {
            ll = -0.5 * (double)J.tau_out * ssq;
        }
        J.lik[c] = (float)ll;
        J.gp[c * J.gp_cs] = (float)gs;   // d ll / d b0 (packed slot 0)
        if (J.fit) J.fit[c] = (float)(ssq / fmax(*J.ysq, 1e-300));
    }
}

__global__ __launch_bounds__(256) void k_contract_stats(StatsJob J) { contract_stats_body(J, blockIdx.x); }


// Fixed-order sum of partial slabs (p = 0, 1, ... sequentially -- bitwise reproducible); grid slice y = n_jobs
// (when present) runs the likelihood statistics instead (saves their launch after side A); 4 consecutive
// elements per thread as float4 when the job's strides allow, 8 slab loads in flight ahead of the adds.
__global__ __launch_bounds__(256) void k_reduce(const ReduceJob* jobs, int n_jobs, StatsJob sj, int sel, ChainBits only) {
    if ((int)blockIdx.y == n_jobs) {                   // the optional likelihood-statistics slice
        if (blockIdx.x == 0) contract_stats_body(sj, blockIdx.z);
        return;
    }
    const ReduceJob J = jobs[blockIdx.y];
    const int c = blockIdx.z;
    if (sel && !chain_bit(only, c)) return;            // fit guard: a chain that ran the Gram form
    if (J.tiled) {
        // float4 quads of the tiled slabs (one accumulator quad of a dW tile each), summed over the slabs in the
        // row-major paths' fixed orders -- so both layouts give bitwise equal gradients -- then scattered to the
        // row-major destination
        __shared__ float4 tsum[3][64];
        const bool grouped = J.n_parts >= REDUCE_GROUP_MIN;
        const int x = grouped ? (int)(threadIdx.x & 63) : (int)threadIdx.x, g = grouped ? (int)(threadIdx.x >> 6) : 0;
        const int q = grouped ? (int)blockIdx.x * 64 + x : (int)blockIdx.x * 256 + x;
        if (grouped && (int)blockIdx.x * 256 >= J.len) return;   // block-uniform
        const bool ok = 4 * q < J.len;
        if (!grouped && !ok) return;
        // quad -> (row tile, column tile, lane) -> rows n = 16 tn + 4 lg + r, column j = 16 t + lr
        const int f = 4 * (ok ? q : 0), big = 6 * J.ntj * 256;
        int tn, t, lane;
        if (f < big) {
            const int T = f >> 8;
            tn = T / J.ntj;
            t = T - tn * J.ntj;
            lane = (f & 255) >> 2;
        } else {
            tn = 6;
            t = (f - big) >> 6;
            lane = ((f - big) & 63) >> 2;
        }
        const int j = 16 * t + (lane & 15), ni4 = (J.n_in + 3) & ~3;
        bool need = ok;
        if (J.samp && ok) {
            need = false;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nn = 16 * tn + 4 * (lane >> 4) + r;
                if (nn >= J.n_out) continue;
                if (j < J.n_in) need |= J.samp[(int64_t)nn * J.ldi + j] != 0;
                else if (j == ni4) need |= J.samp[(int64_t)J.n_out * J.ldi + nn] != 0;
            }
        }
        const float* sp = J.src + c * J.in_cs + (ok ? 4 * q : 0);
        const int64_t st = J.part_stride;
        const int n = need ? J.n_parts : 0;
        float4 s = {0.f, 0.f, 0.f, 0.f};
        if (grouped) {
            int p = g;
            for (; p + 28 < n; p += 32) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(sp + (p + 4 * u) * st);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s.x += v[u].x;
                    s.y += v[u].y;
                    s.z += v[u].z;
                    s.w += v[u].w;
                }
            }
            for (; p < n; p += 4) {
                const float4 v = *reinterpret_cast<const float4*>(sp + p * st);
                s.x += v.x;
                s.y += v.y;
                s.z += v.z;
                s.w += v.w;
            }
            if (g > 0) tsum[g - 1][x] = s;
            __syncthreads();
            if (g != 0 || !need) return;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s.x += tsum[k][x].x;
                s.y += tsum[k][x].y;
                s.z += tsum[k][x].z;
                s.w += tsum[k][x].w;
            }
        } else {
            int p = 0;
            for (; p + 8 <= n; p += 8) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(sp + (p + u) * st);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    s.x += v[u].x;
                    s.y += v[u].y;
                    s.z += v[u].z;
                    s.w += v[u].w;
                }
            }
            for (; p < n; ++p) {
                const float4 v = *reinterpret_cast<const float4*>(sp + p * st);
                s.x += v.x;
                s.y += v.y;
                s.z += v.z;
                s.w += v.w;
            }
        }
        if (!need) return;
        float* d = J.dst + c * J.dst_cs;
        const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int nn = 16 * tn + 4 * (lane >> 4) + r;
            if (nn >= J.n_out) continue;
            if (j < ni4) d[(int64_t)nn * J.ldi + j] = j < J.n_in ? sv[r] : 0.f;
            else if (j == ni4) d[(int64_t)J.n_out * J.ldi + nn] = sv[r];
        }
        return;
    }
    const bool vec =((J.len | J.part_stride | J.in_cs | J.dst_cs) & 3) == 0 &&
                     ((reinterpret_cast<uintptr_t>(J.src) | reinterpret_cast<uintptr_t>(J.dst)) & 15) == 0;
    if (vec && J.n_parts >= REDUCE_GROUP_MIN) {
        // many slabs (the weight-gradient partials of a one-chain plan: ~160 row chunks per trunk layer): the block's
        // four waves split the slabs (wave g sums p = g, g + 4, ... in order), then wave 0 adds the three other
        // waves' sums in order -- still a fixed order; one thread walking 160 slabs was latency-bound (17.7 us for
        // 60 MB at C = 1). Block-uniform branch (J and vec are per block), so the barrier is safe.
        __shared__ float4 gsum[3][64];
        if ((int)blockIdx.x * 256 >= J.len) return;   // whole block past this job (the grid fits the longest job)
        const int x = threadIdx.x & 63, g = threadIdx.x >> 6;
        const int eg = (blockIdx.x * 64 + x) * 4;
        bool ok = eg < J.len;
        if (J.samp && ok) ok = (J.samp[eg] | J.samp[eg + 1] | J.samp[eg + 2] | J.samp[eg + 3]) != 0;
        const float* sp = J.src + c * J.in_cs + (ok ? eg : 0);
        const int64_t st = J.part_stride;
        const int n = ok ? J.n_parts : 0;               // lanes past the end (or with no sampled output) load nothing
        float4 s = {0.f, 0.f, 0.f, 0.f};
        int p = g;
        for (; p + 28 < n; p += 32) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(sp + (p + 4 * u) * st);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s.x += v[u].x;
                s.y += v[u].y;
                s.z += v[u].z;
                s.w += v[u].w;
            }
        }
        for (; p < n; p += 4) {
            const float4 v = *reinterpret_cast<const float4*>(sp + p * st);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        if (g > 0) gsum[g - 1][x] = s;
        __syncthreads();
        if (g == 0 && ok) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                s.x += gsum[q][x].x;
                s.y += gsum[q][x].y;
                s.z += gsum[q][x].z;
                s.w += gsum[q][x].w;
            }
            *reinterpret_cast<float4*>(J.dst + c * J.dst_cs + eg) = s;
        }
        return;
    }
    const int e = (blockIdx.x * blockDim.x + threadIdx.x) * (vec ? 4 : 1);
    if (e >= J.len) return;
    if (J.samp && !(vec ? (J.samp[e] | J.samp[e + 1] | J.samp[e + 2] | J.samp[e + 3]) : J.samp[e])) return;
    const float* src = J.src + c * J.in_cs + e;
    const int n = J.n_parts;
    const int64_t st = J.part_stride;
    if (vec) {
        float4 s = {0.f, 0.f, 0.f, 0.f};
        int p = 0;
        for (; p + 8 <= n; p += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (p + u) * st);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s.x += v[u].x;
                s.y += v[u].y;
                s.z += v[u].z;
                s.w += v[u].w;
            }
        }
        for (; p < n; ++p) {
            const float4 v = *reinterpret_cast<const float4*>(src + p * st);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(J.dst + c * J.dst_cs + e) = s;
        return;
    }
    float s = 0.f;
    int p = 0;
    for (; p + 8 <= n; p += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(p + u) * st];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; p < n; ++p) s += src[p * st];
    J.dst[c * J.dst_cs + e] = s;
}

// Gradient gather + prior: grid (GATHER_SPLIT slices, C); each block writes its partial log-prior
// and the last kernel of the pair adds them in a fixed order.

constexpr int GATHER_SPLIT = GATHER_SPLIT_N;
static_assert(GATHER_SPLIT <= GATHER_SPLIT_MAX, "lp_part slots");

// 1024 threads, GATHER_U elements a thread per pass with every load of the pass issued before the first use: a
// one-element loop waited out the dependent smap -> gp gather latency per element (12.5 us for config 4's
// 172,401 parameters in 64 slices; one pass now)
constexpr int GATHER_THREADS = 1024, GATHER_U = 4;
template <bool LEAP>
__global__ __launch_bounds__(GATHER_THREADS) void k_gather_prior(const float* gp, int64_t gp_cs, const int32_t* smap,
                                                                 const float* theta, int K, const float* prior_mu,
                                                                 const float* prior_inv_var, float prior_scale,
                                                                 float* grad, double* lp_part, LeapArgs lf,
                                                                 FinalizeArgs fin) {
    __shared__ double sh[GATHER_THREADS / 64];
    const int c = blockIdx.y;
    const int per = (K + gridDim.x - 1) / gridDim.x;
    const int k0 = blockIdx.x * per, k1 = min(K, k0 + per);
    const float inv_scale = 1.f / prior_scale;
    const float* gpc = gp + c * gp_cs;
    double lp = 0.0;
    // leapfrog step: its operands (momentum, inverse mass, the scatter's offsets) are loaded with the gather's
    float e = 0.f;
    if (LEAP && lf.mode == 0) e = lf.eps[c];
    const bool scat = LEAP && !lf.last && lf.sc.packed != nullptr;
    for (int kb = k0 + threadIdx.x; kb < k1; kb += GATHER_U * GATHER_THREADS) {
        float thv[GATHER_U], muv[GATHER_U], ivv[GATHER_U], gpv[GATHER_U], pv[GATHER_U], imv[GATHER_U];
        ScatterIdx sx[GATHER_U];
#pragma unroll
        for (int u = 0; u < GATHER_U; ++u) {
            const int k = min(kb + u * GATHER_THREADS, k1 - 1);
            thv[u] = theta[(int64_t)c * K + k];
            muv[u] = prior_mu[k];
            ivv[u] = prior_inv_var[k];
            gpv[u] = gpc[smap[k]];
            if (LEAP) {
                pv[u] = lf.p[(int64_t)c * K + k];
                imv[u] = lf.inv_mass ? lf.inv_mass[k] : 1.f;
                if (scat) sx[u] = scatter_idx(lf.sc.smap_w, lf.sc.smap_wt, lf.sc.si, k);
            }
        }
#pragma unroll
        for (int u = 0; u < GATHER_U; ++u) {
            const int k = kb + u * GATHER_THREADS;
            if (k >= k1) break;
            const int64_t o = (int64_t)c * K + k;
            const float th = thv[u];
            const float d = th - muv[u];
            const float iv = ivv[u];
            lp += -0.5 * (double)d * (double)d * (double)iv;
            // one explicit fma after a rounded product: the same rounding in both instantiations whatever the
            // contraction pragma around them (the fused trajectory is bitwise the step-by-step path)
            const float g = __builtin_fmaf(-__fmul_rn(d, iv), inv_scale, gpv[u]);
            if (grad) grad[o] = g;
            if (LEAP && lf.mode != 0) {
                // the splitting integrator's kicks and drift (LeapArgs.mode), one fma each as torch.add(alpha=)
                float pn = __builtin_fmaf(lf.kick, g, pv[u]);
                if (lf.mode == 1) {
                    pn = __builtin_fmaf(lf.kick, g, pn);
                    const float tn = __builtin_fmaf(lf.drift, pn, th);
                    lf.th[o] = tn;
                    if (scat) scatter_store(lf.sc.packed, lf.sc.dp, lf.sc.si, c, sx[u], tn);
                }
                lf.p[o] = pn;
            } else if (LEAP) {
#pragma clang fp contract(off)
                float pn = pv[u] + e * g;
                if (lf.last) {
                    pn = pn - (0.5f * e) * g;
                } else {
                    const float step = lf.inv_mass ? (e * imv[u]) * pn : e * pn;
                    const float tn = th + step;
                    if (!(GATHER_ABL & 2)) lf.th[o] = tn;
                    if (scat && !GATHER_ABL) scatter_store(lf.sc.packed, lf.sc.dp, lf.sc.si, c, sx[u], tn);
                }
                if (!(GATHER_ABL & 2)) lf.p[o] = pn;
            }
        }
    }
    lp = block_sum(lp, sh);
    if (threadIdx.x == 0) lp_part[c * gridDim.x + blockIdx.x] = lp;
    if (fin.logp == nullptr) return;
    // log-prob finalisation by the chain's last block to finish (k_logp_finalize's fixed butterfly, so bitwise the
    // separate launch it replaces): release the partial, count it, and the block that completes the count
    // acquires every partial and resets the counter for the next evaluation (or graph replay)
    __shared__ int is_last;
    if (threadIdx.x == 0) {
        __threadfence();
        is_last = atomicAdd(fin.cnt + c, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!is_last || threadIdx.x >= 64) return;
    __threadfence();
    const int lane = threadIdx.x;
    // lane l adds partials l, l + 64, ... in order (one term each up to 64 slices: the round-4 order), then the butterfly
    double t = 0.0;
    for (int i = lane; i < (int)gridDim.x; i += 64)
        t += __hip_atomic_load(lp_part + c * gridDim.x + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) {
        fin.logp[c] = (float)((double)fin.lik[c] + (t + fin.prior_const) / (double)prior_scale);
        fin.cnt[c] = 0u;
    }
}

__global__ __launch_bounds__(256) void k_leap_open(const float* th_in, float* th_out, const float* p_in, float* p_out,
                                                   const float* g_in, const float* eps, const float* inv_mass, int K,
                                                   ScatterArgs sc) {
#pragma clang fp contract(off)
    const int c = blockIdx.y;
    const float e = eps[c], he = 0.5f * e;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
        const int64_t o = (int64_t)c * K + k;
        // every load before the first store (a load after a float store may alias it and waits for it)
        const float pi = p_in[o], gi = g_in[o], ti = th_in[o];
        const float im = inv_mass ? inv_mass[k] : 1.f;
        ScatterIdx sx{};
        if (sc.packed) sx = scatter_idx(sc.smap_w, sc.smap_wt, sc.si, k);
        const float pn = pi + he * gi;
        const float step = inv_mass ? (e * im) * pn : e * pn;
        p_out[o] = pn;
        const float tn = ti + step;
        th_out[o] = tn;
        if (sc.packed) scatter_store(sc.packed, sc.dp, sc.si, c, sx, tn);
    }
}

// =============================================================================================
// Metropolis step of one HMC iteration for every chain (hamiltorch sample loop body, SURVEY.md App. A.1;
// vihmc.samplers.HMCRunner.step): H0 = -lp0 + ke0, H1 = -lp1 + ke1 (the caller's kinetic energies, so the
// decisions keep the sampler's own summation), rho = min(H0 - H1, 0) (NaN -> 0), ok = both log-probs finite,
// accept = ok && rho >= log u, and the state selection -- after burn-in the accepted proposal overwrites the last
// returned state in place and (store) is written as the chain's next sample row (a failed chain's row goes to the
// spare last row, not counted); during burn-in the current state is the proposal, else (failed) the last returned
// state, else the burn-in fallback, which an accepted proposal replaces. A [C, K] launch and a [C] launch replace ~25 small
// elementwise launches.
// =============================================================================================
// the per-chain decision (every block of the chain recomputes it from the [C] inputs)
struct AcceptDecision {
    float rho;
    bool ok, acc;
};
__device__ __forceinline__ AcceptDecision accept_decision(const AcceptArgs& a, int c) {
#pragma clang fp contract(off)
    const float lp0 = a.lp0[c], lp1 = a.lp1[c];
    const float h0 = -lp0 + a.ke0[c], h1 = -lp1 + a.ke1[c];
    const float d = h0 - h1;
    AcceptDecision r;
    r.rho = d != d ? 0.f : fminf(d, 0.f);
    r.ok = isfinite(lp0) && isfinite(lp1);
    r.acc = r.ok && r.rho >= a.logu[c];
    return r;
}

// [C, K] part: grid (ceil(K / 1024), C), 4 elements per thread with every load issued before the first store (a
// one-element loop waited out one load per trip: 116 us at 16 chains); reads counts[c] before k_hmc_accept_chain
// advances it (stream order)
constexpr int ACC_U = 4;
__global__ __launch_bounds__(256) void k_hmc_accept(AcceptArgs a) {
    const int c = blockIdx.y;
    const int64_t o = (int64_t)c * a.K;
    __shared__ int flags[2];
    __shared__ int64_t row_s;
    if (threadIdx.x == 0) {
        const AcceptDecision r = accept_decision(a, c);
        flags[0] = r.acc ? 1 : 0;
        flags[1] = r.ok ? 0 : 1;
        // a full sample store (counts[c] reached the spare row s_cap - 1) writes the spare row and stops counting
        if (!a.burn && a.samples) row_s = (r.ok && a.counts[c] < a.s_cap - 1) ? a.counts[c] : a.s_cap - 1;
    }
    __syncthreads();
    const bool acc = flags[0] != 0, err = flags[1] != 0;
    const int k0 = blockIdx.x * (ACC_U * 256) + threadIdx.x;
    if (!a.burn) {
        float* srow = a.samples ? a.samples + ((int64_t)c * a.s_cap + row_s) * a.K : nullptr;
        float th[ACC_U], gn[ACC_U];
#pragma unroll
        for (int u = 0; u < ACC_U; ++u) {
            const int k = min(k0 + 256 * u, a.K - 1);
            th[u] = acc ? a.th1[o + k] : a.th_last[o + k];
            gn[u] = acc ? a.g1[o + k] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < ACC_U; ++u) {
            const int k = k0 + 256 * u;
            if (k >= a.K) break;
            if (acc) {
                a.th_last[o + k] = th[u];
                a.g_last[o + k] = gn[u];
            }
            if (srow) srow[k] = th[u];
        }
    } else {
        float tn[ACC_U], gn[ACC_U], tf[ACC_U], gf[ACC_U];
#pragma unroll
        for (int u = 0; u < ACC_U; ++u) {
            const int k = min(k0 + 256 * u, a.K - 1);
            tn[u] = a.th1[o + k];
            gn[u] = a.g1[o + k];
            tf[u] = err ? a.th_last[o + k] : a.th_bp[o + k];
            gf[u] = err ? a.g_last[o + k] : a.g_bp[o + k];
        }
#pragma unroll
        for (int u = 0; u < ACC_U; ++u) {
            const int k = k0 + 256 * u;
            if (k >= a.K) break;
            a.th_cur[o + k] = acc ? tn[u] : tf[u];
            a.g_cur[o + k] = acc ? gn[u] : gf[u];
            if (acc) {
                a.th_bp[o + k] = tn[u];
                a.g_bp[o + k] = gn[u];
            }
        }
    }
}

// [C] part, after the [C, K] part: log-probs, counts, accepted, trace, rho, err
__global__ __launch_bounds__(256) void k_hmc_accept_chain(AcceptArgs a, int C) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const AcceptDecision r = accept_decision(a, c);
    const float lp1 = a.lp1[c];
    a.rho[c] = r.ok ? r.rho : __builtin_nanf("");
    a.err[c] = r.ok ? 0 : 1;
    a.accepted[(int64_t)c * a.acc_ld + a.n] = r.acc ? 1 : 0;
    float lp_next;
    if (!a.burn) {
        if (r.acc) a.lp_last[c] = lp1;
        lp_next = r.acc ? lp1 : a.lp_last[c];
        if (a.samples) a.counts[c] += (r.ok && a.counts[c] < a.s_cap - 1) ? 1 : 0;
    } else {
        lp_next = r.acc ? lp1 : (r.ok ? a.lp_bp[c] : a.lp_last[c]);
        a.lp_cur[c] = lp_next;
        if (r.acc) a.lp_bp[c] = lp1;
    }
    a.trace[(int64_t)c * a.tr_ld + a.n] = lp_next;
}

// Kinetic energies 0.5 sum_k p[c][k] (m[k] p[c][k]) (m = the inverse mass, or 1) of C chains in ONE launch: grid
// (S slices, C), each block sums its contiguous slice in fp64 (4 loads per thread in flight), fixed-order block tree;
// the chain's last block to finish (arrival counter, reset by it) adds the S partials in order and writes the fp32
// energy. Replaces the sampler's 0.5 * (p * p).sum(1) -- a product, a memset, a reduction and a scale, four launches
// (~21 us at config 4's 172,401 parameters, profiles/r05lt_c1_trace.txt) -- twice per HMC iteration.
constexpr int KIN_THREADS = 1024, KIN_U = 4;
__global__ __launch_bounds__(KIN_THREADS) void k_kinetic(const float* p, const float* inv_mass, int K, float* ke,
                                                         double* part, uint32_t* cnt) {
    __shared__ double sh[KIN_THREADS / 64];
    __shared__ int is_last;
    const int c = blockIdx.y, S = gridDim.x;
    const int per = (K + S - 1) / S;
    const int k0 = blockIdx.x * per, k1 = min(K, k0 + per);
    const float* pc = p + (int64_t)c * K;
    double s = 0.0;
    for (int kb = k0 + threadIdx.x; kb < k1; kb += KIN_U * KIN_THREADS) {
        float v[KIN_U], m[KIN_U];
#pragma unroll
        for (int u = 0; u < KIN_U; ++u) {
            const int k = min(kb + u * KIN_THREADS, k1 - 1);
            v[u] = pc[k];
            m[u] = inv_mass ? inv_mass[k] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < KIN_U; ++u)
            if (kb + u * KIN_THREADS < k1) s += (double)(v[u] * (m[u] * v[u]));
    }
    s = block_sum(s, sh);
    if (threadIdx.x == 0) {
        part[(int64_t)c * S + blockIdx.x] = s;
        __threadfence();
        is_last = atomicAdd(cnt + c, 1u) == (uint32_t)S - 1;
    }
    __syncthreads();
    if (!is_last || threadIdx.x >= 64) return;
    __threadfence();
    const int lane = threadIdx.x;
    double t = 0.0;
    for (int i = lane; i < S; i += 64)
        t += __hip_atomic_load(part + (int64_t)c * S + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) {
        ke[c] = (float)(0.5 * t);
        cnt[c] = 0u;
    }
}

int kinetic_slices(int K) { return std::max(1, std::min(KINETIC_MAX_SLICES, (K + KIN_U * KIN_THREADS - 1) / (KIN_U * KIN_THREADS))); }

hipError_t launch_kinetic(const float* p, const float* inv_mass, int C, int K, float* ke, double* part, uint32_t* cnt,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_kinetic, dim3(kinetic_slices(K), C), dim3(KIN_THREADS), 0, s, p, inv_mass, K, ke, part, cnt);
    return hipGetLastError();
}

hipError_t launch_hmc_accept(const AcceptArgs& a, int C, hipStream_t s) {
    hipLaunchKernelGGL(k_hmc_accept, dim3((a.K + ACC_U * 256 - 1) / (ACC_U * 256), C), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hmc_accept_chain, dim3((C + 255) / 256), dim3(256), 0, s, a, C);
    return hipGetLastError();
}

// =============================================================================================
// BNN: one wave per chain. Lanes are data rows; the flat weights live in LDS (broadcast reads);
// parameter gradients are wave-reduced into LDS and gathered at the sampled indices.
// =============================================================================================
__device__ __forceinline__ float act_grad_z(int act, float z, float h) {
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    if (act == ACT_SINE) return cosf(z);
    return 1.f;
}

// LDS plan per block (floats): w[D] | gw[D] | h[(NL+1)*W][SLD] | z[NL*W][SLD] | d[W][SLD] | g[W][SLD]
// where [unit][SLD] columns hold one value per lane (row); SLD = 65 keeps the per-unit row sums
// (lanes reading different units at the same row) on distinct banks.
constexpr int MLP_SLD = 65;

// One log-posterior (+ gradient) evaluation of chain c by one wave. On entry w[] holds the chain's full weight
// vector (frozen values with its sampled entries written); theta_at(k) is its k-th sampled value (prior term).
// grad_out(k, value) receives the gradient at the sampled indices; returns logp (lane 0's value is the result).
// Loops over layer widths / staged rows, optionally with a compile-time bound (MAXW > 0: fully unrolled with a
// guard; the iteration order -- and so every rounding -- is that of the plain loop). Measured on the shipped BNN
// (widths 10): MAXW = 16 took 34 us per leapfrog step against 21-23 us for the plain loops (MAXW = 0, shipped).
#define VIHMC_MLP_FOR(v, n) \
    _Pragma("unroll") for (int v = 0; v < (MAXW > 0 ? MAXW : (n)); ++v) if (MAXW == 0 || v < (n))
// the row sums (run-time count: the data rows of one 64-row pass) unrolled by 4 so each group's LDS reads are issued
// together; the accumulation order, and so the rounding, is that of the plain loop
#define VIHMC_MLP_ROWS(v, n) \
    _Pragma("unroll 4") for (int v = 0; v < (MAXW > 0 ? 64 : (n)); ++v) if (MAXW == 0 || v < (n))

// Layer widths: MlpDyn reads them from the plan at run time; MlpFix<in, w1, ..., out> fixes them at compile time,
// so every width loop (and the layer loop) unrolls completely and the LDS reads of a layer are issued ahead of its
// FMA chains. Same loops, same order: the rounding is that of the run-time form.
struct MlpDyn {
    static constexpr int NL = 0;
    static constexpr int dim(int) { return 0; }
};
template <int... Ds>
struct MlpFix {
    static constexpr int NL = (int)sizeof...(Ds) - 1;
    static constexpr int dim(int i) {
        constexpr int d[] = {Ds...};
        return d[i];
    }
};
using MlpBnn = MlpFix<1, 10, 10, 1>;     // the reference's BNN (Neural_network/*: 1 -> 10 -> 10 -> 1, D = 141)

// the per-step read-only operands, from the plan (global) or from an LDS copy (k_mlp_traj); passed beside the
// kernel arguments rather than in a modified copy of them (a private MlpArgs went to scratch memory)
struct MlpRead {
    const float* x; const float* y; const int32_t* idx; const float* prior_mu; const float* prior_inv_var;
};

template <int MAXW, class SH = MlpDyn, class ThetaAt, class GradOut>
__device__ __forceinline__ double mlp_eval_core(const MlpArgs& a, MlpRead rd, int W, float* sm, int c,
                                                ThetaAt theta_at, GradOut grad_out, bool want_grad, float* out) {
    // no implicit contraction into fma: the two kernels that inline this body (k_mlp, k_mlp_traj) must round
    // identically (explicit fmaf calls stay fused)
#pragma clang fp contract(off)
    constexpr int SLD = MLP_SLD;
    constexpr bool FIX = SH::NL > 0;
    const int NL = FIX ? SH::NL : a.n_layers;
    const int in_dim = FIX ? SH::dim(0) : a.in_dim;
    const int out_dim = FIX ? SH::dim(FIX ? SH::NL : 0) : a.out_dim;
    float* w = sm;
    float* gw = w + a.D;
    float* hs = gw + a.D;
    float* zs = hs + (NL + 1) * W * SLD;
    float* ds = zs + NL * W * SLD;
    float* gs = ds + W * SLD;
    const int lane = threadIdx.x;
    for (int i = lane; i < a.D; i += 64) gw[i] = 0.f;
    __syncthreads();
    const float v = fmaxf(a.tau_out, 1e-6f);
    const float gscale = (a.loss == 0) ? -1.f / v : -a.tau_out;
    double ssq = 0.0;

    for (int r0 = 0; r0 < a.N; r0 += 64) {
        const int row = r0 + lane;
        const bool ok = row < a.N;
        const int rr = ok ? row : 0;
#pragma unroll
        for (int i = 0; i < in_dim; ++i) hs[i * SLD + lane] = rd.x[(int64_t)rr * in_dim + i];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const MlpLayer L = a.L[l];
            const int nin = FIX ? SH::dim(l) : L.n_in, nout = FIX ? SH::dim(l + 1) : L.n_out;
            const float* hin = hs + l * W * SLD;
            VIHMC_MLP_FOR(j, nout) {
                float s = 0.f;
                VIHMC_MLP_FOR(i, nin) s = fmaf(w[L.w_off + j * nin + i], hin[i * SLD + lane], s);
                if (L.b_off >= 0) s += w[L.b_off + j];
                zs[(l * W + j) * SLD + lane] = s;
                hs[((l + 1) * W + j) * SLD + lane] = act_apply(L.act, s);
            }
        }
        const float* hout = hs + NL * W * SLD;
#pragma unroll
        for (int o = 0; o < out_dim; ++o) {
            const float yv = rd.y[(int64_t)rr * out_dim + o];
            const float pred = hout[o * SLD + lane];
            const float rv = pred - yv;
            float g = 0.f;
            if (ok) {
                ssq += (double)rv * (double)rv;
                g = gscale * rv;
                if (out) out[((int64_t)c * a.N + row) * out_dim + o] = pred;
            }
            gs[o * SLD + lane] = g;
        }
        if (!want_grad) continue;
#pragma unroll
        for (int l = NL - 1; l >= 0; --l) {
            const MlpLayer L = a.L[l];
            const int nin = FIX ? SH::dim(l) : L.n_in, nout = FIX ? SH::dim(l + 1) : L.n_out;
            const float* hin = hs + l * W * SLD;
            VIHMC_MLP_FOR(j, nout) {
                const float z = zs[(l * W + j) * SLD + lane];
                const float h = hs[((l + 1) * W + j) * SLD + lane];
                ds[j * SLD + lane] = gs[j * SLD + lane] * act_grad_z(L.act, z, h);
            }
            __syncthreads();
            // dW[j][i] = sum_rows d[j] h[i], db[j] = sum_rows d[j]: every lane owns distinct entries and
            // sums the staged rows in a fixed order. Rows past N carry d = 0 and are skipped (fmaf(0, h, s) = s:
            // the same sums, 64 / N times fewer dependent steps -- 20 of 64 rows on the shipped BNN data).
            const int nw = nout * nin;
            const int ne = nw + (L.b_off >= 0 ? nout : 0);
            const int nrow = min(64, a.N - r0);
            for (int e = lane; e < ne; e += 64) {
                float s = 0.f;
                if (e < nw) {
                    const int j = e / nin, i = e - j * nin;
                    VIHMC_MLP_ROWS(m, nrow) s = fmaf(ds[j * SLD + m], hin[i * SLD + m], s);
                    gw[L.w_off + e] += s;
                } else {
                    const int j = e - nw;
                    VIHMC_MLP_ROWS(m, nrow) s += ds[j * SLD + m];
                    gw[L.b_off + j] += s;
                }
            }
            if (l > 0) {
                VIHMC_MLP_FOR(i, nin) {
                    float s = 0.f;
                    VIHMC_MLP_FOR(j, nout) s = fmaf(ds[j * SLD + lane], w[L.w_off + j * nin + i], s);
                    gs[i * SLD + lane] = s;
                }
            }
            __syncthreads();
        }
    }
    __syncthreads();
    ssq = wave_sum(ssq);
    double ll;
    if (a.loss == 0) ll = -0.5 * ((double)a.N * a.out_dim * log((double)v) + ssq / (double)v);
    else ll = -0.5 * (double)a.tau_out * ssq;
    const float inv_scale = 1.f / a.prior_scale;
    double lp = 0.0;
    for (int k = lane; k < a.K; k += 64) {
        const float th = theta_at(k);
        const float dd = th - rd.prior_mu[k];
        const float iv = rd.prior_inv_var[k];
        lp += -0.5 * (double)dd * (double)dd * (double)iv;
        if (want_grad) grad_out(k, gw[rd.idx[k]] - dd * iv * inv_scale);
    }
    lp = wave_sum(lp);
    return ll + (lp + a.prior_const) / (double)a.prior_scale;
}

template <int MAXW, class SH = MlpDyn>
__global__ __launch_bounds__(64) void k_mlp(MlpArgs a, int W) {
    extern __shared__ float sm[];
    float* w = sm;
    const int c = blockIdx.x, lane = threadIdx.x;
    for (int i = lane; i < a.D; i += 64) w[i] = a.frozen[i];
    __syncthreads();
    for (int k = lane; k < a.K; k += 64) w[a.idx[k]] = a.theta[(int64_t)c * a.K + k];
    __syncthreads();
    const float* th = a.theta + (int64_t)c * a.K;
    float* gr = a.grad ? a.grad + (int64_t)c * a.K : nullptr;
    const MlpRead rd{a.x, a.y, a.idx, a.prior_mu, a.prior_inv_var};
    const double lp = mlp_eval_core<MAXW, SH>(
        a, rd, W, sm, c, [&](int k) { return th[k]; }, [&](int k, float g) { gr[k] = g; }, gr != nullptr, a.out);
    if (lane == 0) a.logp[c] = (float)lp;
}

// A leapfrog trajectory per chain (hamiltorch leapfrog, Sampler.HMC, non-splitting integrator):
//   p += (eps/2) g(th0);  L x { th += eps p  [eps inv_mass p];  g = grad log p(th);  p += eps g };  p -= (eps/2) g
// every product and sum rounded separately (fp contract off: no fma), as the torch
// elementwise ops round them, so the result is bitwise the step-by-step path. theta / momentum / gradient of
// the chain live in LDS after the evaluation's workspace; one wave per chain, no host round trip per step.
template <int MAXW, class SH = MlpDyn>
__global__ __launch_bounds__(64) void k_mlp_traj(MlpArgs a, int W, MlpTrajArgs t) {
    // products and sums written here are rounded separately (the HIP __fmul_rn / __fadd_rn helpers are plain * and
    // + defined in a header, outside this pragma's reach: the compiler fused them into fma)
#pragma clang fp contract(off)
    extern __shared__ float sm[];
    const int c = blockIdx.x, lane = threadIdx.x, K = a.K;
    float* w = sm;
    float* th = sm + t.ws_floats;
    float* pm = th + K;
    float* gk = pm + K;
    // t.cache: the per-step read-only operands (data rows, sampled-index map, prior, mass) copied into LDS once per
    // trajectory, so a leapfrog step issues no global loads (each was an L2 round trip per step before)
    MlpRead rd{a.x, a.y, a.idx, a.prior_mu, a.prior_inv_var};
    const float* im = t.inv_mass;
    if (t.cache) {
        float* xs = gk + K;
        float* ys = xs + a.N * a.in_dim;
        float* pmu = ys + a.N * a.out_dim;
        float* piv = pmu + K;
        float* ims = piv + K;
        int32_t* ids = reinterpret_cast<int32_t*>(ims + K);
        for (int i = lane; i < a.N * a.in_dim; i += 64) xs[i] = a.x[i];
        for (int i = lane; i < a.N * a.out_dim; i += 64) ys[i] = a.y[i];
        for (int k = lane; k < K; k += 64) {
            pmu[k] = a.prior_mu[k];
            piv[k] = a.prior_inv_var[k];
            ids[k] = a.idx[k];
            if (im) ims[k] = im[k];
        }
        rd = MlpRead{xs, ys, ids, pmu, piv};
        if (im) im = ims;
    }
    for (int i = lane; i < a.D; i += 64) w[i] = a.frozen[i];
    const float e = t.eps[c], he = 0.5f * e;
    const int64_t off = (int64_t)c * K;
    for (int k = lane; k < K; k += 64) {
        th[k] = t.th_in[off + k];
        gk[k] = t.g_in[off + k];
        pm[k] = t.p_in[off + k] + he * gk[k];
    }
    double lp = 0.0;
    for (int s = 0; s < t.L; ++s) {
        for (int k = lane; k < K; k += 64) {
            const float step = im ? (e * im[k]) * pm[k] : e * pm[k];
            th[k] = th[k] + step;
        }
        __syncthreads();
        for (int k = lane; k < K; k += 64) w[rd.idx[k]] = th[k];
        __syncthreads();
        lp = mlp_eval_core<MAXW, SH>(
            a, rd, W, sm, c, [&](int k) { return th[k]; }, [&](int k, float g) { gk[k] = g; }, true, nullptr);
        for (int k = lane; k < K; k += 64) pm[k] = pm[k] + e * gk[k];
    }
    for (int k = lane; k < K; k += 64) {
        t.th_out[off + k] = th[k];
        t.g_out[off + k] = gk[k];
        t.p_out[off + k] = pm[k] - he * gk[k];
    }
    if (lane == 0) t.lp_out[c] = (float)lp;
}

// cfg.sample_data (Operator_network/VI_HMC/main_VI_HMC_burgers.py:131-134): the evaluation sees the trunk rows
// ind[0..P) of the full sensor grid -- trunk features [P_all][in_t] -> plan input [P][ld_in] (pad columns stay
// zero), targets y_all[n][ind[j]] -> y [N][P]. Pure copy (bit-exact); indices checked on the host.
__global__ __launch_bounds__(256) void k_gather_trunk(const float* __restrict__ feat_all, int in_t,
                                                     const float* __restrict__ y_all, int64_t P_all,
                                                     const int32_t* __restrict__ ind, int P, int N,
                                                     float* __restrict__ input, int ld_in, float* __restrict__ y) {
    const int64_t total = (int64_t)N * P, nin = (int64_t)P * in_t;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total + nin; i += (int64_t)gridDim.x * 256) {
        if (i < total) {
            const int64_t n = i / P, j = i - n * P;
            y[i] = y_all[n * P_all + ind[j]];
        } else {
            const int64_t k = i - total, j = k / in_t, f = k - j * in_t;
            input[j * ld_in + f] = feat_all[(int64_t)ind[j] * in_t + f];
        }
    }
}

// =============================================================================================
// launchers
// =============================================================================================
hipError_t launch_gather_trunk(const float* feat_all, int in_t, const float* y_all, int64_t P_all,
                               const int32_t* ind, int P, int N, float* input, int ld_in, float* y, hipStream_t s) {
    const int64_t work = (int64_t)N * P + (int64_t)P * in_t;
    hipLaunchKernelGGL(k_gather_trunk, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 2048)), dim3(256), 0, s,
                       feat_all, in_t, y_all, P_all, ind, P, N, input, ld_in, y);
    return hipGetLastError();
}

#define VIHMC_LAUNCH(kern, grid, block, shm, s, ...) \
    do { hipLaunchKernelGGL(kern, grid, block, shm, s, __VA_ARGS__); return hipGetLastError(); } while (0)

hipError_t launch_init_packed(float* packed, int64_t dp, int C, const float* frozen, const int32_t* map_w,
                              const int32_t* map_wt, int64_t D, hipStream_t s) {
    dim3 g((unsigned)std::min<int64_t>((D + 255) / 256, 1024), C), blk(256);
    VIHMC_LAUNCH(k_init_packed, g, blk, 0, s, packed, dp, frozen, map_w, map_wt, D);
}

hipError_t launch_scatter(float* packed, int64_t dp, int C, const float* theta, int K, const int32_t* smap_w,
                          const int32_t* smap_wt, hipStream_t s, const ScatterImg* si) {
    dim3 g((unsigned)((K + 255) / 256), C), blk(256);
    VIHMC_LAUNCH(k_scatter, g, blk, 0, s, packed, dp, theta, K, smap_w, smap_wt, si ? *si : ScatterImg{});
}

hipError_t launch_reduce(const ReduceJob* jobs_dev, int n_jobs, int max_len, int C, hipStream_t s,
                         const StatsJob* stats, const ChainBits* only) {
    // grid sized for the scalar path; vectorised jobs leave 3/4 of the x-blocks idle (cheap exits)
    dim3 g((max_len + 255) / 256, n_jobs + (stats ? 1 : 0), C), blk(256);
    VIHMC_LAUNCH(k_reduce, g, blk, 0, s, jobs_dev, n_jobs, stats ? *stats : StatsJob{}, only ? 1 : 0,
                 only ? *only : ChainBits{});
}

hipError_t launch_contract_stats(const StatsJob& J, int C, hipStream_t s) {
    VIHMC_LAUNCH(k_contract_stats, dim3(C), dim3(256), 0, s, J);
}

// sum of y^2 and sum of y in fixed order: YSQ_PARTS contiguous chunks (thread-strided fp64 sums + block tree), then
// one block over the partials: out[0] = sum y^2, out[1] = sum y (part holds YSQ_PARTS pairs)
__global__ __launch_bounds__(256) void k_ysq_part(const float* y, int64_t n, double* part) {
    __shared__ double sh[8];
    const int64_t chunk = (n + YSQ_PARTS - 1) / YSQ_PARTS;
    const int64_t e0 = (int64_t)blockIdx.x * chunk, e1 = e0 + chunk < n ? e0 + chunk : n;
    double v = 0.0, w = 0.0;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
        const double x = (double)y[e];
        v += x * x;
        w += x;
    }
    v = block_sum(v, sh);
    __syncthreads();
    w = block_sum(w, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = v;
        part[YSQ_PARTS + blockIdx.x] = w;
    }
}
__global__ __launch_bounds__(256) void k_ysq_final(const double* part, double* out) {
    __shared__ double sh[8];
    double v = 0.0, w = 0.0;
    for (int i = threadIdx.x; i < YSQ_PARTS; i += 256) {
        v += part[i];
        w += part[YSQ_PARTS + i];
    }
    v = block_sum(v, sh);
    __syncthreads();
    w = block_sum(w, sh);
    if (threadIdx.x == 0) {
        out[0] = v;
        out[1] = w;
    }
}
hipError_t launch_ysq(const float* y, int64_t n, double* part, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_ysq_part, dim3(YSQ_PARTS), dim3(256), 0, s, y, n, part);
    VIHMC_LAUNCH(k_ysq_final, dim3(1), dim3(256), 0, s, part, out);
}

hipError_t launch_gather_prior(const float* gp, int64_t gp_cs, const int32_t* smap, const float* theta, int K,
                               const float* prior_mu, const float* prior_inv_var, double prior_const,
                               float prior_scale, const float* lik, int C, float* logp, float* grad,
                               double* lp_part, uint32_t* fin_cnt, hipStream_t s, const LeapArgs* leap) {
    // logp == null: no log-prob wanted (inner leapfrog steps); else the last block of each chain finalises it
    const FinalizeArgs fin{logp, lik, prior_const, fin_cnt};
    if (logp && !fin_cnt) return hipErrorInvalidValue;
    // slices per chain: at least one element per thread (K / 1024) and ~256 blocks over all chains where each keeps
    // >= 256 elements, at most GATHER_SPLIT (C = 16, K = 17,240: 17 slices of ~1,014 elements instead of 64 of 270 --
    // 3/4 of the threads idle; config 4 at one chain, K = 172,401: 256 slices, every CU, instead of 64)
    const int split = std::min(GATHER_SPLIT, std::max({1, (K + GATHER_THREADS - 1) / GATHER_THREADS,
                                                       std::min((256 + C - 1) / C, (K + 255) / 256)}));
    if (leap)
        hipLaunchKernelGGL(k_gather_prior<true>, dim3(split, C), dim3(GATHER_THREADS), 0, s, gp, gp_cs, smap,
                           theta, K, prior_mu, prior_inv_var, prior_scale, grad, lp_part, *leap, fin);
    else
        hipLaunchKernelGGL(k_gather_prior<false>, dim3(split, C), dim3(GATHER_THREADS), 0, s, gp, gp_cs, smap,
                           theta, K, prior_mu, prior_inv_var, prior_scale, grad, lp_part, LeapArgs{}, fin);
    return hipGetLastError();
}

hipError_t launch_leap_open(const float* th_in, float* th_out, const float* p_in, float* p_out, const float* g_in,
                            const float* eps, const float* inv_mass, int K, int C, hipStream_t s, const ScatterArgs* sc) {
    // one element per thread: with the scatter inside, a 4-iteration loop per thread left its scattered stores'
    // latency serial (18 us at C = 16)
    VIHMC_LAUNCH(k_leap_open, dim3((K + 255) / 256, C), dim3(256), 0, s, th_in, th_out, p_in, p_out, g_in, eps,
                 inv_mass, K, sc ? *sc : ScatterArgs{});
}

// the plan's layers are exactly MlpBnn's widths (then the compile-time form runs)
static bool mlp_is_bnn(const MlpArgs& a, int maxw) {
    if (a.n_layers != MlpBnn::NL || maxw != 10 || a.in_dim != MlpBnn::dim(0) || a.out_dim != MlpBnn::dim(MlpBnn::NL))
        return false;
    for (int l = 0; l < MlpBnn::NL; ++l)
        if (a.L[l].n_in != MlpBnn::dim(l) || a.L[l].n_out != MlpBnn::dim(l + 1)) return false;
    return true;
}

size_t mlp_lds_bytes(int D, int n_layers, int maxw) {
    return sizeof(float) * (2 * (size_t)D + (size_t)(2 * n_layers + 3) * maxw * MLP_SLD);
}

hipError_t launch_mlp(const MlpArgs& a, int C, int maxw, hipStream_t s) {
    const size_t shm = mlp_lds_bytes(a.D, a.n_layers, maxw);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    if (mlp_is_bnn(a, maxw)) VIHMC_LAUNCH((k_mlp<0, MlpBnn>), dim3(C), dim3(64), shm, s, a, maxw);
    VIHMC_LAUNCH(k_mlp<0>, dim3(C), dim3(64), shm, s, a, maxw);
}

hipError_t launch_mlp_traj(const MlpArgs& a, const MlpTrajArgs& t, int C, int maxw, hipStream_t s) {
    const size_t ws = mlp_lds_bytes(a.D, a.n_layers, maxw);
    size_t shm = ws + 3 * sizeof(float) * (size_t)a.K;
    if (shm > 160 * 1024 || t.L < 1) return hipErrorInvalidValue;
    MlpTrajArgs tt = t;
    tt.ws_floats = (int32_t)(ws / sizeof(float));
    const size_t cache = sizeof(float) * ((size_t)a.N * (a.in_dim + a.out_dim) + 4 * (size_t)a.K);
    tt.cache = shm + cache <= 160 * 1024 ? 1 : 0;
    if (tt.cache) shm += cache;
    if (mlp_is_bnn(a, maxw)) VIHMC_LAUNCH((k_mlp_traj<0, MlpBnn>), dim3(C), dim3(64), shm, s, a, maxw, tt);
    VIHMC_LAUNCH(k_mlp_traj<0>, dim3(C), dim3(64), shm, s, a, maxw, tt);
}

// Shader-clock stamp (measurement, vihmc_clock_stamp): CLOCK_STAMP_WG one-wave workgroups record their XCD id, their
// HW_ID (CU / shader array / shader engine of the wave), s_memtime (shader-clock ticks) and s_memrealtime (100 MHz); two
// stamps around a timed region give each CU's average shader clock over it, from the SAME CU's two readings (the
// s_memtime counters of different CUs are not one clock domain: pairing medians across CUs read 2.58 GHz on one XCD
// in round 4) -- MI355X_MICROARCH.md "DVFS give-back" item 6. Vector stores only.
__global__ __launch_bounds__(64) void k_clock_stamp(unsigned long long* out) {
    unsigned x, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    const int i = threadIdx.x;
    if (i < 4) out[blockIdx.x * 4 + i] = i == 0 ? (unsigned long long)x : i == 1 ? (unsigned long long)hw : i == 2 ? t : r;
}

hipError_t launch_clock_stamp(unsigned long long* out, hipStream_t s) {
    VIHMC_LAUNCH(k_clock_stamp, dim3(CLOCK_STAMP_WG), dim3(64), 0, s, out);
}

}  // namespace vihmc
