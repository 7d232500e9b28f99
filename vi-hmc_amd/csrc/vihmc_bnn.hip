// Register-resident BNN evaluation and leapfrog trajectory for the reference's three-layer MLP
// (Neural_network/*: 1 -> 10 -> 10 -> 1, D = 141; Functional_Net.functional_model,
// Neural_network/VI_HMC/my_make_func.py:52-73, its log-posterior main_VI_HMC.py:96-151 and the hamiltorch
// leapfrog that drives it).
//
// One wave per chain. Lanes are data rows (64 per pass); every per-row quantity (z, h, delta of each layer) stays in
// registers. The weights live once in LDS in a canonical packed layout [W1 | b1 | W2 | b2 | W3 | b3] (4-float
// aligned blocks) and are read into registers by wave-uniform b128 broadcasts. The weight gradient is the only
// reduction over rows; it is two fp32 MFMA tiles (v_mfma_f32_16x16x4_f32, exact fp32 products, k = 4 rows a step):
//   T1 = D1^T H1m   D1 = [delta2]            H1m = [h1 | 1]        -> dW2, db2
//   T2 = D2^T H2m   D2 = [delta1 | delta3]   H2m = [x | 1 | h2]    -> dW1, db1, dW3, db3 (cross blocks unused)
// with the operand rows staged through LDS as [row][16] images, which a 16x16x4 step reads lane-linearly
// (lane l: image[64 s + l]). The trajectory kernel keeps theta / momentum / gradient of the chain in registers
// (k = lane + 64 j) and runs hamiltorch's leapfrog with every product and sum rounded separately, exactly as the
// torch elementwise updates round them; the evaluation core is shared with the evaluation kernel, so a fused
// trajectory is bitwise the step-by-step path. The log-likelihood and prior sums (fp64) are formed only where a
// log-prob is returned (the last step of a trajectory).
#include "vihmc_internal.h"

namespace vihmc {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IN = BNN_IN, H1 = BNN_H1, H2 = BNN_H2, OUT = BNN_OUT;
// canonical weight layout (floats), blocks 4-aligned
constexpr int r4c(int n) { return (n + 3) & ~3; }
constexpr int CW1 = 0, CB1 = CW1 + r4c(H1 * IN), CW2 = CB1 + r4c(H1), CB2 = CW2 + r4c(H2 * H1), CW3 = CB2 + r4c(H2),
              CB3 = CW3 + r4c(OUT * H2), CWN = CB3 + r4c(OUT);
static_assert(CWN == BNN_CANON, "canonical layout size");
static_assert(H2 <= 16 && H1 + 1 <= 16 && H1 + OUT <= 16 && IN + 1 + H2 <= 16, "two 16x16 gradient tiles");
constexpr int IMG = 64 * 16;                           // one operand image: 64 rows x 16 columns
constexpr int GLD = 17;                                // gradient tile row pitch in LDS
// LDS (floats): canonical weights | 4 operand images | 2 gradient tiles
constexpr int L_W = 0, L_IMG = r4c(CWN), L_G = L_IMG + 4 * IMG;
constexpr int L_TOTAL = L_G + 2 * 16 * GLD;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// hidden layers tanh, output identity (the reference BNN, Neural_network/VI_HMC/main_VI_HMC.py:297-334); the
// activation and its derivative as the generic kernel computes them (tanhf; 1 - h^2 from the output)
constexpr int ACT1 = ACT_TANH, ACT2 = ACT_TANH, ACT3 = ACT_ID;
template <int ACT>
__device__ __forceinline__ float act_f(float z) {
    return ACT == ACT_TANH ? tanhf(z) : z;
}
template <int ACT>
__device__ __forceinline__ float act_g(float h) {
    return ACT == ACT_TANH ? 1.f - h * h : 1.f;
}
template <typename T>
__device__ __forceinline__ T wsum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// the canonical weights from LDS into registers (wave-uniform values), 4 at a time
struct Wts {
    float w[CWN];
    __device__ __forceinline__ void load(const float* lw) {
#pragma unroll
        for (int i = 0; i < CWN; i += 4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(lw + i);
            w[i] = v[0];
            w[i + 1] = v[1];
            w[i + 2] = v[2];
            w[i + 3] = v[3];
        }
    }
};

// One evaluation of the chain whose weights are in LDS (sm + L_W). Returns the per-lane share of nothing: the
// gradient tiles are left in LDS (sm + L_G) for the caller's gather; *ssq_out gets this lane's sum of squared
// residuals (fp64). Rows = lanes; N rows in passes of 64 (x / y from global; the trajectory kernel passes its
// register copies through xr / yr when N <= 64).
template <bool GRAD>
__device__ __forceinline__ double bnn_core(const MlpArgs& a, float* sm, int c, const float (&xr)[IN],
                                           const float (&yr)[OUT], bool rows_in_regs, float* out) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x;
    Wts W;
    W.load(sm + L_W);
    const float v = fmaxf(a.tau_out, 1e-6f);
    const float gscale = (a.loss == 0) ? -1.f / v : -a.tau_out;
    double ssq = 0.0;
    f32x4 t1 = {0.f, 0.f, 0.f, 0.f}, t2 = {0.f, 0.f, 0.f, 0.f};
    float* img = sm + L_IMG;
    for (int r0 = 0; r0 < a.N; r0 += 64) {
        const int row = r0 + lane;
        const bool ok = row < a.N;
        const int rr = ok ? row : 0;
        float x[IN], y[OUT];
#pragma unroll
        for (int i = 0; i < IN; ++i) x[i] = rows_in_regs ? xr[i] : a.x[(int64_t)rr * IN + i];
#pragma unroll
        for (int o = 0; o < OUT; ++o) y[o] = rows_in_regs ? yr[o] : a.y[(int64_t)rr * OUT + o];
        // ---- forward (the generic kernel's order: sum of products from i = 0, then + bias) ----
        float h1[H1], h2[H2], h3[OUT];
#pragma unroll
        for (int j = 0; j < H1; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < IN; ++i) s = fmaf(W.w[CW1 + j * IN + i], x[i], s);
            s += W.w[CB1 + j];
            h1[j] = act_f<ACT1>(s);
        }
#pragma unroll
        for (int j = 0; j < H2; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < H1; ++i) s = fmaf(W.w[CW2 + j * H1 + i], h1[i], s);
            s += W.w[CB2 + j];
            h2[j] = act_f<ACT2>(s);
        }
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < H2; ++i) s = fmaf(W.w[CW3 + o * H2 + i], h2[i], s);
            s += W.w[CB3 + o];
            h3[o] = act_f<ACT3>(s);
        }
        float g[OUT];
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
            const float rv = h3[o] - y[o];
            g[o] = 0.f;
            if (ok) {
                ssq += (double)rv * (double)rv;
                g[o] = gscale * rv;
                if (out) out[((int64_t)c * a.N + row) * OUT + o] = h3[o];
            }
        }
        if (!GRAD) continue;
        // ---- backward: deltas per row ----
        float d3[OUT], d2[H2], d1[H1];
#pragma unroll
        for (int o = 0; o < OUT; ++o) d3[o] = g[o] * act_g<ACT3>(h3[o]);
#pragma unroll
        for (int j = 0; j < H2; ++j) {
            float s = 0.f;
#pragma unroll
            for (int o = 0; o < OUT; ++o) s = fmaf(d3[o], W.w[CW3 + o * H2 + j], s);
            d2[j] = s * act_g<ACT2>(h2[j]);
        }
#pragma unroll
        for (int i = 0; i < H1; ++i) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < H2; ++j) s = fmaf(d2[j], W.w[CW2 + j * H1 + i], s);
            d1[i] = s * act_g<ACT1>(h1[i]);
        }
        // ---- operand images [row][16]: D1 = [d2], H1m = [h1 | 1], D2 = [d1 | d3], H2m = [x | 1 | h2] ----
        float e1[16], f1[16], e2[16], f2[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            e1[q] = q < H2 ? d2[q] : 0.f;
            f1[q] = q < H1 ? h1[q] : (q == H1 ? 1.f : 0.f);
            e2[q] = q < H1 ? d1[q] : (q < H1 + OUT ? d3[q - H1] : 0.f);
            f2[q] = q < IN ? x[q] : (q == IN ? 1.f : (q < IN + 1 + H2 ? h2[q - IN - 1] : 0.f));
        }
        __syncthreads();                       // the previous pass's MFMA reads are done
#pragma unroll
        for (int q = 0; q < 16; q += 4) {
            *reinterpret_cast<f32x4*>(img + 0 * IMG + lane * 16 + q) = f32x4{e1[q], e1[q + 1], e1[q + 2], e1[q + 3]};
            *reinterpret_cast<f32x4*>(img + 1 * IMG + lane * 16 + q) = f32x4{f1[q], f1[q + 1], f1[q + 2], f1[q + 3]};
            *reinterpret_cast<f32x4*>(img + 2 * IMG + lane * 16 + q) = f32x4{e2[q], e2[q + 1], e2[q + 2], e2[q + 3]};
            *reinterpret_cast<f32x4*>(img + 3 * IMG + lane * 16 + q) = f32x4{f2[q], f2[q + 1], f2[q + 2], f2[q + 3]};
        }
        __syncthreads();
        // ---- weight-gradient tiles: k = 4 rows a step, lane-linear operand reads ----
        const int nk = (min(64, a.N - r0) + 3) >> 2;
        for (int s = 0; s < nk; ++s) {
            const int o = 64 * s + lane;
            t1 = mfma4(img[0 * IMG + o], img[1 * IMG + o], t1);
            t2 = mfma4(img[2 * IMG + o], img[3 * IMG + o], t2);
        }
    }
    if (GRAD) {
        // tile element [4 (l >> 4) + r][l & 15] of each accumulator -> LDS [m][GLD]
        float* gt = sm + L_G;
        const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            gt[(4 * lg + r) * GLD + lr] = t1[r];
            gt[16 * GLD + (4 * lg + r) * GLD + lr] = t2[r];
        }
        __syncthreads();
    }
    return ssq;
}

// the log-posterior from this lane's squared-residual sum and prior partial (both fp64; wave-summed here)
__device__ __forceinline__ double bnn_logp(const MlpArgs& a, double ssq, double lp_prior) {
    ssq = wsum(ssq);
    lp_prior = wsum(lp_prior);
    const double v = (double)fmaxf(a.tau_out, 1e-6f);
    const double ll = a.loss == 0 ? -0.5 * ((double)a.N * OUT * log(v) + ssq / v) : -0.5 * (double)a.tau_out * ssq;
    return ll + (lp_prior + a.prior_const) / (double)a.prior_scale;
}

// the canonical weights of chain c: frozen values, then the sampled ones
__device__ __forceinline__ void bnn_init_weights(const MlpArgs& a, float* sm) {
    for (int f = threadIdx.x; f < a.D; f += 64) sm[L_W + a.canon[f]] = a.frozen[f];
}
}  // namespace

__global__ __launch_bounds__(64) void k_mlp_bnn(MlpArgs a) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int c = blockIdx.x, lane = threadIdx.x, K = a.K;
    bnn_init_weights(a, sm);
    __syncthreads();
    const float* th = a.theta + (int64_t)c * K;
    for (int k = lane; k < K; k += 64) sm[L_W + a.cpos[k]] = th[k];
    __syncthreads();
    const float xr[IN] = {}, yr[OUT] = {};
    const bool grad = a.grad != nullptr;
    const double ssq = grad ? bnn_core<true>(a, sm, c, xr, yr, false, a.out) : bnn_core<false>(a, sm, c, xr, yr, false, a.out);
    const float inv_scale = 1.f / a.prior_scale;
    double lp = 0.0;
    for (int k = lane; k < K; k += 64) {
        const float t = th[k];
        const float dd = t - a.prior_mu[k];
        const float iv = a.prior_inv_var[k];
        lp += -0.5 * (double)dd * (double)dd * (double)iv;
        if (grad) a.grad[(int64_t)c * K + k] = sm[L_G + a.goff[k]] - dd * iv * inv_scale;
    }
    const double logp = bnn_logp(a, ssq, lp);
    if (lane == 0) a.logp[c] = (float)logp;
}

// hamiltorch leapfrog (Sampler.HMC, non-splitting integrator):
//   p += (eps/2) g(th0);  L x { th += eps p  [eps inv_mass p];  g = grad log p(th);  p += eps g };  p -= (eps/2) g
// theta, momentum and gradient of the chain in registers (k = lane + 64 j, j < BNN_KS)
__global__ __launch_bounds__(64) void k_mlp_traj_bnn(MlpArgs a, MlpTrajArgs t) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int c = blockIdx.x, lane = threadIdx.x, K = a.K;
    bnn_init_weights(a, sm);
    const int64_t off = (int64_t)c * K;
    const float e = t.eps[c], he = 0.5f * e;
    float th[BNN_KS], pm[BNN_KS], gk[BNN_KS], mu[BNN_KS], iv[BNN_KS], im[BNN_KS];
    int cp[BNN_KS], go[BNN_KS];
    bool on[BNN_KS];
#pragma unroll
    for (int j = 0; j < BNN_KS; ++j) {
        const int k = lane + 64 * j;
        on[j] = k < K;
        const int kk = on[j] ? k : 0;
        th[j] = t.th_in[off + kk];
        gk[j] = t.g_in[off + kk];
        pm[j] = t.p_in[off + kk] + he * gk[j];
        mu[j] = a.prior_mu[kk];
        iv[j] = a.prior_inv_var[kk];
        im[j] = t.inv_mass ? t.inv_mass[kk] : 1.f;
        cp[j] = a.cpos[kk];
        go[j] = a.goff[kk];
    }
    // data rows in registers when one pass covers them
    const bool rows_in_regs = a.N <= 64;
    float xr[IN], yr[OUT];
    {
        const int rr = lane < a.N ? lane : 0;
#pragma unroll
        for (int i = 0; i < IN; ++i) xr[i] = a.x[(int64_t)rr * IN + i];
#pragma unroll
        for (int o = 0; o < OUT; ++o) yr[o] = a.y[(int64_t)rr * OUT + o];
    }
    const float inv_scale = 1.f / a.prior_scale;
    double ssq = 0.0;
    for (int s = 0; s < t.L; ++s) {
#pragma unroll
        for (int j = 0; j < BNN_KS; ++j) {
            const float step = t.inv_mass ? (e * im[j]) * pm[j] : e * pm[j];
            th[j] = th[j] + step;
        }
        __syncthreads();                       // the previous evaluation's weight reads are done
#pragma unroll
        for (int j = 0; j < BNN_KS; ++j)
            if (on[j]) sm[L_W + cp[j]] = th[j];
        __syncthreads();
        ssq = bnn_core<true>(a, sm, c, xr, yr, rows_in_regs, nullptr);
#pragma unroll
        for (int j = 0; j < BNN_KS; ++j) {
            const float dd = th[j] - mu[j];
            gk[j] = sm[L_G + go[j]] - dd * iv[j] * inv_scale;
            pm[j] = pm[j] + e * gk[j];
        }
    }
    double lp = 0.0;
#pragma unroll
    for (int j = 0; j < BNN_KS; ++j) {
        if (!on[j]) continue;
        const int k = lane + 64 * j;
        const float dd = th[j] - mu[j];
        lp += -0.5 * (double)dd * (double)dd * (double)iv[j];
        t.th_out[off + k] = th[j];
        t.g_out[off + k] = gk[j];
        t.p_out[off + k] = pm[j] - he * gk[j];
    }
    const double logp = bnn_logp(a, ssq, lp);
    if (lane == 0) t.lp_out[c] = (float)logp;
}

// the plan's MLP is the reference BNN (shape, tanh / tanh / identity, a bias on every layer) with at most
// BNN_KS * 64 sampled indices
bool mlp_bnn_fast_ok(const MlpArgs& a) {
    const int dims[4] = {IN, H1, H2, OUT};
    if (a.n_layers != 3 || a.in_dim != IN || a.out_dim != OUT || a.K > 64 * BNN_KS || !a.canon) return false;
    const int acts[3] = {ACT1, ACT2, ACT3};
    for (int l = 0; l < 3; ++l)
        if (a.L[l].n_in != dims[l] || a.L[l].n_out != dims[l + 1] || a.L[l].b_off < 0 || a.L[l].act != acts[l])
            return false;
    return true;
}

// canonical position of every flat parameter (w_off / b_off blocks of the layer table) and the gradient-tile
// position of its derivative; -1 where the shape is not the fast kernel's
void mlp_bnn_maps(const MlpArgs& a, std::vector<int32_t>& canon, std::vector<int32_t>& gpos) {
    canon.assign(a.D, -1);
    gpos.assign(a.D, -1);
    const int cw[3] = {CW1, CW2, CW3}, cb[3] = {CB1, CB2, CB3};
    for (int l = 0; l < 3; ++l) {
        const MlpLayer& L = a.L[l];
        for (int j = 0; j < L.n_out; ++j) {
            for (int i = 0; i < L.n_in; ++i) {
                const int f = L.w_off + j * L.n_in + i;
                canon[f] = cw[l] + j * L.n_in + i;
                // T1 (layer 2): [j][i]; T2: layer 1 [j][i], layer 3 [H1 + j][IN + 1 + i]
                gpos[f] = l == 1 ? j * GLD + i : 16 * GLD + (l == 0 ? j * GLD + i : (H1 + j) * GLD + IN + 1 + i);
            }
            const int f = L.b_off + j;
            canon[f] = cb[l] + j;
            gpos[f] = l == 1 ? j * GLD + H1 : 16 * GLD + (l == 0 ? j * GLD + IN : (H1 + j) * GLD + IN);
        }
    }
}

size_t mlp_bnn_lds_bytes() { return sizeof(float) * (size_t)L_TOTAL; }

hipError_t launch_mlp_bnn(const MlpArgs& a, int C, hipStream_t s) {
    hipLaunchKernelGGL(k_mlp_bnn, dim3(C), dim3(64), mlp_bnn_lds_bytes(), s, a);
    return hipGetLastError();
}

hipError_t launch_mlp_traj_bnn(const MlpArgs& a, const MlpTrajArgs& t, int C, hipStream_t s) {
    if (t.L < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mlp_traj_bnn, dim3(C), dim3(64), mlp_bnn_lds_bytes(), s, a, t);
    return hipGetLastError();
}

}  // namespace vihmc
