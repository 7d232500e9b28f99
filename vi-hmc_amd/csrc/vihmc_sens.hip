// Sensitivity scores of the VI parameters: S_i = sigma_i^2 * mean over outputs of (d f / d theta_i)^2.
//
// Replaces eval_std_dydw / eval_jac of Operator_network/VI/sensitivity.py:62-126 (torch.func.jacrev of
// Functional_DeepONet.functional_model over all D parameters, squared, averaged over the p sampled trunk
// points of every validation function, batch_size 1) and of Neural_network/VI/sensitivity.py:71-126
// (jacrev of the BNN over the validation inputs, mean over (0, 1)).
//
// DeepONet, f[n][p] = Z_b[n] . Z_t[p] + b. For one output pair (n, p):
//   d f / d theta_branch = backprop through the branch at row n seeded with Z_t[p],
//   d f / d theta_trunk  = backprop through the trunk  at row p seeded with Z_b[n],   d f / d b = 1.
// A weight's gradient is delta_l[i] h_{l-1}[j]; the pairs of one row ("group": branch row n with its p
// points, trunk point p with the functions that sampled it) share h, so their squared gradients sum to
// q_l[i] h_{l-1}[j]^2 with q_l = sum over the group's seeds of delta_l^2 (and q_l[i] for the bias).
//   k_sens_seeds  one wave per task (<= 16 seeds of one group): the seeds' deltas go down the net in LDS
//                 (16 x 16 x 4 f32 MFMA, exact fp32; the W_l image is shared by the 8 waves of the
//                 workgroup) and q_l of every layer is written per task.
//   k_sens_outer  per (net, layer, task chunk): part[i][j] = sum_tasks q_l[i] h_{l-1}[group][j]^2 and the
//                 bias part sum_tasks q_l[i] (LDS-staged, 8 x 8 register tile per thread).
//   k_sens_reduce fixed-order sum of the chunk partials into the packed layout (deterministic).
//   k_sens_flat   flat (named_parameters) order, * sigma^2 / pairs.
// Sums of squares have no cancellation: fp32 accumulation throughout.
#include "vihmc_internal.h"

namespace vihmc {

namespace {
typedef float f32x4_s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sens_act_grad(int act, float h) {
    // derivative from the activation's output (DeepONet plans: tanh / relu hidden layers)
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}
}  // namespace

size_t sens_seeds_lds_bytes(int ldd, int ldw) {
    return sizeof(float) * ((size_t)128 * ldw + (size_t)SENS_WAVES * SENS_SEEDS * ldd);
}

__global__ __launch_bounds__(SENS_WAVES * 64, 1) void k_sens_seeds(const SensArgs* __restrict__ Ap) {
    const SensArgs& A = *Ap;      // in global memory: runtime net / layer indexing stays a load, not scratch
    extern __shared__ __attribute__((aligned(16))) float ssm[];
    int b = blockIdx.x;
    const int net = b < A.net[0].n_wg ? 0 : 1;
    if (net) b -= A.net[0].n_wg;
    const SensNet& N = A.net[net];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int ldd = A.ldd, ldw = A.ldw;
    float* wimg = ssm;                                              // [<= 128][ldw]
    float* dimg = ssm + 128 * ldw + wave * SENS_SEEDS * ldd;        // this wave's deltas [16][ldd]
    const int t = b * SENS_WAVES + wave;
    const bool active = t < N.n_tasks;
    int grp = 0, sb = 0, sc = 0;
    if (active) {
        grp = N.tasks[3 * t];
        sb = N.tasks[3 * t + 1];
        sc = N.tasks[3 * t + 2];
    }
    const int nl = N.nl;
    const int wlast = N.L[nl - 1].n_out;
    // the seeds are the deltas of the (linear) last layer; unused rows / columns are zero and stay zero
    for (int e = lane; e < SENS_SEEDS * ldd; e += 64) {
        const int i = e / ldd, k = e - i * ldd;
        float v = 0.f;
        if (active && i < sc && k < wlast) v = N.seeds[(int64_t)N.seed_idx[sb + i] * N.ld_seed + k];
        dimg[e] = v;
    }
    __syncthreads();
    float* Qt = N.Q + (int64_t)(active ? t : 0) * nl * SENS_QLD;
    if (active) {
        for (int k = lane; k < SENS_QLD; k += 64) {
            float s = 0.f;
            if (k < wlast)
                for (int i = 0; i < SENS_SEEDS; ++i) {
                    const float v = dimg[i * ldd + k];
                    s = fmaf(v, v, s);
                }
            Qt[(nl - 1) * SENS_QLD + k] = s;
        }
    }
    for (int l = nl - 1; l >= 1; --l) {
        const SensLayer& L = N.L[l];
        // all 8 column tiles always (zero-padded W image): a runtime tile count made the compiler spill
        const int kext = (L.n_out + 15) & ~15, jext = 128;
        __syncthreads();                      // every wave is done with the previous W image
        for (int e = tid; e < kext * jext; e += SENS_WAVES * 64) {
            const int k = e / jext, j = e - k * jext;
            wimg[k * ldw + j] = (k < L.n_out && j < L.n_in) ? L.W[(int64_t)k * L.ldi + j] : 0.f;
        }
        __syncthreads();
        if (!active) continue;
        // delta_{l-1} = (delta_l W_l) * act'(h_{l-1}): A = deltas [seed][k], B = W_l [k][j]; float4 A reads
        // with MFMA step s using k = kb + 4 lg + s (the same permutation on both operands)
        f32x4_s acc[8];
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) acc[jt] = f32x4_s{0.f, 0.f, 0.f, 0.f};
        for (int kb = 0; kb < kext; kb += 16) {
            const f32x4_s a = *reinterpret_cast<const f32x4_s*>(dimg + lr * ldd + kb + 4 * lg);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float* wrow = wimg + (kb + 4 * lg + s) * ldw + lr;
#pragma unroll
                for (int jt = 0; jt < 8; ++jt)
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], wrow[16 * jt], acc[jt], 0, 0, 0);
            }
        }
        const float* hrow = L.Hprev + (int64_t)grp * L.ldh;
        float* Ql = Qt + (l - 1) * SENS_QLD;
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
            const int j = 16 * jt + lr;
            const float ag = j < L.n_in ? sens_act_grad(L.act_prev, hrow[j]) : 0.f;
            float sq = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[jt][r] *= ag;
                sq = fmaf(acc[jt][r], acc[jt][r], sq);
            }
            sq += __shfl_xor(sq, 16, 64);
            sq += __shfl_xor(sq, 32, 64);
            if (lg == 0) Ql[j] = sq;
        }
        // every A read of this wave fed an MFMA whose result is consumed above: safe to overwrite
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dimg[(4 * lg + r) * ldd + 16 * jt + lr] = acc[jt][r];
        }
    }
}

// part[l][ch][i][j] = sum_{tasks in ch} q_l[i] h_{l-1}[grp][j]^2, part[..][128*128 + i] = sum q_l[i]
__global__ __launch_bounds__(256) void k_sens_outer(const SensArgs* __restrict__ Ap) {
    const SensArgs& A = *Ap;
    __shared__ float qs[SENS_TCH][129];
    __shared__ float hs[SENS_TCH][129];
    __shared__ int gs[SENS_TCH];
    int b = blockIdx.x;
    const int nb0 = A.net[0].nl * A.net[0].chunks;
    const int net = b < nb0 ? 0 : 1;
    if (net) b -= nb0;
    const SensNet& N = A.net[net];
    const int l = b / N.chunks, ch = b - l * N.chunks;
    const SensLayer& L = N.L[l];
    const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
    const int t0 = ch * N.tasks_per_chunk, t1 = min(t0 + N.tasks_per_chunk, N.n_tasks);
    float acc[8][8];
    float bsum[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        bsum[a] = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[a][c] = 0.f;
    }
    for (int r0 = t0; r0 < t1; r0 += SENS_TCH) {
        __syncthreads();
        if (tid < SENS_TCH) gs[tid] = r0 + tid < t1 ? N.tasks[3 * (r0 + tid)] : -1;
        __syncthreads();
        for (int e = tid; e < SENS_TCH * 128; e += 256) {
            const int t = e >> 7, c = e & 127;
            const int g = gs[t];
            float qv = 0.f, hv = 0.f;
            if (g >= 0) {
                if (c < L.n_out) qv = N.Q[((int64_t)(r0 + t) * N.nl + l) * SENS_QLD + c];
                if (c < L.n_in) {
                    const float h = L.Hprev[(int64_t)g * L.ldh + c];
                    hv = h * h;
                }
            }
            qs[t][c] = qv;
            hs[t][c] = hv;
        }
        __syncthreads();
        const int nt = min(SENS_TCH, t1 - r0);
        for (int t = 0; t < nt; ++t) {
            float qv[8], hv[8];
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                qv[a] = qs[t][ti + 16 * a];
                hv[a] = hs[t][tj + 16 * a];
            }
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                bsum[a] += qv[a];
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[a][c] = fmaf(qv[a], hv[c], acc[a][c]);
            }
        }
    }
    float* out = N.part + ((int64_t)l * N.chunks + ch) * SENS_PART;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        const int i = ti + 16 * a;
        if (i >= L.n_out) continue;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int j = tj + 16 * c;
            if (j < L.n_in) out[i * 128 + j] = acc[a][c];
        }
        if (tj == 0) out[128 * 128 + i] = bsum[a];
    }
}

__global__ __launch_bounds__(256) void k_sens_reduce(const SensArgs* __restrict__ Ap) {
    const SensArgs& A = *Ap;
    const int net = blockIdx.z, l = blockIdx.y;
    const SensNet& N = A.net[net];
    if (l >= N.nl) return;
    const SensLayer& L = N.L[l];
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= SENS_PART) return;
    int64_t dst;
    if (e < 128 * 128) {
        const int i = e >> 7, j = e & 127;
        if (i >= L.n_out || j >= L.n_in) return;
        dst = L.wp + (int64_t)i * L.ldi + j;
    } else {
        const int i = e - 128 * 128;
        if (i >= L.n_out) return;
        dst = L.bias + i;
    }
    const float* p = N.part + (int64_t)l * N.chunks * SENS_PART + e;
    float s = 0.f;
    for (int c = 0; c < N.chunks; ++c) s += p[(int64_t)c * SENS_PART];
    A.S[dst] = s;
}

__global__ __launch_bounds__(256) void k_sens_flat(const float* S, const int32_t* fmap, int64_t D, const float* sigma,
                                                   float inv_count, float* out) {
    const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (d >= D) return;
    const int32_t m = fmap[d];
    const float v = m == 0 ? 1.f : S[m] * inv_count;    // packed slot 0 = output bias b: d f / d b = 1
    const float sg = sigma ? sigma[d] : 1.f;
    out[d] = v * (sg * sg);
}

hipError_t launch_sens(const SensArgs& a, const SensArgs* dev_a, const int32_t* fmap, int64_t D, const float* sigma,
                       float* out, hipStream_t s) {
    const int blocks = a.net[0].n_wg + a.net[1].n_wg;
    hipLaunchKernelGGL(k_sens_seeds, dim3(blocks), dim3(SENS_WAVES * 64), sens_seeds_lds_bytes(a.ldd, a.ldw), s, dev_a);
    if (hipError_t e = hipGetLastError()) return e;
    const int ob = a.net[0].nl * a.net[0].chunks + a.net[1].nl * a.net[1].chunks;
    hipLaunchKernelGGL(k_sens_outer, dim3(ob), dim3(256), 0, s, dev_a);
    if (hipError_t e = hipGetLastError()) return e;
    const int nlm = a.net[0].nl > a.net[1].nl ? a.net[0].nl : a.net[1].nl;
    hipLaunchKernelGGL(k_sens_reduce, dim3((SENS_PART + 255) / 256, nlm, 2), dim3(256), 0, s, dev_a);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL(k_sens_flat, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, s, a.S, fmap, D, sigma,
                       1.f / a.count, out);
    return hipGetLastError();
}

// =============================================================================================
// BNN: one 64-lane block per 64 data rows (lanes = rows), the k_mlp layout (vihmc_kernels.hip). For every
// output o the block backpropagates the unit seed e_o and adds sum_rows (delta_j h_i)^2 (weights) and
// sum_rows delta_j^2 (biases) to its partial; k_sens_mlp_reduce sums the partials in block order.
// =============================================================================================
namespace {
constexpr int SMLP_SLD = 65;
__device__ __forceinline__ float smlp_act(int act, float z) {
    if (act == ACT_TANH) return tanhf(z);
    if (act == ACT_RELU) return fmaxf(z, 0.f);
    if (act == ACT_SINE) return sinf(z);
    return z;
}
__device__ __forceinline__ float smlp_act_grad(int act, float z, float h) {
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    if (act == ACT_SINE) return cosf(z);
    return 1.f;
}
size_t smlp_lds_bytes(int D, int n_layers, int maxw) {
    return sizeof(float) * (2 * (size_t)D + (size_t)(2 * n_layers + 3) * maxw * SMLP_SLD);
}
}  // namespace

__global__ __launch_bounds__(64) void k_sens_mlp(MlpArgs a, float* slab, int W) {
    constexpr int SLD = SMLP_SLD;
    extern __shared__ float sm[];
    const int NL = a.n_layers;
    float* w = sm;
    float* gq = w + a.D;
    float* hs = gq + a.D;
    float* zs = hs + (NL + 1) * W * SLD;
    float* ds = zs + NL * W * SLD;
    float* gs = ds + W * SLD;
    const int lane = threadIdx.x;
    for (int i = lane; i < a.D; i += 64) {
        w[i] = a.frozen[i];
        gq[i] = 0.f;
    }
    __syncthreads();
    for (int k = lane; k < a.K; k += 64) w[a.idx[k]] = a.theta[k];      // chain 0
    __syncthreads();
    const int row = blockIdx.x * 64 + lane;
    const bool ok = row < a.N;
    const int rr = ok ? row : 0;
    for (int i = 0; i < a.in_dim; ++i) hs[i * SLD + lane] = a.x[(int64_t)rr * a.in_dim + i];
    for (int l = 0; l < NL; ++l) {
        const MlpLayer L = a.L[l];
        const float* hin = hs + l * W * SLD;
        for (int j = 0; j < L.n_out; ++j) {
            float s = 0.f;
            for (int i = 0; i < L.n_in; ++i) s = fmaf(w[L.w_off + j * L.n_in + i], hin[i * SLD + lane], s);
            if (L.b_off >= 0) s += w[L.b_off + j];
            zs[(l * W + j) * SLD + lane] = s;
            hs[((l + 1) * W + j) * SLD + lane] = smlp_act(L.act, s);
        }
    }
    for (int o = 0; o < a.out_dim; ++o) {
        for (int j = 0; j < a.out_dim; ++j) gs[j * SLD + lane] = (ok && j == o) ? 1.f : 0.f;
        for (int l = NL - 1; l >= 0; --l) {
            const MlpLayer L = a.L[l];
            const float* hin = hs + l * W * SLD;
            for (int j = 0; j < L.n_out; ++j) {
                const float z = zs[(l * W + j) * SLD + lane];
                const float h = hs[((l + 1) * W + j) * SLD + lane];
                ds[j * SLD + lane] = gs[j * SLD + lane] * smlp_act_grad(L.act, z, h);
            }
            __syncthreads();
            const int nw = L.n_out * L.n_in;
            const int ne = nw + (L.b_off >= 0 ? L.n_out : 0);
            for (int e = lane; e < ne; e += 64) {
                float s = 0.f;
                if (e < nw) {
                    const int j = e / L.n_in, i = e - j * L.n_in;
                    for (int m = 0; m < 64; ++m) {
                        const float g = ds[j * SLD + m] * hin[i * SLD + m];
                        s = fmaf(g, g, s);
                    }
                    gq[L.w_off + e] += s;
                } else {
                    const int j = e - nw;
                    for (int m = 0; m < 64; ++m) s = fmaf(ds[j * SLD + m], ds[j * SLD + m], s);
                    gq[L.b_off + j] += s;
                }
            }
            if (l > 0) {
                for (int i = 0; i < L.n_in; ++i) {
                    float s = 0.f;
                    for (int j = 0; j < L.n_out; ++j) s = fmaf(ds[j * SLD + lane], w[L.w_off + j * L.n_in + i], s);
                    gs[i * SLD + lane] = s;
                }
            }
            __syncthreads();
        }
    }
    for (int i = lane; i < a.D; i += 64) slab[(int64_t)blockIdx.x * a.D + i] = gq[i];
}

__global__ __launch_bounds__(256) void k_sens_mlp_reduce(const float* slab, int nblk, int D, const float* sigma,
                                                         float inv_count, float* out) {
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d >= D) return;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += slab[(int64_t)b * D + d];
    const float sg = sigma ? sigma[d] : 1.f;
    out[d] = s * inv_count * (sg * sg);
}

hipError_t launch_sens_mlp(const MlpArgs& a, float* slab, const float* sigma, float* out, int maxw, hipStream_t s) {
    const size_t shm = smlp_lds_bytes(a.D, a.n_layers, maxw);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    const int nblk = (a.N + 63) / 64;
    hipLaunchKernelGGL(k_sens_mlp, dim3(nblk), dim3(64), shm, s, a, slab, maxw);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL(k_sens_mlp_reduce, dim3((a.D + 255) / 256), dim3(256), 0, s, slab, nblk, a.D, sigma,
                       1.f / ((float)a.N * (float)a.out_dim), out);
    return hipGetLastError();
}

}  // namespace vihmc
