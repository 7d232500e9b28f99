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
// Row-dot GEMM (forward layers, backward input gradients). One wave per block, 16*MS rows x NT*16
// output columns per wave, operands streamed from L1/L2 (weights are <= 64 KB per chain-layer).
// =============================================================================================
template <int NT, int MS, int MODE>
__global__ __launch_bounds__(64) void k_rowdot(RowdotArgs args) {
    int b = blockIdx.x;
    const int first = args.C * args.p[0].tiles;
    const bool second = b >= first;
    const RowdotProb P = second ? args.p[1] : args.p[0];
    if (second) b -= first;
    const int c = b / P.tiles;
    const int tile = b - c * P.tiles;
    const int lane = threadIdx.x, lr = lane & 15, lg = lane >> 4;
    const float* A = P.A + c * P.a_cs;
    const float* B = P.B + c * P.b_cs;
    const int m0 = tile * 16 * MS;

    const float* ar[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) ar[s] = A + (int64_t)min(m0 + 16 * s + lr, P.M - 1) * P.lda;
    const float* br[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) br[t] = B + (int64_t)min(16 * t + lr, P.Nn - 1) * P.ldb;

    f32x4 acc[MS][NT];
#pragma unroll
    for (int s = 0; s < MS; ++s)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int kfull = P.K & ~15;
    for (int kb = 0; kb < kfull; kb += 16) {
        float4 a[MS], w[NT];
#pragma unroll
        for (int s = 0; s < MS; ++s) a[s] = *reinterpret_cast<const float4*>(ar[s] + kb + 4 * lg);
#pragma unroll
        for (int t = 0; t < NT; ++t) w[t] = *reinterpret_cast<const float4*>(br[t] + kb + 4 * lg);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int s = 0; s < MS; ++s) {
                acc[s][t] = mfma(a[s].x, w[t].x, acc[s][t]);
                acc[s][t] = mfma(a[s].y, w[t].y, acc[s][t]);
                acc[s][t] = mfma(a[s].z, w[t].z, acc[s][t]);
                acc[s][t] = mfma(a[s].w, w[t].w, acc[s][t]);
            }
    }
    // tail: K rounded up to 4; the padding columns of every operand buffer are zero
    const int kend = (P.K + 3) & ~3;
    for (int kb = kfull; kb < kend; kb += 4) {
        float a[MS], w[NT];
#pragma unroll
        for (int s = 0; s < MS; ++s) a[s] = ar[s][kb + lg];
#pragma unroll
        for (int t = 0; t < NT; ++t) w[t] = br[t][kb + lg];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int s = 0; s < MS; ++s) acc[s][t] = mfma(a[s], w[t], acc[s][t]);
    }

    float* O = P.O + c * P.o_cs;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int n = 16 * t + lr;
        if (n >= P.ldo) continue;
        const bool live = n < P.Nn;
        float bv = 0.f;
        if (MODE == MODE_FWD && live && P.bias) bv = P.bias[c * P.bias_cs + n];
#pragma unroll
        for (int s = 0; s < MS; ++s)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 16 * s + 4 * lg + r;
                if (m >= P.M) continue;
                float o = 0.f;
                if (live) {
                    const float v = acc[s][t][r];
                    if (MODE == MODE_FWD) {
                        o = act_apply(P.act, v + bv);
                    } else {
                        const float h = P.H[c * P.h_cs + (int64_t)m * P.ldh + n];
                        o = v * act_grad_from_out(P.act, h);
                    }
                }
                O[(int64_t)m * P.ldo + n] = o;
            }
    }
}

// =============================================================================================
// Column-sum GEMM (weight + bias gradients): one wave per (chain, row chunk, pair of 16-row
// output sub-tiles); partial slabs are reduced in fixed order afterwards.
// =============================================================================================
template <int JT>
__global__ __launch_bounds__(64) void k_colsum(ColsumArgs args) {
    int b = blockIdx.x;
    const int per0 = args.C * args.p[0].n_chunks * args.p[0].n_pairs;
    const bool second = b >= per0;
    const ColsumProb P = second ? args.p[1] : args.p[0];
    if (second) b -= per0;
    const int per_chain = P.n_chunks * P.n_pairs;
    const int c = b / per_chain;
    b -= c * per_chain;
    const int chunk = b / P.n_pairs;
    const int pair = b - chunk * P.n_pairs;
    const int lane = threadIdx.x, lr = lane & 15, lg = lane >> 4;
    const float* D = P.D + c * P.d_cs;
    const float* H = P.H + c * P.h_cs;
    const int r0 = chunk * P.rows_per_chunk;
    const int r1 = min(r0 + P.rows_per_chunk, P.M);

    int ncol[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) ncol[s] = min(32 * pair + 16 * s + lr, P.n_out - 1);
    int jcol[JT];
#pragma unroll
    for (int t = 0; t < JT; ++t) jcol[t] = min(16 * t + lr, P.n_in - 1);

    f32x4 acc[2][JT];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < JT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dsum[2] = {0.f, 0.f};

    for (int m = r0; m < r1; m += 4) {
        const int mm = m + lg;
        const bool mok = mm < r1;
        const int mr = mok ? mm : r0;
        const float* drow = D + (int64_t)mr * P.ldd;
        const float* hrow = H + (int64_t)mr * P.ldh;
        float a[2], h[JT];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const float v = drow[ncol[s]];
            a[s] = mok ? v : 0.f;
        }
#pragma unroll
        for (int t = 0; t < JT; ++t) h[t] = hrow[jcol[t]];
#pragma unroll
        for (int t = 0; t < JT; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) acc[s][t] = mfma(a[s], h[t], acc[s][t]);
        dsum[0] += a[0];
        dsum[1] += a[1];
    }

    float* part = P.part + c * P.part_cs + (int64_t)chunk * P.part_stride;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < JT; ++t) {
            const int j = 16 * t + lr;
            if (j >= P.ldh) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 32 * pair + 16 * s + 4 * lg + r;
                if (n < P.n_out) part[(int64_t)n * P.ldh + j] = (j < P.n_in) ? acc[s][t][r] : 0.f;
            }
        }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        float v = dsum[s];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int n = 32 * pair + 16 * s + lr;
        if (lg == 0 && n < P.n_out) part[(int64_t)P.n_out * P.ldh + n] = v;
    }
}

// =============================================================================================
// Fused contraction + Gaussian likelihood (+ its backward). See ContractProb.
// =============================================================================================
template <int WMAX, bool GRAD>
__global__ __launch_bounds__(64) void k_contract(ContractProb P) {
    constexpr int NB = WMAX / 16;
    int b = blockIdx.x;
    const int per_chain = P.o_tiles * P.q_chunks;
    const int c = b / per_chain;
    b -= c * per_chain;
    const int qc = b / P.o_tiles;
    const int ot = b - qc * P.o_tiles;
    const int lane = threadIdx.x, lr = lane & 15, lg = lane >> 4;
    const float* Own = P.Own + c * P.own_cs;
    const float* Q = P.Q + c * P.q_cs;
    const float b0 = P.b0[c * P.b0_cs];
    const int o0 = ot * 32;
    const int W = P.W;
    const int nkb = W >> 4;
    const int ntail = ((((W + 3) & ~3)) - (nkb << 4)) >> 2;
    const int JT = (W + 15) >> 4;

    // owner rows stay in registers for the whole q sweep (B operand of S = Q . Own^T)
    float4 ob[2][NB];
    float otl[2][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const float* orow = Own + (int64_t)min(o0 + 16 * s + lr, P.Mo - 1) * P.ldown;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
            ob[s][bb] = (bb < nkb) ? *reinterpret_cast<const float4*>(orow + 16 * bb + 4 * lg)
                                   : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ts = 0; ts < 3; ++ts) otl[s][ts] = (ts < ntail) ? orow[16 * nkb + 4 * ts + lg] : 0.f;
    }

    f32x4 dacc[2][NB];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < NB; ++t) dacc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int q_lo = qc * P.q_per_chunk;
    const int q_hi = min(q_lo + P.q_per_chunk, P.Mq);
    double ssq = 0.0, gsum = 0.0;
    float* sout = P.out + c * P.out_cs;

    for (int q = q_lo; q < q_hi; q += 16) {
        f32x4 sacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const float* qrow = Q + (int64_t)min(q + lr, P.Mq - 1) * P.ldq;
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
            if (bb < nkb) {
                const float4 qa = *reinterpret_cast<const float4*>(qrow + 16 * bb + 4 * lg);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    sacc[s] = mfma(qa.x, ob[s][bb].x, sacc[s]);
                    sacc[s] = mfma(qa.y, ob[s][bb].y, sacc[s]);
                    sacc[s] = mfma(qa.z, ob[s][bb].z, sacc[s]);
                    sacc[s] = mfma(qa.w, ob[s][bb].w, sacc[s]);
                }
            }
        }
#pragma unroll
        for (int ts = 0; ts < 3; ++ts) {
            if (ts < ntail) {
                const float qa = qrow[16 * nkb + 4 * ts + lg];
#pragma unroll
                for (int s = 0; s < 2; ++s) sacc[s] = mfma(qa, otl[s][ts], sacc[s]);
            }
        }
        // likelihood epilogue on the 2 S tiles held by this wave
        float g[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qq = q + 4 * lg + r;
                const int oo = o0 + 16 * s + lr;
                const bool ok = (qq < q_hi) && (oo < P.Mo);
                const float yv = P.Y[(int64_t)min(qq, P.Mq - 1) * P.ldy + min(oo, P.Mo - 1)];
                const float sv = sacc[s][r] + b0;
                if (!GRAD && P.write_s && ok) sout[(int64_t)qq * P.ldout + oo] = sv;
                const float rv = sv - yv;
                g[s][r] = ok ? P.gscale * rv : 0.f;
                if (ok) {
                    ssq += (double)rv * (double)rv;
                    gsum += (double)g[s][r];
                }
            }
        if (GRAD) {
            // dOwn[o][j] += sum_q G[q][o] Q[q][j]: G's C-layout register rr is the A operand of
            // MFMA step rr (k' = lane group <-> q = q + 4*lg + rr); the B operand is Q[q][j].
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const float* qr = Q + (int64_t)min(q + 4 * lg + rr, P.Mq - 1) * P.ldq;
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    if (t < JT) {
                        const float bq = qr[min(16 * t + lr, W - 1)];
#pragma unroll
                        for (int s = 0; s < 2; ++s) dacc[s][t] = mfma(g[s][rr], bq, dacc[s][t]);
                    }
                }
            }
        }
    }

    if (GRAD) {
        float* out = P.out + c * P.out_cs + (int64_t)qc * P.out_chunk_stride;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                const int j = 16 * t + lr;
                if (t >= JT || j >= P.ldout) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int oo = o0 + 16 * s + 4 * lg + r;
                    if (oo < P.Mo) out[(int64_t)oo * P.ldout + j] = (j < W) ? dacc[s][t][r] : 0.f;
                }
            }
    }
    if (P.with_stats) {
        ssq = wave_sum(ssq);
        gsum = wave_sum(gsum);
        if (lane == 0) {
            double* st = P.stats + c * P.stats_cs + 2 * (int64_t)(qc * P.o_tiles + ot);
            st[0] = ssq;
            st[1] = gsum;
        }
    }
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

__global__ void k_scatter(float* packed, int64_t dp, const float* theta, int K, const int32_t* smap_w,
                          const int32_t* smap_wt) {
    const int c = blockIdx.y;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
        const float v = theta[(int64_t)c * K + k];
        packed[c * dp + smap_w[k]] = v;
        const int32_t t = smap_wt[k];
        if (t >= 0) packed[c * dp + t] = v;
    }
}

__global__ void k_reduce(const ReduceJob* jobs) {
    const ReduceJob J = jobs[blockIdx.y];
    const int c = blockIdx.z;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= J.len) return;
    const float* src = J.src + c * J.in_cs + e;
    float s = 0.f;
    for (int p = 0; p < J.n_parts; ++p) s += src[p * J.part_stride];
    J.dst[c * J.dst_cs + e] = s;
}

__device__ double block_sum_256(double v, double* sh) {
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

__global__ __launch_bounds__(256) void k_contract_stats(const double* stats, int64_t stats_cs, int n_waves,
                                                        float* lik, float* gp, int64_t gp_cs, double count,
                                                        int loss, float tau_out) {
    __shared__ double sh[8];
    const int c = blockIdx.x;
    const double* st = stats + c * stats_cs;
    double ssq = 0.0, gs = 0.0;
    for (int i = threadIdx.x; i < n_waves; i += blockDim.x) {
        ssq += st[2 * i];
        gs += st[2 * i + 1];
    }
    ssq = block_sum_256(ssq, sh);
    gs = block_sum_256(gs, sh);
    if (threadIdx.x == 0) {
        double ll;
        if (loss == 0) {
            const double v = fmax((double)tau_out, 1e-6);
            ll = -0.5 * (count * log(v) + ssq / v);
        } else {
            ll = -0.5 * (double)tau_out * ssq;
        }
        lik[c] = (float)ll;
        gp[c * gp_cs] = (float)gs;   // d ll / d b0 (packed slot 0)
    }
}

__global__ __launch_bounds__(256) void k_gather_prior(const float* gp, int64_t gp_cs, const int32_t* smap,
                                                      const float* theta, int K, const float* prior_mu,
                                                      const float* prior_inv_var, double prior_const,
                                                      float prior_scale, const float* lik, float* logp,
                                                      float* grad) {
    __shared__ double sh[8];
    const int c = blockIdx.x;
    const float inv_scale = 1.f / prior_scale;
    double lp = 0.0;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const float th = theta[(int64_t)c * K + k];
        const float d = th - prior_mu[k];
        const float iv = prior_inv_var[k];
        lp += -0.5 * (double)d * (double)d * (double)iv;
        if (grad) grad[(int64_t)c * K + k] = gp[c * gp_cs + smap[k]] - d * iv * inv_scale;
    }
    lp = block_sum_256(lp, sh);
    if (threadIdx.x == 0) logp[c] = (float)((double)lik[c] + (lp + prior_const) / (double)prior_scale);
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

__global__ __launch_bounds__(64) void k_mlp(MlpArgs a, int W) {
    constexpr int SLD = MLP_SLD;
    extern __shared__ float sm[];
    const int NL = a.n_layers;
    float* w = sm;
    float* gw = w + a.D;
    float* hs = gw + a.D;
    float* zs = hs + (NL + 1) * W * SLD;
    float* ds = zs + NL * W * SLD;
    float* gs = ds + W * SLD;
    const int c = blockIdx.x, lane = threadIdx.x;
    for (int i = lane; i < a.D; i += 64) {
        w[i] = a.frozen[i];
        gw[i] = 0.f;
    }
    __syncthreads();
    for (int k = lane; k < a.K; k += 64) w[a.idx[k]] = a.theta[(int64_t)c * a.K + k];
    __syncthreads();
    const bool want_grad = a.grad != nullptr;
    const float v = fmaxf(a.tau_out, 1e-6f);
    const float gscale = (a.loss == 0) ? -1.f / v : -a.tau_out;
    double ssq = 0.0;

    for (int r0 = 0; r0 < a.N; r0 += 64) {
        const int row = r0 + lane;
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
                hs[((l + 1) * W + j) * SLD + lane] = act_apply(L.act, s);
            }
        }
        const float* hout = hs + NL * W * SLD;
        for (int o = 0; o < a.out_dim; ++o) {
            const float yv = a.y[(int64_t)rr * a.out_dim + o];
            const float pred = hout[o * SLD + lane];
            const float rv = pred - yv;
            float g = 0.f;
            if (ok) {
                ssq += (double)rv * (double)rv;
                g = gscale * rv;
                if (a.out) a.out[((int64_t)c * a.N + row) * a.out_dim + o] = pred;
            }
            gs[o * SLD + lane] = g;
        }
        if (!want_grad) continue;
        for (int l = NL - 1; l >= 0; --l) {
            const MlpLayer L = a.L[l];
            const float* hin = hs + l * W * SLD;
            for (int j = 0; j < L.n_out; ++j) {
                const float z = zs[(l * W + j) * SLD + lane];
                const float h = hs[((l + 1) * W + j) * SLD + lane];
                ds[j * SLD + lane] = gs[j * SLD + lane] * act_grad_z(L.act, z, h);
            }
            __syncthreads();
            // dW[j][i] = sum_rows d[j] h[i], db[j] = sum_rows d[j]: every lane owns distinct entries and
            // sums the 64 staged rows in a fixed order (masked rows carry d = 0).
            const int nw = L.n_out * L.n_in;
            const int ne = nw + (L.b_off >= 0 ? L.n_out : 0);
            for (int e = lane; e < ne; e += 64) {
                float s = 0.f;
                if (e < nw) {
                    const int j = e / L.n_in, i = e - j * L.n_in;
                    for (int m = 0; m < 64; ++m) s = fmaf(ds[j * SLD + m], hin[i * SLD + m], s);
                    gw[L.w_off + e] += s;
                } else {
                    const int j = e - nw;
                    for (int m = 0; m < 64; ++m) s += ds[j * SLD + m];
                    gw[L.b_off + j] += s;
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
    __syncthreads();
    ssq = wave_sum(ssq);
    double ll;
    if (a.loss == 0) ll = -0.5 * ((double)a.N * a.out_dim * log((double)v) + ssq / (double)v);
    else ll = -0.5 * (double)a.tau_out * ssq;
    const float inv_scale = 1.f / a.prior_scale;
    double lp = 0.0;
    for (int k = lane; k < a.K; k += 64) {
        const float th = a.theta[(int64_t)c * a.K + k];
        const float dd = th - a.prior_mu[k];
        const float iv = a.prior_inv_var[k];
        lp += -0.5 * (double)dd * (double)dd * (double)iv;
        if (want_grad) a.grad[(int64_t)c * a.K + k] = gw[a.idx[k]] - dd * iv * inv_scale;
    }
    lp = wave_sum(lp);
    if (lane == 0) a.logp[c] = (float)(ll + (lp + a.prior_const) / (double)a.prior_scale);
}

// =============================================================================================
// launchers
// =============================================================================================
#define VIHMC_LAUNCH(kern, grid, block, shm, s, ...) \
    do { hipLaunchKernelGGL(kern, grid, block, shm, s, __VA_ARGS__); return hipGetLastError(); } while (0)

template <int MS, int MODE>
static hipError_t rowdot_nt(const RowdotArgs& a, int nt, hipStream_t s) {
    int blocks = a.C * a.p[0].tiles + (a.nprob > 1 ? a.C * a.p[1].tiles : 0);
    dim3 g(blocks), blk(64);
    switch (nt) {
        case 1: VIHMC_LAUNCH((k_rowdot<1, MS, MODE>), g, blk, 0, s, a);
        case 2: VIHMC_LAUNCH((k_rowdot<2, MS, MODE>), g, blk, 0, s, a);
        case 3: VIHMC_LAUNCH((k_rowdot<3, MS, MODE>), g, blk, 0, s, a);
        case 4: VIHMC_LAUNCH((k_rowdot<4, MS, MODE>), g, blk, 0, s, a);
        case 5: VIHMC_LAUNCH((k_rowdot<5, MS, MODE>), g, blk, 0, s, a);
        case 6: VIHMC_LAUNCH((k_rowdot<6, MS, MODE>), g, blk, 0, s, a);
        case 7: VIHMC_LAUNCH((k_rowdot<7, MS, MODE>), g, blk, 0, s, a);
        case 8: VIHMC_LAUNCH((k_rowdot<8, MS, MODE>), g, blk, 0, s, a);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rowdot(const RowdotArgs& a, int nt, int ms, int mode, hipStream_t s) {
    if (ms == 1) return mode == MODE_FWD ? rowdot_nt<1, MODE_FWD>(a, nt, s) : rowdot_nt<1, MODE_BWD>(a, nt, s);
    return mode == MODE_FWD ? rowdot_nt<2, MODE_FWD>(a, nt, s) : rowdot_nt<2, MODE_BWD>(a, nt, s);
}

hipError_t launch_colsum(const ColsumArgs& a, int jt, hipStream_t s) {
    int blocks = a.C * a.p[0].n_chunks * a.p[0].n_pairs +
                 (a.nprob > 1 ? a.C * a.p[1].n_chunks * a.p[1].n_pairs : 0);
    dim3 g(blocks), blk(64);
    switch (jt) {
        case 1: VIHMC_LAUNCH(k_colsum<1>, g, blk, 0, s, a);
        case 2: VIHMC_LAUNCH(k_colsum<2>, g, blk, 0, s, a);
        case 3: VIHMC_LAUNCH(k_colsum<3>, g, blk, 0, s, a);
        case 4: VIHMC_LAUNCH(k_colsum<4>, g, blk, 0, s, a);
        case 5: VIHMC_LAUNCH(k_colsum<5>, g, blk, 0, s, a);
        case 6: VIHMC_LAUNCH(k_colsum<6>, g, blk, 0, s, a);
        case 7: VIHMC_LAUNCH(k_colsum<7>, g, blk, 0, s, a);
        case 8: VIHMC_LAUNCH(k_colsum<8>, g, blk, 0, s, a);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_contract(const ContractProb& p, int C, bool with_grad, hipStream_t s) {
    dim3 g(C * p.o_tiles * p.q_chunks), blk(64);
    const int w = p.W;
    if (with_grad) {
        if (w <= 16) VIHMC_LAUNCH((k_contract<16, true>), g, blk, 0, s, p);
        if (w <= 32) VIHMC_LAUNCH((k_contract<32, true>), g, blk, 0, s, p);
        if (w <= 64) VIHMC_LAUNCH((k_contract<64, true>), g, blk, 0, s, p);
        if (w <= 112) VIHMC_LAUNCH((k_contract<112, true>), g, blk, 0, s, p);
        if (w <= 128) VIHMC_LAUNCH((k_contract<128, true>), g, blk, 0, s, p);
    } else {
        if (w <= 16) VIHMC_LAUNCH((k_contract<16, false>), g, blk, 0, s, p);
        if (w <= 32) VIHMC_LAUNCH((k_contract<32, false>), g, blk, 0, s, p);
        if (w <= 64) VIHMC_LAUNCH((k_contract<64, false>), g, blk, 0, s, p);
        if (w <= 112) VIHMC_LAUNCH((k_contract<112, false>), g, blk, 0, s, p);
        if (w <= 128) VIHMC_LAUNCH((k_contract<128, false>), g, blk, 0, s, p);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_init_packed(float* packed, int64_t dp, int C, const float* frozen, const int32_t* map_w,
                              const int32_t* map_wt, int64_t D, hipStream_t s) {
    dim3 g((unsigned)std::min<int64_t>((D + 255) / 256, 1024), C), blk(256);
    VIHMC_LAUNCH(k_init_packed, g, blk, 0, s, packed, dp, frozen, map_w, map_wt, D);
}

hipError_t launch_scatter(float* packed, int64_t dp, int C, const float* theta, int K, const int32_t* smap_w,
                          const int32_t* smap_wt, hipStream_t s) {
    dim3 g((unsigned)std::min((K + 255) / 256, 256), C), blk(256);
    VIHMC_LAUNCH(k_scatter, g, blk, 0, s, packed, dp, theta, K, smap_w, smap_wt);
}

hipError_t launch_reduce(const ReduceJob* jobs_dev, int n_jobs, int max_len, int C, hipStream_t s) {
    dim3 g((max_len + 255) / 256, n_jobs, C), blk(256);
    VIHMC_LAUNCH(k_reduce, g, blk, 0, s, jobs_dev);
}

hipError_t launch_contract_stats(const double* stats, int64_t stats_cs, int n_waves, int C, float* lik,
                                 float* gp, int64_t gp_cs, double count, int loss, float tau_out, hipStream_t s) {
    VIHMC_LAUNCH(k_contract_stats, dim3(C), dim3(256), 0, s, stats, stats_cs, n_waves, lik, gp, gp_cs, count,
                 loss, tau_out);
}

hipError_t launch_gather_prior(const float* gp, int64_t gp_cs, const int32_t* smap, const float* theta, int K,
                               const float* prior_mu, const float* prior_inv_var, double prior_const,
                               float prior_scale, const float* lik, int C, float* logp, float* grad,
                               hipStream_t s) {
    VIHMC_LAUNCH(k_gather_prior, dim3(C), dim3(256), 0, s, gp, gp_cs, smap, theta, K, prior_mu, prior_inv_var,
                 prior_const, prior_scale, lik, logp, grad);
}

size_t mlp_lds_bytes(int D, int n_layers, int maxw) {
    return sizeof(float) * (2 * (size_t)D + (size_t)(2 * n_layers + 3) * maxw * MLP_SLD);
}

hipError_t launch_mlp(const MlpArgs& a, int C, int maxw, hipStream_t s) {
    const size_t shm = mlp_lds_bytes(a.D, a.n_layers, maxw);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    VIHMC_LAUNCH(k_mlp, dim3(C), dim3(64), shm, s, a, maxw);
}

}  // namespace vihmc
