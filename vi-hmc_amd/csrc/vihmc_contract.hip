// Fused branch x trunk contraction + Gaussian likelihood (+ its backward) -- v2.
//
// Replaces torch.einsum("...i,...i->...", xb, xtr) + b (Operator_network/VI_HMC/my_make_func.py:79-82),
// GaussianNLLLoss / regression ll (main_VI_HMC_burgers.py:157-163) and their autograd backward.
//
// Owner form (see ContractProb): a 256-thread workgroup owns 128 rows of `Own` (32 per wave, held in
// registers as the B operand of S = Q . Own^T for the whole sweep) and streams `Q` in 16-row chunks
// through a double-buffered LDS image that all four waves share; the next chunk is prefetched
// global -> registers while the current one is consumed, then written to the other buffer.
//   S tile (16 q x 16 o per MFMA tile)  : A = Q rows   (ds_read_b128, 16 k per float4, k-permuted)
//   dOwn += G^T Q (16 o x 16 j tiles)   : A = G (the S accumulator registers, MFMA step rr = register rr)
//                                          B = Q[q][j] (ds_read_b32)
// The LDS row stride LDQ satisfies LDQ/4 odd, which makes both read patterns bank-conflict free:
// b128 row reads of 16 consecutive rows hit 16 distinct 4-bank groups, and the b32 reads of row pairs
// 4 apart (lane groups 0/1 and 2/3 of each half-wave) are 16 banks apart.
#include "vihmc_internal.h"


namespace vihmc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_c(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ T wave_sum_c(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__host__ __device__ constexpr int contract_ldq(int W) {
    return ((((W + 3) & ~3) / 4) & 1) ? ((W + 3) & ~3) : ((W + 3) & ~3) + 4;
}

// SNKB/SNTAIL >= 0 fix the k-block structure at compile time (the production width W = 100 is
// SNKB = 6 full 16-wide blocks + SNTAIL = 1 four-wide step); -1 reads it from W at run time.
// LOADG (side B): G is read from Y (written by side A, already scaled) instead of recomputing S; the
// owner rows are then not needed in registers.
template <int WMAX, int SNKB, int SNTAIL, bool GRAD, bool LOADG>
__global__ __launch_bounds__(256, 2) void k_contract2(ContractProb P) {
    constexpr int NB = WMAX / 16;
    constexpr int QC = CONTRACT_QC;
    extern __shared__ float qs[];                           // 2 x QC x LDQ
    const int W = P.W;
    const int W4 = (W + 3) & ~3;
    const int LDQ = contract_ldq(W);
    const int LDQ4 = LDQ >> 2;
    float4* qs4 = reinterpret_cast<float4*>(qs);
    int b = blockIdx.x;
    if (P.xcd_group) {
        // workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8): send the o_tiles workgroups of
        // one (chain, Q chunk) group to one XCD so the chunk is fetched into one L2 once
        const int xcd = b & 7, k = b >> 3;
        const int gx = k / P.o_tiles, og = k - gx * P.o_tiles;
        b = (gx * 8 + xcd) * P.o_tiles + og;
    }
    const int per_chain = P.o_tiles * P.q_chunks;
    const int c = b / per_chain;
    b -= c * per_chain;
    const int qc = b / P.o_tiles;
    const int og = b - qc * P.o_tiles;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const float* Own = P.Own + c * P.own_cs;
    const float* Q = P.Q + c * P.q_cs;
    const float b0 = P.b0[c * P.b0_cs];
    const float* Yc = P.Y + c * P.y_cs;
    const int o0 = og * CONTRACT_OWN_PER_WG + wave * 32;
    const int nkb = SNKB >= 0 ? SNKB : (W >> 4);
    const int ntail = SNTAIL >= 0 ? SNTAIL : ((W4 - (nkb << 4)) >> 2);
    const int JT = SNKB >= 0 ? SNKB + (SNTAIL > 0 ? 1 : 0) : ((W + 15) >> 4);

    float4 ob[2][NB];
    float otl[2][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if (LOADG) break;
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
    const int nchunks = q_hi > q_lo ? (q_hi - q_lo + QC - 1) / QC : 0;
    const int w4q = W4 >> 2;
    const int n4 = QC * w4q;
    // Q chunk staging: QC*W4/4 <= 512 float4 -> two per thread, always loaded (clamped index) so the
    // staging values live in registers across the compute of the current chunk.
    static_assert(QC * (WMAX / 4) <= 512, "chunk staging assumes <= 2 float4 per thread");
    const int i0 = min(tid, n4 - 1), i1 = min(tid + 256, n4 - 1);
    const int r0s = i0 / w4q, c0s = i0 - r0s * w4q, r1s = i1 / w4q, c1s = i1 - r1s * w4q;
    const bool st0 = tid < n4, st1 = tid + 256 < n4;
    float4 stg0, stg1;
#define VIHMC_LOAD_CHUNK(QROW0)                                                                       \
    stg0 = reinterpret_cast<const float4*>(Q + (int64_t)min((QROW0) + r0s, P.Mq - 1) * P.ldq)[c0s]; \
    stg1 = reinterpret_cast<const float4*>(Q + (int64_t)min((QROW0) + r1s, P.Mq - 1) * P.ldq)[c1s];
#define VIHMC_STORE_CHUNK(BUF4)                     \
    if (st0) (BUF4)[r0s * LDQ4 + c0s] = stg0;      \
    if (st1) (BUF4)[r1s * LDQ4 + c1s] = stg1;

    double ssq = 0.0, gsum = 0.0;
    float* sout = P.out + c * P.out_cs;
    if (nchunks > 0) {
        VIHMC_LOAD_CHUNK(q_lo)
        VIHMC_STORE_CHUNK(qs4)
    }
    // targets (side B: G) are loaded one chunk ahead so their HBM latency hides under the previous chunk
    float yn[2][4];
#define VIHMC_C2_YLOAD(QROW0)                                                                         \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                    \
        _Pragma("unroll") for (int r = 0; r < 4; ++r)                                                \
            yn[s][r] = Yc[(int64_t)min((QROW0) + 4 * lg + r, P.Mq - 1) * P.ldy + min(o0 + 16 * s + lr, P.Mo - 1)];
    VIHMC_C2_YLOAD(q_lo)
    __syncthreads();
    for (int ci = 0; ci < nchunks; ++ci) {
        const int q0 = q_lo + ci * QC;
        const float* cur = qs + (ci & 1) * QC * LDQ;
        const bool more = ci + 1 < nchunks;
        {
            const int h = 0;
            float yv[2][4];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int r = 0; r < 4; ++r) yv[s][r] = yn[s][r];
            VIHMC_C2_YLOAD(min(q0 + QC, q_hi - 1))
            if (more) {
                VIHMC_LOAD_CHUNK(q0 + QC)
            }
            f32x4 sacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            const float* qrow = cur + (16 * h + lr) * LDQ;
            const float4* qrow4 = reinterpret_cast<const float4*>(cur) + (16 * h + lr) * LDQ4;
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) {
                if (!LOADG && bb < nkb) {
                    const float4 qa = qrow4[4 * bb + lg];
                    sacc[0] = mfma_c(qa.x, ob[0][bb].x, sacc[0]);
                    sacc[1] = mfma_c(qa.x, ob[1][bb].x, sacc[1]);
                    sacc[0] = mfma_c(qa.y, ob[0][bb].y, sacc[0]);
                    sacc[1] = mfma_c(qa.y, ob[1][bb].y, sacc[1]);
                    sacc[0] = mfma_c(qa.z, ob[0][bb].z, sacc[0]);
                    sacc[1] = mfma_c(qa.z, ob[1][bb].z, sacc[1]);
                    sacc[0] = mfma_c(qa.w, ob[0][bb].w, sacc[0]);
                    sacc[1] = mfma_c(qa.w, ob[1][bb].w, sacc[1]);
                }
            }
#pragma unroll
            for (int ts = 0; ts < 3; ++ts) {
                if (!LOADG && ts < ntail) {
                    const float qa = qrow[16 * nkb + 4 * ts + lg];
                    sacc[0] = mfma_c(qa, otl[0][ts], sacc[0]);
                    sacc[1] = mfma_c(qa, otl[1][ts], sacc[1]);
                }
            }
            float g[2][4];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int qq = q0 + 16 * h + 4 * lg + r;
                    const int oo = o0 + 16 * s + lr;
                    const bool ok = (qq < q_hi) && (oo < P.Mo);
                    if (LOADG) {
                        g[s][r] = ok ? yv[s][r] : 0.f;
                        continue;
                    }
                    const float sv = sacc[s][r] + b0;
                    if (!GRAD && P.write_s && ok) sout[(int64_t)qq * P.ldout + oo] = sv;
                    const float rv = sv - yv[s][r];
                    const bool okm = ok && (!P.masked || yv[s][r] == yv[s][r]);   // NaN target: excluded pair
                    g[s][r] = okm ? P.gscale * rv : 0.f;
                    if (okm) {
                        ssq += (double)rv * (double)rv;
                        gsum += (double)g[s][r];
                    }
                }
            if (GRAD && !LOADG && P.gout) {
                // G^T[o][q .. q+3] for side B: 4 consecutive q of one o per lane -> one float4 store
                float* gw = P.gout + c * P.gout_cs;
                const int qq = q0 + 16 * h + 4 * lg;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int oo = o0 + 16 * s + lr;
                    if (oo >= P.Mo) continue;
                    float* dst = gw + (int64_t)oo * P.ldg + qq;
                    if (qq + 3 < q_hi) {
                        *reinterpret_cast<float4*>(dst) = float4{g[s][0], g[s][1], g[s][2], g[s][3]};
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (qq + r < q_hi) dst[r] = g[s][r];
                    }
                }
            }
            if (GRAD) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const float* qr = cur + (16 * h + 4 * lg + rr) * LDQ;
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if (t < JT) {
                            const float bq = qr[min(16 * t + lr, W - 1)];
                            dacc[0][t] = mfma_c(g[0][rr], bq, dacc[0][t]);
                            dacc[1][t] = mfma_c(g[1][rr], bq, dacc[1][t]);
                        }
                    }
                }
            }
        }
        if (more) {
            VIHMC_STORE_CHUNK(qs4 + ((ci + 1) & 1) * QC * LDQ4)
        }
        __syncthreads();
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
        ssq = wave_sum_c(ssq);
        gsum = wave_sum_c(gsum);
        if (lane == 0) {
            double* st = P.stats + c * P.stats_cs + 2 * (int64_t)((qc * P.o_tiles + og) * 4 + wave);
            st[0] = ssq;
            st[1] = gsum;
        }
    }
}

#undef VIHMC_LOAD_CHUNK
#undef VIHMC_STORE_CHUNK

// =============================================================================================
// Side A (gradient), width 100, wave-specialised: a 512-thread workgroup = 4 S waves + 4 D waves for
// the same 128 owner rows.
//   S wave w : owns 32 rows of Own in registers; per 16-row Q chunk computes S, G = gscale (S + b0 - y),
//              the likelihood sums, stores G^T for side B and hands G (its accumulator registers, as
//              two float4 per lane) to D wave w through LDS.
//   D wave w : one chunk behind, dOwn += G^T Q with G from LDS and Q[q][j] from the chunk's LDS image.
// Each role fits in 128 VGPRs (4 waves/SIMD at 2 workgroups/CU) where the single-role kernel needs 184
// (2 waves/SIMD). Q chunks rotate through 3 LDS buffers (S reads i, D reads i-1, the prefetch of i+1 is
// written), G through 2; one barrier per step; the two roles run separate loops with the same barrier
// sequence so each is register-allocated for its own work.
// =============================================================================================
namespace {
constexpr int CWS_QBUF = CONTRACT_QC * 100;                 // floats per Q chunk image (LDQ = 100)
constexpr int CWS_GBUF = 4 * 2 * 64;                        // float4 per G buffer (4 waves x 2 x 64 lanes)
}

__global__ __launch_bounds__(512, 2) void k_contract_ws(ContractProb P) {
    constexpr int QC = CONTRACT_QC;
    constexpr int LDQ = 100, LDQ4 = 25;
    static_assert(QC == 16, "k_contract_ws: 16-row chunks");
    extern __shared__ float sm[];
    f32x4* qs4 = reinterpret_cast<f32x4*>(sm);
    f32x4* gb = reinterpret_cast<f32x4*>(sm + 3 * CWS_QBUF);
    int b = blockIdx.x;
    const int per_chain = P.o_tiles * P.q_chunks;
    const int c = b / per_chain;
    b -= c * per_chain;
    const int qc = b / P.o_tiles;
    const int og = b - qc * P.o_tiles;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int w = wave & 3;
    const float* Q = P.Q + c * P.q_cs;
    const int o0 = og * CONTRACT_OWN_PER_WG + w * 32;
    const int q_lo = qc * P.q_per_chunk;
    const int q_hi = min(q_lo + P.q_per_chunk, P.Mq);
    const int nchunks = q_hi > q_lo ? (q_hi - q_lo + QC - 1) / QC : 0;

    // chunk staging: 16 x 25 float4, one per thread (threads >= 400 stage a duplicate into a dump slot)
    const int sr = min(tid, 399) / 25, sc = min(tid, 399) % 25;
    const int sdst = tid < 400 ? sr * LDQ4 + sc : -1;
    f32x4 stg;
#define VIHMC_CWS_LOAD(CI) \
    stg = reinterpret_cast<const f32x4*>(Q + (int64_t)min(q_lo + (CI) * QC + sr, P.Mq - 1) * P.ldq)[sc];
#define VIHMC_CWS_STORE(BUF) \
    if (sdst >= 0) qs4[(BUF) * (CWS_QBUF / 4) + sdst] = stg;

    if (nchunks > 0) {
        VIHMC_CWS_LOAD(0)
        VIHMC_CWS_STORE(0)
        VIHMC_CWS_LOAD(min(1, nchunks - 1))
    }

    if (wave < 4) {
        // ---------------- S role ----------------
        const float* Own = P.Own + c * P.own_cs;
        const float* Yc = P.Y + c * P.y_cs;
        const float b0 = P.b0[c * P.b0_cs];
        float4 ob[2][6];
        float otl[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const float* orow = Own + (int64_t)min(o0 + 16 * s + lr, P.Mo - 1) * P.ldown;
#pragma unroll
            for (int bb = 0; bb < 6; ++bb) ob[s][bb] = *reinterpret_cast<const float4*>(orow + 16 * bb + 4 * lg);
            otl[s] = orow[96 + lg];
        }
        double ssq = 0.0, gsum = 0.0;
        float* gw = P.gout ? P.gout + c * P.gout_cs : nullptr;
        // targets are loaded one chunk ahead (HBM latency hidden under a chunk of MFMAs)
        float yn[2][4];
#define VIHMC_CWS_YLOAD(CI)                                                                          \
        _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                \
            _Pragma("unroll") for (int r = 0; r < 4; ++r)                                            \
                yn[s][r] = Yc[(int64_t)min(q_lo + (CI) * QC + 4 * lg + r, P.Mq - 1) * P.ldy +         \
                              min(o0 + 16 * s + lr, P.Mo - 1)];
        VIHMC_CWS_YLOAD(0)
        for (int i = 0; i <= nchunks; ++i) {
            __syncthreads();
            if (i < nchunks) {
                const int q0 = q_lo + i * QC;
                const float* cur = sm + (i % 3) * CWS_QBUF;
                float yv[2][4];
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int r = 0; r < 4; ++r) yv[s][r] = yn[s][r];
                // drained right after the next chunk's y loads (measured faster than leaving them in flight: 0.64 vs 0.67 ms)
                VIHMC_CWS_YLOAD(min(i + 1, nchunks - 1))
                __builtin_amdgcn_s_waitcnt(0x0F70);
                f32x4 sacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
                const float4* qrow4 = reinterpret_cast<const float4*>(cur) + lr * LDQ4;
#pragma unroll
                for (int bb = 0; bb < 6; ++bb) {
                    const float4 qa = qrow4[4 * bb + lg];
                    sacc[0] = mfma_c(qa.x, ob[0][bb].x, sacc[0]);
                    sacc[1] = mfma_c(qa.x, ob[1][bb].x, sacc[1]);
                    sacc[0] = mfma_c(qa.y, ob[0][bb].y, sacc[0]);
                    sacc[1] = mfma_c(qa.y, ob[1][bb].y, sacc[1]);
                    sacc[0] = mfma_c(qa.z, ob[0][bb].z, sacc[0]);
                    sacc[1] = mfma_c(qa.z, ob[1][bb].z, sacc[1]);
                    sacc[0] = mfma_c(qa.w, ob[0][bb].w, sacc[0]);
                    sacc[1] = mfma_c(qa.w, ob[1][bb].w, sacc[1]);
                }
                {
                    const float qa = cur[lr * LDQ + 96 + lg];
                    sacc[0] = mfma_c(qa, otl[0], sacc[0]);
                    sacc[1] = mfma_c(qa, otl[1], sacc[1]);
                }
                f32x4 g[2];
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int qq = q0 + 4 * lg + r;
                        const int oo = o0 + 16 * s + lr;
                        const bool ok = (qq < q_hi) && (oo < P.Mo);
                        const float rv = sacc[s][r] + b0 - yv[s][r];
                        const bool okm = ok && (!P.masked || yv[s][r] == yv[s][r]);   // NaN target: excluded
                        g[s][r] = okm ? P.gscale * rv : 0.f;
                        if (okm) {
                            ssq += (double)rv * (double)rv;
                            gsum += (double)g[s][r];
                        }
                    }
                f32x4* gdst = gb + ((i & 1) * 4 + w) * 128;
                gdst[lane] = g[0];
                gdst[64 + lane] = g[1];
                if (gw) {
                    const int qq = q0 + 4 * lg;
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int oo = o0 + 16 * s + lr;
                        if (oo >= P.Mo) continue;
                        float* dst = gw + (int64_t)oo * P.ldg + qq;
                        if (qq + 3 < q_hi) {
                            *reinterpret_cast<f32x4*>(dst) = g[s];
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (qq + r < q_hi) dst[r] = g[s][r];
                        }
                    }
                }
            }
            VIHMC_CWS_STORE((i + 1) % 3)
            VIHMC_CWS_LOAD(max(min(i + 2, nchunks - 1), 0))
        }
        if (P.with_stats) {
            ssq = wave_sum_c(ssq);
            gsum = wave_sum_c(gsum);
            if (lane == 0) {
                double* st = P.stats + c * P.stats_cs + 2 * (int64_t)((qc * P.o_tiles + og) * 4 + w);
                st[0] = ssq;
                st[1] = gsum;
            }
        }
        return;
    }

    // ---------------- D role ----------------
    f32x4 dacc[2][7];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 7; ++t) dacc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i <= nchunks; ++i) {
        __syncthreads();
        if (i >= 1) {
            const float* cur = sm + ((i - 1) % 3) * CWS_QBUF;
            const f32x4* gsrc = gb + (((i - 1) & 1) * 4 + w) * 128;
            const f32x4 g0 = gsrc[lane], g1 = gsrc[64 + lane];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const float* qr = cur + (4 * lg + rr) * LDQ;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const float bq = qr[min(16 * t + lr, 99)];
                    dacc[0][t] = mfma_c(g0[rr], bq, dacc[0][t]);
                    dacc[1][t] = mfma_c(g1[rr], bq, dacc[1][t]);
                }
            }
        }
        VIHMC_CWS_STORE((i + 1) % 3)
        VIHMC_CWS_LOAD(max(min(i + 2, nchunks - 1), 0))
    }
    float* out = P.out + c * P.out_cs + (int64_t)qc * P.out_chunk_stride;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int j = 16 * t + lr;
            if (j >= P.ldout) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int oo = o0 + 16 * s + 4 * lg + r;
                if (oo < P.Mo) out[(int64_t)oo * P.ldout + j] = (j < 100) ? dacc[s][t][r] : 0.f;
            }
        }
#undef VIHMC_CWS_LOAD
#undef VIHMC_CWS_STORE
#undef VIHMC_CWS_YLOAD
}

size_t contract_lds_bytes(int W) { return sizeof(float) * 2 * CONTRACT_QC * contract_ldq(W); }

#define VIHMC_LAUNCH_C(kern, grid, block, shm, s, ...) \
    do { hipLaunchKernelGGL(kern, grid, block, shm, s, __VA_ARGS__); return hipGetLastError(); } while (0)

template <bool GRAD, bool LOADG>
static hipError_t launch_contract_t(const ContractProb& p, int C, hipStream_t s) {
    dim3 g(C * p.o_tiles * p.q_chunks), blk(256);
    const size_t shm = contract_lds_bytes(p.W);
    const int w = p.W;
    if (w == 100 && GRAD && !LOADG && p.bf16x6) return launch_contract_bf(p, C, s);
    if (w == 100 && GRAD && LOADG && p.bf16x6) return launch_contract_bf_b(p, C, s);
    if (w == 100 && GRAD && !LOADG && VIHMC_CONTRACT_WS) {
        dim3 blk2(512);
        VIHMC_LAUNCH_C(k_contract_ws, g, blk2, sizeof(float) * 3 * CWS_QBUF + 16 * 2 * CWS_GBUF, s, p);
    }
    if (w == 100) VIHMC_LAUNCH_C((k_contract2<112, 6, 1, GRAD, LOADG>), g, blk, shm, s, p);
    if (w <= 16) VIHMC_LAUNCH_C((k_contract2<16, -1, -1, GRAD, LOADG>), g, blk, shm, s, p);
    if (w <= 32) VIHMC_LAUNCH_C((k_contract2<32, -1, -1, GRAD, LOADG>), g, blk, shm, s, p);
    if (w <= 64) VIHMC_LAUNCH_C((k_contract2<64, -1, -1, GRAD, LOADG>), g, blk, shm, s, p);
    if (w <= 112) VIHMC_LAUNCH_C((k_contract2<112, -1, -1, GRAD, LOADG>), g, blk, shm, s, p);
    if (w <= 128) VIHMC_LAUNCH_C((k_contract2<128, -1, -1, GRAD, LOADG>), g, blk, shm, s, p);
    return hipErrorInvalidValue;
}

hipError_t launch_contract(const ContractProb& p, int C, bool with_grad, hipStream_t s) {
    if (p.load_g) return with_grad ? launch_contract_t<true, true>(p, C, s) : hipErrorInvalidValue;
    return with_grad ? launch_contract_t<true, false>(p, C, s) : launch_contract_t<false, false>(p, C, s);
}

}  // namespace vihmc
