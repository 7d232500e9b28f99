// Layer GEMMs of the two MLPs (branch: N rows, trunk: P rows), batched over chains and grouped
// branch+trunk per launch.
//   k_rowdot2 : forward layer  h = act(x W^T + b)   (F.linear + tanh, my_make_func.py:52-77); used for the
//               input layers (K = 101 / 5) and any shape the fused forward (vihmc_fused.hip) does not take
//   k_bwd_ws  : layer backward (autograd of the same): delta_{l-1} = (delta_l W) * act'(h) and the dW / db
//               partial slabs in one pass
// fp32 MFMA v_mfma_f32_16x16x4_f32; operand maps and the float4 k-permutation: see vihmc_kernels.hip.
#include "vihmc_internal.h"

namespace vihmc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float act_apply_l(int act, float z) {
    if (act == ACT_TANH) return tanh_acc(z);
    if (act == ACT_TANH_CR) return tanh_cr(z);
    if (act == ACT_RELU) return fmaxf(z, 0.f);
    return z;
}

__device__ __forceinline__ float act_grad_from_out_l(int act, float h) {
    if (act == ACT_TANH || act == ACT_TANH_CR) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}

// LDS row stride (floats) for row-major operand images read by the MFMA k-permuted float4 pattern
// (lane l reads row l&15, float4 column kb/4 + (l>>4)). ds_read_b128 services the lanes in the groups
// {0-3,12-15,20-27} and {4-11,16-19,28-31} (+32); a stride == 8 (mod 16) puts the 16 lanes of each
// group on 16 distinct 4-bank groups (stride/4 odd alone leaves the lg=0/lg=1 halves 2-way; exhaustive
// check in DESIGN.md section 4). 100 -> 104.
__host__ __device__ constexpr int rowdot_ldb(int k4) { return k4 + ((24 - (k4 & 15)) & 15); }

// =============================================================================================
// Row-dot GEMM v2: 256-thread workgroup = 4 waves x 16*MS rows, the whole weight block B [Nn x K]
// staged once in LDS and shared; A rows streamed from HBM/L2 as float4 with a one-block register
// prefetch; MFMAs interleaved over MS*NT independent accumulators.
// =============================================================================================
// KF > 0: the contraction length is KF for every problem of the launch (hidden 100x100 layers), which
// makes the k-loop a compile-time loop the compiler can software-pipeline; KF = 0 reads P.K.
// Epilogue of one row tile: bias + activation (FWD) or * act'(h) (BWD), float4 stores; columns in
// [Nn, ldo) are written as zeros (padding read by the next GEMM). (A branch-free variant templated on
// the activation measured ~10% slower on the hidden layers; see profiles/README.md.)
// (Staging the output block through LDS for 1-KB row-major stores was measured slower: input layers 44.3 vs
// 35.6 us at C = 16, the staging LDS halves the resident workgroups; profiles/r02_input/README.md.)
template <int NT, int MS, int MODE>
__device__ __forceinline__ void rowdot_epilogue(const RowdotProb& P, int c, int m0, int lr, int lg,
                                                const f32x4 (&acc)[MS][NT]) {
    float* O = P.O + c * P.o_cs;
    const float* H = P.H + c * P.h_cs;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int n = 16 * t + 4 * lg;
        if (n >= P.ldo) continue;
        float4 bv = {0.f, 0.f, 0.f, 0.f};
        if (MODE == MODE_FWD && P.bias) bv = *reinterpret_cast<const float4*>(P.bias + c * P.bias_cs + n);
#pragma unroll
        for (int s = 0; s < MS; ++s) {
            const int m = m0 + 16 * s + lr;
            if (m >= P.M) continue;
            float4 o;
            if (MODE == MODE_FWD) {
                o.x = act_apply_l(P.act, acc[s][t][0] + bv.x);
                o.y = act_apply_l(P.act, acc[s][t][1] + bv.y);
                o.z = act_apply_l(P.act, acc[s][t][2] + bv.z);
                o.w = act_apply_l(P.act, acc[s][t][3] + bv.w);
            } else {
                const float4 h = *reinterpret_cast<const float4*>(H + (int64_t)m * P.ldh + n);
                o.x = acc[s][t][0] * act_grad_from_out_l(P.act, h.x);
                o.y = acc[s][t][1] * act_grad_from_out_l(P.act, h.y);
                o.z = acc[s][t][2] * act_grad_from_out_l(P.act, h.z);
                o.w = acc[s][t][3] * act_grad_from_out_l(P.act, h.w);
            }
            if (n + 3 >= P.Nn) {
                if (n + 0 >= P.Nn) o.x = 0.f;
                if (n + 1 >= P.Nn) o.y = 0.f;
                if (n + 2 >= P.Nn) o.z = 0.f;
                if (n + 3 >= P.Nn) o.w = 0.f;
            }
            *reinterpret_cast<float4*>(O + (int64_t)m * P.ldo + n) = o;
        }
    }
}

// KF > 0: the contraction length is KF for every problem of the launch (hidden 100x100 layers). The
// wave's whole A tile (MS x 16 rows x KF, k-permuted float4 per lane) is then loaded into registers at
// once, and the NEXT tile's loads are issued before the current tile's epilogue, so the HBM latency hides
// under the activation math instead of stalling the MFMA stream. KF = 0 reads P.K and prefetches one
// 16-wide k-block ahead.
template <int NT, int MS, int MODE, int KF>
__device__ __forceinline__ void rowdot_body(const RowdotProb& P, int b, float* bs) {
    const int c = b / P.tiles;
    const int grp = b - c * P.tiles;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const float* A = P.A + c * P.a_cs;
    const float* B = P.B + c * P.b_cs;
    const int KK = KF > 0 ? KF : P.K;
    const int K4 = (KK + 3) & ~3;
    const int LDB = rowdot_ldb(K4);

    // stage B (rows n < Nn, K4 floats each; global row stride ldb >= K4, zero padded). The loads of a thread's
    // pieces go out together (a plain strided loop waited out one load per piece: ~10 serial round trips for the
    // branch input layer's 100 x 104 block, which set the launch at one chain)
    {
        const int q4 = K4 >> 2;
        const int n4 = P.Nn * q4;
        constexpr int SP = 11;                          // pieces in flight per thread: 100 x 104 in one round
        for (int i0 = tid; i0 < n4; i0 += 256 * SP) {
            float4 v[SP];
#pragma unroll
            for (int u = 0; u < SP; ++u) {
                const int i = min(i0 + 256 * u, n4 - 1);   // clamped: every slot loads (stored only if in range)
                const int r = i / q4, c4 = i - r * q4;
                v[u] = *reinterpret_cast<const float4*>(B + (int64_t)r * P.ldb + 4 * c4);
            }
#pragma unroll
            for (int u = 0; u < SP; ++u) {                 // (clamped slots rewrite the last piece, same value)
                const int i = min(i0 + 256 * u, n4 - 1);
                const int r = i / q4, c4 = i - r * q4;
                *reinterpret_cast<float4*>(bs + r * LDB + 4 * c4) = v[u];
            }
        }
    }
    const float* br[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) br[t] = bs + min(16 * t + lr, P.Nn - 1) * LDB;
    const int tile_end = min(P.ntiles, (grp + 1) * P.tpw);
    // acc[s][t] holds the TRANSPOSED 16x16 tile O^T (MFMA A operand = weight rows n, B operand = data
    // rows m): lane l, register r = O[m0 + 16s + (l&15)][16t + 4(l>>4) + r], i.e. 4 consecutive output
    // columns of one row per lane -> float4 epilogue loads/stores.
    f32x4 acc[MS][NT];

    if constexpr (KF > 0) {
        constexpr int NKB = KF / 16;
        constexpr int NTL = ((KF & 15) + 3) / 4;     // 4-wide tail steps
        float4 abuf[MS][NKB];
        float atl[MS][NTL > 0 ? NTL : 1];
#define VIHMC_RD_LOAD_A(TILE, K0, K1, TL)                                                           \
        {                                                                                           \
            const int mt = (TILE) * (ROWDOT_WAVES * 16 * MS) + wave * 16 * MS;                      \
            _Pragma("unroll") for (int s = 0; s < MS; ++s) {                                        \
                const float* ap = A + (int64_t)min(mt + 16 * s + lr, P.M - 1) * P.lda;              \
                _Pragma("unroll") for (int k = (K0); k < (K1); ++k)                                 \
                    abuf[s][k] = *reinterpret_cast<const float4*>(ap + 16 * k + 4 * lg);            \
                if (TL) {                                                                           \
                    _Pragma("unroll") for (int k = 0; k < NTL; ++k) atl[s][k] = ap[16 * NKB + 4 * k + lg]; \
                }                                                                                   \
            }                                                                                       \
        }
        if (grp * P.tpw < tile_end) VIHMC_RD_LOAD_A(grp * P.tpw, 0, NKB, true)
        __syncthreads();
        for (int tile = grp * P.tpw; tile < tile_end; ++tile) {
            const int m0 = tile * (ROWDOT_WAVES * 16 * MS) + wave * 16 * MS;
#pragma unroll
            for (int s = 0; s < MS; ++s)
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            // weights of k-block k+1 are read from LDS while the MFMAs of block k run; the scheduling
            // barrier keeps the compiler from hoisting further blocks' reads (register pressure)
            float4 wc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) wc[t] = *reinterpret_cast<const float4*>(br[t] + 4 * lg);
#pragma unroll
            for (int k = 0; k < NKB; ++k) {
                float4 w[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) w[t] = wc[t];
                if (k + 1 < NKB) {
#pragma unroll
                    for (int t = 0; t < NT; ++t) wc[t] = *reinterpret_cast<const float4*>(br[t] + 16 * (k + 1) + 4 * lg);
                }
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].x, abuf[s][k].x, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].y, abuf[s][k].y, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].z, abuf[s][k].z, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].w, abuf[s][k].w, acc[s][t]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int k = 0; k < NTL; ++k) {
                float w[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) w[t] = br[t][16 * NKB + 4 * k + lg];
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t], atl[s][k], acc[s][t]);
            }
            // first half of the next tile's A goes out before the epilogue (hidden under it), the rest
            // after it (register budget: 3 waves/SIMD = 168 VGPRs)
            if (tile + 1 < tile_end) VIHMC_RD_LOAD_A(tile + 1, 0, NKB / 2, false)
            rowdot_epilogue<NT, MS, MODE>(P, c, m0, lr, lg, acc);
            if (tile + 1 < tile_end) VIHMC_RD_LOAD_A(tile + 1, NKB / 2, NKB, true)
        }
#undef VIHMC_RD_LOAD_A
    } else {
        __syncthreads();
        for (int tile = grp * P.tpw; tile < tile_end; ++tile) {
            const int m0 = tile * (ROWDOT_WAVES * 16 * MS) + wave * 16 * MS;
            const float* ar[MS];
#pragma unroll
            for (int s = 0; s < MS; ++s) ar[s] = A + (int64_t)min(m0 + 16 * s + lr, P.M - 1) * P.lda;
#pragma unroll
            for (int s = 0; s < MS; ++s)
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int kfull = KK & ~15;
            float4 a_cur[MS];
            if (kfull > 0) {
#pragma unroll
                for (int s = 0; s < MS; ++s) a_cur[s] = *reinterpret_cast<const float4*>(ar[s] + 4 * lg);
            }
            for (int kb = 0; kb < kfull; kb += 16) {
                float4 a_nxt[MS];
                const bool more = kb + 16 < kfull;
                if (more) {
#pragma unroll
                    for (int s = 0; s < MS; ++s) a_nxt[s] = *reinterpret_cast<const float4*>(ar[s] + kb + 16 + 4 * lg);
                }
                float4 w[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) w[t] = *reinterpret_cast<const float4*>(br[t] + kb + 4 * lg);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].x, a_cur[s].x, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].y, a_cur[s].y, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].z, a_cur[s].z, acc[s][t]);
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t].w, a_cur[s].w, acc[s][t]);
                if (more) {
#pragma unroll
                    for (int s = 0; s < MS; ++s) a_cur[s] = a_nxt[s];
                }
            }
            // tail: K rounded up to 4 (operand padding columns are zero)
            for (int kb = kfull; kb < K4; kb += 4) {
                float a[MS], w[NT];
#pragma unroll
                for (int s = 0; s < MS; ++s) a[s] = ar[s][kb + lg];
#pragma unroll
                for (int t = 0; t < NT; ++t) w[t] = br[t][kb + lg];
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int s = 0; s < MS; ++s) acc[s][t] = mfma(w[t], a[s], acc[s][t]);
            }
            rowdot_epilogue<NT, MS, MODE>(P, c, m0, lr, lg, acc);
        }
    }
}

template <int NT, int MS, int MODE, int KF>
__global__ __launch_bounds__(256, 3) void k_rowdot2(RowdotArgs args) {
    extern __shared__ float bs[];
    int b = blockIdx.x;
    const int first = args.C * args.p[0].tiles;
    const bool second = b >= first;
    const RowdotProb P = second ? args.p[1] : args.p[0];
    if (second) b -= first;
    rowdot_body<NT, MS, MODE, KF>(P, b, bs);
}

// Input layers (round 2): the first problem (branch, K = 101 padded to KF0 = 104) takes the whole-tile
// register preload of the KF path, the second (trunk, K = 5) the run-time-K path, instead of the run-time-K
// body (26 serial 16-long k blocks with one dependent global load each) for both. Measured neutral on one
// box: 37.1 vs 37.3 us per launch at C = 16 (profiles/r02_input/README.md) -- the branch workgroups do not
// set this launch; VIHMC_ROWDOT_IN_KF=0 selects the run-time-K body. A VALU kernel for both input layers
// (LDS-staged 4 x 4 register blocks for the branch, 4 outputs per thread for the trunk) measured 45-51 us
// and was not kept (profiles/r02_input/input_layer_valu_experiment.patch).
// MS0: row sub-tiles per wave of the branch (1: twice the workgroups of MS = 2 for its 16,000 rows at C = 16).
template <int NT, int MS, int KF0, int MS0>
__global__ __launch_bounds__(256, 3) void k_rowdot_in(RowdotArgs args) {
    extern __shared__ float bs[];
    int b = blockIdx.x;
    const int first = args.C * args.p[0].tiles;
    if (b >= first) {
        rowdot_body<NT, MS, MODE_FWD, 0>(args.p[1], b - first, bs);
    } else {
        rowdot_body<NT, MS0, MODE_FWD, KF0>(args.p[0], b, bs);
    }
}

// =============================================================================================
// Fused layer backward (see BwdProb), wave-specialised: a 512-thread workgroup = 4 dX waves + 4 dW
// waves sharing one LDS image of W^T (staged once) and of each 32-row sub-tile of delta_l and h_{l-1}
// (register prefetch of the next sub-tile by all 8 waves while the current one is consumed).
//   dX waves : Dout = (delta W) * act'(h) -- 2 row halves x 2 column-tile parities, transposed
//              accumulators (4 consecutive output columns per lane, float4 epilogue, h from LDS)
//   dW waves : part += delta^T h, db += sum delta -- wave w owns output rows n in subtiles {2w, 2w+1};
//              the 2 + NTI operands of step i+1 are read from LDS while the 2*NTI MFMAs of step i run
// Splitting the roles keeps each wave under 128 VGPRs (4 waves/SIMD at 2 workgroups/CU), which is what
// lets the LDS latency hide; the single-role v1 kernel needed 233 and serialised read -> wait -> MFMA.
// Deterministic: every partial slab has exactly one writer.
// =============================================================================================
constexpr int BWD_THREADS = 512;
constexpr int BWD_SLOTS = 4;   // staged float4 per thread per sub-tile (2 x 32 rows x <= 32 float4)

// dX of one 32-row sub-tile for one wave: 16 rows (half xh) x NUV column tiles of parity xpar
// (NUV = the tiles that exist: with n_in = 100 -> 7 tiles, parity 0 has 4 and parity 1 has 3; the
// 8th tile would be all padding)
template <int NUV, int KF>
__device__ __forceinline__ void bwd_dx_sub(const BwdProb& P, const float* dt, const float* wt, const float* ht,
                                           int LDT, int LDW, int LDH, int NO4, int NI4, int xh, int xpar,
                                           int lr, int lg, int sub, int r1, int c) {
    const int n_out = KF > 0 ? KF : P.n_out;
    const int kfull = n_out & ~15;
    const float4* drow = reinterpret_cast<const float4*>(dt + (16 * xh + lr) * LDT);
    const float* wrow[NUV];
#pragma unroll
    for (int u = 0; u < NUV; ++u) wrow[u] = wt + min(16 * (2 * u + xpar) + lr, P.n_in - 1) * LDW;
    f32x4 acc_x[NUV];
#pragma unroll
    for (int u = 0; u < NUV; ++u) acc_x[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < kfull; kb += 16) {
        const float4 dv = drow[(kb >> 2) + lg];
        float4 wv[NUV];
#pragma unroll
        for (int u = 0; u < NUV; ++u) wv[u] = reinterpret_cast<const float4*>(wrow[u])[(kb >> 2) + lg];
#pragma unroll
        for (int u = 0; u < NUV; ++u) acc_x[u] = mfma(wv[u].x, dv.x, acc_x[u]);
#pragma unroll
        for (int u = 0; u < NUV; ++u) acc_x[u] = mfma(wv[u].y, dv.y, acc_x[u]);
#pragma unroll
        for (int u = 0; u < NUV; ++u) acc_x[u] = mfma(wv[u].z, dv.z, acc_x[u]);
#pragma unroll
        for (int u = 0; u < NUV; ++u) acc_x[u] = mfma(wv[u].w, dv.w, acc_x[u]);
    }
    for (int kb = kfull; kb < NO4; kb += 4) {
        const float dv = dt[(16 * xh + lr) * LDT + kb + lg];
#pragma unroll
        for (int u = 0; u < NUV; ++u) acc_x[u] = mfma(wrow[u][kb + lg], dv, acc_x[u]);
    }
    const int m = sub + 16 * xh + lr;
    if (m < r1) {
        const float* hrow = ht + (16 * xh + lr) * LDH;
        float* orow = P.Dout + c * P.o_cs + (int64_t)m * P.ldh;
#pragma unroll
        for (int u = 0; u < NUV; ++u) {
            const int i = 16 * (2 * u + xpar) + 4 * lg;
            if (i >= NI4) continue;
            const float4 h = reinterpret_cast<const float4*>(hrow)[i >> 2];
            float4 o;
            o.x = (i + 0 < P.n_in) ? acc_x[u][0] * act_grad_from_out_l(P.act, h.x) : 0.f;
            o.y = (i + 1 < P.n_in) ? acc_x[u][1] * act_grad_from_out_l(P.act, h.y) : 0.f;
            o.z = (i + 2 < P.n_in) ? acc_x[u][2] * act_grad_from_out_l(P.act, h.z) : 0.f;
            o.w = (i + 3 < P.n_in) ? acc_x[u][3] * act_grad_from_out_l(P.act, h.w) : 0.f;
            reinterpret_cast<float4*>(orow)[i >> 2] = o;
        }
    }
}

// dW of one 32-row sub-tile for one wave: NS (1 or 2) 16-row output subtiles (rows ncol0/ncol1 of delta^T)
template <int NS, int NTI>
__device__ __forceinline__ void bwd_dw_sub(const float* dt, const float* ht, int LDT, int LDH, int ncol0, int ncol1,
                                           int jlast, int lr, int lg, f32x4 (&acc_w)[2][NTI], float (&dsum)[2]) {
    // step i covers rows base + 2*lg (base = 0,1,8,9,16,17,24,25): the two rows one b32 lane group
    // {0-31} touches are 2 apart, i.e. 2*LD == 16 (mod 32) banks apart -> conflict free.
#pragma unroll 2
    for (int mi = 0; mi < BWD_SUB / 4; ++mi) {
        const int mrow = (mi & 1) + 8 * (mi >> 1) + 2 * lg;
        const float* drw = dt + mrow * LDT;
        const float* hrw = ht + mrow * LDH + lr;
        const float a0 = drw[ncol0];
        const float a1 = NS > 1 ? drw[ncol1] : 0.f;
        float hv[NTI];
#pragma unroll
        for (int t = 0; t < NTI - 1; ++t) hv[t] = hrw[16 * t];
        hv[NTI - 1] = hrw[jlast];
#pragma unroll
        for (int t = 0; t < NTI; ++t) {
            acc_w[0][t] = mfma(a0, hv[t], acc_w[0][t]);
            if (NS > 1) acc_w[1][t] = mfma(a1, hv[t], acc_w[1][t]);
        }
        dsum[0] += a0;
        if (NS > 1) dsum[1] += a1;
    }
}

template <int NTI, int KF>
__global__ __launch_bounds__(BWD_THREADS, 4) void k_bwd_ws(BwdArgs args) {
    constexpr int NU = (NTI + 1) / 2;          // dX column tiles per wave (parity split)
    extern __shared__ float sm[];
    int b = blockIdx.x;
    const int per0 = args.C * args.p[0].n_wg;
    const bool second = b >= per0;
    const BwdProb P = second ? args.p[1] : args.p[0];
    if (second) b -= per0;
    const int c = b / P.n_wg;
    const int wg = b - c * P.n_wg;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const bool xrole = wave < 4;
    const int rw = wave & 3;
    const int n_out = KF > 0 ? KF : P.n_out;
    const int NO4 = (n_out + 3) & ~3, NI4 = (P.n_in + 3) & ~3;
    const int LDW = rowdot_ldb(NO4), LDT = rowdot_ldb(NO4), LDH = rowdot_ldb(NI4);
    float* wt = sm;
    float* dt = wt + (P.has_dx ? P.n_in * LDW : 0);
    float* ht = dt + BWD_SUB * LDT;
    const float* D = P.D + c * P.d_cs;
    const float* H = P.H + c * P.h_cs;
    const int r0 = wg * P.rows_per_wg;
    const int r1 = min(P.M, r0 + P.rows_per_wg);

    if (P.has_dx) {
        const float* WT = P.WT + c * P.wt_cs;
        const int q4 = NO4 >> 2, n4 = P.n_in * q4;
        for (int i = tid; i < n4; i += BWD_THREADS) {
            const int r = i / q4, c4 = i - r * q4;
            reinterpret_cast<float4*>(wt + r * LDW)[c4] = reinterpret_cast<const float4*>(WT + (int64_t)r * P.ldw)[c4];
        }
    }

    // staging geometry (identical for every sub-tile): slot v of this thread moves one float4 of a delta
    // (bit v of st_d) or h row
    const int dq4 = NO4 >> 2, hq4 = NI4 >> 2;
    const int nd4 = BWD_SUB * dq4, ntot = nd4 + BWD_SUB * hq4;
    float4 pf[BWD_SLOTS];
    int st[BWD_SLOTS];         // (row << 8) | float4 column, -1 = idle slot
    unsigned st_d = 0;         // bit v: slot v stages delta (else h)
#pragma unroll
    for (int v = 0; v < BWD_SLOTS; ++v) {
        const int idx = tid + BWD_THREADS * v;
        const bool isd = idx < nd4;
        const int e = isd ? idx : idx - nd4;
        const int q = isd ? dq4 : hq4;
        const int r = e / q, c4 = e - r * q;
        st[v] = idx < ntot ? (r << 8) | c4 : -1;
        st_d |= (isd ? 1u : 0u) << v;
    }
    const float4* Dv = reinterpret_cast<const float4*>(D);
    const float4* Hv = reinterpret_cast<const float4*>(H);
    float4* dt4 = reinterpret_cast<float4*>(dt);
    float4* ht4 = reinterpret_cast<float4*>(ht);
// An idle slot (st = -1) loads row SUB, column 0 -- an address inside the tile -- and never stores it. (It used to
// take the column from st & 255 = 255: a read 4 KB past the row, beyond the end of the delta / h buffer for narrow
// layers. Harmless while the next allocation was mapped there; the illegal-address faults of round 3
// (deeponet_odd_full) and round 4 (deeponet_small) were this read, found with VIHMC_GUARD=1: DESIGN §7.)
#define VIHMC_BWD_LOAD(SUB)                                                                         \
    _Pragma("unroll") for (int v = 0; v < BWD_SLOTS; ++v) {                                         \
        const int sv = max(st[v], 0);                                                               \
        const int row = min((SUB) + (sv >> 8), P.M - 1);                                            \
        const int c4 = sv & 255;                                                                    \
        pf[v] = ((st_d >> v) & 1) ? Dv[(int64_t)row * (P.ldd >> 2) + c4]                            \
                                  : Hv[(int64_t)row * (P.ldh >> 2) + c4];                           \
    }
#define VIHMC_BWD_STORE(SUB)                                                                        \
    _Pragma("unroll") for (int v = 0; v < BWD_SLOTS; ++v) {                                         \
        if (st[v] >= 0) {                                                                           \
            const int r = st[v] >> 8, c4 = st[v] & 255;                                             \
            const float4 val = ((SUB) + r < r1) ? pf[v] : float4{0.f, 0.f, 0.f, 0.f};               \
            if ((st_d >> v) & 1) dt4[r * (LDT >> 2) + c4] = val;                                    \
            else ht4[r * (LDH >> 2) + c4] = val;                                                    \
        }                                                                                           \
    }

    if (r0 < r1) {
        VIHMC_BWD_LOAD(r0)
    }
    // The two roles run separate sub-tile loops with the same barrier sequence (s_barrier counts waves),
    // so each role's registers are allocated for its own loop only.
    if (xrole) {
        // the parity is fixed per wave, so each parity gets its own loop (one dispatch, not one per sub-tile:
        // a per-sub-tile choice kept both variants' loop invariants live and spilled)
        const int xh = rw & 1, xpar = rw >> 1;
#define VIHMC_BWD_XLOOP(NUV)                                                                          \
        for (int sub = r0; sub < r1; sub += BWD_SUB) {                                                \
            VIHMC_BWD_STORE(sub)                                                                      \
            __syncthreads();                                                                          \
            if (sub + BWD_SUB < r1) {                                                                 \
                VIHMC_BWD_LOAD(sub + BWD_SUB)                                                         \
            }                                                                                         \
            if (P.has_dx)                                                                             \
                bwd_dx_sub<NUV, KF>(P, dt, wt, ht, LDT, LDW, LDH, NO4, NI4, xh, xpar, lr, lg, sub, r1, c); \
            __syncthreads();                                                                          \
        }
        if (xpar == 0 || (NTI & 1) == 0) {
            VIHMC_BWD_XLOOP(NU)
        } else {
            VIHMC_BWD_XLOOP((NTI / 2 > 0 ? NTI / 2 : 1))
        }
#undef VIHMC_BWD_XLOOP
        return;
    }

    // dW role: this wave's two 16-row output subtiles of dW
    const int ns0 = 2 * rw, ns1 = 2 * rw + 1;
    const bool dw0 = 16 * ns0 < P.n_out, dw1 = 16 * ns1 < P.n_out;
    f32x4 acc_w[2][NTI];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int t = 0; t < NTI; ++t) acc_w[s2][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dsum[2] = {0.f, 0.f};
    const int ncol0 = min(16 * ns0 + lr, P.n_out - 1), ncol1 = min(16 * ns1 + lr, P.n_out - 1);
    // h column of the last 16-wide tile, clamped (earlier tiles are always in range: NTI = ceil(n_in/16))
    const int jlast = min(16 * (NTI - 1) + lr, P.n_in - 1) - lr;
    for (int sub = r0; sub < r1; sub += BWD_SUB) {
        VIHMC_BWD_STORE(sub)
        __syncthreads();
        if (sub + BWD_SUB < r1) {
            VIHMC_BWD_LOAD(sub + BWD_SUB)
        }
        if (dw1) bwd_dw_sub<2, NTI>(dt, ht, LDT, LDH, ncol0, ncol1, jlast, lr, lg, acc_w, dsum);
        else if (dw0) bwd_dw_sub<1, NTI>(dt, ht, LDT, LDH, ncol0, ncol1, jlast, lr, lg, acc_w, dsum);
        __syncthreads();
    }
#undef VIHMC_BWD_LOAD
#undef VIHMC_BWD_STORE

    if (!dw0) return;
    float* part = P.part + c * P.part_cs + (int64_t)wg * P.part_stride;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const int ns = s2 == 0 ? ns0 : ns1;
        if (s2 == 1 && !dw1) continue;
#pragma unroll
        for (int t = 0; t < NTI; ++t) {
            const int j = 16 * t + lr;
            if (j >= NI4) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * ns + 4 * lg + r;
                if (n < P.n_out) part[(int64_t)n * NI4 + j] = (j < P.n_in) ? acc_w[s2][t][r] : 0.f;
            }
        }
        float v = dsum[s2];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int n = 16 * ns + lr;
        if (lg == 0 && n < P.n_out) part[(int64_t)P.n_out * NI4 + n] = v;
    }
}

// =============================================================================================
// launchers
// =============================================================================================
#define VIHMC_LAUNCH_L(kern, grid, block, shm, s, ...) \
    do { hipLaunchKernelGGL(kern, grid, block, shm, s, __VA_ARGS__); return hipGetLastError(); } while (0)

size_t rowdot_lds_bytes(const RowdotArgs& a) {
    // B image [Nn][ldb]
    size_t m = 0;
    for (int i = 0; i < a.nprob; ++i) {
        const int k4 = (a.p[i].K + 3) & ~3;
        m = std::max(m, sizeof(float) * (size_t)a.p[i].Nn * rowdot_ldb(k4));
    }
    return m;
}


// branch + trunk input layers of the Burgers DeepONet (K = 101 -> 104 padded columns, K <= 100 run time): the
// padded operand columns are zero (packed W rows, the uploaded input rows), so KF0 = 104 is exact
bool rowdot_in_ok(const RowdotArgs& a, int nt) {
    return nt == 7 && a.nprob == 2 && (a.p[0].K + 3) / 4 * 4 == 104 && a.p[0].lda >= 104 &&
           a.p[0].ldb >= 104 && a.p[1].K <= 100;
}

template <int MS, int MODE>
static hipError_t rowdot_nt(const RowdotArgs& a, int nt, hipStream_t s) {
    const int blocks = a.C * a.p[0].tiles + (a.nprob > 1 && !RD_ONLY_FIRST ? a.C * a.p[1].tiles : 0);
    const size_t shm = rowdot_lds_bytes(a);
    dim3 g(blocks), blk(256);
    const bool k100 = a.p[0].K == 100 && (a.nprob < 2 || a.p[1].K == 100);
    if (k100 && nt == 7) VIHMC_LAUNCH_L((k_rowdot2<7, MS, MODE, 100>), g, blk, shm, s, a);
    if (MODE == MODE_FWD && rowdot_in_ok(a, nt)) VIHMC_LAUNCH_L((k_rowdot_in<7, MS, 104, MS>), g, blk, shm, s, a);
    switch (nt) {
        case 1: VIHMC_LAUNCH_L((k_rowdot2<1, MS, MODE, 0>), g, blk, shm, s, a);
        case 2: VIHMC_LAUNCH_L((k_rowdot2<2, MS, MODE, 0>), g, blk, shm, s, a);
        case 3: VIHMC_LAUNCH_L((k_rowdot2<3, MS, MODE, 0>), g, blk, shm, s, a);
        case 4: VIHMC_LAUNCH_L((k_rowdot2<4, MS, MODE, 0>), g, blk, shm, s, a);
        case 5: VIHMC_LAUNCH_L((k_rowdot2<5, MS, MODE, 0>), g, blk, shm, s, a);
        case 6: VIHMC_LAUNCH_L((k_rowdot2<6, MS, MODE, 0>), g, blk, shm, s, a);
        case 7: VIHMC_LAUNCH_L((k_rowdot2<7, MS, MODE, 0>), g, blk, shm, s, a);
        case 8: VIHMC_LAUNCH_L((k_rowdot2<8, MS, MODE, 0>), g, blk, shm, s, a);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rowdot(const RowdotArgs& a, int nt, int ms, int mode, hipStream_t s) {
    // only the forward mode is launched (the layer backward is k_bwd_ws)
    if (mode != MODE_FWD) return hipErrorInvalidValue;
    return ms == 1 ? rowdot_nt<1, MODE_FWD>(a, nt, s) : rowdot_nt<2, MODE_FWD>(a, nt, s);
}

size_t bwd_lds_bytes(const BwdArgs& a) {
    size_t m = 0;
    for (int i = 0; i < a.nprob; ++i) {
        const BwdProb& p = a.p[i];
        const int no4 = (p.n_out + 3) & ~3, ni4 = (p.n_in + 3) & ~3;
        const size_t f = (size_t)(p.has_dx ? p.n_in * rowdot_ldb(no4) : 0) + (size_t)BWD_SUB * rowdot_ldb(no4) +
                         (size_t)BWD_SUB * rowdot_ldb(ni4);
        m = std::max(m, f * sizeof(float));
    }
    return m;
}

hipError_t launch_bwd(const BwdArgs& a, int nti, hipStream_t s) {
    const int blocks = a.C * a.p[0].n_wg + (a.nprob > 1 ? a.C * a.p[1].n_wg : 0);
    const size_t shm = bwd_lds_bytes(a);
    dim3 g(blocks), blk(BWD_THREADS);
    const bool k100 = a.p[0].n_out == 100 && (a.nprob < 2 || a.p[1].n_out == 100);
    if (k100 && nti == 7) VIHMC_LAUNCH_L((k_bwd_ws<7, 100>), g, blk, shm, s, a);
    switch (nti) {
        case 1: VIHMC_LAUNCH_L((k_bwd_ws<1, 0>), g, blk, shm, s, a);
        case 2: VIHMC_LAUNCH_L((k_bwd_ws<2, 0>), g, blk, shm, s, a);
        case 3: VIHMC_LAUNCH_L((k_bwd_ws<3, 0>), g, blk, shm, s, a);
        case 4: VIHMC_LAUNCH_L((k_bwd_ws<4, 0>), g, blk, shm, s, a);
        case 5: VIHMC_LAUNCH_L((k_bwd_ws<5, 0>), g, blk, shm, s, a);
        case 6: VIHMC_LAUNCH_L((k_bwd_ws<6, 0>), g, blk, shm, s, a);
        case 7: VIHMC_LAUNCH_L((k_bwd_ws<7, 0>), g, blk, shm, s, a);
        case 8: VIHMC_LAUNCH_L((k_bwd_ws<8, 0>), g, blk, shm, s, a);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace vihmc
