// Fused layer backward with fp32 products on the bf16 MFMA (bf16x6, vihmc_bf16x6.h): the same BwdProb
// contract and outputs as k_bwd_ws (vihmc_layers.hip), for layers with n_out = 100 and n_in <= 112.
//
// Replaces the autograd backward of one nn.Linear + activation of the branch / trunk MLPs
// (Operator_network/VI_HMC/my_make_func.py:53-82, torch autograd through F.linear and tanh):
//   Dout[m][i] = (sum_k D[m][k] W[k][i]) * act'(H[m][i])        (dX, when has_dx)
//   part[n][j] = sum_m D[m][n] H[m][j],  part[n_out][n] = sum_m D[m][n]   (dW, db partial of this chunk)
//
// One 1024-thread workgroup per CU (16 waves, 4 per SIMD, <= 128 VGPRs) per row chunk; 32-row sub-tiles
// of D and H are split into bf16 planes by all threads (register prefetch one sub-tile ahead, two LDS
// buffers, one barrier per sub-tile). LDS (150 KB):
//   2 x [D planes [3][32][224 B], H planes [3][32][224 B], D fp32 tail [32][4] (features 96..99)]
//   W^T planes [3][100][208 B] + fp32 tail [100][4], split once per workgroup
//   dX waves (8): i-tiles {2p, 2p+1} x 16-row half h. A = W^T rows, B = D rows (ds_read_b128 of the
//                 planes); the 4-long k tail is one exact f32 MFMA that seeds the accumulator.
//                 Epilogue: act'(h) from the H planes (exact reconstruction h = h2 + h1 + h0), float4 stores.
//   dW waves (8): output row tiles {2q, 2q+1} x column tiles 0..3 or 4..6; A = D^T and B = H, both by
//                 transposed reads (k = the 32 rows of the sub-tile).
//   db: summed from the staged D values by the staging threads (fixed slot -> column map), reduced
//       in a fixed order at the end. Deterministic: every partial slab has exactly one writer.
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"
#include <cstdlib>
#include <type_traits>

#ifndef BB_ABL
#define BB_ABL 0    // timing-only ablations (wrong results): 1 no loads after the first sub-tile, 2 no dX
                    // MFMAs, 3 no dW MFMAs, 4 no three-way split (one cvt), 5 dX W operands not re-read
                    // from LDS per sub-tile, 6 no LDS plane stores after the first sub-tile, 7 no dX (Dout) stores
#endif

#ifndef BB_ROW32
#define BB_ROW32 1        // staging slots row-aligned (32 per row) instead of packed 25 per row
#endif

#ifndef BB_WREG
#define BB_WREG 2         // dX waves keep W^T fragments in registers (loaded once) instead of LDS re-reads:
                          // 1 both i-tiles (spills at 128 VGPRs), 2 the first i-tile only
#endif

#ifndef BB_WPITCH_B
#define BB_WPITCH_B 224   // W^T plane row pitch (bytes)
#endif

namespace vihmc {

namespace {
using bf6::f32x4;
using bf6::bf16x8;
using bf6::bf16x4;
using bf6::split4;
using bf6::cat8;
using bf6::six;
using bf6::tr_frag;

constexpr int BB_SUB = BWD_SUB;                        // 32 rows per sub-tile
constexpr int BB_PITCH = bf6::PITCH;                   // D / H plane rows (transposed reads: 7 x 32 B)
constexpr int BB_PLANE = BB_SUB * BB_PITCH;            // 7168
constexpr int BB_DP = 0;                               // D planes
constexpr int BB_HP = 3 * BB_PLANE;                    // H planes
constexpr int BB_DT = 6 * BB_PLANE;                    // D fp32 tail [32][4]
constexpr int BB_BUF = BB_DT + BB_SUB * 16;            // 43520 bytes per buffer
// W^T plane rows: read like the D planes (lane l: row l & 15, 16-B column l >> 4), so the same pitch
// residue (8 mod 16 dwords) keeps the b128 reads conflict free; 208 B (4 mod 16) measured 2-way
constexpr int BB_WPITCH = BB_WPITCH_B;
constexpr int BB_WPLANE = 100 * BB_WPITCH;             // 20800 (rows 0..99; tile-6 reads clamp to row 99)
constexpr int BB_W = 2 * BB_BUF;                       // W^T planes after the two sub-tile buffers
constexpr int BB_WT = BB_W + 3 * BB_WPLANE;            // W^T fp32 tail [100][4]
constexpr int BB_LDS = BB_WT + 100 * 16;               // 154880 (pitch 224)
static_assert(BB_LDS <= 160 * 1024, "LDS");
constexpr int BB_THREADS = 1024;                       // 8 dX + 8 dW waves, 4 per SIMD
constexpr int BB_SLOTS = 2;                            // staged float4 per thread (<= 800 D + 896 H)

__device__ __forceinline__ float act_grad_bf(int act, float h) {
    // derivative from the activation's output (tanh: 1 - h^2, relu: h > 0), as act_grad_from_out_l
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}
}  // namespace

#ifndef BB_STAMP
#define BB_STAMP 0        // timing-only instrumentation (variant builds): in-kernel phase stamps
#endif
#if BB_STAMP
// every 16th trunk workgroup of the launches with a dX part (the last one written wins: layer 1): per wave and
// sub-tile s_memtime at the barrier exit [0], after the staging of the next sub-tile [1], when the MFMA results
// exist [2]; per workgroup s_memtime / s_memrealtime at start and end (scripts/diag/stamps_bwd.py)
constexpr int BBS_WG = 16, BBS_SUB = 32;
__device__ unsigned long long bb_stamps[BBS_WG][16][BBS_SUB][3];
__device__ unsigned long long bb_real[BBS_WG][2][2];
#define VIHMC_BB_STAMP(I, K)                                                                                  \
    if (samp && lane == 0 && (I) < BBS_SUB) bb_stamps[sidx][wave][(I)][(K)] = __builtin_amdgcn_s_memtime();
#else
#define VIHMC_BB_STAMP(I, K)
#endif

__global__ __launch_bounds__(BB_THREADS, 1) void k_bwd_bf(BwdArgs args) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smw[];
    int b = blockIdx.x;
    const int per0 = args.C * args.p[0].n_wg;
    const bool second = b >= per0;
    const BwdProb P = second ? args.p[1] : args.p[0];
    if (second) b -= per0;
    const int c = b / P.n_wg;
    const int wg = b - c * P.n_wg;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int NI4 = (P.n_in + 3) & ~3;
#if BB_STAMP
    const bool samp = second && P.has_dx && (b % 16) == 0 && b / 16 < BBS_WG;
    const int sidx = b / 16;
    if (samp && tid == 0) {
        bb_real[sidx][0][0] = __builtin_amdgcn_s_memtime();
        bb_real[sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const int hq4 = NI4 >> 2;                          // H float4 per row (<= 28)
    const float* D = P.D + c * P.d_cs;
    const float* H = P.H + c * P.h_cs;
    const int r0 = wg * P.rows_per_wg;
    const int r1 = min(P.M, r0 + P.rows_per_wg);

    // ---- W^T planes (once per workgroup): rows i < n_in, features k < 100 ----
    if (P.has_dx) {
        const float* WT = P.WT + c * P.wt_cs;
        for (int idx = tid; idx < P.n_in * 25; idx += BB_THREADS) {
            const int r = idx / 25, c4 = idx - r * 25;
            const f32x4 x = *reinterpret_cast<const f32x4*>(WT + (int64_t)r * P.ldw + 4 * c4);
            bf16x4 p0, p1, p2;
            split4(x, p0, p1, p2);
            unsigned char* o = smw + BB_W + r * BB_WPITCH + 8 * c4;
            *reinterpret_cast<bf16x4*>(o) = p0;
            *reinterpret_cast<bf16x4*>(o + BB_WPLANE) = p1;
            *reinterpret_cast<bf16x4*>(o + 2 * BB_WPLANE) = p2;
            if (c4 == 24) *reinterpret_cast<f32x4*>(smw + BB_WT + r * 16) = x;
        }
    }

    // ---- staging geometry: slot v of this thread moves float4 (row, c4) of D (idx < 800) or H ----
    int st[BB_SLOTS];                                  // (row << 8) | c4, -1 idle
    unsigned st_d = 0;
#if BB_ROW32
    // slot 0 = D, slot 1 = H, 32 slots per row (c4 = tid & 31; 25 / hq4 of them active): the 16-lane groups of
    // the bf16x4 plane stores never straddle two rows (25 float4 per row did: 2-way bank conflicts)
    static_assert(BB_SLOTS == 2 && BB_SUB * 32 == BB_THREADS, "row-aligned staging map");
#pragma unroll
    for (int v = 0; v < BB_SLOTS; ++v) {
        const int r = tid >> 5, c4 = tid & 31;
        st[v] = c4 < (v == 0 ? 25 : hq4) ? (r << 8) | c4 : -1;
    }
    st_d = 1u;
#else
    const int ntot = BB_SUB * 25 + BB_SUB * hq4;
#pragma unroll
    for (int v = 0; v < BB_SLOTS; ++v) {
        const int idx = tid + BB_THREADS * v;
        const bool isd = idx < BB_SUB * 25;
        const int e = isd ? idx : idx - BB_SUB * 25;
        const int q = isd ? 25 : hq4;
        const int r = e / q, c4 = e - r * q;
        st[v] = idx < ntot ? (r << 8) | c4 : -1;
        st_d |= (isd ? 1u : 0u) << v;
    }
#endif
    f32x4 pf[BB_SLOTS];
    f32x4 dcol = {0.f, 0.f, 0.f, 0.f};                 // db partial of this thread's D slot (slot 0 only:
                                                       // idx < 800 < 1024)
#define VIHMC_BB_LOAD(SUB)                                                                              \
    _Pragma("unroll") for (int v = 0; v < BB_SLOTS; ++v) {                                              \
        const int row = min((SUB) + (max(st[v], 0) >> 8), P.M - 1);                                     \
        const int c4 = max(st[v], 0) & 255;            /* idle slots read column 0: in bounds */        \
        pf[v] = ((st_d >> v) & 1) ? reinterpret_cast<const f32x4*>(D + (int64_t)row * P.ldd)[c4]        \
                                  : reinterpret_cast<const f32x4*>(H + (int64_t)row * P.ldh)[c4];       \
    }
#define VIHMC_BB_STORE(SUB, BUF)                                                                        \
    _Pragma("unroll") for (int v = 0; v < BB_SLOTS; ++v) {                                              \
        if (st[v] >= 0) {                                                                               \
            const int r = st[v] >> 8, c4 = st[v] & 255;                                                 \
            const f32x4 x = ((SUB) + r < r1) ? pf[v] : f32x4{0.f, 0.f, 0.f, 0.f};                       \
            const bool isd = (st_d >> v) & 1;                                                           \
            unsigned char* base = smw + (BUF) * BB_BUF + (isd ? BB_DP : BB_HP) + r * BB_PITCH + 8 * c4; \
            bf16x4 p0, p1, p2;                                                                          \
            if (BB_ABL == 4) {                                                                          \
                for (int j_ = 0; j_ < 4; ++j_) p0[j_] = (__bf16)x[j_];                                  \
                p1 = p0;                                                                                \
                p2 = p0;                                                                                \
            } else {                                                                                    \
                split4(x, p0, p1, p2);                                                                  \
            }                                                                                           \
            if (BB_ABL != 6 || (SUB) == r0) {                                                           \
                *reinterpret_cast<bf16x4*>(base) = p0;                                                  \
                *reinterpret_cast<bf16x4*>(base + BB_PLANE) = p1;                                       \
                *reinterpret_cast<bf16x4*>(base + 2 * BB_PLANE) = p2;                                   \
            }                                                                                           \
            if (isd) {                                                                                  \
                if (v == 0) dcol += x;                                                                  \
                if (c4 == 24) *reinterpret_cast<f32x4*>(smw + (BUF) * BB_BUF + BB_DT + r * 16) = x;     \
            }                                                                                           \
        }                                                                                               \
    }

    const int nsub = r1 > r0 ? (r1 - r0 + BB_SUB - 1) / BB_SUB : 0;
    if (nsub > 0) {
        VIHMC_BB_LOAD(r0)
        VIHMC_BB_STORE(r0, 0)
        if (nsub > 1) {
            VIHMC_BB_LOAD(r0 + BB_SUB)
        }
    }

#ifndef BB_PRIO
#define BB_PRIO 2       // static wave priority: 1 dW waves (dispatched second) at 1: 69 -> 76 us; 2 dX waves at 1: 68.5 -> 67 us
#endif
    if (BB_PRIO == 1 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 512) __builtin_amdgcn_s_setprio(1);
    if (BB_PRIO == 2 && __builtin_amdgcn_readfirstlane(threadIdx.x) < 512) __builtin_amdgcn_s_setprio(1);
    if (wave < 8) {
        // ---------------- dX role: i-tiles {2p, 2p+1} x row half h ----------------
        const int h = wave & 1, p2 = wave >> 1;
        const int t0 = 2 * p2;
        const bool two = t0 + 1 < 7;
        const unsigned char* wrow0 = smw + BB_W + min(16 * t0 + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const unsigned char* wrow1 = smw + BB_W + min(16 * (t0 + 1) + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const float* wtl = reinterpret_cast<const float*>(smw + BB_WT);
        const int wr0 = min(16 * t0 + lr, P.n_in - 1), wr1 = min(16 * (t0 + 1) + lr, P.n_in - 1);
#if BB_WREG
        bf16x8 wra[3][3], wrb[3][3];                   // [kb][plane] W^T fragments, loaded once (after barrier 0)
        float wta = 0.f, wtb = 0.f;
#endif
        for (int i = 0; i < nsub; ++i) {
            const int sub = r0 + i * BB_SUB;
            __syncthreads();                           // buffer i&1 holds sub-tile i
            VIHMC_BB_STAMP(i, 0)
#if BB_WREG
            if (i == 0 && P.has_dx) {
#pragma unroll
                for (int kb = 0; kb < 3; ++kb)
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        wra[kb][p] = *reinterpret_cast<const bf16x8*>(wrow0 + p * BB_WPLANE + 64 * kb);
                        if (BB_WREG == 1) wrb[kb][p] = *reinterpret_cast<const bf16x8*>(wrow1 + p * BB_WPLANE + 64 * kb);
                    }
                wta = wtl[wr0 * 4 + lg];
                wtb = wtl[wr1 * 4 + lg];
            }
#endif
            if (i + 1 < nsub) {
                VIHMC_BB_STORE(sub + BB_SUB, (i + 1) & 1)
                if (i + 2 < nsub && BB_ABL != 1) {
                    VIHMC_BB_LOAD(sub + 2 * BB_SUB)
                }
            }
            VIHMC_BB_STAMP(i, 1)
            if (!P.has_dx) continue;
            const unsigned char* buf = smw + (i & 1) * BB_BUF;
            const unsigned char* drow = buf + BB_DP + (16 * h + lr) * BB_PITCH + 16 * lg;
            // the exact f32 tail (features 96..99) seeds each accumulator
            const float dtl = reinterpret_cast<const float*>(buf + BB_DT)[(16 * h + lr) * 4 + lg];
            f32x4 acc[2];
#if BB_WREG
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wta, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            acc[1] = two ? __builtin_amdgcn_mfma_f32_16x16x4f32(wtb, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < 3; ++kb) {
                bf16x8 db[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) db[p] = *reinterpret_cast<const bf16x8*>(drow + p * BB_PLANE + 64 * kb);
                acc[0] = six(wra[kb], db, acc[0]);
                if (BB_WREG == 2) {
                    // only the first i-tile's W^T in registers (VGPR budget); the second re-read from LDS
#pragma unroll
                    for (int p = 0; p < 3; ++p) wrb[kb][p] = *reinterpret_cast<const bf16x8*>(wrow1 + p * BB_WPLANE + 64 * kb);
                }
                if (two) acc[1] = six(wrb[kb], db, acc[1]);
            }
            if (false)
#else
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wtl[wr0 * 4 + lg], dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            acc[1] = two ? __builtin_amdgcn_mfma_f32_16x16x4f32(wtl[wr1 * 4 + lg], dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
#endif
#pragma unroll
            for (int kb = 0; kb < 3; ++kb) {
                bf16x8 db[3], wa[3], wb[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    db[p] = *reinterpret_cast<const bf16x8*>(drow + p * BB_PLANE + 64 * kb);
                    if (BB_ABL == 5) {
                        wa[p] = db[p];
                        wb[p] = db[(p + 1) % 3];
                    } else {
                        wa[p] = *reinterpret_cast<const bf16x8*>(wrow0 + p * BB_WPLANE + 64 * kb);
                        wb[p] = *reinterpret_cast<const bf16x8*>(wrow1 + p * BB_WPLANE + 64 * kb);
                    }
                }
                if (BB_ABL != 2) {
                    acc[0] = six(wa, db, acc[0]);
                    if (two) acc[1] = six(wb, db, acc[1]);
                }
            }
#if BB_STAMP
            asm volatile("" :: "v"(acc[0]), "v"(acc[1]));
            VIHMC_BB_STAMP(i, 2)
#endif
            const int m = sub + 16 * h + lr;
            if (m < r1) {
                const unsigned char* hrow = buf + BB_HP + (16 * h + lr) * BB_PITCH;
                float* orow = P.Dout + c * P.o_cs + (int64_t)m * P.ldh;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int col = 16 * (t0 + u) + 4 * lg;
                    if ((u == 1 && !two) || col >= NI4) continue;
                    const bf16x4 h0 = *reinterpret_cast<const bf16x4*>(hrow + 2 * col);
                    const bf16x4 h1 = *reinterpret_cast<const bf16x4*>(hrow + BB_PLANE + 2 * col);
                    const bf16x4 h2 = *reinterpret_cast<const bf16x4*>(hrow + 2 * BB_PLANE + 2 * col);
                    f32x4 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float hv = ((float)h2[r] + (float)h1[r]) + (float)h0[r];
                        o[r] = (col + r < P.n_in) ? acc[u][r] * act_grad_bf(P.act, hv) : 0.f;
                    }
                    if (BB_ABL == 7) asm volatile("" :: "v"(o));
                    else *reinterpret_cast<f32x4*>(orow + col) = o;
                }
            }
        }
    } else {
        // ---------------- dW role: row tiles {2q, 2q+1} x column tiles 0..3 or 4..6 ----------------
        const int v8 = wave - 8;
        const int tn0 = 2 * (v8 >> 1);
        const bool two = tn0 + 1 < 7;
        const int tj0 = (v8 & 1) ? 4 : 0;
        const int ntj = (v8 & 1) ? 3 : 4;
        f32x4 acc[2][4];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[s2][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int tro = bf6::tr_lane_off(lr, lg);
        for (int i = 0; i < nsub; ++i) {
            const int sub = r0 + i * BB_SUB;
            __syncthreads();
            VIHMC_BB_STAMP(i, 0)
            if (i + 1 < nsub) {
                VIHMC_BB_STORE(sub + BB_SUB, (i + 1) & 1)
                if (i + 2 < nsub && BB_ABL != 1) {
                    VIHMC_BB_LOAD(sub + 2 * BB_SUB)
                }
            }
            VIHMC_BB_STAMP(i, 1)
            const unsigned char* buf = smw + (i & 1) * BB_BUF;
            bf16x8 da[2][3];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int p = 0; p < 3; ++p) da[s2][p] = tr_frag(buf + BB_DP + p * BB_PLANE, tro, 16 * (tn0 + (two ? s2 : 0)));
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t >= ntj || 16 * (tj0 + t) >= NI4) break;   // column tiles past n_in (trunk layer 0: 5 inputs)
                bf16x8 hb[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) hb[p] = tr_frag(buf + BB_HP + p * BB_PLANE, tro, 16 * (tj0 + t));
                if (BB_ABL != 3) {
                    acc[0][t] = six(da[0], hb, acc[0][t]);
                    if (two) acc[1][t] = six(da[1], hb, acc[1][t]);
                }
            }
#if BB_STAMP
            asm volatile("" :: "v"(acc[0][0]), "v"(acc[1][2]));
            VIHMC_BB_STAMP(i, 2)
#endif
        }
        float* part = P.part + c * P.part_cs + (int64_t)wg * P.part_stride;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            if (s2 == 1 && !two) continue;
            const int tn = tn0 + s2;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = 16 * (tj0 + t) + lr;
                if (t >= ntj || j >= NI4) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = 16 * tn + 4 * lg + r;
                    if (n < P.n_out) part[(int64_t)n * NI4 + j] = (j < P.n_in) ? acc[s2][t][r] : 0.f;
                }
            }
        }
    }
#undef VIHMC_BB_LOAD
#undef VIHMC_BB_STORE

    // ---- db: per-slot column partials -> LDS [32 rows][25 float4] -> fixed-order sum over rows ----
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smw);
    if (st[0] >= 0 && (st_d & 1)) red[(st[0] >> 8) * 25 + (st[0] & 255)] = dcol;
    __syncthreads();
    if (tid < 25) {
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < BB_SUB; ++r) sacc += red[r * 25 + tid];
        float* part = P.part + c * P.part_cs + (int64_t)wg * P.part_stride + (int64_t)P.n_out * NI4;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (4 * tid + e < P.n_out) part[4 * tid + e] = sacc[e];
    }
#if BB_STAMP
    if (samp && tid == 0) {
        bb_real[sidx][1][0] = __builtin_amdgcn_s_memtime();
        bb_real[sidx][1][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ---------------------------------------------------------------------------------------------------------
// k_bwd_bf2: the same contract with a third role. 16 waves = 8 dX + 4 dW + 4 staging waves (one of each of the
// latter two per SIMD). In k_bwd_bf every thread stages (global load + three-way split + LDS plane stores) before
// its MFMAs, so the split VALU sits in the MFMA waves' instruction streams and the dW role (younger, lower
// priority) reaches its MFMAs ~2,000 cycles into a ~5,000-cycle sub-tile period (stamps, profiles/README.md).
// Here the staging waves alone move sub-tile i+1 into the free LDS buffer (and keep i+2 in flight in registers)
// while the dX and dW waves compute sub-tile i; their VALU issues in the MFMA issue gaps of the other waves on
// the SIMD. dW: wave q owns output row tiles {q, q + 4} (q + 4 < 7) x every column tile.
// ---------------------------------------------------------------------------------------------------------
constexpr int B2_SLOTS = 7;                            // staged float4 per staging thread (<= 800 D + 896 H)

__global__ __launch_bounds__(BB_THREADS, 1) void k_bwd_bf2(BwdArgs args) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smw[];
    int b = blockIdx.x;
    const int per0 = args.C * args.p[0].n_wg;
    const bool second = b >= per0;
    const BwdProb P = second ? args.p[1] : args.p[0];
    if (second) b -= per0;
    const int c = b / P.n_wg;
    const int wg = b - c * P.n_wg;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int NI4 = (P.n_in + 3) & ~3;
    const int hq4 = NI4 >> 2;                          // H float4 per row (<= 28)
    const float* D = P.D + c * P.d_cs;
    const float* H = P.H + c * P.h_cs;
    const int r0 = wg * P.rows_per_wg;
    const int r1 = min(P.M, r0 + P.rows_per_wg);
    const int nsub = r1 > r0 ? (r1 - r0 + BB_SUB - 1) / BB_SUB : 0;
#if BB_STAMP
    const bool samp = second && P.has_dx && (b % 16) == 0 && b / 16 < BBS_WG;
    const int sidx = b / 16;
    if (samp && tid == 0) {
        bb_real[sidx][0][0] = __builtin_amdgcn_s_memtime();
        bb_real[sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif

    // ---- W^T planes (once per workgroup): rows i < n_in, features k < 100 ----
    if (P.has_dx && wave < 12) {
        // by the dX and dW waves only (the staging waves start their first sub-tiles' loads meanwhile), all of a
        // thread's W^T loads (n_in * 25 <= 2800 float4 over 768 threads: <= 4) issued before the first split, so
        // the prologue waits out one HBM latency instead of one per iteration
        const float* WT = P.WT + c * P.wt_cs;
        constexpr int WTH = 768;
        constexpr int WSL = (112 * 25 + WTH - 1) / WTH;
        f32x4 wx[WSL];
#pragma unroll
        for (int v = 0; v < WSL; ++v) {
            const int idx = min(tid + WTH * v, P.n_in * 25 - 1);
            const int r = idx / 25, c4 = idx - r * 25;
            wx[v] = *reinterpret_cast<const f32x4*>(WT + (int64_t)r * P.ldw + 4 * c4);
        }
#pragma unroll
        for (int v = 0; v < WSL; ++v) {
            const int idx = tid + WTH * v;
            if (idx >= P.n_in * 25) break;
            const int r = idx / 25, c4 = idx - r * 25;
            bf16x4 p0, p1, p2;
            split4(wx[v], p0, p1, p2);
            unsigned char* o = smw + BB_W + r * BB_WPITCH + 8 * c4;
            *reinterpret_cast<bf16x4*>(o) = p0;
            *reinterpret_cast<bf16x4*>(o + BB_WPLANE) = p1;
            *reinterpret_cast<bf16x4*>(o + 2 * BB_WPLANE) = p2;
            if (c4 == 24) *reinterpret_cast<f32x4*>(smw + BB_WT + r * 16) = wx[v];
        }
    }

#ifndef B2_PRIO
#define B2_PRIO 1       // static wave priority: 1 = staging waves at 1 (the youngest waves, and the critical path
                        // of the sub-tile period without it: stamps, profiles/r02p_stamps.log); 2 = staging 2, dW 1
#endif
    if (B2_PRIO >= 1 && wave >= 12) __builtin_amdgcn_s_setprio(B2_PRIO);
    if (B2_PRIO == 2 && wave >= 8 && wave < 12) __builtin_amdgcn_s_setprio(1);
    if (wave >= 12) {
        // ---------------- staging role: item idx = t + 256 v -> D (row, c4) for idx < 800, else H ----------------
        const int t = tid - 768;
        const int nd = BB_SUB * 25, ntot = nd + BB_SUB * hq4;
        int st[B2_SLOTS];
#pragma unroll
        for (int v = 0; v < B2_SLOTS; ++v) {
            const int idx = t + 256 * v;
            const bool isd = idx < nd;
            const int e = isd ? idx : idx - nd;
            const int q = isd ? 25 : hq4;
            const int r = e / q, c4 = e - r * q;
            st[v] = idx < ntot ? (r << 8) | c4 : -1;
        }
        // db column: H column NI4 of both buffers is the constant 1 (planes 1, 0, 0), never overwritten by the
        // H stores (columns < NI4), so the dW MFMAs produce part[n][NI4] = sum_m D[m][n] = db[n] exactly
        // (the products D x 1 are exact; fp32 accumulation) in the column tile that already covers it
        if (t < 2 * BB_SUB) {
            unsigned char* o = smw + (t >> 5) * BB_BUF + BB_HP + (t & 31) * BB_PITCH + 2 * NI4;
            *reinterpret_cast<unsigned short*>(o) = 0x3F80;
            *reinterpret_cast<unsigned short*>(o + BB_PLANE) = 0;
            *reinterpret_cast<unsigned short*>(o + 2 * BB_PLANE) = 0;
        }
        // two register sets: sub-tile s is loaded into set s & 1 two sub-tiles before its store, so a load has
        // a whole sub-tile period plus the store phase to land (one set: issued ~500 cycles before its use,
        // the staging waves waited out the HBM latency every period -- profiles/r02_bwd/v2_stamps.log)
        f32x4 pfa[B2_SLOTS], pfb[B2_SLOTS];
        // slots 0-2 are D items, slot 3 D for t < 32, slots 4-6 H: per slot a 32-bit byte offset from the
        // sub-tile's (uniform) row base, so the loads take the SGPR-base form and no 64-bit addresses stay live
        static_assert(3 * 256 < BB_SUB * 25 && BB_SUB * 25 <= 3 * 256 + 32, "D slots");
        auto load = [&](int sub, f32x4 (&pf)[B2_SLOTS]) __attribute__((always_inline)) {
            const int rmax = P.M - 1 - sub;
            const char* db = reinterpret_cast<const char*>(D + (int64_t)sub * P.ldd);
            const char* hb = reinterpret_cast<const char*>(H + (int64_t)sub * P.ldh);
#pragma unroll
            for (int v = 0; v < B2_SLOTS; ++v) {
                const int sv = max(st[v], 0);            // idle slots read column 0 of a valid row: in bounds
                const int r = min(sv >> 8, rmax), c4 = sv & 255;
                const bool isd = v < 3 || (v == 3 && t < 32);
                const unsigned off = 4u * (unsigned)(r * (isd ? P.ldd : P.ldh) + 4 * c4);
                pf[v] = *reinterpret_cast<const f32x4*>((isd ? db : hb) + off);
            }
        };
        auto store = [&](int sub, int buf, const f32x4 (&pf)[B2_SLOTS]) __attribute__((always_inline)) {
#pragma unroll
            for (int v = 0; v < B2_SLOTS; ++v) {
                if (st[v] < 0) continue;
                const int r = st[v] >> 8, c4 = st[v] & 255;
                const f32x4 x = (sub + r < r1) ? pf[v] : f32x4{0.f, 0.f, 0.f, 0.f};
                const bool isd = v < 3 || (v == 3 && t < 32);
                unsigned char* base = smw + buf * BB_BUF + (isd ? BB_DP : BB_HP) + r * BB_PITCH + 8 * c4;
                bf16x4 p0, p1, p2;
                split4(x, p0, p1, p2);
                *reinterpret_cast<bf16x4*>(base) = p0;
                *reinterpret_cast<bf16x4*>(base + BB_PLANE) = p1;
                *reinterpret_cast<bf16x4*>(base + 2 * BB_PLANE) = p2;
                if (isd && c4 == 24) *reinterpret_cast<f32x4*>(smw + buf * BB_BUF + BB_DT + r * 16) = x;
            }
        };
        // Loop unrolled by two so set A is always the newest in flight at the loop head, and every load issued
        // unconditionally (rows past the chunk read its last sub-tile again, an L2 hit): with a conditional load or
        // a set index that alternates at run time, the compiler's merged wait state treated both sets as newest
        // and waited for the sub-tile two ahead (vmcnt(0)) before every store.
        const int slast = r0 + max(nsub - 1, 0) * BB_SUB;
        auto sub_at = [&](int k) { return min(r0 + k * BB_SUB, slast); };
        if (nsub > 0) {
            load(sub_at(0), pfa);
            load(sub_at(1), pfb);
            store(r0, 0, pfa);
            load(sub_at(2), pfa);
        }
        int i = 0;
        for (; i + 1 < nsub; i += 2) {
            __syncthreads();                           // buffer 0 holds sub-tile i, buffer 1 is free
            VIHMC_BB_STAMP(i, 0)
            store(r0 + (i + 1) * BB_SUB, 1, pfb);
            load(sub_at(i + 3), pfb);
            VIHMC_BB_STAMP(i, 1)
            VIHMC_BB_STAMP(i, 2)
            __syncthreads();                           // buffer 1 holds sub-tile i + 1, buffer 0 is free
            VIHMC_BB_STAMP(i + 1, 0)
            if (i + 2 < nsub) store(r0 + (i + 2) * BB_SUB, 0, pfa);
            load(sub_at(i + 4), pfa);
            VIHMC_BB_STAMP(i + 1, 1)
            VIHMC_BB_STAMP(i + 1, 2)
        }
        if (i < nsub) {
            __syncthreads();                           // the last sub-tile (odd count): nothing left to stage
            VIHMC_BB_STAMP(i, 0)
            VIHMC_BB_STAMP(i, 1)
            VIHMC_BB_STAMP(i, 2)
        }
    } else if (wave < 8) {
        // ---------------- dX role: i-tiles {2p, 2p+1} x row half h (as k_bwd_bf) ----------------
        // The role body is instantiated per tile count (TWO) and the epilogue per activation (tanh or the rest),
        // so no exec-masked branch splits the LDS reads from the MFMAs that consume them: hipcc then issues
        // the nine D fragment reads of a sub-tile ahead with counted lgkmcnt waits (with `if (two)` regions
        // between them every read was waited for right before its MFMA).
        const int h = wave & 1, p2 = wave >> 1;
        const int t0 = 2 * __builtin_amdgcn_readfirstlane(p2);
        const unsigned char* wrow0 = smw + BB_W + min(16 * t0 + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const unsigned char* wrow1 = smw + BB_W + min(16 * (t0 + 1) + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const float* wtl = reinterpret_cast<const float*>(smw + BB_WT);
        const int wr0 = min(16 * t0 + lr, P.n_in - 1), wr1 = min(16 * (t0 + 1) + lr, P.n_in - 1);
#ifndef B2_HGLOBAL
#define B2_HGLOBAL 0    // 1: the dX epilogue's h as fp32 global loads (L2) issued at the sub-tile head, instead of three
                        // LDS plane reads + reconstruction (same values: the split is exact)
#endif
#ifndef B2_DEFER
#define B2_DEFER 0      // 1: the dX epilogue of sub-tile i runs after sub-tile i+1's MFMAs are issued (branch-free, in
                        // their basic block, so its VALU fills their issue gaps); 0: right after its own MFMAs
#endif
        // Dout through a buffer resource: rows past r1 (another workgroup's) and columns past NI4 get an out-of-range
        // offset instead of a branch around the store
        const __amdgpu_buffer_rsrc_t drs =
            bf6::make_rsrc(P.Dout + c * P.o_cs, (uint32_t)((int64_t)P.M * P.ldh * 4));
        auto dx_run = [&](auto two_c, auto tanh_c) __attribute__((always_inline)) {
            constexpr bool TWO = decltype(two_c)::value;
            constexpr bool TANH = decltype(tanh_c)::value;
            constexpr int NU = TWO ? 2 : 1;
            bf16x8 wra[3][3];
            float wta = 0.f, wtb = 0.f;
            // the pending epilogue: accumulators, the H planes of its rows (read before the buffer is reused) and the
            // store offsets (OOB: nothing pending / not this workgroup's row / past NI4)
            f32x4 accp[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            bf16x4 hq[2][3] = {};
            f32x4 hgp[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            uint32_t offp[2] = {bf6::OOB, bf6::OOB};
            auto epilogue = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int col = 16 * (t0 + u) + 4 * lg;
                    f32x4 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float hv = B2_HGLOBAL ? hgp[u][r]
                                                    : ((float)hq[u][2][r] + (float)hq[u][1][r]) + (float)hq[u][0][r];
                        const float gd = TANH ? 1.f - hv * hv : act_grad_bf(P.act, hv);
                        o[r] = (col + r < P.n_in) ? accp[u][r] * gd : 0.f;
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bf6::u32x4, o), drs, offp[u], 0, 0);
                }
            };
            for (int i = 0; i < nsub; ++i) {
                const int sub = r0 + i * BB_SUB;
                __syncthreads();
                VIHMC_BB_STAMP(i, 0)
                if (!P.has_dx) continue;
#if B2_HGLOBAL
                // act'(h) operands as fp32 straight from H (the rows the staging waves just read: L2 hits), issued
                // before this sub-tile's MFMAs: no plane reads / reconstruction VALU in the epilogue
                f32x4 hgv[2];
                {
                    const int mm = min(sub + 16 * h + lr, P.M - 1);
#pragma unroll
                    for (int u = 0; u < NU; ++u) {
                        const int col = min(16 * (t0 + u) + 4 * lg, NI4 - 4);
                        hgv[u] = *reinterpret_cast<const f32x4*>(H + (int64_t)mm * P.ldh + col);
                    }
                }
#endif
                if (i == 0) {
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            wra[kb][p] = *reinterpret_cast<const bf16x8*>(wrow0 + p * BB_WPLANE + 64 * kb);
                    wta = wtl[wr0 * 4 + lg];
                    if (TWO) wtb = wtl[wr1 * 4 + lg];
                }
                const unsigned char* buf = smw + (i & 1) * BB_BUF;
                const unsigned char* drow = buf + BB_DP + (16 * h + lr) * BB_PITCH + 16 * lg;
                bf16x8 db[3][3];
#pragma unroll
                for (int kb = 0; kb < 3; ++kb)
#pragma unroll
                    for (int p = 0; p < 3; ++p) db[kb][p] = *reinterpret_cast<const bf16x8*>(drow + p * BB_PLANE + 64 * kb);
                const float dtl = reinterpret_cast<const float*>(buf + BB_DT)[(16 * h + lr) * 4 + lg];
                f32x4 acc[2];
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wta, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                acc[1] = TWO ? __builtin_amdgcn_mfma_f32_16x16x4f32(wtb, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) {
                    acc[0] = six(wra[kb], db[kb], acc[0]);
                    if (TWO) {
                        bf16x8 wb[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p) wb[p] = *reinterpret_cast<const bf16x8*>(wrow1 + p * BB_WPLANE + 64 * kb);
                        acc[1] = six(wb, db[kb], acc[1]);
                    }
                }
                if (B2_DEFER) epilogue();                  // sub-tile i-1 (nothing stored when i = 0)
#if BB_STAMP
                asm volatile("" :: "v"(acc[0]), "v"(acc[1]));
                VIHMC_BB_STAMP(i, 1)
#endif
                const int m = sub + 16 * h + lr;
                const unsigned char* hrow = buf + BB_HP + (16 * h + lr) * BB_PITCH;
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int col = 16 * (t0 + u) + 4 * lg;
#if B2_HGLOBAL
                    hgp[u] = hgv[u];
#else
#pragma unroll
                    for (int p = 0; p < 3; ++p) hq[u][p] = *reinterpret_cast<const bf16x4*>(hrow + p * BB_PLANE + 2 * col);
#endif
                    offp[u] = (m < r1 && col < NI4) ? (uint32_t)(m * P.ldh + col) * 4u : bf6::OOB;
                    accp[u] = acc[u];
                }
                if (!B2_DEFER) epilogue();
                VIHMC_BB_STAMP(i, 2)
            }
            if (B2_DEFER && P.has_dx && nsub > 0) epilogue();
        };
        const bool tanh_act = P.act == ACT_TANH;
        if (t0 + 1 < 7) {
            if (tanh_act) dx_run(std::true_type{}, std::true_type{});
            else dx_run(std::true_type{}, std::false_type{});
        } else {
            if (tanh_act) dx_run(std::false_type{}, std::true_type{});
            else dx_run(std::false_type{}, std::false_type{});
        }
    } else {
        // ---------------- dW role: two row tiles per wave, the second over a column range ----------------
        // Waves w, w + 4, w + 8, w + 12 share a SIMD. The dX waves of SIMD groups 0 and 1 (waves 0/4, 1/5) carry
        // four tile-jobs of 20 MFMA-equivalents, those of groups 2 and 3 three; a dW (row, column) tile-job is 6
        // MFMAs. Groups 2 and 3 (waves 10, 11) take row tiles {0, 1} and {2, 3} whole (14 jobs), groups 0 and 1
        // (waves 8, 9) row tile 4 or 5 whole plus row tile 6 (rows 96..99 of n_out) over columns 0..3 or 4..6:
        // at most 146 MFMA-equivalents per SIMD (row tiles {q, q + 4} per wave: 164 on one SIMD).
        const int g = __builtin_amdgcn_readfirstlane(wave - 8);
        const int rta = g == 2 ? 0 : g == 3 ? 2 : 4 + g;               // first row tile, all column tiles
        const int rtb = g == 2 ? 1 : g == 3 ? 3 : 6;                   // second row tile over [cb0, cb1)
        const int cb0 = g == 1 ? 4 : 0, cb1 = g == 0 ? 4 : 7;
        const int ntj = __builtin_amdgcn_readfirstlane((NI4 + 16) >> 4);   // through the db column NI4
        f32x4 acc[2][7];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int t = 0; t < 7; ++t) acc[s2][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int tro = bf6::tr_lane_off(lr, lg);
        // instantiated for 7 column tiles (every layer but the trunk input layer) with the tile loop's reads
        // unconditional, so the next tile's H reads stay in flight under this tile's MFMAs (a run-time tile count
        // made them conditional, and hipcc then waited lgkmcnt(0) -- for the prefetch too -- before each tile)
        auto dw_run = [&](auto nt_c) __attribute__((always_inline)) {
            constexpr int NT = decltype(nt_c)::value;                  // 0: ntj at run time
            const int nt = NT ? NT : ntj;
            for (int i = 0; i < nsub; ++i) {
                __syncthreads();
                VIHMC_BB_STAMP(i, 0)
                const unsigned char* buf = smw + (i & 1) * BB_BUF;
                bf16x8 da[2][3], hb[2][3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    da[0][p] = tr_frag(buf + BB_DP + p * BB_PLANE, tro, 16 * rta);
                    da[1][p] = tr_frag(buf + BB_DP + p * BB_PLANE, tro, 16 * rtb);
                    hb[0][p] = tr_frag(buf + BB_HP + p * BB_PLANE, tro, 0);
                }
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= nt) break;                    // wave-uniform (NT = 0 only)
                    if (t + 1 < nt) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) hb[(t + 1) & 1][p] = tr_frag(buf + BB_HP + p * BB_PLANE, tro, 16 * (t + 1));
                    }
                    acc[0][t] = six(da[0], hb[t & 1], acc[0][t]);
                    if (t >= cb0 && t < cb1) acc[1][t] = six(da[1], hb[t & 1], acc[1][t]);
                }
#if BB_STAMP
                asm volatile("" :: "v"(acc[0][0]), "v"(acc[1][6]));
                VIHMC_BB_STAMP(i, 1)
                VIHMC_BB_STAMP(i, 2)
#endif
            }
        };
        if (ntj == 7) dw_run(std::integral_constant<int, 7>{});
        else dw_run(std::integral_constant<int, 0>{});
        float* part = P.part + c * P.part_cs + (int64_t)wg * P.part_stride;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int tn = s2 == 0 ? rta : rtb;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                const int j = 16 * t + lr;
                if (t >= ntj || j > NI4 || (s2 == 1 && (t < cb0 || t >= cb1))) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = 16 * tn + 4 * lg + r;
                    if (n >= P.n_out) continue;
                    if (j == NI4) part[(int64_t)P.n_out * NI4 + n] = acc[s2][t][r];     // db
                    else part[(int64_t)n * NI4 + j] = (j < P.n_in) ? acc[s2][t][r] : 0.f;
                }
            }
        }
    }
#if BB_STAMP
    if (samp && tid == 0) {
        bb_real[sidx][1][0] = __builtin_amdgcn_s_memtime();
        bb_real[sidx][1][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

bool bwd_bf_ok(const BwdArgs& a) {
    for (int i = 0; i < a.nprob; ++i) {
        const BwdProb& p = a.p[i];
        if (p.n_out != 100 || p.n_in > 112 || (p.has_dx && p.n_in != 100)) return false;
        if ((p.ldd & 3) || (p.ldh & 3) || (p.has_dx && (p.ldw & 3))) return false;
    }
    return true;
}

#if BB_STAMP
extern "C" int vihmc_debug_bb_stamps(void* stamps, size_t stamp_bytes, void* real, size_t real_bytes) {
    if (stamp_bytes != sizeof(bb_stamps) || real_bytes != sizeof(bb_real)) return -1;
    hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(bb_stamps), stamp_bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(real, HIP_SYMBOL(bb_real), real_bytes, 0, hipMemcpyDeviceToHost);
    return (int)e;
}
#endif

// layer-backward kernel: VIHMC_BWD_V2 = 0 k_bwd_bf, otherwise (default) k_bwd_bf2 (read once per process)
static int bwd_v2() {
    static const int v = [] {
        const char* e = std::getenv("VIHMC_BWD_V2");
        return e ? std::atoi(e) : 2;
    }();
    return v;
}

hipError_t launch_bwd_bf(const BwdArgs& a, hipStream_t s) {
    if (!bwd_bf_ok(a)) return hipErrorInvalidValue;
    const int blocks = a.C * a.p[0].n_wg + (a.nprob > 1 ? a.C * a.p[1].n_wg : 0);
    // k_bwd_bf2 keeps its db column at H column NI4 inside the last column tile: NI4 < 112
    bool v2 = bwd_v2() != 0;
    for (int i = 0; i < a.nprob; ++i) v2 = v2 && ((a.p[i].n_in + 3) & ~3) < 112;
    if (v2) hipLaunchKernelGGL(k_bwd_bf2, dim3(blocks), dim3(BB_THREADS), BB_LDS, s, a);
    else hipLaunchKernelGGL(k_bwd_bf, dim3(blocks), dim3(BB_THREADS), BB_LDS, s, a);
    return hipGetLastError();
}

// timing-only / instrumentation switches this translation unit was built with (0 = product build)
int diag_switches_bwd_bf() { return BB_ABL | (BB_STAMP << 8); }

}  // namespace vihmc
