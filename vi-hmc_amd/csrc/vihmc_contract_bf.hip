// Side-A contraction (branch x trunk S, Gaussian NLL, G, dZ_trunk) with fp32 products emulated on the
// bf16 MFMA: the "bf16x6" form of k_contract_ws (vihmc_contract.hip), same ContractProb, same outputs.
//
// Replaces torch.einsum("...i,...i->...", xb, xtr) + b (Operator_network/VI_HMC/my_make_func.py:79-82),
// GaussianNLLLoss / regression ll (main_VI_HMC_burgers.py:157-163) and their autograd backward.
//
// Every fp32 operand x is split exactly into three bf16 planes x = x0 + x1 + x2 (x0 = bf16(x),
// x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)); a.b keeps the six products of order <= 2
// (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0, small first) accumulated in fp32: the dropped terms are
// < 2^-24 |a||b|, so the result is as accurate as the sequential fp32 dot product
// (profiles/bf16x6_precision.py). Six 16x16x32 bf16 MFMAs (16 cycles each) replace eight 16x16x4 f32
// MFMAs (32 cycles each) per 32-long k-block: 2.7x fewer matrix-core cycles. The 4-long k tail
// (features 96..99) is one exact 16x16x4 f32 MFMA.
//
// Workgroup = 8 S waves + 8 D waves (4 waves per SIMD, 1 workgroup per CU, <= 128 VGPRs a wave) for
// 128 owner (trunk) rows, 16 per wave pair; the branch rows stream through LDS in 32-row chunks:
//   Q image  (3 rotating buffers): the chunk's three bf16 planes, row-major [32 q][112 j], 224-B rows,
//            plus the fp32 tail [32 q][4]. S waves read it by rows (ds_read_b128, the A operand of
//            S = Q Own^T); D waves read it by columns (ds_read_b64_tr_b16, the B operand of G^T Q).
//            224 B = 32 * 7 (odd multiple of 32 B): the transposed reads of 8 consecutive rows are
//            bank-conflict free.
//   G image  (2 buffers): each S wave's G (fp32, its accumulator registers) for its D partner, lane-
//            linear. The D role's k order is chosen so that its A operand IS that register layout:
//            lane (lr, lg) element jj <-> branch row 4lg + jj (jj < 4) or 16 + 4lg + jj - 4 (jj >= 4),
//            and the two transposed reads fetch exactly those rows.
//   S wave w: 16 owner rows, their three planes in registers (36 VGPRs) as the B operand; per chunk two
//             16-row S tiles, G = gscale (S + b0 - y), likelihood sums, G^T stores for side B.
//   D wave w: one chunk behind: splits G, dOwn[16 rows][112] += G^T Q over the chunk's 32 rows.
// Likelihood sums: 2 doubles per S wave at stats[(qc * o_tiles + og) * 8 + w].
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"

namespace vihmc {

namespace {
using bf6::f32x4;
using bf6::bf16x8;
using bf6::bf16x4;
using bf6::lds_bf16x4;
using bf6::split4;
using bf6::cat8;
using bf6::six;
typedef bf6::u32x4 u32x4_c;
constexpr uint32_t OOB_C = bf6::OOB;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_c(const void* p, uint32_t bytes) {
    return bf6::make_rsrc(p, bytes);
}

constexpr int CB_QC = CONTRACT_SPLIT_ROWS;         // branch rows per chunk (32)
constexpr int CB_PITCH = bf6::PITCH;               // bytes per bf16 image row (112 features)
constexpr int CB_PLANE = CB_QC * CB_PITCH;         // 7168
constexpr int CB_TAIL = 3 * CB_PLANE;              // fp32 [32][4] tail image offset
constexpr int CB_BLOCK = CONTRACT_SPLIT_BLOCK;     // 22528: 3 planes + tail, padded to 22 KB
static_assert(CB_TAIL + CB_QC * 16 <= CB_BLOCK && CB_BLOCK % 1024 == 0, "split block layout");
constexpr int CB_QIMG = CB_BLOCK;                  // bytes per Q buffer (one pre-split block)
constexpr int CBA_DW = 8;                         // D waves (DMA stride)
constexpr int CBA_THREADS = 1024;
// G image per buffer: 8 S waves x 64 lanes x 2 f32x4 (the S waves' accumulators as they stand; handing G over
// pre-split measured no change, 412 vs 411 us). Sum G: per chunk an fp32 partial of the lane's 8 terms, then fp64
// (as sum r^2); its rounding, ~1e-6 of the b gradient, is below the reference's own fp32 sum over N x P terms.
constexpr int CB_GIMG = 8 * 2 * 64 * 16;
constexpr int CB_NQBUF = 3;
constexpr int CB_LDS = CB_NQBUF * CB_QIMG + 2 * CB_GIMG;  // 98816
constexpr int CB_GLDS = CB_BLOCK / 1024;           // 22 wave-wide 16-B-per-lane DMA copies per block

}  // namespace

#if CB_STAMP
// every 64th workgroup: per wave and chunk, s_memtime at the barrier exit [0] and when the chunk's results
// exist [1]; per workgroup s_memtime / s_memrealtime (100 MHz) at start and end (scripts/diag/stamps_side_a.py)
constexpr int CBS_WG = 24, CBS_CH = 40;
__device__ unsigned long long cb_stamps[CBS_WG][16][CBS_CH][3];
__device__ unsigned long long cb_real[CBS_WG][2][2];
#define VIHMC_CB_STAMP(I, K)                                                                                  \
    if (samp && lane == 0 && (I) < CBS_CH) cb_stamps[sidx][wave][(I)][(K)] = __builtin_amdgcn_s_memtime();
#else
#define VIHMC_CB_STAMP(I, K)
#endif

__global__ __launch_bounds__(CBA_THREADS, 1) void k_contract_bf(ContractProb P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smc[];
    int b = blockIdx.x;
#if CB_STAMP
    const bool samp = (blockIdx.x % 64) == 0 && blockIdx.x / 64 < CBS_WG;
    const int sidx = blockIdx.x / 64;
    if (samp && threadIdx.x == 0) {
        cb_real[sidx][0][0] = __builtin_amdgcn_s_memtime();
        cb_real[sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const int per_chain = P.o_tiles * P.q_chunks;
    const int c = b / per_chain;
    if (P.sel && !chain_bit(P.bits, c)) return;          // fit guard: a chain that runs the Gram form
    b -= c * per_chain;
    const int qc = b / P.o_tiles;
    const int og = b - qc * P.o_tiles;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int w = wave & 7;                            // S wave w and D wave w share owner rows o0 .. o0+15
    const int o0 = og * CONTRACT_OWN_PER_WG + w * 16;
    const int q_lo = qc * P.q_per_chunk;
    const int q_hi = min(q_lo + P.q_per_chunk, P.Mq);
    const int nchunks = q_hi > q_lo ? (q_hi - q_lo + CB_QC - 1) / CB_QC : 0;

    // Q chunks: blocks of the pre-split image (vihmc_split_blocks), copied global -> LDS by the D waves
    // with wave-wide DMA (global_load_lds_dwordx4: 1 KB per instruction, no VGPRs, no VALU), issued by asm:
    // with the builtin, hipcc waited vmcnt(0) -- for the copies just issued -- before the D waves' first LDS
    // read of every chunk; the asm copies are retired by the wave's own vmcnt(0) before the next barrier.
    // r03: side A 0.366 vs 0.385 ms at 16 chains, neutral at one chain (profiles/r03_side_a/asm_dma_*).
    // Moving the copies to the S waves (4 buffers, two chunks ahead) and a one-role kernel with G kept in
    // registers (8 waves, both products in every wave) were bitwise equal and slower: profiles/r03_side_a/.
    const unsigned char* qblk = P.qimg + c * P.qimg_cs + (int64_t)(q_lo / CB_QC) * CB_BLOCK;
#define VIHMC_CB_BAR() __syncthreads();
#define VIHMC_CB_GLDS(CI, BUF)                                                                              \
    for (int k = wave - 8; k < CB_GLDS; k += CBA_DW)                                                        \
        bf6::glds16_asm(qblk + (int64_t)(CI) * CB_BLOCK + k * 1024 + lane * 16, smc + (BUF) * CB_QIMG + k * 1024);
    if (wave < 8) {
        // ---------------- S role ----------------
        const float* Own = P.Own + c * P.own_cs;
        const float* Yc = P.Y + c * P.y_cs;
        const float b0 = P.b0[c * P.b0_cs];
        bf16x8 ob[3][3];        // [kb][plane]: Own[o0 + lr][32kb + 8lg + j]
        float otl;              // Own[o0 + lr][96 + lg]
        {
            const float* orow = Own + (int64_t)min(o0 + lr, P.Mo - 1) * P.ldown;
#pragma unroll
            for (int kb = 0; kb < 3; ++kb) {
                const f32x4 x0 = *reinterpret_cast<const f32x4*>(orow + 32 * kb + 8 * lg);
                const f32x4 x1 = *reinterpret_cast<const f32x4*>(orow + 32 * kb + 8 * lg + 4);
                bf16x4 a0, a1, a2, c0, c1, c2;
                split4(x0, a0, a1, a2);
                split4(x1, c0, c1, c2);
                ob[kb][0] = cat8(a0, c0);
                ob[kb][1] = cat8(a1, c1);
                ob[kb][2] = cat8(a2, c2);
            }
            otl = orow[96 + lg];
        }
        double ssq = 0.0, gsum = 0.0;
        // targets and G^T through buffer resources: 32-bit offsets, rows past the end read 0 and owner
        // rows past Mo are dropped by the hardware range check (no exec-mask branches per element)
        const __amdgpu_buffer_rsrc_t yrs = make_rsrc_c(Yc, (uint32_t)((int64_t)P.Mq * P.ldy * 4));
        // G^T exchange buffer, 16-row blocked: element (o, q) at ((q / 16) * ldg + o) * 16 + q % 16 (ldg = Mo rows
        // per block). A 16-row S tile of one wave's 16 owner rows is 16 x 64 B = 1 KB contiguous, and lane (lr, lg)
        // holds its 16-B piece (q = 4lg .. 4lg+3 of owner row o0 + lr) as the accumulator quad: one whole-line store
        // per tile straight from the accumulators (no lane exchange)
        const __amdgpu_buffer_rsrc_t grs = make_rsrc_c(
            P.gout ? P.gout + c * P.gout_cs : P.Y,
            P.gout ? (uint32_t)((int64_t)((P.Mq + CB_QC - 1) / CB_QC) * P.ldg * CB_QC * 4) : 0u);
        const int oo = o0 + lr;
        const bool ovalid = oo < P.Mo;
        // every owner row of this wave exists (all but the last owner tile): with a whole chunk, no masking
        const bool wave_valid = o0 + 16 <= P.Mo;
        const uint32_t yoff = (uint32_t)((4 * lg) * P.ldy + min(oo, P.Mo - 1)) * 4u;
        const uint32_t g_off = ovalid ? (uint32_t)(((q_lo / 16) * P.ldg + oo) * 16 + 4 * lg) * 4u : OOB_C;
        const uint32_t gblk = (uint32_t)P.ldg * 64u;            // bytes per 16-row block
        const uint32_t ystep = (uint32_t)P.ldy * 4u;
        // targets [sub][r] one chunk ahead in two register sets used alternately (the loop is unrolled by
        // two), so no register copy forces a wait on the newest loads and the G^T stores
        float ya[2][4], yb[2][4];
#define VIHMC_CB_YLOAD(YN, CI)                                                                           \
        _Pragma("unroll") for (int sub = 0; sub < 2; ++sub)                                              \
            _Pragma("unroll") for (int r = 0; r < 4; ++r)                                                \
                YN[sub][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(              \
                    yrs, yoff, (uint32_t)(q_lo + (CI) * CB_QC + 16 * sub + r) * ystep, 0));
        VIHMC_CB_YLOAD(ya, 0)
        // chunk i < nchunks, called with no condition around its loads or stores (below): hipcc's wait counts
        // stay exact (a conditional chunk body or a store count that depends on the path made it wait vmcnt(0)
        // -- for this wave's own G^T stores -- at the head of every other chunk)
        auto s_chunk = [&](int i, float (&yv)[2][4], float (&yn)[2][4]) __attribute__((always_inline)) {
            VIHMC_CB_BAR()
            VIHMC_CB_STAMP(i, 0)
            {
                const int q0 = q_lo + i * CB_QC;
                const bool nomask = q0 + CB_QC <= q_hi && wave_valid && !P.masked;   // wave-uniform
                const unsigned char* img = smc + (i % CB_NQBUF) * CB_QIMG;
                VIHMC_CB_YLOAD(yn, min(i + 1, nchunks - 1))
                unsigned char* gimg = smc + CB_NQBUF * CB_QIMG + (i & 1) * CB_GIMG + w * (CB_GIMG / 8);
                float ps = 0.f, gp = 0.f;
                f32x4 rv[2];
#pragma unroll
                for (int sub = 0; sub < 2; ++sub) {
                    const unsigned char* row = img + (16 * sub + lr) * CB_PITCH + 16 * lg;
                    const float qt = reinterpret_cast<const float*>(img + CB_TAIL)[(16 * sub + lr) * 4 + lg];
                    // the exact f32 tail (features 96..99) on top of the output bias b0 seeds the accumulator
                    f32x4 sacc = __builtin_amdgcn_mfma_f32_16x16x4f32(qt, otl, f32x4{b0, b0, b0, b0}, 0, 0, 0);
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb) {
                        bf16x8 qa[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            qa[p] = *reinterpret_cast<const bf16x8*>(row + p * CB_PLANE + 64 * kb);
                        sacc = six(qa, ob[kb], sacc);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) rv[sub][r] = sacc[r] - yv[sub][r];
                }
                if (!nomask) {
                    // a partial last chunk (branch rows past q_hi: zero image rows, so S = b0) or owner rows past Mo
                    // (the last owner tile): those residuals are not the workgroup's; a masked plan's NaN targets
                    // (pairs outside an item's trunk subset) count as residual 0
#pragma unroll
                    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            rv[sub][r] = (ovalid && q0 + 16 * sub + 4 * lg + r < q_hi &&
                                          (!P.masked || yv[sub][r] == yv[sub][r])) ? rv[sub][r] : 0.f;
                }
#pragma unroll
                for (int sub = 0; sub < 2; ++sub) {
                    f32x4 g;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        g[r] = P.gscale * rv[sub][r];
                        ps = fmaf(rv[sub][r], rv[sub][r], ps);
                        gp += g[r];
                    }
                    reinterpret_cast<f32x4*>(gimg)[sub * 64 + lane] = g;
#if CB_STAMP
                    if (sub == 0) {
                        asm volatile("" :: "v"(g));
                        VIHMC_CB_STAMP(i, 2)
                    }
#endif
                    // whole lines in a partial chunk too: its q >= q_hi elements are G = 0 (rv zeroed above) and
                    // land in the padding of the blocked layout (q_hi < Mq only at chunk boundaries, qperA being a
                    // multiple of 32), which no workgroup owns
                    if (P.gout)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c, g), grs,
                                                               g_off + (uint32_t)(2 * i + sub) * gblk, 0, 0);
                }
                // sum r^2 (no cancellation): per-chunk fp32 partial of 8 terms per lane, then fp64
                ssq += (double)ps;
                gsum += (double)gp;
#if CB_STAMP
                asm volatile("" :: "v"(ps));
                VIHMC_CB_STAMP(i, 1)
#endif
            }
        };
        int i = 0;
        for (; i + 1 < nchunks; i += 2) {
            s_chunk(i, ya, yb);
            s_chunk(i + 1, yb, ya);
        }
        if (i < nchunks) s_chunk(i, ya, yb);
        VIHMC_CB_BAR()                                 // the D role's last barrier (it runs one chunk behind)
        if (P.with_stats) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                ssq += __shfl_xor(ssq, o, 64);
                gsum += __shfl_xor(gsum, o, 64);
            }
            if (lane == 0) {
                double* st = P.stats + c * P.stats_cs + 2 * (int64_t)((qc * P.o_tiles + og) * 8 + w);
                st[0] = ssq;
                st[1] = gsum;
            }
        }
        return;
    }

    // ---------------- D role ----------------
    if (nchunks > 0) {
        VIHMC_CB_GLDS(0, 0)
    }
    f32x4 dacc[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) dacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int tro = bf6::tr_lane_off(lr, lg);
    for (int i = 0; i <= nchunks; ++i) {
        bf6::wait_vmcnt0();                            // this wave's copies of chunk i (invisible to hipcc) landed
        VIHMC_CB_BAR()
        VIHMC_CB_STAMP(i, 0)
        // chunk i+1 -> buffer (i+1)%3 (last read by this role in iteration i-1, by S in i-2); the copies
        // land while this iteration computes and are drained by the next barrier (vmcnt(0)).
        if (i + 1 < nchunks) {
            VIHMC_CB_GLDS(i + 1, (i + 1) % CB_NQBUF)
        }
#if CB_STAMP == 2
        VIHMC_CB_STAMP(i, 2)                           // D waves: mid = the copies issued
#endif
        if (i >= 1) {
            const unsigned char* img = smc + ((i - 1) % CB_NQBUF) * CB_QIMG;
            const unsigned char* gimg = smc + CB_NQBUF * CB_QIMG + ((i - 1) & 1) * CB_GIMG + w * (CB_GIMG / 8);
            bf16x8 ga[3];
            {
                const f32x4* gsrc = reinterpret_cast<const f32x4*>(gimg);
                bf16x4 l0, l1, l2, h0, h1, h2;
                split4(gsrc[lane], l0, l1, l2);          // sub 0
                split4(gsrc[64 + lane], h0, h1, h2);     // sub 1
                ga[0] = cat8(l0, h0);
                ga[1] = cat8(l1, h1);
                ga[2] = cat8(l2, h2);
            }
#if CB_STAMP
            asm volatile("" :: "v"(ga[0]), "v"(ga[2]));
#if CB_STAMP == 1
            VIHMC_CB_STAMP(i, 2)
#endif
#endif
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                bf16x8 qb[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) qb[p] = bf6::tr_frag(img + p * CB_PLANE, tro, 16 * t);
                dacc[t] = six(ga, qb, dacc[t]);
            }
#if CB_STAMP
            asm volatile("" :: "v"(dacc[0]), "v"(dacc[6]));
            VIHMC_CB_STAMP(i, 1)
#endif
        }
    }
    float* out = P.out + c * P.out_cs + (int64_t)qc * P.out_chunk_stride;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        const int j = 16 * t + lr;
        if (j >= P.ldout) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oo = o0 + 4 * lg + r;
            if (oo < P.Mo) out[(int64_t)oo * P.ldout + j] = (j < 100) ? dacc[t][r] : 0.f;
        }
    }
#if CB_STAMP
    if (samp && wave == 8 && lane == 0) {
        cb_real[sidx][1][0] = __builtin_amdgcn_s_memtime();
        cb_real[sidx][1][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
#undef VIHMC_CB_GLDS
#undef VIHMC_CB_YLOAD
}

// Split rows [rows][ld] (width 100) of every chain into the blocked bf16x6 image: block b holds rows
// 32b .. 32b+31 as planes [3][32][112] bf16 (features 100..111 and rows past `rows` zero) followed by the
// fp32 tail [32][4] (features 96..99), CONTRACT_SPLIT_BLOCK bytes per block.
// 8 features per lane, 16-B stores, one pass of 448 lanes per block (4 per lane over 256 lanes: 24.4 vs 23.4 us)
constexpr int CBS_THREADS = CB_QC * 14;     // 14 groups of 8 features per 112-feature image row
__global__ __launch_bounds__(CBS_THREADS) void k_split_blocks(const float* src, int64_t src_cs, int ld, int rows,
                                                             unsigned char* dst, int64_t dst_cs, int nblk) {
    const int c = blockIdx.x / nblk, blk = blockIdx.x - c * nblk;
    const int r = threadIdx.x / 14, g = threadIdx.x - r * 14, row = blk * CB_QC + r;
    const float* sr = src + c * src_cs + (int64_t)row * ld + 8 * g;
    unsigned char* d = dst + c * dst_cs + (int64_t)blk * CB_BLOCK;
    f32x4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = x0;
    if (row < rows && g < 13) {                    // features 8g .. 8g+7; group 12 holds 96..99 only
        x0 = *reinterpret_cast<const f32x4*>(sr);
        if (g < 12) x1 = *reinterpret_cast<const f32x4*>(sr + 4);
    }
    bf16x4 a0, a1, a2, b0, b1, b2;
    split4(x0, a0, a1, a2);
    split4(x1, b0, b1, b2);
    unsigned char* o = d + r * CB_PITCH + 16 * g;
    struct alignas(16) bf16x4x2 { bf16x4 lo, hi; };
    *reinterpret_cast<bf16x4x2*>(o) = bf16x4x2{a0, b0};
    *reinterpret_cast<bf16x4x2*>(o + CB_PLANE) = bf16x4x2{a1, b1};
    *reinterpret_cast<bf16x4x2*>(o + 2 * CB_PLANE) = bf16x4x2{a2, b2};
    if (g == 12) *reinterpret_cast<f32x4*>(d + CB_TAIL + r * 16) = x0;
}

hipError_t launch_split_blocks(const float* src, int64_t src_cs, int ld, int rows, unsigned char* dst,
                               int64_t dst_cs, int C, hipStream_t s) {
    const int nblk = (rows + CB_QC - 1) / CB_QC;
    hipLaunchKernelGGL(k_split_blocks, dim3(C * nblk), dim3(CBS_THREADS), 0, s, src, src_cs, ld, rows, dst, dst_cs,
                       nblk);
    return hipGetLastError();
}


// =============================================================================================
// Side B (load-G), bf16x6: dOwn[o][j] += sum_q G[q][o] Q[q][j] with G read from side A's chunk-blocked
// G^T (P.Y) and Q = the trunk outputs pre-split into blocks. No S role: all 8 waves are alike,
// 32 owner (branch) rows each (256 per workgroup); per 32-row chunk each wave loads its G (one chunk
// ahead, two register sets), splits it into the A operand (same k order as the side-A D role) and runs
// 7 column tiles x 2 row tiles x 6 products against transposed reads of the shared chunk image.
// =============================================================================================
constexpr int CBB_OWN = 256;        // owner rows per workgroup (8 waves x 32, or 16 x 16)
// 16 waves of 16 owner rows (4 per SIMD, <= 128 VGPRs; 8 waves of 32 rows at 2 per SIMD: 240 vs 226 us)
constexpr int CBB_NS = 1;                               // 16-row owner tiles per wave
constexpr int CBB_WAVES = CBB_OWN / (16 * CBB_NS);
constexpr int CBB_THREADS = 64 * CBB_WAVES;

__global__ __launch_bounds__(CBB_THREADS, 1) void k_contract_bf_b(ContractProb P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smb[];
    int b = blockIdx.x;
    if (P.xcd_group) {
        const int xcd = b & 7, k = b >> 3;
        const int gx = k / P.o_tiles, og = k - gx * P.o_tiles;
        b = (gx * 8 + xcd) * P.o_tiles + og;
    }
    const int per_chain = P.o_tiles * P.q_chunks;
    const int c = b / per_chain;
    if (P.sel && !chain_bit(P.bits, c)) return;          // fit guard: a chain that runs the Gram form
    b -= c * per_chain;
    const int qc = b / P.o_tiles;
    const int og = b - qc * P.o_tiles;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int o0 = og * CBB_OWN + wave * 16 * CBB_NS;
    const int q_lo = qc * P.q_per_chunk;
    const int q_hi = min(q_lo + P.q_per_chunk, P.Mq);
    const int nchunks = q_hi > q_lo ? (q_hi - q_lo + CB_QC - 1) / CB_QC : 0;
    const unsigned char* qblk = P.qimg + c * P.qimg_cs + (int64_t)(q_lo / CB_QC) * CB_BLOCK;
    // image by asm LDS-DMA (with the builtin, hipcc waited vmcnt(0) before the LDS reads of every chunk: 266 -> 237 us)
#define VIHMC_CBB_GLDS(CI, BUF)                                                                             \
    for (int k = wave; k < CB_GLDS; k += CBB_WAVES)                                                         \
        bf6::glds16_asm(qblk + (int64_t)(CI) * CB_BLOCK + k * 1024 + lane * 16, smb + (BUF) * CB_QIMG + k * 1024);

    // G[q][o] for this lane: rows 4lg + jj (jj < 4) and 16 + 4lg + jj - 4 of the chunk, column o0+16s+lr;
    // buffer loads with the whole offset in the range-checked VGPR: rows past Mq read 0, rows past q_hi
    // (another workgroup's range, only in a partial last chunk) are sent out of range
    const float* Gc = P.Y + c * P.y_cs;
    // 16-row blocked G^T (see k_contract_bf): element (q, o) at ((o / 16) * ldy + q) * 16 + o % 16 with ldy = Mq
    // rows per block; this wave's 16 owner rows are one block (64 B per trunk row q)
    static_assert(CBB_NS == 1, "one 16-row owner block per wave");
    const __amdgpu_buffer_rsrc_t grs =
        make_rsrc_c(Gc, (uint32_t)((int64_t)((P.Mo + CB_QC - 1) / CB_QC) * P.ldy * CB_QC * 4));
    uint32_t gcol[CBB_NS];
    gcol[0] = (uint32_t)((o0 / 16) * P.ldy * 16 + lr) * 4u;
    const uint32_t ystep = 16 * 4u;
    float ga_[CBB_NS][8], gb_[CBB_NS][8];
#define VIHMC_CBB_GLOAD(GN, CI)                                                                             \
    {                                                                                                       \
        const int qb0 = q_lo + (CI) * CB_QC;                                                                \
        _Pragma("unroll") for (int jj = 0; jj < 8; ++jj) {                                                  \
            const int qq = qb0 + (jj < 4 ? 4 * lg + jj : 12 + 4 * lg + jj);                                 \
            const uint32_t roff = qq < q_hi ? (uint32_t)qq * ystep : OOB_C;                                 \
            _Pragma("unroll") for (int s = 0; s < CBB_NS; ++s)                                              \
                GN[s][jj] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, roff + gcol[s], 0, 0)); \
        }                                                                                                   \
    }

    // G one chunk ahead in two register sets (rotated by a 2x unrolled loop), the image one chunk ahead by asm
    // LDS-DMA. Per chunk the DMA is issued before the G loads, so the chunk ends with a counted vmcnt(8 NS) -- the
    // image (invisible to hipcc) landed, G(i+1) left in flight for the next chunk's split -- instead of vmcnt(0),
    // which made every chunk wait out the HBM latency of the G loads it had just issued (the previous design
    // loaded G two chunks ahead in three sets to survive that drain). The G loads are unconditional (clamped
    // chunk index) and the loop runs whole pairs, so hipcc's own counted wait before the split of G(i) is exact.
    if (nchunks > 0) {
        VIHMC_CBB_GLDS(0, 0)
        VIHMC_CBB_GLOAD(ga_, 0)
        bf6::wait_vmcnt0();                          // chunk 0 published by the first barrier
    }
    f32x4 dacc[CBB_NS][7];
#pragma unroll
    for (int s = 0; s < CBB_NS; ++s)
#pragma unroll
        for (int t = 0; t < 7; ++t) dacc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int tr_off = (4 * lg + (lr >> 2)) * CB_PITCH + 8 * (lr & 3);
    auto chunk = [&](int i, float (&gv)[CBB_NS][8], float (&gn)[CBB_NS][8]) __attribute__((always_inline)) {
        __syncthreads();                      // chunk i landed; buffer (i+1)%3 free
        // split G(i) first: hipcc's wait for its loads then sits before this chunk's DMA (which it cannot see and
        // would otherwise wait for too); the empty asm pins the split ahead of the DMA's asm
        bf16x8 ga[CBB_NS][3];
#pragma unroll
        for (int s = 0; s < CBB_NS; ++s) {
            bf16x4 l0, l1, l2, h0, h1, h2;
            split4(f32x4{gv[s][0], gv[s][1], gv[s][2], gv[s][3]}, l0, l1, l2);
            split4(f32x4{gv[s][4], gv[s][5], gv[s][6], gv[s][7]}, h0, h1, h2);
            ga[s][0] = cat8(l0, h0);
            ga[s][1] = cat8(l1, h1);
            ga[s][2] = cat8(l2, h2);
            asm volatile("" :: "v"(ga[s][0]), "v"(ga[s][1]), "v"(ga[s][2]));
        }
        if (i + 1 < nchunks) {
            VIHMC_CBB_GLDS(i + 1, (i + 1) % 3)
        }
        VIHMC_CBB_GLOAD(gn, min(i + 1, nchunks - 1))
        const unsigned char* img = smb + (i % 3) * CB_QIMG;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            bf16x8 qb[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const unsigned char* a = img + p * CB_PLANE + tr_off + 32 * t;
                const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
                const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 16 * CB_PITCH));
                qb[p] = cat8(lo, hi);
            }
#pragma unroll
            for (int s = 0; s < CBB_NS; ++s) dacc[s][t] = six(ga[s], qb, dacc[s][t]);
        }
        // the image of chunk i+1 landed before the next barrier; G(i+1) may stay in flight
        if (CBB_NS == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    };
    int i = 0;
    for (; i + 1 < nchunks; i += 2) {
        chunk(i, ga_, gb_);
        chunk(i + 1, gb_, ga_);
    }
    if (i < nchunks) chunk(i, ga_, gb_);
    bf6::wait_vmcnt0();                              // the clamped tail loads retired
    float* out = P.out + c * P.out_cs + (int64_t)qc * P.out_chunk_stride;
#pragma unroll
    for (int s = 0; s < CBB_NS; ++s)
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
#undef VIHMC_CBB_GLDS
#undef VIHMC_CBB_GLOAD
}

#if CB_STAMP
extern "C" int vihmc_debug_cb_stamps(void* stamps, size_t stamp_bytes, void* real, size_t real_bytes) {
    if (stamp_bytes != sizeof(cb_stamps) || real_bytes != sizeof(cb_real)) return -1;
    hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(cb_stamps), stamp_bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(real, HIP_SYMBOL(cb_real), real_bytes, 0, hipMemcpyDeviceToHost);
    return (int)e;
}
#endif

hipError_t launch_contract_bf_b(const ContractProb& p, int C, hipStream_t s) {
    if (p.W != 100 || !p.load_g || !p.qimg || p.q_per_chunk % CB_QC) return hipErrorInvalidValue;
    dim3 g(C * p.o_tiles * p.q_chunks), blk(CBB_THREADS);
    hipLaunchKernelGGL(k_contract_bf_b, g, blk, 3 * CB_QIMG, s, p);
    return hipGetLastError();
}

hipError_t launch_contract_bf(const ContractProb& p, int C, hipStream_t s) {
    if (p.W != 100 || p.load_g || !p.qimg || p.q_per_chunk % CB_QC) return hipErrorInvalidValue;
    dim3 g(C * p.o_tiles * p.q_chunks), blk(CBA_THREADS);
    hipLaunchKernelGGL(k_contract_bf, g, blk, CB_LDS, s, p);
    return hipGetLastError();
}


}  // namespace vihmc
