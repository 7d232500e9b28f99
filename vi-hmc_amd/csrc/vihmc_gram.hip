// Gradient-only contraction in Gram form (the leapfrog's inner evaluations, where no log-prob is returned).
//
// Replaces the autograd backward of torch.einsum("...i,...i->...", xb, xtr) + b and the Gaussian NLL
// (Operator_network/VI_HMC/my_make_func.py:79-82, main_VI_HMC_burgers.py:157-163) when only the gradient is
// needed. With the augmented outputs Zb^ = [Z_b | 1] (N x 101) and Zt^ = [Z_t | b0] (P x 101) the prediction is
// S + b0 = Zb^ Zt^T and G = gscale (Zb^ Zt^T - y), so
//     dZb^ = G Zt^ = gscale (Zb^ Gt - y Zt^),      Gt = Zt^T Zt^   (101 x 101)
//     dZt^ = G^T Zb^ = gscale (Zt^ Gb - y^T Zb^),  Gb = Zb^T Zb^
// and d ll / d b0 = sum G = sum_p dZt^[p][100]. The N x P residual is never formed: the two products with the
// data y (shared by every chain, pre-split once per plan) are plain GEMMs over all chains, and the Gram terms are
// W x W. Per chain 2 N P W + O((N + P) W^2) MACs instead of 3 N P W, no G^T hand-off, no per-element VALU.
// The log-likelihood value itself (sum r^2) is not computed here: with a good fit it is a small difference of
// large Gram-form terms, so evaluations that return the log-prob keep the residual form (k_contract_bf).
//
// Products are bf16x6 (vihmc_bf16x6.h): every operand pre-split into three bf16 planes, six MFMA products per
// 32-long k-block, fp32 accumulation -- fp32-level accuracy, no splits inside the loops.
//
// Kernels (one evaluation, C chains):
//   k_gram_aug   feature 100 of the pre-split output images: 1 (branch rows < N), b0 (trunk rows < P) -- only when
//                the fused forward did not write the images (it writes that column itself, FusedNet::aug)
//   k_gram_a     T_b = y Zt^ over the trunk image, Gt = Zt^T Zt^, Gb = Zb^T Zb^: split-K partial slabs
//   k_gram_sum   fixed-order slab sums: Gt (both halves), -Gb pre-split as the B blocks of k_gram_b's extension,
//                and (more than GRAM_TB_DIRECT T_b slabs) the T_b sum the dZb epilogue units read
//   k_gram_b     dZt = -gscale (y^T Zb^ - Zt^ Gb) over the branch image + 4 extension blocks; d ll / d b0 slots
//   (k_gram_b)   dZb = gscale (Zb^ Gt - sum_s T_b slab s): epilogue units after the T_t units of k_gram_b
//   k_gram_tt    (T_t split over the branch blocks, few chains) fixed-order sum of the T_t slabs, dZt, d ll / d b0
// Images: the contraction's pre-split blocks (k_split_blocks' layout, written by the fused forward): block =
// 3 planes [32 rows][112 features] bf16, 224-B rows. The B operand (rows = k) is read with ds_read_b64_tr_b16
// (bf6::tr_frag), which delivers k rows 4lg..4lg+3 and 16+4lg..+3 of a 32-row block; the pre-split data images
// YA = y[n][p] and YB = y^T[p][n] store each 32-long k block in that order, so a lane's A fragment is one 16-B load.
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"
#include <type_traits>

namespace vihmc {

namespace {
using bf6::bf16x4;
using bf6::bf16x8;
using bf6::f32x4;
using bf6::six;

constexpr int GR_PL = CONTRACT_SPLIT_ROWS * bf6::PITCH;   // 7168 B per plane of a block
constexpr int GR_BLK = 3 * GR_PL;                         // 21504 B of planes per block (the fp32 tail is not used)
constexpr int GR_PIECES = GR_BLK / 1024;                  // 21 one-KB DMA pieces per block
static_assert(GR_PIECES * 1024 == GR_BLK, "whole DMA pieces");
constexpr int GR_NBUF = 3;
constexpr int GR_LDS = GR_NBUF * GR_BLK;                  // 64.5 KB
// k_gram_b: the ring, then the 4th planes of the 4 -Gb extension blocks (DMA'd first); its dZb epilogue units stage
// Gt in fp64 [101][112] and Zb^T [101][32] fp32 over the same LDS
constexpr int GRB_P3 = GR_LDS;
constexpr int GRB_LDS_T = GRB_P3 + 4 * GRAM_P3_BLOCK;     // 92.5 KB
constexpr int GRB_DZB = 101 * 112 * 8 + 101 * 32 * 4;     // 103,424 B
constexpr int GRB_LDS = GRB_LDS_T > GRB_DZB ? GRB_LDS_T : GRB_DZB;
static_assert(GRB_LDS <= 160 * 1024, "k_gram_b LDS");
static_assert(GRAM_P3_BLOCK % 1024 == 0, "whole DMA pieces");
constexpr int GR_CW = 8;                                  // compute waves (32 rows each)
constexpr int GR_THREADS = 64 * (GR_CW + 1);              // + one DMA wave
// centred form (GramArgs::center): k_gram_a's Gram units stream the output image AND the centre's image (ring slots
// of two blocks); k_gram_b runs 8 extension blocks (-Gb, then -Hb) and its dZb units stage Gt (fp64), Ht (fp32),
// dB^T and B0^T
constexpr int GR_LDS_C = GR_NBUF * 2 * GR_BLK;            // 126 KB
constexpr int GRB_LDS_TC = GR_LDS;                       // 64.5 KB: no 4th planes
constexpr int GRB_DZBC = 2 * 101 * 112 * 4 + 2 * 101 * 32 * 4;               // 116,352 B
constexpr int GRB_LDS_C = GRB_LDS_TC > GRB_DZBC ? GRB_LDS_TC : GRB_DZBC;
static_assert(GR_LDS_C <= 160 * 1024 && GRB_LDS_C <= 160 * 1024, "centred Gram LDS");

// position of k (0..31) inside a 32-long block of the A images: lane group lg holds k = 4lg..4lg+3, 16+4lg..+3
__host__ __device__ inline int kpos(int k) { return k < 16 ? 8 * (k >> 2) + (k & 3) : 8 * ((k - 16) >> 2) + 4 + (k & 3); }

// the DMA wave of a block ring: block i -> buffer i % 3, copies of block i+2 issued after the barrier of
// iteration i (every wave is past block i-1 = buffer (i+2) % 3), then wait for block i+1 (21 newer copies may stay
// in flight) so the next barrier publishes it. SRC(i) gives block i's global address.
#define GRAM_DMA_PIECES(SRC, BUF)                                                                             \
    for (int k = 0; k < (GR_ABL & 2 ? 0 : GR_PIECES); ++k)                                                     \
        bf6::glds16_asm((SRC) + k * 1024 + lane * 16, lds + (BUF) * GR_BLK + k * 1024);

struct NoStamp {
    __device__ void operator()(int, int) const {}
};
template <typename F, typename ST = NoStamp>
__device__ __forceinline__ void dma_role(unsigned char* lds, int lane, int nb, F src, ST st = ST{}) {
    if (nb > 0) { GRAM_DMA_PIECES(src(0), 0) }
    if (nb > 1) { GRAM_DMA_PIECES(src(1), 1) }
    if (nb > 1) asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < nb; ++i) {
        __syncthreads();
        st(i, 0);
        if (i + 2 < nb) {
            GRAM_DMA_PIECES(src(i + 2), (i + 2) % GR_NBUF)
            st(i, 1);
            asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
        } else {
            st(i, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        st(i, 2);
    }
}

__device__ __forceinline__ void load_b(const unsigned char* buf, int tro, int t, bf16x8 (&b)[3]) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) b[pl] = bf6::tr_frag(buf + pl * GR_PL, tro, 16 * t);
}

// the centred Gram units' DMA wave: block i of the output image (s0) and of the centre's image (s1) into ring slot
// i % 3 (two blocks, 42 one-KB pieces), the order and counted waits of dma_role
__device__ __forceinline__ void dma_role2(unsigned char* lds, int lane, int nb, const unsigned char* s0,
                                          const unsigned char* s1) {
    auto issue = [&](int i) __attribute__((always_inline)) {
        const unsigned char* a = s0 + (int64_t)i * CONTRACT_SPLIT_BLOCK;
        const unsigned char* b = s1 + (int64_t)i * CONTRACT_SPLIT_BLOCK;
        unsigned char* d = lds + (i % GR_NBUF) * 2 * GR_BLK;
        for (int k = 0; k < (GR_ABL & 2 ? 0 : GR_PIECES); ++k) bf6::glds16_asm(a + k * 1024 + lane * 16, d + k * 1024);
        for (int k = 0; k < (GR_ABL & 2 ? 0 : GR_PIECES); ++k)
            bf6::glds16_asm(b + k * 1024 + lane * 16, d + GR_BLK + k * 1024);
    };
    if (nb > 0) issue(0);
    if (nb > 1) issue(1);
    if (nb > 1) asm volatile("s_waitcnt vmcnt(42)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < nb; ++i) {
        __syncthreads();
        if (i + 2 < nb) {
            issue(i + 2);
            asm volatile("s_waitcnt vmcnt(42)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
}

// fp32 value of three exact bf16 planes ((x0 + x1) + x2 is exact: the partial sums are x rounded to 16 / 24 bits)
__device__ __forceinline__ float unsplit(__bf16 a, __bf16 b, __bf16 c) { return ((float)a + (float)b) + (float)c; }

// d = z - r of two pre-split fragments: one rounded fp32 subtraction, then the exact three-way split
__device__ __forceinline__ void delta_frag(const bf16x8 (&z)[3], const bf16x8 (&r)[3], bf16x8 (&d)[3]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = unsplit(z[0][j], z[1][j], z[2][j]) - unsplit(r[0][j], r[1][j], r[2][j]);
        const __bf16 a = (__bf16)x;
        const float rr = x - (float)a;
        const __bf16 b = (__bf16)rr;
        d[0][j] = a;
        d[1][j] = b;
        d[2][j] = (__bf16)(rr - (float)b);
    }
}

#if GR_STAMP
// every 16th T_b unit (at most 32) of the last k_gram_a launch: per wave (8 compute + the DMA wave) and k block
// s_memtime at the barrier exit [0], after the next block's loads / DMA pieces are issued [1], after the block's MFMAs
// are issued (compute) or the DMA wait (DMA wave) [2]; per workgroup s_memtime / s_memrealtime at start and end
// (profiles/scripts/diag/stamps_gram.py)
constexpr int GRS_WG = 32, GRS_BLK = 48;
__device__ unsigned long long gr_stamps[GRS_WG][GR_CW + 1][GRS_BLK][3];
__device__ unsigned long long gr_real[GRS_WG][2][2];
#define GR_ST(I, K)                                                                                             \
    if (gr_samp && lane == 0 && (I) < GRS_BLK) gr_stamps[gr_sidx][wave][(I)][(K)] = __builtin_amdgcn_s_memtime();
#else
#define GR_ST(I, K)
#endif

// one 32-long k block of a wave's 32 x 112 tile: B fragments of column tile t+1 read while tile t's 12 MFMAs run
// (double-buffered fragments, so the wait before tile t's products leaves the next tile's reads in flight)
// pre(t) runs before tile t's products: the T_b / T_t loops issue one of the next block's six A loads there, so
// the loads spread over the block's MFMAs. Issued all at once after the barrier (with the DMA wave's 21 pieces), the
// loads queued behind each other for ~1,200 cycles before the first MFMA of a 4,400-cycle block period (stamps:
// profiles/r04s_stamps_gram.txt).
struct NoPre {
    __device__ void operator()(int) const {}
};
template <typename PRE = NoPre>
__device__ __forceinline__ void mma_block(const unsigned char* buf, int tro, const bf16x8 (&a)[2][3],
                                          f32x4 (&acc)[2][7], PRE pre = PRE{}) {
    bf16x8 b[2][3];
    load_b(buf, tro, 0, b[0]);
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        if (t < 6) load_b(buf, tro, t + 1, b[(t + 1) & 1]);
        pre(t);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt][t] = six(a[rt], b[t & 1], acc[rt][t]);
    }
}

// the extension blocks' product with a FOUR-plane B (the -Gb image, k_gram_sum): the three order-3 products
// (a2 b1, a1 b2, a0 b3: ~2^-24 of the product each) first, then bf6::six's six -- the B value carried to ~32 bits
__device__ __forceinline__ f32x4 nine(const bf16x8 (&a)[3], const bf16x8 (&b)[3], const bf16x8& b3, f32x4 acc) {
    acc = bf6::mfma_bf(a[2], b[1], acc);
    acc = bf6::mfma_bf(a[1], b[2], acc);
    acc = bf6::mfma_bf(a[0], b3, acc);
    return six(a, b, acc);
}
__device__ __forceinline__ void mma_block9(const unsigned char* buf, const unsigned char* p3, int tro,
                                           const bf16x8 (&a)[2][3], f32x4 (&acc)[2][7]) {
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        bf16x8 b[3];
        load_b(buf, tro, t, b);
        const bf16x8 b3 = bf6::tr_frag(p3, tro, 16 * t);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt][t] = nine(a[rt], b, b3, acc[rt][t]);
        __builtin_amdgcn_sched_barrier(0);             // one tile's fragments live at a time (no hoisting: spills)
    }
}

// unit of a workgroup with XCD-contiguous unit ranges (workgroup b runs on XCD b % 8, checked by
// scripts/diag/xcc_probe.hip): `upx` slots of every XCD take units [x upx, (x + 1) upx) of the grouped list, `gpx`
// slots round-robin units of the second list; -1 = idle slot. second_first: k_gram_a's Gram units are shorter than
// the GEMM units, which then fill the chip behind them (gradient-only evaluation at 16 chains: Gram form 0.542 ->
// 0.525 ms, profiles/r03u_ab_gram.txt; raising the wave priority around the MFMAs measured neutral)
__device__ __forceinline__ void unit_of(int b, int upx, int n1, int n2, int& list, int& u, bool second_first = true) {
    const int x = b & 7, gpx = (n2 + 7) / 8;
    int k = b >> 3;
    if (second_first) k = k < gpx ? k + upx : k - gpx;
    if (k < upx) {
        list = 0;
        u = x * upx + k;
        if (u >= n1) list = -1;
    } else {
        list = 1;
        u = (k - upx) * 8 + x;
        if (u >= n2) list = -1;
    }
}
}  // namespace

// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gram_aug(GramArgs A) {
    const int c = blockIdx.y;
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int f = 2 * 100;                                    // byte offset of feature 100 in a plane row
    if (r < A.N) {
        unsigned char* row = A.bimg + c * A.bimg_cs + (int64_t)(r / 32) * CONTRACT_SPLIT_BLOCK + (r % 32) * bf6::PITCH;
        *reinterpret_cast<__bf16*>(row + f) = (__bf16)1.0f;
        *reinterpret_cast<__bf16*>(row + GR_PL + f) = (__bf16)0.0f;
        *reinterpret_cast<__bf16*>(row + 2 * GR_PL + f) = (__bf16)0.0f;
    } else if (r < A.N + A.P) {
        const int q = r - A.N;
        const float b0 = A.b0[c * A.b0_cs];
        const __bf16 a = (__bf16)b0;
        const float rr = b0 - (float)a;
        const __bf16 bb = (__bf16)rr;
        unsigned char* row = A.timg + c * A.timg_cs + (int64_t)(q / 32) * CONTRACT_SPLIT_BLOCK + (q % 32) * bf6::PITCH;
        *reinterpret_cast<__bf16*>(row + f) = a;
        *reinterpret_cast<__bf16*>(row + GR_PL + f) = bb;
        *reinterpret_cast<__bf16*>(row + 2 * GR_PL + f) = (__bf16)(rr - (float)bb);
        // column 101 = 1: Gt[v][101] = sum_p Zt^[p][v] (the exact d ll / d b0, gram_tt_epilogue)
        *reinterpret_cast<__bf16*>(row + f + 2) = (__bf16)1.0f;
        *reinterpret_cast<__bf16*>(row + GR_PL + f + 2) = (__bf16)0.0f;
        *reinterpret_cast<__bf16*>(row + 2 * GR_PL + f + 2) = (__bf16)0.0f;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// k_gram_a: list 0 = T_b units (g = s * NG + ng major, chain minor: with 8 slabs, XCD x runs slab x -- the chains
// sharing one YA slab and the n groups sharing one chain's trunk slab are co-resident on one XCD, and its Gram-t units
// (c * S + s, round robin) land there too), list 1 = Gram units (C * S Gram-t slabs, then C Gram-b).
//   T_b unit (ng, s, c): rows n0 = 256 ng + 32 w of wave w, trunk blocks [s SL, (s+1) SL): acc[2][7] tiles, stored
//     tile-major to tb_part[c][s][ng][w][rt][t] (256 floats = 64 lanes x float4 each).
//   Gram-t (c, s): the 28 upper 16x16 tiles of Zt^T Zt^ over the slab (4 per wave, A = the B fragment of the tile's
//     row); stored to gt_part[c][s][28][256] (fp64); k_gram_sum adds the St slabs up in order s = 0.. into gt[c]
//     ([112 v][112 w] fp32, both halves).
//   Gram-b (c, s): the same over the branch blocks [s SLb, (s+1) SLb) into gb_part; k_gram_sum writes -Gb pre-split
//     as 4 blocks (rows v, k of the extension).
// ---------------------------------------------------------------------------------------------------------------
template <int GT>
__global__ __launch_bounds__(GR_THREADS, 1) void k_gram_a(GramArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    int list, u;
    constexpr int NGT = GT > 0 ? 0 : 1;  // Gram-t units of their own (GT = 0: the T_b units take no Gram-t tiles)
    unit_of(blockIdx.x, A.upx_a, A.NG * A.S * A.C, A.C * (NGT * A.St + A.Sb), list, u);
    if (list < 0) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    // decode the unit
    int c, s = 0, ng = 0, kind;          // kind 0 = T_b (GT > 0: + its share of the slab's Gram-t tiles), 1 = Gram-t,
                                         // 2 = Gram-b
    if (list == 0) {
        const int g = u / A.C;
        c = u - g * A.C;
        s = g / A.NG;
        ng = g - s * A.NG;
        kind = 0;
    } else if (u < NGT * A.C * A.St) {
        c = u / A.St;
        s = u - c * A.St;
        kind = 1;
    } else {
        const int u2 = u - NGT * A.C * A.St;
        c = u2 / A.Sb;
        s = u2 - c * A.Sb;
        kind = 2;
    }
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain (unit-uniform)
    const unsigned char* src0;
    int nb, kb0 = 0;
    if (kind == 2) {
        kb0 = s * A.SLb;                  // Gram-b slab s: SLb branch blocks
        nb = min(A.SLb, A.nblkN - kb0);
        src0 = A.bimg + c * A.bimg_cs + (int64_t)kb0 * CONTRACT_SPLIT_BLOCK;
    } else if (kind == 1) {
        kb0 = s * A.SLt;                  // Gram-t slab s: the T_b slab's trunk blocks
        nb = min(A.SLt, A.nblkP - kb0);
        src0 = A.timg + c * A.timg_cs + (int64_t)kb0 * CONTRACT_SPLIT_BLOCK;
    } else {
        kb0 = s * A.SL;
        nb = min(A.SL, A.nblkP - kb0);
        src0 = A.timg + c * A.timg_cs + (int64_t)kb0 * CONTRACT_SPLIT_BLOCK;
    }
    const int tro = bf6::tr_lane_off(lr, lg);
#if GR_STAMP
    const bool gr_samp = kind == 0 && (u & 15) == 0 && (u >> 4) < GRS_WG;
    const int gr_sidx = u >> 4;
    if (gr_samp && tid == 0) {
        gr_real[gr_sidx][0][0] = __builtin_amdgcn_s_memtime();
        gr_real[gr_sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const bool cgram = A.center && kind != 0;             // centred Gram unit: G and H over the slab
    if (wave == GR_CW) {
        if (cgram) {
            const unsigned char* ref = (kind == 2 ? A.cbimg : A.ctimg) + (int64_t)kb0 * CONTRACT_SPLIT_BLOCK;
            dma_role2(lds, lane, nb, src0, ref);
        } else {
#if GR_STAMP
        dma_role(lds, lane, nb, [&](int i) { return src0 + (int64_t)i * CONTRACT_SPLIT_BLOCK; },
                 [&](int i, int k) { GR_ST(i, k) });
#else
        dma_role(lds, lane, nb, [&](int i) { return src0 + (int64_t)i * CONTRACT_SPLIT_BLOCK; });
#endif
        }
    } else if (cgram) {
        // ---------------- centred Gram unit (c, s): G = Z^T Z (28 upper tiles) and H = dZ^T Z (49 tiles) ----------
        // over the slab's blocks of one side (kind 1: Z = Zt^, dZ = Zt^ - T0; kind 2: Z = Zb^, dZ = Zb^ - B0). Compute
        // wave vt < 7 owns row tile vt: H (vt, 0..6) and G (vt, vt..6), sharing each column fragment; its dZ fragment
        // is formed once per block from the two images' planes (delta_frag). fp32 MFMA accumulation over the slab
        // (in the centred form both matrices multiply residual-sized operands), fp64 across the slabs (k_gram_sum).
        // Balance: compute wave 7 takes G (0, 4..6), (1, 5..6), (2, 6), so the four SIMDs (waves w, w + 4) carry 21 / 20 /
        // 19 / 17 tiles per block instead of 24 / 20 / 16 / 11 (wave vt keeps G (vt, vt .. lim(vt) - 1))
        const int vt = wave;
        const int lim = vt < 3 ? 4 + vt : 7;
        f32x4 hacc[7], gacc[7];
#pragma unroll
        for (int t = 0; t < 7; ++t) hacc[t] = gacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int i = 0; i < nb; ++i) {
            __syncthreads();
            const unsigned char* zbuf = lds + (i % GR_NBUF) * 2 * GR_BLK;
            if (vt < 7) {
                bf16x8 za[3], ra[3], da[3];
                load_b(zbuf, tro, vt, za);
                load_b(zbuf + GR_BLK, tro, vt, ra);
                delta_frag(za, ra, da);
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    bf16x8 b[3];
                    load_b(zbuf, tro, t, b);
                    hacc[t] = six(da, b, hacc[t]);
                    if (t >= vt && t < lim) gacc[t] = six(za, b, gacc[t]);
                }
            } else {
                // wave 7: the six G tiles of rows 0..2 the first three waves leave (gacc[k], k = 0..5)
                bf16x8 a0f[3], a1f[3], a2f[3];
                load_b(zbuf, tro, 0, a0f);
                load_b(zbuf, tro, 1, a1f);
                load_b(zbuf, tro, 2, a2f);
#pragma unroll
                for (int t = 4; t < 7; ++t) {
                    bf16x8 b[3];
                    load_b(zbuf, tro, t, b);
                    gacc[t - 4] = six(a0f, b, gacc[t - 4]);                       // (0, 4), (0, 5), (0, 6)
                    if (t >= 5) gacc[t - 2] = six(a1f, b, gacc[t - 2]);           // (1, 5), (1, 6)
                    if (t == 6) gacc[5] = six(a2f, b, gacc[5]);                   // (2, 6)
                }
            }
        }
        double* gp = (kind == 1 ? A.gt_part + c * A.gt_cs : A.gb_part + c * A.gb_cs) + (int64_t)s * 28 * 256 + 4 * lane;
        // index of (v, t) in the row-major upper-triangle list (k_gram_sum's decode)
        auto tri = [](int v, int t) { return 7 * v - v * (v - 1) / 2 + t - v; };
        if (vt < 7) {
            float* hp = (kind == 1 ? A.ht_part + c * A.ht_cs : A.hb_part + c * A.hb_cs) +
                        ((int64_t)s * 49 + vt * 7) * 256 + 4 * lane;
#pragma unroll
            for (int t = 0; t < 7; ++t) *reinterpret_cast<f32x4*>(hp + t * 256) = hacc[t];
#pragma unroll
            for (int t = 0; t < 7; ++t)
                if (t >= vt && t < lim) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) gp[tri(vt, t) * 256 + r] = (double)gacc[t][r];
                }
        } else {
            const int tv[6] = {0, 0, 0, 1, 1, 2}, tt[6] = {4, 5, 6, 5, 6, 6};
#pragma unroll
            for (int k = 0; k < 6; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) gp[tri(tv[k], tt[k]) * 256 + r] = (double)gacc[k][r];
        }
    } else if (kind == 0) {
        // ---------------- T_b = y Zt^ (A = YA rows, 16-B loads one block ahead in two register sets) ----------
        const int n0 = 256 * ng + 32 * wave;
        const __bf16* ya = A.ya + (int64_t)(n0 + lr) * A.ya_ld + (int64_t)kb0 * 32 + 8 * lg;
        const int64_t rt16 = 16 * (int64_t)A.ya_ld;
        bf16x8 a0[2][3], a1[2][3];
        auto load_a = [&](bf16x8 (&a)[2][3], int i) __attribute__((always_inline)) {
            const int ii = (GR_ABL & 1) ? 0 : min(i, nb - 1);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    a[rt][pl] = *reinterpret_cast<const bf16x8*>(ya + pl * A.ya_plane + rt * rt16 + 32 * ii);
        };
        f32x4 acc[2][7];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        // this unit's share of the slab's Gram-t tiles: the NG units of (s, c) stream the same trunk blocks, so wave
        // w of unit ng takes tiles j = 8 ng + w + 8 NG q (q < GT) of the 28 upper tiles -- no Gram-t units of their
        // own (which re-streamed the blocks: 128 of 656 k_gram_a units at 16 chains). Per block and tile the same
        // products and fp64 accumulation as a Gram unit: the same slab values bit for bit.
        constexpr int G1 = GT > 0 ? GT : 1;
        double accg[G1][4];
        int gvt[G1], gtt[G1], gj[G1];
#pragma unroll
        for (int q = 0; q < G1; ++q) {
            gj[q] = GT > 0 ? GR_CW * ng + wave + GR_CW * A.NG * q : 28;     // wave-uniform
            int rem = min(gj[q], 27), vt = 0;
            while (rem >= 7 - vt) rem -= 7 - vt++;
            gvt[q] = vt;
            gtt[q] = vt + rem;
#pragma unroll
            for (int r = 0; r < 4; ++r) accg[q][r] = 0.0;
        }
        auto step = [&](int i, bf16x8 (&a)[2][3], bf16x8 (&an)[2][3]) __attribute__((always_inline)) {
            __syncthreads();
            GR_ST(i, 0)
            const int ii = (GR_ABL & 1) ? 0 : min(i + 1, nb - 1);
            GR_ST(i, 1)
            const unsigned char* buf = lds + (i % GR_NBUF) * GR_BLK;
            // the next block's A loads, one per tile under this block's MFMAs
            mma_block(buf, tro, a, acc, [&](int t) __attribute__((always_inline)) {
                if (t < 6) {
                    const int rt = t / 3, pl = t % 3;
                    an[rt][pl] = *reinterpret_cast<const bf16x8*>(ya + pl * A.ya_plane + rt * rt16 + 32 * ii);
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
#pragma unroll
            for (int q = 0; q < G1; ++q) {
                if (GT > 0 && gj[q] < 28) {
                    bf16x8 ga[3], gb[3];
                    load_b(buf, tro, gvt[q], ga);
                    load_b(buf, tro, gtt[q], gb);
                    const f32x4 blk = six(ga, gb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                    for (int r = 0; r < 4; ++r) accg[q][r] += (double)blk[r];
                }
            }
#if GR_STAMP
            __builtin_amdgcn_sched_barrier(0);
#endif
            GR_ST(i, 2)
        };
        load_a(a0, 0);
        int i = 0;
        for (; i + 1 < nb; i += 2) {
            step(i, a0, a1);
            step(i + 1, a1, a0);
        }
        if (i < nb) step(i, a0, a1);
        float* dst = A.tb_part + c * A.tb_cs + ((int64_t)((s * A.NG + ng) * GR_CW + wave) * 14) * 256 + 4 * lane;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) *reinterpret_cast<f32x4*>(dst + (rt * 7 + t) * 256) = acc[rt][t];
        double* gpart = A.gt_part + c * A.gt_cs;
#pragma unroll
        for (int q = 0; q < G1; ++q)
            if (GT > 0 && gj[q] < 28) {
#pragma unroll
                for (int r = 0; r < 4; ++r) gpart[((s * 28) + gj[q]) * 256 + 4 * lane + r] = accg[q][r];
            }
#if GR_STAMP
        if (gr_samp && tid == 0) {
            gr_real[gr_sidx][1][0] = __builtin_amdgcn_s_memtime();
            gr_real[gr_sidx][1][1] = __builtin_amdgcn_s_memrealtime();
        }
#endif
    } else {
    // ---------------- Gram tiles: the 28 tiles (vt <= t) of the symmetric 112 x 112 matrix, 4 per wave ------------
    // Every element of Gt / Gb enters all N (P) rows of the other side's correction product, so its rounding error
    // adds up coherently in the last layer's bias gradient (a sum over rows): each block's six products are summed
    // from zero in fp32 (one 32-long dot) and the blocks in fp64 -- not 240 fp32 roundings of one running sum.
    // Wave w < 7 owns tiles j = w, w+7, w+14, w+21 of the row-major upper-triangle list (A = the B fragment of row
    // tile vt); the mirror half is written from them.
    double acc[4][4];
    int tvt[4], tt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int rem = min(wave, 6) + 7 * q, vt = 0;
        while (rem >= 7 - vt) rem -= 7 - vt++;
        tvt[q] = vt;
        tt[q] = vt + rem;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[q][r] = 0.0;
    }
    for (int i = 0; i < nb; ++i) {
        __syncthreads();
        if (wave < 7) {
            const unsigned char* buf = lds + (i % GR_NBUF) * GR_BLK;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bf16x8 a[3], b[3];
                load_b(buf, tro, tvt[q], a);
                load_b(buf, tro, tt[q], b);
                const f32x4 blk = six(a, b, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[q][r] += (double)blk[r];
            }
        }
    }
    if (wave < 7) {
        // Gram-t / Gram-b slab s of chain c: the 28 upper tiles
        double* part = kind == 1 ? A.gt_part + c * A.gt_cs : A.gb_part + c * A.gb_cs;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[((s * 28) + wave + 7 * q) * 256 + 4 * lane + r] = acc[q][r];
    }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// k_gram_sum: the slab sums, fixed order s = 0.. (fp64 for the Gram slabs), block (x, chain):
//   x < 28       Gt tile x: Gt = sum of the St Gram-t slabs, fp32, both halves
//   28 <= x < 56 Gb tile x - 28: -sum of the Sb Gram-b slabs, pre-split into the 4 extension blocks of k_gram_b
//   x >= 56      (S > GRAM_TB_DIRECT only) 4 T_b tiles: tb_sum = sum of the S T_b slabs, for the dZb epilogue units
// A launch of its own: the slabs come from workgroups on all 8 XCDs, and a kernel boundary makes them visible.
// The mirror half is written off the diagonal tiles only: a diagonal tile holds both (v, x) and (x, v), computed in
// different product orders (not bitwise equal), and mirroring there made two threads write one element with different
// values -- the nondeterminism of profiles/r04e_nondet.txt / r04j_nondet3.txt (one element of Gt, then dZb).
// ---------------------------------------------------------------------------------------------------------------
// -Gb / -Hb pre-split from an fp64 sum into FOUR bf16 planes (~32 significant bits): element (v, x) -> extension block
// v / 32, row v % 32, feature x; planes 0..2 in the block image, plane 3 in the P3 image
__device__ __forceinline__ void put4(unsigned char* img, unsigned char* p3, int vv, int xx, double val) {
    double rr = val;
    __bf16 pl[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        pl[k] = (__bf16)(float)rr;         // rr -> fp32 -> bf16: the fp32 step is exact for k >= 1 (|rr| small)
        rr -= (double)(float)pl[k];
    }
    unsigned char* q = img + (vv / 32) * CONTRACT_SPLIT_BLOCK + (vv % 32) * bf6::PITCH + 2 * xx;
    *reinterpret_cast<__bf16*>(q) = pl[0];
    *reinterpret_cast<__bf16*>(q + GR_PL) = pl[1];
    *reinterpret_cast<__bf16*>(q + 2 * GR_PL) = pl[2];
    *reinterpret_cast<__bf16*>(p3 + (vv / 32) * GRAM_P3_BLOCK + (vv % 32) * bf6::PITCH + 2 * xx) = pl[3];
}

__global__ __launch_bounds__(256) void k_gram_sum(GramArgs A) {
    const int x0 = blockIdx.x, c = blockIdx.y;
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int nh = A.center ? 98 : 0;                     // centred: 49 Ht tiles, then 49 Hb tiles
    if (x0 >= 56 && x0 < 56 + nh) {
        // H tile: fixed-order fp64 sum of the fp32 slab partials; Ht -> fp32 [112][112] (the dZb epilogue), -Hb -> the
        // 4-plane B blocks of k_gram_b's second extension set; the column sums of the exact d ll / d b0:
        // Ht[v][101] = sum_p dT[p][v], Hb[v][100] = sum_n dB[n][v]
        const bool hb = x0 - 56 >= 49;
        const int tile = (x0 - 56) % 49, vt = tile / 7, t = tile % 7;
        const int l = threadIdx.x >> 2, r = threadIdx.x & 3;
        const float* part = (hb ? A.hb_part + c * A.hb_cs : A.ht_part + c * A.ht_cs) + tile * 256 + threadIdx.x;
        const int ns = hb ? A.Sb : A.St;
        double sum = 0.0;
#pragma unroll 16
        for (int ss = 0; ss < ns; ++ss) sum += (double)part[(int64_t)ss * 49 * 256];
        const int v = 16 * vt + 4 * (l >> 4) + r, x = 16 * t + (l & 15);
        if (!hb) {
            A.ht[c * A.gt_cs2 + v * 112 + x] = (float)sum;
            if (x == 101) A.gcol[c * A.gcol_cs + 3 * 112 + v] = sum;
        } else {
            put4(A.hbimg + c * A.gbimg_cs, A.hb3img + c * 4 * GRAM_P3_BLOCK, v, x, -sum);
            if (x == 100) A.gcol[c * A.gcol_cs + 2 * 112 + v] = sum;
        }
        return;
    }
    if (x0 >= 56) {
        const int64_t sstride = (int64_t)A.NG * GR_CW * 14 * 256;
        const int64_t e = ((int64_t)(x0 - 56 - nh) * 256 + threadIdx.x) * 4;
        const float* src = A.tb_part + c * A.tb_cs + e;
        double v[4] = {0.0, 0.0, 0.0, 0.0};               // fp64 over the slabs, one rounding at the end
#pragma unroll 16
        for (int ss = 0; ss < A.S; ++ss) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(src + ss * sstride);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (double)w[r];
        }
        *reinterpret_cast<f32x4*>(A.tb_sum + c * A.tbs_cs + e) = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        return;
    }
    const bool gb = x0 >= 28;
    const int tile = gb ? x0 - 28 : x0;
    const int e = tile * 256 + threadIdx.x, l = threadIdx.x >> 2, r = threadIdx.x & 3;
    const double* part = gb ? A.gb_part + c * A.gb_cs : A.gt_part + c * A.gt_cs;
    const int ns = gb ? A.Sb : A.St;
    double sum = 0.0;
#pragma unroll 16
    for (int ss = 0; ss < ns; ++ss) sum += part[ss * 28 * 256 + e];
    int rem = tile, vt = 0;
    while (rem >= 7 - vt) rem -= 7 - vt++;
    const int t = vt + rem, v = 16 * vt + 4 * (l >> 4) + r, x = 16 * t + (l & 15);
    // the fp64 column sums of the exact d ll / d b0: sum_n Zb^[n][v] = Gb[v][100], sum_p Zt^[p][v] = Gt[v][101]
    if (x == (gb ? 100 : 101)) A.gcol[c * A.gcol_cs + (gb ? 0 : 112) + v] = sum;
    if (!gb) {
        float* gt = A.gt + c * A.gt_cs2;
        double* g64 = A.gt64 + c * A.gt_cs2;
        gt[v * 112 + x] = (float)sum;
        g64[v * 112 + x] = sum;
        if (vt != t) {
            gt[x * 112 + v] = (float)sum;
            g64[x * 112 + v] = sum;
        }
        return;
    }
    // -Gb pre-split from the fp64 sum into FOUR bf16 planes (~32 significant bits): every trunk row's extension product
    // Zt^ Gb uses the same Gb, so its representation error is coherent over the P rows -- rounded to fp32 it cost
    // 4.2e-4 of the gradient norm at fit 0.13 (profiles/r05d_gram_parts.txt); k_gram_b adds the order-3 products.
    // Element (v, x) -> extension block v / 32, row v % 32, feature x; planes 0..2 in the block image, plane 3 in gb3img
    unsigned char* gbi = A.gbimg + c * A.gbimg_cs;
    unsigned char* gb3 = A.gb3img + c * 4 * GRAM_P3_BLOCK;
    put4(gbi, gb3, v, x, -sum);
    if (vt != t) put4(gbi, gb3, x, v, -sum);
}

// ---------------------------------------------------------------------------------------------------------------
// k_gram_b: unit (pt, sb, c), chains minor (the chains sharing one YB slab on one XCD). Waves own 32 trunk rows
// p0 = 256 pt + 32 w; k runs over the split's branch blocks [sb SLB, (sb+1) SLB) (A = YB rows, 16-B loads) and, in
// the last split, 4 extension blocks (A = Zt^ rows from the trunk image, k = feature v; B = -Gb blocks). With SB = 1
// (enough chains to fill the chip) dZt = -gscale acc is written directly; with SB > 1 (few chains: 5 splits at one
// chain) each split stores its partial tiles and the last one to finish sums them. Column 100 goes to the
// d ll / d b0 slot (pt * 8 + w) of the chain.
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ void dzb_unit(const GramArgs& A, int u, unsigned char* lds);
__device__ __forceinline__ void dzb_unit_c(const GramArgs& A, int u, unsigned char* lds);
__device__ __forceinline__ void gram_tt_epilogue(const GramArgs& A, int c, int pt, int wave, int lane,
                                                 const f32x4 (&acc)[2][7]);

template <int CEN>
__global__ __launch_bounds__(GR_THREADS, 1) void k_gram_b(GramArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    int list, u;
    // the dZb epilogue units go last: they fill the half round the 640 T_t units leave at 16 chains (0.531 -> 0.519 ms,
    // profiles/r03z_ab_gram_epi_last.txt)
    unit_of(blockIdx.x, A.upx_b, (A.PT - A.pt2) * A.SB * A.C, A.C * ((A.N + 31) / 32), list, u, false);
    if (list < 0) return;
    if (list == 1) {                   // the dZb epilogue units fill the tail of the T_t rounds (k_gram_a is done)
        if (CEN) dzb_unit_c(A, u, lds);
        else dzb_unit(A, u, lds);
        return;
    }
    // T_t unit (pt, sb, c): chains minor, so the chains sharing one YB slab (rows, k range) run on one XCD
    const int g = u / A.C, c = u - g * A.C;
    const int pt = A.pt2 + g / A.SB, sb = g % A.SB;       // row groups [0, pt2): k_gram_b2's chain pairs
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int kb0 = sb * A.SLB;
    const int nbm = min(A.SLB, A.nblkN - kb0);            // this split's branch blocks (>= 1: SB = cdiv(nblkN, SLB))
    const bool ext = sb == A.SB - 1;                      // the last split also runs the extension blocks
    const int next = CEN ? 8 : 4;                         // centred: -Gb (A = dT rows), then -Hb (A = T0 rows)
    const int nb = nbm + (ext ? next : 0);
    const int p0 = 256 * pt + 32 * wave;
    f32x4 acc[2][7];
    if (wave == GR_CW) {
        const unsigned char* bsrc = A.bimg + c * A.bimg_cs + (int64_t)kb0 * CONTRACT_SPLIT_BLOCK;
        const unsigned char* gsrc = A.gbimg + c * A.gbimg_cs;
        const unsigned char* hsrc = CEN ? A.hbimg + c * A.gbimg_cs : nullptr;
        if (ext && !CEN) {
            // the 4th -Gb planes of the extension blocks, first: dma_role's counted waits retire them with block 0
            // (centred: the extension terms are of the residual's size, three planes carry them to fp32)
            const unsigned char* p3 = A.gb3img + c * 4 * GRAM_P3_BLOCK;
            for (int k = 0; k < 4 * GRAM_P3_BLOCK / 1024; ++k)
                bf6::glds16_asm(p3 + k * 1024 + lane * 16, lds + GRB_P3 + k * 1024);
        }
        dma_role(lds, lane, nb, [&](int i) {
            return i < nbm ? bsrc + (int64_t)i * CONTRACT_SPLIT_BLOCK
                           : (i - nbm < 4 ? gsrc + (int64_t)(i - nbm) * CONTRACT_SPLIT_BLOCK
                                          : hsrc + (int64_t)(i - nbm - 4) * CONTRACT_SPLIT_BLOCK);
        });
    } else {
        const int tro = bf6::tr_lane_off(lr, lg);
        const __bf16* yb = A.yb + (int64_t)(p0 + lr) * A.yb_ld + (int64_t)kb0 * 32 + 8 * lg;
        const int64_t rt16 = 16 * (int64_t)A.yb_ld;
        bf16x8 a0[2][3], a1[2][3];
        auto load_a = [&](bf16x8 (&a)[2][3], int i) __attribute__((always_inline)) {
            const int ii = (GR_ABL & 1) ? 0 : min(i, nbm - 1);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    a[rt][pl] = *reinterpret_cast<const bf16x8*>(yb + pl * A.yb_plane + rt * rt16 + 32 * ii);
        };
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        auto step = [&](int i, bf16x8 (&a)[2][3], bf16x8 (&an)[2][3]) __attribute__((always_inline)) {
            __syncthreads();
            const int ii = (GR_ABL & 1) ? 0 : min(i + 1, nbm - 1);
            // the next block's A loads, one per tile under this block's MFMAs (see mma_block)
            mma_block(lds + (i % GR_NBUF) * GR_BLK, tro, a, acc, [&](int t) __attribute__((always_inline)) {
                if (t < 6) {
                    const int rt = t / 3, pl = t % 3;
                    an[rt][pl] = *reinterpret_cast<const bf16x8*>(yb + pl * A.yb_plane + rt * rt16 + 32 * ii);
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
        };
        load_a(a0, 0);
        int i = 0;
        for (; i + 1 < nbm; i += 2) {
            step(i, a0, a1);
            step(i + 1, a1, a0);
        }
        if (i < nbm) step(i, a0, a1);
        if (CEN && ext) {
            // centred extension: acc -= dT Gb (blocks 0..3, B = -Gb) and acc -= T0 Hb (blocks 4..7, B = -Hb). A lane (lr,
            // lg) = row p, features 32f + 4lg + j (j < 4) and 32f + 16 + 4lg + j - 4 (j >= 4) of dT = Zt^ - T0 (formed
            // from the two images' planes: exact fp32 values, one rounded subtraction, an exact re-split) or of T0;
            // rows past P read 0
            const unsigned char* trow[2];
            const unsigned char* crow[2];
            bool pval[2];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int p = p0 + 16 * rt + lr;
                pval[rt] = p < A.P;
                const int pc = min(p, A.P - 1);
                const int64_t off = (int64_t)(pc / 32) * CONTRACT_SPLIT_BLOCK + (pc % 32) * bf6::PITCH;
                trow[rt] = A.timg + c * A.timg_cs + off;
                crow[rt] = A.ctimg + off;
            }
            auto load_ext_c = [&](int e, bf16x8 (&a)[2][3]) __attribute__((always_inline)) {
                const int f = e & 3;
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) {
                    bf16x4 lo[3], hi[3], clo[3], chi[3];
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) {
                        const int q = pl * GR_PL + 2 * (32 * f + 4 * lg);
                        clo[pl] = *reinterpret_cast<const bf16x4*>(crow[rt] + q);
                        chi[pl] = f < 3 ? *reinterpret_cast<const bf16x4*>(crow[rt] + q + 32) : bf16x4{};
                        if (e < 4) {
                            lo[pl] = *reinterpret_cast<const bf16x4*>(trow[rt] + q);
                            hi[pl] = f < 3 ? *reinterpret_cast<const bf16x4*>(trow[rt] + q + 32) : bf16x4{};
                        }
                    }
                    if (e < 4) {
                        const bf16x8 z[3] = {bf6::cat8(lo[0], hi[0]), bf6::cat8(lo[1], hi[1]), bf6::cat8(lo[2], hi[2])};
                        const bf16x8 r[3] = {bf6::cat8(clo[0], chi[0]), bf6::cat8(clo[1], chi[1]),
                                             bf6::cat8(clo[2], chi[2])};
                        delta_frag(z, r, a[rt]);
                    } else {
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) a[rt][pl] = bf6::cat8(clo[pl], chi[pl]);
                    }
                    if (!pval[rt]) {
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) a[rt][pl] = bf16x8{};
                    }
                }
            };
            load_ext_c(0, a0);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __syncthreads();
                if (e + 1 < 8) load_ext_c(e + 1, (e & 1) ? a0 : a1);
                mma_block(lds + ((nbm + e) % GR_NBUF) * GR_BLK, tro, (e & 1) ? a1 : a0, acc);
            }
        } else if (ext) {
            // extension: acc -= Zt^ Gb (B blocks hold -Gb); A lane (lr, lg) = Zt^[p][32e + 4lg + j] (j < 4) and
            // [32e + 16 + 4lg + j - 4] (j >= 4), two 8-B loads per plane from the trunk image row; rows past P read 0
            const unsigned char* trow[2];
            bool pval[2];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int p = p0 + 16 * rt + lr;
                pval[rt] = p < A.P;
                const int pc = min(p, A.P - 1);
                trow[rt] = A.timg + c * A.timg_cs + (int64_t)(pc / 32) * CONTRACT_SPLIT_BLOCK + (pc % 32) * bf6::PITCH;
            }
            // the A operand of extension block e + 1 loaded under block e's products (two register sets; loaded at
            // use, each of the four blocks waited out an L2 / HBM latency)
            auto load_ext = [&](int e, bf16x8 (&a)[2][3]) __attribute__((always_inline)) {
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) {
                        const unsigned char* q = trow[rt] + pl * GR_PL + 2 * (32 * e + 4 * lg);
                        bf16x4 lo = *reinterpret_cast<const bf16x4*>(q);
                        bf16x4 hi = e < 3 ? *reinterpret_cast<const bf16x4*>(q + 32) : bf16x4{};
                        if (!pval[rt]) lo = bf16x4{}, hi = bf16x4{};
                        a[rt][pl] = bf6::cat8(lo, hi);
                    }
            };
            load_ext(0, a0);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                __syncthreads();
                if (e + 1 < 4) load_ext(e + 1, (e & 1) ? a0 : a1);
                mma_block9(lds + ((nbm + e) % GR_NBUF) * GR_BLK, lds + GRB_P3 + e * GRAM_P3_BLOCK, tro, (e & 1) ? a1 : a0,
                           acc);
            }
        }
    }
    if (A.SB > 1) {
        // split-K: this split's tiles as they stand; k_gram_tt sums the SB slabs in fixed order and writes dZt
        if (wave == GR_CW) return;
        const int64_t sstride = (int64_t)GR_CW * 14 * 256;
        float* tp = A.tt_part + c * A.tt_cs + (int64_t)pt * A.SB * sstride + sb * sstride + (int64_t)wave * 14 * 256 +
                    4 * lane;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) *reinterpret_cast<f32x4*>(tp + (rt * 7 + t) * 256) = acc[rt][t];
        return;
    }
    if (wave == GR_CW) return;
    gram_tt_epilogue(A, c, pt, wave, lane, acc);
}

// ---------------------------------------------------------------------------------------------------------------
// k_gram_b2 (centred form, SB = 1, round 6): T_t units of TWO chains. Unit (pt, pair): chains c0 = 2 pair, c1 = c0 + 1,
// rows p0 = 256 pt + 32 w of wave w; the 8 waves stream the shared YB rows once for both chains (one A fragment feeds
// the two chains' products), the two chains' branch-image blocks share a ring slot (2 x 21 KB, 3 slots). No DMA wave:
// its 256-VGPR share holds the two chains' 112 accumulator registers, so the compute waves issue the block DMA
// themselves (42 one-KB pieces per block, q = w, w + 8, ...) right after the wait that retires the block before it
// -- wait_vmcnt0 at every block start: the builtin half tells hipcc every earlier load is retired (its own waits after
// it do not count the DMA issued next), the asm half covers the DMA it cannot see. A DMA issued at block i is retired
// by the wait of block i + 1 and read at block i + 2. The extension runs per chain (16 blocks: chain c0's dT Gb, T0 Hb,
// then c1's), A formed from the chain's trunk image and the centre's. Row groups [0, pt2): launch_gram sizes pt2 so
// these units fill whole rounds of the chip; k_gram_b takes the rest (and the dZb epilogue units).
// ---------------------------------------------------------------------------------------------------------------
constexpr int GB2_THREADS = 64 * GR_CW;
constexpr int GB2_SLOT = 2 * GR_BLK;
constexpr int GB2_LDS = GR_NBUF * GB2_SLOT;               // 126 KB
static_assert(GB2_LDS <= 160 * 1024, "k_gram_b2 LDS");

namespace {
// one 32-long k block of a wave's two 32 x 112 tiles (chains c0, c1: slot halves 0 / 1), the A fragment shared:
// B fragments of (tile, chain) step q + 1 read while step q's 12 MFMAs run
template <typename PRE>
__device__ __forceinline__ void mma_block2(const unsigned char* slot, int tro, const bf16x8 (&a)[2][3],
                                           f32x4 (&acc)[2][2][7], PRE pre) {
    bf16x8 b[2][3];
    load_b(slot, tro, 0, b[0]);
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        load_b(slot + GR_BLK, tro, t, b[1]);
        pre(t);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[0][rt][t] = six(a[rt], b[0], acc[0][rt][t]);
        if (t < 6) load_b(slot, tro, t + 1, b[0]);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[1][rt][t] = six(a[rt], b[1], acc[1][rt][t]);
    }
}
}  // namespace

__global__ __launch_bounds__(GB2_THREADS, 1) void k_gram_b2(GramArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int np = A.C / 2, n2 = A.pt2 * np, u2x = (n2 + 7) / 8;
    const int k = blockIdx.x >> 3, j = (blockIdx.x & 7) * u2x + k;   // XCD x: units [x u2x, (x + 1) u2x)
    if (k >= u2x || j >= n2) return;
    const int pt = j / np, c0 = 2 * (j - pt * np), c1 = c0 + 1;      // pairs minor: one YB slab per XCD at a time
    const bool on0 = !(A.sel && chain_bit(A.bits, c0)), on1 = !(A.sel && chain_bit(A.bits, c1));
    if (!on0 && !on1) return;                             // fit guard: both chains in the residual form
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int nbm = A.nblkN, nb = nbm + 16;
    const int p0 = 256 * pt + 32 * wave;
    const int tro = bf6::tr_lane_off(lr, lg);
    const unsigned char* bsrc0 = A.bimg + c0 * A.bimg_cs;
    const unsigned char* bsrc1 = A.bimg + c1 * A.bimg_cs;
    auto dma = [&](int i) __attribute__((always_inline)) {
        unsigned char* slot = lds + (i % GR_NBUF) * GB2_SLOT;
        if (i < nbm) {
            const unsigned char* s0 = bsrc0 + (int64_t)i * CONTRACT_SPLIT_BLOCK + lane * 16;
            const unsigned char* s1 = bsrc1 + (int64_t)i * CONTRACT_SPLIT_BLOCK + lane * 16;
            for (int q = wave; q < 2 * GR_PIECES; q += GR_CW)
                bf6::glds16_asm(q < GR_PIECES ? s0 + q * 1024 : s1 + (q - GR_PIECES) * 1024, slot + q * 1024);
        } else {
            // extension step s: chain s / 8, block e = s % 8 (-Gb blocks 0..3, then -Hb blocks 0..3)
            const int s = i - nbm, e = s & 7;
            const int c = s < 8 ? c0 : c1;
            const unsigned char* src = (e < 4 ? A.gbimg : A.hbimg) + c * A.gbimg_cs +
                                       (int64_t)(e & 3) * CONTRACT_SPLIT_BLOCK + lane * 16;
            for (int q = wave; q < GR_PIECES; q += GR_CW) bf6::glds16_asm(src + q * 1024, slot + q * 1024);
        }
    };
    f32x4 acc[2][2][7];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) acc[ch][rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __bf16* yb = A.yb + (int64_t)(p0 + lr) * A.yb_ld + 8 * lg;
    const int64_t rt16 = 16 * (int64_t)A.yb_ld;
    bf16x8 a0[2][3], a1[2][3];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a0[rt][pl] = *reinterpret_cast<const bf16x8*>(yb + pl * A.yb_plane + rt * rt16);
    dma(0);
    dma(1);
    bf6::wait_vmcnt0();                                   // block 0 is read after the first barrier: retire it before
    auto step = [&](int i, bf16x8 (&a)[2][3], bf16x8 (&an)[2][3]) __attribute__((always_inline)) {
        __syncthreads();                                  // every wave retired block i's pieces; slot (i + 2) % 3 free
        bf6::wait_vmcnt0();                               // A(i) and the pieces of block i + 1
        dma(i + 2);                                       // nb >= 18: always a block i + 2
        const int ii = min(i + 1, nbm - 1);
        mma_block2(lds + (i % GR_NBUF) * GB2_SLOT, tro, a, acc, [&](int t) __attribute__((always_inline)) {
            if (t < 6) {
                const int rt = t / 3, pl = t % 3;
                an[rt][pl] = *reinterpret_cast<const bf16x8*>(yb + pl * A.yb_plane + rt * rt16 + 32 * ii);
                __builtin_amdgcn_sched_barrier(0);
            }
        });
    };
    int i = 0;
    for (; i + 1 < nbm; i += 2) {
        step(i, a0, a1);
        step(i + 1, a1, a0);
    }
    if (i < nbm) step(i, a0, a1);
    // extension, per chain: acc[ch] -= dT Gb (blocks 0..3) and -= T0 Hb (blocks 4..7); A lane (lr, lg) = row p, features
    // 32f + 4lg + j (j < 4) and 32f + 16 + 4lg + j - 4 (j >= 4) of dT = Zt^ - T0 or of T0; rows past P read 0
    int64_t roff[2];
    bool pval[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int p = p0 + 16 * rt + lr;
        pval[rt] = p < A.P;
        const int pc = min(p, A.P - 1);
        roff[rt] = (int64_t)(pc / 32) * CONTRACT_SPLIT_BLOCK + (pc % 32) * bf6::PITCH;
    }
    // the A operand of extension step s + 1 is loaded (raw bf16 pieces) under step s's products and formed after step
    // s + 1's wait: formed at load time, hipcc's wait for the loads would also wait for the DMA issued after them
    struct ExtRaw {
        bf16x4 lo[2][3], hi[2][3], clo[2][3], chi[2][3];
    } raw;
    auto ext_load = [&](int s) __attribute__((always_inline)) {
        const int e = s & 7, f = e & 3;
        const unsigned char* tim = A.timg + (s < 8 ? c0 : c1) * A.timg_cs;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                const int64_t q = roff[rt] + pl * GR_PL + 2 * (32 * f + 4 * lg);
                raw.clo[rt][pl] = *reinterpret_cast<const bf16x4*>(A.ctimg + q);
                raw.chi[rt][pl] = f < 3 ? *reinterpret_cast<const bf16x4*>(A.ctimg + q + 32) : bf16x4{};
                if (e < 4) {
                    raw.lo[rt][pl] = *reinterpret_cast<const bf16x4*>(tim + q);
                    raw.hi[rt][pl] = f < 3 ? *reinterpret_cast<const bf16x4*>(tim + q + 32) : bf16x4{};
                }
            }
    };
    auto ext_form = [&](int s, bf16x8 (&a)[2][3]) __attribute__((always_inline)) {
        const int e = s & 7;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            if (e < 4) {
                bf16x8 z[3], r[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    z[pl] = bf6::cat8(raw.lo[rt][pl], raw.hi[rt][pl]);
                    r[pl] = bf6::cat8(raw.clo[rt][pl], raw.chi[rt][pl]);
                }
                delta_frag(z, r, a[rt]);
            } else {
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) a[rt][pl] = bf6::cat8(raw.clo[rt][pl], raw.chi[rt][pl]);
            }
            if (!pval[rt]) {
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) a[rt][pl] = bf16x8{};
            }
        }
    };
    ext_load(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int ie = nbm + s;
        __syncthreads();
        bf6::wait_vmcnt0();
        if (s + 2 < 16) dma(ie + 2);
        bf16x8 a[2][3];
        ext_form(s, a);
        if (s + 1 < 16) ext_load(s + 1);
        mma_block(lds + (ie % GR_NBUF) * GB2_SLOT, tro, a, acc[s >> 3]);
    }
    if (on0) gram_tt_epilogue(A, c0, pt, wave, lane, acc[0]);
    if (on1) gram_tt_epilogue(A, c1, pt, wave, lane, acc[1]);
}

__device__ __forceinline__ void gram_tt_epilogue(const GramArgs& A, int c, int pt, int wave, int lane,
                                                 const f32x4 (&acc)[2][7]) {
    const int lr = lane & 15, lg = lane >> 4;
    const int p0 = 256 * pt + 32 * wave;
    // dZt = -gscale acc
    const float sc = -A.gscale;
    float* out = A.dzt + c * A.dzt_cs;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int x = 16 * t + lr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = p0 + 16 * rt + 4 * lg + r;
                if (x < 100 && p < A.P) out[(int64_t)p * A.ldz + x] = sc * acc[rt][t][r];
            }
        }
    // d ll / d b0 = sum G = gscale (sum_{n,p} (S + b0) - sum y) = gscale (sum_v colsum_b[v] colsum_t[v] - sum y), all in
    // fp64 from the fp64 Gram slab sums (k_gram_sum) and the plan's sum y: the column-100 sum of acc (sum over p of
    // sum_n y[n][p] - Zt^ Gb, each ~sqrt(N) |y| / |S - y| larger than sum_n G[n][p]) was the Gram form's largest
    // error, 8.5e-3 absolute on a 16.6 derivative at fit 0.13 (~1e-3 of the gradient norm: profiles/r05d_gram_parts.txt).
    // One slot per chain carries it (slot 0; the statistics slice adds the PT * 8 slots).
    if (lane == 0) {
        double* st = A.stats + c * A.stats_cs + 2 * (int64_t)(pt * GR_CW + wave);
        double db = 0.0;
        if (pt == 0 && wave == 0) {
            const double* col = A.gcol + c * A.gcol_cs;
            double ss = 0.0;
            if (A.center) {
                // centred: sum (S + b0 - y) = sum_v (sum_n dB[n][v]) (sum_p Zt^[p][v]) + (sum_n B0[n][v]) (sum_p dT[p][v])
                // - sum y~, every term of the residual's size
                for (int v = 0; v <= 100; ++v) ss = fma(col[2 * 112 + v], col[112 + v], ss);
                for (int v = 0; v <= 100; ++v) ss = fma(A.ccol[v], col[3 * 112 + v], ss);
                db = (double)A.gscale * (ss - *A.cysum);
            } else {
                for (int v = 0; v <= 100; ++v) ss = fma(col[v], col[112 + v], ss);
                db = (double)A.gscale * (ss - *A.ysum);
            }
        }
        st[0] = 0.0;
        st[1] = db;
    }
}

// T_t split-K sum (few chains, SB > 1): one one-wave block per (256-row group pt, 32-row wave slot w, chain) sums
// its 14 tiles over the SB slabs in the order s = 0.. and runs the dZt epilogue. A launch of its own (k_gram_sum).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_gram_tt(GramArgs A) {
    const int pt = blockIdx.x >> 3, wave = blockIdx.x & 7, c = blockIdx.y, lane = threadIdx.x;
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int64_t sstride = (int64_t)GR_CW * 14 * 256;
    const float* tp = A.tt_part + c * A.tt_cs + (int64_t)pt * A.SB * sstride + (int64_t)wave * 14 * 256 + 4 * lane;
    f32x4 acc[2][7];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // slab-major: the 14 tile loads of one slab are issued together (a tile-major loop waited out one load latency
    // per (tile, slab): 24 us at one chain, profiles/r04q_c1_kstats.txt); per element the order is still s = 0..
    for (int ss = 0; ss < A.SB; ++ss) {
        f32x4 v[2][7];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) v[rt][t] = *reinterpret_cast<const f32x4*>(tp + ss * sstride + (rt * 7 + t) * 256);
        __builtin_amdgcn_sched_barrier(0);        // keep the 14 loads ahead of the adds (hipcc paired them)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 7; ++t) acc[rt][t] += v[rt][t];
    }
    gram_tt_epilogue(A, c, pt, wave, lane, acc);
}

// ---------------------------------------------------------------------------------------------------------------
// dZb epilogue unit (c, 32-row group m) of k_gram_b: dZb[n][x] = gscale (sum_{v <= 100} Zb^[n][v] Gt[v][x] - sum_s T_b[s][n][x]).
// Wave wv handles the group's accumulator tiles (rt, t) = wv, wv + 9, ... of 14, lane layout of the T_b slabs (rows
// 4lg + r, column lr). Gt (101 x 112) and Zb^T (101 x 32) staged in the workgroup's LDS ring.
// Both sums in fp64 (round 5): Zb^ Gt and sum_s T_b are each ~sqrt(P) |y| / |S - y| larger than their difference (the
// data term is coherent over the P points, the residual is not), so the fp32 running sum over v, rounded 101 times at
// the magnitude of Zb^ Gt, set the Gram form's gradient error (4.8e-4 of its norm at fit 0.13 in an fp32 emulation,
// 3e-5 with this sum exact: profiles/r05_gram_fit_table.json). The products of fp32 values are exact in fp64.
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ void dzb_unit(const GramArgs& A, int u, unsigned char* lds) {
    double* gts = reinterpret_cast<double*>(lds);                // Gt [101][112], fp64 (k_gram_sum's gt64)
    float* zbt = reinterpret_cast<float*>(gts + 101 * 112);      // Zb^T [101][32]
    const int ngroups = (A.N + 31) / 32;
    const int c = u / ngroups, m = u - c * ngroups;
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    // staging: every load of a thread issued before its first LDS store (a load -> store loop waited out one L2 / HBM
    // latency per trip: ~10 trips for the 90-KB fp64 Gt)
    const double* gt = A.gt64 + c * A.gt_cs2;
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    constexpr int GSL = (101 * 56 + GR_THREADS - 1) / GR_THREADS;       // 10 f64x2 per thread
    f64x2 gv[GSL];
#pragma unroll
    for (int k = 0; k < GSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 101 * 56 - 1);        // clamped slots rewrite the last pair
        const int v = e / 56, q = e - v * 56;
        gv[k] = *reinterpret_cast<const f64x2*>(gt + v * 112 + 2 * q);
    }
    const float* zb = A.zb + c * A.zb_cs;
    constexpr int ZSL = (32 * 101 + GR_THREADS - 1) / GR_THREADS;        // 6 per thread
    float zv[ZSL];
#pragma unroll
    for (int k = 0; k < ZSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 32 * 101 - 1);
        const int row = e / 101, v = e - row * 101, n = 32 * m + row;
        zv[k] = v < 100 ? zb[(int64_t)min(n, A.N - 1) * A.ldz + v] : 1.f;
        if (n >= A.N) zv[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < GSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 101 * 56 - 1);
        const int v = e / 56, q = e - v * 56;
        *reinterpret_cast<f64x2*>(gts + v * 112 + 2 * q) = gv[k];
    }
#pragma unroll
    for (int k = 0; k < ZSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 32 * 101 - 1);
        const int row = e / 101, v = e - row * 101;
        zbt[v * 32 + row] = zv[k];
    }
    __syncthreads();
    const int n32 = 32 * m, ng = n32 / 256, w8 = (n32 % 256) / 32;
    const bool pre = A.tb_sum != nullptr;                 // S > GRAM_TB_DIRECT: k_gram_sum added the slabs up
    const float* tb = (pre ? A.tb_sum + c * A.tbs_cs : A.tb_part + c * A.tb_cs) +
                      ((int64_t)(ng * GR_CW + w8) * 14) * 256 + 4 * lane;
    const int64_t sstride = (int64_t)A.NG * GR_CW * 14 * 256;
    const int nslab = pre ? 1 : A.S;
    float* out = A.dzb + c * A.dzb_cs;
    for (int tile = wv; tile < 14; tile += GR_THREADS / 64) {
        const int rt = tile / 7, t = tile - rt * 7;
        using acc_t = std::conditional_t<GRAM_DZB_FP64 != 0, double, float>;
        acc_t ts[4] = {0, 0, 0, 0};
        int ss = 0;
        for (; ss + 8 <= nslab; ss += 8) {                // eight slab loads in flight, then the adds in order
            f32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const f32x4*>(tb + (ss + k) * sstride + tile * 256);
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) ts[r] += (acc_t)v[k][r];
        }
        for (; ss < nslab; ++ss) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(tb + ss * sstride + tile * 256);
#pragma unroll
            for (int r = 0; r < 4; ++r) ts[r] += (acc_t)v[r];
        }
        acc_t gz[4] = {0, 0, 0, 0};
        const int x = 16 * t + lr;
        for (int v = 0; v < 101; ++v) {
            const f32x4 z = *reinterpret_cast<const f32x4*>(zbt + v * 32 + 16 * rt + 4 * lg);
            const acc_t g = (acc_t)gts[v * 112 + x];     // fp64 Gt (with GRAM_DZB_FP64 = 0 rounded to fp32)
#pragma unroll
            for (int r = 0; r < 4; ++r) gz[r] = fma((acc_t)z[r], g, gz[r]);
        }
        if (x < 100) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n32 + 16 * rt + 4 * lg + r;
                if (n < A.N) out[(int64_t)n * A.ldz + x] = (float)((acc_t)A.gscale * (gz[r] - ts[r]));
            }
        }
    }
}

// Centred dZb epilogue unit (c, 32-row group m): dZb[n][x] = gscale (sum_v dB[n][v] Gt[v][x] + B0[n][v] Ht[v][x]
// - sum_s T~_b[s][n][x]), dB = Zb^ - B0 (column 100: 1 - 1 = 0, B0[n][100] = 1), the T_b slabs over y~. LDS: Gt and Ht
// fp32 [101][112], dB^T and B0^T [101][32]. Both Gram terms are of the residual's size here, so their 202-term sum runs
// in fp32 (dzb_unit's fp64 guarded the uncentred Zb^ Gt, ~sqrt(P) |y| / |S - y| larger than the result); the T~_b
// slabs are added in fp64.
__device__ __forceinline__ void dzb_unit_c(const GramArgs& A, int u, unsigned char* lds) {
    float* gts = reinterpret_cast<float*>(lds);
    float* hts = gts + 101 * 112;
    float* dbt = hts + 101 * 112;
    float* b0t = dbt + 101 * 32;
    const int ngroups = (A.N + 31) / 32;
    const int c = u / ngroups, m = u - c * ngroups;
    if (A.sel && chain_bit(A.bits, c)) return;            // fit guard: residual form for this chain
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const float* gt = A.gt + c * A.gt_cs2;
    const float* ht = A.ht + c * A.gt_cs2;
    constexpr int HSL = (101 * 28 + GR_THREADS - 1) / GR_THREADS;       // f32x4 of Gt / Ht per thread
    constexpr int ZSL = (32 * 101 + GR_THREADS - 1) / GR_THREADS;
    f32x4 gv[HSL], hv[HSL];
#pragma unroll
    for (int k = 0; k < HSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 101 * 28 - 1);
        const int v = e / 28, q = e - v * 28;
        gv[k] = *reinterpret_cast<const f32x4*>(gt + v * 112 + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < HSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 101 * 28 - 1);
        const int v = e / 28, q = e - v * 28;
        hv[k] = *reinterpret_cast<const f32x4*>(ht + v * 112 + 4 * q);
    }
    const float* zb = A.zb + c * A.zb_cs;
    float dv[ZSL], bv[ZSL];
#pragma unroll
    for (int k = 0; k < ZSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 32 * 101 - 1);
        const int row = e / 101, v = e - row * 101, n = 32 * m + row;
        const int64_t o = (int64_t)min(n, A.N - 1) * A.ldz + min(v, 99);
        const float z = zb[o], b0 = A.cb0[o];
        dv[k] = v < 100 ? z - b0 : 0.f;
        bv[k] = v < 100 ? b0 : 1.f;
        if (n >= A.N) dv[k] = bv[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < HSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 101 * 28 - 1);
        const int v = e / 28, q = e - v * 28;
        *reinterpret_cast<f32x4*>(gts + v * 112 + 4 * q) = gv[k];
        *reinterpret_cast<f32x4*>(hts + v * 112 + 4 * q) = hv[k];
    }
#pragma unroll
    for (int k = 0; k < ZSL; ++k) {
        const int e = min(tid + GR_THREADS * k, 32 * 101 - 1);
        const int row = e / 101, v = e - row * 101;
        dbt[v * 32 + row] = dv[k];
        b0t[v * 32 + row] = bv[k];
    }
    __syncthreads();
    const int n32 = 32 * m, ng = n32 / 256, w8 = (n32 % 256) / 32;
    const bool pre = A.tb_sum != nullptr;
    const float* tb = (pre ? A.tb_sum + c * A.tbs_cs : A.tb_part + c * A.tb_cs) +
                      ((int64_t)(ng * GR_CW + w8) * 14) * 256 + 4 * lane;
    const int64_t sstride = (int64_t)A.NG * GR_CW * 14 * 256;
    const int nslab = pre ? 1 : A.S;
    float* out = A.dzb + c * A.dzb_cs;
    // tiles wv and wv + 9 (< 14) of the 2 x 7 accumulator tiles. Zb^ Gt + B0 Ht as exact f32 MFMAs (16x16x4: the products
    // of one instruction accumulate as a sequential fmaf chain over k, MI355X_MICROARCH.md): k step j takes v = 2j, 2j + 1
    // as (B0 Ht, dB Gt, B0 Ht, dB Gt) -- the order of the former VALU loop (per v: fma(b, h), then fma(d, g)), so the
    // same roundings, bit for bit (profiles/r06o_dzb_mfma_ab.txt); 51 dependent MFMAs per tile, two tiles' chains
    // interleaved. The units' time is their staging loads, not these products: 46.6 -> 46.0 us for all 512 units
    constexpr int NWV = GR_THREADS / 64;
    const bool two = wv + NWV < 14;
    const float* asrc = (lg & 1) ? dbt : b0t;
    const float* bsrc = (lg & 1) ? gts : hts;
    double ts[2][4];
    int tl[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int tile = min(wv + NWV * q, 13);
        tl[q] = tile;
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[q][r] = 0.0;
        if (q == 1 && !two) continue;
        int ss = 0;
        for (; ss + 8 <= nslab; ss += 8) {
            f32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const f32x4*>(tb + (ss + k) * sstride + tile * 256);
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) ts[q][r] += (double)v[k][r];
        }
        for (; ss < nslab; ++ss) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(tb + ss * sstride + tile * 256);
#pragma unroll
            for (int r = 0; r < 4; ++r) ts[q][r] += (double)v[r];
        }
    }
    f32x4 gz[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int ao[2] = {16 * (tl[0] / 7) + lr, 16 * (tl[1] / 7) + lr};
    const int bo[2] = {16 * (tl[0] % 7) + lr, 16 * (tl[1] % 7) + lr};
    for (int j = 0; j < 51; ++j) {
        const int v = 2 * j + (lg >> 1);
        const bool vok = v < 101;
        const int vc = min(v, 100);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q == 1 && !two) break;
            const float av = vok ? asrc[vc * 32 + ao[q]] : 0.f;
            const float bv = vok ? bsrc[vc * 112 + bo[q]] : 0.f;
            gz[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, gz[q], 0, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        if (q == 1 && !two) break;
        const int rt = tl[q] / 7, t = tl[q] - rt * 7;
        const int x = 16 * t + lr;
        if (x < 100) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n32 + 16 * rt + 4 * lg + r;
                if (n < A.N) out[(int64_t)n * A.ldz + x] = (float)((double)A.gscale * ((double)gz[q][r] - ts[q][r]));
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Pre-split data images (once per plan / data change): YA = y [n][p] (k = p blocks in kpos order), YB = y^T [p][n]
// (k = n blocks). Padding rows / columns stay zero (the plan zeroes the allocation).
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gram_yimg(const float* y, int N, int P, __bf16* ya, int64_t ya_plane, int ya_ld,
                                                   __bf16* yb, int64_t yb_plane, int yb_ld) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)N * P) return;
    const int n = (int)(e / P), p = (int)(e - (int64_t)n * P);
    const float x = y[e];
    const __bf16 a = (__bf16)x;
    const float r = x - (float)a;
    const __bf16 b = (__bf16)r;
    const __bf16 cc = (__bf16)(r - (float)b);
    const int64_t ia = (int64_t)n * ya_ld + 32 * (p / 32) + kpos(p % 32);
    ya[ia] = a;
    ya[ia + ya_plane] = b;
    ya[ia + 2 * ya_plane] = cc;
    const int64_t ib = (int64_t)p * yb_ld + 32 * (n / 32) + kpos(n % 32);
    yb[ib] = a;
    yb[ib + yb_plane] = b;
    yb[ib + 2 * yb_plane] = cc;
}

// ---------------------------------------------------------------------------------------------------------------
// Centred data (once per plan / data change, gram_center): yc[n][p] = y[n][p] - (sum_v B0[n][v] T0[p][v] + b0), the
// products and sums in fp64 (exact products of fp32 values), rounded once; 64 x 64 output tiles, B0 / T0 rows staged
// in LDS. Block (0, 0) also writes col[v] = sum_n B0[n][v] in fp64 (v < W), col[W] = N.
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_center_y(const float* y, const float* B0, const float* T0, const float* b0p, int N,
                                                  int P, int W, int ldz, float* yc, double* col) {
    __shared__ float bs[64][101];
    __shared__ float ts[64][101];
    const int p0 = blockIdx.x * 64, n0 = blockIdx.y * 64, tid = threadIdx.x;
    for (int e = tid; e < 64 * W; e += 256) {
        const int r = e / W, v = e - r * W;
        bs[r][v] = n0 + r < N ? B0[(int64_t)(n0 + r) * ldz + v] : 0.f;
        ts[r][v] = p0 + r < P ? T0[(int64_t)(p0 + r) * ldz + v] : 0.f;
    }
    __syncthreads();
    const int tx = tid & 15, ty = tid >> 4;                  // 4 x 4 outputs: n = n0 + ty + 16 i, p = p0 + tx + 16 j
    double acc[4][4] = {};
    for (int v = 0; v < W; ++v) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = bs[ty + 16 * i][v], b[i] = ts[tx + 16 * i][v];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
    }
    const double bb = (double)*b0p;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + ty + 16 * i, p = p0 + tx + 16 * j;
            if (n < N && p < P) {
                const int64_t e = (int64_t)n * P + p;
                yc[e] = (float)((double)y[e] - (acc[i][j] + bb));
            }
        }
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid <= W) {
        double sum = 0.0;
        if (tid < W)
            for (int n = 0; n < N; ++n) sum += (double)B0[(int64_t)n * ldz + tid];
        else sum = (double)N;
        col[tid] = sum;
    }
}

hipError_t launch_center_y(const float* y, const float* B0, const float* T0, const float* b0, int N, int P, int W,
                           int ldz, float* yc, double* col, hipStream_t s) {
    if (W < 1 || W > 101 || W >= 112) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_center_y, dim3((P + 63) / 64, (N + 63) / 64), dim3(256), 0, s, y, B0, T0, b0, N, P, W, ldz, yc,
                       col);
    return hipGetLastError();
}

hipError_t launch_gram_aug(const GramArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gram_aug, dim3((a.N + a.P + 255) / 256, a.C), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gram_yimg(const float* y, int N, int P, __bf16* ya, int64_t ya_plane, int ya_ld, __bf16* yb,
                            int64_t yb_plane, int yb_ld, hipStream_t s) {
    const int64_t n = (int64_t)N * P;
    hipLaunchKernelGGL(k_gram_yimg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, N, P, ya, ya_plane, ya_ld, yb,
                       yb_plane, yb_ld);
    return hipGetLastError();
}


#if GR_STAMP
extern "C" int vihmc_debug_gram_stamps(void* stamps, size_t stamp_bytes, void* real, size_t real_bytes) {
    if (stamp_bytes != sizeof(gr_stamps) || real_bytes != sizeof(gr_real)) return -1;
    hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(gr_stamps), stamp_bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(real, HIP_SYMBOL(gr_real), real_bytes, 0, hipMemcpyDeviceToHost);
    return (int)e;
}
#endif


hipError_t launch_gram(const GramArgs& a0, hipStream_t s) {
    GramArgs a = a0;
    if (a.ya_ld % 8 || a.yb_ld % 8 || a.NG * 256 < a.N || a.PT * 256 < a.P || a.nblkN * 32 < a.N ||
        a.nblkP * 32 < a.P || a.S * a.SL < a.nblkP || a.C < 1)
        return hipErrorInvalidValue;
    if (a.SB < 1 || a.SLB < 1 || a.SB * a.SLB < a.nblkN || (a.SB - 1) * a.SLB >= a.nblkN || (a.SB > 1 && !a.tt_part))
        return hipErrorInvalidValue;
    if (a.St < 1 || a.SLt < 1 || a.St * a.SLt < a.nblkP || (a.St - 1) * a.SLt >= a.nblkP) return hipErrorInvalidValue;
    if (a.Sb < 1 || a.SLb < 1 || a.Sb * a.SLb < a.nblkN || (a.Sb - 1) * a.SLb >= a.nblkN || !a.gb_part)
        return hipErrorInvalidValue;
    if (a.S > GRAM_TB_DIRECT ? !a.tb_sum : a.tb_sum != nullptr) return hipErrorInvalidValue;
    if (a.center && (!a.cbimg || !a.ctimg || !a.cb0 || !a.ccol || !a.cysum || !a.ht_part || !a.hb_part || !a.ht ||
                     !a.hbimg || !a.hb3img))
        return hipErrorInvalidValue;
    // the T_b units take the Gram-t tiles (one per wave) when a slab has >= 4 of them (>= 32 waves for 28 tiles);
    // fewer n groups keep the Gram-t units (two or four tiles per T_b wave spill registers). Centred: the Gram units
    // stream the centre's image beside the outputs' and compute G with H (Gram-t units of their own)
    const int gt = a.NG >= 4 && !a.center ? 1 : 0;
    if (gt && (a.St != a.S || a.SLt != a.SL)) return hipErrorInvalidValue;   // the Gram-t tiles ride the T_b slabs
    const int n1 = a.NG * a.S * a.C, n2 = a.C * ((gt ? 0 : a.St) + a.Sb);
    a.upx_a = (n1 + 7) / 8;
    const int gpx = (n2 + 7) / 8;
    // two-chain T_t units (k_gram_b2): the row-group count pt2 minimising the rounds of the two launches' T_t units (a
    // two-chain unit costs GRAM_B2_RATIO one-chain units; ties: the most pairs)
    a.pt2 = 0;
    if (a.pair2 == 2 && a.center && a.SB == 1 && a.C >= 2 && a.C % 2 == 0) a.pt2 = a.PT;   // tests: every row group
    else if (a.pair2 && a.center && a.SB == 1 && a.C >= 2 && a.C % 2 == 0) {
        double best = 1e30;
        for (int g = 0; g <= a.PT; ++g) {
            const int u2x = (g * (a.C / 2) + 7) / 8, u1x = ((a.PT - g) * a.C + 7) / 8;
            const double cost = GRAM_B2_RATIO * ((u2x + 31) / 32) + (u1x + 31) / 32;
            if (cost <= best) best = cost, a.pt2 = g;
        }
    }
    a.upx_b = ((a.PT - a.pt2) * a.SB * a.C + 7) / 8;
    const int cpx = (a.C * ((a.N + 31) / 32) + 7) / 8;
    if (!a.aug_done) hipLaunchKernelGGL(k_gram_aug, dim3((a.N + a.P + 255) / 256, a.C), dim3(256), 0, s, a);
    const dim3 ga(8 * (a.upx_a + gpx));
    if (gt) hipLaunchKernelGGL(k_gram_a<1>, ga, dim3(GR_THREADS), GR_LDS, s, a);
    else hipLaunchKernelGGL(k_gram_a<0>, ga, dim3(GR_THREADS), a.center ? GR_LDS_C : GR_LDS, s, a);
    hipLaunchKernelGGL(k_gram_sum, dim3(56 + (a.center ? 98 : 0) + (a.tb_sum ? a.NG * 28 : 0), a.C), dim3(256), 0, s, a);
    if (a.pt2 > 0)
        hipLaunchKernelGGL(k_gram_b2, dim3(8 * ((a.pt2 * (a.C / 2) + 7) / 8)), dim3(GB2_THREADS), GB2_LDS, s, a);
    if (a.center) hipLaunchKernelGGL(k_gram_b<1>, dim3(8 * (a.upx_b + cpx)), dim3(GR_THREADS), GRB_LDS_C, s, a);
    else hipLaunchKernelGGL(k_gram_b<0>, dim3(8 * (a.upx_b + cpx)), dim3(GR_THREADS), GRB_LDS, s, a);
    if (a.SB > 1) hipLaunchKernelGGL(k_gram_tt, dim3(a.PT * GR_CW, a.C), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace vihmc
