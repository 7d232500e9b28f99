// Internal declarations shared by the kernels (vihmc_kernels.hip) and the plan / C-ABI layer
// (vihmc_plan.hip). Nothing here crosses the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "vihmc_diag.h"

namespace vihmc {

enum { ACT_ID = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_SINE = 3 };

// tanh of the DeepONet layer epilogues (fused forward, row-dot input layers): <= 0.9 ulp below |x| = 0.625, ~1-2 ulp
// above (v_exp_f32 / v_rcp_f32), and UNBIASED -- the contraction sums 10^4-10^7 products of these outputs, so a
// systematic error adds up where a random one averages out. Until round 5 the epilogues used (1 - t) / (1 + t),
// t = exp(-2|x|): absolute error ~6e-8 near 0 (2e4 ulp at |x| ~ 1e-3) and a -0.08-ulp bias from log2(e) rounded to
// fp32; at a good fit the likelihood gradient came out ~50x the reference's own fp32 error.
//   |x| < 0.625: x + x^3 P(x^2), P of degree 4 fitted to tanh with each fp32 coefficient chosen for zero mean error
//   else:        1 - 2 t / (1 + t), t = 2^(-2 log2(e) |x|) <= 0.287, log2(e) as two fp32 parts in one fma
__device__ __forceinline__ float tanh_acc(float x) {
    const float ax = fabsf(x);
    const float u = x * x;
    float p = fmaf(u, -0.005816340912133455f, 0.020738132297992706f);
    p = fmaf(u, p, -0.053769949823617935f);
    p = fmaf(u, p, 0.13331805169582367f);
    p = fmaf(u, p, -0.33333295583724976f);
    const float small = fmaf(x * u, p, x);
    const float t = __builtin_amdgcn_exp2f(fmaf(ax, -2.885390043258667f, ax * -3.851926067000022e-08f));
    const float big = copysignf(fmaf(-2.f, t * __builtin_amdgcn_rcpf(1.f + t), 1.f), x);
    return ax < 0.625f ? small : big;
}
// tanh correctly rounded to fp32 (all but ~1 in 10^6 arguments, where the fp64 value lies within 2^-44 of a rounding
// midpoint): tanh(a) = em / (em + 2), em = expm1(2a) evaluated in fp64 (Cody-Waite reduction 2a = k ln2 + r,
// |r| <= ln2 / 2, expm1(r) to r^11, 2^k expm1(r) + (2^k - 1)), the quotient from v_rcp_f64 with one correction. The
// epilogue of each net's LAST hidden layer (plan option tanh_cr, round 6): the output layer is linear, so that layer's
// rounding reaches Z, and through the N x P contraction S - y, without an averaging nonlinearity in between -- and
// tanh_acc's rounding, although unbiased over [-inf, inf], is a smooth function of the argument, so over a smooth grid of
// 10^4 trunk points its local bias adds up coherently: the reference's fp32 closure with tanh_acc in that one layer
// has 3.4x its gradient error against fp64 at fit 1.5e-3, with tanh_acc in the other seven layers 1.0x
// (profiles/r06_tanh_layers.txt). ~25 fp64 instructions.
__device__ __forceinline__ float tanh_cr(float x) {
    const double a = fmin(fabs((double)x), 20.0);
    const double u = 2.0 * a;
    const double k = __builtin_rint(u * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, u);      // ln2_hi (32 significant bits: k ln2_hi exact)
    r = fma(-k, 1.90821492927058770002e-10, r);             // ln2_lo
    double p = 2.505210838544172e-08;                       // 1/11!
    p = fma(p, r, 2.755731922398589e-07);
    p = fma(p, r, 2.7557319223985893e-06);
    p = fma(p, r, 2.48015873015873e-05);
    p = fma(p, r, 1.984126984126984e-04);
    p = fma(p, r, 1.388888888888889e-03);
    p = fma(p, r, 8.333333333333333e-03);
    p = fma(p, r, 4.1666666666666664e-02);
    p = fma(p, r, 1.6666666666666666e-01);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    const double s = __builtin_ldexp(1.0, (int)k);
    const double em = fma(s, p * r, s - 1.0);
    const double den = em + 2.0;
    const double rc = __builtin_amdgcn_rcp(den);
    const double y0 = em * rc;
    const double y = fma(fma(-y0, den, em), rc, y0);
    return copysignf((float)y, x);
}
// forward-epilogue activation code of a layer whose tanh is tanh_cr (the plans set it on each net's last hidden layer;
// the backward treats it as ACT_TANH)
enum { ACT_TANH_CR = 4 };
enum { MODE_FWD = 0, MODE_BWD = 1 };

// contraction geometry (vihmc_contract.hip): 4 waves x 32 owner rows per workgroup, 16-row Q chunks
constexpr int CONTRACT_OWN_PER_WG = 128;
constexpr int CONTRACT_QC = 16;
constexpr int CONTRACT_SPLIT_ROWS = 32;      // rows per block of the pre-split (bf16x6) contraction image
constexpr int CONTRACT_SPLIT_BLOCK = 22528;  // bytes per block: 3 x [32][112] bf16 + [32][4] fp32, padded
// row-dot geometry (vihmc_layers.hip): 4 waves per workgroup, 16*MS rows per wave
constexpr int ROWDOT_WAVES = 4;

// ---------------------------------------------------------------------------------------------
// Row-dot GEMM: O[m][n] = epilogue( sum_k A[m][k] * B[n][k] ), both operands row-major with the
// contraction index contiguous. Used for every forward layer (A = activations, B = W[n_out][n_in])
// and for the backward input-gradient (A = delta, B = W^T[n_in][n_out]).
//   FWD epilogue: O = act(acc + bias[n])
//   BWD epilogue: O = acc * act'(H[m][n])      (H = the stored activation of the layer below)
// Columns [Nn, ldo) of O are written as zeros so the next GEMM can read whole 4-float groups.
// ---------------------------------------------------------------------------------------------
struct RowdotProb {
    const float* A; int64_t a_cs; int32_t lda;
    const float* B; int64_t b_cs; int32_t ldb;
    float* O;       int64_t o_cs; int32_t ldo;
    const float* bias; int64_t bias_cs;
    const float* H; int64_t h_cs; int32_t ldh;
    int32_t M, Nn, K, act;
    int32_t tiles;          // workgroups per chain = ceil(ntiles / tpw)
    int32_t ntiles;         // ceil(M / (ROWDOT_WAVES*16*MS)) row tiles
    int32_t tpw;            // row tiles per workgroup (amortises the LDS weight staging)
};
struct RowdotArgs {
    RowdotProb p[2];
    int32_t nprob, C;
    int32_t ms0;            // row sub-tiles per wave of problem 0 when it differs from the launch's (input layers)
};

// ---------------------------------------------------------------------------------------------
// Column-sum GEMM for weight gradients: part[chunk][n][j] = sum_{m in chunk} D[m][n] * H[m][j],
// plus the bias gradient part[chunk][n_out*ldh + n] = sum_m D[m][n]. One partial per row chunk,
// reduced in fixed order by k_reduce_partials (deterministic, no atomics).
// ---------------------------------------------------------------------------------------------


// ---------------------------------------------------------------------------------------------
// Fused backward of one linear layer l (grouped branch + trunk):
//   Dout = (D W) * act'(H)        (D = delta_l [M][ldd], W^T = WT [n_in][ldw], H = h_{l-1} [M][ldh])
//   part[wg] = D^T H (weight gradient partial) and sum_rows D (bias gradient partial)
// One 256-thread workgroup per rows_per_wg rows; D and H are staged in LDS in 32-row sub-tiles (read
// once from HBM for both products), W^T is staged once per workgroup.
// ---------------------------------------------------------------------------------------------
constexpr int BWD_SUB = 32;

constexpr int GATHER_SPLIT_MAX = 256;
struct BwdProb {
    const float* D;  int64_t d_cs;  int32_t ldd;
    const float* WT; int64_t wt_cs; int32_t ldw;
    const float* H;  int64_t h_cs;  int32_t ldh;
    float* Dout;     int64_t o_cs;
    float* part;     int64_t part_cs; int32_t part_stride;
    int32_t M, n_out, n_in, act, has_dx;
    int32_t rows_per_wg, n_wg;
};
struct BwdArgs {
    BwdProb p[2];
    int32_t nprob, C;
};
hipError_t launch_bwd(const BwdArgs& a, int nti, hipStream_t s);
bool bwd_bf_ok(const BwdArgs& a);                       // k_bwd_bf handles every problem of the launch
hipError_t launch_bwd_bf(const BwdArgs& a, hipStream_t s);

// Whole-network backward in one launch for chunks of 64 rows (vihmc_bwd_chain.hip): every layer of both nets,
// the deltas on chip, the same partial slabs as the per-layer k_bwd_bf2 launches. W_j^T from the pre-split W^T
// image of layer j (BWD_WTIMG layout, index j - 1 of the net's images).
constexpr int BWD_CHAIN_MAXL = 12;
struct BwdChainLayer {
    const float* H; int64_t h_cs; int32_t ldh;    // h_{j-1} rows (j >= 1) or the net input (j = 0)
    int32_t n_in, n_out;
    int32_t act;                                  // activation of layer j - 1 (j >= 1)
    int64_t part_off; int32_t part_stride;        // layer j's partial slabs inside the net's dwpart
};
struct BwdChainNet {
    BwdChainLayer L[BWD_CHAIN_MAXL];
    int32_t nl, M, n_wg;                          // n_wg = ceil(M / 64) workgroups per chain
    int32_t tanh_all;                             // every layer j >= 1 has a tanh below it (compile-time act')
    const float* D; int64_t d_cs; int32_t ldd;    // delta of the top layer (dZ) [M][ldd]
    float* dwpart; int64_t dwpart_cs;
    const unsigned char* wtimg; int64_t wtimg_cs; // the net's W^T images (layers 1 .. nl - 1)
};
struct BwdChainArgs {
    BwdChainNet net[2];
    int32_t C;
};
bool bwd_chain_ok(const BwdChainArgs& a);
hipError_t launch_bwd_chain(const BwdChainArgs& a, hipStream_t s);
int bwd_chain_rows();

// ---------------------------------------------------------------------------------------------
// Fused branch x trunk contraction with the Gaussian likelihood, owner form.
//   S[q][o] = sum_k Q[q][k] * Own[o][k] + b0;  r = S - Y[q][o];  G = gscale * r
//   dOwn[o][j] = sum_q G[q][o] * Q[q][j]            (WITH_GRAD)
// The wave owns 32 rows of `Own` and streams `Q` in 16-row steps; S is never stored.
// Side A: Own = Z_trunk [P], Q = Z_branch [N], Y = y [N][P]   -> dZ_trunk (complete) + sum r^2, sum G
// Side B: Own = Z_branch [N], Q = Z_trunk chunk, Y = G^T [P][N] written by side A (load_g: no S
//         recompute; y^T with load_g = 0) -> dZ_branch partial per chunk
// Forward-only (predict) writes out[q][o] = S into `out` (side A, o = p contiguous).
// ---------------------------------------------------------------------------------------------
// Gram-form fit guard (vihmc_plan.hip, plan option gram_guard): per-chain selection of the contraction form in a
// gradient-only evaluation. Bit c set: chain c runs the residual form (k_contract_bf + k_contract_bf_b + reduce);
// clear: the Gram form. The selection is a launch argument, so every kernel sees it without a memory read.
constexpr int GUARD_MAXC = 256;
struct ChainBits {
    uint32_t w[GUARD_MAXC / 32];
};
__host__ __device__ inline bool chain_bit(const ChainBits& b, int c) {
    return c < GUARD_MAXC && ((b.w[c >> 5] >> (c & 31)) & 1u) != 0u;
}

struct ContractProb {
    const float* Own; int64_t own_cs; int32_t ldown;
    const float* Q;   int64_t q_cs;   int32_t ldq;
    const float* Y;   int32_t ldy; int64_t y_cs;   // y_cs = 0: targets shared by all chains
    float* gout;      int64_t gout_cs; int32_t ldg;  // side A (optional): G^T[o][q] written for side B
    const float* b0;  int64_t b0_cs;
    float* out;       int64_t out_cs; int32_t ldout; int64_t out_chunk_stride;
    double* stats;    int64_t stats_cs;   // 2 doubles per wave (sum r^2, sum G) when with_stats
                                          // (4 waves per workgroup, index ((qc*o_tiles+og)*4+wave))
    int32_t Mo, Mq, W;
    int32_t o_tiles, q_chunks, q_per_chunk;   // o_tiles = ceil(Mo / CONTRACT_OWN_PER_WG)
    int32_t with_stats, write_s;
    int32_t load_g;                       // side B: Y holds G (already scaled); no S recompute
    int32_t masked;                       // side A: a NaN target marks an excluded (row, point) pair (residual 0)
    int32_t xcd_group;                    // 1: the o_tiles workgroups sharing one Q chunk run on one XCD
                                          //    (requires C * q_chunks % 8 == 0; speed only)
    int32_t bf16x6;                       // side A, W = 100: products on the bf16 MFMA, 3-way split
                                          //    operands, six products (k_contract_bf)
    const unsigned char* qimg; int64_t qimg_cs;   // bf16x6: Q pre-split into blocks (launch_split_blocks)
    float gscale;
    int32_t sel; ChainBits bits;          // sel = 1: only the chains whose bit is set (the others' workgroups exit)
};

// ---------------------------------------------------------------------------------------------
// Gradient-only contraction in Gram form (vihmc_gram.hip): dZ_b and dZ_t from y Zt^, y^T Zb^ and the two
// 101 x 101 Gram matrices of the augmented outputs Zb^ = [Z_b | 1], Zt^ = [Z_t | b0]; no residual, no G^T.
// ---------------------------------------------------------------------------------------------
struct GramArgs {
    unsigned char* bimg; int64_t bimg_cs; int32_t nblkN;   // branch outputs, pre-split blocks (qsplitA)
    unsigned char* timg; int64_t timg_cs; int32_t nblkP;   // trunk outputs, pre-split blocks (qsplitB)
    const __bf16* ya; int64_t ya_plane; int32_t ya_ld;     // y [NG*256 rows n][32 nblkP], 3 planes, kpos order
    const __bf16* yb; int64_t yb_plane; int32_t yb_ld;     // y^T [PT*256 rows p][32 nblkN], 3 planes
    float* tb_part; int64_t tb_cs;                         // [C][S][NG][8 waves][14 tiles][256]
    double* gt_part; int64_t gt_cs;                        // [C][St][28 tiles][256] (fp64 slab sums)
    double* gb_part; int64_t gb_cs; int32_t Sb, SLb;       // [C][Sb][28 tiles][256] Gram-b slabs of SLb branch blocks
    float* tb_sum; int64_t tbs_cs;                         // [C][NG][8][14][256] sum of the S T_b slabs (S > 8), else null
    float* gt; int64_t gt_cs2;                             // [C][112][112] Zt^T Zt^
    double* gt64;                                          // [C][112][112] the same in fp64 (dZb epilogue), gt_cs2
    unsigned char* gb3img;                                 // [C][4][GRAM_P3_BLOCK]: 4th bf16 plane of -Gb
    unsigned char* gbimg; int64_t gbimg_cs;                // [C][4 blocks] -Zb^T Zb^ pre-split
    const float* zb; int64_t zb_cs;                        // fp32 Z_b rows [N][ldz]
    float* dzb; int64_t dzb_cs;                            // dZ_b [N][ldz]
    float* dzt; int64_t dzt_cs;                            // dZ_t [P][ldz]
    double* stats; int64_t stats_cs;                       // (0, sum G) pairs, PT * 8 per chain (slot 0: d ll / d b0)
    double* gcol; int64_t gcol_cs;                         // [C][2][112] fp64 column sums of Zb^ (Gb[v][100]), Zt^ (Gt[v][101])
    const double* ysum;                                    // sum y (fp64, with sum y^2 by k_ysq)
    const float* b0; int64_t b0_cs;
    int32_t N, P, ldz, NG, S, SL, PT, C;
    int32_t St, SLt;                                       // Gram-t split of the trunk blocks (gt_part: St slabs)
    // split-K of T_t = y^T Zb^ over the branch blocks (SB splits of SLB blocks; the last also runs the 4 extension
    // blocks): SB > 1 writes partial slabs tt_part [C][PT][SB][8 waves][14 tiles][256] and k_gram_tt (a launch of its
    // own) sums them in order s = 0.. and writes dZt
    int32_t SB, SLB;
    float* tt_part; int64_t tt_cs;
    int32_t upx_a, upx_b;                                  // set by launch_gram
    // two-chain T_t units (k_gram_b2, round 6): row groups [0, pt2) of chain pairs (2c, 2c + 1) run there; k_gram_b
    // takes the row groups [pt2, PT) of every chain. Set by launch_gram (pair2 = 0: k_gram_b alone)
    int32_t pair2, pt2;
    int32_t aug_done;                                      // feature 100 of both images already written
    float gscale;
    int32_t sel; ChainBits bits;                           // sel = 1: chains whose bit is set exit (residual form)
    // Centred data (plan option gram_center, round 6): y = S0 + y~ with S0 = B0 T0^T the output at the plan's centre
    // weights (the frozen vector); ya / yb then hold y~, and with dB = Zb^ - B0, dT = Zt^ - T0
    //     dZb^ = gscale (dB Gt + B0 Ht - y~ Zt^),   Ht = dT^T Zt^
    //     dZt^ = gscale (dT Gb + T0 Hb - y~^T Zb^), Hb = dB^T Zb^
    // every term of the size of the residual, not of y. center = 0: the uncentred form above.
    int32_t center;
    const unsigned char* cbimg;                            // B0 pre-split image (one chain's qsplitA layout)
    const unsigned char* ctimg;                            // T0 pre-split image (one chain's qsplitB layout)
    const float* cb0;                                      // B0 fp32 rows [N][ldz]
    const double* ccol;                                    // [112] sum_n B0[n][v] (fp64)
    const double* cysum;                                   // sum y~ (fp64)
    float* ht_part; int64_t ht_cs;                         // [C][St][49 tiles][256] Ht slabs (fp32 per slab)
    float* hb_part; int64_t hb_cs;                         // [C][Sb][49 tiles][256] Hb slabs
    float* ht;                                             // [C][112][112] Ht (fp32, gt_cs2)
    unsigned char* hbimg;                                  // [C][4 blocks] -Hb pre-split (gbimg_cs)
    unsigned char* hb3img;                                 // [C][4][GRAM_P3_BLOCK]: 4th bf16 plane of -Hb
};
constexpr int GRAM_P3_BLOCK = 32 * 224;   // bytes of one 32-row plane of a pre-split block (the 4th plane of -Gb)
constexpr int GRAM_TB_DIRECT = 8;   // up to this many T_b slabs the dZb epilogue units sum them themselves
hipError_t launch_gram(const GramArgs& a, hipStream_t s);
// feature 100 (and trunk feature 101) of the pre-split output images of a.C chains (k_gram_aug)
hipError_t launch_gram_aug(const GramArgs& a, hipStream_t s);
// the centred data y~ = y - (B0 T0^T + b0) in fp64, rounded once (B0 [N][ldz], T0 [P][ldz] fp32 rows, b0 at *b0),
// and col[v] = sum_n B0[n][v] (v < W; col[W] = N) in fp64
hipError_t launch_center_y(const float* y, const float* B0, const float* T0, const float* b0, int N, int P, int W,
                           int ldz, float* yc, double* col, hipStream_t s);
hipError_t launch_gram_yimg(const float* y, int N, int P, __bf16* ya, int64_t ya_plane, int ya_ld, __bf16* yb,
                            int64_t yb_plane, int yb_ld, hipStream_t s);

// launchers (vihmc_kernels.hip)
hipError_t launch_rowdot(const RowdotArgs& a, int nt, int ms, int mode, hipStream_t s);
// The grouped input-layer launch (branch K = 101 on the whole-tile KF = 104 path, trunk run-time K) applies:
// problem 0 may then use its own row sub-tiles per wave (RowdotArgs::ms0).
bool rowdot_in_ok(const RowdotArgs& a, int nt);
hipError_t launch_contract(const ContractProb& p, int C, bool with_grad, hipStream_t s);
hipError_t launch_contract_bf(const ContractProb& p, int C, hipStream_t s);
hipError_t launch_contract_bf_b(const ContractProb& p, int C, hipStream_t s);
constexpr int CONTRACT_BF_B_OWN = 256;       // side-B bf16x6 owner rows per workgroup
hipError_t launch_split_blocks(const float* src, int64_t src_cs, int ld, int rows, unsigned char* dst,
                               int64_t dst_cs, int C, hipStream_t s);
size_t contract_lds_bytes(int W);
hipError_t launch_init_packed(float* packed, int64_t dp, int C, const float* frozen, const int32_t* map_w,
                              const int32_t* map_wt, int64_t D, hipStream_t s);
// Optional: the bf16x6 forward's pre-split weight images kept current by the scatter itself (plane triple and the
// fp32 copies -- k tail or bias -- of every sampled weight of a fused layer), so they are split from the full
// weights only once per plan instead of once per evaluation (k_split_wimg). img_w / img_f: byte offsets inside a
// chain's image region, -1 = none; null maps: packed only.
struct ScatterImg {
    unsigned char* img; int64_t img_cs; const int32_t* img_w; const int32_t* img_f; int32_t plane;  // plane stride (B)
    // the backward's transposed images (BWD_WTIMG bytes per fused layer): W^T planes and the fp32 n tail
    unsigned char* timg; int64_t timg_cs; const int32_t* timg_w; const int32_t* timg_f; int32_t tplane;
};
// Pre-split W^T of every fused layer (layers 1.. of both nets), for the whole-network backward's dX: planes
// [3][112 i][112 n] bf16 (224-B rows, zero past n_in / n_out) and the fp32 n tail [112 i][4] = W[96 + q][i].
constexpr int BWD_WTPITCH = 224;
constexpr int BWD_WTPLANE = 112 * BWD_WTPITCH;           // 25088
constexpr int BWD_WTTAIL = 3 * BWD_WTPLANE;              // 75264
constexpr int BWD_WTIMG = 77824;                         // 76 KB per layer
static_assert(BWD_WTTAIL + 112 * 16 <= BWD_WTIMG, "W^T image");
hipError_t launch_split_wtimg(const struct FusedArgs& a, unsigned char* timg, int64_t timg_cs, hipStream_t s);
hipError_t launch_scatter(float* packed, int64_t dp, int C, const float* theta, int K, const int32_t* smap_w,
                          const int32_t* smap_wt, hipStream_t s, const ScatterImg* si = nullptr);
// Sum `n_parts` partial slabs of `len` floats (slab stride `part_stride`, chain stride `in_cs`) into
// dst[c*dst_cs + e] (e < len), fixed order.
struct ReduceJob {
    const float* src; int64_t in_cs; int64_t part_stride; int32_t n_parts; int32_t len;
    float* dst; int64_t dst_cs;
    // tiled = 1: the slabs hold the bf16x6 backward's dW accumulator tiles as they stand (bwd_tile_off), len = the
    // tiled slab's floats; the sums are scattered to dst = [n_out][ldi] weights + [n_out] bias (the db column NI4)
    int32_t tiled, ntj, n_out, n_in, ldi;
    // samp != null (weight-gradient jobs of a plan that samples a subset of the parameters): samp[dst offset] = 1
    // where the gather reads the sum (a sampled parameter); a quad of four outputs none of which is read is neither
    // summed nor written (the slab loads are most of the reduce's bytes)
    const uint8_t* samp;
};
// Tiled dW partial slab of the bf16x6 backward kernels: 16x16 tiles (row tile tn of the outputs n, column tile t of
// the inputs j, t < ntj), lane-major float4 quads (lane l = 16 lg + lr holds rows n = 16 tn + 4 lg + r, column
// j = 16 t + lr): tile (tn < 6, t) at (tn ntj + t) 256 floats, row tile 6 (n 96..111) keeps only its lg = 0 lanes.
constexpr int bwd_tile_floats(int ntj) { return 6 * ntj * 256 + ntj * 64; }
__host__ __device__ inline int bwd_tile_off(int tn, int t, int ntj, int lane) {
    return tn < 6 ? (tn * ntj + t) * 256 + 4 * lane : 6 * ntj * 256 + t * 64 + 4 * lane;
}
// Likelihood statistics of the contraction (k_contract_stats): ll from the per-wave (sum r^2, sum G) pairs and
// d ll / d b0 into packed slot 0 of gp. Optionally run as one extra grid slice of the weight-gradient reduce.
// Mixed Gram / residual evaluation (fit guard): chains whose bit is set read (stats2, n_waves2). fit != null: the
// fit ratio sum r^2 / sum y^2 (*ysq) of every chain is written to fit[c] (all-residual evaluations only).
struct StatsJob {
    const double* stats; int64_t stats_cs; int32_t n_waves;
    float* lik; float* gp; int64_t gp_cs; double count; int32_t loss; float tau_out;
    const double* stats2; int64_t stats2_cs; int32_t n_waves2;
    int32_t sel; ChainBits bits;
    float* fit; const double* ysq;
};
hipError_t launch_reduce(const ReduceJob* jobs_dev, int n_jobs, int max_len, int C, hipStream_t s,
                         const StatsJob* stats = nullptr, const ChainBits* only = nullptr);
constexpr int CLOCK_STAMP_WG = 256;    // k_clock_stamp workgroups; 4 uint64 each
hipError_t launch_clock_stamp(unsigned long long* out, hipStream_t s);
hipError_t launch_contract_stats(const StatsJob& J, int C, hipStream_t s);
// sum of y^2 over n elements (fixed order, fp64): `parts` partial sums into part[], then *out (the fit guard's scale)
constexpr int YSQ_PARTS = 1024;
hipError_t launch_ysq(const float* y, int64_t n, double* part, double* out, hipStream_t s);
// Leapfrog update fused into the gradient gather (vihmc_trajectory on DeepONet plans), hamiltorch's order with
// every product and sum rounded separately: p += eps g; then on the last step p -= (eps / 2) g, otherwise
// theta += eps p (eps inv_mass p with a diagonal mass). p and theta are updated in place (theta is the
// evaluation's own input, read by the same thread first).
// The scatter of a new position into the plan's packed weights (+ kept weight images), done by the kernel that
// computes that position (the gradient gather of the previous leapfrog step, or the trajectory's opening kernel)
// instead of a k_scatter launch at the head of the next evaluation. packed == null: none.
struct ScatterArgs {
    float* packed; int64_t dp; const int32_t* smap_w; const int32_t* smap_wt; ScatterImg si;
};
struct LeapArgs {
    float* p;               // [C, K]
    float* th;              // [C, K]
    const float* eps;       // [C] (mode 0)
    const float* inv_mass;  // [K] or null (mode 0)
    int32_t last;
    ScatterArgs sc;         // scatter the new theta (not on the last step); packed == null: the next evaluation does
    int32_t scattered_in;   // this evaluation's theta is already scattered (skip its k_scatter)
    // mode 1 / 2: the splitting integrator's steps around one shard's gradient g (hamiltorch Integrator.SPLITTING with
    // two shards and the reused end gradient, HMCRunner._trajectory): 1 = p += kick g twice (this shard's kick of the
    // forward sweep and of the reverse sweep, or the reverse sweep's last kick and the next step's first), then
    // theta += drift p; 2 = p += kick g once (the trajectory's last kick). Each update one fma, as torch.add(alpha=).
    int32_t mode;
    float kick, drift;
};
// the log-prob finalisation fused into the gradient gather (logp == null: none); cnt: [maxC] zeroed counters
struct FinalizeArgs {
    float* logp;
    const float* lik;
    double prior_const;
    uint32_t* cnt;
};
hipError_t launch_gather_prior(const float* gp, int64_t gp_cs, const int32_t* smap, const float* theta, int K,
                               const float* prior_mu, const float* prior_inv_var, double prior_const,
                               float prior_scale, const float* lik, int C, float* logp, float* grad,
                               double* lp_part, uint32_t* fin_cnt, hipStream_t s, const LeapArgs* leap = nullptr);
// the opening half step and first position step of a trajectory: p_out = p_in + (eps / 2) g_in,
// th_out = th_in + eps p_out (eps inv_mass p_out)
hipError_t launch_leap_open(const float* th_in, float* th_out, const float* p_in, float* p_out, const float* g_in,
                            const float* eps, const float* inv_mass, int K, int C, hipStream_t s,
                            const ScatterArgs* sc = nullptr);
hipError_t launch_gather_trunk(const float* feat_all, int in_t, const float* y_all, int64_t P_all,
                               const int32_t* ind, int P, int N, float* input, int ld_in, float* y, hipStream_t s);

// Fused hidden-layer forward (width 100 -> 100 layers of both nets, one launch): every wave keeps 16 rows
// of activations in registers through all fused layers; per layer the weights + bias of the next layer
// are prefetched into registers and written to the second of two LDS buffers. h_j of every layer is
// stored (the backward needs it). Layer j's W block and bias are contiguous in the packed layout.
constexpr int FUSED_MAXL = 16;
// vihmc_hmc_accept (k_hmc_accept): one HMC iteration's Metropolis step for C chains of K parameters
struct AcceptArgs {
    int32_t K, n, burn;
    const float *lp0, *lp1, *ke0, *ke1, *logu, *th1, *g1;
    float *th_last, *lp_last, *g_last;          // the last returned state (updated in place after burn-in)
    float *th_bp, *lp_bp, *g_bp;                // burn-in fallback (updated in place during burn-in)
    float *th_cur, *lp_cur, *g_cur;             // burn-in: the current state (output)
    float* samples; int64_t s_cap; int64_t* counts;   // after burn-in, or null: the sample rows [C][s_cap][K]
    uint8_t* accepted; int64_t acc_ld;          // accepted[c * acc_ld + n]
    float* trace; int64_t tr_ld;                // trace[c * tr_ld + n] = the current state's log-prob
    float* rho; uint8_t* err;                   // [C]: rho (NaN where the chain failed), 1 = failed
};
hipError_t launch_hmc_accept(const AcceptArgs& a, int C, hipStream_t s);
// vihmc_kinetic (k_kinetic): kinetic energies of C chains; part [C][kinetic_slices(K)] fp64, cnt [C] zeroed once
constexpr int KINETIC_MAX_SLICES = 256;
int kinetic_slices(int K);
hipError_t launch_kinetic(const float* p, const float* inv_mass, int C, int K, float* ke, double* part, uint32_t* cnt,
                          hipStream_t s);

struct FusedNet {
    const float* in; int64_t in_cs; int32_t ldin;   // activations feeding the first fused layer
    float* out; int64_t out_cs; int32_t ldo;        // per-chain activation buffer, row stride of h_j
    int64_t h_off[FUSED_MAXL];                      // h_j offset inside the activation buffer
    int64_t w_off[FUSED_MAXL];                      // packed offset of W_j [100][100] (+ bias right after)
    int32_t act[FUSED_MAXL];
    int32_t nl, rows, nblk;                         // nblk = ceil(rows / (16 * waves per workgroup))
    const unsigned char* wimg; int64_t wimg_cs;     // bf16x6: pre-split [W_j | bias] LDS images of layers
                                                    // 1..nl, FWD_WIMG bytes each (k_split_wimg), or null
    unsigned char* qimg; int64_t qimg_cs;           // or null: the last layer's output also written as the
                                                    // contraction's pre-split block image (k_split_blocks'
                                                    // layout; padding pre-zeroed by the plan)
    int32_t aug;                                    // feature 100 of that image: 0 = zero, 1 = one (branch),
                                                    // 2 = the chain's output bias b0 (trunk): the Gram form's
                                                    // augmented outputs (vihmc_gram.hip; unused by the other paths)
    // the input layer (network layer 0) in the same launch (x != null; the pre-split-image form only): h_0 = act0(x
    // W0^T + b0) on the f32 MFMA in k_rowdot_in's product order, stored at `in` (row stride ldin) and carried on in
    // registers instead of re-read; W0 [n0 = 100][k0] (packed, row stride ldw0) staged in LDS buffer 1
    const float* x; int32_t ldx, k0, ldw0, act0;
    int64_t w0_off, b0_off;
    int32_t skip_last;                              // the last layer's fp32 rows not stored (its image carries them;
                                                    // a Gram-form evaluation reads no other copy of the trunk's)
};
struct FusedArgs {
    FusedNet net[2];
    const float* packed; int64_t dp;
    int32_t C;
};
constexpr int FWD_WIMG = 69632;                     // one pre-split weight image: 3 x [100][112] bf16 + fp32
                                                    // bias [112], zero padded to 68 KB (whole 1-KB DMA pieces)
hipError_t launch_split_wimg(const FusedArgs& a, hipStream_t s);
// byte offsets inside one layer image (k_split_wimg's layout): plane-0 bf16 of W[n][col], the plane stride, the
// fp32 bias[n], and the fp32 k-tail copy of W[n][col] for col in 96..99
int fwd_img_plane_off(int n, int col);
int fwd_img_plane_stride();
int fwd_img_bias_off(int n);
int fwd_img_tail_off(int n, int col);
bool fwd_fused_bf_needs_wimg();                     // the bf16x6 forward reads the fp32 k tail of the image
bool fwd_fused_in0_ok(int n_in, int ldx, int ldw);  // an input layer of this shape fits the fused forward
int fwd_fused_bf_waves();                           // its waves per workgroup (16 rows each)
// VIHMC_DIAG (vihmc_diag.h): nonzero in a build with timing-only ablations (wrong results) or phase stamps.
// vihmc_version() reports it and plan creation refuses such a library unless VIHMC_ALLOW_DIAG=1.
int diag_switches();
hipError_t launch_fwd_fused(const FusedArgs& a, int nwaves, hipStream_t s);   // nwaves: 12 or 4
hipError_t launch_fwd_fused_bf(const FusedArgs& a, int nw, hipStream_t s);     // bf16x6, 12 (or 4) waves

size_t fwd_fused_lds_bytes();

// BNN: one wave per chain, everything in registers / LDS.
struct MlpLayer { int32_t w_off, b_off, n_out, n_in, act; };
struct MlpArgs {
    MlpLayer L[6];
    int32_t n_layers, D, K, N, in_dim, out_dim;
    const float* x; const float* y; const float* frozen; const int32_t* idx;
    const float* prior_mu; const float* prior_inv_var;
    double prior_const; float prior_scale; int32_t loss; float tau_out;
    const float* theta; float* logp; float* grad; float* out;
    // register-resident BNN kernels (vihmc_bnn.hip): canonical weight position of every flat parameter, of every
    // sampled index, and the gradient-tile position of every sampled index (null: the shape is not the BNN's)
    const int32_t* canon; const int32_t* cpos; const int32_t* goff;
};
hipError_t launch_mlp(const MlpArgs& a, int C, int maxw, hipStream_t s);
size_t mlp_lds_bytes(int D, int n_layers, int maxw);
// A whole leapfrog trajectory of every chain in one launch (k_mlp_traj): hamiltorch's op sequence in fp32
// with no fused multiply-adds, so positions / momenta / gradients are bitwise those of L separate
// evaluations driven by the torch elementwise updates.
struct MlpTrajArgs {
    const float* th_in; float* th_out; const float* p_in; float* p_out; const float* g_in; float* g_out;
    float* lp_out; const float* eps; const float* inv_mass; int32_t L;
    int32_t ws_floats;             // set by launch_mlp_traj: the evaluation workspace (mlp_lds_bytes) in floats
    int32_t cache;                 // set by launch_mlp_traj: 1 = data rows / index map / prior / mass cached in LDS
};
hipError_t launch_mlp_traj(const MlpArgs& a, const MlpTrajArgs& t, int C, int maxw, hipStream_t s);
// the reference BNN shape (1 -> 10 -> 10 -> 1, a bias on every layer) as register-resident kernels
constexpr int BNN_IN = 1, BNN_H1 = 10, BNN_H2 = 10, BNN_OUT = 1;
constexpr int BNN_CANON = 152;      // canonical weight floats ([W1 | b1 | W2 | b2 | W3 | b3], 4-aligned blocks)
constexpr int BNN_KS = 3;           // sampled indices per lane (K <= 192)
bool mlp_bnn_fast_ok(const MlpArgs& a);
void mlp_bnn_maps(const MlpArgs& a, std::vector<int32_t>& canon, std::vector<int32_t>& gpos);
hipError_t launch_mlp_bnn(const MlpArgs& a, int C, hipStream_t s);
hipError_t launch_mlp_traj_bnn(const MlpArgs& a, const MlpTrajArgs& t, int C, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Sensitivity scores (vihmc_sens.hip): mean over the selected outputs f[n][p] of (df/dtheta)^2 for every
// parameter of both DeepONet MLPs, by pair backprop. A pair (n, p) seeds the branch at row n with the
// trunk output row Z_t[p] and the trunk at row p with Z_b[n]; within one row ("group") the pairs share
// every activation, so sum_pairs (delta_l[i] h_{l-1}[j])^2 = q_l[i] h_{l-1}[j]^2 with
// q_l = sum_pairs delta_l^2. k_sens_seeds propagates 16 seeds of one group per wave and writes q_l per
// layer; k_sens_outer forms sum_tasks q_l[i] h^2[j] per task chunk; k_sens_reduce sums the chunks in a
// fixed order into the packed layout; k_sens_flat maps to flat order and applies sigma^2 / count.
// ---------------------------------------------------------------------------------------------
constexpr int SENS_MAXL = 16;
constexpr int SENS_WAVES = 8;          // tasks (waves) per k_sens_seeds workgroup, sharing the W_l image
constexpr int SENS_SEEDS = 16;         // seeds per task
constexpr int SENS_QLD = 128;          // q row stride (floats)
constexpr int SENS_PART = 128 * 128 + 128;
constexpr int SENS_TCH = 64;           // tasks staged per k_sens_outer LDS round
struct SensLayer {
    const float* W;          // packed Wp [n_out][ldi] of layer l
    const float* Hprev;      // input rows of layer l: h_{l-1} [rows][ldh] (l > 0) or the net input (l = 0)
    int64_t wp, bias;        // packed offsets of W_l and b_l (output image)
    int32_t ldi, n_out, n_in, ldh, act_prev;   // act_prev: activation of layer l-1 (unused for l = 0)
};
struct SensNet {
    SensLayer L[SENS_MAXL];
    int32_t nl, n_tasks, n_wg, chunks, tasks_per_chunk;
    const float* seeds; int32_t ld_seed;   // the other net's output rows
    const int32_t* tasks;                  // [n_tasks][3]: group row, first seed, seed count (<= 16)
    const int32_t* seed_idx;
    float* Q;                              // [n_tasks][nl][SENS_QLD]
    float* part;                           // [nl][chunks][SENS_PART]
};
struct SensArgs {
    SensNet net[2];
    int32_t ldd, ldw;        // LDS strides of the delta and W images (floats)
    float* S;                // packed-layout output (one chain), slot 0 = the output bias b
    float count;             // pairs = outputs averaged over
};
hipError_t launch_sens(const SensArgs& a, const SensArgs* dev_a, const int32_t* fmap, int64_t D, const float* sigma,
                       float* out, hipStream_t s);    // dev_a: a copy of `a` in device memory
size_t sens_seeds_lds_bytes(int ldd, int ldw);
hipError_t launch_sens_mlp(const MlpArgs& a, float* slab, const float* sigma, float* out, int maxw, hipStream_t s);

}  // namespace vihmc
