// Whole-network backward of one row chunk in ONE launch (bf16x6 products): the nine per-layer k_bwd_bf2
// launches of a single-chain evaluation fused, the deltas kept on chip from layer to layer.
//
// Replaces the autograd backward of the branch / trunk MLPs (Operator_network/VI_HMC/my_make_func.py:53-82,
// torch autograd through F.linear and tanh), layer j = nl-1 .. 0 of each net:
//   delta_{j-1}[m][i] = (sum_n delta_j[m][n] W_j[n][i]) * act'(h_{j-1}[m][i])        (j >= 1)
//   part_j[n][i] = sum_m delta_j[m][n] h_{j-1}[m][i],  part_j[n_out][n] = sum_m delta_j[m][n]
// with k_bwd_bf2's tiled partial slabs (reduced by the same k_reduce jobs), so the two paths are interchangeable
// per evaluation and bitwise equal: every product and every accumulation order is k_bwd_bf2's.
//
// One 768-thread workgroup (8 dX + 4 dW waves, 3 per SIMD) per 64-row chunk of one net of one chain -- the
// plan's chunk when a single chain's rows fill the chip in one round (C = 1: 16 + 160 workgroups). LDS (153 KB):
//   2 sub-tiles x [delta_j planes [3][32][224 B] | delta_j fp32 tail [32][4]], 2 h sets x 2 sub-tiles x planes,
//   act'(h) of the epilogue [64][104] fp32
// W_j^T never touches LDS: each dX wave keeps the fragments of its two input tiles in registers, loaded from the
// pre-split W^T image (BWD_WTIMG, kept current by the scatter) right after its last MFMA of the layer before, so
// they land while the workgroup writes the next deltas.
// Per layer: [A] the dX waves issue the loads of the next h rows, compute delta_{j-1} (kept in registers), load the
// next W^T fragments and split the next h rows into the other h set, while the dW waves compute the weight gradient
// of both sub-tiles; [B] the dX waves split delta_{j-1} into the planes, the dW waves store the partial slab; loop.
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"
#include <type_traits>

namespace vihmc {

namespace {
using bf6::f32x4;
using bf6::bf16x8;
using bf6::bf16x4;
using bf6::split4;
using bf6::six;
using bf6::tr_frag;

constexpr int CH_SUB = BWD_SUB;                        // 32 rows per sub-tile
constexpr int CH_ROWS = 2 * CH_SUB;                    // rows per workgroup
constexpr int CH_PITCH = bf6::PITCH;                   // 224 B
constexpr int CH_PLANE = CH_SUB * CH_PITCH;            // 7168
// LDS: per sub-tile s a delta buffer [planes [3][32][224 B] | fp32 tail [32][4]] at s CH_BUF, then two h sets
// (k = 0, 1) of per-sub-tile planes [3][32][224 B] at CH_HOFF + (2 k + s) CH_HSUB: layer j reads h_{j-1} from set
// k while the dX waves write h_{j-2} into set k ^ 1 before barrier B (their slack while the dW waves finish), so the
// write phase after B only splits the next deltas
constexpr int CH_DP = 0;
constexpr int CH_DT = 3 * CH_PLANE;
constexpr int CH_BUF = CH_DT + CH_SUB * 16;            // 22016 per sub-tile
constexpr int CH_HSUB = 3 * CH_PLANE;                  // 21504
constexpr int CH_HOFF = 2 * CH_BUF;                    // 44032
// act'(h) of the dX epilogue, fp32 [64 rows][104] (stride 8 mod 16 dwords: the k-permuted float4 pattern of the
// epilogue lanes is conflict free), written when the h rows are staged, read by the same lane one layer later
constexpr int CH_AG = CH_HOFF + 4 * CH_HSUB;           // 130048
constexpr int CH_AGLD = 104;
constexpr int CH_LDS = CH_AG + CH_ROWS * CH_AGLD * 4;  // 156672
static_assert(CH_LDS <= 160 * 1024, "LDS");
constexpr int CH_THREADS = 768;
constexpr int CH_HSLOTS = 4;                           // h float4 per dX lane: 64 rows x <= 32 float4 / 512

// h * h rounded before the subtraction (no fused multiply-add), as k_bwd_bf2 computes it
__device__ __forceinline__ float act_grad(int act, float h) {
#pragma clang fp contract(off)
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}
}  // namespace

#if CH_STAMP
// every 8th workgroup (the first 16 of them): per wave and layer, s_memtime after barrier A [0], when the compute
// phase is done [2], after barrier B [3], when the write phase is done [4] ([1] = [0]); per workgroup s_memtime /
// s_memrealtime at start and end (scripts/diag/stamps_chain.py)
constexpr int CHS_WG = 16;
__device__ unsigned long long ch_stamps[CHS_WG][12][BWD_CHAIN_MAXL][5];
__device__ unsigned long long ch_real[CHS_WG][2][2];
#define VIHMC_CH_STAMP(J, K) \
    if (samp && lane == 0) ch_stamps[sidx][wave][(J)][(K)] = __builtin_amdgcn_s_memtime();
#else
#define VIHMC_CH_STAMP(J, K)
#endif

__global__ __launch_bounds__(CH_THREADS, 1) void k_bwd_chain(BwdChainArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    int b = blockIdx.x;
    const int per0 = A.C * A.net[0].n_wg;
    const int net = b >= per0 ? 1 : 0;
    if (net) b -= per0;
    const BwdChainNet& N = A.net[net];
    const int c = b / N.n_wg;
    const int wg = b - c * N.n_wg;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int r0 = wg * CH_ROWS;
    const int M = N.M;
    const int nl = N.nl;
    const unsigned char* wtimg = N.wtimg + c * N.wtimg_cs;
#if CH_STAMP
    const bool samp = (blockIdx.x % 8) == 0 && blockIdx.x / 8 < CHS_WG;
    const int sidx = blockIdx.x / 8;
    if (samp && tid == 0) {
        ch_real[sidx][0][0] = __builtin_amdgcn_s_memtime();
        ch_real[sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif

    // rows [r0, r0 + 64) of a [M][ld] fp32 matrix, float4 item e = row * q + c4 -> (global byte offset, LDS plane
    // offset in the delta buffers (HS < 0) or in h set HS); rows past M read 0 through the buffer resource
    auto item_offsets = [&](int e, int q, int ld, int hs, uint32_t& voff, uint32_t& loff, int& c4o, int& rowo) {
        const int row = e / q, c4 = e - row * q;
        voff = (uint32_t)(row * ld + 4 * c4) * 4u;
        loff = (uint32_t)((hs < 0 ? (row >> 5) * CH_BUF : CH_HOFF + (2 * hs + (row >> 5)) * CH_HSUB) +
                          (row & 31) * CH_PITCH + 8 * c4);
        c4o = c4;
        rowo = row;
    };
    auto hset = [&](int hs, int s) { return sm + CH_HOFF + (2 * hs + s) * CH_HSUB; };
    auto store_planes = [&](unsigned char* base, f32x4 x) {
        bf16x4 p0, p1, p2;
        split4(x, p0, p1, p2);
        *reinterpret_cast<bf16x4*>(base) = p0;
        *reinterpret_cast<bf16x4*>(base + CH_PLANE) = p1;
        *reinterpret_cast<bf16x4*>(base + 2 * CH_PLANE) = p2;
    };
    // the db column of h set hs: constant one at column NI4 of both sub-tiles (planes 1, 0, 0)
    auto db_column = [&](int hs, int ni4, int t) {
        if (t < CH_ROWS) {
            unsigned char* o = hset(hs, t >> 5) + (t & 31) * CH_PITCH + 2 * ni4;
            *reinterpret_cast<unsigned short*>(o) = 0x3F80;
            *reinterpret_cast<unsigned short*>(o + CH_PLANE) = 0;
            *reinterpret_cast<unsigned short*>(o + 2 * CH_PLANE) = 0;
        }
    };

    // ---------------- prologue (all waves): delta of the top layer and its h rows ----------------
    {
        const int jt = nl - 1;
        const BwdChainLayer& L = N.L[jt];
        const int hq = (L.n_in + 3) >> 2;
        const float* D = N.D + c * N.d_cs + (int64_t)r0 * N.ldd;
        const float* H = L.H + c * L.h_cs + (int64_t)r0 * L.ldh;
        const __amdgpu_buffer_rsrc_t drs = bf6::make_rsrc(D, (uint32_t)((M - r0) * N.ldd * 4));
        const __amdgpu_buffer_rsrc_t hrs = bf6::make_rsrc(H, (uint32_t)((M - r0) * L.ldh * 4));
        // every piece's load issued before the first store (the strided loops waited out one load per piece: 6
        // serial round trips before the first layer)
        constexpr int NP = (CH_ROWS * 25 + CH_THREADS - 1) / CH_THREADS;
        static_assert(NP == 3, "prologue pieces per thread");
        f32x4 xd[NP], xh[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int e = tid + CH_THREADS * u;
            uint32_t voff, loff;
            int c4, row;
            if (e < CH_ROWS * 25) {
                item_offsets(e, 25, N.ldd, -1, voff, loff, c4, row);
                xd[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(drs, voff, 0, 0));
            }
            if (e < CH_ROWS * hq) {
                item_offsets(e, hq, L.ldh, 0, voff, loff, c4, row);
                xh[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs, voff, 0, 0));
            }
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int e = tid + CH_THREADS * u;
            uint32_t voff, loff;
            int c4, row;
            if (e < CH_ROWS * 25) {
                item_offsets(e, 25, N.ldd, -1, voff, loff, c4, row);
                store_planes(sm + CH_DP + loff, xd[u]);
                if (c4 == 24) *reinterpret_cast<f32x4*>(sm + (row >> 5) * CH_BUF + CH_DT + (row & 31) * 16) = xd[u];
            }
            if (e < CH_ROWS * hq) {
                item_offsets(e, hq, L.ldh, 0, voff, loff, c4, row);
                store_planes(sm + loff, xh[u]);
            }
        }
        db_column(0, 4 * hq, tid);
    }

    if (wave < 8) {
        // ---------------- dX role: i-tiles {2 p2, 2 p2 + 1} x row half h of both sub-tiles ----------------
        // instantiated per tile count (TWO) and activation (every hidden activation tanh, or any), so no branch
        // splits the loads from the MFMAs; every global load of the loop is unconditional (clamped layer index),
        // so hipcc's counted waits stay exact across the loop edge (the W^T fragments wait for themselves only)
        const int h = wave & 1, p2 = wave >> 1;
        const int t0 = 2 * __builtin_amdgcn_readfirstlane(p2);
        auto dx_run = [&](auto two_c, auto tanh_c) __attribute__((always_inline)) {
            constexpr bool TWO = decltype(two_c)::value;
            constexpr bool TANH = decltype(tanh_c)::value;
            constexpr int NU = TWO ? 2 : 1;
            // W_j^T fragments: lane (lr, lg) holds W^T[16 t + lr][32 kb + 8 lg + jj] (jj = 0..7, the k order of the
            // delta rows' b128 reads) of every plane, and the exact fp32 n tail W^T[16 t + lr][96 + lg]
            bf16x8 wf[NU][3][3];
            float wt[NU];
            auto load_w = [&](int jj) __attribute__((always_inline)) {
                const unsigned char* ti = wtimg + (int64_t)(jj - 1) * BWD_WTIMG;
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int row = 16 * (t0 + u) + lr;
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            wf[u][kb][p] = *reinterpret_cast<const bf16x8*>(ti + p * BWD_WTPLANE + row * BWD_WTPITCH +
                                                                            2 * (32 * kb + 8 * lg));
                    wt[u] = *reinterpret_cast<const float*>(ti + BWD_WTTAIL + 4 * (row * 4 + lg));
                }
            };
            // act'(h_{j-1}) of this lane's epilogue elements (rows 32 s + 16 h + lr, columns 16 (t0 + u) + 4 lg),
            // computed from the fp32 h rows when they are staged (one layer ahead) and kept in the CH_AG array, which
            // only this lane reads back, instead of rebuilding h from the three LDS planes per element (as k_bwd_bf2
            // does since round 5; the same h, bitwise the same deltas). Slot v = 2 s + u of the aligned staging
            // map; columns past 99 clamp to float4 24 (a duplicate item: the same value to the same address).
            auto aligned_item = [&](int v, int& row, int& c4) {
                row = 32 * (v >> 1) + 16 * h + lr;
                c4 = min(4 * (t0 + (v & 1)) + lg, 24);
            };
            auto ag_at = [&](int v) {
                int row, c4;
                aligned_item(v, row, c4);
                return reinterpret_cast<f32x4*>(sm + CH_AG + (row * CH_AGLD + 4 * c4) * 4);
            };
            auto act_of = [&](int act, const f32x4& x) __attribute__((always_inline)) {
                f32x4 out;
#pragma unroll
                for (int r = 0; r < 4; ++r) out[r] = TANH ? act_grad(ACT_TANH, x[r]) : act_grad(act, x[r]);
                return out;
            };
            if (nl >= 2) {                             // the top layer's epilogue: h_{nl-2}, loaded again (L2)
                const BwdChainLayer& L = N.L[nl - 1];
                const float* H = L.H + c * L.h_cs + (int64_t)r0 * L.ldh;
                const __amdgpu_buffer_rsrc_t hrs = bf6::make_rsrc(H, (uint32_t)((M - r0) * L.ldh * 4));
                f32x4 x[2 * NU];
#pragma unroll
                for (int v = 0; v < 2 * NU; ++v) {
                    int row, c4;
                    aligned_item(2 * (v / NU) + v % NU, row, c4);
                    x[v] = __builtin_bit_cast(
                        f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs, (uint32_t)(row * L.ldh + 4 * c4) * 4u, 0, 0));
                }
#pragma unroll
                for (int v = 0; v < 2 * NU; ++v) *ag_at(2 * (v / NU) + v % NU) = act_of(N.L[nl - 1].act, x[v]);
            }
            load_w(max(nl - 1, 1));
            for (int j = nl - 1; j >= 0; --j) {
                const int hs = (nl - 1 - j) & 1;       // h set of this layer's h_{j-1}
                __syncthreads();                       // A: delta_j, h_{j-1} in LDS
                VIHMC_CH_STAMP(j, 0)
                VIHMC_CH_STAMP(j, 1)
                const bool dx = j >= 1;
                // the next layer's h rows (h_{j-2}, or the net input when j = 1) into registers, stored after B
                f32x4 hx[CH_HSLOTS];
                uint32_t hl[CH_HSLOTS];
                const BwdChainLayer& Ln = N.L[max(j - 1, 0)];
                const int hq_n = (Ln.n_in + 3) >> 2;
                // the next layer has a dX part (j - 1 >= 1, n_in = 100): the aligned map, whose items are this lane's
                // epilogue elements of that layer; else (the input layer next) item e = tid + 512 v, wrapped
                const bool aligned = j >= 2;
                {
                    const float* H = Ln.H + c * Ln.h_cs + (int64_t)r0 * Ln.ldh;
                    const __amdgpu_buffer_rsrc_t hrs = bf6::make_rsrc(H, (uint32_t)((M - r0) * Ln.ldh * 4));
                    const int tot = CH_ROWS * hq_n;
#pragma unroll
                    for (int v = 0; v < CH_HSLOTS; ++v) {
                        // wrapped: a lane past the end moves an item another lane moves too (same value and address)
                        int row, c4;
                        if (aligned) {
                            aligned_item(v, row, c4);
                        } else {
                            const int e = (tid + 512 * v) % tot;
                            row = e / hq_n;
                            c4 = e - row * hq_n;
                        }
                        const uint32_t voff = (uint32_t)(row * Ln.ldh + 4 * c4) * 4u;
                        hl[v] = (uint32_t)(CH_HOFF + (2 * (hs ^ 1) + (row >> 5)) * CH_HSUB + (row & 31) * CH_PITCH + 8 * c4);
                        hx[v] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs, voff, 0, 0));
                    }
                }
                f32x4 o[2][NU];                        // [sub][u] delta_{j-1} of rows 32 sub + 16 h + lr
                if (dx) {
                    const int act = N.L[j].act;
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const unsigned char* buf = sm + s * CH_BUF;
                        const unsigned char* drow = buf + CH_DP + (16 * h + lr) * CH_PITCH + 16 * lg;
                        const float dtl = reinterpret_cast<const float*>(buf + CH_DT)[(16 * h + lr) * 4 + lg];
                        f32x4 ac[NU];
#pragma unroll
                        for (int u = 0; u < NU; ++u)
                            ac[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[u], dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                        for (int kb = 0; kb < 3; ++kb) {
                            bf16x8 db[3];
#pragma unroll
                            for (int p = 0; p < 3; ++p) db[p] = *reinterpret_cast<const bf16x8*>(drow + p * CH_PLANE + 64 * kb);
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                if (CH_ABL == 2) asm volatile("" :: "v"(wf[u][kb][0]), "v"(db[0]), "v"(db[1]), "v"(db[2]));
                                else ac[u] = six(wf[u][kb], db, ac[u]);
                            }
                        }
                        // epilogue: act'(h_{j-1}), staged with h_{j-1} one layer ago (or in the prologue)
                        (void)act;
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            const f32x4 ag = *ag_at(2 * s + u);
#pragma unroll
                            for (int r = 0; r < 4; ++r) ac[u][r] = ac[u][r] * ag[r];
                            o[s][u] = ac[u];
                        }
                    }
                }
                // the next layer's fragments, in flight through B; the scheduling barrier keeps hipcc from hoisting
                // them above this layer's MFMAs (which would need a second set of 72 fragment registers)
                __builtin_amdgcn_sched_barrier(0);
                load_w(max(j - 1, 1));
                // the next layer's h rows into the other h set (its last readers were layer j + 1's, before A)
                if (dx) {
#pragma unroll
                    for (int v = 0; v < CH_HSLOTS; ++v) store_planes(sm + hl[v], hx[v]);
                    db_column(hs ^ 1, 4 * hq_n, tid);
                    if (aligned) {                     // act'(h_{j-2}) for the next layer's epilogue
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                            for (int u = 0; u < NU; ++u) *ag_at(2 * s2 + u) = act_of(N.L[j - 1].act, hx[2 * s2 + u]);
                    }
                }
#if CH_STAMP
                asm volatile("" :: "v"(o[0][0]), "v"(o[1][0]));
#endif
                VIHMC_CH_STAMP(j, 2)
                __syncthreads();                       // B: every read of delta_j done
                VIHMC_CH_STAMP(j, 3)
                if (dx) {
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            const int col = 16 * (t0 + u) + 4 * lg;
                            unsigned char* buf = sm + s * CH_BUF;
                            store_planes(buf + CH_DP + (16 * h + lr) * CH_PITCH + 2 * col, o[s][u]);
                            if (col == 96) *reinterpret_cast<f32x4*>(buf + CH_DT + (16 * h + lr) * 16) = o[s][u];
                        }
                }
                VIHMC_CH_STAMP(j, 4)
            }
        };
        const bool tanh_all = N.tanh_all != 0;
        if (t0 + 1 < 7) {
            if (tanh_all) dx_run(std::true_type{}, std::true_type{});
            else dx_run(std::true_type{}, std::false_type{});
        } else {
            if (tanh_all) dx_run(std::false_type{}, std::true_type{});
            else dx_run(std::false_type{}, std::false_type{});
        }
    } else {
        // ---------------- dW role ----------------
        // the tile assignment of k_bwd_bf2's dW role: waves 10, 11 take row tiles {0, 1} and {2, 3} whole, waves
        // 8, 9 row tile 4 or 5 whole plus row tile 6 over column tiles 0..3 or 4..6
        const int g = __builtin_amdgcn_readfirstlane(wave - 8);
        const int rta = g == 2 ? 0 : g == 3 ? 2 : 4 + g;
        const int rtb = g == 2 ? 1 : g == 3 ? 3 : 6;
        const int cb0 = g == 1 ? 4 : 0, cb1 = g == 0 ? 4 : 7;
        const int tro = bf6::tr_lane_off(lr, lg);
        f32x4 acc[2][7];
        // weight gradient over the 64 rows (k = the rows, two 32-row blocks); instantiated for 7 column tiles (all
        // but an input layer), so the next tile's h reads stay in flight under this tile's MFMAs
        auto dw_layer = [&](auto nt_c, int ntj, int hs) __attribute__((always_inline)) {
            constexpr int NT = decltype(nt_c)::value;  // 0: ntj at run time
            const int nt = NT ? NT : ntj;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int t = 0; t < 7; ++t) acc[s2][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
            for (int s = 0; s < 2; ++s) {
                const unsigned char* buf = sm + s * CH_BUF;
                const unsigned char* hbuf = hset(hs, s);
                bf16x8 da[2][3], hb[2][3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    da[0][p] = tr_frag(buf + CH_DP + p * CH_PLANE, tro, 16 * rta);
                    da[1][p] = tr_frag(buf + CH_DP + p * CH_PLANE, tro, 16 * rtb);
                    hb[0][p] = tr_frag(hbuf + p * CH_PLANE, tro, 0);
                }
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= nt) break;
                    if (t + 1 < nt) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) hb[(t + 1) & 1][p] = tr_frag(hbuf + p * CH_PLANE, tro, 16 * (t + 1));
                    }
                    if (CH_ABL == 1) {
                        asm volatile("" :: "v"(da[0][0]), "v"(da[1][0]), "v"(hb[t & 1][0]), "v"(hb[t & 1][1]), "v"(hb[t & 1][2]));
                        continue;
                    }
                    acc[0][t] = six(da[0], hb[t & 1], acc[0][t]);
                    if (t >= cb0 && t < cb1) acc[1][t] = six(da[1], hb[t & 1], acc[1][t]);
                }
            }
        };
        for (int j = nl - 1; j >= 0; --j) {
            const int hs = (nl - 1 - j) & 1;
            __syncthreads();                           // A
            VIHMC_CH_STAMP(j, 0)
            VIHMC_CH_STAMP(j, 1)
            const BwdChainLayer& L = N.L[j];
            const int NI4 = (L.n_in + 3) & ~3;
            const int ntj = __builtin_amdgcn_readfirstlane((NI4 + 16) >> 4);
            if (ntj == 7) dw_layer(std::integral_constant<int, 7>{}, 7, hs);
            else dw_layer(std::integral_constant<int, 0>{}, ntj, hs);
#if CH_STAMP
            asm volatile("" :: "v"(acc[0][0]), "v"(acc[1][6]));
#endif
            VIHMC_CH_STAMP(j, 2)
            __syncthreads();                           // B
            VIHMC_CH_STAMP(j, 3)
            // the tiled partial slab of layer j (bwd_tile_off, as k_bwd_bf2): one 1-KB store per tile through a
            // buffer resource (row tile 6 keeps its lg = 0 lanes: the others get an out-of-range offset)
            const __amdgpu_buffer_rsrc_t prs = bf6::make_rsrc(N.dwpart + c * N.dwpart_cs + L.part_off +
                                                              (int64_t)wg * L.part_stride,
                                                              (uint32_t)bwd_tile_floats(ntj) * 4u);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int tn = s2 == 0 ? rta : rtb;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= ntj || (s2 == 1 && (t < cb0 || t >= cb1))) continue;
                    const uint32_t off = (tn < 6 || lg == 0) ? (uint32_t)bwd_tile_off(tn, t, ntj, lane) * 4u : bf6::OOB;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bf6::u32x4, acc[s2][t]), prs, off, 0, 0);
                }
            }
            VIHMC_CH_STAMP(j, 4)
        }
    }
#if CH_STAMP
    __syncthreads();
    if (samp && tid == 0) {
        ch_real[sidx][1][0] = __builtin_amdgcn_s_memtime();
        ch_real[sidx][1][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

#if CH_STAMP
extern "C" int vihmc_debug_ch_stamps(void* stamps, size_t stamp_bytes, void* real, size_t real_bytes) {
    if (stamp_bytes != sizeof(ch_stamps) || real_bytes != sizeof(ch_real)) return -1;
    hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(ch_stamps), stamp_bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(real, HIP_SYMBOL(ch_real), real_bytes, 0, hipMemcpyDeviceToHost);
    return (int)e;
}
#endif

// W^T of every fused layer of every chain -> the backward's transposed image (BWD_WTIMG layout): one block per
// (chain, net, layer); the three planes exactly as k_split_wimg / the scatter split them
__global__ __launch_bounds__(256) void k_split_wtimg(FusedArgs args, unsigned char* timg, int64_t timg_cs) {
    const int C = args.C;
    int b = blockIdx.x;
    const int c = b % C;
    b /= C;
    const int net = b < args.net[0].nl ? 0 : 1;
    const int j = net ? b - args.net[0].nl : b;
    const float* W = args.packed + c * args.dp + args.net[net].w_off[j];   // [100 n][100 i]
    unsigned char* img = timg + c * timg_cs + (int64_t)b * BWD_WTIMG;
    for (int e = threadIdx.x; e < 112 * 112; e += 256) {
        const int i = e / 112, n = e - i * 112;
        const float v = (i < 100 && n < 100) ? W[n * 100 + i] : 0.f;
        const __bf16 a = (__bf16)v;
        const float r = v - (float)a;
        const __bf16 bb = (__bf16)r;
        const __bf16 cc = (__bf16)(r - (float)bb);
        __bf16* o = reinterpret_cast<__bf16*>(img + i * BWD_WTPITCH + 2 * n);
        o[0] = a;
        o[BWD_WTPLANE / 2] = bb;
        o[BWD_WTPLANE] = cc;
    }
    float* tail = reinterpret_cast<float*>(img + BWD_WTTAIL);
    for (int e = threadIdx.x; e < 112 * 4; e += 256) {
        const int i = e >> 2, q = e & 3;
        tail[e] = i < 100 ? W[(96 + q) * 100 + i] : 0.f;
    }
}

hipError_t launch_split_wtimg(const FusedArgs& a, unsigned char* timg, int64_t timg_cs, hipStream_t s) {
    hipLaunchKernelGGL(k_split_wtimg, dim3(a.C * (a.net[0].nl + a.net[1].nl)), dim3(256), 0, s, a, timg, timg_cs);
    return hipGetLastError();
}

bool bwd_chain_ok(const BwdChainArgs& a) {
    for (int net = 0; net < 2; ++net) {
        const BwdChainNet& n = a.net[net];
        if (n.nl < 2 || n.nl > BWD_CHAIN_MAXL || !n.wtimg || (n.ldd & 3) || n.ldd < 100 || n.n_wg * CH_ROWS < n.M ||
            (n.n_wg - 1) * CH_ROWS >= n.M)
            return false;
        for (int j = 0; j < n.nl; ++j) {
            const BwdChainLayer& L = n.L[j];
            if (L.n_out != 100 || (L.ldh & 3) || ((L.n_in + 3) & ~3) >= 112 || (j >= 1 && L.n_in != 100) ||
                ((L.n_in + 3) >> 2) * CH_ROWS > 512 * CH_HSLOTS)
                return false;
        }
    }
    return true;
}

hipError_t launch_bwd_chain(const BwdChainArgs& a, hipStream_t s) {
    if (!bwd_chain_ok(a)) return hipErrorInvalidValue;
    const int blocks = a.C * (a.net[0].n_wg + a.net[1].n_wg);
    hipLaunchKernelGGL(k_bwd_chain, dim3(blocks), dim3(CH_THREADS), CH_LDS, s, a);
    return hipGetLastError();
}

int bwd_chain_rows() { return CH_ROWS; }


}  // namespace vihmc
