// Whole-network backward of one row chunk in ONE launch (bf16x6 products): the nine per-layer k_bwd_bf2
// launches of a single-chain evaluation fused, the deltas kept on chip from layer to layer.
//
// Replaces the autograd backward of the branch / trunk MLPs (Operator_network/VI_HMC/my_make_func.py:53-82,
// torch autograd through F.linear and tanh), layer j = nl-1 .. 0 of each net:
//   delta_{j-1}[m][i] = (sum_n delta_j[m][n] W_j[n][i]) * act'(h_{j-1}[m][i])        (j >= 1)
//   part_j[n][i] = sum_m delta_j[m][n] h_{j-1}[m][i],  part_j[n_out][n] = sum_m delta_j[m][n]
// with the same partial-slab layout as k_bwd_bf2 (reduced by the same k_reduce jobs), so the two paths are
// interchangeable per evaluation and bitwise equal: every product and every accumulation order is k_bwd_bf2's.
//
// One 768-thread workgroup (8 dX + 4 dW waves, 3 per SIMD) per 64-row chunk of one net of one chain -- the
// plan's chunk when a single chain's rows fill the chip in one round (C = 1: 16 + 160 workgroups). LDS (151 KB):
//   2 sub-tiles x [delta_j planes [3][32][224 B] | h_{j-1} planes [3][32][224 B] | delta_j fp32 tail [32][4]]
//   W_j: the forward's pre-split weight image (k_split_wimg: planes [3][100 n][112 permuted i]), one DMA copy
//        per layer. dX reads it with transposed reads whose per-lane addresses undo the permutation and give
//        the k order of the delta row reads; its n tail (rows 96..99) is rebuilt exactly from the planes.
// Per layer: [A] the dX waves take their W fragments into registers; [A2] the dW waves start the DMA of the
// next layer's image, the dX waves the loads of its h rows, then compute delta_{j-1} (kept in registers) while
// the dW waves compute the weight gradient of both sub-tiles; [B] the dX waves split delta_{j-1} and the next h
// rows into the planes, the dW waves store the partial slab; loop.
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"
#include <type_traits>

namespace vihmc {

namespace {
using bf6::f32x4;
using bf6::bf16x8;
using bf6::bf16x4;
using bf6::lds_bf16x4;
using bf6::split4;
using bf6::cat8;
using bf6::six;
using bf6::tr_frag;

constexpr int CH_SUB = BWD_SUB;                        // 32 rows per sub-tile
constexpr int CH_ROWS = 2 * CH_SUB;                    // rows per workgroup
constexpr int CH_PITCH = bf6::PITCH;                   // 224 B
constexpr int CH_PLANE = CH_SUB * CH_PITCH;            // 7168
constexpr int CH_DP = 0;
constexpr int CH_HP = 3 * CH_PLANE;
constexpr int CH_DT = 6 * CH_PLANE;
constexpr int CH_BUF = CH_DT + CH_SUB * 16;            // 43520 per sub-tile
constexpr int CH_W = 2 * CH_BUF;                       // 87040: the W image planes
constexpr int CH_WPLANE = 100 * 224;                   // plane stride of the forward's image (fwd_img_plane_stride)
constexpr int CH_WPIECES = (3 * CH_WPLANE + 1023) / 1024;   // 66 DMA pieces of 1 KB
constexpr int CH_LDS = CH_W + CH_WPIECES * 1024;       // 154624
static_assert(CH_LDS <= 160 * 1024 && CH_WPIECES * 1024 <= FWD_WIMG, "LDS / image");
static_assert(CH_BUF + 2 * CH_PLANE < 65536, "LDS store offsets fit the ds_write immediate");
constexpr int CH_THREADS = 768;
constexpr int CH_HSLOTS = 4;                           // h float4 per dX lane: 64 rows x <= 32 float4 / 512

// image position of input column col (k_split_wimg's permuted order; fwd_img_plane_off)
__device__ __forceinline__ int img_pos(int col) {
    const int t = col >> 4, g = (col >> 2) & 3, e = col & 3;
    return t < 6 ? (t >> 1) * 32 + g * 8 + (t & 1) * 4 + e : col;
}

// h * h rounded before the subtraction (no fused multiply-add), as k_bwd_bf2 computes it
__device__ __forceinline__ float act_grad(int act, float h) {
#pragma clang fp contract(off)
    if (act == ACT_TANH) return 1.f - h * h;
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}
}  // namespace

#ifndef CH_STAMP
#define CH_STAMP 0        // timing-only instrumentation (variant builds): in-kernel phase stamps
#endif
#if CH_STAMP
// every 8th workgroup (the first 16 of them): per wave and layer, s_memtime after barrier A [0], after A2 [1], when
// the compute phase is done [2], after barrier B [3], when the write phase is done [4]; per workgroup s_memtime /
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
    const unsigned char* wimg = N.wimg + c * N.wimg_cs;
#if CH_STAMP
    const bool samp = (blockIdx.x % 8) == 0 && blockIdx.x / 8 < CHS_WG;
    const int sidx = blockIdx.x / 8;
    if (samp && tid == 0) {
        ch_real[sidx][0][0] = __builtin_amdgcn_s_memtime();
        ch_real[sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif

    // rows [r0, r0 + 64) of a [M][ld] fp32 matrix, float4 item e = row * q + c4 -> (global byte offset, LDS plane
    // offset); rows past M read 0 through the buffer resource
    auto item_offsets = [&](int e, int q, int ld, uint32_t& voff, uint32_t& loff, int& c4o, int& rowo) {
        const int row = e / q, c4 = e - row * q;
        voff = (uint32_t)(row * ld + 4 * c4) * 4u;
        loff = (uint32_t)((row >> 5) * CH_BUF + (row & 31) * CH_PITCH + 8 * c4);
        c4o = c4;
        rowo = row;
    };
    auto store_planes = [&](unsigned char* base, f32x4 x) {
        bf16x4 p0, p1, p2;
        split4(x, p0, p1, p2);
        *reinterpret_cast<bf16x4*>(base) = p0;
        *reinterpret_cast<bf16x4*>(base + CH_PLANE) = p1;
        *reinterpret_cast<bf16x4*>(base + 2 * CH_PLANE) = p2;
    };
    // the db column of the h planes: constant one at column NI4 of both sub-tiles (planes 1, 0, 0)
    auto db_column = [&](int ni4, int t) {
        if (t < CH_ROWS) {
            unsigned char* o = sm + (t >> 5) * CH_BUF + CH_HP + (t & 31) * CH_PITCH + 2 * ni4;
            *reinterpret_cast<unsigned short*>(o) = 0x3F80;
            *reinterpret_cast<unsigned short*>(o + CH_PLANE) = 0;
            *reinterpret_cast<unsigned short*>(o + 2 * CH_PLANE) = 0;
        }
    };
    auto dma_image = [&](int j, int w0, int nw) {       // W_j's image (index j - 1) -> the W buffer
        const unsigned char* src = wimg + (int64_t)(j - 1) * FWD_WIMG;
        for (int k = w0; k < CH_WPIECES; k += nw) bf6::glds16_asm(src + k * 1024 + lane * 16, sm + CH_W + k * 1024);
    };

    // ---------------- prologue (all waves): delta of the top layer, h rows and W image of the top layer ------
    {
        const int jt = nl - 1;
        const BwdChainLayer& L = N.L[jt];
        const int hq = (L.n_in + 3) >> 2;
        const float* D = N.D + c * N.d_cs + (int64_t)r0 * N.ldd;
        const float* H = L.H + c * L.h_cs + (int64_t)r0 * L.ldh;
        const __amdgpu_buffer_rsrc_t drs = bf6::make_rsrc(D, (uint32_t)((M - r0) * N.ldd * 4));
        const __amdgpu_buffer_rsrc_t hrs = bf6::make_rsrc(H, (uint32_t)((M - r0) * L.ldh * 4));
        if (jt >= 1 && wave >= 8) dma_image(jt, wave - 8, 4);
        for (int e = tid; e < CH_ROWS * 25; e += CH_THREADS) {
            uint32_t voff, loff;
            int c4, row;
            item_offsets(e, 25, N.ldd, voff, loff, c4, row);
            const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(drs, voff, 0, 0));
            store_planes(sm + CH_DP + loff, x);
            if (c4 == 24) *reinterpret_cast<f32x4*>(sm + (row >> 5) * CH_BUF + CH_DT + (row & 31) * 16) = x;
        }
        for (int e = tid; e < CH_ROWS * hq; e += CH_THREADS) {
            uint32_t voff, loff;
            int c4, row;
            item_offsets(e, hq, L.ldh, voff, loff, c4, row);
            const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs, voff, 0, 0));
            store_planes(sm + CH_HP + loff, x);
        }
        db_column(4 * hq, tid);
        if (jt >= 1 && wave >= 8) bf6::wait_vmcnt0();
    }

    if (wave < 8) {
        // ---------------- dX role: i-tiles {2 p2, 2 p2 + 1} x row half h of both sub-tiles ----------------
        const int h = wave & 1, p2 = wave >> 1;
        const int t0 = 2 * __builtin_amdgcn_readfirstlane(p2);
        const bool two = t0 + 1 < 7;                   // wave-uniform (p2 = 3: i-tile 6 only)
        // transposed image reads: lane (qq = lr >> 2, pp = lr & 3) of group lg supplies image row 32 kb + 8 lg + qq
        // (+ 4: the second read) at the position of input column 16 t + 4 pp, so result lane (lr, lg) holds
        // W[32 kb + 8 lg + jj][16 t + lr], jj = 0..7: the k order of the delta rows' b128 reads
        uint32_t wtr[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
            wtr[u] = (uint32_t)(CH_W + (8 * lg + (lr >> 2)) * CH_PITCH + 2 * img_pos(16 * (t0 + u) + 4 * (lr & 3)));
        for (int j = nl - 1; j >= 0; --j) {
            __syncthreads();                           // A: delta_j, h_{j-1}, W_j in LDS
            VIHMC_CH_STAMP(j, 0)
            const bool dx = j >= 1;
            bf16x8 wf[2][3][3];                        // [u][kb][plane]
            float wt[2] = {0.f, 0.f};
            if (dx) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (u == 1 && !two) break;
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
                        for (int p = 0; p < 3; ++p) {
                            const unsigned char* a = sm + wtr[u] + p * CH_WPLANE + 32 * kb * CH_PITCH;
                            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
                            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 4 * CH_PITCH));
                            wf[u][kb][p] = cat8(lo, hi);
                        }
                    // n tail: W[96 + lg][16 t + lr], rebuilt exactly from the planes
                    const __bf16* pl = reinterpret_cast<const __bf16*>(sm + CH_W + (96 + lg) * CH_PITCH) +
                                       img_pos(16 * (t0 + u) + lr);
                    wt[u] = ((float)pl[CH_WPLANE] + (float)pl[CH_WPLANE / 2]) + (float)pl[0];   // (x2 + x1) + x0
                }
            }
            __syncthreads();                           // A2: the W buffer is free (the dW waves refill it)
            VIHMC_CH_STAMP(j, 1)
            // the next layer's h rows (h_{j-2}, or the net input when j = 1) into registers, stored after B
            f32x4 hx[CH_HSLOTS];
            uint32_t hl[CH_HSLOTS];
            int hq_n = 0;
            if (dx) {
                const BwdChainLayer& Ln = N.L[j - 1];
                hq_n = (Ln.n_in + 3) >> 2;
                const float* H = Ln.H + c * Ln.h_cs + (int64_t)r0 * Ln.ldh;
                const __amdgpu_buffer_rsrc_t hrs = bf6::make_rsrc(H, (uint32_t)((M - r0) * Ln.ldh * 4));
                const int tot = CH_ROWS * hq_n;
#pragma unroll
                for (int v = 0; v < CH_HSLOTS; ++v) {
                    // wrapped: a lane past the end moves an item another lane moves too (same value, same address)
                    const int e = (tid + 512 * v) % tot;
                    uint32_t voff, loff;
                    int c4, row;
                    item_offsets(e, hq_n, Ln.ldh, voff, loff, c4, row);
                    hl[v] = loff;
                    hx[v] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hrs, voff, 0, 0));
                }
            }
            f32x4 o[2][2];                             // [sub][u] delta_{j-1} of rows 32 sub + 16 h + lr
            if (dx) {
                const int act = N.L[j].act;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const unsigned char* buf = sm + s * CH_BUF;
                    const unsigned char* drow = buf + CH_DP + (16 * h + lr) * CH_PITCH + 16 * lg;
                    const float dtl = reinterpret_cast<const float*>(buf + CH_DT)[(16 * h + lr) * 4 + lg];
                    f32x4 ac[2];
                    ac[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[0], dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    ac[1] = two ? __builtin_amdgcn_mfma_f32_16x16x4f32(wt[1], dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int kb = 0; kb < 3; ++kb) {
                        bf16x8 db[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p) db[p] = *reinterpret_cast<const bf16x8*>(drow + p * CH_PLANE + 64 * kb);
                        ac[0] = six(wf[0][kb], db, ac[0]);
                        if (two) ac[1] = six(wf[1][kb], db, ac[1]);
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        if (u == 1 && !two) {
                            o[s][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                            break;
                        }
                        f32x4 acc = ac[u];
                        // epilogue: act'(h_{j-1}) from the exact h planes
                        const int col = 16 * (t0 + u) + 4 * lg;
                        const unsigned char* hrow = buf + CH_HP + (16 * h + lr) * CH_PITCH + 2 * col;
                        bf16x4 hq[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p) hq[p] = *reinterpret_cast<const bf16x4*>(hrow + p * CH_PLANE);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float hv = ((float)hq[2][r] + (float)hq[1][r]) + (float)hq[0][r];
                            acc[r] = acc[r] * act_grad(act, hv);
                        }
                        o[s][u] = acc;
                    }
                }
            }
#if CH_STAMP
            if (dx) asm volatile("" :: "v"(o[0][0]), "v"(o[1][0]));
#endif
            VIHMC_CH_STAMP(j, 2)
            __syncthreads();                           // B: every read of delta_j / h_{j-1} done
            VIHMC_CH_STAMP(j, 3)
            if (dx) {
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        if (u == 1 && !two) break;
                        const int col = 16 * (t0 + u) + 4 * lg;
                        unsigned char* buf = sm + s * CH_BUF;
                        store_planes(buf + CH_DP + (16 * h + lr) * CH_PITCH + 2 * col, o[s][u]);
                        if (col == 96) *reinterpret_cast<f32x4*>(buf + CH_DT + (16 * h + lr) * 16) = o[s][u];
                    }
#pragma unroll
                for (int v = 0; v < CH_HSLOTS; ++v) store_planes(sm + CH_HP + hl[v], hx[v]);
                db_column(4 * hq_n, tid);
            }
            VIHMC_CH_STAMP(j, 4)
        }
    } else {
        // ---------------- dW role (and the staging of the next layer) ----------------
        // the tile assignment of k_bwd_bf2's dW role: waves 10, 11 take row tiles {0, 1} and {2, 3} whole, waves
        // 8, 9 row tile 4 or 5 whole plus row tile 6 over column tiles 0..3 or 4..6
        const int g = __builtin_amdgcn_readfirstlane(wave - 8);
        const int rta = g == 2 ? 0 : g == 3 ? 2 : 4 + g;
        const int rtb = g == 2 ? 1 : g == 3 ? 3 : 6;
        const int cb0 = g == 1 ? 4 : 0, cb1 = g == 0 ? 4 : 7;
        const int tro = bf6::tr_lane_off(lr, lg);
        for (int j = nl - 1; j >= 0; --j) {
            __syncthreads();                           // A
            VIHMC_CH_STAMP(j, 0)
            const BwdChainLayer& L = N.L[j];
            const int NI4 = (L.n_in + 3) & ~3;
            const int ntj = __builtin_amdgcn_readfirstlane((NI4 + 16) >> 4);
            __syncthreads();                           // A2: the dX waves hold their W fragments
            VIHMC_CH_STAMP(j, 1)
            if (j >= 2) dma_image(j - 1, g, 4);       // the next layer's image (layers >= 1)
            // weight gradient of layer j over the 64 rows (k = the rows, two 32-row blocks)
            f32x4 acc[2][7];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int t = 0; t < 7; ++t) acc[s2][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int s = 0; s < 2; ++s) {
                const unsigned char* buf = sm + s * CH_BUF;
                bf16x8 da[2][3], hb[2][3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    da[0][p] = tr_frag(buf + CH_DP + p * CH_PLANE, tro, 16 * rta);
                    da[1][p] = tr_frag(buf + CH_DP + p * CH_PLANE, tro, 16 * rtb);
                    hb[0][p] = tr_frag(buf + CH_HP + p * CH_PLANE, tro, 0);
                }
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= ntj) break;
                    if (t + 1 < ntj) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) hb[(t + 1) & 1][p] = tr_frag(buf + CH_HP + p * CH_PLANE, tro, 16 * (t + 1));
                    }
                    acc[0][t] = six(da[0], hb[t & 1], acc[0][t]);
                    if (t >= cb0 && t < cb1) acc[1][t] = six(da[1], hb[t & 1], acc[1][t]);
                }
            }
#if CH_STAMP
            asm volatile("" :: "v"(acc[0][0]), "v"(acc[1][6]));
#endif
            VIHMC_CH_STAMP(j, 2)
            if (j >= 2) bf6::wait_vmcnt0();            // the image DMA landed
            __syncthreads();                           // B
            VIHMC_CH_STAMP(j, 3)
            // the tiled partial slab of layer j (bwd_tile_off, as k_bwd_bf2): one 1-KB store per tile
            float* part = N.dwpart + c * N.dwpart_cs + L.part_off + (int64_t)wg * L.part_stride;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int tn = s2 == 0 ? rta : rtb;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= ntj || (s2 == 1 && (t < cb0 || t >= cb1))) continue;
                    if (tn < 6 || lg == 0) *reinterpret_cast<f32x4*>(part + bwd_tile_off(tn, t, ntj, lane)) = acc[s2][t];
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

bool bwd_chain_ok(const BwdChainArgs& a) {
    for (int net = 0; net < 2; ++net) {
        const BwdChainNet& n = a.net[net];
        if (n.nl < 2 || n.nl > BWD_CHAIN_MAXL || !n.wimg || (n.ldd & 3) || n.ldd < 100 || n.n_wg * CH_ROWS < n.M ||
            (n.n_wg - 1) * CH_ROWS >= n.M)
            return false;
        for (int j = 0; j < n.nl; ++j) {
            const BwdChainLayer& L = n.L[j];
            if (L.n_out != 100 || (L.ldh & 3) || ((L.n_in + 3) & ~3) >= 112 || (j >= 1 && L.n_in != 100) ||
                ((L.n_in + 3) >> 2) * CH_ROWS > 512 * CH_HSLOTS)
                return false;
        }
    }
    return fwd_img_plane_stride() == CH_WPLANE;
}

hipError_t launch_bwd_chain(const BwdChainArgs& a, hipStream_t s) {
    if (!bwd_chain_ok(a)) return hipErrorInvalidValue;
    const int blocks = a.C * (a.net[0].n_wg + a.net[1].n_wg);
    hipLaunchKernelGGL(k_bwd_chain, dim3(blocks), dim3(CH_THREADS), CH_LDS, s, a);
    return hipGetLastError();
}

int bwd_chain_rows() { return CH_ROWS; }

// timing-only / instrumentation switches this translation unit was built with (0 = product build)
int diag_switches_bwd_chain() { return CH_STAMP << 8; }

}  // namespace vihmc
