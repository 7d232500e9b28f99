// Fused layer backward with fp32 products on the bf16 MFMA (bf16x6, vihmc_bf16x6.h): the same BwdProb
// contract and outputs as k_bwd_ws (vihmc_layers.hip), for layers with n_out = 100 and n_in < 109.
//
// Replaces the autograd backward of one nn.Linear + activation of the branch / trunk MLPs
// (Operator_network/VI_HMC/my_make_func.py:53-82, torch autograd through F.linear and tanh):
//   Dout[m][i] = (sum_k D[m][k] W[k][i]) * act'(H[m][i])        (dX, when has_dx)
//   part[n][j] = sum_m D[m][n] H[m][j],  part[n_out][n] = sum_m D[m][n]   (dW, db partial of this chunk)
//
// One 1024-thread workgroup per CU (16 waves, 4 per SIMD, <= 128 VGPRs) per row chunk (a multiple of 32 rows);
// 32-row sub-tiles of D and H are split into bf16 planes in LDS, two buffers, one barrier per sub-tile.
// 16 waves = 8 dX + 4 dW + 4 staging waves (one dW and one staging wave per SIMD). LDS (151 KB):
//   2 x [D planes [3][32][224 B], H planes [3][32][224 B], D fp32 tail [32][4] (features 96..99)]
//   W^T planes [3][100][224 B] + fp32 tail [100][4], split once per workgroup
//   staging (4 waves): the deltas of sub-tile i+1 into the free buffer while the others compute sub-tile i, i+2 in
//                 flight in registers (3 slots per lane on layers with a dX part, whose two single-tile dX waves
//                 carry the last 32 items; 4 otherwise). Branch-free: per-lane global and LDS offsets fixed at kernel
//                 start, loads through buffer resources based at the sub-tile (rows past M read 0), so a slot costs
//                 its loads, the exact split and three LDS stores. The h rows are staged by the dX waves.
//   dX waves (8): i-tiles {2p, 2p+1} x 16-row half h. A = W^T rows, B = D rows (ds_read_b128 of the planes);
//                 the 4-long k tail is one exact f32 MFMA that seeds the accumulator. Epilogue: act'(h) from
//                 the fp32 h rows the wave staged itself, buffer stores (rows past the chunk and columns past n_in
//                 dropped by the range check).
//   dW waves (4): output row tiles x column tiles by transposed reads (k = the 32 rows of the sub-tile); db[n]
//                 from the MFMAs through a constant-one column of H at column NI4 (exact products).
// Deterministic: every partial slab has exactly one writer, reduced in a fixed order by k_reduce.
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

constexpr int BB_SUB = BWD_SUB;                        // 32 rows per sub-tile
constexpr int BB_PITCH = bf6::PITCH;                   // D / H plane rows (transposed reads: 7 x 32 B)
constexpr int BB_PLANE = BB_SUB * BB_PITCH;            // 7168
constexpr int BB_DP = 0;                               // D planes
constexpr int BB_HP = 3 * BB_PLANE;                    // H planes
constexpr int BB_DT = 6 * BB_PLANE;                    // D fp32 tail [32][4]
constexpr int BB_BUF = BB_DT + BB_SUB * 16;            // 43520 bytes per buffer
// W^T plane rows: read like the D planes (lane l: row l & 15, 16-B column l >> 4), so the same pitch residue
// (8 mod 16 dwords) keeps the b128 reads conflict free; 208 B (4 mod 16) measured 2-way
constexpr int BB_WPITCH = 224;
constexpr int BB_WPLANE = 100 * BB_WPITCH;             // 22400 (rows 0..99; tile-6 reads clamp to row 99)
constexpr int BB_W = 2 * BB_BUF;                       // W^T planes after the two sub-tile buffers
constexpr int BB_WT = BB_W + 3 * BB_WPLANE;            // W^T fp32 tail [100][4]
constexpr int BB_LDS = BB_WT + 100 * 16;               // 154880
static_assert(BB_LDS <= 160 * 1024, "LDS");
static_assert(BB_BUF + 2 * BB_PLANE < 65536, "LDS store offsets fit the ds_write immediate");
constexpr int BB_THREADS = 1024;                       // 8 dX + 4 dW + 4 staging waves, 4 per SIMD
constexpr int B2_HSLOTS = 2;                           // staged H float4 per dX lane (<= 32 x 28 per sub-tile / 512)

// H planes: 8-B slot c4 of sub-tile row r sits at slot c4 ^ ((r >> 2) & 3) (a permutation inside each aligned group of
// four slots). The dX waves store h in the epilogue's layout -- 16 lanes of a store group on 16 rows, one slot each --
// and the 224-B pitch puts rows r and r + 4 on one bank (56 r mod 32 dwords): 4-way conflicts on every h store (~670
// of the sub-tile's LDS-array cycles) without the swizzle. The transposed reads of the dW waves stay conflict free:
// a read group's rows 4lg .. 4lg + 3 share (r >> 2) & 3 = lg, so it reads each row's 32 bytes in a permuted order.
__device__ __forceinline__ int hslot(int r, int c4) { return c4 ^ ((r >> 2) & 3); }

__device__ __forceinline__ float act_grad_bf(int act, float h) {
#pragma clang fp contract(off)
    // derivative from the activation's output (tanh: 1 - h^2, relu: h > 0), as act_grad_from_out_l
    if (act == ACT_TANH) return 1.f - h * h;   // h * h rounded first (no fused multiply-add)
    if (act == ACT_RELU) return h > 0.f ? 1.f : 0.f;
    return 1.f;
}
__device__ __forceinline__ float tanh_grad(float h) {
#pragma clang fp contract(off)
    return 1.f - h * h;                                // h * h rounded first (no fused multiply-add)
}
}  // namespace

#if BB_STAMP
// every 16th trunk workgroup of the launches with a dX part (the last one written wins: layer 1): per wave and
// sub-tile s_memtime at the barrier exit [0] and at the role's phase ends [1..5] (staging: stores, loads; dX: MFMAs
// issued, epilogue stores, h stores, act', h loads; dW: fragment reads, MFMAs issued), each fenced by a scheduling
// barrier; per workgroup s_memtime / s_memrealtime at start and end (scripts/diag/stamps_bwd.py)
constexpr int BBS_WG = 16, BBS_SUB = 32, BBS_K = 6;
__device__ unsigned long long bb_stamps[BBS_WG][16][BBS_SUB][BBS_K];
__device__ unsigned long long bb_real[BBS_WG][2][2];
#define VIHMC_BB_STAMP(I, K)                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                        \
    if (samp && lane == 0 && (I) < BBS_SUB) bb_stamps[sidx][wave][(I)][(K)] = __builtin_amdgcn_s_memtime();   \
    __builtin_amdgcn_sched_barrier(0);
#else
#define VIHMC_BB_STAMP(I, K)
#endif
constexpr int BBS_NONE = 1 << 20;                      // stamp index of the prologue's h stage: never recorded

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
    const int hq4 = NI4 >> 2;                          // H float4 per row (<= 27)
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
        // thread's W^T loads (n_in * 25 <= 2500 float4 over 768 threads: <= 4) issued before the first split, so
        // the prologue waits out one HBM latency instead of one per iteration
        const float* WT = P.WT + c * P.wt_cs;
        constexpr int WTH = 768;
        constexpr int WSL = (100 * 25 + WTH - 1) / WTH;
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

    // no static wave priority: with 3 staging slots (round 5) the staging waves are no longer the critical path, and
    // at priority 1 (round 2, profiles/r02p_stamps.log) their split VALU held back the dX waves' epilogues: 52.5 ->
    // 51.0 us per launch without it, the dX waves at priority 1 or the dW waves at 1 no better (profiles/r05r_ab.txt)
    if (wave >= 12) {
        // ---------------- staging role ----------------
        // wave-slot ws = 4 v + g (g = staging wave, v = slot) carries D items e = 64 ws + lane (800 of them: 32 rows x
        // 25 float4) wrapped modulo 800: a lane past the end moves an item another lane moves too (the same value to the
        // same LDS address), so no slot is ever skipped; the offsets are constant over the sub-tiles. The h rows are
        // the dX waves' (below): split between the two roles, neither is the period's critical path alone.
        const int g = __builtin_amdgcn_readfirstlane(wave - 12);
        // db column: H column NI4 of both buffers is the constant 1 (planes 1, 0, 0), never overwritten by the
        // H stores (columns < NI4), so the dW MFMAs produce part[n][NI4] = sum_m D[m][n] = db[n] exactly
        // (the products D x 1 are exact; fp32 accumulation) in the column tile that already covers it
        {
            const int t = tid - 768;
            if (t < 2 * BB_SUB) {
                unsigned char* o = smw + (t >> 5) * BB_BUF + BB_HP + (t & 31) * BB_PITCH + 8 * hslot(t & 31, NI4 >> 2);
                *reinterpret_cast<unsigned short*>(o) = 0x3F80;
                *reinterpret_cast<unsigned short*>(o + BB_PLANE) = 0;
                *reinterpret_cast<unsigned short*>(o + 2 * BB_PLANE) = 0;
            }
        }
        // NS = 3 slots (items 0..767) on layers with a dX part, whose two single-tile dX waves carry the last 32
        // items (dX role); 4 (items wrapped modulo 800) on the others
        auto stage_run = [&](auto ns_c) __attribute__((always_inline)) {
        constexpr int B2_SLOTS = decltype(ns_c)::value;
        uint32_t voff[B2_SLOTS], loff[B2_SLOTS], toff[B2_SLOTS];
        bool tl[B2_SLOTS];
#pragma unroll
        for (int v = 0; v < B2_SLOTS; ++v) {
            const int e = ((4 * v + g) * 64 + lane) % (BB_SUB * 25);
            const int r = e / 25, c4 = e - r * 25;
            voff[v] = (uint32_t)(r * P.ldd + 4 * c4) * 4u;
            loff[v] = (uint32_t)(BB_DP + r * BB_PITCH + 8 * c4);
            tl[v] = c4 == 24;
            toff[v] = (uint32_t)(BB_DT + r * 16);
        }
        // two register sets: sub-tile s is loaded into set s & 1 two sub-tiles before its store, so a load has
        // a whole sub-tile period plus the store phase to land
        f32x4 pfa[B2_SLOTS], pfb[B2_SLOTS];
        auto load = [&](int sub, f32x4 (&pf)[B2_SLOTS]) __attribute__((always_inline)) {
            // resources based at the sub-tile's first row: rows past M read 0 (a partial last sub-tile)
            const __amdgpu_buffer_rsrc_t rs = bf6::make_rsrc(D + (int64_t)sub * P.ldd, (uint32_t)((P.M - sub) * P.ldd * 4));
#pragma unroll
            for (int v = 0; v < B2_SLOTS; ++v)
                pf[v] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[v], 0, 0));
        };
        auto store = [&](int buf, const f32x4 (&pf)[B2_SLOTS]) __attribute__((always_inline)) {
#pragma unroll
            for (int v = 0; v < B2_SLOTS; ++v) {
                bf16x4 p0, p1, p2;
                split4(pf[v], p0, p1, p2);
                unsigned char* base = smw + buf * BB_BUF + loff[v];
                *reinterpret_cast<bf16x4*>(base) = p0;
                *reinterpret_cast<bf16x4*>(base + BB_PLANE) = p1;
                *reinterpret_cast<bf16x4*>(base + 2 * BB_PLANE) = p2;
                if (tl[v]) *reinterpret_cast<f32x4*>(smw + buf * BB_BUF + toff[v]) = pf[v];
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
            store(0, pfa);
            load(sub_at(2), pfa);
        }
        int i = 0;
        for (; i + 1 < nsub; i += 2) {
            __syncthreads();                           // buffer 0 holds sub-tile i, buffer 1 is free
            VIHMC_BB_STAMP(i, 0)
            store(1, pfb);
            VIHMC_BB_STAMP(i, 1)
            load(sub_at(i + 3), pfb);
            VIHMC_BB_STAMP(i, 2)
            __syncthreads();                           // buffer 1 holds sub-tile i + 1, buffer 0 is free
            VIHMC_BB_STAMP(i + 1, 0)
            if (i + 2 < nsub) store(0, pfa);
            VIHMC_BB_STAMP(i + 1, 1)
            load(sub_at(i + 4), pfa);
            VIHMC_BB_STAMP(i + 1, 2)
        }
        if (i < nsub) {
            __syncthreads();                           // the last sub-tile (odd count): nothing left to stage
            VIHMC_BB_STAMP(i, 0)
            VIHMC_BB_STAMP(i, 1)
            VIHMC_BB_STAMP(i, 2)
        }
        };
        if (P.has_dx) stage_run(std::integral_constant<int, 3>{});
        else stage_run(std::integral_constant<int, 4>{});
    } else if (wave < 8) {
        // ---------------- dX role: i-tiles {2p, 2p+1} x row half h ----------------
        // The role body is instantiated per tile count (TWO) and the epilogue per activation (tanh or the rest),
        // so no exec-masked branch splits the LDS reads from the MFMAs that consume them: hipcc then issues
        // the nine D fragment reads of a sub-tile ahead with counted lgkmcnt waits. has_dx implies n_in = 100
        // (bwd_bf_ok), so the columns past n_in are exactly the ones the store offsets send out of range.
        const int h = wave & 1, p2 = wave >> 1;
        const int t0 = 2 * __builtin_amdgcn_readfirstlane(p2);
        const unsigned char* wrow0 = smw + BB_W + min(16 * t0 + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const unsigned char* wrow1 = smw + BB_W + min(16 * (t0 + 1) + lr, P.n_in - 1) * BB_WPITCH + 16 * lg;
        const float* wtl = reinterpret_cast<const float*>(smw + BB_WT);
        const int wr0 = min(16 * t0 + lr, P.n_in - 1), wr1 = min(16 * (t0 + 1) + lr, P.n_in - 1);
        // Dout through a buffer resource: rows past r1 (another workgroup's) and columns past NI4 get an out-of-range
        // offset instead of a branch around the store
        const __amdgpu_buffer_rsrc_t drs =
            bf6::make_rsrc(P.Dout + c * P.o_cs, (uint32_t)((int64_t)P.M * P.ldh * 4));
        // h-row staging (the staging waves move the deltas); sub-tile s is loaded into set s & 1 two sub-tiles before
        // its store. Layers with a dX part (n_in = 100): lane (lr, lg) stages exactly the float4 its own epilogue
        // multiplies -- row 16 h + lr, columns 16 (t0 + v) + 4 lg, clamped to float4 24 (columns 96..99: a duplicate of
        // lane lg = 0's item, never the constant-1 db column 100) -- so act'(h) comes from the fp32 rows at staging
        // time and waits in registers for the epilogue instead of being rebuilt from the three LDS planes per element
        // (5 VALU and 3 LDS reads per element less; the same h, so bitwise the same deltas). Other layers: item
        // e = tid + 512 v of the sub-tile's 32 x hq4 float4, wrapped like the staging role's.
        const int slast = r0 + max(nsub - 1, 0) * BB_SUB;
        auto hsub_at = [&](int k) { return min(r0 + k * BB_SUB, slast); };
        auto dx_run = [&](auto dx_c, auto two_c, auto tanh_c) __attribute__((always_inline)) {
            constexpr bool DX = decltype(dx_c)::value;
            constexpr bool TWO = decltype(two_c)::value;
            constexpr bool TANH = decltype(tanh_c)::value;
            constexpr int NU = TWO ? 2 : 1;
            // The single-tile dX waves of a dX layer (i-tile 6: only lanes lg = 0 have an h item, columns 96..99) stage
            // ONE slot: lanes lg >= 1 carry the staging role's last 32 delta items (768..799, wrapped; the staging
            // waves then take 3 slots instead of 4 -- 1,024 staged items for 800 before)
            constexpr bool MIX = DX && !TWO;
            constexpr int NS = MIX ? 1 : B2_HSLOTS;
            const bool dlane = MIX && lg != 0;
            uint32_t hvoff[NS], hloff[NS], dvoff = bf6::OOB;
            bool dtail = false;
            uint32_t dtoff = 0;
#pragma unroll
            for (int v = 0; v < NS; ++v) {
                int r, c4;
                if (DX) {
                    r = 16 * h + lr;
                    c4 = min(4 * (t0 + v) + lg, 24);
                } else {
                    const int e = (tid + 512 * v) % (BB_SUB * hq4);
                    r = e / hq4;
                    c4 = e - r * hq4;
                }
                hvoff[v] = (uint32_t)(r * P.ldh + 4 * c4) * 4u;
                hloff[v] = (uint32_t)(BB_HP + r * BB_PITCH + 8 * hslot(r, c4));
            }
            if (MIX) {
                const int e = 768 + (48 * h + 16 * (lg - 1) + lr) % 32;
                const int r = e / 25, c4 = e - r * 25;
                if (dlane) {
                    dvoff = (uint32_t)(r * P.ldd + 4 * c4) * 4u;
                    hvoff[0] = bf6::OOB;
                    hloff[0] = (uint32_t)(BB_DP + r * BB_PITCH + 8 * c4);
                    dtail = c4 == 24;
                    dtoff = (uint32_t)(BB_DT + r * 16);
                }
            }
            auto hload = [&](int sub, f32x4 (&hs)[NS]) __attribute__((always_inline)) {
                const __amdgpu_buffer_rsrc_t rs = bf6::make_rsrc(H + (int64_t)sub * P.ldh, (uint32_t)((P.M - sub) * P.ldh * 4));
#pragma unroll
                for (int v = 0; v < NS; ++v)
                    hs[v] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, hvoff[v], 0, 0));
                if (MIX) {
                    // both loads by every lane, one of them out of range (reads 0, no memory traffic)
                    const __amdgpu_buffer_rsrc_t ds = bf6::make_rsrc(D + (int64_t)sub * P.ldd, (uint32_t)((P.M - sub) * P.ldd * 4));
                    const f32x4 dv = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ds, dvoff, 0, 0));
                    if (dlane) hs[0] = dv;
                }
            };
            auto hstore = [&](int buf, const f32x4 (&hs)[NS]) __attribute__((always_inline)) {
#pragma unroll
                for (int v = 0; v < NS; ++v) {
                    bf16x4 p0, p1, p2;
                    split4(hs[v], p0, p1, p2);
                    unsigned char* base = smw + buf * BB_BUF + hloff[v];
                    *reinterpret_cast<bf16x4*>(base) = p0;
                    *reinterpret_cast<bf16x4*>(base + BB_PLANE) = p1;
                    *reinterpret_cast<bf16x4*>(base + 2 * BB_PLANE) = p2;
                }
                if (MIX && dtail) *reinterpret_cast<f32x4*>(smw + buf * BB_BUF + dtoff) = hs[0];
            };
            f32x4 hsa[NS], hsb[NS];                    // per instantiation: no register set live across the dispatch
            f32x4 ag[NU];                              // act'(h) of the staged sub-tile (dX layers), epilogue operand
            auto hstage = [&](int buf, const f32x4 (&hs)[NS], int si) __attribute__((always_inline)) {
                hstore(buf, hs);
                VIHMC_BB_STAMP(si, 3)
                if (DX) {
#pragma unroll
                    for (int u = 0; u < NU; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) ag[u][r] = TANH ? tanh_grad(hs[u][r]) : act_grad_bf(P.act, hs[u][r]);
                }
                VIHMC_BB_STAMP(si, 4)
            };
            if (nsub > 0) {
                hload(hsub_at(0), hsa);
                hload(hsub_at(1), hsb);
                hstage(0, hsa, BBS_NONE);
                hload(hsub_at(2), hsa);
            }
            bf16x8 wra[3][3];                          // [kb][plane] W^T fragments of the first i-tile (registers)
            float wta = 0.f, wtb = 0.f;
            auto dx_sub = [&](int i) __attribute__((always_inline)) {
                const int sub = r0 + i * BB_SUB;
                if (!DX) return;
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
                const float dtl = reinterpret_cast<const float*>(buf + BB_DT)[(16 * h + lr) * 4 + lg];
                f32x4 acc[2];
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wta, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                acc[1] = TWO ? __builtin_amdgcn_mfma_f32_16x16x4f32(wtb, dtl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < 3; ++kb) {
                    bf16x8 db[3];                      // the delta fragments of this k-block (12 VGPRs at a time)
#pragma unroll
                    for (int p = 0; p < 3; ++p) db[p] = *reinterpret_cast<const bf16x8*>(drow + p * BB_PLANE + 64 * kb);
                    acc[0] = six(wra[kb], db, acc[0]);
                    if (TWO) {
                        // only the first i-tile's W^T in registers (VGPR budget); the second re-read from LDS
                        bf16x8 wb[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p) wb[p] = *reinterpret_cast<const bf16x8*>(wrow1 + p * BB_WPLANE + 64 * kb);
                        acc[1] = six(wb, db, acc[1]);
                    }
                }
#if BB_STAMP
                asm volatile("" :: "v"(acc[0]), "v"(acc[1]));
                VIHMC_BB_STAMP(i, 1)
#endif
                const int m = sub + 16 * h + lr;
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int col = 16 * (t0 + u) + 4 * lg;
                    const uint32_t off = (m < r1 && col < NI4) ? (uint32_t)(m * P.ldh + col) * 4u : bf6::OOB;
                    f32x4 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) o[r] = acc[u][r] * ag[u][r];
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bf6::u32x4, o), drs, off, 0, 0);
                }
                VIHMC_BB_STAMP(i, 2)
            };
            // unrolled by two (static register sets, every load unconditional: see the staging role)
            int i = 0;
            for (; i + 1 < nsub; i += 2) {
                __syncthreads();                       // buffer 0 holds sub-tile i
                VIHMC_BB_STAMP(i, 0)
                dx_sub(i);
                hstage(1, hsb, i);                     // h of sub-tile i + 1 into the free buffer (+ its act')
                hload(hsub_at(i + 3), hsb);
                VIHMC_BB_STAMP(i, 5)
                __syncthreads();                       // buffer 1 holds sub-tile i + 1
                VIHMC_BB_STAMP(i + 1, 0)
                dx_sub(i + 1);
                if (i + 2 < nsub) hstage(0, hsa, i + 1);
                hload(hsub_at(i + 4), hsa);
                VIHMC_BB_STAMP(i + 1, 5)
            }
            if (i < nsub) {
                __syncthreads();
                VIHMC_BB_STAMP(i, 0)
                dx_sub(i);
            }
        };
        // instantiated per dX part too: with a run-time has_dx the Dout stores were conditional, so hipcc's counted
        // wait before each h split had to assume they might be missing and also waited for the NEXT set's loads,
        // issued half a period earlier (vmcnt(2) instead of 4: the dX waves' ~1,100-cycle split phase in the stamps)
        const bool tanh_act = P.act == ACT_TANH;
        if (!P.has_dx) dx_run(std::false_type{}, std::true_type{}, std::true_type{});
        else if (t0 + 1 < 7) {
            if (tanh_act) dx_run(std::true_type{}, std::true_type{}, std::true_type{});
            else dx_run(std::true_type{}, std::true_type{}, std::false_type{});
        } else {
            if (tanh_act) dx_run(std::true_type{}, std::false_type{}, std::true_type{});
            else dx_run(std::true_type{}, std::false_type{}, std::false_type{});
        }
    } else {
        // ---------------- dW role: two row tiles per wave, the second over a column range ----------------
        // Waves w, w + 4, w + 8, w + 12 share a SIMD. The dX waves of SIMD groups 0 and 1 (waves 0/4, 1/5) carry
        // four tile-jobs of 20 MFMA-equivalents, those of groups 2 and 3 three; a dW (row, column) tile-job is 6
        // MFMAs. Groups 2 and 3 (waves 10, 11) take row tiles {0, 1} and {2, 3} whole (14 jobs), groups 0 and 1
        // (waves 8, 9) row tile 4 or 5 whole plus row tile 6 (rows 96..99 of n_out) over columns 0..3 or 4..6:
        // at most 146 MFMA-equivalents per SIMD.
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
        const int troh = (4 * lg + (lr >> 2)) * BB_PITCH + 8 * ((lr & 3) ^ lg);   // the H planes' slot swizzle (hslot)
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
                    hb[0][p] = tr_frag(buf + BB_HP + p * BB_PLANE, troh, 0);
                }
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    if (t >= nt) break;                    // wave-uniform (NT = 0 only)
                    if (t + 1 < nt) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) hb[(t + 1) & 1][p] = tr_frag(buf + BB_HP + p * BB_PLANE, troh, 16 * (t + 1));
                    }
                    acc[0][t] = six(da[0], hb[t & 1], acc[0][t]);
                    if (t >= cb0 && t < cb1) acc[1][t] = six(da[1], hb[t & 1], acc[1][t]);
                }
#if BB_STAMP
                asm volatile("" :: "v"(acc[0][0]), "v"(acc[1][6]));
                VIHMC_BB_STAMP(i, 2)
#endif
            }
        };
        if (ntj == 7) dw_run(std::integral_constant<int, 7>{});
        else dw_run(std::integral_constant<int, 0>{});
        // the tiled partial slab (bwd_tile_off): each accumulator quad as it stands, one 1-KB store per tile
        float* part = P.part + c * P.part_cs + (int64_t)wg * P.part_stride;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int tn = s2 == 0 ? rta : rtb;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                if (t >= ntj || (s2 == 1 && (t < cb0 || t >= cb1))) continue;
                if (tn < 6 || lg == 0) *reinterpret_cast<f32x4*>(part + bwd_tile_off(tn, t, ntj, lane)) = acc[s2][t];
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
        // the db column sits at H column NI4 inside the last column tile: NI4 < 112; chunks of whole sub-tiles
        // (a sub-tile never straddles two workgroups' rows)
        if (p.n_out != 100 || ((p.n_in + 3) & ~3) >= 112 || (p.has_dx && p.n_in != 100)) return false;
        if ((p.ldd & 3) || (p.ldh & 3) || (p.has_dx && (p.ldw & 3)) || p.rows_per_wg % BWD_SUB) return false;
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

hipError_t launch_bwd_bf(const BwdArgs& a, hipStream_t s) {
    if (!bwd_bf_ok(a)) return hipErrorInvalidValue;
    const int blocks = a.C * a.p[0].n_wg + (a.nprob > 1 ? a.C * a.p[1].n_wg : 0);
    hipLaunchKernelGGL(k_bwd_bf2, dim3(blocks), dim3(BB_THREADS), BB_LDS, s, a);
    return hipGetLastError();
}


}  // namespace vihmc
