// Fused hidden-layer forward of both DeepONet MLPs (branch + trunk), width 100.
//
// Replaces, for layers 1..L-1 of each net, the per-layer F.linear + tanh of
// Operator_network/VI_HMC/my_make_func.py:52-77 (Functional_DeepONet branch/trunk loops).
//
// Why fused: with the transposed accumulator layout (MFMA A operand = weight rows n, B operand =
// activation rows m), lane l of a wave ends a layer holding O[m = l&15][n = 16t + 4(l>>4) + r] in
// register r of accumulator t -- which is exactly the k-permuted float4 B operand the next layer needs
// for k-block t. So a wave can carry its 16 rows through every hidden layer in registers: HBM sees only
// the h_j stores (kept for the backward) instead of a load + store per layer, and the per-layer kernels'
// separate memory and MFMA phases disappear. Only the 4-wide k tail (columns 96..99) needs a cross-lane
// move (4 ds_bpermute).
//
// Workgroup = 12 waves (192 rows; 4 waves for small chain batches); the weights + bias of layer j sit in LDS buffer j&1 (row stride 104:
// conflict-free b128 row reads, see rowdot_ldb), layer j+1's are prefetched into registers by all 768
// threads while layer j computes and stored into the other buffer: one barrier per layer.
// Blocks are chain-fastest (c = blockIdx % C) so, with C a multiple of 8, all blocks of one chain run on
// one XCD and share its L2 copy of that chain's weights.
#include "vihmc_internal.h"
#include "vihmc_bf16x6.h"

namespace vihmc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int FW = 100;                  // layer width (n_in == n_out)
constexpr int FLDB = 104;                // LDS row stride (== 8 mod 16)
constexpr int FBUF = FW * FLDB + 116;    // one weight buffer: 100 rows + bias (zero padded to 112) + dump float4
constexpr int FBLK4 = (FW * FW + FW) / 4;                        // float4 in W + bias (2525)

__device__ __forceinline__ f32x4 mfma_f(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}


__device__ __forceinline__ float tanh_f(float x) { return tanh_acc(x); }

template <int ACT>
__device__ __forceinline__ float act_t(float z) {
    if constexpr (ACT == ACT_TANH) return (FWD_ABL & 2) ? z : tanh_f(z);
    else if constexpr (ACT == ACT_TANH_CR) return (FWD_ABL & 2) ? z : tanh_cr(z);   // each net's last hidden layer
    else if constexpr (ACT == ACT_RELU) return fmaxf(z, 0.f);
    else return z;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Buffer resource over [p, p + bytes) from wave-uniform inputs; out-of-range stores are dropped by the
// hardware range check, which keeps the epilogue free of exec-mask branches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

constexpr uint32_t OOB = 0x80000000u;

// One fused layer for one wave: acc = W a (+ bias, activation), h stored, next operand returned in
// na / h6. Straight-line (no runtime branches) so the scheduler can interleave a column-tile pair's
// epilogue with the next pair's MFMAs.
template <int ACT>
__device__ __forceinline__ void fused_layer(const float* wb, const float4 (&a)[6], float atl, int lr, int lg,
                                            __amdgpu_buffer_rsrc_t orsrc, uint32_t ooff, float4 (&na)[6],
                                            float4& h6) {
    const float* bb = wb + FW * FLDB;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int t0 = 2 * p, t1 = 2 * p + 1;          // t1 == 7 does not exist
        const float* w0r = wb + min(16 * t0 + lr, FW - 1) * FLDB;
        const float* w1r = wb + min(16 * t1 + lr, FW - 1) * FLDB;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) {
            const float4 w0 = *reinterpret_cast<const float4*>(w0r + 16 * kb + 4 * lg);
            if (t1 < 7) {
                const float4 w1 = *reinterpret_cast<const float4*>(w1r + 16 * kb + 4 * lg);
                acc0 = mfma_f(w0.x, a[kb].x, acc0);
                acc1 = mfma_f(w1.x, a[kb].x, acc1);
                acc0 = mfma_f(w0.y, a[kb].y, acc0);
                acc1 = mfma_f(w1.y, a[kb].y, acc1);
                acc0 = mfma_f(w0.z, a[kb].z, acc0);
                acc1 = mfma_f(w1.z, a[kb].z, acc1);
                acc0 = mfma_f(w0.w, a[kb].w, acc0);
                acc1 = mfma_f(w1.w, a[kb].w, acc1);
            } else {
                acc0 = mfma_f(w0.x, a[kb].x, acc0);
                acc0 = mfma_f(w0.y, a[kb].y, acc0);
                acc0 = mfma_f(w0.z, a[kb].z, acc0);
                acc0 = mfma_f(w0.w, a[kb].w, acc0);
            }
        }
        acc0 = mfma_f(w0r[96 + lg], atl, acc0);
        if (t1 < 7) acc1 = mfma_f(w1r[96 + lg], atl, acc1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int t = u == 0 ? t0 : t1;
            if (t >= 7) continue;
            const f32x4& acc = u == 0 ? acc0 : acc1;
            const int n = 16 * t + 4 * lg;
            const float4 bv = *reinterpret_cast<const float4*>(bb + n);
            float4 h;
            h.x = n + 0 < FW ? act_t<ACT>(acc[0] + bv.x) : 0.f;
            h.y = n + 1 < FW ? act_t<ACT>(acc[1] + bv.y) : 0.f;
            h.z = n + 2 < FW ? act_t<ACT>(acc[2] + bv.z) : 0.f;
            h.w = n + 3 < FW ? act_t<ACT>(acc[3] + bv.w) : 0.f;
            // columns >= 100 (t = 6, lg >= 1) and rows >= M (ooff already OOB) are dropped
            const uint32_t off = (t < 6 || lg == 0) ? ooff + 4u * n : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), orsrc, off, 0, 0);
            if (t < 6) na[t] = h;
            else h6 = h;
        }
    }
}

}  // namespace

// NW waves per workgroup (16 NW rows): 12 for a full-chip batch of chains, 4 when the 12-wave grid
// would leave most CUs idle (single chain: 60 workgroups)
template <int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_fwd_fused(FusedArgs args) {
    constexpr int FTHREADS = NW * 64;
    constexpr int FSLOTS = (FBLK4 + FTHREADS - 1) / FTHREADS;
    extern __shared__ float fsm[];       // 2 x FBUF
    const int C = args.C;
    const int c = blockIdx.x % C;
    int item = blockIdx.x / C;
    const int net = item < args.net[0].nblk ? 0 : 1;
    if (net) item -= args.net[0].nblk;
    const FusedNet& N = args.net[net];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int row = item * (16 * NW) + wave * 16 + lr;
    const int rowc = min(row, N.rows - 1);
    const bool rok = row < N.rows;
    const float* Wc = args.packed + c * args.dp;

    // staging slots: float4 idx of the contiguous [W | bias] block -> LDS position
    int sl[FSLOTS];
#pragma unroll
    for (int v = 0; v < FSLOTS; ++v) {
        const int i = tid + FTHREADS * v;
        sl[v] = i < FW * FW / 4 ? (i / (FW / 4)) * FLDB + 4 * (i % (FW / 4))
                                : (i < FBLK4 ? FW * FLDB + 4 * (i - FW * FW / 4) : FW * FLDB + 112);  // idle: dump
    }
    // zero the bias padding (columns 100..111) of both buffers once
    if (tid < 24) fsm[(tid / 12) * FBUF + FW * FLDB + FW + (tid % 12)] = 0.f;
    f32x4 pf[FSLOTS];   // native vector type: a HIP float4 struct array here was left in scratch (memcpy)
#define VIHMC_FW_LOAD(J)                                                                              \
    {                                                                                                 \
        const f32x4* src = reinterpret_cast<const f32x4*>(Wc + N.w_off[J]);                           \
        _Pragma("unroll") for (int v = 0; v < FSLOTS; ++v)                                            \
            pf[v] = src[min(tid + FTHREADS * v, FBLK4 - 1)];                                          \
    }
#define VIHMC_FW_STORE(BUF)                                                                           \
    _Pragma("unroll") for (int v = 0; v < FSLOTS; ++v)                                                \
        *reinterpret_cast<f32x4*>(fsm + (BUF) * FBUF + sl[v]) = pf[v];

    VIHMC_FW_LOAD(0)
    // A operand of the first fused layer: k-permuted float4 per 16-wide k-block + the 4-wide tail
    float4 a[6];
    float atl;
    {
        const float* ar = N.in + c * N.in_cs + (int64_t)rowc * N.ldin;
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) a[kb] = *reinterpret_cast<const float4*>(ar + 16 * kb + 4 * lg);
        atl = ar[96 + lg];
    }
    VIHMC_FW_STORE(0)
    // drain the entry loads here: otherwise the waitcnt pass, merging the loop-entry state (a[] still in
    // flight) with the back edge, puts vmcnt waits before the MFMAs of EVERY layer -- which then also
    // wait for the previous layer's h stores (stores count in vmcnt)
    __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0) expcnt(7) lgkmcnt(15)

    const float* outc = N.out + c * N.out_cs;
    const uint32_t ooff = rok ? (uint32_t)row * (uint32_t)N.ldo * 4u : OOB;
    const uint32_t obytes = (uint32_t)N.rows * (uint32_t)N.ldo * 4u;
    for (int j = 0; j < N.nl; ++j) {
        __syncthreads();                        // buffer j&1 complete; buffer (j+1)&1 no longer read
        // unconditional prefetch (the last layer reloads its own block into the idle buffer): keeps pf in
        // registers -- a conditional load/store pair around the layer body put it in scratch
        VIHMC_FW_LOAD(min(j + 1, N.nl - 1))
        const float* wb = fsm + (j & 1) * FBUF;
        const __amdgpu_buffer_rsrc_t orsrc = make_rsrc(outc + N.h_off[j], obytes);
        float4 na[6];
        float4 h6;
        const int act = N.act[j];
        if (act == ACT_TANH) fused_layer<ACT_TANH>(wb, a, atl, lr, lg, orsrc, ooff, na, h6);
        else if (act == ACT_TANH_CR) fused_layer<ACT_TANH_CR>(wb, a, atl, lr, lg, orsrc, ooff, na, h6);
        else if (act == ACT_RELU) fused_layer<ACT_RELU>(wb, a, atl, lr, lg, orsrc, ooff, na, h6);
        else fused_layer<ACT_ID>(wb, a, atl, lr, lg, orsrc, ooff, na, h6);
        VIHMC_FW_STORE((j + 1) & 1)
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) a[kb] = na[kb];
        // tail operand: lane (lr, lg) needs h[lr][96 + lg], held by lane lr (lg = 0) in component lg
        {
            const float x0 = __shfl(h6.x, lr, 64), x1 = __shfl(h6.y, lr, 64);
            const float x2 = __shfl(h6.z, lr, 64), x3 = __shfl(h6.w, lr, 64);
            atl = lg == 0 ? x0 : (lg == 1 ? x1 : (lg == 2 ? x2 : x3));
        }
    }
#undef VIHMC_FW_LOAD
#undef VIHMC_FW_STORE
}

// =============================================================================================
// bf16x6 variant: the same register-resident layer walk with every product done on the bf16 MFMA.
// Each fp32 operand is split exactly into three bf16 planes x = x0 + x1 + x2 and W.h keeps the six
// terms of order <= 2 (w2h0, w1h1, w0h2, w1h0, w0h1, w0h0, smallest first), accumulated in fp32: as
// accurate as an fp32 dot product (profiles/bf16x6_precision.py) at 6/16 of the fp32 MFMA cycles.
//   k order: 16x16x32 k-block kb covers the column tiles t0 = 2kb, t1 = 2kb + 1; lane (l&15, g = l>>4)
//   holds slots 8g..8g+7 = h[m][16 t0 + 4g + 0..3] and h[m][16 t1 + 4g + 0..3] -- exactly registers
//   0..3 of accumulators t0 and t1 of the previous layer, so activations need no lane movement. The
//   weights are stored in LDS in that permuted order (one b128 per plane per fragment). The k tail
//   (columns 96..99) is one exact 16x16x4 f32 MFMA per tile (FWD_TAILF32, below; the FWD_TAILF32 = 0 form
//   runs six 16x16x16 bf16 MFMAs, whose k layout 4g + j is the accumulator's).
// =============================================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BROW = 112;                         // bf16 per plane row (3 k-blocks x 32 + tile 6 x 16)
constexpr int BPLANE = FW * BROW;                 // bf16 per plane
constexpr int BBUF = 3 * BPLANE * 2 + 112 * 4;    // bytes per buffer: 3 planes + fp32 bias [112]

__device__ __forceinline__ void split3(float x, __bf16& a, __bf16& b, __bf16& c) {
    a = (__bf16)x;
    const float r = x - (float)a;
    b = (__bf16)r;
    c = (__bf16)(r - (float)b);
}

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c,
                                                      0, 0, 0);
}

// one 16-row output tile t: acc += W[16t + lr][:] . h (six bf16 products per k-block)
__device__ __forceinline__ f32x4 bf_tile(const __bf16* wb, int t, int lr, int lg, const bf16x8 (&hp)[3][3],
                                         const bf16x4 (&h6)[3]) {
    const int n = min(16 * t + lr, FW - 1);
    const __bf16* row0 = wb + n * BROW;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 3; ++kb) {
        const int o = kb * 32 + lg * 8;
        const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(row0 + o);
        const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(row0 + BPLANE + o);
        const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(row0 + 2 * BPLANE + o);
        acc = mfma32(w2, hp[0][kb], acc);
        acc = mfma32(w1, hp[1][kb], acc);
        acc = mfma32(w0, hp[2][kb], acc);
        acc = mfma32(w1, hp[0][kb], acc);
        acc = mfma32(w0, hp[1][kb], acc);
        acc = mfma32(w0, hp[0][kb], acc);
    }
    // the K = 16 tail accumulates into its own registers: no accumulator chain crosses the two MFMA shapes.
    // (Chaining a 16x16x32 result straight into a 16x16x16 MFMA's C operand gave wrong tiles with the
    // ROCm 7.2 compiler -- which tile depended on the schedule; scripts/diag/fused_bf_vs_fp32.hip.)
    f32x4 acc6 = {0.f, 0.f, 0.f, 0.f};
    {
        const int o = 96 + lg * 4;
        const bf16x4 w0 = *reinterpret_cast<const bf16x4*>(row0 + o);
        const bf16x4 w1 = *reinterpret_cast<const bf16x4*>(row0 + BPLANE + o);
        const bf16x4 w2 = *reinterpret_cast<const bf16x4*>(row0 + 2 * BPLANE + o);
        acc6 = mfma16(w2, h6[0], acc6);
        acc6 = mfma16(w1, h6[1], acc6);
        acc6 = mfma16(w0, h6[2], acc6);
        acc6 = mfma16(w1, h6[0], acc6);
        acc6 = mfma16(w0, h6[1], acc6);
        acc6 = mfma16(w0, h6[0], acc6);
    }
    return acc + acc6;
}

template <int ACT>
__device__ __forceinline__ float4 bf_epi(const float* bias, int t, int lg, const f32x4& acc,
                                         __amdgpu_buffer_rsrc_t orsrc, uint32_t ooff) {
    const int n = 16 * t + 4 * lg;
    const float4 bv = *reinterpret_cast<const float4*>(bias + n);
    float4 h;
    h.x = n + 0 < FW ? act_t<ACT>(acc[0] + bv.x) : 0.f;
    h.y = n + 1 < FW ? act_t<ACT>(acc[1] + bv.y) : 0.f;
    h.z = n + 2 < FW ? act_t<ACT>(acc[2] + bv.z) : 0.f;
    h.w = n + 3 < FW ? act_t<ACT>(acc[3] + bv.w) : 0.f;
    // one per-lane offset (row + 16 lg bytes) for every tile, the tile's 64 t bytes as the scalar offset: with
    // per-tile lane offsets hipcc hoisted seven of them out of the layer loop and spilled them at 168 VGPRs, and
    // each reload's vmcnt(0) then also waited for this wave's earlier h stores (OOB + 64 t stays out of range)
    const uint32_t off = (t < 6 || lg == 0) ? ooff + 16u * lg : OOB;
#if FWD_ABL & 1
    asm volatile("" :: "v"(h.x), "v"(h.y), "v"(h.z), "v"(h.w));
    (void)off;
    (void)orsrc;
#else
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), orsrc, off, 64 * t, 0);
#endif
    return h;
}

template <int ACT>
__device__ __forceinline__ void bf_layer(const __bf16* wb, const float* bias, const bf16x8 (&hp)[3][3],
                                         const bf16x4 (&h6)[3], int lr, int lg, __amdgpu_buffer_rsrc_t orsrc,
                                         uint32_t ooff, float4 (&hn)[7]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const f32x4 a0 = bf_tile(wb, 2 * p, lr, lg, hp, h6);
        const f32x4 a1 = bf_tile(wb, 2 * p + 1, lr, lg, hp, h6);
        hn[2 * p] = bf_epi<ACT>(bias, 2 * p, lg, a0, orsrc, ooff);
        hn[2 * p + 1] = bf_epi<ACT>(bias, 2 * p + 1, lg, a1, orsrc, ooff);
    }
    const f32x4 a6 = bf_tile(wb, 6, lr, lg, hp, h6);
    hn[6] = bf_epi<ACT>(bias, 6, lg, a6, orsrc, ooff);
}

// fp32 h tiles (this lane: 4 columns 16t + 4lg of its row) -> the three bf16 B-operand planes
__device__ __forceinline__ void bf_split_operand(const float4 (&h)[7], bf16x8 (&hp)[3][3], bf16x4 (&h6)[3]) {
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        const float v[4] = {h[t].x, h[t].y, h[t].z, h[t].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            __bf16 a, b, c;
            split3(v[j], a, b, c);
            if (t < 6) {
                hp[0][t >> 1][(t & 1) * 4 + j] = a;
                hp[1][t >> 1][(t & 1) * 4 + j] = b;
                hp[2][t >> 1][(t & 1) * 4 + j] = c;
            } else {
                h6[0][j] = a;
                h6[1][j] = b;
                h6[2][j] = c;
            }
        }
    }
}

// ---- f32 k tail (FWD_TAILF32): the 4-long k tail (features 96..99) as ONE exact 16x16x4 f32 MFMA that seeds
// each tile's accumulator, instead of six 16x16x16 bf16 MFMAs -- which issue at 16 cycles each on gfx950, the
// same as a 16x16x32 (scripts/diag/mfma_rate.hip): 6 x 16 = 96 -> 32 matrix cycles per tile. Its B operand
// B[k = lg][m = lr] = h[m][96 + lg] must sit in lane (lr, lg): tile 6's A rows are W rows 96 + (lr >> 2)
// (rows 4g .. 4g+3 all W row 96 + g), so accumulator register 0 of lane (lr, lg) is exactly h[lr][96 + lg] --
// no cross-lane move. The image carries the fp32 tail W[n][96..99] ([100][4] after the bias).
constexpr int FWD_WTAIL = 3 * BPLANE * 2 + 112 * 4;   // byte offset of the fp32 W tail [100][4] in an image
constexpr int QI_PITCH = 224;                           // contraction block image (vihmc_contract_bf.hip): plane
constexpr int QI_PLANE = CONTRACT_SPLIT_ROWS * QI_PITCH;  // rows of 112 bf16, 3 planes, then the fp32 tail [32][4]
static_assert(3 * QI_PLANE + CONTRACT_SPLIT_ROWS * 16 <= CONTRACT_SPLIT_BLOCK, "block image");
constexpr int QI_HALF = 16 * QI_PITCH;                  // a wave's 16 rows of one plane (3584 B)
constexpr int QI_WAVE = 3 * QI_HALF + 16 * 16;          // + its tail rows: 11008 B of LDS per wave

__device__ __forceinline__ int tf_row(int t, int lr) { return t < 6 ? 16 * t + lr : 96 + (lr >> 2); }

__device__ __forceinline__ f32x4 tf_tile(const __bf16* wb, const float* wtail, int t, int lr, int lg,
                                         const bf16x8 (&hp)[3][3], float h6) {
    const int n = tf_row(t, lr);
    const __bf16* row0 = wb + n * BROW;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (FWD_ABL & 8) return __builtin_amdgcn_mfma_f32_16x16x4f32(wtail[4 * n + lg], h6, acc, 0, 0, 0);
#pragma unroll
    for (int kb = 0; kb < 3; ++kb) {
        const int o = kb * 32 + lg * 8;
        const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(row0 + o);
        const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(row0 + BPLANE + o);
        const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(row0 + 2 * BPLANE + o);
        acc = mfma32(w2, hp[0][kb], acc);
        acc = mfma32(w1, hp[1][kb], acc);
        acc = mfma32(w0, hp[2][kb], acc);
        acc = mfma32(w1, hp[0][kb], acc);
        acc = mfma32(w0, hp[1][kb], acc);
        acc = mfma32(w0, hp[0][kb], acc);
    }
    // the tail closes the chain (as the last MFMA it cannot be hoisted ahead of the tile: no extra live
    // accumulators; seeding the chain with it spilled 67 VGPRs)
    return __builtin_amdgcn_mfma_f32_16x16x4f32(wtail[4 * n + lg], h6, acc, 0, 0, 0);
}

template <int ACT>
__device__ __forceinline__ void tf_layer(const __bf16* wb, const float* bias, const float* wtail,
                                         const bf16x8 (&hp)[3][3], float h6, int lr, int lg,
                                         __amdgpu_buffer_rsrc_t orsrc, uint32_t ooff, float4 (&hn)[7]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const f32x4 a0 = tf_tile(wb, wtail, 2 * p, lr, lg, hp, h6);
        const f32x4 a1 = tf_tile(wb, wtail, 2 * p + 1, lr, lg, hp, h6);
        hn[2 * p] = bf_epi<ACT>(bias, 2 * p, lg, a0, orsrc, ooff);
        hn[2 * p + 1] = bf_epi<ACT>(bias, 2 * p + 1, lg, a1, orsrc, ooff);
    }
    // tile 6: register 0 of lane (lr, lg) = pre-activation of h[lr][96 + lg]
    const f32x4 a6 = tf_tile(wb, wtail, 6, lr, lg, hp, h6);
    const float v = act_t<ACT>(a6[0] + bias[96 + lg]);
#if FWD_ABL & 1
    asm volatile("" :: "v"(v));
#else
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, ooff + 4u * lg, 4 * 96, 0);
#endif
    hn[6].x = v;
}

// ---- input layer in the forward launch (FusedNet::x): network layer 0 of the wave's 16 rows on the f32 MFMA, every
// tile's products in k_rowdot_in's order (16-long k blocks .x .y .z .w, then the 4-wide tail steps) and its epilogue
// (tanh_f = the row-dot epilogue's tanh_acc; columns >= 100 zero), so h_0 is bitwise the separate launch's. Saves
// that launch and the re-read of h_0: the lanes' accumulators are the layer walk's operand layout already (tile 6
// moved into its f32-tail form by four shuffles).
constexpr int IN0_KMAX = 111;                       // 6 full 16-long k blocks + <= 4 tail steps
__host__ __device__ constexpr int in0_ldw(int k4) { return k4 + ((24 - (k4 & 15)) & 15); }   // rowdot_ldb
__device__ __forceinline__ float in0_act(int act, float z) {
    if (act == ACT_TANH) return tanh_f(z);
    if (act == ACT_TANH_CR) return tanh_cr(z);
    if (act == ACT_RELU) return fmaxf(z, 0.f);
    return z;
}

// x operand of the wave's row: a[kb] = x[16 kb + 4 lg .. + 3] (kb < nkb), atl[q] = x[16 nkb + 4 q + lg] (q < ntl)
__device__ __forceinline__ void in0_load_x(const FusedNet& N, int rowc, int lg, float4 (&a)[6], float (&atl)[4]) {
    const float* xr = N.x + (int64_t)rowc * N.ldx;
    const int nkb = N.k0 >> 4, ntl = (((N.k0 + 3) & ~3) - 16 * nkb) >> 2;
#pragma unroll
    for (int kb = 0; kb < 6; ++kb)
        if (kb < nkb) a[kb] = *reinterpret_cast<const float4*>(xr + 16 * kb + 4 * lg);
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (q < ntl) atl[q] = xr[16 * nkb + 4 * q + lg];
}

__device__ __forceinline__ void in0_layer(const FusedNet& N, const float* w0s, const float* bias, const float4 (&a)[6],
                                          const float (&atl)[4], int lr, int lg, __amdgpu_buffer_rsrc_t hrs,
                                          uint32_t hoff, float4 (&h)[7]) {
    const int nkb = N.k0 >> 4, ntl = (((N.k0 + 3) & ~3) - 16 * nkb) >> 2;
    const int ldw = in0_ldw((N.k0 + 3) & ~3);
    float4 o6;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        const float* wr = w0s + min(16 * t + lr, FW - 1) * ldw;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) {
            if (kb < nkb) {
                const float4 w = *reinterpret_cast<const float4*>(wr + 16 * kb + 4 * lg);
                acc = mfma_f(w.x, a[kb].x, acc);
                acc = mfma_f(w.y, a[kb].y, acc);
                acc = mfma_f(w.z, a[kb].z, acc);
                acc = mfma_f(w.w, a[kb].w, acc);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < ntl) acc = mfma_f(wr[16 * nkb + 4 * q + lg], atl[q], acc);
        const int n = 16 * t + 4 * lg;
        const float4 bv = n < FW ? *reinterpret_cast<const float4*>(bias + n) : float4{0.f, 0.f, 0.f, 0.f};
        float4 o;
        o.x = n + 0 < FW ? in0_act(N.act0, acc[0] + bv.x) : 0.f;
        o.y = n + 1 < FW ? in0_act(N.act0, acc[1] + bv.y) : 0.f;
        o.z = n + 2 < FW ? in0_act(N.act0, acc[2] + bv.z) : 0.f;
        o.w = n + 3 < FW ? in0_act(N.act0, acc[3] + bv.w) : 0.f;
        // columns past the row stride and rows >= M (hoff already out of range) are dropped
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), hrs, n < N.ldin ? hoff + 4u * n : OOB, 0,
                                               0);
        if (t < 6) h[t] = o;
        else o6 = o;
    }
    // tile 6: lane (lr, 0) holds h[96..99]; the layer walk wants h[96 + lg] in register 0 of lane (lr, lg)
    // (FWD_TAILF32), or the accumulator form itself (zeros beyond column 99)
    if (FWD_TAILF32) {
        const float v0 = __shfl(o6.x, lr, 64), v1 = __shfl(o6.y, lr, 64), v2 = __shfl(o6.z, lr, 64),
                    v3 = __shfl(o6.w, lr, 64);
        h[6] = float4{lg == 0 ? v0 : (lg == 1 ? v1 : (lg == 2 ? v2 : v3)), 0.f, 0.f, 0.f};
    } else {
        h[6] = o6;
    }
}

#if FWD_STAMP
// every 8th workgroup (the first 16): per wave (compute, then DMA) and layer s_memtime after the layer's barrier [0],
// after the operand split (compute) / the DMA issue (DMA waves) [1], after the layer's MFMAs + epilogue + h stores
// are issued [2], after the wait before the next barrier [3]; per workgroup s_memtime / s_memrealtime at start and
// end (profiles/scripts/diag/stamps_fwd.py)
constexpr int FWS_WG = 16, FWS_L = 10;
__device__ unsigned long long fw_stamps[FWS_WG][16][FWS_L][4];
__device__ unsigned long long fw_real[FWS_WG][2][2];
#define FW_ST(J, K) \
    if (fw_samp && lane == 0 && (J) < FWS_L) fw_stamps[fw_sidx][wave][(J)][(K)] = __builtin_amdgcn_s_memtime();
#else
#define FW_ST(J, K)
#endif

// ND > 0 (images only): ND extra waves that only issue the weight-image DMA. With four compute waves (one chain) each
// of them otherwise issues 17 one-KB DMA pieces per layer (~100 cycles each among its MFMAs).
template <int NW, int ND = 0>
__global__ __launch_bounds__((NW + ND) * 64, 1) void k_fwd_fused_bf(FusedArgs args) {
    constexpr int FTHREADS = NW * 64;
    constexpr int FSLOTS = (FBLK4 + FTHREADS - 1) / FTHREADS;
    extern __shared__ __attribute__((aligned(16))) unsigned char fsmb[];      // 2 x BBUF
    const int C = args.C;
    const int c = blockIdx.x % C;
    int item = blockIdx.x / C;
    const int net = item < args.net[0].nblk ? 0 : 1;
    if (net) item -= args.net[0].nblk;
    const FusedNet& N = args.net[net];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int row = item * (16 * NW) + wave * 16 + lr;
    const int rowc = min(row, N.rows - 1);
    const bool rok = row < N.rows;
    const float* Wc = args.packed + c * args.dp;
#if FWD_STAMP
    const bool fw_samp = (blockIdx.x % 8) == 0 && blockIdx.x / 8 < FWS_WG;
    const int fw_sidx = blockIdx.x / 8;
    if (fw_samp && tid == 0) {
        fw_real[fw_sidx][0][0] = __builtin_amdgcn_s_memtime();
        fw_real[fw_sidx][0][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (ND > 0 && wave >= NW) {
        // DMA waves: image 0 before the first barrier, image j + 1 after barrier j, each drained before the barrier
        // that publishes it; the same barrier sequence as the compute waves (zero fill, one per layer, epilogue)
        const unsigned char* wimgd = N.wimg + c * N.wimg_cs;
        for (int k = wave - NW; k < FWD_WIMG / 1024; k += ND)
            bf6::glds16_asm(wimgd + k * 1024 + lane * 16, fsmb + k * 1024);
        bf6::wait_vmcnt0();
        __syncthreads();
        for (int j = 0; j < N.nl; ++j) {
            __syncthreads();
            FW_ST(j, 0)
            if (j + 1 < N.nl && !(FWD_ABL & 4)) {
                for (int k = wave - NW; k < FWD_WIMG / 1024; k += ND)
                    bf6::glds16_asm(wimgd + (int64_t)(j + 1) * FWD_WIMG + k * 1024 + lane * 16,
                                    fsmb + ((j + 1) & 1) * FWD_WIMG + k * 1024);
            }
            FW_ST(j, 1)
            bf6::wait_vmcnt0();
            FW_ST(j, 3)
        }
        if (N.qimg != nullptr) __syncthreads();
        return;
    }

    // zero the never-written tail columns 100..111 of every plane row and the bias pad, both buffers
    // (register staging only: the pre-split images carry their zeros)
    if (!N.wimg) {
        for (int i = tid; i < 2 * 3 * FW; i += FTHREADS) {
            __bf16* r = reinterpret_cast<__bf16*>(fsmb + (i / (3 * FW)) * BBUF) + (i % (3 * FW)) * BROW + 100;
#pragma unroll
            for (int z = 0; z < 12; ++z) r[z] = (__bf16)0.f;
        }
        if (tid < 24) reinterpret_cast<float*>(fsmb + (tid / 12) * BBUF + 3 * BPLANE * 2)[100 + tid % 12] = 0.f;
    }

    // staging slot v: float4 i of [W | bias] -> (plane row position) or bias position
    int sdst[FSLOTS];
#pragma unroll
    for (int v = 0; v < FSLOTS; ++v) {
        const int i = tid + FTHREADS * v;
        if (i < FW * FW / 4) {
            const int n = i / (FW / 4), c4 = i % (FW / 4), tq = c4 >> 2, g = c4 & 3;
            const int pos = tq < 6 ? (tq >> 1) * 32 + g * 8 + (tq & 1) * 4 : 96 + g * 4;
            sdst[v] = n * BROW + pos;                     // bf16 index within a plane
        } else {
            sdst[v] = i < FBLK4 ? -1 - 4 * (i - FW * FW / 4) : INT32_MIN;   // bias float index, encoded
        }
    }
    f32x4 pf[FSLOTS];
#define VIHMC_FB_LOAD(J)                                                                              \
    {                                                                                                 \
        const f32x4* src = reinterpret_cast<const f32x4*>(Wc + N.w_off[J]);                           \
        _Pragma("unroll") for (int v = 0; v < FSLOTS; ++v)                                            \
            pf[v] = src[min(tid + FTHREADS * v, FBLK4 - 1)];                                          \
    }
#define VIHMC_FB_STORE(BUF)                                                                           \
    _Pragma("unroll") for (int v = 0; v < FSLOTS; ++v) {                                              \
        unsigned char* bb = fsmb + (BUF) * BBUF;                                                      \
        if (sdst[v] >= 0) {                                                                           \
            bf16x4 a, b, cc;                                                                          \
            _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                           \
                __bf16 x0, x1, x2;                                                                    \
                split3(pf[v][j], x0, x1, x2);                                                         \
                a[j] = x0; b[j] = x1; cc[j] = x2;                                                     \
            }                                                                                         \
            __bf16* pl = reinterpret_cast<__bf16*>(bb) + sdst[v];                                     \
            *reinterpret_cast<bf16x4*>(pl) = a;                                                       \
            *reinterpret_cast<bf16x4*>(pl + BPLANE) = b;                                              \
            *reinterpret_cast<bf16x4*>(pl + 2 * BPLANE) = cc;                                         \
        } else if (sdst[v] != INT32_MIN) {                                                            \
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(bb + 3 * BPLANE * 2) + (-1 - sdst[v])) = pf[v]; \
        }                                                                                             \
    }

    // pre-split weight images (k_split_wimg): layer j's image is DMA-copied into buffer j&1 one layer ahead
    // (global_load_lds, 1 KB per wave-instruction, no VGPRs / VALU); the barrier drains it (vmcnt(0))
    const bool dma = FWD_TAILF32 || FWD_DMA_ONLY || N.wimg != nullptr;  // FWD_TAILF32: images only (host-checked)
    const unsigned char* wimgc = dma ? N.wimg + c * N.wimg_cs : nullptr;
#define VIHMC_FB_DMA(J, BUF)                                                                          \
    if (ND == 0)                                                                                      \
    for (int k = wave; k < FWD_WIMG / 1024; k += NW)                                                  \
        bf6::glds16_asm(wimgc + (int64_t)(J) * FWD_WIMG + k * 1024 + lane * 16, fsmb + (BUF) * FWD_WIMG + k * 1024);
    if (dma) {
        VIHMC_FB_DMA(0, 0)
    } else {
        VIHMC_FB_LOAD(0)
    }
    float4 h[7];
    float4 xa[6];
    float xt[4];
    if (N.x != nullptr) {
        // input layer in this launch: W0 into buffer 1 (layer 1's image goes there only after the first loop barrier),
        // every piece's load issued before the stores; the row's x operand prefetched
        const int q4 = ((N.k0 + 3) & ~3) >> 2, n4 = FW * q4, ldw = in0_ldw(4 * q4);
        const float* W0 = Wc + N.w0_off;
        float* w0s = reinterpret_cast<float*>(fsmb + FWD_WIMG);
        constexpr int SP = (FW * ((IN0_KMAX + 3) / 4) + FTHREADS - 1) / FTHREADS;
        f32x4 wv[SP];
#pragma unroll
        for (int u = 0; u < SP; ++u) {
            const int i = min(tid + FTHREADS * u, n4 - 1);        // clamped slots rewrite the last piece (same value)
            const int r = i / q4, c4 = i - r * q4;
            wv[u] = *reinterpret_cast<const f32x4*>(W0 + (int64_t)r * N.ldw0 + 4 * c4);
        }
        in0_load_x(N, rowc, lg, xa, xt);
#pragma unroll
        for (int u = 0; u < SP; ++u) {
            const int i = min(tid + FTHREADS * u, n4 - 1);
            const int r = i / q4, c4 = i - r * q4;
            *reinterpret_cast<f32x4*>(w0s + r * ldw + 4 * c4) = wv[u];
        }
    } else {
        const float* ar = N.in + c * N.in_cs + (int64_t)rowc * N.ldin;
#pragma unroll
        for (int t = 0; t < 6; ++t) h[t] = *reinterpret_cast<const float4*>(ar + 16 * t + 4 * lg);
        if (FWD_TAILF32) h[6] = float4{ar[96 + lg], 0.f, 0.f, 0.f};
        else h[6] = lg == 0 ? *reinterpret_cast<const float4*>(ar + 96) : float4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();                            // zero fill done before the staging writes (and W0 staged)
    if (!dma) {
        VIHMC_FB_STORE(0)
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);         // see k_fwd_fused: no vmcnt waits inside the layer loop
    if (N.x != nullptr) {
        float* h0 = const_cast<float*>(N.in) + c * N.in_cs;
        const __amdgpu_buffer_rsrc_t hrs = make_rsrc(h0, (uint32_t)N.rows * (uint32_t)N.ldin * 4u);
        in0_layer(N, reinterpret_cast<const float*>(fsmb + FWD_WIMG), Wc + N.b0_off, xa, xt, lr, lg, hrs,
                  rok ? (uint32_t)row * (uint32_t)N.ldin * 4u : OOB, h);
    }
    const float* outc = N.out + c * N.out_cs;
    const uint32_t ooff = rok ? (uint32_t)row * (uint32_t)N.ldo * 4u : OOB;
    const uint32_t obytes = (uint32_t)N.rows * (uint32_t)N.ldo * 4u;
    for (int j = 0; j < N.nl; ++j) {
        __syncthreads();
        FW_ST(j, 0)
        if (dma) {
            if (j + 1 < N.nl) {
                VIHMC_FB_DMA(j + 1, (j + 1) & 1)
            }
        } else {
            VIHMC_FB_LOAD(min(j + 1, N.nl - 1))
        }
        const unsigned char* bbuf = fsmb + (j & 1) * (dma ? FWD_WIMG : BBUF);
        const __bf16* wb = reinterpret_cast<const __bf16*>(bbuf);
        const float* bias = reinterpret_cast<const float*>(bbuf + 3 * BPLANE * 2);
        const __amdgpu_buffer_rsrc_t orsrc = make_rsrc(outc + N.h_off[j], obytes);
        const uint32_t hoffj = (N.skip_last && j == N.nl - 1) ? OOB : ooff;   // stores issued, dropped (vmcnt count)
        bf16x8 hp[3][3];
        const int act = N.act[j];
        if (FWD_TAILF32) {
            bf16x4 h6u[3];
            bf_split_operand(h, hp, h6u);          // tile 6 planes unused (the f32 MFMA takes h[6].x)
#if FWD_STAMP
            __builtin_amdgcn_sched_barrier(0);
#endif
            FW_ST(j, 1)
            const float* wtail = reinterpret_cast<const float*>(bbuf + FWD_WTAIL);
            const float h6f = h[6].x;
            if (act == ACT_TANH) tf_layer<ACT_TANH>(wb, bias, wtail, hp, h6f, lr, lg, orsrc, hoffj, h);
            else if (act == ACT_TANH_CR) tf_layer<ACT_TANH_CR>(wb, bias, wtail, hp, h6f, lr, lg, orsrc, hoffj, h);
            else if (act == ACT_RELU) tf_layer<ACT_RELU>(wb, bias, wtail, hp, h6f, lr, lg, orsrc, hoffj, h);
            else tf_layer<ACT_ID>(wb, bias, wtail, hp, h6f, lr, lg, orsrc, hoffj, h);
#if FWD_STAMP
            __builtin_amdgcn_sched_barrier(0);
#endif
            FW_ST(j, 2)
        } else {
            bf16x4 h6[3];
            bf_split_operand(h, hp, h6);
            if (act == ACT_TANH) bf_layer<ACT_TANH>(wb, bias, hp, h6, lr, lg, orsrc, hoffj, h);
            else if (act == ACT_TANH_CR) bf_layer<ACT_TANH_CR>(wb, bias, hp, h6, lr, lg, orsrc, hoffj, h);
            else if (act == ACT_RELU) bf_layer<ACT_RELU>(wb, bias, hp, h6, lr, lg, orsrc, hoffj, h);
            else bf_layer<ACT_ID>(wb, bias, hp, h6, lr, lg, orsrc, hoffj, h);
        }
        if (!dma) {
            VIHMC_FB_STORE((j + 1) & 1)
        }
        // layer j+1's image landed before the next barrier. The DMA was issued ahead of this layer's seven h stores
        // (six b128 + the tile-6 b32), so a counted wait leaves those stores in flight (vmcnt(0) waited for them)
        if (dma) {
            if (FWD_TAILF32) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else bf6::wait_vmcnt0();
        }
        FW_ST(j, 3)
    }
#if FWD_STAMP
    if (fw_samp && tid == 0) {
        fw_real[fw_sidx][1][0] = __builtin_amdgcn_s_memtime();
        fw_real[fw_sidx][1][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    // the output layer's rows as the contraction's pre-split image (bit-identical to k_split_blocks on the fp32
    // rows just stored: same conversions), which saves that kernel's re-read of the outputs and its launch
    if (N.qimg != nullptr) {
        auto split_tile = [&](int t, bf16x4& a, bf16x4& b, bf16x4& cc) __attribute__((always_inline)) {
            const float v[4] = {h[t].x, h[t].y, h[t].z, h[t].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                __bf16 x0, x1, x2;
                split3(v[e], x0, x1, x2);
                a[e] = x0;
                b[e] = x1;
                cc[e] = x2;
            }
        };
        __bf16 y0, y1, y2;
        split3(h[6].x, y0, y1, y2);                       // column 96 + lg: its planes and the fp32 tail
        unsigned char* blk = N.qimg + c * N.qimg_cs + (int64_t)(min(row, N.rows - 1) / CONTRACT_SPLIT_ROWS) *
                                                          CONTRACT_SPLIT_BLOCK;
        // through LDS (the weight buffers are free after the last layer): each wave lays its 16 rows out as in
        // the image -- three 16-row plane slices and the tail slice, 11,008 B -- then copies them out in whole
        // 1-KB wave stores (direct 8-B stores per lane and tile measured slower)
        __syncthreads();
        unsigned char* reg = fsmb + wave * QI_WAVE;
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            bf16x4 a, b, cc;
            split_tile(t, a, b, cc);
            unsigned char* o = reg + lr * QI_PITCH + 2 * (16 * t + 4 * lg);
            *reinterpret_cast<bf16x4*>(o) = a;
            *reinterpret_cast<bf16x4*>(o + QI_HALF) = b;
            *reinterpret_cast<bf16x4*>(o + 2 * QI_HALF) = cc;
        }
        {
            unsigned char* o = reg + lr * QI_PITCH + 2 * (96 + lg);
            *reinterpret_cast<__bf16*>(o) = y0;
            *reinterpret_cast<__bf16*>(o + QI_HALF) = y1;
            *reinterpret_cast<__bf16*>(o + 2 * QI_HALF) = y2;
            if (lg < 3) {                                  // columns 100..111 of plane lg (8-B aligned): zero, but
                uint64_t* z = reinterpret_cast<uint64_t*>(reg + lg * QI_HALF + lr * QI_PITCH + 200);
                uint64_t f100 = 0;                         // column 100 = plane lg of the augmentation value
                if (N.aug) {
                    const float av = N.aug == 1 ? 1.f : args.packed[c * args.dp];
                    __bf16 a0, a1, a2;
                    split3(av, a0, a1, a2);
                    const __bf16 al = lg == 0 ? a0 : (lg == 1 ? a1 : a2);
                    f100 = (uint64_t)__builtin_bit_cast(uint16_t, al);
                    // trunk: column 101 = 1 (planes 1, 0, 0), so the Gram-t tiles carry the column sums sum_p Zt^[p][v]
                    // in fp64 (Gt[v][101]) for the exact d ll / d b0 (vihmc_gram.hip gram_tt_epilogue)
                    if (N.aug == 2 && lg == 0) f100 |= (uint64_t)0x3F80u << 16;
                }
                z[0] = f100;
                z[1] = 0;
                z[2] = 0;
            }
            reinterpret_cast<float*>(reg + 3 * QI_HALF + lr * 16)[lg] = h[6].x;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);               // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();
        const int row0 = row - lr;                         // the wave's first row (16-row aligned)
        const int hb = (row0 % CONTRACT_SPLIT_ROWS) / 16;  // which half of the 32-row block
#pragma unroll
        for (int k = 0; k < (QI_WAVE / 16 + 63) / 64; ++k) {
            const int i = k * 64 + lane;                   // 16-B piece of the wave's region
            if (i >= QI_WAVE / 16) break;
            int r, off;
            if (i < 3 * QI_HALF / 16) {
                const int pl = i / (QI_HALF / 16), w16 = i % (QI_HALF / 16);
                r = w16 / (QI_PITCH / 16);
                off = pl * QI_PLANE + hb * QI_HALF + w16 * 16;
            } else {
                r = i - 3 * QI_HALF / 16;
                off = 3 * QI_PLANE + (hb * 16 + r) * 16;
            }
            if (row0 + r < N.rows)
                *reinterpret_cast<u32x4*>(blk + off) = *reinterpret_cast<const u32x4*>(reg + i * 16);
        }
    }
#undef VIHMC_FB_LOAD
#undef VIHMC_FB_STORE
#undef VIHMC_FB_DMA
}

// [W_j | bias_j] of every fused layer of every chain -> the LDS image k_fwd_fused_bf stages (same permuted
// column order as VIHMC_FB_STORE, zero padding, bias fp32 [112]); one block per (chain, net, layer)
__global__ __launch_bounds__(1024) void k_split_wimg(FusedArgs args) {
    const int C = args.C;
    int b = blockIdx.x;
    const int c = b % C;
    b /= C;
    const int net = b < args.net[0].nl ? 0 : 1;
    const int j = net ? b - args.net[0].nl : b;
    const FusedNet& N = args.net[net];
    const float* src = args.packed + c * args.dp + N.w_off[j];
    unsigned char* img = const_cast<unsigned char*>(N.wimg) + c * N.wimg_cs + (int64_t)j * FWD_WIMG;
    __bf16* pl = reinterpret_cast<__bf16*>(img);
    for (int i = threadIdx.x; i < FW * 112 / 4; i += 1024) {          // plane positions, 4 at a time
        const int n = i / 28, q = i % 28;                            // row n, positions 4q..4q+3
        const int pos = 4 * q;
        // inverse of VIHMC_FB_STORE's map: position -> source column
        int col;
        if (pos < 96) {
            const int kb = pos >> 5, g = (pos & 31) >> 3, hi = (pos >> 2) & 1;
            col = 16 * (2 * kb + hi) + 4 * g;
        } else {
            col = pos;                                               // 96..99 real, 100..111 zero
        }
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (col < FW) x = *reinterpret_cast<const f32x4*>(src + n * FW + col);
        bf16x4 a, bb, cc;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            __bf16 x0, x1, x2;
            split3(x[e], x0, x1, x2);
            a[e] = x0;
            bb[e] = x1;
            cc[e] = x2;
        }
        *reinterpret_cast<bf16x4*>(pl + n * BROW + pos) = a;
        *reinterpret_cast<bf16x4*>(pl + BPLANE + n * BROW + pos) = bb;
        *reinterpret_cast<bf16x4*>(pl + 2 * BPLANE + n * BROW + pos) = cc;
    }
    float* bias = reinterpret_cast<float*>(img + 3 * BPLANE * 2);
    for (int i = threadIdx.x; i < 112; i += 1024) bias[i] = i < FW ? src[FW * FW + i] : 0.f;
    // fp32 k tail W[n][96..99] (FWD_TAILF32), then zeros to the end of the image
    float* wtail = reinterpret_cast<float*>(img + FWD_WTAIL);
    for (int i = threadIdx.x; i < FW * 4; i += 1024) wtail[i] = src[(i >> 2) * FW + 96 + (i & 3)];
    for (int i = FWD_WTAIL + FW * 16 + threadIdx.x * 4; i < FWD_WIMG; i += 1024 * 4)
        *reinterpret_cast<float*>(img + i) = 0.f;
}

hipError_t launch_split_wimg(const FusedArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_split_wimg, dim3(a.C * (a.net[0].nl + a.net[1].nl)), dim3(1024), 0, s, a);
    return hipGetLastError();
}

int fwd_img_plane_off(int n, int col) {
    // inverse of k_split_wimg's position -> column map (VIHMC_FB_STORE's permuted column order)
    const int t = col >> 4, g = (col >> 2) & 3, e = col & 3;
    const int pos = t < 6 ? (t >> 1) * 32 + g * 8 + (t & 1) * 4 + e : 96 + g * 4 + e;
    return 2 * (n * BROW + pos);
}
int fwd_img_plane_stride() { return 2 * BPLANE; }
int fwd_img_bias_off(int n) { return 3 * BPLANE * 2 + 4 * n; }
int fwd_img_tail_off(int n, int col) { return FWD_WTAIL + 4 * (n * 4 + (col - 96)); }

size_t fwd_fused_bf_lds_bytes() { return 2 * (size_t)FWD_WIMG; }
static_assert(BBUF <= FWD_WIMG && FWD_WTAIL + FW * 16 <= FWD_WIMG && FWD_WIMG % 1024 == 0 &&
              2 * FWD_WIMG <= 160 * 1024, "weight image");
bool fwd_fused_bf_needs_wimg() { return FWD_TAILF32 != 0; }

// an input layer [100][n_in] (x row stride ldx, W0 row stride ldw) the bf16x6 forward can run in its launch (the
// pre-split-image form: FWD_TAILF32; W0 staged in one image buffer; its tanh the row-dot epilogue's)
bool fwd_fused_in0_ok(int n_in, int ldx, int ldw) {
    const int k4 = (n_in + 3) & ~3;
    return FWD_TAILF32 && FWD_ABL == 0 && n_in >= 1 && n_in <= IN0_KMAX && ldx >= k4 &&
           (n_in < 16 || (ldx & 3) == 0) && ldw >= k4 && (ldw & 3) == 0 &&
           (size_t)FW * in0_ldw(k4) * sizeof(float) <= (size_t)FWD_WIMG;
}

#if FWD_STAMP
extern "C" int vihmc_debug_fwd_stamps(void* stamps, size_t stamp_bytes, void* real, size_t real_bytes) {
    if (stamp_bytes != sizeof(fw_stamps) || real_bytes != sizeof(fw_real)) return -1;
    hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(fw_stamps), stamp_bytes, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(real, HIP_SYMBOL(fw_real), real_bytes, 0, hipMemcpyDeviceToHost);
    return (int)e;
}
#endif
int fwd_fused_bf_waves() { return FWD_BF_NW; }

hipError_t launch_fwd_fused_bf(const FusedArgs& a, int nw, hipStream_t s) {
    dim3 g(a.C * (a.net[0].nblk + a.net[1].nblk));
    // 4 waves (64 rows per workgroup) for chain counts whose 12-wave grid would leave most CUs idle (single chain:
    // 176 workgroups instead of 60)
    if (nw == 4 && FWD_TAILF32 && a.net[0].wimg && a.net[1].wimg)
        hipLaunchKernelGGL((k_fwd_fused_bf<4, 4>), g, dim3(8 * 64), fwd_fused_bf_lds_bytes(), s, a);
    else if (nw == 4) hipLaunchKernelGGL(k_fwd_fused_bf<4>, g, dim3(4 * 64), fwd_fused_bf_lds_bytes(), s, a);
    else hipLaunchKernelGGL(k_fwd_fused_bf<FWD_BF_NW>, g, dim3(FWD_BF_NW * 64), fwd_fused_bf_lds_bytes(), s, a);
    return hipGetLastError();
}

size_t fwd_fused_lds_bytes() { return sizeof(float) * 2 * FBUF; }

hipError_t launch_fwd_fused(const FusedArgs& a, int nwaves, hipStream_t s) {
    dim3 g(a.C * (a.net[0].nblk + a.net[1].nblk));
    if (nwaves == 12) hipLaunchKernelGGL(k_fwd_fused<12>, g, dim3(12 * 64), fwd_fused_lds_bytes(), s, a);
    else if (nwaves == 4) hipLaunchKernelGGL(k_fwd_fused<4>, g, dim3(4 * 64), fwd_fused_lds_bytes(), s, a);
    else if (nwaves == 16) hipLaunchKernelGGL(k_fwd_fused<16>, g, dim3(16 * 64), fwd_fused_lds_bytes(), s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}


}  // namespace vihmc
