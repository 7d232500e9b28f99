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

__device__ __forceinline__ float tanh_f(float x) {
    const float ax = fabsf(x);
    const float x2 = x * x;
    float p = fmaf(x2, -0.0088632355f, 0.0218694885f);
    p = fmaf(x2, p, -0.0539682540f);
    p = fmaf(x2, p, 0.1333333333f);
    p = fmaf(x2, p, -0.3333333333f);
    const float small = fmaf(x * x2, p, x);
    const float e = __expf(2.f * ax);
    const float big = copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f), x);
    return ax < 0.25f ? small : big;
}

template <int ACT>
__device__ __forceinline__ float act_t(float z) {
    if constexpr (ACT == ACT_TANH) return tanh_f(z);
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
