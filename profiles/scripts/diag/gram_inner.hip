// Microbenchmark of the Gram kernels' inner block (vihmc_gram.hip mma_block): one 32-long k block of a wave's 32 x 112
// tile = 7 column tiles x 2 row tiles x six bf16 MFMAs, B fragments by ds_read_b64_tr_b16 from an LDS block image,
// the A fragment in registers. No global memory in the loop. One workgroup per CU over the whole chip.
//   v0: as shipped (B fragments of tile t + 1 read under tile t's MFMAs), 8 waves (2 per SIMD)
//   v1: B fragments read once before the loop (registers only): the MFMA issue alone
//   v2: v0 with a workgroup barrier per block (the kernels' per-block barrier)
//   v3: v0 with 4 waves (1 per SIMD)
//   v4: v0 with 12 waves (3 per SIMD)
// Prints per variant: us, the shader clock from s_memtime / s_memrealtime, and the matrix-core busy fraction
// (MFMAs x 16 cycles per SIMD over the measured cycles).
//   hipcc --offload-arch=gfx950 -O3 -o gram_inner gram_inner.hip && ./gram_inner
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int PITCH = 224, PL = 32 * PITCH, BLK = 3 * PL;
constexpr int ITERS = 2000;

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 six(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 acc) {
    acc = mfma_bf(a[2], b[0], acc);
    acc = mfma_bf(a[1], b[1], acc);
    acc = mfma_bf(a[0], b[2], acc);
    acc = mfma_bf(a[1], b[0], acc);
    acc = mfma_bf(a[0], b[1], acc);
    acc = mfma_bf(a[0], b[0], acc);
    return acc;
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* plane, int tr_off, int col0) {
    const unsigned char* a = plane + tr_off + 2 * col0;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 16 * PITCH));
    return cat8(lo, hi);
}
__device__ __forceinline__ void load_b(const unsigned char* buf, int tro, int t, bf16x8 (&b)[3]) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) b[pl] = tr_frag(buf + pl * PL, tro, 16 * t);
}

template <int V, int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_inner(const bf16x8* src, float* out, unsigned long long* clk) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[BLK];
    const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    for (int i = tid; i < BLK / 16; i += NW * 64) reinterpret_cast<bf16x8*>(lds)[i] = src[i % 4096];
    bf16x8 a[2][3];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[rt][pl] = src[(tid + 64 * (rt * 3 + pl)) % 4096];
    __syncthreads();
    const int tro = (4 * lg + (lr >> 2)) * PITCH + 8 * (lr & 3);
    f32x4 acc[2][7];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bb[7][3];
    if (V == 1) {
#pragma unroll
        for (int t = 0; t < 7; ++t) load_b(lds, tro, t, bb[t]);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
        if (V == 2) __syncthreads();
        if (V == 1) {
#pragma unroll
            for (int t = 0; t < 7; ++t)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][t] = six(a[rt], bb[t], acc[rt][t]);
            asm volatile("" ::: "memory");
        } else {
            bf16x8 b[2][3];
            load_b(lds, tro, 0, b[0]);
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                if (t < 6) load_b(lds, tro, t + 1, b[(t + 1) & 1]);
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][t] = six(a[rt], b[t & 1], acc[rt][t]);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) s += acc[rt][t][0] + acc[rt][t][1] + acc[rt][t][2] + acc[rt][t][3];
    out[blockIdx.x * NW * 64 + tid] = s;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// RT row tiles per wave (RT = 4: 64 rows, each B fragment feeds four row tiles), NWG workgroups per CU via the grid
template <int RT, int NW>
__global__ __launch_bounds__(NW * 64) void k_inner_rt(const bf16x8* src, float* out, unsigned long long* clk) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[BLK];
    const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    for (int i = tid; i < BLK / 16; i += NW * 64) reinterpret_cast<bf16x8*>(lds)[i] = src[i % 4096];
    bf16x8 a[RT][3];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[rt][pl] = src[(tid + 64 * (rt * 3 + pl)) % 4096];
    __syncthreads();
    const int tro = (4 * lg + (lr >> 2)) * PITCH + 8 * (lr & 3);
    f32x4 acc[RT][7];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS * 2 / RT; ++it) {
        bf16x8 b[2][3];
        load_b(lds, tro, 0, b[0]);
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            if (t < 6) load_b(lds, tro, t + 1, b[(t + 1) & 1]);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt][t] = six(a[rt], b[t & 1], acc[rt][t]);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < 7; ++t) s += acc[rt][t][0] + acc[rt][t][1] + acc[rt][t][2] + acc[rt][t][3];
    out[blockIdx.x * NW * 64 + tid] = s;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// same MFMA count per SIMD as run<0, 8>: (waves per SIMD) x (ITERS x 2 / RT blocks) x (RT x 7 x 6 MFMAs)
template <int RT, int NW>
void run_rt(const char* name, const bf16x8* src, float* out, unsigned long long* clk, int nblk, int wg_per_cu) {
    hipLaunchKernelGGL((k_inner_rt<RT, NW>), dim3(nblk), dim3(NW * 64), 0, 0, src, out, clk);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_inner_rt<RT, NW>), dim3(nblk), dim3(NW * 64), 0, 0, src, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * nblk);
    hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < nblk; ++b) cyc += h[2 * b], rt += h[2 * b + 1];
    const double mhz = cyc / rt * 100.0;
    const double mfma_per_simd = (NW / 4.0) * wg_per_cu * (ITERS * 2.0 / RT) * RT * 42.0;
    const double us_floor = mfma_per_simd * 16.0 / mhz;
    printf("%-34s %8.1f us  clock %6.0f MHz  MFMA busy (wall, at that clock) %.3f\n", name, ms * 1e3, mhz,
           us_floor / (ms * 1e3));
}

template <int V, int NW>
void run(const char* name, const bf16x8* src, float* out, unsigned long long* clk, int nblk) {
    hipLaunchKernelGGL((k_inner<V, NW>), dim3(nblk), dim3(NW * 64), 0, 0, src, out, clk);   // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_inner<V, NW>), dim3(nblk), dim3(NW * 64), 0, 0, src, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * nblk);
    hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < nblk; ++b) cyc += h[2 * b], rt += h[2 * b + 1];
    cyc /= nblk;
    rt /= nblk;
    const double mhz = cyc / rt * 100.0;
    // MFMAs per SIMD: waves per SIMD x ITERS x 84; 16 cycles each
    const double wps = NW / 4.0;
    const double busy = wps * ITERS * 84.0 * 16.0 / cyc;
    printf("%-34s %8.1f us  clock %6.0f MHz  cycles/block/wave-set %7.0f  MFMA busy %.3f\n", name, ms * 1e3, mhz,
           cyc / ITERS, busy);
}

int main() {
    int nblk = 256;
    bf16x8* src;
    float* out;
    unsigned long long* clk;
    hipMalloc(&src, 4096 * sizeof(bf16x8));
    std::vector<__bf16> hs(4096 * 8);
    for (size_t i = 0; i < hs.size(); ++i) hs[i] = (__bf16)(0.001f * (float)((i * 7919) % 1000));
    hipMemcpy(src, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&out, nblk * 12 * 64 * 4);
    hipMalloc(&clk, nblk * 2 * 8);
    run<0, 8>("v0 shipped, 8 waves", src, out, clk, nblk);
    run<1, 8>("v1 B in registers, 8 waves", src, out, clk, nblk);
    run<2, 8>("v2 + barrier per block, 8 waves", src, out, clk, nblk);
    run<0, 4>("v3 shipped, 4 waves", src, out, clk, nblk);
    run<0, 12>("v4 shipped, 12 waves", src, out, clk, nblk);
    run<1, 4>("v5 B in registers, 4 waves", src, out, clk, nblk);
    // row tiles per wave: RT = 2 (shipped, 8 waves per CU) vs RT = 4 (4-wave workgroups, two per CU: 512 blocks)
    hipFree(out);
    hipFree(clk);
    hipMalloc(&out, 2 * nblk * 12 * 64 * 4);
    hipMalloc(&clk, 2 * nblk * 2 * 8);
    run_rt<2, 8>("rt2 8 waves, 1 wg/CU", src, out, clk, nblk, 1);
    run_rt<4, 4>("rt4 4 waves, 2 wg/CU", src, out, clk, 2 * nblk, 2);
    run_rt<2, 8>("rt2 8 waves, 1 wg/CU (again)", src, out, clk, nblk, 1);
    run_rt<4, 4>("rt4 4 waves, 2 wg/CU (again)", src, out, clk, 2 * nblk, 2);
    return 0;
}
