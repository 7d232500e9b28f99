// bf16x6: fp32 products on the bf16 MFMA (shared by the bf16x6 contraction and layer-backward kernels).
//
// Every fp32 operand x is split exactly into three bf16 planes x = x0 + x1 + x2 (x0 = bf16(x),
// x1 = bf16(x - x0), x2 = bf16(x - x0 - x1); the last conversion is exact). a.b keeps the six products of
// order <= 2 (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0, small first) accumulated in fp32 by the MFMA: the
// dropped terms are < 2^-24 |a||b|, so a dot product is as accurate as the sequential fp32 one
// (profiles/bf16x6_precision.py). Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight
// v_mfma_f32_16x16x4f32 (32 cycles each) per 32-long k-block: 2.7x fewer matrix-core cycles.
//
// Operand maps (16x16x32 bf16): lane l holds A[l & 15][8(l >> 4) + j] and B[8(l >> 4) + j][l & 15],
// j = 0..7; accumulator lane l holds D[4(l >> 4) + r][l & 15], r = 0..3. Any k permutation shared by A
// and B is allowed; the kernels use "rows 4lg .. 4lg+3 and 16 + 4lg .. +3" of a 32-row block, which is
// both the accumulator layout of two 16-row tiles and what two ds_read_b64_tr_b16 of a row-major
// [rows][224 B] plane deliver.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace vihmc {
namespace bf6 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int PITCH = 224;                 // bytes per bf16 plane row (112 features): 7 x 32 B, odd
constexpr uint32_t OOB = 0x80000000u;      // buffer offset the range check always drops

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// exact three-way split of 4 values into bf16 planes
__device__ __forceinline__ void split4(f32x4 x, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        p0[j] = a;
        p1[j] = b;
        p2[j] = (__bf16)(r - (float)b);
    }
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// acc += a.b over one 32-long k-block, six products, small terms first
__device__ __forceinline__ f32x4 six(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 acc) {
    acc = mfma_bf(a[2], b[0], acc);
    acc = mfma_bf(a[1], b[1], acc);
    acc = mfma_bf(a[0], b[2], acc);
    acc = mfma_bf(a[1], b[0], acc);
    acc = mfma_bf(a[0], b[1], acc);
    acc = mfma_bf(a[0], b[0], acc);
    return acc;
}

// the 8-row k fragment of a 32-row block of a row-major [rows][PITCH] plane, columns col0 .. col0+15,
// as the B (or A) operand: rows 4lg .. 4lg+3 and 16 + 4lg .. +3 (two transposed reads)
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* plane, int tr_off, int col0) {
    const unsigned char* a = plane + tr_off + 2 * col0;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 16 * PITCH));
    return cat8(lo, hi);
}
// per-lane byte offset for tr_frag: lane 4qq + pp of group lg supplies row 4lg + qq, columns +4pp
__device__ __forceinline__ int tr_lane_off(int lr, int lg) { return (4 * lg + (lr >> 2)) * PITCH + 8 * (lr & 3); }

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4: lane l's bytes land at lds_dst + 16 l) issued from inline
// asm, so hipcc does not put it in its vmcnt bookkeeping: with the builtin form, hipcc waits vmcnt(0) before
// the next LDS read of ANY buffer (it cannot prove the DMA target disjoint) -- which serialised the DMA
// latency into every chunk. The issuing wave must wait for completion itself (s_waitcnt vmcnt(0)) before the
// barrier that publishes the buffer. M0 is written and restored in the same statement.
__device__ __forceinline__ void glds16_asm(const void* gsrc, const void* lds_generic) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_generic);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// vmcnt(0) twice: through the builtin, so hipcc's waitcnt bookkeeping sees every earlier load retired (its
// counted waits after this point do not wait on loads issued before it), and as asm volatile, which hipcc
// cannot drop or merge -- the asm DMA it guards is invisible to its bookkeeping
__device__ __forceinline__ void wait_vmcnt0() {
    __builtin_amdgcn_s_waitcnt(0x0F70);                 // vmcnt(0) expcnt(7) lgkmcnt(15)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// buffer resource over [p, p + bytes) from wave-uniform inputs (out-of-range loads read 0, stores drop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

}  // namespace bf6
}  // namespace vihmc
