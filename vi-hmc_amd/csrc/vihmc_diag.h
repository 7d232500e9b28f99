// Compile-time configuration of the kernels, in one place.
//
// 1. Instrumentation: ONE enable macro, VIHMC_DIAG (default 0 = the product build). A variant build sets it on the
//    hipcc line (make -C vi-hmc_amd OUT=$PWD/_ab/<v>.so BUILD=$PWD/build/<v> EXTRA=-DVIHMC_DIAG=<value>); its fields
//    select in-kernel phase stamps (s_memtime per phase into a __device__ array of their own, read back by
//    profiles/scripts/diag/stamps_*.py) and timing-only ablations (wrong results by design). vihmc_version() reports
//    the value ("diag=<n>"); plan creation and vihmc._lib refuse a library with VIHMC_DIAG != 0 unless
//    VIHMC_ALLOW_DIAG=1 (the A/B timing scripts only).
//
//    field (bits)         name            meaning
//    0-3                  FWD_ABL         bf16x6 forward ablations: 1 = no h stores, 2 = tanh -> identity,
//                                         4 = the DMA waves issue no weight-image copies, 8 = no bf16 MFMAs
//    4                    FWD_STAMP       per-layer phase stamps of k_fwd_fused_bf (stamps_fwd.py)
//    5                    BB_STAMP        per-sub-tile stamps of k_bwd_bf2 (stamps_bwd.py)
//    6                    CH_STAMP        per-layer stamps of k_bwd_chain (stamps_chain.py)
//    7-8                  CB_STAMP        side-A contraction stamps, two placements 1 / 2 (stamps_side_a.py)
//    9                    GR_STAMP        per-block stamps of k_gram_a's T_b units (stamps_gram.py)
//    10-11                GR_ABL          Gram ablations: 1 = no A loads in the main loops (block 0's), 2 = no block
//                                         DMA (the ring keeps stale data), 3 = both
//    12-13                CH_ABL          k_bwd_chain ablations: 1 = no dW MFMAs, 2 = no dX bf16 MFMAs
//    14-15                GATHER_ABL      leapfrog gather: 1 = no scatter into packed weights / images, 2 = nor theta/p
//    16                   RD_ONLY_FIRST   grouped row-dot launches run their first problem's workgroups only
//
// 2. Tuning constants of the shipped kernels (not switches: an A/B edits this header and builds into _ab/).
#pragma once

#ifndef VIHMC_DIAG
#define VIHMC_DIAG 0
#endif

#define VIHMC_DIAG_FIELD(shift, bits) ((VIHMC_DIAG >> (shift)) & ((1 << (bits)) - 1))
#define FWD_ABL VIHMC_DIAG_FIELD(0, 4)
#define FWD_STAMP VIHMC_DIAG_FIELD(4, 1)
#define BB_STAMP VIHMC_DIAG_FIELD(5, 1)
#define CH_STAMP VIHMC_DIAG_FIELD(6, 1)
#define CB_STAMP VIHMC_DIAG_FIELD(7, 2)
#define GR_STAMP VIHMC_DIAG_FIELD(9, 1)
#define GR_ABL VIHMC_DIAG_FIELD(10, 2)
#define CH_ABL VIHMC_DIAG_FIELD(12, 2)
#define GATHER_ABL VIHMC_DIAG_FIELD(14, 2)
#define RD_ONLY_FIRST VIHMC_DIAG_FIELD(16, 1)

// bf16x6 forward: the 4-wide k tail as one f32 MFMA per tile (0: six 16x16x16 bf16 MFMAs, register-staged weights)
#define FWD_TAILF32 1
// waves per workgroup of the bf16x6 forward (16 rows each): 12 = 3 per SIMD at 168 VGPRs
#define FWD_BF_NW 12
// the register-staging path compiled out with FWD_TAILF32 = 0 too (timing variants of round 2)
#define FWD_DMA_ONLY 0
// slab count from which a reduce block's four waves split the slabs (k_reduce)
#define REDUCE_GROUP_MIN 32
// gradient-gather K slices per chain at most (launch_gather_prior picks ~256 blocks over all chains)
#define GATHER_SPLIT_N 256
// the fp32-MFMA contraction (k_contract_ws + k_contract2) and fused forward forms (0: the round-1 generic kernels)
#define VIHMC_CONTRACT_WS 1
#define VIHMC_FUSED_FWD 1
// Gram form: the dZb epilogue's sums (Zb^ Gt over v, the T_b slabs) in fp64 (0: fp32 fma)
#define GRAM_DZB_FP64 1
// Gram form, centred: cost of a two-chain T_t unit (k_gram_b2) in one-chain units, for launch_gram's row-group split
#define GRAM_B2_RATIO 1.7
// centred Gram form, 8+ chains: Gram-t slabs per T_b slab (k_gram_a's Gram-t units GRAM_T_SPLIT times shorter)
#define GRAM_T_SPLIT 2
