// Every compile-time switch of the srmi kernels, in one place.  The values below are
// the production build (the measured winners, DESIGN.md sections 3-4); a variant build
// for an A/B overrides one with -DNAME=value (tools/build_variant.sh) and never ships.
// Run-time choices (A/B and tests) are the srmi_model_config.flags bits, include/srmi.h.
#pragma once

// Write-through (sc1) stores for the large outputs (common.hpp st_wt*): the kernel
// boundary then finds no dirty lines to flush (the slabs alone: +1.1 % in the step).
#ifndef SRMI_TRAIN_WT
#define SRMI_TRAIN_WT 1
#endif
// the one-launch inference RCAB (rcab_infer.hip): write-back stores -- t is re-read by
// the workgroup that wrote it and the pair by the next launch (+1 % C5 over write-through)
#ifndef SRMI_INFER_WT
#define SRMI_INFER_WT 0
#endif

// Deferred conv epilogues (conv64_body.hpp conv64_defers), a bit mask: 1 RELU, 2 POOL,
// 4 DG_RELUMASK, 8 DG_ACC_CA, 16 RELU_POOL, 32 CA_RESID, 64 DG_ACC_CA16; 128: DG_ACC_CA16 in the
// deferred body's register-direct form but right after its own strip (no LDS staging, one
// barrier per strip).  Training: DG_RELUMASK and 128 (F1: +0.3 / +0.4 / +0.9 % on three boxes,
// profiles/r06_ab_f1_epilogue_forms.txt, r06_ab_f1_imm_final.txt) gain in the step; 64 lost;
// inference (an image is one run of 12 strips): conv1's RELU_POOL
// (CA_RESID deferred measured 5 % slower: its pair codec competes with the next strip's
// MFMA issue).
#ifndef SRMI_TRAIN_DEFER
#define SRMI_TRAIN_DEFER 132
#endif
#ifndef SRMI_INFER_DEFER
#define SRMI_INFER_DEFER 16
#endif

// F1 (EPI_DG_ACC_CA16) in the deferred body (SRMI_TRAIN_DEFER bit 64 or 128): dgrad strips per
// run handed to the paired filter-gradient workgroup (1, as the staged form's)
#ifndef SRMI_F1_DEFER_TAIL
#define SRMI_F1_DEFER_TAIL 1
#endif

// du formed from g in the fused conv2 backward (ConvParams / WgradParams gx): where the
// dgrad forms it on group k+2's ring pieces -- 2 = one piece every other K-step from K-step
// 18 - 2 x pieces, each read the K-step before (profiles/r06_ab_gx_spread.txt: +0.2-0.4 %),
// 1 = one piece per K-step over the last K-steps, 0 = after the strip's wait for the pieces,
// before the barrier that publishes them; the filter gradient forms a pair's dY rows behind
// the MFMAs of the pair before's first K-step (1, 2) or before its barrier (0)
#ifndef SRMI_GX_INLOOP
#define SRMI_GX_INLOOP 2
#endif

// the CALayer backward with du formed in the fused conv2 backward: its MLP in that launch's
// prologue (every workgroup, 1; the filter-gradient reductions then wait for the group's end)
// or in a small launch of its own before it (0; the reductions ride in it)
#ifndef SRMI_F2_MLP
#define SRMI_F2_MLP 1
#endif

// the inference conv2's h' = h + s u with u rounded to bf16 (as the training conv2 and
// the round-3 three-launch inference did; staged once as bf16, one barrier), 0 = fp32 u
// (staged as fp32 in two halves, four barriers)
#ifndef SRMI_INFER_BF16U
#define SRMI_INFER_BF16U 1
#endif

// rcab_infer.hip defines SRMI_TU_INFER before its includes: the inference policies
#ifdef SRMI_TU_INFER
#define SRMI_WT SRMI_INFER_WT
#define SRMI_DEFER SRMI_INFER_DEFER
#else
#define SRMI_WT SRMI_TRAIN_WT
#define SRMI_DEFER SRMI_TRAIN_DEFER
#endif

// Training CA forward (engine.cpp ca_fwd_mode): 1 = inside conv2's launch (the scale in
// every conv2 workgroup, after its first strip's MFMAs), 0 = the CA pass of its own.
#ifndef SRMI_CA_FWD
#define SRMI_CA_FWD 1
#endif

// the training CA mean from conv1's partial means (ca_scale.hpp ca_matvec in conv1's run
// end, conv2 sums them: 1) or conv2 computing it from t's border lines (0)
#ifndef SRMI_CA_MPART
#define SRMI_CA_MPART 1
#endif

// the fused backward's tail strips (wgrad3x3.hip rcab_bwd_kernel): run by the paired
// filter-gradient workgroup after its chunk (0) or before it (1: +0.2-0.4 % in the step,
// profiles/r05_ab_tail_first.txt; the chunk's slab stores no longer meet the dgrad runs' loads)
#ifndef SRMI_FUSE_TAIL_FIRST
#define SRMI_FUSE_TAIL_FIRST 1
#endif

// the RCAB filter gradients' partial slabs (the fused backward's wgrad48 body) stored as
// bf16 and summed in fp32 by the reduction (1), or fp32 (0): half the slab bytes
#ifndef SRMI_SLAB16
#define SRMI_SLAB16 1
#endif

// waves per workgroup of the exact-fp32 conv (conv_f32.hip)
#ifndef SRMI_F32_NW
#define SRMI_F32_NW 8
#endif

// workgroups of the tail conv's forward (small.hip tail_fwd_launch)
#ifndef SRMI_TAIL_FWD_BLOCKS
#define SRMI_TAIL_FWD_BLOCKS 512
#endif

// 8-channel groups per thread of the CA elementwise passes (small.hip): 4 amortises the
// per-block MLP over twice the data of 2 (ca_fwd 22.6 -> 20.0 us, ca_bwd 15.1 -> 13.7 us)
#ifndef SRMI_CA_VEC
#define SRMI_CA_VEC 4
#endif

// SRMI_STAMPS (undefined in production): s_memtime stamps per workgroup phase into
// ConvParams / WgradParams .stamps (srmi_debug_conv_stamps, tools/stamps_run.sh)
