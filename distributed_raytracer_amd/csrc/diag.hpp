// diag.hpp — build-time switches of kernels.hip, in one place.
//
// The product build (the Makefile, no -D flags) uses the defaults below.  Everything else is
// a measurement or ablation build made with EXTRA=-D... (tools/variants.sh, tools/ab_lib.sh,
// tools/diag_stages.py, tools/item_trace.py): those builds change what the kernels compute
// or record, never the default library.  Run-time variants are MIRT_OPT_* (mirt.h) instead.
#pragma once

// ---- diagnostics: record, never change results
// MIRT_DIAG: wave-level event counts per stage of the triangle test (kernels.hip diag(),
// read with mirt_debug_counters).
#ifndef MIRT_DIAG
#define MIRT_DIAG 0
#endif
// MIRT_PHASE_TIMING: shader-clock cycles per phase of the primary blocks in the timeline.
#ifndef MIRT_PHASE_TIMING
#define MIRT_PHASE_TIMING 0
#endif
// MIRT_ITEM_TRACE: one timeline record per work item (with MIRT_OPT_TIMELINE).
#ifndef MIRT_ITEM_TRACE
#define MIRT_ITEM_TRACE 0
#endif

// ---- measurement builds: each removes one phase of the frame; results WRONG
#ifndef MIRT_EXP_NO_PRIMARY_TRACE  // every traced primary ray misses
#define MIRT_EXP_NO_PRIMARY_TRACE 0
#endif
#ifndef MIRT_EXP_NO_TRI_TESTS  // leaves are entered but never tested
#define MIRT_EXP_NO_TRI_TESTS 0
#endif
#ifndef MIRT_EXP_NO_SHADOW_TESTS  // shadow leaves entered, never tested (all lit)
#define MIRT_EXP_NO_SHADOW_TESTS 0
#endif
#ifndef MIRT_EXP_NO_PHONG  // ambient colour only
#define MIRT_EXP_NO_PHONG 0
#endif
#ifndef MIRT_EXP_NO_SHADOW_TRACE  // every light reaches every hit
#define MIRT_EXP_NO_SHADOW_TRACE 0
#endif
#ifndef MIRT_SKIP_MISS_STORES  // miss outputs left unwritten
#define MIRT_SKIP_MISS_STORES 0
#endif

// ---- ablations: same results, other shapes (DESIGN.md §4.8 measured each)
// Occupancy target of the tracing kernels (waves per SIMD; 4 = 128 VGPRs).
#ifndef MIRT_WAVES_PER_EU
#define MIRT_WAVES_PER_EU 4
#endif
// k_shadow's occupancy (the split kernels' shadow items: reflection levels, configs[4]).
#ifndef MIRT_SHADOW_WAVES_PER_EU
#define MIRT_SHADOW_WAVES_PER_EU MIRT_WAVES_PER_EU
#endif
// k_reflect's occupancy (chains option; 2 waves: no spill but 30% slower).
#ifndef MIRT_REFLECT_WAVES_PER_EU
#define MIRT_REFLECT_WAVES_PER_EU 4
#endif
// Meshes up to kLdsTris faces staged whole in LDS (0: read from HBM with scalar loads).
#ifndef MIRT_LDS_MESH
#define MIRT_LDS_MESH 1
#endif
// Whole-block frustum pre-test of primary blocks (one-object frames).
#ifndef MIRT_BLOCK_FRUSTUM
#define MIRT_BLOCK_FRUSTUM 1
#endif
// Traversal per query: 1 = wide cone traversal (shared-origin packets), 0 = the 8-child
// sweep with scalar node loads (faster on suzanne for both, profiles/r01_*).
#ifndef MIRT_PRIMARY_WIDE
#define MIRT_PRIMARY_WIDE 0
#endif
#ifndef MIRT_SHADOW_WIDE
#define MIRT_SHADOW_WIDE 0
#endif
// Wide traversal: leaves tested per lane before the wave tests them (1) or wave-wide (0).
#ifndef MIRT_LEAF_LANE_TEST
#define MIRT_LEAF_LANE_TEST 1
#endif
// Bounce waves: k_bounce also traces each level's shadow rays and phong (1: slower), or
// leaves them to k_shadow on the packed records (0).
#ifndef MIRT_BOUNCE_SHADE
#define MIRT_BOUNCE_SHADE 0
#endif
// k_shadow: a three-face leaf's light-table records loaded at once (1) or two per step (0,
// fewer spilled VGPRs there; k_trace always loads three).
#ifndef MIRT_SHADOW_LT3
#define MIRT_SHADOW_LT3 0
#endif
// The reference's face/object Box.Intersect gate compiled in (1) or out (0:
// brute-force semantics, as MIRT_OPT_NO_BOX_GATE at run time; measures the gate's cost; 2: the
// gates evaluated but a failure only counted (overflow statistic), no second pass; 3: every box
// passes without a test, the rest kept; 4: no NaN tracking in Best: measurement builds).
#ifndef MIRT_BOX_GATE
#define MIRT_BOX_GATE 1
#endif
// One-object frames of an HBM mesh (beyond the LDS) run k_trace instantiations that take the
// object count and the segment shadow mode as constants (1), or the generic HBM kernel (0:
// measurement builds).  MIRT_OPT_LDS_STREAM selects the one that streams the triangles through
// LDS; MIRT_STREAM_SHADOW: its shadow segments stream too (1) or read HBM (0: the default —
// at configs[3] streaming the shadow sweeps cost 11% (15 VGPR spills), primary-only
// streaming ties the HBM kernel: DESIGN.md §4.6).
#ifndef MIRT_HBM1
#define MIRT_HBM1 1
#endif
#ifndef MIRT_STREAM_SHADOW
#define MIRT_STREAM_SHADOW 0
#endif
