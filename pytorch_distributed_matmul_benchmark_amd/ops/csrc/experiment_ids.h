// Experiment / diagnostic kernel ids (A/B arms and timing-only builds behind
// the profiles/ tables, docs/REPRODUCE.md). Accepted only by a library built
// with PDMB_EXPERIMENTS=1 (ops/build.py; ops/gemm.py EXPERIMENT_KERNELS); the
// dispatch for them is experiments.h.
#pragma once

namespace pdmb {

enum ExperimentKernel : int {
  kMfma256 = 1,       // SCHED 0 (ping-pong)
  kMfma256b = 3,      // SCHED 1: DMA issued in the read slot
  kMfma256c = 4,      // SCHED 2: fragment reads balanced over the read slots
  kMfma256Stamp = 5,  // SCHED 2 with in-kernel barrier-wait stamps (needs a debug buffer)
  kF32_256 = 6,       // exact-fp32 256x256 without the staggered DMA
  kMfma256X1 = 10,    // SCHED 2 + per-cluster setprio
  kMfma256X2 = 11,    // SCHED 2 + static priority of waves 4..7
  kMfma256X4 = 13,    // SCHED 2 + XCD sub-block 8x4
  kFp8 = 15,          // fp8 8-wave 256x256 (block-scaled MFMA 16x16x128)
  kFp8W4Diag = 17,    // timing only (wrong results): kFp8W4 without the DMA wait
  kFp8W4Diag2 = 18,   // timing only: no wait at all before the barrier
  kFp8W4Diag3 = 19,   // timing only: MFMAs + barriers, no loads
  kF32NoDma = 20,     // timing only: f32 K-loop without loads
  kMfmaW4Tall = 22,   // kMfmaW4 (bf16) with the 8x4 XCD sub-block
  kMfmaW4Wide = 23,   // kMfmaW4 (bf16) with the 2x16 XCD sub-block
  kFp8W4Tall = 24,    // kFp8W4 with the 8x4 XCD sub-block
  kFp8W4Wide = 25,    // kFp8W4 with the 2x16 XCD sub-block
  kFp8W4Scaled = 31,  // kFp8W4 on the block-scaled MFMA form (scales 1)
  kMfmaW4Trace = 32,  // kMfmaW4 (bf16) writing the tile timeline into the debug buffer
  kFp8W4Trace = 33,   // kFp8W4 writing the tile timeline into the debug buffer
  kMfmaW4Pers = 34,   // persistent W4 (one workgroup per CU, per-XCD work queues)
  kMfmaW4PersTrace = 35,  // kMfmaW4Pers writing the tile timeline
  kMfmaW4STrace = 38,  // W4S writing per-workgroup start / end stamps
  kMfmaW4SRot = 39,    // W4S with the per-round rotating XCD block map (supertile 6)
  kMfmaW4SRotTrace = 40,  // kMfmaW4SRot with per-workgroup start / end stamps
  kMfmaW4Il32 = 30,   // kMfmaW4 (bf16) with the 8-wave kernel's 32-column B-half interleave
  kFp8W4TS = 43,      // kFp8W4 with plain (temporal) C stores (shipping: non-temporal)
  kFp8W4STS = 44,     // kFp8W4S with plain C stores
  kMfmaW4STS = 45,    // kMfmaW4S (bf16) with plain C stores
  kF32_256sDirect = 46,  // kF32_256s with direct (not LDS-staged, temporal) C stores
  kFp8W4Unfused = 47,    // kFp8W4 with the epilogue after (not inside) the last K-tile
  kT128Unfused = 48,     // kT128 (bf16 / fp16) with the epilogue after the last K-tile
  kFp8T128Unfused = 49,  // kFp8T128 with the epilogue after the last K-tile
  kMfmaW4Unfused = 50,   // kMfmaW4 (bf16) with the epilogue after the last K-tile
  kF32T128B32 = 52,      // kF32T128 with one b32 LDS read per B operand (round 3's first version)
  kF32W4B32 = 54,        // kF32W4 with one b32 LDS read per B operand (round 2's version)
  kF32_256p = 55,        // kF32_256s with software-pipelined fragments and a mid-tile barrier
  // W4S power attribution (timing only, wrong results; scripts/power_attrib.py):
  kMfmaW4SNoFrag = 56,   // no LDS fragment reads (MFMAs re-use their registers)
  kMfmaW4SNoDma = 57,    // no LDS-DMA refills in the K-loop
  kMfmaW4SNoEpi = 58,    // no C stores (no-access loads in their place)
  kMfmaW4SMfmaOnly = 59, // neither fragment reads nor refills: MFMAs, waits, barriers
  // W4S tile orders (round 6, VERDICT r5 #6: does the clock follow the L2 /
  // Infinity Cache hit rate?), the shipping K-loop with another map_tile order:
  kMfmaW4STall = 70,     // XCD sub-block 8 x 4 (12 panels per K-step, A-heavy)
  kMfmaW4SWide = 71,     // XCD sub-block 2 x 16 (18 panels per K-step: lower L2 hit)
  kMfmaW4SSnake = 72,    // 16 x 16 rounds in snake order (odd rows sweep N backwards)
  kMfmaW4SMcol = 73,     // 16 x 16 rounds sweeping M fastest
  // fp8 W4S's K4 form on any even nk >= 4 (round 6; the
  // shipping W4S runs it at nk == 4 only, K = 512)
  kFp8W4SK4 = 74,
  kFp8W4SK4TS = 75,      // the same with plain (temporal) C stores
  // thin grids (tiles_n = 8: the ws = 8 shards at 16k / 8k): mode 3's 32 x 8
  // round as an 8 x 1 XCD grid of 4 x 8 blocks (supertile 9)
  kMfmaW4SSt9 = 76,
  kMfmaW4St9 = 77,
  kFp8W4SSt9 = 78,
  kFp8W4St9 = 79,
  kF32W4NB = 80,         // exact-fp32 W4 with a branch-free K-loop (round 6)
  kF32W4NBP = 81,        // kF32W4NB with 1024-B B rows: conflict-free b128 B reads (round 6)
  kF32W4NoDma = 82,      // timing-only kF32W4NBP diagnostics (WRONG results): no DMA refills,
  kF32W4NoFrag = 83,     //   no fragment reads,
  kF32W4MfmaBar = 84,    //   MFMAs and the mid-tile barrier only,
  kF32W4MfmaOnly = 85,   //   MFMAs only
  kF32W4Spread = 86,     // kF32W4NBP with the DMA pieces and fragment reads spread over each half,
  kF32W4SpreadDma = 87,  //   the DMA pieces only,
  kF32W4SpreadRd = 88,   //   the fragment reads only
  kF32W4Lean = 89,       // kF32W4NBP with a third of the SALU per K-tile (descriptors built once)
  kF32W4Lean2 = 90,      // kF32W4Lean without the s_nop per DMA piece
  kF32W4S = 91,          // the streamed persistent form of kF32W4Lean2 (hangs, see gemm_f32_w4.hip)
  kF32T128Lean = 92,     // kF32T128 / kF32T128x2 / kF32T64 / kF32T64x2 with the W4 lean K-loop
  kF32T128x2Lean = 93,   //   (descriptors built once per slice, K-tile offsets in the voffsets,
  kF32T64Lean = 94,      //   M0 in one SALU, the DMA piece fused with its gap's MFMA; round 6)
  kF32T64x2Lean = 95,
  kF32W4SDbg = 96,       // f32_w4s stamping its progress into a host-mapped buffer (diagnostic)
  kMfmaW4SLean = 97,
  kFp8W4SThin = 98,      // fp8 W4S / W4S with the thin round that follows the grid's aspect
  kMfmaW4SThin = 99,     //   (common.h thin_supertile) in place of the 16 x 16 round     // W4S with the lean DMA issue (voffset K-offsets, tile descriptors, fused pieces)
};

}  // namespace pdmb
