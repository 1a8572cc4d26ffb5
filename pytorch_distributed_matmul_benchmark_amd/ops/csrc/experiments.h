// Experiment / diagnostic GEMM kernels: the A/B arms and timing-only builds
// behind the profiles/ tables (docs/REPRODUCE.md). Compiled only into a
// library built with PDMB_EXPERIMENTS=1 (ops/build.py): gemm_dispatch.cpp
// includes this file at its end, inside namespace pdmb, so these functions see
// the dispatcher's helpers (plan, supports, tiled_launch, ...); the shipping
// build never includes it and refuses every id below (ops/gemm.py
// EXPERIMENT_KERNELS). The kernels themselves are template variants of the
// shipping ones (a flag of their launch functions), so they stay in the .hip
// sources under #ifdef PDMB_EXPERIMENTS.
// The ids are experiment_ids.h.
#pragma once




static bool is_experiment(int k) {
  switch (k) {
    case kMfma256: case kMfma256b: case kMfma256c: case kMfma256Stamp: case kF32_256:
    case kMfma256X1: case kMfma256X2: case kMfma256X4: case kFp8: case kFp8W4Diag:
    case kFp8W4Diag2: case kFp8W4Diag3: case kF32NoDma: case kMfmaW4Tall: case kMfmaW4Wide: case kMfmaW4Il32:
    case kMfmaW4Pers: case kMfmaW4PersTrace: case kMfmaW4STrace: case kMfmaW4SRot: case kMfmaW4SRotTrace:
    case kFp8W4Tall: case kFp8W4Wide: case kFp8W4Scaled: case kFp8W4Trace: case kMfmaW4Trace:
    case kFp8W4TS: case kFp8W4STS: case kMfmaW4STS: case kF32_256sDirect: case kFp8W4Unfused:
    case kT128Unfused: case kFp8T128Unfused: case kMfmaW4Unfused: case kF32T128B32:
    case kF32W4B32: case kF32_256p: case kMfmaW4SNoFrag: case kMfmaW4SNoDma: case kMfmaW4SNoEpi:
    case kMfmaW4SMfmaOnly: case kMfmaW4STall: case kMfmaW4SWide: case kMfmaW4SSnake: case kMfmaW4SMcol:
    case kFp8W4SK4: case kFp8W4SK4TS: case kMfmaW4SSt9: case kMfmaW4St9: case kFp8W4SSt9: case kFp8W4St9:
    case kF32W4NB: case kF32W4NBP: case kF32W4NoDma: case kF32W4NoFrag: case kF32W4MfmaBar:
    case kF32W4MfmaOnly: case kF32W4Spread: case kF32W4SpreadDma: case kF32W4SpreadRd:
    case kF32W4Lean: case kF32W4Lean2: case kF32T128Lean: case kF32T128x2Lean: case kF32T64Lean:
    case kF32T64x2Lean: case kF32W4S: case kF32W4SDbg: case kMfmaW4SLean: case kFp8W4SThin: case kMfmaW4SThin:
      return true;
    default:
      return false;
  }
}

static bool experiment_is_fp8(int k) {
  return k == kFp8 || k == kFp8W4TS || k == kFp8W4STS || k == kFp8W4Unfused || k == kFp8T128Unfused ||
         k == kFp8W4Diag || k == kFp8W4Diag2 || k == kFp8W4Diag3 || k == kFp8W4Tall || k == kFp8W4Wide ||
         k == kFp8W4Scaled || k == kFp8W4Trace || k == kFp8W4SK4 || k == kFp8W4SK4TS || k == kFp8W4SSt9 ||
         k == kFp8W4St9 || k == kFp8W4SThin;
}

static int experiment_resolve_fp8(const Problem& p, int kernel, bool s_fits) {
  if (kernel == kFp8W4STS) return s_fits ? kernel : -1;
  if (kernel == kFp8W4SSt9 || kernel == kFp8W4SThin) return s_fits ? kernel : -1;
  if (kernel == kFp8W4St9) return kernel;
  if (kernel == kFp8W4SK4 || kernel == kFp8W4SK4TS)
    return gemm_fp8_w4s_k4_fits(shape_args(p)) && device_cus() % 8 == 0 ? kernel : -1;
  if (kernel == kFp8T128Unfused) return supports(p, kFp8T128) ? kernel : -1;
  return kernel;
}

// The shipping kernel whose plan (split) a lean fp32 tile arm runs.
static int ln_base(int k) {
  return k == kF32T128Lean ? kF32T128 : k == kF32T128x2Lean ? kF32T128x2 : k == kF32T64Lean ? kF32T64 : kF32T64x2;
}

static int experiment_resolve(const Problem& p, int kernel, bool fast, bool w4, bool t128, bool f32fast) {
  switch (kernel) {
    case kF32_256: case kF32NoDma: case kF32_256sDirect: case kF32_256p: return f32fast ? kernel : -1;
    case kT128Unfused: return t128 ? kernel : -1;
    case kF32T128B32: return p.dtype == kF32 && supports(p, kF32T128) ? kernel : -1;
    case kF32W4S: case kF32W4SDbg:
      return f32fast && gemm_f32_w4s_fits(shape_args(p)) && device_cus() % 8 == 0 ? kernel : -1;
    case kF32T128Lean: case kF32T128x2Lean: case kF32T64Lean: case kF32T64x2Lean:
      return p.dtype == kF32 && supports(p, kF32T128) && gemm_f32_tile_ln_fits(shape_args(p)) ? kernel : -1;
    case kF32W4B32: case kF32W4NB: case kF32W4NBP: case kF32W4NoDma: case kF32W4NoFrag:
    case kF32W4MfmaBar: case kF32W4MfmaOnly: case kF32W4Spread: case kF32W4SpreadDma: case kF32W4SpreadRd:
    case kF32W4Lean: case kF32W4Lean2:
      return f32fast ? kernel : -1;
    case kMfmaW4Unfused: return (p.dtype == kBF16 && w4) ? kernel : -1;
    case kMfma256: case kMfma256b: case kMfma256c: return fast ? kernel : -1;
    case kMfma256X1: case kMfma256X2: case kMfma256X4: case kMfma256Stamp:
      return (fast && p.dtype == kBF16) ? kernel : -1;
    case kMfmaW4Tall: case kMfmaW4Wide: case kMfmaW4Il32: case kMfmaW4Trace:
    case kMfmaW4PersTrace:
      return (p.dtype == kBF16 && w4) ? kernel : -1;
    case kMfmaW4STrace: case kMfmaW4SRot: case kMfmaW4SRotTrace: case kMfmaW4STS:
    case kMfmaW4SNoFrag: case kMfmaW4SNoDma: case kMfmaW4SNoEpi: case kMfmaW4SMfmaOnly:
    case kMfmaW4STall: case kMfmaW4SWide: case kMfmaW4SSnake: case kMfmaW4SMcol: case kMfmaW4SSt9:
      return (p.dtype == kBF16 && w4 && w4s_fits(p)) ? kernel : -1;
    case kMfmaW4St9: return (p.dtype == kBF16 && w4) ? kernel : -1;
    case kMfmaW4SLean: return w4 && w4s_fits(p) && gemm_w4s_lean_fits(shape_args(p)) ? kernel : -1;
    case kMfmaW4SThin: return w4 && w4s_fits(p) ? kernel : -1;
    case kMfmaW4Pers: return w4 ? kernel : -1;  // bf16 and fp16
    default: return -1;
  }
}

static size_t experiment_workspace_bytes(const Problem& p, int k) {
  if (k == kMfmaW4Tall || k == kMfmaW4Wide || k == kMfmaW4Il32 || k == kMfmaW4Trace ||
      k == kMfmaW4Pers || k == kMfmaW4PersTrace)
    return splitk_bytes(p, kMfmaW4, plan(p, kMfmaW4).splitk);
  if (k == kF32T128B32) return splitk_bytes(p, kF32T128, plan(p, kF32T128).splitk);
  if (k >= kF32T128Lean && k <= kF32T64x2Lean) {
    const int base = ln_base(k);
    return splitk_bytes(p, base, plan(p, base).splitk);
  }
  if (k == kF32W4B32 || (k >= kF32W4NB && k <= kF32W4Lean2)) return splitk_bytes(p, kF32W4, plan(p, kF32W4).splitk);
  return 0;
}

static hipError_t experiment_launch(const Problem& p, int k, const GemmArgs& a, hipStream_t stream) {
  switch (k) {
    case kFp8: return gemm_fp8_launch(a, 0, stream);
    case kFp8W4Diag: return gemm_fp8_launch(a, 9, stream);
    case kFp8W4Diag2: return gemm_fp8_launch(a, 10, stream);
    case kFp8W4Diag3: return gemm_fp8_launch(a, 11, stream);
    case kFp8W4Tall: return gemm_fp8_launch(a, 12, stream);
    case kFp8W4Wide: return gemm_fp8_launch(a, 13, stream);
    case kFp8W4Scaled: return gemm_fp8_launch(a, 14, stream);
    case kFp8W4Trace: return gemm_fp8_launch(a, 15, stream);
    case kFp8W4TS: return gemm_fp8_launch(a, 16, stream);
    case kFp8W4Unfused: return gemm_fp8_launch(a, 18, stream);
    case kT128Unfused:
    case kFp8T128Unfused: return gemm_tile_launch(k, p.dtype, a, stream);  // unsplit (A/B)
    case kMfmaW4Unfused: return gemm_w4_launch(p.dtype, a, stream, 12);   // unsplit (A/B)
    case kFp8W4STS: {
      GemmArgs s = a;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_fp8_launch(s, 17, stream);
    }
    case kFp8W4SK4:
    case kFp8W4SK4TS: {
      GemmArgs s = a;
      s.splitk = 1;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_fp8_launch(s, k == kFp8W4SK4 ? 19 : 20, stream);
    }
    case kMfmaW4STS: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 11);
    case kMfmaW4SNoFrag: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 13);
    case kMfmaW4SNoDma: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 14);
    case kMfmaW4SNoEpi: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 15);
    case kMfmaW4SMfmaOnly: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 16);
    case kMfmaW4STall: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 17);
    case kMfmaW4SWide: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 18);
    case kMfmaW4SSnake: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 19);
    case kMfmaW4SMcol: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 20);
    case kMfmaW4SSt9: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 21);
    case kMfmaW4SLean: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 23);
    case kMfmaW4SThin: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 24);
    case kFp8W4SThin: {
      GemmArgs s = a;
      s.splitk = 1;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_fp8_launch(s, 23, stream);
    }
    case kMfmaW4St9: {
      GemmArgs s = a;
      s.splitk = 1;
      return gemm_w4_launch(p.dtype, s, stream, 22);
    }
    case kFp8W4SSt9: {
      GemmArgs s = a;
      s.splitk = 1;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_fp8_launch(s, 21, stream);
    }
    case kFp8W4St9: {
      GemmArgs s = a;
      s.splitk = 1;
      return gemm_fp8_launch(s, 22, stream);
    }
    case kMfma256: return gemm256_launch(p.dtype, a, 0, stream);
    case kMfma256b: return gemm256_launch(p.dtype, a, 1, stream);
    case kMfma256c: return gemm256_launch(p.dtype, a, 2, stream);
    case kMfma256Stamp: return gemm256_launch(p.dtype, a, 3, stream);
    case kMfmaW4Tall: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 1);
    case kMfmaW4Wide: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 2);
    case kMfmaW4Il32: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 3);
    case kMfmaW4Trace: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 4);
    case kMfmaW4Pers: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 5);
    case kMfmaW4PersTrace: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 6);
    case kMfmaW4STrace: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 8);
    case kMfmaW4SRot: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 9);
    case kMfmaW4SRotTrace: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 10);
    case kF32_256: return gemm_f32_256_launch(a, 0, stream);
    case kF32NoDma: return gemm_f32_256_launch(a, 9, stream);
    case kF32_256sDirect: return gemm_f32_256_launch(a, 10, stream);
    case kF32_256p: return gemm_f32_256_launch(a, 11, stream);
    case kF32T128B32: return tiled_launch(p, kF32T128, a, p.workspace, p.workspace_bytes, stream, 1);
    case kF32W4S: case kF32W4SDbg: {
      GemmArgs s = a;
      s.splitk = 1;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_f32_w4_launch(s, stream, k == kF32W4S ? 14 : 15);
    }
    case kF32T128Lean: case kF32T128x2Lean: case kF32T64Lean: case kF32T64x2Lean:
      return tiled_launch(p, ln_base(k), a, p.workspace, p.workspace_bytes, stream, 5 + (k - kF32T128Lean));
    case kF32W4B32: return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 1);
    case kF32W4NB: return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 2);
    case kF32W4NBP: return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 3);
    case kF32W4NoDma: case kF32W4NoFrag: case kF32W4MfmaBar: case kF32W4MfmaOnly:
      return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 4 + (k - kF32W4NoDma));
    case kF32W4Spread: case kF32W4SpreadDma: case kF32W4SpreadRd:
      return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 8 + (k - kF32W4Spread));
    case kF32W4Lean: return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 11);
    case kF32W4Lean2: return tiled_launch(p, kF32W4, a, p.workspace, p.workspace_bytes, stream, 12);
    case kMfma256X1: case kMfma256X2: case kMfma256X4:
      return gemm256_launch(p.dtype, a, 10 + (k - kMfma256X1 + 1), stream);
    default: return hipErrorInvalidValue;
  }
}

static const char* experiment_name(int kernel) {
  switch (kernel) {
    case kMfma256: return "pdmb_mfma256_nn";
    case kMfma256b: return "pdmb_mfma256b_nn";
    case kMfma256c: return "pdmb_mfma256c_nn";
    case kMfma256Stamp: return "pdmb_mfma256c_stamp";
    case kF32_256: return "pdmb_f32_256_nn";
    case kFp8: return "pdmb_fp8_256_nt";
    case kMfmaW4Tall: return "pdmb_w4_nn_tall";
    case kMfmaW4Wide: return "pdmb_w4_nn_wide";
    case kMfmaW4Il32: return "pdmb_w4_nn_il32";
    case kFp8W4Tall: return "pdmb_fp8_w4_nt_tall";
    case kFp8W4Wide: return "pdmb_fp8_w4_nt_wide";
    case kFp8W4Scaled: return "pdmb_fp8_w4_nt_scaled";
    case kMfmaW4Trace: return "pdmb_w4_nn_trace";
    case kMfmaW4Pers: return "pdmb_w4_pers";
    case kMfmaW4PersTrace: return "pdmb_w4_pers_trace";
    case kMfmaW4STrace: return "pdmb_w4s_trace";
    case kMfmaW4SRot: return "pdmb_w4s_rot";
    case kMfmaW4SRotTrace: return "pdmb_w4s_rot_trace";
    case kFp8W4TS: return "pdmb_fp8_w4_nt_tstore";
    case kFp8W4STS: return "pdmb_fp8_w4s_tstore";
    case kMfmaW4STS: return "pdmb_w4s_tstore";
    case kF32_256sDirect: return "pdmb_f32_256s_direct";
    case kF32_256p: return "pdmb_f32_256p_nn";
    case kFp8W4Unfused: return "pdmb_fp8_w4_nt_unfused";
    case kT128Unfused: return "pdmb_t128_nn_unfused";
    case kFp8T128Unfused: return "pdmb_fp8_t128_nt_unfused";
    case kMfmaW4Unfused: return "pdmb_w4_nn_unfused";
    case kF32T128B32: return "pdmb_f32_t128_b32";
    case kF32W4B32: return "pdmb_f32_w4_b32";
    case kF32W4NB: return "pdmb_f32_w4_nb";
    case kF32W4NBP: return "pdmb_f32_w4_nbp";
    case kF32W4NoDma: return "pdmb_f32_w4_diag_nodma";
    case kF32W4NoFrag: return "pdmb_f32_w4_diag_nofrag";
    case kF32W4MfmaBar: return "pdmb_f32_w4_diag_mfma_bar";
    case kF32W4MfmaOnly: return "pdmb_f32_w4_diag_mfma_only";
    case kF32W4Spread: return "pdmb_f32_w4_spread";
    case kF32W4SpreadDma: return "pdmb_f32_w4_spread_dma";
    case kF32W4SpreadRd: return "pdmb_f32_w4_spread_rd";
    case kF32T128Lean: return "pdmb_f32_t128_lean";
    case kF32T128x2Lean: return "pdmb_f32_t128x2_lean";
    case kF32T64Lean: return "pdmb_f32_t64_lean";
    case kF32T64x2Lean: return "pdmb_f32_t64x2_lean";
    case kF32W4S: return "pdmb_f32_w4s";
    case kF32W4SDbg: return "pdmb_f32_w4s_dbg";
    case kMfmaW4SLean: return "pdmb_w4s_lean";
    case kF32W4Lean: return "pdmb_f32_w4_lean";
    case kF32W4Lean2: return "pdmb_f32_w4_lean2";
    case kFp8W4Trace: return "pdmb_fp8_w4_nt_trace";
    case kMfmaW4SNoFrag: return "pdmb_w4s_diag_nofrag";
    case kMfmaW4SNoDma: return "pdmb_w4s_diag_nodma";
    case kMfmaW4SNoEpi: return "pdmb_w4s_diag_noepi";
    case kMfmaW4SMfmaOnly: return "pdmb_w4s_diag_mfma_only";
    case kMfmaW4STall: return "pdmb_w4s_tall";
    case kMfmaW4SWide: return "pdmb_w4s_wide";
    case kMfmaW4SSnake: return "pdmb_w4s_snake";
    case kMfmaW4SMcol: return "pdmb_w4s_mcol";
    case kFp8W4SK4: return "pdmb_fp8_w4s_k4";
    case kFp8W4SK4TS: return "pdmb_fp8_w4s_k4_tstore";
    case kMfmaW4SSt9: return "pdmb_w4s_st9";
    case kMfmaW4St9: return "pdmb_w4_nn_st9";
    case kFp8W4SSt9: return "pdmb_fp8_w4s_st9";
    case kFp8W4SThin: return "pdmb_fp8_w4s_thin";
    case kMfmaW4SThin: return "pdmb_w4s_thin";
    case kFp8W4St9: return "pdmb_fp8_w4_nt_st9";
    default: return "auto";
  }
}
