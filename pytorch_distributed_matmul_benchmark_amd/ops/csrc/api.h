// Host-side C++ API of the native GEMM library (no torch dependency).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>

namespace pdmb {

enum Kernel : int {
  kAuto = 0,      // fastest kernel that supports the problem
  kMfma256 = 1,   // gemm_mfma256.hip (LDS-DMA, 256x256, ping-pong)
  kGeneric = 2,   // gemm_generic.hip (any shape)
  kMfma256b = 3,  // gemm_mfma256.hip, DMA issued in the read slot (SCHED 1)
  kMfma256c = 4,  // SCHED 1 + fragment reads balanced over the read slots (SCHED 2)
  kMfma256d = 9,  // SCHED 3: two quadrants (32 MFMAs) per compute slot, 4 barriers per K-tile
  kF32_256 = 6,   // gemm_f32_256.hip: exact-fp32 MFMA, 256x256 LDS-DMA tile
  kF32_256s = 7,  // same, DMA issue staggered between the two waves of a SIMD
  kF32NoDma = 20,  // diagnostic: f32 K-loop without loads (timing only, wrong results)
  kMfma256X1 = 10,  // SCHED 2 experiment builds (A/B only): 10 = per-cluster setprio,
  kMfma256X2 = 11,  //   11 = static priority of waves 4..7,
  kMfma256X4 = 13,  //   13 = XCD sub-block 8x4 (12 unused)
  kMfma256Stamp = 5,  // diagnostic: SCHED 2 with in-kernel barrier-wait stamps (needs a debug buffer)
  kFp8W4 = 16,    // gemm_fp8.hip experiment: 4 waves x 128x128, AGPR accumulators via asm MFMA
  kFp8W4Diag = 17,  // diagnostic: kFp8W4 without the DMA wait (timing only, wrong results)
  kFp8W4Diag2 = 18,  // diagnostic: kFp8W4 with no wait at all before the barrier
  kFp8W4Diag3 = 19,  // diagnostic: kFp8W4 MFMAs + barriers only (no loads)
  kMfmaW4 = 21,   // gemm_w4.hip: bf16/fp16 NN, 4 waves x 128x128, AGPR accumulators (M, N % 256)
  kMfmaW4Tall = 22,  // experiment (A/B only): kMfmaW4 (bf16) with the 8x4 XCD sub-block
  kMfmaW4Wide = 23,  // experiment (A/B only): kMfmaW4 (bf16) with the 2x16 XCD sub-block
  kFp8W4Tall = 24,   // experiment (A/B only): kFp8W4 with the 8x4 XCD sub-block
  kFp8W4Wide = 25,   // experiment (A/B only): kFp8W4 with the 2x16 XCD sub-block
  kFp8 = 15,      // gemm_fp8.hip: e4m3 A [M,K] x column-major B, block-scaled MFMA 16x16x128, bf16 out
};

// dtype kFP8: A, B are OCP fp8 e4m3, B is COLUMN-major (ldb = distance between
// columns, i.e. B is stored as Bt [N,K]), C is bf16 and C = alpha * (A @ B).
struct Problem {
  int dtype;  // DType
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  int lda, ldb, ldc;
  long long sA, sB, sC;
  int batch;
  float alpha = 1.0f;
};

// Which kernel `kernel` (kAuto allowed) resolves to for this problem;
// -1 if the requested kernel cannot run it.
int resolve_kernel(const Problem& p, int kernel);

// Enqueue C = A @ B on `stream`. Returns hipSuccess or an error; *used (if
// non-null) receives the kernel that ran. With kAuto, a large problem whose K /
// N / alignment miss the fast kernels runs on them through zero-padded
// workspace copies (gemm_dispatch.cpp "padded fast path").
hipError_t gemm(const Problem& p, int kernel, hipStream_t stream, int* used);

// Native timing loop: `warmup` untimed launches, then `iters` launches
// bracketed by hipEvents on `stream` (optionally captured once into a
// hipGraph and replayed, which removes host launch gaps). Returns the
// total elapsed milliseconds of the timed region in *ms.
hipError_t bench_gemm(const Problem& p, int kernel, int iters, int warmup, bool use_graph,
                      hipStream_t stream, float* ms);

const char* kernel_name(int kernel);

// Diagnostic builds write per-wave stamps here (device memory; nullptr = off).
void set_debug_buffer(void* p);

}  // namespace pdmb
