// gemm_generic.hip — shape-general MFMA GEMM for gfx950: any M, N, K, any
// leading dimensions / alignment, batched, for fp32 (exact f32 MFMA
// v_mfma_f32_16x16x4_f32 — gfx950 has no TF32/xf32), fp16 and bf16
// (v_mfma_f32_16x16x32_*). Row-major NN: C[b] = A[b] @ B[b].
//
// This is the fallback behind gemm_mfma256.hip (which needs K % 64 == 0,
// N % 8 == 0 and 16-B alignment) and the fp32 path of the benchmark
// (reference `--dtype float32`, matmul_benchmark.py:163-174).
//
// Structure: 128x128 tile, BK = 32, 256 threads = 4 waves (2x2), each wave
// 64x64 = 4x4 MFMA tiles. Global -> registers (bounds-checked, 16-B
// vectors when alignment allows) -> LDS, with the next tile's global loads
// issued before the current tile's MFMAs (register double-buffering).
// Several workgroups per CU hide the two barriers per K-tile.
// Like the fast kernel, MFMA operands are swapped so each lane holds 4
// consecutive output columns of one row.
#include "common.h"

namespace pdmb {
namespace kgen {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

// ---- 16-bit variant -----------------------------------------------------
constexpr int A16_LD = BK + 8;    // 40 el = 80 B rows (16-B aligned)
constexpr int B16_LD = BN + 8;    // 136 el = 272 B rows (16-B aligned)

template <int DT, bool VEC>
__global__ void __launch_bounds__(NT) gemm_generic16(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short As[BM * A16_LD];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[BK * B16_LD];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const unsigned short* A = (const unsigned short*)a.A + (long long)bz * a.sA;
  const unsigned short* B = (const unsigned short*)a.B + (long long)bz * a.sB;
  unsigned short* C = (unsigned short*)a.C + (long long)bz * a.sC;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int l16 = lane & 15, g = lane >> 4;

  s16x8 ra[2], rb[2];  // staged global data (2 vectors each for A and B)
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * NT;
      {  // A: row = idx>>2, k = (idx&3)*8
        const int r = idx >> 2, kc = (idx & 3) * 8;
        const int gm = m0 + r, gk = k0 + kc;
        s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (gm < a.M) {
          const unsigned short* p = A + (long long)gm * a.lda + gk;
          if (VEC && gk + 8 <= a.K) {
            v = *(const s16x8*)p;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (gk + e < a.K) ? (short)p[e] : (short)0;
          }
        }
        ra[i] = v;
      }
      {  // B: k = idx>>4, n = (idx&15)*8
        const int kr = idx >> 4, nc = (idx & 15) * 8;
        const int gk = k0 + kr, gn = n0 + nc;
        s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (gk < a.K) {
          const unsigned short* p = B + (long long)gk * a.ldb + gn;
          if (VEC && gn + 8 <= a.N) {
            v = *(const s16x8*)p;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (gn + e < a.N) ? (short)p[e] : (short)0;
          }
        }
        rb[i] = v;
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + i * NT;
      *(s16x8*)&As[(idx >> 2) * A16_LD + (idx & 3) * 8] = ra[i];
      *(s16x8*)&Bs[(idx >> 4) * B16_LD + (idx & 15) * 8] = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  gload(0);
  for (int t = 0; t < nk; ++t) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (t + 1 < nk) gload((t + 1) * BK);
    s16x8 fa[4], fb[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
      fa[mi] = *(const s16x8*)&As[(wr * 64 + mi * 16 + l16) * A16_LD + g * 8];
    const int q4 = l16 >> 2, p4 = l16 & 3;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const unsigned short* p = &Bs[(8 * g + q4) * B16_LD + wc * 64 + ni * 16 + 4 * p4];
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * B16_LD));
      fb[ni] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16x16x32<DT>(fb[ni], fa[mi], acc[mi][ni]);
  }

#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int row = m0 + wr * 64 + mi * 16 + l16;
    if (row >= a.M) continue;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wc * 64 + ni * 16 + 4 * g;
      unsigned short* p = C + (long long)row * a.ldc + col;
      const unsigned int lo = pack2<DT>(acc[mi][ni].x, acc[mi][ni].y);
      const unsigned int hi = pack2<DT>(acc[mi][ni].z, acc[mi][ni].w);
      if (VEC && col + 4 <= a.N) {
        *(u32x2*)p = u32x2{lo, hi};
      } else {
        const unsigned short v[4] = {(unsigned short)lo, (unsigned short)(lo >> 16),
                                     (unsigned short)hi, (unsigned short)(hi >> 16)};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < a.N) p[e] = v[e];
      }
    }
  }
}

// ---- fp32 variant -------------------------------------------------------
constexpr int A32_LD = BK + 2;     // 34: ds_read_b32 of A[l16][g] conflict-free
constexpr int B32_LD = BN + 16;    // 144: B[g][l16] rows land on disjoint banks

template <bool VEC>
__global__ void __launch_bounds__(NT) gemm_generic32(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) float As[BM * A32_LD];
  __shared__ __attribute__((aligned(16))) float Bs[BK * B32_LD];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = (const float*)a.A + (long long)bz * a.sA;
  const float* B = (const float*)a.B + (long long)bz * a.sB;
  float* C = (float*)a.C + (long long)bz * a.sC;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int l16 = lane & 15, g = lane >> 4;

  f32x4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NT;
      {  // A: row = idx>>3, k = (idx&7)*4
        const int r = idx >> 3, kc = (idx & 7) * 4;
        const int gm = m0 + r, gk = k0 + kc;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gm < a.M) {
          const float* p = A + (long long)gm * a.lda + gk;
          if (VEC && gk + 4 <= a.K) {
            v = *(const f32x4*)p;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (gk + e < a.K) ? p[e] : 0.f;
          }
        }
        ra[i] = v;
      }
      {  // B: k = idx>>5, n = (idx&31)*4
        const int kr = idx >> 5, nc = (idx & 31) * 4;
        const int gk = k0 + kr, gn = n0 + nc;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gk < a.K) {
          const float* p = B + (long long)gk * a.ldb + gn;
          if (VEC && gn + 4 <= a.N) {
            v = *(const f32x4*)p;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (gn + e < a.N) ? p[e] : 0.f;
          }
        }
        rb[i] = v;
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NT;
      const int r = idx >> 3, kc = (idx & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) As[r * A32_LD + kc + e] = ra[i][e];
      *(f32x4*)&Bs[(idx >> 5) * B32_LD + (idx & 31) * 4] = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  gload(0);
  for (int t = 0; t < nk; ++t) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (t + 1 < nk) gload((t + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      float fa[4], fb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) fa[mi] = As[(wr * 64 + mi * 16 + l16) * A32_LD + ks * 4 + g];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) fb[ni] = Bs[(ks * 4 + g) * B32_LD + wc * 64 + ni * 16 + l16];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[ni], fa[mi], acc[mi][ni], 0, 0, 0);
    }
  }

#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int row = m0 + wr * 64 + mi * 16 + l16;
    if (row >= a.M) continue;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wc * 64 + ni * 16 + 4 * g;
      float* p = C + (long long)row * a.ldc + col;
      if (VEC && col + 4 <= a.N) {
        *(f32x4*)p = acc[mi][ni];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < a.N) p[e] = acc[mi][ni][e];
      }
    }
  }
}

}  // namespace kgen

hipError_t gemm_generic_launch(int dt, GemmArgs a, bool vec, hipStream_t stream) {
  a.tiles_m = (a.M + kgen::BM - 1) / kgen::BM;
  a.tiles_n = (a.N + kgen::BN - 1) / kgen::BN;
  a.supertile = 0;
  const long long nblocks = (long long)a.tiles_m * a.tiles_n * a.batch;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  dim3 grid((unsigned)nblocks), block(kgen::NT);
  if (dt == kF32) {
    if (vec)
      hipLaunchKernelGGL(kgen::gemm_generic32<true>, grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL(kgen::gemm_generic32<false>, grid, block, 0, stream, a);
  } else if (dt == kBF16) {
    if (vec)
      hipLaunchKernelGGL((kgen::gemm_generic16<kBF16, true>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kgen::gemm_generic16<kBF16, false>), grid, block, 0, stream, a);
  } else {
    if (vec)
      hipLaunchKernelGGL((kgen::gemm_generic16<kF16, true>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kgen::gemm_generic16<kF16, false>), grid, block, 0, stream, a);
  }
  return hipGetLastError();
}

}  // namespace pdmb
