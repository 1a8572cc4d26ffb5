// gemm_f32_256.hip — exact-fp32 C = A @ B (row-major NN) on gfx950 MFMA
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate; gfx950 has no TF32/xf32,
// so this IS the fp32 path of the reference's `--dtype float32`,
// matmul_benchmark.py:163-174 / matmul_scaling_benchmark.py:365-374).
//
// fp32 MFMA runs at 64 FLOP/clk/SIMD (1/16 of bf16), so a 256×256 tile is
// MFMA-bound by a wide margin: per K-tile of 32 each wave issues 256 MFMAs
// (8192 cycles) against 48 LDS reads and 8 LDS-DMA pieces. The design goal is
// therefore just "never let the MFMA pipe idle":
//  * 256×256 tile, BK = 32, 8 waves (2 M × 4 N), each wave 128×64 =
//    8×4 MFMA tiles → 128 accumulators/lane, 2 waves per SIMD.
//  * Operands land in LDS by LDS-DMA, double-buffered (2 × 65 KiB). One
//    barrier per K-tile; the next tile's DMA is in flight for a whole tile.
//  * A image [256][32] fp32 (128-B rows), 16-B chunk c of row r stored at
//    c ^ ((r>>1)&7) (swizzle applied on the DMA source address): the
//    ds_read_b128 A fragments are conflict-free. One b128 read gives a lane
//    4 consecutive k of its row: k-step e of the 16-k block uses element e,
//    i.e. MFMA k-slot g holds k = 4g + e (a k-permutation the B read copies).
//  * B image [32][260] fp32 (1040-B rows: one DMA wave-instruction = one
//    256-column k-row, the 4-float pad puts k-rows 4 apart on opposite bank
//    halves): B fragment element = ds_read_b32 of B[4g+e][col] — conflict-free.
//  * Operands swapped in the MFMA (B fragment as "A") so each lane owns 4
//    consecutive output columns → 16-B stores.
// Fast-path constraints (host-checked, else gemm_generic.hip): K % 32 == 0,
// N % 4 == 0, lda/ldb % 4 == 0, ldc % 4 == 0, 16-B aligned A/B/C.
#include "common.h"

namespace pdmb {
namespace kf32 {

constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int A_BYTES = BM * BK * 4;         // 32 KiB
constexpr int B_PITCH = (BN + 4) * 4;        // 1040 B per k-row
constexpr int B_BYTES = BK * B_PITCH;        // 33,280 B
constexpr int STAGE = A_BYTES + B_BYTES;     // 66,048 B (16-B multiple)
constexpr int LDS_BYTES = 2 * STAGE;         // 132,096 B

struct Ctx {
  const char* Ab;
  const char* Bb;
  long long a_bytes, b_bytes;
  int lda4, ldb4, nk, wu;
  uint32_t voffA[4], voffB[4];
  uint32_t lds0;
};

// DMA of K-tile `tile` into stage STG: 4 A pieces (8 rows each) + 4 B pieces
// (one k-row each) per wave.
template <int STG>
__device__ __forceinline__ void issue_tile(const Ctx& c, int tile) {
  constexpr int ST = STAGE, BP = B_PITCH;
  const long long offA = (long long)tile * BK * 4;
  const u32x4 ra = make_rsrc(c.Ab + offA, c.a_bytes - offA);
  const long long offB = (long long)tile * BK * c.ldb4;
  const u32x4 rb = make_rsrc(c.Bb + offB, c.b_bytes - offB);
#pragma unroll
  for (int h = 0; h < 4; ++h)
    dma16(ra, c.voffA[h], c.lds0 + STG * ST + (h * 8 + c.wu) * 8 * 128);
#pragma unroll
  for (int h = 0; h < 4; ++h)
    dma16(rb, c.voffB[h], c.lds0 + STG * ST + A_BYTES + (h * 8 + c.wu) * BP);
}

template <int STG, int KB>
__device__ __forceinline__ void compute_half(const char* smem, int wr, int wc, int l16, int g,
                                             f32x4 (&acc)[8][4]) {
  {
    constexpr int kb = KB;
    f32x4 af[8];
    float bf[4][4];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int r = wr * 128 + mi * 16 + l16;
      const int ch = (kb * 4 + g) ^ ((r >> 1) & 7);
      af[mi] = *(const f32x4*)(smem + STG * STAGE + r * 128 + ch * 16);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int k = kb * 16 + 4 * g + e;
        const int col = wc * 64 + ni * 16 + l16;
        bf[ni][e] = *(const float*)(smem + STG * STAGE + A_BYTES + k * B_PITCH + col * 4);
      }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[ni][e], af[mi][e], acc[mi][ni],
                                                             0, 0, 0);
  }
}

// One K-tile from stage STG with the prefetch of tile `next` into the other
// stage. STAGGER: the two waves that share a SIMD (wave w and w+4) issue
// their DMA pieces at different points — waves 0..3 before the first 16-k
// half, waves 4..7 between the halves — so while one wave of the pair is
// issuing DMA (~60 cycles per piece) its partner keeps the MFMA pipe busy.
template <int STG, bool STAGGER, bool NODMA = false>
__device__ __forceinline__ void tile_step(const Ctx& c, const char* smem, int wr, int wc, int l16,
                                          int g, f32x4 (&acc)[8][4], int next) {
  const bool pf = !NODMA && next < c.nk;
  if (pf && (!STAGGER || wr == 0)) issue_tile<STG ^ 1>(c, next);
  compute_half<STG, 0>(smem, wr, wc, l16, g, acc);
  if (STAGGER && pf && wr == 1) issue_tile<STG ^ 1>(c, next);
  compute_half<STG, 1>(smem, wr, wc, l16, g, acc);
}

__device__ __forceinline__ void tile_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// NODMA: timing-only diagnostic (the K-loop issues no loads, results are
// wrong): the ceiling of the compute + barrier structure alone.
// LDSEPI: C through LDS as whole rows with non-temporal stores (common.h
// store_block16_f32; the shipping form); false: direct 16-B stores (A/B).
template <bool STAGGER, bool NODMA = false, bool LDSEPI = true>
__global__ void __launch_bounds__(NT, 2) gemm_f32_256(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wu >> 2, wc = wu & 3;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda4 = a.lda * 4;
  c.ldb4 = a.ldb * 4;
  c.nk = a.K / BK;
  c.Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda) * 4;
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + n0) * 4;
  c.a_bytes = ((long long)(a.M - m0 - 1) * a.lda + a.K) * 4;
  c.b_bytes = ((long long)(a.kb - 1) * a.ldb + (a.N - n0)) * 4;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int r = (h * 8 + wu) * 8 + (lane >> 3);
    const int src_chunk = (lane & 7) ^ ((r >> 1) & 7);
    c.voffA[h] = (uint32_t)(r * c.lda4 + src_chunk * 16);
    const int k = h * 8 + wu;
    c.voffB[h] = (uint32_t)(k * c.ldb4 + lane * 16);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = c.nk;
  issue_tile<0>(c, 0);
  tile_barrier();
  for (int t = 0; t < nk; t += 2) {
    // The stage being refilled was last read in the previous K-tile, which
    // ended with a barrier (WAR); the refill has a whole K-tile to land and
    // is retired by the vmcnt(0) + barrier that closes this one (RAW).
    tile_step<0, STAGGER, NODMA>(c, smem, wr, wc, l16, g, acc, t + 1);
    tile_barrier();
    if (t + 1 < nk) {
      tile_step<1, STAGGER, NODMA>(c, smem, wr, wc, l16, g, acc, t + 2);
      tile_barrier();
    }
  }

  if constexpr (LDSEPI) {  // the loop ended at a barrier: every wave is done with the stages
    char* Cb = (char*)a.C + (long long)bz * a.sC * 4;
    char* ebuf = smem + wu * epi_buf_f32<4>();
    const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      if (interior)
        store_block16_f32<false, 4>(ebuf, acc[mi], Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                    n0 + wc * 64, a.M, a.N, lane);
      else
        store_block16_f32<true, 4>(ebuf, acc[mi], Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                   n0 + wc * 64, a.M, a.N, lane);
    }
    return;
  }
  float* Cb = (float*)a.C + (long long)bz * a.sC;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int row = m0 + wr * 128 + mi * 16 + l16;
    if (row < a.M) {
      float* crow = Cb + (long long)row * a.ldc;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + wc * 64 + ni * 16 + 4 * g;
        if (col < a.N) *(f32x4*)(crow + col) = acc[mi][ni];
      }
    }
  }
}

// ---- f32_256p: the same tile with software-pipelined fragments -------------
// PMC of f32_256s at 16k (profiles/r2_pmc_fp32.md): 97.4 % MFMA busy vs 98.6 %
// for hipBLASLt at the same clock, with twice its WAIT_INST cycles — each wave
// starts a 16-k half by waiting for that half's LDS reads, and the barrier at
// the end of every K-tile lines the two waves of a SIMD up so they wait
// together. Here the K-tile runs as four quarters (8 k each: 64 MFMAs per
// wave) and quarter q+1's fragments are read while quarter q's MFMAs run (two
// 24-register sets; accumulators pinned to AGPRs by asm MFMAs, so 128 VGPRs
// suffice). The loop body is branch-free; the one barrier per K-tile comes
// before the last quarter:
//   tile t (stage s): q0: DMA A pieces of tile t+1 -> stage s^1, read q1, MFMAs q0
//                     q1: DMA B pieces, read q2, MFMAs q1;  q2: read q3, MFMAs q2
//                     q3: vmcnt(0) lgkmcnt(0) + barrier, read tile t+1's q0
//                         from stage s^1, MFMAs q3
// WAR: stage s^1 (tile t-1) was last read before tile t-1's barrier; RAW: tile
// t+1 is read only after tile t's barrier, its DMA has >= half a K-tile
// (~3.5 us at 2.38 GHz) to land. The last tile's DMA re-reads tile nk-1 into
// the idle stage (clamped, harmless).
// Measured (experiment id x_f32_256p, profiles/r3i_f32_256p_ab.jsonl, same
// process): 144.7 / 145.2 TF at 8k / 16k vs 149.5 / 150.0 for f32_256s and
// 151.9 / 152.0 for f32_t128x2 — slower: kept as the recorded negative result.
struct Frag32 {
  float a[8][2];  // [mi][e - e0]: A row k 4g + e of block mi (one b64 read per mi)
  float b[4][2];  // [ni][e - e0]
};

// Per-lane LDS byte offsets of one stage (opaque, so every read is base +
// immediate: a stage is 66,048 B, past ds_read's 16-bit offset): A block mi of
// half kb at a[kb] + mi * 2048 (the row swizzle (r >> 1) & 7 does not depend
// on mi); B element (k = 4 g + k', ni) at b + k' * B_PITCH + ni * 64.
struct StageBase {
  uint32_t a[2];
  uint32_t b;
};

template <int Q>
__device__ __forceinline__ void read_q(const char* smem, const StageBase& bs, Frag32& F) {
  constexpr int KB = Q >> 1, E0 = (Q & 1) * 2;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const float2 v = *(const float2*)(smem + bs.a[KB] + mi * 2048 + E0 * 4);
    F.a[mi][0] = v.x;
    F.a[mi][1] = v.y;
  }
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      F.b[ni][e] = *(const float*)(smem + bs.b + (KB * 16 + E0 + e) * B_PITCH + ni * 64);
}

// Accumulators pinned to AGPRs (inline asm on "+a" operands): the builtin form
// keeps them in VGPRs and spills at two waves per SIMD.
__device__ __forceinline__ void mfma_q(const Frag32& F, f32x4 (&acc)[8][4]) {
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0"
                     : "+a"(acc[mi][ni])
                     : "v"(F.b[ni][e]), "v"(F.a[mi][e]));
}

// DMA of K-tile `tile` into the stage at byte offset `so` (runtime): A pieces
// (8 rows each) or B pieces (one k-row each), 4 per wave.
template <bool B>
__device__ __forceinline__ void issue_half(const Ctx& c, int tile, uint32_t so) {
  if constexpr (!B) {
    const long long offA = (long long)tile * BK * 4;
    const u32x4 ra = make_rsrc(c.Ab + offA, c.a_bytes - offA);
#pragma unroll
    for (int h = 0; h < 4; ++h) dma16(ra, c.voffA[h], c.lds0 + so + (h * 8 + c.wu) * 8 * 128);
  } else {
    const long long offB = (long long)tile * BK * c.ldb4;
    const u32x4 rb = make_rsrc(c.Bb + offB, c.b_bytes - offB);
#pragma unroll
    for (int h = 0; h < 4; ++h) dma16(rb, c.voffB[h], c.lds0 + so + A_BYTES + (h * 8 + c.wu) * B_PITCH);
  }
}

__global__ void __launch_bounds__(NT, 2) gemm_f32_256p(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wu >> 2, wc = wu & 3;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda4 = a.lda * 4;
  c.ldb4 = a.ldb * 4;
  c.nk = a.K / BK;
  c.Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda) * 4;
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + n0) * 4;
  c.a_bytes = ((long long)(a.M - m0 - 1) * a.lda + a.K) * 4;
  c.b_bytes = ((long long)(a.kb - 1) * a.ldb + (a.N - n0)) * 4;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int r = (h * 8 + wu) * 8 + (lane >> 3);
    const int src_chunk = (lane & 7) ^ ((r >> 1) & 7);
    c.voffA[h] = (uint32_t)(r * c.lda4 + src_chunk * 16);
    const int k = h * 8 + wu;
    c.voffB[h] = (uint32_t)(k * c.ldb4 + lane * 16);
  }
  StageBase cur, nxt;
  {
    const int r = wr * 128 + l16;  // + 16 mi: same swizzle
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      uint32_t ao = (uint32_t)(r * 128 + (((kb * 4 + g) ^ ((r >> 1) & 7)) * 16));
      uint32_t an = ao + STAGE;
      asm volatile("" : "+v"(ao), "+v"(an));
      cur.a[kb] = ao;
      nxt.a[kb] = an;
    }
    uint32_t bo = (uint32_t)(A_BYTES + 4 * g * B_PITCH + (wc * 64 + l16) * 4);
    uint32_t bn = bo + STAGE;
    asm volatile("" : "+v"(bo), "+v"(bn));
    cur.b = bo;
    nxt.b = bn;
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = c.nk;
  issue_half<false>(c, 0, 0);
  issue_half<true>(c, 0, 0);
  tile_barrier();
  Frag32 F0, F1;
  read_q<0>(smem, cur, F0);
  for (int t = 0; t < nk; ++t) {
    const int td = t + 1 < nk ? t + 1 : nk - 1;
    const uint32_t so = (uint32_t)((t + 1) & 1) * STAGE;
    issue_half<false>(c, td, so);
    read_q<1>(smem, cur, F1);
    mfma_q(F0, acc);
    issue_half<true>(c, td, so);
    read_q<2>(smem, cur, F0);
    mfma_q(F1, acc);
    read_q<3>(smem, cur, F1);
    mfma_q(F0, acc);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    read_q<0>(smem, nxt, F0);
    mfma_q(F1, acc);
    const StageBase tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  // Every wave done with the stages before the epilogue reuses LDS; the nops
  // give the last asm MFMAs time to write their AGPRs (invisible to hipcc's
  // hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_barrier" ::: "memory");

  char* Cb = (char*)a.C + (long long)bz * a.sC * 4;
  char* ebuf = smem + wu * epi_buf_f32<4>();
  const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    if (interior)
      store_block16_f32<false, 4>(ebuf, acc[mi], Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                  n0 + wc * 64, a.M, a.N, lane);
    else
      store_block16_f32<true, 4>(ebuf, acc[mi], Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                 n0 + wc * 64, a.M, a.N, lane);
  }
}

}  // namespace kf32

bool gemm_f32_256_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (a.K % 32 != 0 || a.K <= 0 || a.N % 4 != 0 || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 4 || a.ldb % 4 || a.ldc % 4) return false;
  if (a.batch > 1 && (a.sA % 4 || a.sB % 4 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 16) return false;
  // 32-bit per-lane DMA offsets: 255 rows * lda and 31 rows * ldb.
  if ((long long)256 * a.lda * 4 >= (1LL << 31) || (long long)32 * a.ldb * 4 >= (1LL << 31))
    return false;
  return true;
}

hipError_t gemm_f32_256_launch(GemmArgs a, int variant, hipStream_t stream) {
  a.tiles_m = (a.M + kf32::BM - 1) / kf32::BM;
  a.tiles_n = (a.N + kf32::BN - 1) / kf32::BN;
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const long long nblocks = (long long)a.tiles_m * a.tiles_n * a.batch;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblocks), block(kf32::NT);
  if (variant == 1) {  // the shipping exact-fp32 kernel (kF32_256s)
    hipLaunchKernelGGL(kf32::gemm_f32_256<true>, grid, block, 0, stream, a);
    return hipGetLastError();
  }
#ifdef PDMB_EXPERIMENTS
  if (variant == 9)
    hipLaunchKernelGGL((kf32::gemm_f32_256<false, true>), grid, block, 0, stream, a);
  else if (variant == 10)  // kF32_256sDirect: the shipping kernel with direct C stores
    hipLaunchKernelGGL((kf32::gemm_f32_256<true, false, false>), grid, block, 0, stream, a);
  else if (variant == 11)  // kF32_256p: software-pipelined fragments, mid-tile barrier
    hipLaunchKernelGGL(kf32::gemm_f32_256p, grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL(kf32::gemm_f32_256<false>, grid, block, 0, stream, a);
  return hipGetLastError();
#else
  return hipErrorInvalidValue;  // experiment variants are not built
#endif
}

}  // namespace pdmb
