// gemm_f32_w4.hip — exact-fp32 C = A @ B (row-major NN) on v_mfma_f32_16x16x4_f32
// with W4's structure: 4 waves per 256x256 workgroup, one per SIMD, each
// owning 128x128 outputs in 256 AGPR accumulators.
//
// Why: gemm_f32_256.hip (8 waves x 128x64, 2 waves per SIMD) reaches 148 TF at
// 16k, 95 % MFMA busy at 2.38 GHz — fp32 MFMA is not power-bound — while
// hipBLASLt's one-wave-per-SIMD 128x128-per-wave kernel is 98.7 % busy
// (154 TF, profiles/r1_fp32_ablation.md). Round 1 could not build that shape:
// hipcc spilled and broke the accumulator chains. Here, as in gemm_w4.hip,
// the MFMAs are inline asm on "+a" accumulator operands, so the 256
// accumulators stay in AGPRs and the operands in VGPRs.
//
// Layout (gemm_f32_256.hip's conflict-free images, unchanged):
//  * A [256 rows][32 fp32 = 128 B], 16-B chunk c of row r at c ^ ((r >> 1) & 7);
//    one ds_read_b128 gives a lane 4 consecutive k of its row, so MFMA e of a
//    16-k block uses k = 16 kb + 4 g + e in lane group g (a k-permutation).
//  * B [32 k][260 fp32] (1040-B rows; the pad puts k-rows 4 apart on opposite
//    bank halves): the matching B element is ds_read_b32 of B[16 kb + 4 g + e][col].
//  * 2 stages x 66,048 B, filled by LDS-DMA (buffer_load ... lds): per K-tile
//    32 A pieces (8 rows x 128 B) + 32 B pieces (one k-row) = 16 per wave.
// Schedule per K-tile t (stage s = t & 1): 512 MFMAs (2 halves x 4 e x 8 m
// x 8 n, 32 cycles each = ~7 us) from registers; during half 0 the wave
// reads half 1's fragments of t; then ONE barrier mid-tile (vmcnt(0): tile
// t+1 landed; lgkmcnt(0): done reading s); during half 1 it refills s with
// tile t+2 (16 DMA pieces, so each tile has a whole tile of flight) and reads
// half 0 of tile t+1 from s ^ 1. No wave waits at a tile boundary and no LDS
// read latency is exposed (round 2's first version waited at the top of each
// tile and ran 1 % behind f32_256s).
// Operands swapped (B element as the MFMA's A) so each lane owns 4
// consecutive output columns; C leaves through LDS as whole rows. Edges: the DMA descriptors'
// extents read zeros past M / N / K, the stores are masked, so any M and
// N % 4 == 0 runs here (the host checks K % 32, alignment).
#include "api.h"
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace kf32w4 {

constexpr int BM = 256, BN = 256, BK = 32, NT = 256;
constexpr int A_BYTES = BM * BK * 4;      // 32 KiB
constexpr int B_PITCH = (BN + 4) * 4;     // 1040 B per k-row
constexpr int B_BYTES = BK * B_PITCH;     // 33,280 B
constexpr int STAGE = A_BYTES + B_BYTES;  // 66,048 B (16-B multiple)
constexpr int LDS_BYTES = 2 * STAGE;      // 132,096 B

__device__ __forceinline__ void mfma(f32x4& acc, float b, float a) {
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// LDS-DMA with a scalar offset; M0 is clobbered (declared), not saved.
__device__ __forceinline__ void dma16_m0(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  asm volatile(
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
      : "memory", "m0");
}

struct Ctx {
  const char* Ab;
  const char* Bb;
  long long a_bytes, b_bytes;
  int lda4, ldb4, nk, wu;
  uint32_t voffA, voffB;
  uint32_t lds0;
};

// Fragments of one 16-k block: A rows (4 k each) and B. BV (b128 B reads):
// b4[e][h] = B[k][wc * 128 + 64 h + 4 l16 + j] for j = 0..3 — MFMA ni = 4 h + j
// of the lane's column group uses output column 64 h + 16 g + 4 r + j (a
// column permutation the epilogue undoes), so one read feeds four MFMAs.
// Else b[ni][e] = B[k][16 ni + l16], one b32 read per MFMA operand.
template <bool BV>
struct Half {
  f32x4 a[8];
  float b[8][4];
};
template <>
struct Half<true> {
  f32x4 a[8];
  f32x4 b4[4][2];
};

// DMA piece h (0..15) of K-tile `tile` into stage `stg`: h < 8: A rows
// (h*4 + wu)*8 + [0,8) (8 x 128 B); h >= 8: B k-row (h-8)*4 + wu (1 KiB).
// A's swizzle depends on (r >> 1) & 7, which the h*32-row offset keeps.
__device__ __forceinline__ void issue_piece(const Ctx& c, u32x4 ra, u32x4 rb, int stg, int h) {
  if (h < 8) {
    dma16_m0(ra, c.voffA, (uint32_t)(h * 32 * c.lda4),
             c.lds0 + stg * STAGE + ((h * 4 + c.wu) * 8) * 128);
  } else {
    const int kr = (h - 8) * 4 + c.wu;
    dma16_m0(rb, c.voffB, (uint32_t)((h - 8) * 4 * c.ldb4), c.lds0 + stg * STAGE + A_BYTES + kr * B_PITCH);
  }
}

// Fragment reads of 16-k block kb from stage stg. mi / ni index the wave's
// 8 row blocks / 8 column blocks; each is issued separately so the schedule
// can place it in an MFMA gap.
__device__ __forceinline__ f32x4 read_a(const char* smem, int stg, int kb, int mi, int wr, int l16,
                                        int g) {
  const int r = wr * 128 + mi * 16 + l16;
  const int ch = (kb * 4 + g) ^ ((r >> 1) & 7);
  return *(const f32x4*)(smem + stg * STAGE + r * 128 + ch * 16);
}
__device__ __forceinline__ float read_b(const char* smem, int stg, int kb, int ni, int e, int wc,
                                        int l16, int g) {
  const int k = kb * 16 + 4 * g + e;
  const int col = wc * 128 + ni * 16 + l16;
  return *(const float*)(smem + stg * STAGE + A_BYTES + k * B_PITCH + col * 4);
}
__device__ __forceinline__ f32x4 read_b4(const char* smem, int stg, int kb, int h, int e, int wc,
                                         int l16, int g) {
  const int k = kb * 16 + 4 * g + e;
  const int col = wc * 128 + h * 64 + 4 * l16;
  return *(const f32x4*)(smem + stg * STAGE + A_BYTES + k * B_PITCH + col * 4);
}

// One 16-k half: 256 MFMAs from `cur`; in their gaps read the other half's
// fragments into `nxt` (kb_next >= 0) and issue DMA pieces [p0, p0 + np) of
// the next tile (one per 4 MFMAs from the start).
template <bool BV>
__device__ __forceinline__ void half_step(const Ctx& c, const char* smem, f32x4 (&acc)[8][8],
                                          const Half<BV>& cur, Half<BV>& nxt, int stg_rd, int kb_next,
                                          int wr, int wc, int l16, int g, u32x4 ra, u32x4 rb,
                                          int stg_dma, int p0, int np) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) {
        const int gap = (e * 8 + mi) * 8 + ni;  // 0..255
        if constexpr (BV)
          mfma(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e]);
        else
          mfma(acc[mi][ni], cur.b[ni][e], cur.a[mi][e]);
        if (gap % 4 == 3 && gap / 4 < np) {
          issue_piece(c, ra, rb, stg_dma, p0 + gap / 4);
        } else if (kb_next >= 0 && gap % 4 == 1 && gap / 4 < (BV ? 16 : 40)) {
          // 8 A rows (b128) then the B reads (BV: 8 b128; else 32 b32), one per 4 MFMAs
          const int q = gap / 4;
          if (q < 8) {
            nxt.a[q] = read_a(smem, stg_rd, kb_next, q, wr, l16, g);
          } else if constexpr (BV) {
            const int e2 = (q - 8) >> 1, h2 = (q - 8) & 1;
            nxt.b4[e2][h2] = read_b4(smem, stg_rd, kb_next, h2, e2, wc, l16, g);
          } else {
            const int e2 = (q - 8) >> 3, ni2 = (q - 8) & 7;
            nxt.b[ni2][e2] = read_b(smem, stg_rd, kb_next, ni2, e2, wc, l16, g);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
}

// BV: b128 B reads (column-permuted MFMAs) instead of b32 ones.
// NB (experiments, round 6: kF32W4NB): a branch-free K-loop. The shipping loop
// skips the last two tiles' DMA pieces and the last tile's fragment reads
// with runtime conditions: hipcc puts a branch around each of the 16 DMA
// pieces and the reads, 32 branches per 512 MFMAs (PMC: 0.067 branches per
// MFMA against hipBLASLt's 0.002, 95.4 % MFMA busy against its 98.9 %,
// profiles/r8h_*). NB always issues all 16 pieces (the last two tiles
// re-read their own K-tile into the stage they just released: harmless, as
// W4's clamped tail DMAs) and always reads the next fragments (the last
// tile's are never used).
template <bool BV, bool NB = false>
__global__ void __launch_bounds__(NT, 1) gemm_f32_w4(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  // Split-K (under-filled grids: matrix_parallel's fp32 column shards): the
  // grid's batch is batch x S with the slice innermost, as in gemm_w4.hip;
  // slice s runs K-tiles [s * kt_per, +kt_per) and the S slices of a tile
  // meet in the epilogue (splitk.h).
  int slice = 0;
  if (a.splitk > 1) {
    slice = bz % a.splitk;
    bz /= a.splitk;
  }
  const int kt0 = slice * a.kt_per;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda4 = a.lda * 4;
  c.ldb4 = a.ldb * 4;
  c.nk = a.splitk > 1 ? min(a.kt_per, a.K / BK - kt0) : a.K / BK;
  const long long k0 = (long long)kt0 * BK;
  c.Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda + k0) * 4;
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + k0 * a.ldb + n0) * 4;
  c.a_bytes = ((long long)(a.M - m0 - 1) * a.lda + (a.K - k0)) * 4;
  c.b_bytes = ((long long)(a.kb - k0 - 1) * a.ldb + (a.N - n0)) * 4;
  {
    const int r = wu * 8 + (lane >> 3);  // row of A piece 0
    c.voffA = (uint32_t)(r * c.lda4 + (((lane & 7) ^ ((r >> 1) & 7)) * 16));
    c.voffB = (uint32_t)(wu * c.ldb4 + lane * 16);  // k-row wu of piece 8
  }
  auto rsrc_a = [&](int tile) {
    const long long off = (long long)tile * BK * 4;
    return make_rsrc(c.Ab + off, c.a_bytes - off);
  };
  auto rsrc_b = [&](int tile) {
    const long long off = (long long)tile * BK * c.ldb4;
    return make_rsrc(c.Bb + off, c.b_bytes - off);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue: tiles 0 and 1 into stages 0 and 1; tile 0 landed everywhere;
  // half 0 of tile 0 to registers.
  const int nk = c.nk;
  {
    const u32x4 ra = rsrc_a(0), rb = rsrc_b(0);
#pragma unroll
    for (int h = 0; h < 16; ++h) issue_piece(c, ra, rb, 0, h);
  }
  if (nk > 1) {
    const u32x4 ra = rsrc_a(1), rb = rsrc_b(1);
#pragma unroll
    for (int h = 0; h < 16; ++h) issue_piece(c, ra, rb, 1, h);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  Half<BV> h0, h1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // in the order the MFMAs consume them
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
      if (e == 0) h0.a[mi] = read_a(smem, 0, 0, mi, wr, l16, g);
    if constexpr (BV) {
#pragma unroll
      for (int h = 0; h < 2; ++h) h0.b4[e][h] = read_b4(smem, 0, 0, h, e, wc, l16, g);
    } else {
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) h0.b[ni][e] = read_b(smem, 0, 0, ni, e, wc, l16, g);
    }
  }
  // K-tile t (stage s = t & 1; tile t+1 in s ^ 1 was issued a tile ago):
  //   half 0: MFMAs from h0 | read half 1 of t from s into h1
  //   mid-tile: vmcnt(0) (t+1 landed) lgkmcnt(0) (this wave done reading s),
  //             s_barrier — so nobody waits at the top of a tile
  //   half 1: MFMAs from h1 | DMA tile t+2 into s | read half 0 of t+1 from
  //           s ^ 1 into h0
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const bool more = t + 1 < nk, more2 = t + 2 < nk;
    const int td = more2 ? t + 2 : t;  // the last two tiles issue no DMA (np = 0; NB: a re-read)
    const u32x4 ra = rsrc_a(td), rb = rsrc_b(td);
    half_step(c, smem, acc, h0, h1, s, 1, wr, wc, l16, g, ra, rb, s, 0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NB)
      half_step(c, smem, acc, h1, h0, s ^ 1, 0, wr, wc, l16, g, ra, rb, s, 0, 16);
    else
      half_step(c, smem, acc, h1, h0, s ^ 1, more ? 0 : -1, wr, wc, l16, g, ra, rb, s,
                0, more2 ? 16 : 0);
  }
  // Give the last MFMAs time to write their AGPRs (asm MFMAs are invisible to
  // hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  // Split-K: only the last slice of a tile to arrive writes C, summing the
  // slices' fp32 slots in slice order (bitwise reproducible).
  SplitSlots sl;
  const bool split = a.splitk > 1;
  if (split && !splitk_meet<8, 8, NT>(a, smem, ((long long)bz * a.tiles_m + tm) * a.tiles_n + tn, slice,
                                      acc, sl))
    return;
  // Epilogue through LDS as whole 512-B rows, non-temporal (common.h
  // store_block16_f32), once every wave is done with the stages.
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  char* Cb = (char*)a.C + (long long)bz * a.sC * 4;
  char* ebuf = smem + 1024 + wu * epi_buf_f32<8>();  // past splitk_meet's ticket word
  const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    f32x4 v[8];
    if (!split) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[mi][j];
    } else {
      splitk_row<8, 8, NT>(a, sl, slice, mi, acc, v);
    }
    if constexpr (BV) {  // v[4 h + j][r] is column 64 h + 16 g + 4 r + j: regroup by r
      f32x4 w[8];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          w[4 * h + r] = f32x4{v[4 * h][r], v[4 * h + 1][r], v[4 * h + 2][r], v[4 * h + 3][r]};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = w[j];
    }
    if (interior)
      store_block16_f32<false, 8, BV>(ebuf, v, Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                      n0 + wc * 128, a.M, a.N, lane);
    else
      store_block16_f32<true, 8, BV>(ebuf, v, Cb, (long long)a.ldc * 4, m0 + wr * 128 + mi * 16,
                                     n0 + wc * 128, a.M, a.N, lane);
  }
}

}  // namespace kf32w4

// a.splitk > 1: split-K with a.part / a.flags (gemm_dispatch.cpp f32_split).
// variant 0: the shipping kernel (b128 B reads); 1 (experiment builds): b32 B reads.
hipError_t gemm_f32_w4_launch(GemmArgs a, hipStream_t stream, int variant) {
  a.tiles_m = (a.M + kf32w4::BM - 1) / kf32w4::BM;
  a.tiles_n = (a.N + kf32w4::BN - 1) / kf32w4::BN;
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const int S = a.splitk > 1 ? a.splitk : 1;
  if (S > 1) {
    const int nk = a.K / kf32w4::BK;
    a.kt_per = (nk + S - 1) / S;
    if ((S - 1) * a.kt_per >= nk || !a.part || !a.flags ||
        (long long)a.tiles_m * a.tiles_n * a.batch > kMaxSplitTiles)
      return hipErrorInvalidValue;  // every slice must own >= 1 K-tile
  } else {
    a.splitk = 1;
  }
  const long long nblocks = (long long)a.tiles_m * a.tiles_n * a.batch * S;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
#ifdef PDMB_EXPERIMENTS
  if (variant == 1) {
    hipLaunchKernelGGL(kf32w4::gemm_f32_w4<false>, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 2) {  // kF32W4NB: the branch-free K-loop
    hipLaunchKernelGGL((kf32w4::gemm_f32_w4<true, true>), dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream,
                       a);
    return hipGetLastError();
  }
#endif
  if (variant != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kf32w4::gemm_f32_w4<true>, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace pdmb
