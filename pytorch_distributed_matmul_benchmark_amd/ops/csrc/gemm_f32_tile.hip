// gemm_f32_tile.hip — exact-fp32 C = A @ B (row-major NN) on v_mfma_f32_16x16x4_f32
// with a 128x128 output tile: the fp32 member of the tile family (gemm_tile.hip)
// for grids that under-fill the 256 CUs with 256x256 tiles.
//
// Why: matrix_parallel's fp32 column shards at the reference's default sizes
// (matmul_scaling_benchmark.py:179-188 at :351-352; --dtype float32 is a
// reference choice, matmul_benchmark.py:163-174) are 4096 x {2048, 1024, 512} x
// 4096 = 128 / 64 / 32 256x256 tiles, and 2048^3 has 64. gemm_f32_w4.hip fills
// them only by splitting K over 256 KiB fp32 slabs per slice (95-120 TF vs
// hipBLASLt 127-140). A 128x128 tile gives 4x the workgroups, a
// 64 KiB slab per slice, and needs no split at all on the 64-tile shapes.
//
// Structure (W4 / tile-family idioms):
//  * 4 waves as 2 x 2, one per SIMD, each owning 64x64 outputs: 4 x 4 MFMA
//    16x16 blocks, 64 fp32 accumulators in AGPRs (asm MFMAs on "+a" operands);
//    operands swapped (the B element is the MFMA's A) so a lane owns 4
//    consecutive output columns and C leaves through LDS as whole rows.
//  * K-tile = 32 (128 B of A per row). LDS images per stage (32 KiB):
//      A [128 rows][128 B], 16-B chunk c of row r at c ^ ((r >> 1) & 7)
//        (gemm_f32_w4.hip's image; one ds_read_b128 = 4 consecutive k);
//      B [32 k][512 B], UNPADDED so one 64-lane LDS-DMA fills two k-rows; for
//        the b32 reads (A/B build) 16-B chunk c of k-row k sits at c ^ 4 *
//        ((k >> 2) & 3) (a wave's four B pieces all have (k >> 2) & 3 == wave
//        id, so the swizzle is one per-lane source offset) and a fragment read
//        (16 columns x k = 16 kb + 4 g + e over the lane groups g) hits chunk
//        groups 4 (q ^ g): all 64 banks once; the shipping b128 reads use the
//        unswizzled image (kBSwz: conflict-free for ds_read_b128's lane groups).
//  * 4-stage ring filled by LDS-DMA (buffer_load ... lds), 8 x 1 KiB pieces
//    per wave per K-tile; one barrier per K-tile (s_waitcnt vmcnt(16): tile
//    t+1 landed, t+2 / t+3 may fly; lgkmcnt(0): this wave's reads of t's
//    stage done). Tile t+1's fragments are read during t's 128 MFMAs into a
//    second register set; every load sits in an MFMA gap (Sched).
//  * Split-K over K-tile ranges with the in-launch combine of splitk.h.
// Edges: A rows past M and B past its extent read zeros through the DMA
// descriptors; B columns past N feed only C columns the masked epilogue drops
// (N % 4 == 0; the host checks K % 32, lda / ldb % 4, 16-B alignment).
#include "api.h"
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace kf32t {

constexpr int BN = 128, BK = 32, NT = 256;
constexpr int NB = 4;                         // 16x16 column blocks per wave
constexpr int B_BYTES = BK * BN * 4;          // 16 KiB
// Tile rows: 128 (kF32T128 / kF32T128x2) or 64 (kF32T64, round 5: a 64x128
// tile, 4 waves x 32x64). The B image, its DMA pieces and the b128 B reads
// are the same for both; A has BM / 32 pieces per wave and MB = BM / 32 row
// blocks per wave.
template <int BM_>
struct Sh {
  static constexpr int BM = BM_;
  static_assert(BM == 64 || BM == 128, "tile rows");
  static constexpr int MB = BM / 32;                  // 16x16 row blocks per wave
  static constexpr int A_BYTES = BM * BK * 4;         // 16 / 8 KiB
  static constexpr int STAGE = A_BYTES + B_BYTES;     // 32 / 24 KiB
  static constexpr int PA = BM / 32;                  // A DMA pieces per wave per K-tile
  static constexpr int P = PA + 4;                    // + 4 B pieces
  static constexpr int G = 2 * 4 * MB * NB;           // MFMAs per K-tile per wave (kb, e, mi, ni)
};
typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
typedef __attribute__((address_space(3))) float lds_f32;

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

// LN (experiments, round 6): the DMA piece fused with its gap's MFMA — M0 =
// an SGPR stage base + the piece's constant LDS offset in one SALU, and the
// MFMA is the one wait state the M0 write needs before the LDS-DMA (no s_nop;
// gemm_f32_w4.hip mfma_dma, which took the W4 loop from 97.0 to 98.3 % MFMA
// busy, profiles/r8lq_fp32_lean_stream.md).
__device__ __forceinline__ void mfma_dma(f32x4& acc, float b, float a, u32x4 rsrc, uint32_t voff, uint32_t soff,
                                         uint32_t base, int imm) {
  asm volatile(
      "s_add_u32 m0, %5, %6\n\t"
      "v_mfma_f32_16x16x4_f32 %0, %1, %2, %0\n\t"
      "buffer_load_dwordx4 %3, %4, %7 offen lds"
      : "+a"(acc)
      : "v"(b), "v"(a), "v"(voff), "s"(rsrc), "s"(base), "i"(imm), "s"(soff)
      : "memory", "m0", "scc");
}

template <int N>
__device__ __forceinline__ void wait_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Item schedule of one K-tile (gemm_tile.hip Sched, fp32 classes): 8 A
// fragment reads (b128: 2 kb x 4 mi), the B reads (BV: 8 b128, 2 kb x 4 e;
// else 32 b32, 2 kb x 4 ni x 4 e) and 8 DMA pieces spread Bresenham-style
// over the 128 MFMA gaps, at most one per gap. Encoding: 0 none; 1 + piece;
// 100 + B read q; 200 + A read q.
template <class H, bool BV>
struct Sched {
  static constexpr int G = H::G;
  int item[G];
  constexpr Sched() : item() {
    const int T[3] = {BV ? 8 : 32, 2 * H::MB, H::P};
    int n[3] = {0, 0, 0};
    for (int g = 0; g < G; ++g) {
      int best = -1, bd = 0;
      for (int k = 0; k < 3; ++k) {
        const int d = T[k] * (g + 1) - n[k] * G;
        if (n[k] < T[k] && d > bd) {
          bd = d;
          best = k;
        }
      }
      if (best == 0) item[g] = 100 + n[0]++;
      else if (best == 1) item[g] = 200 + n[1]++;
      else if (best == 2) item[g] = 1 + n[2]++;
      else item[g] = 0;
    }
  }
};

// B image chunk swizzle per k-group ((k >> 2) & 3): 4 for the b32 reads (k-
// strided lanes land on distinct bank quads, above), 0 for the b128 reads.
// ds_read_b128 is serviced in four 16-lane groups, {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md, LDS table): group 0 holds
// lanes g = 0, l16 in {0-3, 12-15} and g = 1, l16 in {4-11}. A lane's bank quad
// is (chunk mod 16) = l16 ^ swz(g) (k-rows are 512 B, a whole number of bank
// rows), so swz = 4 g made both halves of every group hit the same 8 quads —
// 2-way conflicts on every B read (PMC: 1.08e9 conflict cycles of 3.24e9 at
// 16k, profiles/r3r_pmc_fp32_t128x2.md); swz = 0 gives 16 distinct quads.
template <bool BV>
constexpr int kBSwz = BV ? 0 : 4;

// One K-tile's fragments: A rows (4 k each) and B. BV (b128 B reads): b4[kb][e]
// holds B[k][c0 + 4 l16 + ni] for ni = 0..3 — MFMA ni of the lane's column
// group uses output column 16 g + 4 r + ni of the wave's 64 (a column
// permutation undone by the epilogue), so one read feeds four MFMAs. Else
// b[kb][ni][e] = B[k][16 ni + l16] (one b32 read per MFMA operand).
template <int MB, bool BV>
struct Frag {
  f32x4 a[2][MB];      // [kb][mi]
  float b[2][NB][4];   // [kb][ni][e]
};
template <int MB>
struct Frag<MB, true> {
  f32x4 a[2][MB];      // [kb][mi]
  f32x4 b4[2][4];      // [kb][e], lanes ni
};

struct Ctx {
  u32x4 ra;             // A descriptor at this slice's first K
  u32x4 rb0;            // LN: B descriptor at this slice's first K (built once)
  const char* Bb;       // B at this slice's first K row, column n0
  long long b_bytes;
  int lda4, ldb4, nk, wu;
  uint32_t voffA, voffB;
  uint32_t lds0;
  // Per-lane fragment bases in stage 0 (the rest of each offset is an
  // immediate): A block mi of half kb at abase[kb] + mi * 2048 (the row
  // swizzle (r >> 1) & 7 does not depend on mi); B element (kb, ni, e) at
  // bbase[ni] + kb * 8192 + e * 512 (k = 16 kb + 4 g + e; g is in the base);
  // BV: B chunk (kb, e) at bbase[0] + kb * 8192 + e * 512.
  uint32_t abase[2];
  uint32_t bbase[NB];
};

__device__ __forceinline__ u32x4 b_rsrc(const Ctx& c, int tile) {
  const long long off = (long long)tile * BK * c.ldb4;
  return make_rsrc(c.Bb + off, c.b_bytes - off);
}

// DMA piece h (0..P-1) of K-tile `tile` into the stage at byte offset `so`.
// h < PA: A rows 32 h + 8 wu + [0, 8) (8 x 128 B). h >= PA: B k-rows k0,
// k0 + 1 with k0 = 16 (j >> 1) + 4 wu + 2 (j & 1), j = h - PA (2 x 512 B).
template <class H>
__device__ __forceinline__ void issue_piece(const Ctx& c, u32x4 rb, uint32_t so, int tile, int h) {
  if (h < H::PA) {
    dma16_m0(c.ra, c.voffA, (uint32_t)tile * (BK * 4) + (uint32_t)(h * 32 * c.lda4),
             c.lds0 + so + (h * 32 + c.wu * 8) * 128);
  } else {
    const int j = h - H::PA;
    const int k0 = 16 * (j >> 1) + 4 * c.wu + 2 * (j & 1);
    dma16_m0(rb, c.voffB, (uint32_t)(k0 * c.ldb4), c.lds0 + so + H::A_BYTES + k0 * 512);
  }
}

// One K-tile: G MFMAs on `cur` (tile t), reading tile t+1's fragments into
// `nxt` from stage `sn`, DMA of tile t + NS into stage `sc`.
// LN (experiments): the slice's descriptors are built once and the K-tile's
// offset rides in the voffsets (one VALU add each) instead of a new B
// descriptor per K-tile (~15 SALU: a 64-bit multiply, the extent, clamps), and
// each piece issues as mfma_dma.
template <class H, int NS, bool BV, bool LN = false>
__device__ __forceinline__ void ktile(const Ctx& c, const char* smem, int t, uint32_t sc, uint32_t sn,
                                      f32x4 (&acc)[H::MB][NB], const Frag<H::MB, BV>& cur,
                                      Frag<H::MB, BV>& nxt) {
  constexpr int MB = H::MB, G = H::G;
  constexpr Sched<H, BV> S{};
  const int td = t + NS < c.nk ? t + NS : c.nk - 1;  // clamped tail DMAs (harmless re-reads)
  const u32x4 rb = LN ? c.rb0 : b_rsrc(c, td);
  // LN: this K-tile's voffsets and the stage's M0 bases (A pieces at h * 4096 +
  // wu * 1024, B k-row pairs at A_BYTES + (16 (j >> 1) + 2 (j & 1)) * 512 + wu * 2048)
  const uint32_t vA = c.voffA + (uint32_t)td * (BK * 4), vB = c.voffB + (uint32_t)td * (uint32_t)(BK * c.ldb4);
  const uint32_t mA = c.lds0 + sc + (uint32_t)c.wu * 1024, mB = c.lds0 + sc + (uint32_t)c.wu * 2048;
  wait_lgkm_barrier<H::P * (NS - 2)>();
  __builtin_amdgcn_sched_barrier(0);
  uint32_t ab[2], bb[NB];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) ab[kb] = c.abase[kb] + sn;
#pragma unroll
  for (int ni = 0; ni < NB; ++ni) bb[ni] = c.bbase[ni] + sn;
  auto step = [&](const int gap) __attribute__((always_inline)) {
    const int ni = gap % NB, mi = (gap / NB) % MB, e = (gap / (NB * MB)) % 4, kb = gap / (NB * MB * 4);
    const int it = S.item[gap];
    if constexpr (LN) {
      static_assert(BV, "LN: the b128 kernel");
      if (it >= 1 && it < 100) {  // the gap's MFMA and DMA piece h in one asm block
        const int h = it - 1;
        if (h < H::PA) {
          mfma_dma(acc[mi][ni], cur.b4[kb][e][ni], cur.a[kb][mi][e], c.ra, vA, (uint32_t)(h * 32 * c.lda4), mA,
                   h * 4096);
        } else {
          const int j = h - H::PA, kr = 16 * (j >> 1) + 2 * (j & 1);
          mfma_dma(acc[mi][ni], cur.b4[kb][e][ni], cur.a[kb][mi][e], rb, vB, (uint32_t)((kr + 4 * c.wu) * c.ldb4),
                   mB, H::A_BYTES + kr * 512);
        }
        __builtin_amdgcn_sched_barrier(0);
        return;
      }
    }
    if constexpr (BV)
      mfma(acc[mi][ni], cur.b4[kb][e][ni], cur.a[kb][mi][e]);
    else
      mfma(acc[mi][ni], cur.b[kb][ni][e], cur.a[kb][mi][e]);
    if (it >= 200) {
      const int q = it - 200, qk = q / MB, qm = q % MB;
      nxt.a[qk][qm] = *(const lds_f32x4*)(smem + ab[qk] + qm * 2048);
    } else if (it >= 100) {
      if constexpr (BV) {
        const int q = it - 100, qk = q >> 2, qe = q & 3;
        nxt.b4[qk][qe] = *(const lds_f32x4*)(smem + bb[0] + qk * 8192 + qe * 512);
      } else {
        const int q = it - 100, qk = q >> 4, qn = (q >> 2) & 3, qe = q & 3;
        nxt.b[qk][qn][qe] = *(const lds_f32*)(smem + bb[qn] + qk * 8192 + qe * 512);
      }
    } else if (it >= 1) {
      issue_piece<H>(c, rb, sc, td, it - 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (LN) {
    // loops of 32 gaps: one loop of 128 fused gaps passes the unroller's size
    // limit, and a rolled loop cannot give the pieces constant M0 offsets
    // (the "i" operands)
#pragma unroll
    for (int gap = 0; gap < 32; ++gap) step(gap);
#pragma unroll
    for (int gap = 32; gap < 64; ++gap) step(gap);
    if constexpr (G == 128) {
#pragma unroll
      for (int gap = 64; gap < 96; ++gap) step(gap);
#pragma unroll
      for (int gap = 96; gap < 128; ++gap) step(gap);
    }
  } else {
#pragma unroll
    for (int gap = 0; gap < G; ++gap) step(gap);
  }
}

// NS: LDS stages (4: 128 KiB, one workgroup per CU; 2: 64 KiB, two per CU).
// BV: b128 B reads (column-permuted MFMAs) instead of b32 ones.
// BM: tile rows (128, or 64 for kF32T64: 4 x 24 KiB stages).
template <int NS, bool BV, int BM = 128, bool LN = false>
__global__ void __launch_bounds__(NT, NS == 2 ? 2 : 1) gemm_f32_t128(GemmArgs a) {
  using H = Sh<BM>;
  constexpr int MB = H::MB, P = H::P, STAGE = H::STAGE;
  constexpr int LDS_BYTES = NS * STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  int slice = 0;  // split-K: grid batch = batch x S, slice innermost (as W4)
  long long meet_tile;
  if (a.tile_span > 0) {
    // the split tail of a tile-range plan (gemm_dispatch.cpp tail_plan): local
    // tile b % span of [tile_base, +span) in map_tile's order, slice b / span
    const int local = blockIdx.x % a.tile_span;
    slice = blockIdx.x / a.tile_span;
    map_tile(a, a.tile_base + local, bz, tm, tn);
    meet_tile = local;
  } else {
    map_tile(a, blockIdx.x, bz, tm, tn);
    if (a.splitk > 1) {
      slice = bz % a.splitk;
      bz /= a.splitk;
    }
    meet_tile = ((long long)bz * a.tiles_m + tm) * a.tiles_n + tn;
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
  {
    const int nk_all = a.K / BK;
    c.nk = a.splitk > 1 ? min(a.kt_per, nk_all - kt0) : nk_all;
  }
  const long long k0 = (long long)kt0 * BK;
  c.ra = make_rsrc((const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda + k0) * 4,
                   ((long long)(a.M - m0 - 1) * a.lda + (a.K - k0)) * 4);
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + k0 * a.ldb + n0) * 4;
  c.b_bytes = ((long long)(a.kb - k0 - 1) * a.ldb + (a.N - n0)) * 4;
  if constexpr (LN) c.rb0 = b_rsrc(c, 0);
  {
    const int r = wu * 8 + (lane >> 3);  // row of A piece 0 (the swizzle is 32-row periodic)
    c.voffA = (uint32_t)(r * c.lda4 + (((lane & 7) ^ ((r >> 1) & 7)) * 16));
    // B: lanes 0-31 row k0, 32-63 row k0 + 1; LDS chunk (lane & 31) holds
    // global chunk (lane & 31) ^ 4 wu ((k0 >> 2) & 3 == wu for every piece) for
    // the b32 reads, and global chunk lane & 31 (no swizzle) for the b128 reads
    // (see kBSwz)
    c.voffB = (uint32_t)((lane >> 5) * c.ldb4 + (((lane & 31) ^ (kBSwz<BV> * wu)) * 16));
    const int rr = wr * (BM / 2) + l16;  // + 16 mi: same swizzle
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      uint32_t ao = (uint32_t)(rr * 128 + (((kb * 4 + g) ^ ((rr >> 1) & 7)) * 16));
      asm volatile("" : "+v"(ao));  // opaque: one base VGPR each
      c.abase[kb] = ao;
    }
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {  // k = 16 kb + 4 g + e: (k >> 2) & 3 == g
      // BV: chunk wc * 16 + l16 (columns wc * 64 + 4 l16 .. + 3), bbase[0] only
      const int col = BV ? wc * 64 + 4 * l16 : wc * 64 + ni * 16 + l16;
      const int ch = (col >> 2) ^ (kBSwz<BV> * g);
      uint32_t bo = (uint32_t)(H::A_BYTES + 4 * g * 512 + ch * 16 + (col & 3) * 4);
      asm volatile("" : "+v"(bo));
      c.bbase[ni] = bo;
      if (BV) break;
    }
  }

  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue: tiles 0 .. NS-1 into stages 0 .. NS-1 (clamped), wait for tile
  // 0 everywhere, read its fragments.
  const int nk = c.nk;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int tl = st < nk ? st : nk - 1;
    const u32x4 rb = b_rsrc(c, tl);
#pragma unroll
    for (int h = 0; h < P; ++h) issue_piece<H>(c, rb, st * STAGE, tl, h);
  }
  wait_barrier<P * (NS - 1)>();
  Frag<MB, BV> F0, F1;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int mi = 0; mi < MB; ++mi) F0.a[kb][mi] = *(const lds_f32x4*)(smem + c.abase[kb] + mi * 2048);
    if constexpr (BV) {
#pragma unroll
      for (int e = 0; e < 4; ++e) F0.b4[kb][e] = *(const lds_f32x4*)(smem + c.bbase[0] + kb * 8192 + e * 512);
    } else {
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          F0.b[kb][ni][e] = *(const lds_f32*)(smem + c.bbase[ni] + kb * 8192 + e * 512);
    }
  }
  // K-tile t computes from set t & 1, reads t+1 into the other set from
  // stage (t+1) % NS, refills stage t % NS with tile t + NS.
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile<H, NS, BV, LN>(c, smem, t, (uint32_t)((t % NS) * STAGE), (uint32_t)(((t + 1) % NS) * STAGE), acc, F0,
                         F1);
    ktile<H, NS, BV, LN>(c, smem, t + 1, (uint32_t)(((t + 1) % NS) * STAGE), (uint32_t)(((t + 2) % NS) * STAGE),
                         acc, F1, F0);
  }
  if (t < nk)  // odd count: the last tile (its "next" reads are clamped re-reads)
    ktile<H, NS, BV, LN>(c, smem, t, (uint32_t)((t % NS) * STAGE), (uint32_t)((t % NS) * STAGE), acc, F0, F1);
  // Drain the tail DMAs and give the last MFMAs time to write their AGPRs
  // (asm MFMAs are invisible to hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  SplitSlots sl;
  const bool split = a.splitk > 1;
  if (split && !splitk_meet<MB, NB, NT>(a, smem, meet_tile, slice, acc, sl))
    return;

  // Epilogue through LDS as whole 256-B rows (common.h store_block16_f32),
  // once every wave is done with the stages.
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  char* Cb = (char*)a.C + (long long)bz * a.sC * 4;
  char* ebuf = smem + 1024 + wu * epi_buf_f32<NB>();  // past splitk_meet's ticket word
  const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
  // S == 2: the other slice's rows prefetched a row ahead (splitk.h
  // splitk_load_other), in the 4-stage kernel only: in the two-stage one the
  // extra live registers made hipcc place register copies right before the asm
  // MFMAs of the odd-count last K-tile (wrong results at K / 32 odd, found by
  // scripts/race_screen.py; tests/test_mfma_hazards.py now screens for it).
  const bool pf2 = NS == 4 && split && a.splitk == 2 && a.meet_prefetch;
  const bool pf3 = NS == 4 && split && a.splitk == 3 && a.meet_prefetch;  // splitk_load_others3
  f32x4 qa[NB], qb[NB];
  f32x4 ta[2][NB], tb[2][NB];
  if (pf2) splitk_load_other<MB, NB, NT>(sl, slice, 0, qa);
  if (pf3) splitk_load_others3<MB, NB, NT>(sl, slice, 0, ta);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    f32x4 v[NB];
    if (!split) {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = acc[mi][j];
    } else if (pf2) {
      if (mi + 1 < MB) splitk_load_other<MB, NB, NT>(sl, slice, mi + 1, (mi & 1) ? qa : qb);
      const f32x4(&q)[NB] = (mi & 1) ? qb : qa;
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = acc[mi][j] + q[j];
    } else if (pf3) {
      if (mi + 1 < MB) splitk_load_others3<MB, NB, NT>(sl, slice, mi + 1, (mi & 1) ? ta : tb);
      splitk_sum3<NB>(slice, acc[mi], (mi & 1) ? tb : ta, v);
    } else {
      splitk_row<MB, NB, NT>(a, sl, slice, mi, acc, v);
    }
    if constexpr (BV) {  // v[ni][r] is column 16 g + 4 r + ni: w[r] = columns 16 g + 4 r .. + 3
      f32x4 w[NB];
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = f32x4{v[0][r], v[1][r], v[2][r], v[3][r]};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = w[r];
    }
    const int row0 = m0 + wr * (BM / 2) + mi * 16, col0 = n0 + wc * 64;
    if (interior)
      store_block16_f32<false, NB, BV>(ebuf, v, Cb, (long long)a.ldc * 4, row0, col0, a.M, a.N, lane);
    else
      store_block16_f32<true, NB, BV>(ebuf, v, Cb, (long long)a.ldc * 4, row0, col0, a.M, a.N, lane);
  }
}

}  // namespace kf32t

// Same operand constraints as gemm_f32_256 / gemm_f32_w4 (K % 32, N % 4,
// lda / ldb % 4, 16-B aligned A / B, 16-B aligned C rows).
bool gemm_f32_tile_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.K % 32 || a.N % 4) return false;
  if (a.lda % 4 || a.ldb % 4 || a.ldc % 4) return false;
  if (a.lda < a.K || a.ldb < a.N || a.ldc < a.N) return false;
  if (a.batch > 1 && (a.sA % 4 || a.sB % 4 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 16) return false;
  // 32-bit offsets: A rows up to 127 * lda (+ K bytes), B rows up to 31 * ldb.
  if ((long long)128 * a.lda * 4 + (long long)a.K * 4 >= (1LL << 31)) return false;
  if ((long long)32 * a.ldb * 4 + 512 >= (1LL << 31)) return false;
  return true;
}

// LN's 32-bit voffsets: the K-tile offset rides in them, so the whole K of A
// (128 B per K-tile, plus 127 rows) and of B (K rows) must stay below 2^31.
bool gemm_f32_tile_ln_fits(const GemmArgs& a) {
  return (long long)128 * a.lda * 4 + (long long)a.K * 4 < (1LL << 31) &&
         (long long)(a.K + 32) * a.ldb * 4 + 512 < (1LL << 31);
}

// a.splitk > 1: split-K with a.part / a.flags (gemm_dispatch.cpp f32 planner).
// variant 0: kF32T128 (4 stages, b128 B reads); 2: kF32T128x2 (2 stages, two
// workgroups per CU); experiment builds: 1 = b32 B reads (round 3's first version).
// Tile-range launches (gemm_dispatch.cpp tail_plan, as gemm_w4.hip's):
// tile_end > 0 runs tiles [0, tile_end) of map_tile's order unsplit (the
// whole waves); tile_span > 0 runs tiles [tile_base, +span), each split
// a.splitk ways (the meet's tile id is the local index).
hipError_t gemm_f32_tile_launch(GemmArgs a, hipStream_t stream, int variant) {
  const int bm = variant == 3 || variant == 4 || variant == 7 || variant == 8 ? 64 : 128;  // kF32T64 (x2)
  a.tiles_m = (a.M + bm - 1) / bm;
  a.tiles_n = (a.N + kf32t::BN - 1) / kf32t::BN;
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const int S = a.splitk > 1 ? a.splitk : 1;
  const long long all_tiles = (long long)a.tiles_m * a.tiles_n * a.batch;
  if (a.tile_span < 0 || a.tile_base < 0 || a.tile_end < 0 || a.tile_end > all_tiles ||
      (a.tile_end > 0 && (a.tile_span > 0 || S > 1)) ||
      (a.tile_span > 0 && (long long)a.tile_base + a.tile_span > all_tiles))
    return hipErrorInvalidValue;
  const long long tiles = a.tile_span > 0 ? a.tile_span : a.tile_end > 0 ? a.tile_end : all_tiles;
  if (S > 1) {
    const int nk = a.K / kf32t::BK;
    a.kt_per = (nk + S - 1) / S;
    if ((S - 1) * a.kt_per >= nk || !a.part || !a.flags || tiles > kMaxSplitTiles)
      return hipErrorInvalidValue;  // every slice must own >= 1 K-tile
  } else {
    a.splitk = 1;
  }
  const long long nblocks = tiles * S;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
#ifdef PDMB_EXPERIMENTS
  if (variant == 1) {
    hipLaunchKernelGGL((kf32t::gemm_f32_t128<4, false>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant >= 5 && variant <= 8) {  // LN forms of kF32T128, kF32T128x2, kF32T64, kF32T64x2
    if (!gemm_f32_tile_ln_fits(a)) return hipErrorInvalidValue;
    auto k = variant == 5 ? kf32t::gemm_f32_t128<4, true, 128, true>
           : variant == 6 ? kf32t::gemm_f32_t128<2, true, 128, true>
           : variant == 7 ? kf32t::gemm_f32_t128<4, true, 64, true>
                          : kf32t::gemm_f32_t128<2, true, 64, true>;
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
    return hipGetLastError();
  }
#endif
  if (variant == 3) {  // kF32T64: 64x128 tiles, 4 stages, one workgroup per CU
    hipLaunchKernelGGL((kf32t::gemm_f32_t128<4, true, 64>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 4) {  // kF32T64x2: 64x128 tiles, 2 stages, two workgroups per CU
    hipLaunchKernelGGL((kf32t::gemm_f32_t128<2, true, 64>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 2) {  // kF32T128x2
    hipLaunchKernelGGL((kf32t::gemm_f32_t128<2, true>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant != 0) return hipErrorInvalidValue;
  if (S == 1 && gemm_f32_tile_ln_fits(a)) {
    // Unsplit kF32T128 runs the lean K-loop (round 6, bitwise equal): +0.6-0.7 %
    // on 4096 x 1024 x 4096, 2048^3, 4096 x 2048 x 4096 (settled, two sessions,
    // profiles/r8v_fp32_tile_lean.md). Split slices keep the plain loop (not
    // measured lean), and so do the two-per-CU and 64-row forms (lean lost there).
    hipLaunchKernelGGL((kf32t::gemm_f32_t128<4, true, 128, true>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0,
                       stream, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((kf32t::gemm_f32_t128<4, true>), dim3((unsigned)nblocks), dim3(kf32t::NT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace pdmb
