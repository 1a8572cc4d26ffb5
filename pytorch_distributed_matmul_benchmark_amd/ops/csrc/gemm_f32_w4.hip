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
// B k-row pitch: 1040 B (BP false) or 1024 B (BP, experiments: kF32W4NBP).
// With 1040-B rows the b128 B reads of lane groups g and g + 1 (k-rows 4
// apart = 4160 B, 64 B mod the 256-B bank row) overlap on 4 bank quads in
// every ds_read_b128 lane group ({0-3,12-15} of g against {4-11} of g + 1,
// MI355X_MICROARCH.md LDS table): 2-way, 4 extra cycles per read, exactly
// the 5.4e8 conflict cycles of profiles/r8h_*; 1024-B rows put a group's 16
// lanes on 16 distinct quads (gemm_f32_tile.hip kBSwz). The pad only helps
// the b32 reads (BV false).
template <bool BP>
constexpr int b_pitch() { return BP ? BN * 4 : (BN + 4) * 4; }
template <bool BP>
constexpr int stage_bytes() { return A_BYTES + BK * b_pitch<BP>(); }  // 66,048 / 65,536 B
constexpr int B_PITCH = b_pitch<false>();
constexpr int STAGE = stage_bytes<false>();
constexpr int LDS_BYTES = 2 * STAGE;      // 132,096 B (the BP stages fit in it)

__device__ __forceinline__ void mfma(f32x4& acc, float b, float a) {
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ void mfma_zero(f32x4& acc, float b, float a) {
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&a"(acc) : "v"(b), "v"(a));
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

// LN (experiments): M0 = an SGPR stage base + the piece's constant LDS
// offset in one SALU (the plain form computes the address, then moves it).
__device__ __forceinline__ void dma16_m0i(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t base, int imm) {
  asm volatile(
      "s_add_u32 m0, %3, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(base), "i"(imm)
      : "memory", "m0", "scc");
}

// LN >= 2 (experiments): the DMA piece fused with its gap's MFMA, which is
// the one wait state the M0 write needs before the LDS-DMA (no s_nop).
__device__ __forceinline__ void mfma_dma(f32x4& acc, float b, float a, u32x4 rsrc, uint32_t voff,
                                         uint32_t soff, uint32_t base, int imm) {
  asm volatile(
      "s_add_u32 m0, %5, %6\n\t"
      "v_mfma_f32_16x16x4_f32 %0, %1, %2, %0\n\t"
      "buffer_load_dwordx4 %3, %4, %7 offen lds"
      : "+a"(acc)
      : "v"(b), "v"(a), "v"(voff), "s"(rsrc), "s"(base), "i"(imm), "s"(soff)
      : "memory", "m0", "scc");
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
template <bool BP>
__device__ __forceinline__ void issue_piece(const Ctx& c, u32x4 ra, u32x4 rb, int stg, int h) {
  constexpr int ST = stage_bytes<BP>();
  if (h < 8) {
    dma16_m0(ra, c.voffA, (uint32_t)(h * 32 * c.lda4),
             c.lds0 + stg * ST + ((h * 4 + c.wu) * 8) * 128);
  } else {
    const int kr = (h - 8) * 4 + c.wu;
    dma16_m0(rb, c.voffB, (uint32_t)((h - 8) * 4 * c.ldb4), c.lds0 + stg * ST + A_BYTES + kr * b_pitch<BP>());
  }
}

// LN (experiments): piece h of the K-tile whose A / B voffsets are vA / vB (the
// K-tile offset rides in the voffset, so the descriptors are the slice's, set
// once), into the stage at LDS byte `base`.
template <bool BP>
__device__ __forceinline__ void issue_piece_ln(const Ctx& c, u32x4 ra, u32x4 rb, uint32_t vA, uint32_t vB,
                                               uint32_t base, int h) {
  static_assert(BP, "LN: the A piece and B k-row wave offsets are both wu * 1 KiB");
  if (h < 8)  // A rows (h * 4 + wu) * 8 + [0, 8): wu * 1 KiB rides in `base`
    dma16_m0i(ra, vA, (uint32_t)(h * 32 * c.lda4), base, h * 4096);
  else  // B k-row (h - 8) * 4 + wu
    dma16_m0i(rb, vB, (uint32_t)((h - 8) * 4 * c.ldb4), base, A_BYTES + (h - 8) * 4 * 1024);
}

// Fragment reads of 16-k block kb from stage stg. mi / ni index the wave's
// 8 row blocks / 8 column blocks; each is issued separately so the schedule
// can place it in an MFMA gap.
template <bool BP>
__device__ __forceinline__ f32x4 read_a(const char* smem, int stg, int kb, int mi, int wr, int l16,
                                        int g) {
  const int r = wr * 128 + mi * 16 + l16;
  const int ch = (kb * 4 + g) ^ ((r >> 1) & 7);
  return *(const f32x4*)(smem + stg * stage_bytes<BP>() + r * 128 + ch * 16);
}
template <bool BP>
__device__ __forceinline__ float read_b(const char* smem, int stg, int kb, int ni, int e, int wc,
                                        int l16, int g) {
  const int k = kb * 16 + 4 * g + e;
  const int col = wc * 128 + ni * 16 + l16;
  return *(const float*)(smem + stg * stage_bytes<BP>() + A_BYTES + k * b_pitch<BP>() + col * 4);
}
template <bool BP>
__device__ __forceinline__ f32x4 read_b4(const char* smem, int stg, int kb, int h, int e, int wc,
                                         int l16, int g) {
  const int k = kb * 16 + 4 * g + e;
  const int col = wc * 128 + h * 64 + 4 * l16;
  return *(const f32x4*)(smem + stg * stage_bytes<BP>() + A_BYTES + k * b_pitch<BP>() + col * 4);
}

// One 16-k half: 256 MFMAs from `cur`; in their gaps read the other half's
// fragments into `nxt` (kb_next >= 0) and issue DMA pieces [p0, p0 + np) of
// the next tile (one per 4 MFMAs from the start). DG: the timing-only
// diagnostic bits of gemm_f32_w4 (1: no DMA, 2: no fragment reads). SP
// (experiments): bit 1 spreads the DMA pieces one per 16 MFMAs over the whole
// half (instead of one per 4 over its first quarter), bit 2 the fragment reads
// one per 12 over its first three quarters (the phases 15 mod 16 and 5 mod 12
// never meet).
template <bool BV, bool BP, int DG = 0, int SP = 0, int LN = 0, bool ZERO = false>
__device__ __forceinline__ void half_step(const Ctx& c, const char* smem, f32x4 (&acc)[8][8],
                                          const Half<BV>& cur, Half<BV>& nxt, int stg_rd, int kb_next,
                                          int wr, int wc, int l16, int g, u32x4 ra, u32x4 rb,
                                          int stg_dma, int p0, int np, uint32_t vA = 0, uint32_t vB = 0,
                                          uint32_t mbase = 0) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) {
        const int gap = (e * 8 + mi) * 8 + ni;  // 0..255
        constexpr int DP = (SP & 1) ? 16 : 4, DR = (SP & 1) ? 15 : 3;  // DMA period / phase
        constexpr int RP = (SP & 2) ? 12 : 4, RR = (SP & 2) ? 5 : 1;   // read period / phase
        static_assert(!(SP & 2) || BV, "spread reads: b128 B reads only");
        if constexpr (LN >= 2) {
          static_assert(BV && BP && DG == 0, "LN 2: on the b128, 1 KiB-row kernel");
          if (gap % DP == DR && gap / DP < np) {  // MFMA + DMA piece h in one asm block
            const int h = p0 + gap / DP;
            if (h < 8)
              mfma_dma(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e], ra, vA,
                       (uint32_t)(h * 32 * c.lda4), mbase, h * 4096);
            else
              mfma_dma(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e], rb, vB,
                       (uint32_t)((h - 8) * 4 * c.ldb4), mbase, A_BYTES + (h - 8) * 4096);
            __builtin_amdgcn_sched_barrier(0);
            continue;
          }
        }
        if constexpr (ZERO && BV) {  // a streamed tile's K-tile 0: e == 0 starts each accumulator
          if (e == 0)
            mfma_zero(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e]);
          else
            mfma(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e]);
        } else if constexpr (BV) {
          mfma(acc[mi][ni], cur.b4[e][ni >> 2][ni & 3], cur.a[mi][e]);
        } else {
          mfma(acc[mi][ni], cur.b[ni][e], cur.a[mi][e]);
        }
        if (gap % DP == DR && gap / DP < np) {
          if constexpr (DG & 1) continue;
          if constexpr (LN)
            issue_piece_ln<BP>(c, ra, rb, vA, vB, mbase, p0 + gap / DP);
          else
            issue_piece<BP>(c, ra, rb, stg_dma, p0 + gap / DP);
        } else if (kb_next >= 0 && gap % RP == RR && gap / RP < (BV ? 16 : 40)) {
          if constexpr (DG & 2) continue;
          // 8 A rows (b128) then the B reads (BV: 8 b128; else 32 b32), one per RP MFMAs
          const int q = gap / RP;
          if (q < 8) {
            nxt.a[q] = read_a<BP>(smem, stg_rd, kb_next, q, wr, l16, g);
          } else if constexpr (BV) {
            const int e2 = (q - 8) >> 1, h2 = (q - 8) & 1;
            nxt.b4[e2][h2] = read_b4<BP>(smem, stg_rd, kb_next, h2, e2, wc, l16, g);
          } else {
            const int e2 = (q - 8) >> 3, ni2 = (q - 8) & 7;
            nxt.b[ni2][e2] = read_b<BP>(smem, stg_rd, kb_next, ni2, e2, wc, l16, g);
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
// DG (experiments, round 6: kF32W4NoDma ..., timing-only, WRONG results): bit 1
// drops the DMA refills, bit 2 the fragment reads, bit 4 the mid-tile wait and
// barrier — what costs the NB kernel its 97.3 % MFMA busy against hipBLASLt's
// 98.7 % (profiles/r8l_*).
// LN (experiments, kF32W4Lean): kF32W4NBP with a third of the SALU work per
// K-tile: the slice's descriptors are built once and each K-tile's offset rides
// in the voffsets (two VALU adds) instead of two new descriptors per K-tile
// (~30 SALU), and M0 takes one SALU per piece (dma16_m0i). r8m: the DMA pieces
// (with their SALU) cost 0.9 % MFMA busy and the fragment reads 0.6 %; the
// kernel's 0.14 SALU per MFMA against hipBLASLt's 0.04 is the largest
// instruction-mix difference left (profiles/r8i_fp32_instruction_mix.md).
// LN 2 (kF32W4Lean2): also no s_nop per DMA piece (mfma_dma). (Unrolling the
// K-loop by two to make each stage a constant made hipcc split an accumulator's
// live range with v_accvgpr moves inside the loop — the hazard class
// tests/test_mfma_hazards.py screens for — so it is not done.)
template <bool BV, bool NB = false, bool BP = false, int DG = 0, int SP = 0, int LN = 0>
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
    for (int h = 0; h < 16; ++h) issue_piece<BP>(c, ra, rb, 0, h);
  }
  if (nk > 1) {
    const u32x4 ra = rsrc_a(1), rb = rsrc_b(1);
#pragma unroll
    for (int h = 0; h < 16; ++h) issue_piece<BP>(c, ra, rb, 1, h);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  Half<BV> h0, h1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // in the order the MFMAs consume them
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
      if (e == 0) h0.a[mi] = read_a<BP>(smem, 0, 0, mi, wr, l16, g);
    if constexpr (BV) {
#pragma unroll
      for (int h = 0; h < 2; ++h) h0.b4[e][h] = read_b4<BP>(smem, 0, 0, h, e, wc, l16, g);
    } else {
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) h0.b[ni][e] = read_b<BP>(smem, 0, 0, ni, e, wc, l16, g);
    }
  }
  // K-tile t (stage s = t & 1; tile t+1 in s ^ 1 was issued a tile ago):
  //   half 0: MFMAs from h0 | read half 1 of t from s into h1
  //   mid-tile: vmcnt(0) (t+1 landed) lgkmcnt(0) (this wave done reading s),
  //             s_barrier — so nobody waits at the top of a tile
  //   half 1: MFMAs from h1 | DMA tile t+2 into s | read half 0 of t+1 from
  //           s ^ 1 into h0
  const u32x4 ra0 = rsrc_a(0), rb0 = rsrc_b(0);  // LN: built once
  static_assert(!LN || (NB && BP && DG == 0), "LN: on the branch-free 1 KiB-row kernel");
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const bool more = t + 1 < nk, more2 = t + 2 < nk;
    const int td = more2 ? t + 2 : t;  // the last two tiles issue no DMA (np = 0; NB: a re-read)
    if constexpr (LN) {
      // the slice's descriptors; this K-tile's offset in the voffsets
      const uint32_t vA = c.voffA + (uint32_t)td * (BK * 4), vB = c.voffB + (uint32_t)td * (BK * c.ldb4);
      const uint32_t mbase = c.lds0 + (uint32_t)s * stage_bytes<BP>() + (uint32_t)c.wu * 1024;
      half_step<BV, BP, DG, SP, LN>(c, smem, acc, h0, h1, s, 1, wr, wc, l16, g, ra0, rb0, s, 0, 0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      half_step<BV, BP, DG, SP, LN>(c, smem, acc, h1, h0, s ^ 1, 0, wr, wc, l16, g, ra0, rb0, s, 0, 16, vA, vB,
                                    mbase);
      continue;
    }
    const u32x4 ra = rsrc_a(td), rb = rsrc_b(td);
    half_step<BV, BP, DG, SP, LN>(c, smem, acc, h0, h1, s, 1, wr, wc, l16, g, ra, rb, s, 0, 0);
    if constexpr (!(DG & 4)) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NB)
      half_step<BV, BP, DG, SP, LN>(c, smem, acc, h1, h0, s ^ 1, 0, wr, wc, l16, g, ra, rb, s, 0, 16);
    else
      half_step<BV, BP, DG, SP, LN>(c, smem, acc, h1, h0, s ^ 1, more ? 0 : -1, wr, wc, l16, g, ra, rb, s,
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

// ---- f32_w4s: the streamed persistent form (round 6) ------
// The lean2 K-loop (1 KiB B rows, descriptors per tile, M0 in one SALU, no
// s_nop per DMA piece: 98.3 % MFMA busy against hipBLASLt's 98.9 %,
// profiles/r8p_*) run as ONE K-tile stream per CU, as gemm_w4.hip's W4S does
// for bf16: the DMA pieces that would fetch K-tiles nk, nk + 1 fetch K-tiles
// 0, 1 of the CU's next tile, the last K-tile reads the next tile's first
// fragments as usual, K-tile 0 starts the accumulators with C = 0 (no zeroing
// pass), and the epilogue leaves through its own LDS region past the two
// stages (16-row x 64-column blocks, 17 KiB for the four waves) while the
// next tile's first K-tiles land. Its 64 stores per wave are not drained:
// vmcnt counts loads, stores and LDS-DMA in issue order, so K-tile 0's
// mid-tile wait is vmcnt(47) (K-tile 1 landed once at most 47 younger stores
// remain; the 16 refills that half issues then keep the count <= 63).
// The count must NEVER pass 63, the counter's largest value: the hardware
// does not hold back a 64th outstanding operation, and the counter wraps.
// (The first form waited vmcnt(63) after 16 K-tile 1 pieces plus 64 stores,
// or 64 no-access loads before the first tile: up to 80 outstanding. With
// K-tile 1 slow to land — a cold first launch — that wrapped the counter and
// a later wait never finished: the launch hung, r8s / r8t.) So the epilogue
// waits vmcnt(43) before its last 20 stores (the 16 pieces of K-tile 1 and the
// first store retired: at most 43 + 20 = 63), and the first tile starts with
// both prologue stages landed. That needs all 64 stores issued on every tile,
// so only whole tiles run here (M, N multiples of 256: no masked store can be
// skipped). Tiles are static (workgroup b: b, b + G, ...; G a multiple
// of 8 keeps a tile on map_tile's XCD); no workgroup waits for another, so
// residency is not required. Host: unsplit, K / 32 even and >= 4, M % 256 ==
// N % 256 == 0, K * ldb * 4 < 2^31.
constexpr int EPI4 = epi_buf_f32<4>();                        // 4352 B per wave
constexpr int S_STAGE = stage_bytes<true>();                   // 65,536 B
constexpr int S_LDS = 2 * S_STAGE + 4 * EPI4;                  // 148,480 B

struct TileSrc {
  u32x4 ra, rb;  // A at row m0 / B at column n0, both from K = 0, to the operand's end
};

__device__ __forceinline__ TileSrc f32_tile_src(const GemmArgs& a, int bz, int tm, int tn) {
  const int m0 = tm * BM, n0 = tn * BN;
  TileSrc t;
  t.ra = make_rsrc((const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda) * 4,
                   ((long long)(a.M - m0 - 1) * a.lda + a.K) * 4);
  t.rb = make_rsrc((const char*)a.B + ((long long)bz * a.sB + n0) * 4,
                   ((long long)(a.kb - 1) * a.ldb + (a.N - n0)) * 4);
  return t;
}

template <int W>
__device__ __forceinline__ void wait_vm_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(W) : "memory");
}

// One K-tile in stage S: half 0 from h0 (reading h1 of this K-tile from S);
// the mid-tile wait (vmcnt(W): the next K-tile landed; lgkmcnt(0): S read);
// half 1 from h1, refilling S with the K-tile two ahead (descriptors ra / rb,
// voffsets vA / vB) and reading h0 of the next K-tile from S ^ 1.
template <int W, bool ZERO>
__device__ __forceinline__ void ktile_s(const Ctx& c, const char* smem, f32x4 (&acc)[8][8], Half<true>& h0,
                                        Half<true>& h1, int S, int wr, int wc, int l16, int g, u32x4 ra,
                                        u32x4 rb, uint32_t vA, uint32_t vB, uint32_t mbase) {
  half_step<true, true, 0, 0, 2, ZERO>(c, smem, acc, h0, h1, S, 1, wr, wc, l16, g, ra, rb, S, 0, 0);
  wait_vm_lgkm_barrier<W>();
  __builtin_amdgcn_sched_barrier(0);
  half_step<true, true, 0, 0, 2>(c, smem, acc, h1, h0, S ^ 1, 0, wr, wc, l16, g, ra, rb, S, 0, 16, vA, vB,
                                 mbase);
}

// DBG (experiments, kF32W4SDbg): lane 0 of every wave stamps its progress
// into a.dbg (host-mapped, coherent: read by the host while the kernel runs)
// at slot (blockIdx.x * 4 + wave) * 4: [0] tiles finished, [1] phase
// (1 prologue issued, 2 prologue landed, 3 K-tile 0 done, 4 K-loop done,
// 5 epilogue done, 9 exit), [2] the last K-tile finished, [3] its tile index.
__device__ __forceinline__ void dbg_stamp(const GemmArgs& a, int lane, int wu, int k, long long v) {
  if (lane == 0)
    __hip_atomic_store(a.dbg + ((long long)blockIdx.x * 4 + wu) * 4 + k, (unsigned long long)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int DBG = 0>
__global__ void __launch_bounds__(NT, 1) gemm_f32_w4s(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[S_LDS];
  const int T = a.tiles_m * a.tiles_n * a.batch;
  const int G = gridDim.x;
  int vb = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda4 = a.lda * 4;
  c.ldb4 = a.ldb * 4;
  c.nk = a.K / BK;
  {
    const int r = wu * 8 + (lane >> 3);  // row of A piece 0
    c.voffA = (uint32_t)(r * c.lda4 + (((lane & 7) ^ ((r >> 1) & 7)) * 16));
    c.voffB = (uint32_t)(wu * c.ldb4 + lane * 16);  // k-row wu of piece 8
  }
  const int nk = c.nk;
  const uint32_t kA = BK * 4, kB = (uint32_t)(BK * c.ldb4);  // voffset steps per K-tile
  const uint32_t mb0 = c.lds0 + (uint32_t)wu * 1024, mb1 = mb0 + S_STAGE;

  int bz, tm, tn;
  map_tile(a, vb, bz, tm, tn);
  TileSrc cur = f32_tile_src(a, bz, tm, tn);
  int nvb = vb + G, nbz = bz, ntm = tm, ntn = tn;
  TileSrc nxt = cur;
  if (nvb < T) {
    map_tile(a, nvb, nbz, ntm, ntn);
    nxt = f32_tile_src(a, nbz, ntm, ntn);
  }

  // Prologue of the first tile: K-tiles 0, 1 -> stages 0, 1; K-tile 0 landed
  // everywhere; its first half's fragments.
#pragma unroll
  for (int h = 0; h < 16; ++h) issue_piece_ln<true>(c, cur.ra, cur.rb, c.voffA, c.voffB, mb0, h);
#pragma unroll
  for (int h = 0; h < 16; ++h) issue_piece_ln<true>(c, cur.ra, cur.rb, c.voffA + kA, c.voffB + kB, mb1, h);
  if constexpr (DBG) dbg_stamp(a, lane, wu, 1, 1);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  Half<true> h0, h1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
      if (e == 0) h0.a[mi] = read_a<true>(smem, 0, 0, mi, wr, l16, g);
#pragma unroll
    for (int h = 0; h < 2; ++h) h0.b4[e][h] = read_b4<true>(smem, 0, 0, h, e, wc, l16, g);
  }
  char* ebuf = smem + 2 * S_STAGE + wu * EPI4;
  // K-tile 1 of the first tile landed too (K-tile 0's vmcnt(47) counts on
  // nothing older than the stores being outstanding)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DBG) dbg_stamp(a, lane, wu, 1, 2);
  int ntiles = 0;

  // Started by each tile's K-tile 0 (ZERO: C = 0 in the first MFMA of every
  // accumulator). Zeroing them with v_accvgpr_write instead put each write 1-4
  // instructions before the asm MFMA reading it: a VALU-write / MFMA-read
  // hazard hipcc cannot see.
  f32x4 acc[8][8];
  for (;;) {
    const bool more = nvb < T;
    // K-tile 0 (stage 0): the epilogue's stores are younger than K-tile 1
    ktile_s<47, true>(c, smem, acc, h0, h1, 0, wr, wc, l16, g, cur.ra, cur.rb, c.voffA + 2 * kA,
                      c.voffB + 2 * kB, mb0);
    if constexpr (DBG) {
      dbg_stamp(a, lane, wu, 1, 3);
      dbg_stamp(a, lane, wu, 3, vb);
    }
    int t = 1;
    for (; t + 2 < nk; ++t) {
      ktile_s<0, false>(c, smem, acc, h0, h1, t & 1, wr, wc, l16, g, cur.ra, cur.rb,
                        c.voffA + (uint32_t)(t + 2) * kA, c.voffB + (uint32_t)(t + 2) * kB, (t & 1) ? mb1 : mb0);
      if constexpr (DBG) dbg_stamp(a, lane, wu, 2, t);
    }
    {
      // K-tiles nk - 2 (stage 0), nk - 1 (stage 1): their refills are the next
      // tile's K-tiles 0 and 1 — or, on the last tile, re-reads of this tile's
      // last K-tile into stages nobody reads again
      const u32x4 ra = more ? nxt.ra : cur.ra, rb = more ? nxt.rb : cur.rb;
      const uint32_t k0 = more ? 0u : (uint32_t)(nk - 1), k1 = more ? 1u : (uint32_t)(nk - 1);
      ktile_s<0, false>(c, smem, acc, h0, h1, 0, wr, wc, l16, g, ra, rb, c.voffA + k0 * kA, c.voffB + k0 * kB,
                        mb0);
      ktile_s<0, false>(c, smem, acc, h0, h1, 1, wr, wc, l16, g, ra, rb, c.voffA + k1 * kA, c.voffB + k1 * kB,
                        mb1);
    }
    if constexpr (DBG) dbg_stamp(a, lane, wu, 1, 4);
    // The last MFMAs write their AGPRs before the epilogue reads them (asm
    // MFMAs are invisible to hipcc's hazard recognizer). Every accumulator is
    // an operand of the padding, so no register copy of one (the epilogue's
    // regroup needs AGPR temporaries) can be placed before it.
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15"
                 : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]), "+a"(acc[0][4]),
                   "+a"(acc[0][5]), "+a"(acc[0][6]), "+a"(acc[0][7])::"memory");
#pragma unroll
    for (int i = 1; i < 8; ++i)
      asm volatile(""
                   : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                     "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    __builtin_amdgcn_sched_barrier(0);
    char* Cb = (char*)a.C + (long long)bz * a.sC * 4;
    const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // acc[mi][4 h + j][r] is column 64 h + 16 g + 4 r + j: regroup by r
        // 4 stores per block: before block 11 (stores 44..), at most 43 outstanding
        if (mi * 2 + h == 11) asm volatile("s_waitcnt vmcnt(43)" ::: "memory");
        f32x4 w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          w[r] = f32x4{acc[mi][4 * h][r], acc[mi][4 * h + 1][r], acc[mi][4 * h + 2][r], acc[mi][4 * h + 3][r]};
        const int row0 = m0 + wr * 128 + mi * 16, col0 = n0 + wc * 128 + 64 * h;
        store_block16_f32<false, 4, true>(ebuf, w, Cb, (long long)a.ldc * 4, row0, col0, a.M, a.N, lane);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DBG) {
      dbg_stamp(a, lane, wu, 1, 5);
      dbg_stamp(a, lane, wu, 0, ++ntiles);
    }
    if (!more) break;
    vb = nvb;
    bz = nbz;
    tm = ntm;
    tn = ntn;
    cur = nxt;
    nvb = vb + G;
    if (nvb < T) {
      map_tile(a, nvb, nbz, ntm, ntn);
      nxt = f32_tile_src(a, nbz, ntm, ntn);
    }
  }
  // No LDS-DMA may still be writing when this workgroup's LDS is handed on.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DBG) dbg_stamp(a, lane, wu, 1, 9);
}

}  // namespace kf32w4

// The lean K-loop's 32-bit voffsets carry the K-tile offset: A's 255 rows plus
// its whole K, and B's whole K of rows, must stay below 2^31 bytes.
bool gemm_f32_w4l_fits(const GemmArgs& a) {
  return (long long)256 * a.lda * 4 + (long long)a.K * 4 < (1LL << 31) &&
         (long long)(a.K + 32) * a.ldb * 4 + 1024 < (1LL << 31);
}

// The streamed form's shape constraints (K-tiles even and >= 4, whole 256x256
// tiles, 32-bit B offsets over the whole K); alignment as gemm_f32_256.
bool gemm_f32_w4s_fits(const GemmArgs& a) {
  const int nk = a.K / kf32w4::BK;
  return a.K % kf32w4::BK == 0 && nk % 2 == 0 && nk >= 4 && a.M > 0 && a.N > 0 && a.M % kf32w4::BM == 0 &&
         a.N % kf32w4::BN == 0 && (long long)a.K * a.ldb * 4 < (1LL << 31);
}

// a.splitk > 1: split-K with a.part / a.flags (gemm_dispatch.cpp f32_split).
// variant 0: the shipping kernel (b128 B reads); 16: kF32W4L, the lean K-loop
// (1 KiB B rows, branch-free, descriptors once per slice, no s_nop per DMA
// piece: bitwise equal to variant 0); experiment builds: 1.. the
// A/B arms, 14 the streamed persistent form (kF32W4S, a.pers_grid workgroups),
// 15 its stamping diagnostic.
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
  if (variant == 14) {  // kF32W4S: the streamed persistent form (unsplit, pers_grid workgroups)
    if (S > 1 || !gemm_f32_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8 || a.tile_span || a.tile_end)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL(kf32w4::gemm_f32_w4s<0>, pg, dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 15) {  // kF32W4SDbg: the streamed form stamping its progress into a.dbg
    if (S > 1 || !gemm_f32_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8 || a.tile_span || a.tile_end ||
        !a.dbg)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL(kf32w4::gemm_f32_w4s<1>, pg, dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
#endif
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
  if (variant == 3) {  // kF32W4NBP: branch-free, 1024-B B rows (conflict-free b128 reads)
    hipLaunchKernelGGL((kf32w4::gemm_f32_w4<true, true, true>), dim3((unsigned)nblocks), dim3(kf32w4::NT), 0,
                       stream, a);
    return hipGetLastError();
  }
  if (variant >= 4 && variant <= 7) {  // timing-only diagnostics of kF32W4NBP (DG 1, 2, 3, 7)
    auto k = variant == 4 ? kf32w4::gemm_f32_w4<true, true, true, 1>
           : variant == 5 ? kf32w4::gemm_f32_w4<true, true, true, 2>
           : variant == 6 ? kf32w4::gemm_f32_w4<true, true, true, 3>
                          : kf32w4::gemm_f32_w4<true, true, true, 7>;
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 11 || variant == 12) {  // kF32W4Lean, kF32W4Lean2
    auto k = variant == 11 ? kf32w4::gemm_f32_w4<true, true, true, 0, 0, 1>
                           : kf32w4::gemm_f32_w4<true, true, true, 0, 0, 2>;
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
  if (variant >= 8 && variant <= 10) {  // kF32W4Spread*: kF32W4NBP with SP 3, 1, 2
    auto k = variant == 8 ? kf32w4::gemm_f32_w4<true, true, true, 0, 3>
           : variant == 9 ? kf32w4::gemm_f32_w4<true, true, true, 0, 1>
                          : kf32w4::gemm_f32_w4<true, true, true, 0, 2>;
    hipLaunchKernelGGL(k, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
    return hipGetLastError();
  }
#endif
  if (variant == 16) {  // kF32W4L: the lean K-loop (experiments' kF32W4Lean2), unsplit or split
    if (!gemm_f32_w4l_fits(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((kf32w4::gemm_f32_w4<true, true, true, 0, 0, 2>), dim3((unsigned)nblocks), dim3(kf32w4::NT),
                       0, stream, a);
    return hipGetLastError();
  }
  if (variant != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kf32w4::gemm_f32_w4<true>, dim3((unsigned)nblocks), dim3(kf32w4::NT), 0, stream, a);
  return hipGetLastError();
}

}  // namespace pdmb
