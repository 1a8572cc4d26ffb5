// gemm_w4.hip — bf16 / fp16 C = A @ B (row-major NN, fp32 accumulate) with
// 4 waves per workgroup, one per SIMD, each owning a 128x128 output block
// (256 fp32 accumulators per lane in AGPRs).
//
// Same job as gemm_mfma256.hip (the GEMM behind the reference's torch.matmul /
// torch.bmm, matmul_scaling_benchmark.py:79,92,120,142,188,211), with the
// structure that took the fp8 kernel from 3079 to 3217 TF (gemm_fp8.hip
// "W4"): the 8-wave kernel reads 192 KiB of LDS fragments per 256x256x64
// K-tile (every A fragment by 4 waves, every B fragment by 2); with 128x128
// per wave a workgroup reads 128 KiB (each by 2). On random bf16 data the
// chip is power-bound (profiles/r1_pmc_sched3.md: 1.75 GHz at 77 % MFMA
// utilisation), so LDS energy is clock.
//
// The LDS images are the 8-wave kernel's, byte for byte (A: [256 rows][128 B]
// with 16-B chunk c at c ^ ((row>>1)&7); B: two halves [64 k][256 B] with
// 32-B unit u at u ^ ((k&3) | ((k>>3)&1)<<2), read by ds_read_b64_tr_b16), so
// the conflict-free read patterns carry over. Only the DMA split (16 pieces of
// 1 KiB per wave per K-tile) and the per-wave fragment offsets change.
//
// B halves and L2 requests (round 2): which 128 columns of the 256-wide tile
// a B half holds is free — the LDS image and every read pattern stay the same.
// The 8-wave kernel's choice (IL = 32: half nq = the four 32-column runs
// [64i + 32nq, +32)) makes each k-row of a half four 64-B segments, so every
// 128-B line of B is fetched as two half-line requests (PMC at 8192^3: W4
// 8.43e7 L2 requests vs hipBLASLt 6.92e7; the A+B minimum is 6.7e7). IL = 64
// (the default: half nq = [128i + 64nq, +64)) fetches whole lines; a wave
// still owns 128 contiguous output columns, 64 from each half.
//
// Schedule (per K-tile t from stage S, tile t+1 in S^1; gemm_fp8.hip ktile_w4):
//   Bar0: B(t+1) landed (vmcnt 16), every wave done reading A(t) (lgkmcnt 0).
//   m-blocks 0-3: 64 MFMAs | read B(t+1) fragments | DMA A(t+2) -> S.A
//   Bar_mid: A(t+1) landed, every wave done reading B(t+1) from S^1.B.
//   m-blocks 4-7: 64 MFMAs | read A(t+1) fragments | DMA B(t+3) -> S^1.B
// Every load sits in the shadow of an MFMA (one item per 16-cycle
// v_mfma_f32_16x16x32 gap at most, kItems), and each operand half gets
// ~1.5 K-tiles of DMA flight.
//
// Fast-path constraints (host-checked; otherwise the 8-wave kernel): M and N
// multiples of 256 (interior tiles only: no edge masking, no out-of-extent
// DMA), K % 64 == 0, lda / ldb % 8 == 0, ldc % 4 == 0, 16-B aligned A / B,
// 8-B aligned C.
#include "api.h"
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace kw4 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 256;
constexpr int A_BYTES = BM * BK * 2;         // 32 KiB
constexpr int BH_BYTES = BK * (BN / 2) * 2;  // 16 KiB per B half
constexpr int STAGE = A_BYTES + 2 * BH_BYTES;  // 64 KiB

// 16 fp32 accumulators x K = 32 per lane, operands swapped (B fragment
// first) so the accumulator holds C^T and a lane owns 4 consecutive columns.
template <int DT>
__device__ __forceinline__ void mfma_acc(f32x4& acc, const s16x8& b, const s16x8& a);
template <>
__device__ __forceinline__ void mfma_acc<kBF16>(f32x4& acc, const s16x8& b, const s16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
template <>
__device__ __forceinline__ void mfma_acc<kF16>(f32x4& acc, const s16x8& b, const s16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
// acc = B * A with C = 0: starts an accumulator without zeroing it first.
template <int DT>
__device__ __forceinline__ void mfma_zero(f32x4& acc, const s16x8& b, const s16x8& a);
template <>
__device__ __forceinline__ void mfma_zero<kBF16>(f32x4& acc, const s16x8& b, const s16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&a"(acc) : "v"(b), "v"(a));
}
template <>
__device__ __forceinline__ void mfma_zero<kF16>(f32x4& acc, const s16x8& b, const s16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&a"(acc) : "v"(b), "v"(a));
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

// LN (experiments, round 6): the MFMA of a DMA item's gap fused with the piece,
// as gemm_f32_w4.hip's mfma_dma: M0 in one SALU from the wave's base, the MFMA
// as the wait state M0 needs (no s_nop).
template <int DT>
__device__ __forceinline__ void mfma_dma_w4(f32x4& acc, const s16x8& b, const s16x8& a, u32x4 rsrc, uint32_t voff,
                                            uint32_t soff, uint32_t lds0w, int imm) {
  if constexpr (DT == kBF16)
    asm volatile(
        "s_add_u32 m0, %5, %6\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
        "buffer_load_dwordx4 %3, %4, %7 offen lds"
        : "+a"(acc)
        : "v"(b), "v"(a), "v"(voff), "s"(rsrc), "s"(lds0w), "i"(imm), "s"(soff)
        : "memory", "m0", "scc");
  else
    asm volatile(
        "s_add_u32 m0, %5, %6\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\t"
        "buffer_load_dwordx4 %3, %4, %7 offen lds"
        : "+a"(acc)
        : "v"(b), "v"(a), "v"(voff), "s"(rsrc), "s"(lds0w), "i"(imm), "s"(soff)
        : "memory", "m0", "scc");
}

struct Frag {  // one 16-row (A) or 16-column (B) block of a K-tile: k 0..31 and 32..63
  s16x8 k[2];
};

struct Ctx {
  u32x4 ra;             // A descriptor at K = 0
  const char* Bb;       // B at row 0, column n0
  long long b_bytes;    // bytes from Bb to the end of B's extent
  int lda2, ldb2, nk;   // leading dims in bytes, K / 64
  uint32_t voffA, voffB;  // per-lane DMA offsets of piece 0
  // Per-lane LDS fragment offsets, one VGPR per stage so every read is
  // ds_read off:imm with no address add (the immediate stops at 64 KiB).
  uint32_t aoff[2][2];  // [stage][ks]
  uint32_t boff[2][4];  // [stage][jj]: B block j uses jj = bjj<IL>(j)
  int wu;
  uint32_t lds0;
  uint32_t lds0w;  // lds0 + wu * 1 KiB: every DMA piece's per-wave LDS offset
};

// B block j (16 output columns wc*128 + 16j of the wave) lives in half bhalf
// at 32-B unit 4 wc + bjj of it (see "B halves" above).
template <int IL>
__device__ __forceinline__ constexpr int bhalf(int j) { return IL == 64 ? j >> 2 : (j >> 1) & 1; }
template <int IL>
__device__ __forceinline__ constexpr int bjj(int j) { return IL == 64 ? j & 3 : 2 * (j >> 2) + (j & 1); }

// DMA piece h (0..15) of tile `tile` into the stage at byte offset `so`.
// h < 8: A rows h*32 + wu*8 + [0,8) (8 x 128 B). h >= 8: B half nq = (h-8)>>2,
// k rows kb*16 + wu*4 + [0,4) with kb = (h-8)&3 (4 x 256 B). B's swizzle
// depends on k & 11 only, which kb*16 leaves alone, so one per-lane offset
// serves all pieces; nq shifts the source by IL columns.
template <int IL>
__device__ __forceinline__ void issue_piece(const Ctx& c, u32x4 rb, int so, int tile, int h) {
  // per-wave part (A: wu * 8 rows * 128 B, B: wu * 4 k-rows * 256 B) in lds0w
  if (h < 8) {
    dma16_at(c.ra, c.voffA, (uint32_t)tile * (BK * 2) + (uint32_t)(h * 32 * c.lda2), c.lds0w,
             so + h * 32 * 128);
  } else {
    const int nq = (h - 8) >> 2, kb = (h - 8) & 3;
    dma16_at(rb, c.voffB, (uint32_t)(kb * 16 * c.ldb2 + nq * IL * 2), c.lds0w,
             so + A_BYTES + nq * BH_BYTES + kb * 16 * 256);
  }
}

__device__ __forceinline__ u32x4 b_rsrc(const Ctx& c, int tile) {
  const long long off = (long long)tile * BK * c.ldb2;
  return make_rsrc(c.Bb + off, c.b_bytes - off);
}

// A fragment half ks of block m (rows 16m..16m+15 of this wave's 128).
__device__ __forceinline__ s16x8 frag_a(const char* smem, uint32_t off, int m) {
  return *(const lds_s16x8*)(smem + m * 16 * 128 + off);
}

// B fragment half ks of block j (16 output columns): two transposed reads.
template <int IL>
__device__ __forceinline__ s16x8 frag_b(const char* smem, uint32_t off, int j, int ks) {
  const char* p = smem + A_BYTES + bhalf<IL>(j) * BH_BYTES + ks * 32 * 256 + off;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 256));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// What a wave issues after MFMA `gap` (0..15: ks*8 + ni) of m-block `blk`.
// 0: nothing; 1: next DMA piece (blocks 0-3: A of t+2, blocks 4-7: B of
// t+3); 100 + 2s + ks: half ks of B fragment s of tile t+1; 200 + 2m + ks:
// half ks of A fragment m of tile t+1 (m = 7: into the second A7 set).
// A fragment m of t+1 is written only after block m of t is done with it.
constexpr int kItems[8][16] = {
    {100, 0, 101, 0, 1, 0, 102, 0, 103, 0, 1, 0, 0, 0, 0, 0},
    {104, 0, 105, 0, 1, 0, 106, 0, 107, 0, 1, 0, 0, 0, 0, 0},
    {108, 0, 109, 0, 1, 0, 110, 0, 111, 0, 1, 0, 0, 0, 0, 0},
    {112, 0, 113, 0, 1, 0, 114, 0, 115, 0, 1, 0, 0, 0, 0, 0},
    {200, 0, 201, 0, 1, 0, 202, 0, 203, 0, 1, 0, 0, 0, 0, 0},
    {204, 0, 205, 0, 1, 0, 206, 0, 207, 0, 1, 0, 0, 0, 0, 0},
    {208, 0, 209, 0, 1, 0, 210, 0, 211, 0, 1, 0, 214, 0, 215, 0},
    {212, 0, 213, 0, 1, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0}};

constexpr int piece_of(int blk, int gap) {  // running index of a DMA item (0..15)
  int n = 0;
  for (int b = 0; b < 8; ++b)
    for (int g = 0; g < 16; ++g) {
      if (b == blk && g == gap) return n;
      if (kItems[b][g] == 1) ++n;
    }
  return n;
}

template <int DT, int IL, int SO>
__device__ __forceinline__ void ktile(const Ctx& c, const char* smem, int t, f32x4 (&acc)[8][8],
                                      Frag (&A)[8], Frag& A7c, Frag& A7n, Frag (&Bc)[8],
                                      Frag (&Bn)[8]) {
  constexpr int SN = STAGE - SO;  // stage of tile t+1
  constexpr int sn = SN / STAGE;
  const int ta = t + 2 < c.nk ? t + 2 : c.nk - 1;  // clamped tail DMAs (harmless re-reads)
  const int tb = t + 3 < c.nk ? t + 3 : c.nk - 1;
  const u32x4 rb = b_rsrc(c, tb);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    if (mi == 0 || mi == 4) {
      asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int gap = 0; gap < 16; ++gap) {
      const int ks = gap >> 3, ni = gap & 7;
      mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], mi == 7 ? A7c.k[ks] : A[mi].k[ks]);
      const int it = kItems[mi][gap];
      if (it == 1) {
        const int h = piece_of(mi, gap);  // 0..7: A of t+2 into S; 8..15: B of t+3 into S^1
        if (h < 8)
          issue_piece<IL>(c, rb, SO, ta, h);
        else
          issue_piece<IL>(c, rb, SN, tb, h);
      } else if (it >= 100 && it < 200) {
        const int s = (it - 100) >> 1, h = (it - 100) & 1;
        Bn[s].k[h] = frag_b<IL>(smem, c.boff[sn][bjj<IL>(s)], s, h);
      } else if (it >= 214) {
        const int h = it - 214;
        A7n.k[h] = frag_a(smem, c.aoff[sn][h], 7);
      } else if (it >= 200) {
        const int m = (it - 200) >> 1, h = (it - 200) & 1;
        A[m].k[h] = frag_a(smem, c.aoff[sn][h], m);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The last K-tile of an unsplit tile with the epilogue folded in (as
// gemm_fp8.hip ktile_w4_last): block row mi - 1 leaves through this wave's
// LDS buffer past the two stages while block row mi's 16 MFMAs run (same
// per-accumulator MFMA order as ktile: bitwise equal). No fragment reads,
// DMAs or barrier.
template <int DT, bool WT = false>
__device__ __forceinline__ void ktile_last(f32x4 (&acc)[8][8], const Frag (&A)[8], const Frag& A7c,
                                           const Frag (&Bc)[8], char* ebuf, char* Cb, long long ldc_b,
                                           int row0, int col0, int M, int N) {
  auto store = [&](int i) {
    unsigned all = ~0u;  // lane id formed here: the stores' addresses are not hoisted
    asm volatile("" : "+s"(all));
    const int eln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
    store_block16<DT, false, false, 8, true, WT>(ebuf, acc[i], 1.0f, Cb, ldc_b, row0 + i * 16, col0, M, N, eln);
  };
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
    for (int gap = 0; gap < 16; ++gap) {
      const int ks = gap >> 3, ni = gap & 7;
      mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], mi == 7 ? A7c.k[ks] : A[mi].k[ks]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (mi >= 1) store(mi - 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  store(7);
}

// SUB: XCD sub-block shape (map_tile): 0 = 4 x 8 (default), 1 = 8 x 4
// (kMfmaW4Tall), 2 = 2 x 16 (kMfmaW4Wide); 1 and 2 are A/B experiments.
// IL: B half interleave in columns (64 default; 32 = kMfmaW4Il32, A/B only).
// TRACE: write the tile timeline (common.h tile_trace_write; kMfmaW4Trace).
// One output tile: virtual block vb (map_tile's order). PERS (persistent
// kernel; no split-K): thread 0 takes the next ticket of its XCD's queue
// `qpre` as the tile starts and returns it; it is first read after the
// K-loop's vmcnt(0), so the atomic's latency hides behind the tile.
// FUSED (needs 4 kEpiBuf of LDS past the stages): an unsplit tile with an
// even K-tile count stores C during its last K-tile (ktile_last); its
// fragments are then in (A7b, B1) — one register set, as in gemm_fp8.hip.
// WT: C stores write-through (GemmArgs::sig). Returns the next ticket (PERS)
// or whether this workgroup wrote C (1; 0: a split-K slice that did not).
template <int DT, int SUB, int IL, int TRACE, bool PERS, bool FUSED = false, bool WT = false>
__device__ __forceinline__ unsigned w4_tile(const GemmArgs& a, char* smem, int vb, unsigned* qpre) {
  TileTrace tr;
  if constexpr (TRACE) tr.t[0] = tile_clock();
  // PERS: an opaque thread id, so nothing lane-derived is hoisted out of the
  // persistent tile loop (live across the epilogue, it spilled).
  int tid = threadIdx.x;
  if constexpr (PERS) asm volatile("" : "+v"(tid));
  unsigned pre = 0;
  if constexpr (PERS) {
    // A per-lane (opaque) address keeps this a plain returning atomic: the
    // compiler's wave-aggregation rewrite would read the result at once and
    // wait for it here instead of after the K-loop.
    unsigned z = 0;
    asm volatile("" : "+v"(z));
    if (tid == 0) pre = __hip_atomic_fetch_add(qpre + z, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  int bz, tm, tn;
  // Split-K: the grid's "batch" is batch x S with the slice innermost, so
  // one slice of every tile is a contiguous block range (map_tile's grouped
  // order) and each workgroup runs K-tiles [kt0, kt0 + nk) of its tile. A
  // tile-range launch (GemmArgs::tile_span, the wave-quantisation tail) maps
  // block vb to local tile vb % span of the range and slice vb / span (a
  // tile's slices share the XCD, vb % 8, so their meet stays in one L2).
  int slice = 0;
  long long meet_tile;
  if (!PERS && a.tile_span > 0) {
    const int local = vb % a.tile_span;
    slice = vb / a.tile_span;
    map_tile(a, a.tile_base + local, bz, tm, tn, SUB);
    meet_tile = local;
  } else {
    map_tile(a, vb, bz, tm, tn, SUB);
    if (!PERS && a.splitk > 1) {
      slice = bz % a.splitk;
      bz /= a.splitk;
    }
    meet_tile = ((long long)bz * a.tiles_m + tm) * a.tiles_n + tn;
  }
  const int kt0 = slice * a.kt_per;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lds0w = c.lds0 + wu * 1024;
  c.lda2 = a.lda * 2;
  c.ldb2 = a.ldb * 2;
  {
    const int nk_all = a.K / BK;
    c.nk = !PERS && a.splitk > 1 ? min(a.kt_per, nk_all - kt0) : nk_all;
  }
  const int k0 = kt0 * BK;
  const char* Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda + k0) * 2;
  c.ra = make_rsrc(Ab, ((long long)(a.M - m0 - 1) * a.lda + (a.K - k0)) * 2);
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + (long long)k0 * a.ldb + n0) * 2;
  c.b_bytes = ((long long)(a.kb - k0 - 1) * a.ldb + (a.N - n0)) * 2;
  {
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;  // row of A piece 0
    c.voffA = (uint32_t)(r * c.lda2 + ((lc8 ^ ((r >> 1) & 7)) * 16));
    const int lr16 = lane >> 4, lc16 = lane & 15;
    const int k = wu * 4 + lr16;  // k row of B piece 0 (kb = 0)
    const int s = (k & 3) | (((k >> 3) & 1) << 2);
    const int p = ((lc16 >> 1) ^ s) * 16 + (lc16 & 1) * 8;
    // unit u = p >> 4 holds columns (u / (IL/16)) * 2 IL + (u % (IL/16)) * 16 (+ nq IL via soffset)
    const int n = (p / IL) * 2 * IL + (p % IL);
    c.voffB = (uint32_t)(k * c.ldb2 + n * 2);
    const int swA = (l16 >> 1) & 7;
    const int q4 = l16 >> 2, p4 = l16 & 3;
    const int sB = q4 | ((g & 1) << 2);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint32_t ao = (uint32_t)(st * STAGE + (wr * 128 + l16) * 128 + (((4 * ks + g) ^ swA) * 16));
        asm volatile("" : "+v"(ao));  // opaque: keep each as its own base VGPR
        c.aoff[st][ks] = ao;
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int u = 4 * wc + jj;  // 32-B unit of the B half
        uint32_t bo = (uint32_t)(st * STAGE + (8 * g + q4) * 256 + ((u ^ sB) * 32) + p4 * 8);
        asm volatile("" : "+v"(bo));
        c.boff[st][jj] = bo;
      }
    }
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue, in the DMA order the loop's counted waits assume:
  // A(0), B(0) -> stage 0; B(1), A(1) -> stage 1; tile 0's fragments to
  // registers; then B(2) -> stage 0.B (the loop's "Bar_mid(-1)" issue).
  const int nk = c.nk;
  const int t1 = nk > 1 ? 1 : 0, t2 = nk > 2 ? 2 : nk - 1;
  {
    const u32x4 rb0 = b_rsrc(c, 0), rb1 = b_rsrc(c, t1);
#pragma unroll
    for (int h = 0; h < 16; ++h) issue_piece<IL>(c, rb0, 0, 0, h);
#pragma unroll
    for (int h = 8; h < 16; ++h) issue_piece<IL>(c, rb1, STAGE, t1, h);
#pragma unroll
    for (int h = 0; h < 8; ++h) issue_piece<IL>(c, rb1, STAGE, t1, h);
  }
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");  // tile 0 landed everywhere
  Frag A[8], A7a, A7b, B0[8], B1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      A[i].k[ks] = frag_a(smem, c.aoff[0][ks], i);
      B0[i].k[ks] = frag_b<IL>(smem, c.boff[0][bjj<IL>(i)], i, ks);
    }
  A7a = A[7];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // stage 0.B read by all
  if constexpr (TRACE) tr.t[1] = tile_clock();
  {
    const u32x4 rb2 = b_rsrc(c, t2);
#pragma unroll
    for (int h = 8; h < 16; ++h) issue_piece<IL>(c, rb2, 0, t2, h);
  }
  const bool split = !PERS && a.splitk > 1;
  const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
  constexpr bool kFuse = FUSED && !PERS && TRACE == 0;
  const bool fuse = kFuse && !split && interior && (nk & 1) == 0;
  const int nloop = fuse ? nk - 1 : nk;
  int t = 0;
  for (; t + 1 < nloop; t += 2) {  // branch-free body: B0/B1 and A7a/A7b swap roles every K-tile
    ktile<DT, IL, 0>(c, smem, t, acc, A, A7a, A7b, B0, B1);
    ktile<DT, IL, STAGE>(c, smem, t + 1, acc, A, A7b, A7a, B1, B0);
  }
  if (t < nloop) ktile<DT, IL, 0>(c, smem, t, acc, A, A7a, A7b, B0, B1);  // odd count
  if constexpr (kFuse) {
    if (fuse) {
      ktile_last<DT, WT>(acc, A, A7b, B1, smem + 2 * STAGE + wu * kEpiBuf,
                         (char*)a.C + (long long)bz * a.sC * 2, (long long)a.ldc * 2, m0 + wr * 128,
                         n0 + wc * 128, a.M, a.N);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs landed before the LDS is released
      return PERS ? pre : 1u;
    }
  }
  // Drain the tail DMAs and give the last MFMAs time to write their AGPRs
  // (asm MFMAs are invisible to hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if constexpr (TRACE) tr.t[2] = tile_clock();

  // Split-K: only the last slice of a tile to arrive writes C, adding the
  // other slices' fp32 slots block row by block row while storing, so no
  // more than 2 x 8 fragments are live in VGPRs (splitk.h).
  SplitSlots sl;
  if (split && !splitk_meet<8, 8, NT>(a, smem, meet_tile, slice, acc, sl))
    return PERS ? pre : 0u;

  // Epilogue: acc[i][j] holds C^T of a 16x16 tile (lane: row l16, columns
  // 4g..4g+3), stored through LDS as whole rows (common.h store_block16;
  // edge tiles masked at M / N). Every wave's DMAs have landed and every
  // fragment read is done before any wave writes its staging buffers.
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
  char* ebuf = smem + 1024 + wu * 2 * kEpiBuf;  // past splitk_meet's ticket word
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f32x4 v[8];
    if (!split) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[i][j];
    } else if constexpr (!PERS) {
      splitk_row<8, 8, NT>(a, sl, slice, i, acc, v);
    }
    if (interior)
      store_block16<DT, false, false, 8, true, WT>(ebuf + (i & 1) * kEpiBuf, v, 1.0f, Cb,
                                                   (long long)a.ldc * 2, m0 + wr * 128 + i * 16,
                                                   n0 + wc * 128, a.M, a.N, lane);
    else
      store_block16<DT, true, false, 8, true, WT>(ebuf + (i & 1) * kEpiBuf, v, 1.0f, Cb,
                                                  (long long)a.ldc * 2, m0 + wr * 128 + i * 16,
                                                  n0 + wc * 128, a.M, a.N, lane);
  }
  if constexpr (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr.t[3] = tile_clock();
    tile_trace_write(a, tr, vb, tm, tn);
  }
  return PERS ? pre : 1u;
}

// FUSED: see w4_tile (false: the A/B kernel kMfmaW4Unfused).
// SIG: completion signals (GemmArgs::sig, common.h signal_tile): the tile's C
// goes out write-through, every wave drains it, the workgroup meets at a
// barrier and one lane signals the tile's slot (Guideline 16 R1: sc1
// payload, drained by every storing wave, one atomic add behind a barrier).
template <int DT, int SUB = 0, int IL = 64, int TRACE = 0, bool FUSED = true, bool SIG = false>
__global__ void __launch_bounds__(NT, 1) gemm_w4_nn(GemmArgs a) {
  constexpr bool kFused = FUSED && TRACE == 0;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + (kFused ? 4 * kEpiBuf : 0)];
  const unsigned wrote = w4_tile<DT, SUB, IL, TRACE, false, kFused, SIG>(a, smem, blockIdx.x, nullptr);
  if constexpr (SIG) {
    if (wrote) {  // uniform: a split-K slice that handed its sums on wrote nothing
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
      __syncthreads();
      if (threadIdx.x == 0) {
        int bz, tm, tn;
        map_tile(a, blockIdx.x, bz, tm, tn, SUB);
        if (a.splitk > 1) bz /= a.splitk;
        signal_tile(a, bz, tm);
      }
    }
  }
}

// Persistent W4: one workgroup per CU, tiles from per-XCD queues. The tile
// timeline (scripts/tile_timeline.py) shows the XCDs running at different
// speeds (16k bf16: 331.9 to 349.3 us per tile) while hardware dispatch
// gives each exactly 1/8 of the tiles, so the fast ones idle at the end (~2 %
// of the kernel). Here XCD x (its real XCC_ID) takes the virtual blocks
// vb = x + 8 i from queue x — map_tile's XCD-local tile sets, so L2 reuse is
// unchanged — and a workgroup whose queue is empty steals from the others.
// a.queue: 8 ticket counters + 1 exit counter, zero at launch; the last
// workgroup to exit re-zeroes them (stream-ordered, like the split-K flags).
// Every workgroup exits when no queue has a tile left.
template <int DT, int TRACE = 0>
__global__ void __launch_bounds__(NT, 1) gemm_w4_pers(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 16];
  volatile int* qword = (volatile int*)(smem + 2 * STAGE);
  unsigned* q = a.queue;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int T = a.tiles_m * a.tiles_n * a.batch;
  auto count = [&](int x) { return T > x ? (T - x + 7) / 8 : 0; };
  auto take = [&](unsigned own) -> int {  // thread 0: own ticket, else steal
    if ((int)own < count(xcc)) return (int)xcc + 8 * (int)own;
    for (int y = 1; y < 8; ++y) {
      const int x = (xcc + y) & 7;
      if (count(x) == 0) continue;
      const unsigned i = __hip_atomic_fetch_add(&q[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)i < count(x)) return x + 8 * (int)i;
    }
    return -1;
  };
  if (threadIdx.x == 0)
    *qword = take(__hip_atomic_fetch_add(&q[xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  int vb = __builtin_amdgcn_readfirstlane(*qword);  // uniform: tile math stays scalar
  while (vb >= 0) {
    const unsigned pre = w4_tile<DT, 0, 64, TRACE, true>(a, smem, vb, &q[xcc]);
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    if (tid == 0) *qword = take(pre);
    // every wave is done with its epilogue staging (lgkmcnt) before the next
    // tile's DMAs land, and sees the next ticket
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    vb = __builtin_amdgcn_readfirstlane(*qword);
  }
  if (threadIdx.x == 0) {
    const unsigned d = __hip_atomic_fetch_add(&q[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1)  // every other workgroup has taken its last ticket
      for (int i = 0; i < 9; ++i) __hip_atomic_store(&q[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- W4S: streaming persistent W4 -----------------------------------------
// The tile timeline (profiles/r2_tile_timeline_*.jsonl) puts ~7.4 us of a
// 16k tile outside its K-loop: the first DMA latency (prologue, 2.2), the C
// epilogue (4.9) and the dispatch gap (0.3-0.7) — ~2 % at K = 16384, ~8 % at
// K = 4096 — and with one workgroup per CU (W4 holds all 512 registers of
// every SIMD) nothing else on the CU can hide them. W4S runs a CU's tiles as
// ONE K-tile stream: the DMA items that would fetch K-tiles nk, nk+1, nk+2
// of the current tile fetch K-tiles 0, 1, 2 of the CU's next tile instead,
// the last K-tile reads the next tile's first fragments as usual, and the
// epilogue goes out through its own LDS region (past the two stages) while
// those land. Its 32 stores per wave are not drained: vmcnt counts loads,
// stores and LDS-DMA together in issue order, so the first two K-tiles of
// the next tile wait with vmcnt(16 + 32) where they would wait vmcnt(16).
// Tiles are assigned statically (workgroup b: tiles b, b + G, b + 2G, ...,
// G = grid, a multiple of 8 so a tile stays on map_tile's XCD): every
// workgroup must be resident at once (one per CU) — the host launches it only
// for grids of >= 2 tiles per workgroup on an unmasked device.
template <int N>
__device__ __forceinline__ void wait_vm_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct Src {  // one output tile's operand sources
  u32x4 ra;           // A at row m0, K = 0
  const char* Bb;     // B at row 0, column n0
  long long b_bytes;  // bytes from Bb to the end of B's extent
};

__device__ __forceinline__ Src tile_src(const GemmArgs& a, int bz, int tm, int tn) {
  const int m0 = tm * BM, n0 = tn * BN;
  Src s;
  s.ra = make_rsrc((const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda) * 2,
                   ((long long)(a.M - m0 - 1) * a.lda + a.K) * 2);
  s.Bb = (const char*)a.B + ((long long)bz * a.sB + n0) * 2;
  s.b_bytes = ((long long)(a.kb - 1) * a.ldb + (a.N - n0)) * 2;
  return s;
}

__device__ __forceinline__ u32x4 src_b(const Src& s, int kt, int ldb2) {
  const long long off = (long long)kt * BK * ldb2;
  return make_rsrc(s.Bb + off, s.b_bytes - off);
}

// ktile with explicit DMA targets (A of the item "t+2": descriptor raT at K
// byte offset kaT; B of "t+3": descriptor rbT at its K-tile) and wait counts
// (W0 at Bar0, W1 at Bar_mid); otherwise ktile<DT, 64, SO> item for item.
// ZERO (K-tile 0 of a tile): the first MFMA of every accumulator takes C = 0.
// DIAG (timing-only experiment builds, WRONG results; the power attribution
// of VERDICT r4 #8, scripts/power_attrib.py): bit 0 drops the fragment reads
// (the MFMAs keep re-using the registers they hold), bit 1 the LDS-DMA refills;
// every MFMA, wait and barrier stays.
// LN (experiments, round 6: kMfmaW4SLean): the descriptors are the tile's, at
// K = 0 (rbT: B's; built once per tile), the K-tile offsets ride in the
// voffsets (kaT for A, kbT for B: one VALU add each per K-tile instead of
// a soffset add per A piece and a new B descriptor per K-tile), and outside
// the first two K-tiles (W0 48, dma16_at_pad) each piece is fused with its
// gap's MFMA (mfma_dma_w4: no s_nop).
template <int DT, int SO, int W0, int W1, bool ZERO = false, int DIAG = 0, bool LN = false>
__device__ __forceinline__ void ktile_s(const Ctx& c, const char* smem, u32x4 raT, uint32_t kaT,
                                        u32x4 rbT, f32x4 (&acc)[8][8], Frag (&A)[8], Frag& A7c,
                                        Frag& A7n, Frag (&Bc)[8], Frag (&Bn)[8], uint32_t kbT = 0) {
  constexpr int IL = 64;
  constexpr int SN = STAGE - SO;
  constexpr int sn = SN / STAGE;
  const uint32_t vA = LN ? c.voffA + kaT : c.voffA, vB = LN ? c.voffB + kbT : c.voffB;
  const uint32_t kaS = LN ? 0u : kaT;  // the A soffsets' K part
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    if (mi == 0) {
      wait_vm_lgkm_barrier<W0>();
      __builtin_amdgcn_sched_barrier(0);
    } else if (mi == 4) {
      wait_vm_lgkm_barrier<W1>();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int gap = 0; gap < 16; ++gap) {
      const int ks = gap >> 3, ni = gap & 7;
      const int it = kItems[mi][gap];
      if constexpr (LN && W0 != 48 && !(DIAG & 2) && !ZERO) {
        if (it == 1) {  // the gap's MFMA and DMA piece in one asm block
          const int h = piece_of(mi, gap);
          const s16x8& av = mi == 7 ? A7c.k[ks] : A[mi].k[ks];
          if (h < 8) {
            mfma_dma_w4<DT>(acc[mi][ni], Bc[ni].k[ks], av, raT, vA, (uint32_t)(h * 32 * c.lda2), c.lds0w,
                            SO + h * 32 * 128);
          } else {
            const int nq = (h - 8) >> 2, kb = (h - 8) & 3;
            mfma_dma_w4<DT>(acc[mi][ni], Bc[ni].k[ks], av, rbT, vB, (uint32_t)(kb * 16 * c.ldb2 + nq * IL * 2),
                            c.lds0w, SN + A_BYTES + nq * BH_BYTES + kb * 16 * 256);
          }
          __builtin_amdgcn_sched_barrier(0);
          continue;
        }
      }
      if (ZERO && ks == 0)
        mfma_zero<DT>(acc[mi][ni], Bc[ni].k[ks], mi == 7 ? A7c.k[ks] : A[mi].k[ks]);
      else
        mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], mi == 7 ? A7c.k[ks] : A[mi].k[ks]);
      if ((DIAG & 2) && it == 1) {
        // no refill (timing-only)
      } else if ((DIAG & 1) && it >= 100) {
        // no fragment read (timing-only)
      } else if (it == 1) {
        const int h = piece_of(mi, gap);
        if (h < 8) {
          // the first two K-tiles of a tile (W0 48): soffsets hipcc may have
          // just restored with v_readlane (common.h dma16_at_pad)
          if constexpr (W0 == 48)
            dma16_at_pad(raT, vA, kaS + (uint32_t)(h * 32 * c.lda2), c.lds0w, SO + h * 32 * 128);
          else
            dma16_at(raT, vA, kaS + (uint32_t)(h * 32 * c.lda2), c.lds0w, SO + h * 32 * 128);
        } else {
          const int nq = (h - 8) >> 2, kb = (h - 8) & 3;
          if constexpr (W0 == 48)
            dma16_at_pad(rbT, vB, (uint32_t)(kb * 16 * c.ldb2 + nq * IL * 2), c.lds0w,
                         SN + A_BYTES + nq * BH_BYTES + kb * 16 * 256);
          else
            dma16_at(rbT, vB, (uint32_t)(kb * 16 * c.ldb2 + nq * IL * 2), c.lds0w,
                     SN + A_BYTES + nq * BH_BYTES + kb * 16 * 256);
        }
      } else if (it >= 100 && it < 200) {
        const int s = (it - 100) >> 1, h = (it - 100) & 1;
        Bn[s].k[h] = frag_b<IL>(smem, c.boff[sn][bjj<IL>(s)], s, h);
      } else if (it >= 214) {
        const int h = it - 214;
        A7n.k[h] = frag_a(smem, c.aoff[sn][h], 7);
      } else if (it >= 200) {
        const int m = (it - 200) >> 1, h = (it - 200) & 1;
        A[m].k[h] = frag_a(smem, c.aoff[sn][h], m);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// TRACE (kMfmaW4STrace): each workgroup stamps its start and end (after the
// final drain) into the tile-trace row blockIdx.x, for the per-XCD tail.
// DIAG: ktile_s's bits, plus bit 2: no C stores — 32 out-of-range LDS-DMA
// loads per wave in their place, as before the first tile, so every vmcnt
// wait counts the same (timing-only, WRONG results).
// SUB: map_tile's XCD sub-block shape (0 = 4 x 8; 1 = 8 x 4 and 2 = 2 x 16 are
// the tile-order A/Bs of kMfmaW4STall / kMfmaW4SWide).
template <int DT, int TRACE = 0, bool NTS = true, int DIAG = 0, int SUB = 0, bool LN = false>  // NTS: non-temporal C stores (false: A/B)
__global__ void __launch_bounds__(NT, 1) gemm_w4s(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 4 * kEpiBuf];
  TileTrace tr;
  if constexpr (TRACE) tr.t[0] = tile_clock();
  constexpr int IL = 64;
  // tile_end > 0: the whole-wave part of a tile-range tail plan
  const int T = a.tile_end > 0 ? a.tile_end : a.tiles_m * a.tiles_n * a.batch;
  const int G = gridDim.x;
  int vb = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lds0w = c.lds0 + wu * 1024;
  c.lda2 = a.lda * 2;
  c.ldb2 = a.ldb * 2;
  c.nk = a.K / BK;
  {
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;
    c.voffA = (uint32_t)(r * c.lda2 + ((lc8 ^ ((r >> 1) & 7)) * 16));
    const int lr16 = lane >> 4, lc16 = lane & 15;
    const int k = wu * 4 + lr16;
    const int s = (k & 3) | (((k >> 3) & 1) << 2);
    const int p = ((lc16 >> 1) ^ s) * 16 + (lc16 & 1) * 8;
    const int n = (p / IL) * 2 * IL + (p % IL);
    c.voffB = (uint32_t)(k * c.ldb2 + n * 2);
    const int swA = (l16 >> 1) & 7;
    const int q4 = l16 >> 2, p4 = l16 & 3;
    const int sB = q4 | ((g & 1) << 2);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint32_t ao = (uint32_t)(st * STAGE + (wr * 128 + l16) * 128 + (((4 * ks + g) ^ swA) * 16));
        asm volatile("" : "+v"(ao));
        c.aoff[st][ks] = ao;
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int u = 4 * wc + jj;
        uint32_t bo = (uint32_t)(st * STAGE + (8 * g + q4) * 256 + ((u ^ sB) * 32) + p4 * 8);
        asm volatile("" : "+v"(bo));
        c.boff[st][jj] = bo;
      }
    }
  }
  const int nk = c.nk;

  int bz, tm, tn;
  map_tile(a, vb, bz, tm, tn, SUB);
  Src cur = tile_src(a, bz, tm, tn);
  int nvb = vb + G, nbz = bz, ntm = tm, ntn = tn;
  Src nxt = cur;
  if (nvb < T) {
    map_tile(a, nvb, nbz, ntm, ntn, SUB);
    nxt = tile_src(a, nbz, ntm, ntn);
  }

  f32x4 acc[8][8];  // started by each tile's K-tile 0 (ktile_s ZERO)

  // Prologue of the first tile, as W4's: A(0), B(0) -> stage 0; B(1), A(1)
  // -> stage 1; fragments of K-tile 0; then B(2) -> stage 0.B.
  auto dma_a = [&](const u32x4& ra, uint32_t ka, int so, int h) {
    dma16_at(ra, c.voffA, ka + (uint32_t)(h * 32 * c.lda2), c.lds0w, so + h * 32 * 128);
  };
  auto dma_b = [&](const u32x4& rb, int so, int h) {
    const int nq = (h - 8) >> 2, kb = (h - 8) & 3;
    dma16_at(rb, c.voffB, (uint32_t)(kb * 16 * c.ldb2 + nq * IL * 2), c.lds0w,
             so + A_BYTES + nq * BH_BYTES + kb * 16 * 256);
  };
  {
    const u32x4 rb0 = src_b(cur, 0, c.ldb2), rb1 = src_b(cur, 1, c.ldb2);
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      if (h < 8)
        dma_a(cur.ra, 0u, 0, h);
      else
        dma_b(rb0, 0, h);
    }
#pragma unroll
    for (int h = 8; h < 16; ++h) dma_b(rb1, STAGE, h);
#pragma unroll
    for (int h = 0; h < 8; ++h) dma_a(cur.ra, BK * 2, STAGE, h);
  }
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  Frag A[8], A7a, A7b, B0[8], B1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      A[i].k[ks] = frag_a(smem, c.aoff[0][ks], i);
      B0[i].k[ks] = frag_b<IL>(smem, c.boff[0][bjj<IL>(i)], i, ks);
    }
  A7a = A[7];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  {
    const u32x4 rb2 = src_b(cur, 2, c.ldb2);
#pragma unroll
    for (int h = 8; h < 16; ++h) dma_b(rb2, 0, h);
  }

  char* ebuf = smem + 2 * STAGE + wu * kEpiBuf;
  // 32 out-of-range LDS-DMA loads (num_records 0: no memory access; zeros
  // into this wave's epilogue buffer) in the place of the 32 epilogue stores
  // that precede every later tile's first K-tile: every tile, the first one
  // included, then runs the same code with the same vmcnt counts.
  {
    u32x4 nul;
    nul.x = 0u;
    nul.y = 0u;
    nul.z = 0u;
    nul.w = 0x00020000u;
    const uint32_t eb = c.lds0 + 2 * STAGE + wu * kEpiBuf;
#pragma unroll
    for (int i = 0; i < 32; ++i) dma16_m0(nul, 0u, 0u, eb);
  }
  for (;;) {
    const bool more = nvb < T;
    // DMA targets of item "kt" (A: t+2, B: t+3): this tile, the next, or
    // (last tile) a harmless re-read of this tile's last K-tile. Scalar
    // selects, then one descriptor: no branch in the MFMA stream.
    // 32-bit bitwise selects (m = all ones: this tile) stay on the SALU
    auto sel = [](uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); };
    auto tgt_a = [&](int kt, u32x4& r, uint32_t& ka) {
      const uint32_t m = (kt < nk || !more) ? ~0u : 0u;
      const int k = kt < nk ? kt : (more ? kt - nk : nk - 1);
      r.x = sel(m, cur.ra.x, nxt.ra.x);
      r.y = sel(m, cur.ra.y, nxt.ra.y);
      r.z = sel(m, cur.ra.z, nxt.ra.z);
      r.w = cur.ra.w;
      ka = (uint32_t)k * (BK * 2);
    };
    auto tgt_b = [&](int kt) -> u32x4 {
      const uint32_t m = (kt < nk || !more) ? ~0u : 0u;
      const int k = kt < nk ? kt : (more ? kt - nk : nk - 1);
      const unsigned long long pc = (unsigned long long)cur.Bb, pn = (unsigned long long)nxt.Bb;
      const unsigned long long bc = (unsigned long long)cur.b_bytes, bn = (unsigned long long)nxt.b_bytes;
      const unsigned long long p = ((unsigned long long)sel(m, (uint32_t)(pc >> 32), (uint32_t)(pn >> 32)) << 32) |
                                   sel(m, (uint32_t)pc, (uint32_t)pn);
      const long long bytes = (long long)(((unsigned long long)sel(m, (uint32_t)(bc >> 32), (uint32_t)(bn >> 32)) << 32) |
                                          sel(m, (uint32_t)bc, (uint32_t)bn));
      const long long off = LN ? 0 : (long long)k * BK * c.ldb2;  // LN: K-tile offset in the voffset
      return make_rsrc((const char*)p + off, bytes - off);
    };
    auto tgt_kb = [&](int kt) -> uint32_t {  // LN: B's K-tile byte offset of item kt
      const int k = kt < nk ? kt : (more ? kt - nk : nk - 1);
      return (uint32_t)k * (uint32_t)(BK * c.ldb2);
    };
    const u32x4 rb0 = make_rsrc(cur.Bb, cur.b_bytes);  // LN: this tile's B from K = 0
    auto bsrc = [&](int kt) { return LN ? rb0 : src_b(cur, kt, c.ldb2); };
    auto bkoff = [&](int kt) { return LN ? (uint32_t)kt * (uint32_t)(BK * c.ldb2) : 0u; };
    // K-tiles 0 and 1 (32 stores or dummies per wave are younger than the
    // DMAs they wait for), then pairs whose DMA targets stay in this tile
    // (W4's instruction mix: no selects), then the last two pairs, whose
    // targets cross into the next tile (nk >= 6: host-checked).
    constexpr int KD = DIAG & 3;
    ktile_s<DT, 0, 48, 48, true, KD, LN>(c, smem, cur.ra, 2 * (BK * 2), bsrc(3), acc, A, A7a, A7b, B0, B1,
                                         bkoff(3));
    ktile_s<DT, STAGE, 48, 16, false, KD, LN>(c, smem, cur.ra, 3 * (BK * 2), bsrc(4), acc, A, A7b, A7a, B1,
                                              B0, bkoff(4));
    int t = 2;
    for (; t + 4 < nk; t += 2) {
      ktile_s<DT, 0, 16, 16, false, KD, LN>(c, smem, cur.ra, (uint32_t)(t + 2) * (BK * 2), bsrc(t + 3), acc, A,
                                            A7a, A7b, B0, B1, bkoff(t + 3));
      ktile_s<DT, STAGE, 16, 16, false, KD, LN>(c, smem, cur.ra, (uint32_t)(t + 3) * (BK * 2), bsrc(t + 4), acc,
                                                A, A7b, A7a, B1, B0, bkoff(t + 4));
    }
    for (; t < nk; t += 2) {
      u32x4 ra;
      uint32_t ka;
      tgt_a(t + 2, ra, ka);
      ktile_s<DT, 0, 16, 16, false, KD, LN>(c, smem, ra, ka, tgt_b(t + 3), acc, A, A7a, A7b, B0, B1,
                                            LN ? tgt_kb(t + 3) : 0u);
      tgt_a(t + 3, ra, ka);
      ktile_s<DT, STAGE, 16, 16, false, KD, LN>(c, smem, ra, ka, tgt_b(t + 4), acc, A, A7b, A7a, B1, B0,
                                                LN ? tgt_kb(t + 4) : 0u);
    }
    // The last MFMAs write their AGPRs before the epilogue reads them (asm
    // MFMAs are invisible to hipcc's hazard recognizer).
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
    // lane id from v_mbcnt (no live-in): the store offsets are formed here
    // instead of being kept live through the K-loop (where they spilled)
    unsigned all = ~0u;
    asm volatile("" : "+s"(all));  // per tile, so the mbcnt is not hoisted either
    const int eln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
    if constexpr (DIAG & 4) {  // timing-only: 32 no-access loads for the 32 stores
      u32x4 nul;
      nul.x = 0u;
      nul.y = 0u;
      nul.z = 0u;
      nul.w = 0x00020000u;
      const uint32_t eb = c.lds0 + 2 * STAGE + wu * kEpiBuf;
#pragma unroll
      for (int i = 0; i < 32; ++i) dma16_m0(nul, 0u, 0u, eb);
      (void)Cb;
      (void)eln;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[i][j];
        store_block16<DT, false, false, 8, NTS>(ebuf, v, 1.0f, Cb, (long long)a.ldc * 2,
                                                tm * BM + wr * 128 + i * 16, tn * BN + wc * 128, a.M,
                                                a.N, eln);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!more) break;
    vb = nvb;
    bz = nbz;
    tm = ntm;
    tn = ntn;
    cur = nxt;
    nvb = vb + G;
    if (nvb < T) {
      map_tile(a, nvb, nbz, ntm, ntn, SUB);
      nxt = tile_src(a, nbz, ntm, ntn);
    }
  }
  // No LDS-DMA may still be writing when this workgroup's LDS is handed on.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (TRACE) {
    tr.t[1] = tr.t[2] = tr.t[3] = tile_clock();
    tile_trace_write(a, tr, blockIdx.x, 0, 0);
  }
}

}  // namespace kw4

// Edge tiles (M or N not a multiple of 256): rows of A past M read zeros
// through the descriptor's extent; B columns past N read the next row's
// elements (or zeros past the end) and only feed C columns the masked
// epilogue drops. N % 8: 16-B B rows for the LDS-DMA.
bool gemm_w4_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (dt != kBF16 && dt != kF16) return false;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.N % 8 || a.K % 64) return false;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 4) return false;
  if (a.lda < a.K || a.ldb < a.N || a.ldc < a.N) return false;
  if (a.batch > 1 && (a.sA % 8 || a.sB % 8 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 8) return false;
  // 32-bit offsets: A rows up to 255 * lda (+ K bytes of the tile offset),
  // B rows up to 63 * ldb (+ 128 B of the half offset).
  if ((long long)256 * a.lda * 2 + (long long)a.K * 2 >= (1LL << 31)) return false;
  if ((long long)64 * a.ldb * 2 + 128 >= (1LL << 31)) return false;
  return true;
}

// kMfmaW4SLean's 32-bit voffsets carry the K-tile offset: A's 256 rows plus
// its whole K, and B's K + 128 rows, must stay below 2^31 bytes.
bool gemm_w4s_lean_fits(const GemmArgs& a) {
  return (long long)256 * a.lda * 2 + (long long)a.K * 2 < (1LL << 31) &&
         (long long)(a.K + 128) * a.ldb * 2 < (1LL << 31);
}

hipError_t gemm_w4_launch(int dt, GemmArgs a, hipStream_t stream, int sub) {
  a.tiles_m = (a.M + kw4::BM - 1) / kw4::BM;  // edge tiles: masked epilogue
  a.tiles_n = (a.N + kw4::BN - 1) / kw4::BN;
  const int S = a.splitk > 1 ? a.splitk : 1;
  const long long all_tiles = (long long)a.tiles_m * a.tiles_n * a.batch;
  // tile-range launches (GemmArgs::tile_end / tile_span): plain W4 (sub 0) for
  // a range, plain W4 or W4S (sub 7) for the leading whole waves
  if (a.tile_span < 0 || a.tile_base < 0 || a.tile_end < 0 || a.tile_end > all_tiles ||
      (a.tile_span > 0 && (sub != 0 || a.sig || (long long)a.tile_base + a.tile_span > all_tiles)) ||
      (a.tile_end > 0 && (a.tile_span > 0 || a.sig || (sub != 0 && sub != 7))))
    return hipErrorInvalidValue;
  const long long tiles = a.tile_span > 0 ? a.tile_span : a.tile_end > 0 ? a.tile_end : all_tiles;
  if (S > 1) {
    const int nk = a.K / kw4::BK;
    a.kt_per = (nk + S - 1) / S;
    if ((S - 1) * a.kt_per >= nk || !a.part || !a.flags || tiles > kMaxSplitTiles)
      return hipErrorInvalidValue;  // every slice must own >= 1 K-tile
  } else {
    a.splitk = 1;
  }
  // The grid's batch is batch x S (slice innermost); the XCD-aware order is
  // chosen from the per-element tile grid as before.
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const long long nblocks = tiles * S;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblocks), block(kw4::NT);
#ifdef PDMB_EXPERIMENTS
  if (dt == kBF16 && sub == 1) {
    hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 1>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16 && sub == 2) {
    hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 2>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16 && sub == 3) {
    hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 0, 32>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16 && sub == 4) {
    hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 0, 64, 1>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16 && sub == 12) {  // kMfmaW4Unfused: the epilogue after the last K-tile
    hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 0, 64, 0, false>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16 && sub == 6) {  // persistent + tile timeline
    if (S > 1 || !a.queue) return hipErrorInvalidValue;
    const unsigned g = (unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid);
    hipLaunchKernelGGL((kw4::gemm_w4_pers<kBF16, 1>), dim3(g), block, 0, stream, a);
    return hipGetLastError();
  }
#endif
#ifdef PDMB_EXPERIMENTS
  if (sub == 11) {  // W4S with plain (temporal) C stores
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, false>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub == 9) {  // W4S with the per-round rotating XCD block map (supertile 6)
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    if (a.supertile == 1) a.supertile = 6;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL((kw4::gemm_w4s<kBF16>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub == 10) {  // the same with per-workgroup start / end stamps
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    if (a.supertile == 1) a.supertile = 6;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 1>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub >= 13 && sub <= 16) {  // W4S power attribution (timing-only): DIAG 1, 2, 4, 3
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6 ||
        dt != kBF16)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (sub == 13) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 1>), pg, block, 0, stream, a);
    if (sub == 14) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 2>), pg, block, 0, stream, a);
    if (sub == 15) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 4>), pg, block, 0, stream, a);
    if (sub == 16) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 3>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub == 21 || sub == 22) {  // W4S / W4 with mode 3's rounds as an 8 x 1 XCD grid of 4 x 8 (supertile 9)
    if (a.supertile == 3) a.supertile = 9;
    if (sub == 22) {
      if (S > 1 || dt != kBF16) return hipErrorInvalidValue;
      hipLaunchKernelGGL(kw4::gemm_w4_nn<kBF16>, grid, block, 0, stream, a);
      return hipGetLastError();
    }
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6 ||
        dt != kBF16)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL((kw4::gemm_w4s<kBF16>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub >= 17 && sub <= 20) {  // W4S tile-order A/Bs: 8x4 / 2x16 sub-blocks, snake / M-fastest rounds
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6 ||
        dt != kBF16)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (sub == 17) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 0, 1>), pg, block, 0, stream, a);
    if (sub == 18) hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 0, 2>), pg, block, 0, stream, a);
    if (sub == 19 || sub == 20) {
      if (a.supertile == 1) a.supertile = sub == 19 ? 7 : 8;
      hipLaunchKernelGGL((kw4::gemm_w4s<kBF16>), pg, block, 0, stream, a);
    }
    return hipGetLastError();
  }
  if (sub == 24) {  // kMfmaW4SThin: W4S with the aspect-following thin round
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    a.supertile = thin_supertile(a.tiles_m, a.tiles_n);
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (dt == kBF16)
      hipLaunchKernelGGL((kw4::gemm_w4s<kBF16>), pg, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kw4::gemm_w4s<kF16>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub == 23) {  // kMfmaW4SLean: W4S on the lean DMA issue (bf16 / fp16)
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6 ||
        !gemm_w4s_lean_fits(a))
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (dt == kBF16)
      hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 0, true, 0, 0, true>), pg, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kw4::gemm_w4s<kF16, 0, true, 0, 0, true>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
  if (sub == 8) {  // W4S with per-workgroup start / end stamps
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL((kw4::gemm_w4s<kBF16, 1>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
#endif
  if (sub == 7) {  // W4S: streaming persistent, static tiles (nk even, >= 6)
    if (S > 1 || a.pers_grid <= 0 || a.pers_grid % 8 || (a.K / kw4::BK) % 2 || a.K / kw4::BK < 6)
      return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (dt == kBF16)
      hipLaunchKernelGGL((kw4::gemm_w4s<kBF16>), pg, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kw4::gemm_w4s<kF16>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
#ifdef PDMB_EXPERIMENTS
  if (sub == 5) {  // persistent (per-XCD work queues), unsplit only
    if (S > 1 || !a.queue || a.pers_grid <= 0) return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (dt == kBF16)
      hipLaunchKernelGGL((kw4::gemm_w4_pers<kBF16>), pg, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kw4::gemm_w4_pers<kF16>), pg, block, 0, stream, a);
    return hipGetLastError();
  }
#endif
  if (sub != 0) return hipErrorInvalidValue;
  if (a.sig) {  // completion signals (overlap schedules)
    if (!a.sig_host || a.sig_rows <= 0 || a.sig_slots * a.sig_rows < a.tiles_m ||
        (long long)a.ldc * 2 * 16 >= (1LL << 31))
      return hipErrorInvalidValue;
    if (dt == kBF16)
      hipLaunchKernelGGL((kw4::gemm_w4_nn<kBF16, 0, 64, 0, true, true>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kw4::gemm_w4_nn<kF16, 0, 64, 0, true, true>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16)
    hipLaunchKernelGGL(kw4::gemm_w4_nn<kBF16>, grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL(kw4::gemm_w4_nn<kF16>, grid, block, 0, stream, a);
  return hipGetLastError();
}

}  // namespace pdmb
