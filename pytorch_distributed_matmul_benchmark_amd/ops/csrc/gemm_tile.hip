// gemm_tile.hip — bf16 / fp16 C = A @ B (row-major NN, fp32 accumulate) and
// fp8 e4m3 C = alpha * (A @ B) (A row-major, B column-major, bf16 out): the
// one-barrier LDS-DMA tile family for grids that under-fill the 256 CUs with
// W4's 256x256 tiles. Members (Cfg<BM, BN, NS>):
//   T128      128 x 128, 4-stage ring, 1 workgroup / CU
//   T128x2    128 x 128, 2-stage ring, 2 workgroups / CU (A/B)
//   T256x128  256 x 128, 3-stage ring, 1 workgroup / CU
//
// Why: matrix_parallel's per-rank column shards at ws >= 2 of the reference's
// default sizes (matmul_scaling_benchmark.py:179-188 at :351-352) include
// [4096^2] @ [4096 x 512] (32 256x256 tiles), [8192^2] @ [8192 x 1024] and
// [4096^2] @ [4096 x 2048] (128 each); 2048^3 has 64. W4 (gemm_w4.hip) leaves
// most CUs idle there, and splitting K over 256x256 tiles costs a 256 KiB
// fp32 slab per slice to combine (profiles/r2_t128_splitk_sweep.jsonl). The
// smaller tiles give 2x / 4x the workgroups with the same LDS images and MFMA
// idiom, and smaller split-K slabs.
//
// Structure (W4's idioms, one barrier per K-tile):
//  * 4 waves, one per SIMD, as 2 x 2, each owning a (BM/2) x 64 output block
//    (MB x NB MFMA 16x16x32 blocks, MB = BM/32, NB = 4; fp32 accumulators in
//    AGPRs; operands swapped so the accumulator holds C^T).
//  * LDS images per stage: A [BM rows][128 B] with 16-B chunk c at
//    c ^ ((row >> 1) & 7); B [64 k][256 B] with 32-B unit u (16 columns) at
//    u ^ ((k & 3) | ((k >> 3) & 1) << 2), read transposed by ds_read_b64_tr_b16
//    (the NN B operand, no transposed copy). Both are W4's conflict-free
//    layouts (A: W4's image at BM rows; B: one W4 B half without its column
//    interleave).
//  * NS-stage ring filled by LDS-DMA (buffer_load ... lds): during K-tile t
//    the workgroup refills t's stage with tile t + NS, so each tile has
//    ~NS-1 K-tiles of flight.
//  * One barrier per K-tile: s_waitcnt vmcnt(P * (NS-2)) (tile t+1 landed;
//    later tiles may be in flight; P DMA pieces per wave per K-tile)
//    lgkmcnt(0) (this wave's reads of tile t's fragments done) then
//    s_barrier; after it t's stage is free and t+1's readable. Fragments of
//    t+1 are read during t's MFMAs into a second register set.
//  * Every load sits in an MFMA gap (Sched: B fragments, A fragments and DMA
//    pieces spread over the K-tile's MFMA gaps, at most one per gap).
//  * Optional split-K over K-tile ranges with the in-launch combine of
//    splitk.h.
//
// fp8 (DT = kFP8; kFp8T128 / kFp8T256x128): a K-tile is 128 e4m3 = 128 B per
// row, so the A image is byte for byte the bf16 one and B (column-major, Bt
// [N,K] rows) is a second A-like image of BN rows; both use gemm_fp8.hip's
// swizzle swz8 (conflict-free for the fp8 fragment: chunks 2g, 2g+1 of a row)
// and ds_read_b128, no transposed read. One v_mfma_f32_16x16x128_f8f6f4 per
// block per K-tile (twice the cycles of the bf16 pair it replaces), so the
// same item schedule runs with the MFMA at every other gap: 16 MFMAs and 24
// loads per K-tile per wave, as many cycles as the bf16 kernel's 32 + 24.
//
// Fast-path constraints (host-checked): N % 8 == 0 (fp8: % 4; M and N edge
// tiles masked at the store), K % 64 == 0 (fp8: K % 128), lda / ldb % 8 == 0
// (fp8: % 16), ldc % 4 == 0, 16-B aligned A / B, 8-B aligned C.
#include "api.h"
#ifdef PDMB_EXPERIMENTS
#include "experiment_ids.h"
#endif
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace ktile {

constexpr int BK = 64;
constexpr int NT = 256;

template <int BM_, int BN_, int NS_, int OCC_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, NS = NS_, OCC = OCC_;
  static_assert(BN == 128 || BN == 192, "B image: 128 columns per k, or three 64-column panels");
  static_assert(BM == 128 || BM == 192 || BM == 256, "A image rows");
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  // bf16 / fp16 B image of a 192-column tile: three 64-column panels (below)
  static constexpr bool PANEL = BN == 192;
  static constexpr int MB = BM / 32, NB = BN / 32;       // 16x16 blocks per wave (2 x 2 waves)
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BK * BN * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int PA = A_BYTES / 4096, PB = B_BYTES / 4096;  // 1 KiB pieces per wave
  static constexpr int P = PA + PB;
  static constexpr int G = MB * NB * 2;                  // MFMAs (gaps) per K-tile per wave
  // the stages, plus (one workgroup per CU) the fused epilogue's wave buffers
  static_assert(NS * STAGE + (OCC == 1 ? 4 * epi_buf<NB>() : 0) <= 160 * 1024 / OCC, "LDS");
};

using CfgT128 = Cfg<128, 128, 4, 1>;
using CfgT128x2 = Cfg<128, 128, 2, 2>;
using CfgT256x128 = Cfg<256, 128, 3, 1>;
// Round 5: 192-row tiles for grids that no 256- or 128-tile cuts into whole
// waves — 3072^2 is 16 x 16 192x192 tiles (one wave of 256 CUs; 144 W4 tiles
// fill 56 %), 2304^2 is 12 x 18 192x128 tiles (84 %; 81 W4 tiles fill 32 %).
using CfgT192 = Cfg<192, 192, 3, 1>;
using CfgT192x128 = Cfg<192, 128, 3, 1>;

// Item schedule of one K-tile: which load follows MFMA `gap`. Three classes —
// B fragment halves (2 NB, each two ds_read_b64_tr_b16), A fragment halves
// (2 MB, ds_read_b128) and DMA pieces (P) — are spread Bresenham-style so each
// class stays within one item of its even share of the gaps; at most one item
// per gap. Encoding: 0 none; 1 + piece; 100 + (2j + half) B; 200 + (2m + half) A.
template <class C>
struct Sched {
  int item[C::G];
  constexpr Sched() : item() {
    const int T[3] = {2 * C::NB, 2 * C::MB, C::P};
    int n[3] = {0, 0, 0};
    for (int g = 0; g < C::G; ++g) {
      int best = -1, bd = 0;
      for (int k = 0; k < 3; ++k) {
        const int d = T[k] * (g + 1) - n[k] * C::G;  // deficit vs the even share (x G)
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
  constexpr int issued(int base, int lo, int hi) const {
    int c = 0;
    for (int g = 0; g < C::G; ++g) c += (item[g] >= lo && item[g] < hi) ? 1 : 0;
    return c + base;
  }
};

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

// fp8: one 16x16x128 e4m3 MFMA on a block's whole fragment (k[0] | k[1]).
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void mfma_acc_f8(f32x4& acc, const s16x8 (&b)[2], const s16x8 (&a)[2]) {
  const s16x8 bv[2] = {b[0], b[1]}, av[2] = {a[0], a[1]};
  const i32x8 bb = __builtin_bit_cast(i32x8, bv), aa = __builtin_bit_cast(i32x8, av);
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(acc) : "v"(bb), "v"(aa));
}

// fp8 row swizzle (gemm_fp8.hip swz): 16-B chunk c of 128-B row r at c ^ swz8(r);
// depends on r & 15 only.
__host__ __device__ __forceinline__ int swz8(int r) {
  return ((r >> 1) & 7) ^ ((((r & 15) - 4) & 15) < 8 ? 2 : 0);
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

// Top-of-K-tile wait (N = P * (NS - 2): pieces of tiles t+2 .. t+NS-1 may be in
// flight, tile t+1's have landed) and the prologue's (N = P * (NS - 1)).
template <int N>
__device__ __forceinline__ void wait_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct Frag {  // one 16-row (A) or 16-column (B) block of a K-tile: k 0..31 and 32..63
  s16x8 k[2];
};

template <class C>
struct Ctx {
  u32x4 ra;               // A descriptor at this slice's first K
  u32x4 rb;               // fp8: Bt descriptor at this slice's first K (row n0)
  const char* Bb;         // B at this slice's first K row, column n0
  long long b_bytes;      // bytes from Bb to the end of B's extent
  int lda2, ldb2, nk;     // leading dims in bytes, K-tiles of this slice
  uint32_t voffA, voffB;  // per-lane DMA offsets of piece 0
  uint32_t aoff[2];       // per-lane A fragment offsets in stage 0, [ks]
  uint32_t boff[C::NB];   // per-lane B fragment offsets in stage 0, [block j] (fp8: [half])
  int wu;
  uint32_t lds0;
};

template <class C>
__device__ __forceinline__ u32x4 b_rsrc(const Ctx<C>& c, int tile) {
  const long long off = (long long)tile * BK * c.ldb2;
  return make_rsrc(c.Bb + off, c.b_bytes - off);
}

// DMA piece h (0 .. P-1) of K-tile `tile` into the stage at byte offset `so`.
// h < PA: A rows h*32 + wu*8 + [0,8) (8 x 128 B); else B k rows
// (h-PA)*16 + wu*4 + [0,4) (4 x 256 B). The swizzles depend on (row >> 1) & 7
// (A) and k & 11 (B) only, which those row offsets leave alone, so one
// per-lane offset serves every piece.
//
// PANEL (BN = 192, bf16 / fp16): B is three images of 64 columns, [64 k][128
// B] each (panel p: columns 64p .. 64p+63 at A_BYTES + 8 KiB p), 32-B unit v
// (16 columns) of row k holding column unit v ^ s(k), s(k) = ((k >> 1) & 1) |
// ((k >> 3) & 1) << 1. A 128-B row pitch puts rows of one parity on one half of
// the 64 banks; a ds_read_b64_tr_b16 half-wave reads rows 8g + q4 (g = 0, 1;
// q4 = 0..3), i.e. four rows per parity, which s(k) sends to four different
// units: 64 distinct banks, conflict-free. DMA pieces: 8-row groups r of one
// panel (1 KiB each); wave wu takes r = wu and wu + 4 of all three panels, so
// (r & 1) — bit 3 of k — is the wave's own and one per-lane offset serves all
// six pieces.
template <int DT, class C>
__device__ __forceinline__ void issue_piece(const Ctx<C>& c, u32x4 rb, uint32_t so, int tile, int h) {
  if constexpr (DT == kFP8) {  // A / Bt rows h' * 32 + wu * 8 + [0,8), K at tile * 128 B
    if (h < C::PA)
      dma16_m0(c.ra, c.voffA, (uint32_t)tile * 128 + (uint32_t)(h * 32 * c.lda2),
               c.lds0 + so + (h * 32 + c.wu * 8) * 128);
    else
      dma16_m0(c.rb, c.voffB, (uint32_t)tile * 128 + (uint32_t)((h - C::PA) * 32 * c.ldb2),
               c.lds0 + so + C::A_BYTES + ((h - C::PA) * 32 + c.wu * 8) * 128);
  } else if (h < C::PA) {
    dma16_m0(c.ra, c.voffA, (uint32_t)tile * (BK * 2) + (uint32_t)(h * 32 * c.lda2),
             c.lds0 + so + (h * 32 + c.wu * 8) * 128);
  } else if constexpr (C::PANEL) {
    const int kb = h - C::PA, pn = kb >> 1, r = c.wu + 4 * (kb & 1);  // panel, 8-row group
    dma16_m0(rb, c.voffB, (uint32_t)(r * 8 * c.ldb2 + pn * 128),
             c.lds0 + so + C::A_BYTES + pn * 8192 + r * 1024);
  } else {
    const int kb = h - C::PA;
    dma16_m0(rb, c.voffB, (uint32_t)(kb * 16 * c.ldb2),
             c.lds0 + so + C::A_BYTES + (kb * 16 + c.wu * 4) * 256);
  }
}

// A fragment half ks of block m (rows 16m..16m+15 of this wave's BM/2).
__device__ __forceinline__ s16x8 frag_a(const char* smem, uint32_t off, int m) {
  return *(const lds_s16x8*)(smem + m * 16 * 128 + off);
}

// B fragment half ks of block j (16 output columns): two transposed reads
// (rows 4 apart; PANEL: 128-B rows within the block's panel, which `off` holds).
template <class C>
__device__ __forceinline__ s16x8 frag_b(const char* smem, uint32_t off, int ks) {
  constexpr int RP = C::PANEL ? 128 : 256;  // B image row pitch
  const char* p = smem + C::A_BYTES + ks * 32 * RP + off;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * RP));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// fp8 B fragment half h of block j (16 output columns = 16 Bt rows).
template <class C>
__device__ __forceinline__ s16x8 frag_b8(const char* smem, uint32_t off, int j) {
  return *(const lds_s16x8*)(smem + C::A_BYTES + j * 16 * 128 + off);
}

// One K-tile: G MFMAs on (Ac, Bc) = fragments of tile t, reading tile t+1's
// fragments into (An, Bn) from stage sn, DMA of tile t + NS into stage sc.
template <int DT, class C>
__device__ __forceinline__ void ktile(const Ctx<C>& c, const char* smem, int t, uint32_t sc,
                                      uint32_t sn, f32x4 (&acc)[C::MB][C::NB], Frag (&Ac)[C::MB],
                                      Frag (&Bc)[C::NB], Frag (&An)[C::MB], Frag (&Bn)[C::NB]) {
  constexpr Sched<C> S{};
  const int td = t + C::NS < c.nk ? t + C::NS : c.nk - 1;  // clamped tail DMAs (harmless re-reads)
  u32x4 rb;
  if constexpr (DT == kFP8) rb = c.rb;
  else rb = b_rsrc(c, td);
  wait_lgkm_barrier<C::P * (C::NS - 2)>();
  __builtin_amdgcn_sched_barrier(0);
  uint32_t ao[2], bo[C::NB];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ao[ks] = c.aoff[ks] + sn;
#pragma unroll
  for (int j = 0; j < C::NB; ++j) bo[j] = c.boff[j] + sn;
#pragma unroll
  for (int gap = 0; gap < C::G; ++gap) {
    constexpr int MN = C::MB * C::NB;
    if constexpr (DT == kFP8) {  // one MFMA per block, at every other gap
      if ((gap & 1) == 0) {
        const int b = gap >> 1, mi = b / C::NB, ni = b % C::NB;
        mfma_acc_f8(acc[mi][ni], Bc[ni].k, Ac[mi].k);
      }
    } else {
      const int ks = gap / MN, mi = (gap % MN) / C::NB, ni = gap % C::NB;
      mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], Ac[mi].k[ks]);
    }
    const int it = S.item[gap];
    if (it >= 200) {
      const int m = (it - 200) >> 1, h = (it - 200) & 1;
      An[m].k[h] = frag_a(smem, ao[h], m);
    } else if (it >= 100) {
      const int j = (it - 100) >> 1, h = (it - 100) & 1;
      if constexpr (DT == kFP8) Bn[j].k[h] = frag_b8<C>(smem, bo[h], j);
      else Bn[j].k[h] = frag_b<C>(smem, bo[j], h);
    } else if (it >= 1) {
      issue_piece<DT, C>(c, rb, sc, td, it - 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The last K-tile of an unsplit tile with the epilogue folded in (as
// gemm_fp8.hip ktile_w4_last): block row mi - 1 leaves through this wave's
// own LDS buffer (past the stages, which tail DMAs may still be writing)
// while block row mi's MFMAs run. MFMAs in block-row order (per accumulator
// the same ks sequence as ktile: bitwise equal); no fragment reads, DMAs or
// barrier. Block mi's MFMAs separate block mi - 1's last accumulator write
// from its AGPR reads.
template <int DT, class C>
__device__ __forceinline__ void ktile_last(f32x4 (&acc)[C::MB][C::NB], const Frag (&Ac)[C::MB],
                                           const Frag (&Bc)[C::NB], char* ebuf, char* Cb, long long ldc_b,
                                           int row0, int col0, int M, int N, float alpha) {
  auto store = [&](int i) {
    unsigned all = ~0u;  // lane id formed here: the stores' addresses are not hoisted
    asm volatile("" : "+s"(all));
    const int eln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
    if constexpr (DT == kFP8)
      store_block16<kBF16, false, true, C::NB>(ebuf, acc[i], alpha, Cb, ldc_b, row0 + i * 16, col0, M, N, eln);
    else
      store_block16<DT, false, false, C::NB>(ebuf, acc[i], 1.0f, Cb, ldc_b, row0 + i * 16, col0, M, N, eln);
  };
#pragma unroll
  for (int mi = 0; mi < C::MB; ++mi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < C::NB; ++ni) {
        if constexpr (DT == kFP8) {
          if (ks == 0) mfma_acc_f8(acc[mi][ni], Bc[ni].k, Ac[mi].k);
        } else {
          mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], Ac[mi].k[ks]);
        }
      }
    __builtin_amdgcn_sched_barrier(0);
    if (mi >= 1) store(mi - 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  store(C::MB - 1);
}

// FUSED: unsplit tiles with an even K-tile count store C during their last
// K-tile (ktile_last; false: the A/B kernels kT128Unfused / kFp8T128Unfused).
template <int DT, class C, bool FUSED = true>
__global__ void __launch_bounds__(NT, C::OCC) gemm_tile_nn(GemmArgs a) {
  // T128x2 (2 workgroups / CU) keeps the separate epilogue: in its 128-register
  // budget the fused last K-tile made hipcc shuffle fragment registers next
  // to the inline-asm MFMAs (wrong results on the GPU).
  constexpr bool kFused = FUSED && C::OCC == 1;
  __shared__ __attribute__((aligned(1024))) char smem[C::NS * C::STAGE + (kFused ? 4 * epi_buf<C::NB>() : 0)];
  constexpr int MB = C::MB, NB = C::NB, NS = C::NS;

  int bz, tm, tn;
  int slice = 0;  // split-K: grid batch = batch x S, slice innermost (as W4)
  if (a.tile_span > 0) {
    // Refined wave-quantisation tail (gemm_dispatch.cpp tail_plan): the tiles
    // [tile_base, +tile_span) of W4's 256x256 order (a.tiles_m / tiles_n /
    // supertile describe that grid), each cut into R = (256/BM) x (256/BN) of
    // this kernel's tiles; block b is part b / span of local tile b % span.
    constexpr int RM = 256 / C::BM, RN = 256 / C::BN;
    const int local = blockIdx.x % a.tile_span, part = blockIdx.x / a.tile_span;
    map_tile(a, a.tile_base + local, bz, tm, tn);
    tm = tm * RM + part / RN;
    tn = tn * RN + part % RN;
    if (tm * C::BM >= a.M || tn * C::BN >= a.N) return;  // a part past an edge tile's rows / columns
  } else {
    map_tile(a, blockIdx.x, bz, tm, tn);
    if (a.splitk > 1) {
      slice = bz % a.splitk;
      bz /= a.splitk;
    }
  }
  const int kt0 = slice * a.kt_per;
  const int m0 = tm * C::BM, n0 = tn * C::BN;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx<C> c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  constexpr int ES = DT == kFP8 ? 1 : 2;       // bytes per element
  constexpr int BKE = DT == kFP8 ? 128 : BK;   // K per K-tile (128 B per row either way)
  c.lda2 = a.lda * ES;
  c.ldb2 = a.ldb * ES;
  {
    const int nk_all = a.K / BKE;
    c.nk = a.splitk > 1 ? min(a.kt_per, nk_all - kt0) : nk_all;
  }
  const int k0 = kt0 * BKE;
  const char* Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda + k0) * ES;
  c.ra = make_rsrc(Ab, ((long long)(a.M - m0 - 1) * a.lda + (a.K - k0)) * ES);
  if constexpr (DT == kFP8) {  // Bt [N,K]: rows n0 .., K-contiguous
    const char* Bt = (const char*)a.B + (long long)bz * a.sB + (long long)n0 * a.ldb + k0;
    c.rb = make_rsrc(Bt, (long long)(a.N - n0 - 1) * a.ldb + (a.K - k0));
    c.Bb = Bt;
    c.b_bytes = 0;
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;  // row of piece 0 (swz8(r + 32h) = swz8(r))
    c.voffA = (uint32_t)(r * c.lda2 + ((lc8 ^ swz8(r)) * 16));
    c.voffB = (uint32_t)(r * c.ldb2 + ((lc8 ^ swz8(r)) * 16));
    const int sw = swz8(l16);  // fragment rows are 16-aligned bases + l16
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t ao = (uint32_t)((wr * (C::BM / 2) + l16) * 128 + (((2 * g + h) ^ sw) * 16));
      uint32_t bo = (uint32_t)((wc * (C::BN / 2) + l16) * 128 + (((2 * g + h) ^ sw) * 16));
      asm volatile("" : "+v"(ao), "+v"(bo));  // opaque: one base VGPR each
      c.aoff[h] = ao;
      c.boff[h] = bo;
    }
#pragma unroll
    for (int j = 2; j < NB; ++j) c.boff[j] = 0u;  // unused by the fp8 reads
  } else {
    c.rb = c.ra;
    c.Bb = (const char*)a.B + ((long long)bz * a.sB + (long long)k0 * a.ldb + n0) * 2;
    c.b_bytes = ((long long)(a.kb - k0 - 1) * a.ldb + (a.N - n0)) * 2;
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;  // row of A piece 0
    c.voffA = (uint32_t)(r * c.lda2 + ((lc8 ^ ((r >> 1) & 7)) * 16));
    if constexpr (C::PANEL) {  // row lane >> 3 of an 8-row group (group parity wu & 1)
      const int kr = lane >> 3;
      const int s = ((kr >> 1) & 1) | ((wu & 1) << 1);
      const int n = ((lc8 >> 1) ^ s) * 16 + (lc8 & 1) * 8;  // column (within the panel) of this lane's 16 B
      c.voffB = (uint32_t)(kr * c.ldb2 + n * 2);
    } else {
      const int lr16 = lane >> 4, lc16 = lane & 15;
      const int k = wu * 4 + lr16;  // k row of B piece 0
      const int s = (k & 3) | (((k >> 3) & 1) << 2);
      const int n = ((lc16 >> 1) ^ s) * 16 + (lc16 & 1) * 8;  // column of this lane's 16 B
      c.voffB = (uint32_t)(k * c.ldb2 + n * 2);
    }
    const int swA = (l16 >> 1) & 7;
    const int q4 = l16 >> 2, p4 = l16 & 3;
    const int sB = C::PANEL ? (((q4 >> 1) & 1) | ((g & 1) << 1)) : (q4 | ((g & 1) << 2));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint32_t ao = (uint32_t)((wr * (C::BM / 2) + l16) * 128 + (((4 * ks + g) ^ swA) * 16));
      asm volatile("" : "+v"(ao));  // opaque: one base VGPR each
      c.aoff[ks] = ao;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int u = NB * wc + j;  // 32-B unit = columns 16u .. 16u+15 of the tile
      uint32_t bo = C::PANEL ? (uint32_t)((u >> 2) * 8192 + (8 * g + q4) * 128 + (((u & 3) ^ sB) * 32) + p4 * 8)
                             : (uint32_t)((8 * g + q4) * 256 + ((u ^ sB) * 32) + p4 * 8);
      asm volatile("" : "+v"(bo));
      c.boff[j] = bo;
    }
  }

  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue: tiles 0 .. NS-1 into stages 0 .. NS-1 (clamped), wait for tile
  // 0 everywhere (tiles 1 .. NS-1 may still fly), read its fragments.
  const int nk = c.nk;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int tl = st < nk ? st : nk - 1;
    u32x4 rb;
    if constexpr (DT == kFP8) rb = c.rb;
    else rb = b_rsrc(c, tl);
#pragma unroll
    for (int h = 0; h < C::P; ++h) issue_piece<DT, C>(c, rb, st * C::STAGE, tl, h);
  }
  wait_barrier<C::P * (NS - 1)>();
  Frag A0[MB], B0[NB], A1[MB], B1[NB];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int i = 0; i < MB; ++i) A0[i].k[ks] = frag_a(smem, c.aoff[ks], i);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if constexpr (DT == kFP8) B0[j].k[ks] = frag_b8<C>(smem, c.boff[ks], j);
      else B0[j].k[ks] = frag_b<C>(smem, c.boff[j], ks);
    }
  }
  // Steady state: K-tile t computes from set (t & 1), reads t+1 into the
  // other set from stage (t+1) % NS, refills stage t % NS with tile t + NS.
  // Fused (unsplit, nk even): the loop stops before K-tile nk-1, whose
  // fragments it leaves in (A1, B1), and ktile_last runs it with the stores.
  const bool split = a.splitk > 1;
  const bool interior = m0 + C::BM <= a.M && n0 + C::BN <= a.N;  // else: masked edge tile
  const bool fuse = kFused && !split && interior && (nk & 1) == 0;
  const int nloop = fuse ? nk - 1 : nk;
  int t = 0;
  for (; t + 1 < nloop; t += 2) {
    ktile<DT, C>(c, smem, t, (uint32_t)((t % NS) * C::STAGE), (uint32_t)(((t + 1) % NS) * C::STAGE),
                 acc, A0, B0, A1, B1);
    ktile<DT, C>(c, smem, t + 1, (uint32_t)(((t + 1) % NS) * C::STAGE),
                 (uint32_t)(((t + 2) % NS) * C::STAGE), acc, A1, B1, A0, B0);
  }
  if (t < nloop)  // odd count: the next tile's reads (fused) or clamped re-reads (the last tile)
    ktile<DT, C>(c, smem, t, (uint32_t)((t % NS) * C::STAGE),
                 (uint32_t)(((fuse ? t + 1 : t) % NS) * C::STAGE), acc, A0, B0, A1, B1);
  if constexpr (kFused) {
    if (fuse) {
      ktile_last<DT, C>(acc, A1, B1, smem + C::NS * C::STAGE + wu * epi_buf<NB>(),
                        (char*)a.C + (long long)bz * a.sC * 2, (long long)a.ldc * 2,
                        m0 + wr * (C::BM / 2), n0 + wc * (C::BN / 2), a.M, a.N, a.alpha);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs landed before the LDS is released
      return;
    }
  }
  // Drain the tail DMAs and give the last MFMAs time to write their AGPRs
  // (asm MFMAs are invisible to hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  SplitSlots sl;
  if (split && !splitk_meet<MB, NB, NT>(a, smem, ((long long)bz * a.tiles_m + tm) * a.tiles_n + tn,
                                        slice, acc, sl))
    return;

  // Epilogue: acc[i][j] holds C^T of a 16x16 block (lane: row l16, columns
  // 4g..4g+3), stored through LDS as whole rows (common.h store_block16;
  // interior tiles only: no masks) once every wave's DMAs have landed and
  // every fragment read is done.
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
  char* ebuf = smem + 1024 + wu * 2 * epi_buf<NB>();  // past splitk_meet's ticket word
  // S == 2: the other slice's rows prefetched a row ahead (splitk.h splitk_load_other)
  // S == 3: both other slices' rows, a row ahead (splitk_load_others3) — in
  // T128 only: its 4 x 4 blocks leave the registers (358 VGPRs, no spills);
  // in T256x128, T128x2 and T192 the two extra row buffers spilled.
  constexpr bool kPf3 = C::BM == 128 && C::BN == 128 && C::NS == 4;
  const bool pf2 = split && a.splitk == 2 && a.meet_prefetch;
  const bool pf3 = kPf3 && split && a.splitk == 3 && a.meet_prefetch;
  f32x4 qa[NB], qb[NB];
  f32x4 ta[2][NB], tb[2][NB];
  if (pf2) splitk_load_other<MB, NB, NT>(sl, slice, 0, qa);
  if constexpr (kPf3)
    if (pf3) splitk_load_others3<MB, NB, NT>(sl, slice, 0, ta);
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    f32x4 v[NB];
    if (!split) {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = acc[i][j];
    } else if (pf2) {
      if (i + 1 < MB) splitk_load_other<MB, NB, NT>(sl, slice, i + 1, (i & 1) ? qa : qb);
      const f32x4(&q)[NB] = (i & 1) ? qb : qa;
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = acc[i][j] + q[j];
    } else if (kPf3 && pf3) {
      if constexpr (kPf3) {
        if (i + 1 < MB) splitk_load_others3<MB, NB, NT>(sl, slice, i + 1, (i & 1) ? ta : tb);
        splitk_sum3<NB>(slice, acc[i], (i & 1) ? tb : ta, v);
      }
    } else {
      splitk_row<MB, NB, NT>(a, sl, slice, i, acc, v);
    }
    char* eb = ebuf + (i & 1) * epi_buf<NB>();
    const int row0 = m0 + wr * (C::BM / 2) + i * 16, col0 = n0 + wc * (C::BN / 2);
    if constexpr (DT == kFP8) {  // alpha (the per-tensor scales), bf16 out
      if (interior)
        store_block16<kBF16, false, true, NB>(eb, v, a.alpha, Cb, (long long)a.ldc * 2, row0, col0, a.M, a.N, lane);
      else
        store_block16<kBF16, true, true, NB>(eb, v, a.alpha, Cb, (long long)a.ldc * 2, row0, col0, a.M, a.N, lane);
    } else {
      if (interior)
        store_block16<DT, false, false, NB>(eb, v, 1.0f, Cb, (long long)a.ldc * 2, row0, col0, a.M, a.N, lane);
      else
        store_block16<DT, true, false, NB>(eb, v, 1.0f, Cb, (long long)a.ldc * 2, row0, col0, a.M, a.N, lane);
    }
  }
}

template <class C, bool FUSED = true>
hipError_t launch(int dt, GemmArgs a, hipStream_t stream) {
  if (a.tile_end != 0 || a.tile_span < 0 || a.tile_base < 0) return hipErrorInvalidValue;
  if (a.tile_span > 0 && (256 % C::BM || 256 % C::BN)) return hipErrorInvalidValue;  // no whole parts
  if (a.tile_span > 0) {  // refined tail: W4's 256x256 tile order, R parts per tile, unsplit
    a.tiles_m = (a.M + 255) / 256;
    a.tiles_n = (a.N + 255) / 256;
    a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
    a.splitk = 1;
    if ((long long)a.tile_base + a.tile_span > (long long)a.tiles_m * a.tiles_n * a.batch)
      return hipErrorInvalidValue;
    constexpr int R = (256 / C::BM) * (256 / C::BN);
    const long long nb = (long long)a.tile_span * R;
    if (nb > 0x7fffffffLL) return hipErrorInvalidValue;
    const dim3 grid((unsigned)nb), block(NT);
    if (dt == kBF16) {
      hipLaunchKernelGGL((gemm_tile_nn<kBF16, C, FUSED>), grid, block, 0, stream, a);
    } else if (dt == kF16) {
      hipLaunchKernelGGL((gemm_tile_nn<kF16, C, FUSED>), grid, block, 0, stream, a);
    } else if (dt == kFP8) {
      if constexpr (C::OCC == 1)
        hipLaunchKernelGGL((gemm_tile_nn<kFP8, C, FUSED>), grid, block, 0, stream, a);
      else
        return hipErrorInvalidValue;
    } else {
      return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  a.tiles_m = (a.M + C::BM - 1) / C::BM;  // edge tiles: masked epilogue
  a.tiles_n = (a.N + C::BN - 1) / C::BN;
  const int S = a.splitk > 1 ? a.splitk : 1;
  if (S > 1) {
    const int nk = a.K / (dt == kFP8 ? 128 : BK);
    a.kt_per = (nk + S - 1) / S;
    if ((S - 1) * a.kt_per >= nk || !a.part || !a.flags ||
        (long long)a.tiles_m * a.tiles_n * a.batch > kMaxSplitTiles)
      return hipErrorInvalidValue;  // every slice must own >= 1 K-tile
  } else {
    a.splitk = 1;
  }
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const long long nblocks = (long long)a.tiles_m * a.tiles_n * a.batch * S;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblocks), block(NT);
  if (dt == kBF16) {
    hipLaunchKernelGGL((gemm_tile_nn<kBF16, C, FUSED>), grid, block, 0, stream, a);
  } else if (dt == kF16) {
    hipLaunchKernelGGL((gemm_tile_nn<kF16, C, FUSED>), grid, block, 0, stream, a);
  } else {
    if constexpr (C::OCC == 1)  // fp8: T128, T256x128
      hipLaunchKernelGGL((gemm_tile_nn<kFP8, C, FUSED>), grid, block, 0, stream, a);
    else
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ktile

// bm x 128 / bm x 192 tiles (bm = 128, 192 or 256).
bool gemm_tile_supported(int dt, int bm, const GemmArgs& a, size_t align_a, size_t align_b,
                         size_t align_c) {
  // Edge tiles (M % bm, N % 128): rows of A (and fp8's Bt) past M / N load
  // zeros through the descriptor extents; bf16 / fp16 B columns past N feed
  // only C columns the masked epilogue drops.
  if (dt == kFP8) {  // A [M,K] row-major, Bt [N,K] row-major, bf16 C
    if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
    if (a.N % 4 || a.K % 128) return false;
    if (a.lda % 16 || a.ldb % 16 || a.ldc % 4) return false;
    if (a.lda < a.K || a.ldb < a.K || a.ldc < a.N) return false;
    if (a.batch > 1 && (a.sA % 16 || a.sB % 16 || a.sC % 4)) return false;
    if (align_a % 16 || align_b % 16 || align_c % 8) return false;
    // 32-bit offsets: rows up to bm-1 (A) / the tile's last Bt row plus the K
    // byte offset. The 192-column fp8 tile (T192, BN = 192) reads Bt rows up
    // to 191; bm = 192 covers both 192-row tiles, so it is bounded by 192.
    const long long bt_rows = bm == 192 ? 192 : 128;
    if ((long long)bm * a.lda + a.K >= (1LL << 31) || bt_rows * a.ldb + a.K >= (1LL << 31))
      return false;
    return true;
  }
  if (dt != kBF16 && dt != kF16) return false;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.N % 8 || a.K % 64) return false;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 4) return false;
  if (a.lda < a.K || a.ldb < a.N || a.ldc < a.N) return false;
  if (a.batch > 1 && (a.sA % 8 || a.sB % 8 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 8) return false;
  // 32-bit offsets: A rows up to bm-1 * lda (+ K bytes of the tile offset),
  // B rows up to 63 * ldb.
  if ((long long)bm * a.lda * 2 + (long long)a.K * 2 >= (1LL << 31)) return false;
  if ((long long)64 * a.ldb * 2 + 64 >= (1LL << 31)) return false;
  return true;
}

// kernel: kT128 | kT128x2 | kT256x128 | kT192 | kT192x128 (bf16 / fp16),
// kFp8T128 | kFp8T256x128 | kFp8T192 | kFp8T192x128 (fp8)
hipError_t gemm_tile_launch(int kernel, int dt, GemmArgs a, hipStream_t stream) {
  bool fp8 = kernel == kFp8T128 || kernel == kFp8T256x128 || kernel == kFp8T192 || kernel == kFp8T192x128;
#ifdef PDMB_EXPERIMENTS
  fp8 = fp8 || kernel == kFp8T128Unfused;
#endif
  if ((dt == kFP8) != fp8) return hipErrorInvalidValue;
  switch (kernel) {
#ifdef PDMB_EXPERIMENTS
    case kT128Unfused: return ktile::launch<ktile::CfgT128, false>(dt, a, stream);
    case kFp8T128Unfused: return ktile::launch<ktile::CfgT128, false>(dt, a, stream);
#endif
    case kFp8T128: return ktile::launch<ktile::CfgT128>(dt, a, stream);
    case kFp8T256x128: return ktile::launch<ktile::CfgT256x128>(dt, a, stream);
    case kT128: return ktile::launch<ktile::CfgT128>(dt, a, stream);
    case kT128x2: return ktile::launch<ktile::CfgT128x2>(dt, a, stream);
    case kT256x128: return ktile::launch<ktile::CfgT256x128>(dt, a, stream);
    case kT192: return ktile::launch<ktile::CfgT192>(dt, a, stream);
    case kT192x128: return ktile::launch<ktile::CfgT192x128>(dt, a, stream);
    case kFp8T192: return ktile::launch<ktile::CfgT192>(dt, a, stream);
    case kFp8T192x128: return ktile::launch<ktile::CfgT192x128>(dt, a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pdmb
