// gemm_t128.hip — bf16 / fp16 C = A @ B (row-major NN, fp32 accumulate) on
// 128x128 output tiles: the kernel for grids that under-fill the 256 CUs with
// 256x256 tiles.
//
// Why: matrix_parallel's per-rank column shards at ws >= 4 of the reference's
// default sizes (matmul_scaling_benchmark.py:179-188 at :351-352) are
// [4096^2] @ [4096 x 512] (32 256x256 tiles) and [8192^2] @ [8192 x 1024]
// (128 tiles); 2048^3 has 64. W4 (gemm_w4.hip) leaves most CUs idle there,
// and splitting K over 256x256 tiles costs a 256 KiB fp32 slab per slice to
// combine (profiles/r2_splitk_sweep.jsonl). A 128x128 tile gives 4x the
// workgroups with the same LDS images and MFMA idiom, and its split-K slab
// is 64 KiB.
//
// Structure (W4's idioms at a quarter of the tile):
//  * 4 waves, one per SIMD, each owning a 64x64 output block (4 x 4 MFMA
//    16x16x32 blocks, 64 fp32 accumulators per lane in AGPRs, operands
//    swapped so the accumulator holds C^T).
//  * LDS images per stage: A [128 rows][128 B] with 16-B chunk c at
//    c ^ ((row >> 1) & 7); B [64 k][256 B] with 32-B unit u (16 columns) at
//    u ^ ((k & 3) | ((k >> 3) & 1) << 2), read transposed by ds_read_b64_tr_b16
//    (the NN B operand, no transposed copy). Both are W4's conflict-free
//    layouts (A: W4's image at half the rows; B: one W4 half without the
//    column interleave).
//  * NS = 4 stage ring (4 x 32 KiB = 128 KiB, 1 workgroup per CU; kT128x2:
//    NS = 2, 64 KiB, 2 workgroups per CU) filled by
//    LDS-DMA (buffer_load ... lds): during K-tile t the workgroup issues tile
//    t + 4 into t's stage, so each tile has ~3 K-tiles of flight (a 128x128
//    K-tile is 1/4 of W4's MFMA time, so the ring is deeper instead).
//  * One barrier per K-tile: s_waitcnt vmcnt(16) (tile t+1 landed; t+2, t+3
//    may be in flight) lgkmcnt(0) (this wave's reads of tile t's fragments
//    done) then s_barrier; after it, tile t's stage is free for tile t+4 and
//    tile t+1's stage is readable. Fragments of t+1 are read during t's 32
//    MFMAs into a second register set (A/B fragments double-buffered).
//  * Every load sits in an MFMA gap: per K-tile 8 A-fragment ds_read_b128,
//    8 B fragments (2 ds_read_b64_tr_b16 each) and 8 DMA pieces over 32
//    gaps (kItems).
//  * Optional split-K over K-tile ranges with the in-launch combine of
//    splitk.h (64 KiB slab per slice).
//
// Fast-path constraints (host-checked): M, N multiples of 128 (interior tiles
// only), K % 64 == 0, lda / ldb % 8 == 0, ldc % 4 == 0, 16-B aligned A / B,
// 8-B aligned C.
#include "api.h"
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace kt128 {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;
constexpr int NS4 = 4;                       // LDS stages (default: 1 workgroup / CU)
constexpr int A_BYTES = BM * BK * 2;         // 16 KiB
constexpr int B_BYTES = BK * BN * 2;         // 16 KiB
constexpr int STAGE = A_BYTES + B_BYTES;     // 32 KiB

// Top-of-K-tile wait: the pieces issued after tile t+1's are those of tiles
// t+2 .. t+NS-1 (8 per tile per wave).
template <int NS>
__device__ __forceinline__ void wait_next_and_barrier() {
  if constexpr (NS == 4)
    asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (NS == 3)
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Prologue wait: tile 0 landed, tiles 1 .. NS-1 may still be in flight.
template <int NS>
__device__ __forceinline__ void wait_first_and_barrier() {
  if constexpr (NS == 4)
    asm volatile("s_waitcnt vmcnt(24)\n\ts_barrier" ::: "memory");
  else if constexpr (NS == 3)
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
}
constexpr int NPIECE = 8;                    // DMA pieces per wave per K-tile (4 A + 4 B)

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

struct Frag {  // one 16-row (A) or 16-column (B) block of a K-tile: k 0..31 and 32..63
  s16x8 k[2];
};

struct Ctx {
  u32x4 ra;               // A descriptor at this slice's first K
  const char* Bb;         // B at this slice's first K row, column n0
  long long b_bytes;      // bytes from Bb to the end of B's extent
  int lda2, ldb2, nk;     // leading dims in bytes, K-tiles of this slice
  uint32_t voffA, voffB;  // per-lane DMA offsets of piece 0
  uint32_t aoff[2];       // per-lane A fragment offsets in stage 0, [ks]
  uint32_t boff[4];       // per-lane B fragment offsets in stage 0, [block j]
  int wu;
  uint32_t lds0;
};

__device__ __forceinline__ u32x4 b_rsrc(const Ctx& c, int tile) {
  const long long off = (long long)tile * BK * c.ldb2;
  return make_rsrc(c.Bb + off, c.b_bytes - off);
}

// DMA piece h (0..7) of K-tile `tile` into the stage at byte offset `so`.
// h < 4: A rows h*32 + wu*8 + [0,8) (8 x 128 B); h >= 4: B k rows
// (h-4)*16 + wu*4 + [0,4) (4 x 256 B). B's swizzle depends on k & 11 only,
// which the (h-4)*16 row offset leaves alone, so one per-lane offset serves
// all pieces (A likewise: rows +32 keep (row >> 1) & 7).
__device__ __forceinline__ void issue_piece(const Ctx& c, u32x4 rb, uint32_t so, int tile, int h) {
  if (h < 4) {
    dma16_m0(c.ra, c.voffA, (uint32_t)tile * (BK * 2) + (uint32_t)(h * 32 * c.lda2),
             c.lds0 + so + (h * 32 + c.wu * 8) * 128);
  } else {
    const int kb = h - 4;
    dma16_m0(rb, c.voffB, (uint32_t)(kb * 16 * c.ldb2),
             c.lds0 + so + A_BYTES + (kb * 16 + c.wu * 4) * 256);
  }
}

// A fragment half ks of block m (rows 16m..16m+15 of this wave's 64).
__device__ __forceinline__ s16x8 frag_a(const char* smem, uint32_t off, int m) {
  return *(const lds_s16x8*)(smem + m * 16 * 128 + off);
}

// B fragment half ks of block j (16 output columns): two transposed reads.
__device__ __forceinline__ s16x8 frag_b(const char* smem, uint32_t off, int ks) {
  const char* p = smem + A_BYTES + ks * 32 * 256 + off;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 256));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// What a wave issues after MFMA `gap` (0..31; ks = gap >> 4, mi = (gap >> 2) & 3,
// ni = gap & 3) of K-tile t: 0 nothing; 1 the next DMA piece (tile t + NS into
// t's stage); 100 + 2j + ks: B fragment j, half ks of tile t+1; 200 + 2m + ks:
// A fragment m, half ks of tile t+1. Reads of t+1 go to the other register set,
// so they may sit anywhere in t; DMA pieces every 4th gap, LDS reads spread.
constexpr int kItems[32] = {100, 200, 0, 1, 101, 201, 0, 1, 102, 202, 0, 1, 103, 203, 0, 1,
                            104, 204, 0, 1, 105, 205, 0, 1, 106, 206, 0, 1, 107, 207, 0, 1};

constexpr int piece_of(int gap) {
  int n = 0;
  for (int g = 0; g < gap; ++g)
    if (kItems[g] == 1) ++n;
  return n;
}

// One K-tile: 32 MFMAs on (Ac, Bc) = fragments of tile t, reading tile t+1's
// fragments into (An, Bn) from stage sn, DMA of tile t + NS into stage sc.
template <int DT, int NS>
__device__ __forceinline__ void ktile(const Ctx& c, const char* smem, int t, uint32_t sc,
                                      uint32_t sn, f32x4 (&acc)[4][4], Frag (&Ac)[4],
                                      Frag (&Bc)[4], Frag (&An)[4], Frag (&Bn)[4]) {
  const int td = t + NS < c.nk ? t + NS : c.nk - 1;  // clamped tail DMAs (harmless re-reads)
  static_assert(NS >= 2 && NS <= 4, "T128 ring depth");
  const u32x4 rb = b_rsrc(c, td);
  wait_next_and_barrier<NS>();
  __builtin_amdgcn_sched_barrier(0);
  uint32_t ao[2], bo[4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ao[ks] = c.aoff[ks] + sn;
#pragma unroll
  for (int j = 0; j < 4; ++j) bo[j] = c.boff[j] + sn;
#pragma unroll
  for (int gap = 0; gap < 32; ++gap) {
    const int ks = gap >> 4, mi = (gap >> 2) & 3, ni = gap & 3;
    mfma_acc<DT>(acc[mi][ni], Bc[ni].k[ks], Ac[mi].k[ks]);
    const int it = kItems[gap];
    if (it == 1) {
      issue_piece(c, rb, sc, td, piece_of(gap));
    } else if (it >= 200) {
      const int m = (it - 200) >> 1, h = (it - 200) & 1;
      An[m].k[h] = frag_a(smem, ao[h], m);
    } else if (it >= 100) {
      const int j = (it - 100) >> 1, h = (it - 100) & 1;
      Bn[j].k[h] = frag_b(smem, bo[j], h);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// NS = 4: 128 KiB ring, 1 workgroup per CU (default). NS = 2: 64 KiB, 2
// workgroups per CU (kT128x2: the other workgroup hides DMA latency).
template <int DT, int NS>
__global__ void __launch_bounds__(NT, NS == 2 ? 2 : 1) gemm_t128_nn(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  int slice = 0;  // split-K: grid batch = batch x S, slice innermost (as W4)
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
  c.lda2 = a.lda * 2;
  c.ldb2 = a.ldb * 2;
  {
    const int nk_all = a.K / BK;
    c.nk = a.splitk > 1 ? min(a.kt_per, nk_all - kt0) : nk_all;
  }
  const int k0 = kt0 * BK;
  const char* Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda + k0) * 2;
  c.ra = make_rsrc(Ab, ((long long)(a.M - m0 - 1) * a.lda + (a.K - k0)) * 2);
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + (long long)k0 * a.ldb + n0) * 2;
  c.b_bytes = ((long long)(a.K - k0 - 1) * a.ldb + (a.N - n0)) * 2;
  {
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;  // row of A piece 0
    c.voffA = (uint32_t)(r * c.lda2 + ((lc8 ^ ((r >> 1) & 7)) * 16));
    const int lr16 = lane >> 4, lc16 = lane & 15;
    const int k = wu * 4 + lr16;  // k row of B piece 0
    const int s = (k & 3) | (((k >> 3) & 1) << 2);
    const int n = ((lc16 >> 1) ^ s) * 16 + (lc16 & 1) * 8;  // column of this lane's 16 B
    c.voffB = (uint32_t)(k * c.ldb2 + n * 2);
    const int swA = (l16 >> 1) & 7;
    const int q4 = l16 >> 2, p4 = l16 & 3;
    const int sB = q4 | ((g & 1) << 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint32_t ao = (uint32_t)((wr * 64 + l16) * 128 + (((4 * ks + g) ^ swA) * 16));
      asm volatile("" : "+v"(ao));  // opaque: one base VGPR each
      c.aoff[ks] = ao;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int u = 4 * wc + j;  // 32-B unit = columns 16u .. 16u+15 of the tile
      uint32_t bo = (uint32_t)((8 * g + q4) * 256 + ((u ^ sB) * 32) + p4 * 8);
      asm volatile("" : "+v"(bo));
      c.boff[j] = bo;
    }
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue: tiles 0 .. NS-1 into stages 0 .. NS-1 (clamped), wait for tile
  // 0 everywhere, read its fragments. The loop's wait then always finds
  // exactly NS-1 tiles (8 pieces each) issued after the one it needs... minus
  // one: vmcnt(16) = tiles t+2, t+3 still in flight, t+1 landed.
  const int nk = c.nk;
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int tl = st < nk ? st : nk - 1;
    const u32x4 rb = b_rsrc(c, tl);
#pragma unroll
    for (int h = 0; h < NPIECE; ++h) issue_piece(c, rb, st * STAGE, tl, h);
  }
  wait_first_and_barrier<NS>();  // tile 0 landed everywhere
  Frag A0[4], B0[4], A1[4], B1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      A0[i].k[ks] = frag_a(smem, c.aoff[ks], i);
      B0[i].k[ks] = frag_b(smem, c.boff[i], ks);
    }
  // Steady state: K-tile t computes from set (t & 1), reads t+1 into the
  // other set from stage (t+1) % NS, refills stage t % NS with tile t + NS.
  // The wait at the top of t: pieces issued after tile t+1's are those of
  // t+2 .. t+NS-1 = 16 pieces (the prologue issued t+NS-1 = 3 for t = 0).
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile<DT, NS>(c, smem, t, (uint32_t)((t % NS) * STAGE), (uint32_t)(((t + 1) % NS) * STAGE),
                  acc, A0, B0, A1, B1);
    ktile<DT, NS>(c, smem, t + 1, (uint32_t)(((t + 1) % NS) * STAGE),
              (uint32_t)(((t + 2) % NS) * STAGE), acc, A1, B1, A0, B0);
  }
  if (t < nk)  // odd count: the last tile's "next" reads are clamped re-reads
    ktile<DT, NS>(c, smem, t, (uint32_t)((t % NS) * STAGE), (uint32_t)((t % NS) * STAGE), acc, A0,
                  B0, A1, B1);
  // Drain the tail DMAs and give the last MFMAs time to write their AGPRs
  // (asm MFMAs are invisible to hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  SplitSlots sl;
  const bool split = a.splitk > 1;
  if (split && !splitk_meet<4, 4, NT>(a, smem, ((long long)bz * a.tiles_m + tm) * a.tiles_n + tn,
                                      slice, acc, sl))
    return;

  // Epilogue: acc[i][j] holds C^T of a 16x16 block: lane owns row l16 and
  // columns 4g..4g+3 (interior tiles only: no masks).
  char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 v[4];
    if (!split) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[i][j];
    } else {
      splitk_row<4, 4, NT>(a, sl, slice, i, acc, v);
    }
    const int row = m0 + wr * 64 + i * 16 + l16;
    char* crow = Cb + (long long)row * a.ldc * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + 4 * g;
      u32x2 w;
      w.x = pack2<DT>(v[j].x, v[j].y);
      w.y = pack2<DT>(v[j].z, v[j].w);
      *(u32x2*)(crow + col * 2) = w;
    }
  }
}

}  // namespace kt128

bool gemm_t128_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (dt != kBF16 && dt != kF16) return false;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return false;
  if (a.M % 128 || a.N % 128 || a.K % 64) return false;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 4) return false;
  if (a.lda < a.K || a.ldb < a.N || a.ldc < a.N) return false;
  if (a.batch > 1 && (a.sA % 8 || a.sB % 8 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 8) return false;
  // 32-bit offsets: A rows up to 127 * lda (+ K bytes of the tile offset),
  // B rows up to 63 * ldb.
  if ((long long)128 * a.lda * 2 + (long long)a.K * 2 >= (1LL << 31)) return false;
  if ((long long)64 * a.ldb * 2 + 64 >= (1LL << 31)) return false;
  return true;
}

hipError_t gemm_t128_launch(int dt, GemmArgs a, hipStream_t stream, int stages) {
  a.tiles_m = a.M / kt128::BM;
  a.tiles_n = a.N / kt128::BN;
  const int S = a.splitk > 1 ? a.splitk : 1;
  if (S > 1) {
    const int nk = a.K / kt128::BK;
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
  const dim3 grid((unsigned)nblocks), block(kt128::NT);
  if (stages == 2) {
    if (dt == kBF16)
      hipLaunchKernelGGL((kt128::gemm_t128_nn<kBF16, 2>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kt128::gemm_t128_nn<kF16, 2>), grid, block, 0, stream, a);
  } else {
    if (dt == kBF16)
      hipLaunchKernelGGL((kt128::gemm_t128_nn<kBF16, kt128::NS4>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((kt128::gemm_t128_nn<kF16, kt128::NS4>), grid, block, 0, stream, a);
  }
  return hipGetLastError();
}

}  // namespace pdmb
