// gemm_fp8.hip — C = alpha * (A @ B) with A, B in OCP fp8 e4m3 (gfx950's
// float8_e4m3fn, not MI300's fnuz), fp32 accumulate, bf16 out, on the fp8
// MFMA v_mfma_f32_16x16x128_f8f6f4 (the W4 kernels; the 8-wave A/B kernel
// keeps the block-scaled form with unit scales).
//
// An MI355X extension beyond the reference's float32/float16/bfloat16
// (matmul_benchmark.py:163-174): the fp8 MFMA with K = 128 runs at twice the
// bf16 rate (MI355X_MICROARCH.md § Matrix cores: ~5 PF dense), so the same
// `--dtype` sweep can show what the matrix cores do at fp8.
//
// Layout: A row-major [M,K]; B column-major, i.e. stored as Bt [N,K]
// row-major (torch._scaled_mm's convention, and what a weight matrix is).
// Both operands are then K-contiguous, so both reach their MFMA fragments
// with ds_read_b128 — no transposed LDS read is needed.
//
// Design: the schedule of gemm_mfma256.hip SCHED 3 carried over byte for
// byte. A K-tile of 128 fp8 is 128 bytes per row — the same LDS image as a
// 64-deep bf16 tile (A 32 KiB + two 16 KiB B halves per stage, 2 stages =
// 128 KiB, 1 workgroup / CU, 8 waves 2 (M) x 4 (N), 128x64 per wave) — and
// each 16x16x128 MFMA takes twice the cycles of a 16x16x32 bf16 one, so a
// compute slot of 16 fp8 MFMAs is as long as SCHED 3's 32 bf16 MFMAs while
// doing twice the FLOPs. LDS-DMA units, counted vmcnt(6), the one-slot
// stagger of waves 4..7 and the XCD-aware tile order are unchanged.
//
// MFMA fragments (16x16x128, e4m3): lane l holds 32 consecutive k of one
// row, k = 32 * (l >> 4) + j (j = 0..31), i.e. two 16-B LDS chunks 2g and
// 2g+1 of the 128-B row. The block scales are fixed at e8m0 127 (= 1.0); the
// per-tensor scale alpha is applied in the epilogue. Operands are swapped
// (B fragment as the MFMA's A) so each lane owns 4 consecutive output
// columns -> 8-byte bf16 stores.
//
// Fast-path constraints (host-checked, no fallback for fp8): K % 128 == 0,
// N % 4 == 0, lda / ldb % 16 == 0 (16-B rows), ldc % 4 == 0, 16-B aligned
// A / B, 8-B aligned C. M and N edges read zeros through the buffer
// descriptor's extent and are masked at the store.
#include "api.h"
#include "common.h"
#include "splitk.h"

namespace pdmb {
namespace k8 {

constexpr int BM = 256, BN = 256, BK = 128;  // BK in fp8 elements (= bytes)
constexpr int NTHREADS = 512;
constexpr int A_BYTES = BM * BK;             // 32 KiB
constexpr int BH_BYTES = (BN / 2) * BK;      // 16 KiB per B half
constexpr int STAGE = A_BYTES + 2 * BH_BYTES;
constexpr int LDS_BYTES = 2 * STAGE;         // 128 KiB
constexpr int kScaleOne = 0x7F7F7F7F;        // e8m0 127 = 2^0 in every byte

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

#define PDMB8_BARRIER()                     \
  do {                                      \
    __builtin_amdgcn_sched_barrier(0);      \
    asm volatile("s_barrier" ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0);      \
  } while (0)
#define PDMB8_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define PDMB8_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

struct Ctx {
  const char* Ab;     // A of this batch element at row m0
  const char* Bb;     // Bt of this batch element at row (= output column) n0
  long long a_bytes;  // bytes from Ab to the end of A's extent
  long long b_bytes;  // bytes from Bb to the end of Bt's extent
  int nk;             // K / 128
  uint32_t voffA[2][2];  // [mq][h] per-lane DMA source offsets
  uint32_t voffB[2][2];  // [nq][h]
  uint32_t aoff[2];      // [h] per-lane LDS read offsets (stage 0, quadrant 0)
  uint32_t boff[2];
  int wu;
  uint32_t lds0;
};

// One LDS-DMA unit (2 wave-instructions per wave). TYPE: 0 = A rows of
// quadrant-row 0, 1 = B half 0, 2 = B half 1, 3 = A rows of quadrant-row 1.
// A unit holds the 128 rows {mq*64 + [0,64)} U {128 + mq*64 + [0,64)}; a B
// half holds the 128 output columns wc*64 + nq*32 + [0,32) of the 4 wave
// columns, LDS row i <-> column (i>>5)*64 + nq*32 + (i&31). 16-B chunk c of
// LDS row r holds source chunk c ^ swz(r) (conflict-free b128 reads).
template <int TYPE, int STG>
__device__ __forceinline__ void issue_unit(const Ctx& c, int tile) {
  tile = tile < c.nk ? tile : c.nk - 1;  // tail re-reads the last tile (harmless)
  const long long off = (long long)tile * BK;
  if constexpr (TYPE == 0 || TYPE == 3) {
    constexpr int mq = TYPE == 0 ? 0 : 1;
    const u32x4 rs = make_rsrc(c.Ab + off, c.a_bytes - off);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      dma16(rs, c.voffA[mq][h], c.lds0 + STG * STAGE + (h * 128 + mq * 64 + c.wu * 8) * BK);
  } else {
    constexpr int nq = TYPE == 1 ? 0 : 1;
    const u32x4 rs = make_rsrc(c.Bb + off, c.b_bytes - off);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      dma16(rs, c.voffB[nq][h],
            c.lds0 + STG * STAGE + A_BYTES + nq * BH_BYTES + (h * 64 + c.wu * 8) * BK);
  }
}

// LDS swizzle of a 128-B row r: 16-B chunk c is stored at c ^ swz(r).
// A lane's fragment is chunks 2g, 2g+1 of row l16, and ds_read_b128 serves
// lanes in the groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): in each
// group the rows are all 16 distinct, but lanes on rows 4..11 fetch a chunk
// 2 apart from the others (g differs by one). The plain (r>>1)&7 swizzle of
// the bf16 kernel then collides (PMC: 4.0e8 conflict cycles of 8.1e8); the
// extra XOR by 2 on rows 4..11 cancels that offset, so each group covers all
// 64 banks once.
__device__ __forceinline__ int swz(int r) {
  return ((r >> 1) & 7) ^ ((((r & 15) - 4) & 15) < 8 ? 2 : 0);
}

__device__ __forceinline__ i32x8 join(u32x4 lo, u32x4 hi) {
  const u32x4 v[2] = {lo, hi};
  return __builtin_bit_cast(i32x8, v);
}

// A fragments of quadrant-row MQ: 4 m-blocks x 32 B.
template <int STG, int MQ>
__device__ __forceinline__ void read_a(const Ctx& c, const char* smem, i32x8 (&ra)[4]) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const char* p = smem + STG * STAGE + (MQ * 64 + mi * 16) * BK;
    ra[mi] = join(*(const lds_u32x4*)(p + c.aoff[0]), *(const lds_u32x4*)(p + c.aoff[1]));
  }
}

// B fragments of half NQ: 2 n-blocks x 32 B.
template <int STG, int NQ>
__device__ __forceinline__ void read_b(const Ctx& c, const char* smem, i32x8 (&rb)[2]) {
#pragma unroll
  for (int nn = 0; nn < 2; ++nn) {
    const char* p = smem + STG * STAGE + A_BYTES + NQ * BH_BYTES + nn * 16 * BK;
    rb[nn] = join(*(const lds_u32x4*)(p + c.boff[0]), *(const lds_u32x4*)(p + c.boff[1]));
  }
}

template <int MQ, int NQ>
__device__ __forceinline__ void mma_quadrant(f32x4 (&acc)[8][4], const i32x8 (&ra)[4],
                                             const i32x8 (&rb)[2]) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
      acc[MQ * 4 + mi][NQ * 2 + nn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
          rb[nn], ra[mi], acc[MQ * 4 + mi][NQ * 2 + nn], 0 /*A: e4m3*/, 0 /*B: e4m3*/, 0,
          kScaleOne, 0, kScaleOne);
}

// One K-tile from stage STG in two phases (SCHED 3 of gemm_mfma256.hip; the
// RAW / WAR argument there carries over unit for unit):
//   X: read B0,B1 | issue B0',B1' of t+1 | MFMA quadrants (0,0),(0,1)
//   Y: read A1 and the next tile's A0 | issue A0,A1 of t+2 | MFMA (1,1),(1,0)
template <int STG>
__device__ __forceinline__ void tile_body(const Ctx& c, char* smem, int t, f32x4 (&acc)[8][4],
                                          i32x8 (&ra)[4], i32x8 (&ra2)[4], i32x8 (&rb0)[2],
                                          i32x8 (&rb1)[2]) {
  read_b<STG, 0>(c, smem, rb0);
  read_b<STG, 1>(c, smem, rb1);
  issue_unit<2, STG ^ 1>(c, t + 1);
  issue_unit<3, STG ^ 1>(c, t + 1);
  PDMB8_LGKM0();
  PDMB8_VMCNT(6);
  PDMB8_BARRIER();
  mma_quadrant<0, 0>(acc, ra2, rb0);
  mma_quadrant<0, 1>(acc, ra2, rb1);
  PDMB8_BARRIER();
  read_a<STG, 1>(c, smem, ra);
  read_a<STG ^ 1, 0>(c, smem, ra2);
  issue_unit<0, STG>(c, t + 2);
  issue_unit<1, STG>(c, t + 2);
  PDMB8_LGKM0();
  PDMB8_VMCNT(6);
  PDMB8_BARRIER();
  mma_quadrant<1, 1>(acc, ra, rb1);
  mma_quadrant<1, 0>(acc, ra, rb0);
  PDMB8_BARRIER();
}

#ifdef PDMB_EXPERIMENTS  // the 8-wave kernel: an A/B build only (kFp8)
__global__ void __launch_bounds__(NTHREADS, 2) gemm_fp8_nt(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wu >> 2, wc = wu & 3;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.nk = a.K / BK;
  c.Ab = (const char*)a.A + (long long)bz * a.sA + (long long)m0 * a.lda;
  c.Bb = (const char*)a.B + (long long)bz * a.sB + (long long)n0 * a.ldb;
  // Exact extents: rows >= M (A) and columns >= N (Bt rows) read zeros.
  c.a_bytes = (long long)(a.M - m0 - 1) * a.lda + a.K;
  c.b_bytes = (long long)(a.N - n0 - 1) * a.ldb + a.K;
  {
    const int lr8 = lane >> 3, lc8 = lane & 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int mq = 0; mq < 2; ++mq) {
        const int r = h * 128 + mq * 64 + wu * 8 + lr8;
        c.voffA[mq][h] = (uint32_t)(r * a.lda + ((lc8 ^ swz(r)) * 16));
      }
#pragma unroll
      for (int nq = 0; nq < 2; ++nq) {
        const int i = h * 64 + wu * 8 + lr8;
        const int col = (i >> 5) * 64 + nq * 32 + (i & 31);
        c.voffB[nq][h] = (uint32_t)(col * a.ldb + ((lc8 ^ swz(i)) * 16));
      }
    }
    const int sw = swz(l16);  // rows read are 16-aligned bases + l16
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      c.aoff[h] = (uint32_t)((wr * 128 + l16) * BK + (((2 * g + h) ^ sw) * 16));
      c.boff[h] = (uint32_t)((wc * 32 + l16) * BK + (((2 * g + h) ^ sw) * 16));
    }
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x8 ra[4], ra2[4], rb0[2], rb1[2];

  // Prologue: units 0..5 = A0,B0,B1,A1 of tile 0 and A0,B0 of tile 1.
  issue_unit<0, 0>(c, 0);
  issue_unit<1, 0>(c, 0);
  issue_unit<2, 0>(c, 0);
  issue_unit<3, 0>(c, 0);
  issue_unit<0, 1>(c, 1);
  issue_unit<1, 1>(c, 1);
  PDMB8_VMCNT(6);  // units 0..2 landed (for this wave); 3..5 in flight
  PDMB8_BARRIER();
  if (wr == 1) PDMB8_BARRIER();  // waves 4..7 run one slot behind waves 0..3
  read_a<0, 0>(c, smem, ra2);

  const int nk = c.nk;
  for (int t = 0; t < nk; t += 2) {
    tile_body<0>(c, smem, t, acc, ra, ra2, rb0, rb1);
    if (t + 1 < nk) tile_body<1>(c, smem, t + 1, acc, ra, ra2, rb0, rb1);
  }
  if (wr == 0) PDMB8_BARRIER();
  PDMB8_VMCNT(0);  // drain the clamped tail DMAs before the LDS is released

  // Epilogue: acc[i][j] holds C^T of a 16x16 tile — lane owns row l16 and
  // columns 4g..4g+3; scale by alpha, round to bf16.
  const float alpha = a.alpha;
  char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + l16;
    if (row < a.M) {
      char* crow = Cb + (long long)row * a.ldc * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + 4 * g;
        if (col < a.N) {
          u32x2 v;
          v.x = pack2<kBF16>(acc[i][j].x * alpha, acc[i][j].y * alpha);
          v.y = pack2<kBF16>(acc[i][j].z * alpha, acc[i][j].w * alpha);
          *(u32x2*)(crow + col * 2) = v;
        }
      }
    }
  }
}
#endif


// ---- W4 (default): 4 waves, one per SIMD, 128x128 output per wave --------
// The 8-wave kernel above reads 192 KiB of LDS fragments per K-tile; with
// 128x128 per wave a workgroup reads 128 KiB (each A / B fragment is shared
// by 2 waves, not 4 / 2), the LDS energy that kept hipBLASLt's fp8 kernel
// ~5 % higher in clock (profiles/r1_s3_pmc_fp8.md). 256 fp32 accumulators
// per lane live in AGPRs: the MFMA is issued by inline asm with "+a"
// operands, since with the builtin hipcc shuffles and spills them
// (profiles/r1_fp32_ablation.md). What it took (each step measured, 16k):
//  * every load in an MFMA's shadow, about one per 32-cycle gap (kW4Items):
//    loads issued back to back after each m-block's MFMAs left the MFMA pipe
//    idle — 66 % utilisation, 2750 TF;
//  * ~1.5 K-tiles of LDS-DMA flight: B of tile t+1 is read in m-blocks 0-3 and
//    A in 4-7, with a second barrier between, so each operand half is
//    refilled half a K-tile after its last read (one K-tile of flight cost
//    17 %, measured with a no-wait diagnostic build);
//  * LDS-DMA pieces that clobber M0 instead of saving / restoring it, and one
//    base VGPR per stage so fragment reads need no address adds: 3157 → 3217 TF.
// 3217 TF vs 3079 for the 8-wave kernel (hipBLASLt 3343).
constexpr int NT4 = 256;
constexpr int STAGE4 = 2 * A_BYTES;  // A [256][128 B] + Bt [256][128 B]

// SCALED = 0 (default): the unscaled v_mfma_f32_16x16x128_f8f6f4 (e4m3 x e4m3,
// same rate as the block-scaled form, scale 1). SCALED = 1: the block-scaled
// form with both scales 2^0 — identical results, but it assembles to TWO
// instructions (a v_mfma_ld_scale_b32 prefix + the MFMA, 16 bytes), an extra
// issue slot in every MFMA gap of a one-wave-per-SIMD schedule (A/B only).
template <int SCALED>
__device__ __forceinline__ void mfma_f8_acc(f32x4& acc, const i32x8& a, const i32x8& b, int sc) {
  if constexpr (SCALED)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                 : "+a"(acc)
                 : "v"(a), "v"(b), "v"(sc));
  else
    asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// LDS-DMA with a scalar offset (the 8 pieces of one operand differ by 32 rows).
__device__ __forceinline__ void dma16_so(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  unsigned int keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
      : "memory");
}

// As dma16_so, but M0 is simply clobbered (declared to hipcc) instead of
// saved and restored around every piece: 3 instructions per piece, not 5.
__device__ __forceinline__ void dma16_m0(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  asm volatile(
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
      : "memory", "m0");
}

struct Ctx4 {
  u32x4 ra, rb;       // buffer descriptors at K = 0
  int lda, ldb, nk;
  uint32_t voffA, voffB;  // per-lane DMA offsets of piece 0
  // Per-lane LDS fragment offsets [stage][16-B chunk h], B's including A_BYTES;
  // one VGPR per (stage, h) so every fragment read is ds_read_b128 off:imm
  // with no address add (the immediate field stops at 64 KiB = one stage).
  uint32_t aoff[2][2], boff[2][2];
  int wu;
  uint32_t lds0;
};

// DMA piece h (0..15) of tile `tile` into stage `so`: h < 8 -> A rows
// (h*4+wu)*8 + [0,8), else Bt rows ((h-8)*4+wu)*8 + [0,8).
__device__ __forceinline__ void issue_piece(const Ctx4& c, int so, int tile, int h) {
  const uint32_t koff = (uint32_t)tile * BK;
  if (h < 8)
    dma16_m0(c.ra, c.voffA, koff + (uint32_t)(h * 32 * c.lda),
             c.lds0 + so + (h * 4 + c.wu) * 8 * BK);
  else
    dma16_m0(c.rb, c.voffB, koff + (uint32_t)((h - 8) * 32 * c.ldb),
             c.lds0 + so + A_BYTES + ((h - 8) * 4 + c.wu) * 8 * BK);
}

__device__ __forceinline__ i32x8 frag(const char* p, const uint32_t (&off)[2]) {
  return join(*(const lds_u32x4*)(p + off[0]), *(const lds_u32x4*)(p + off[1]));
}

// What a wave issues in MFMA gap `gap` of m-block `blk`. With one wave per
// SIMD a load must sit in an MFMA's shadow (~one per 32-cycle gap) or it
// delays the next MFMA: loads issued back to back after each m-block's MFMAs
// ran at 66 % MFMA utilisation. 0: nothing; 1: next LDS-DMA piece (blocks
// 0-3: A of tile t+2, blocks 4-7: B of tile t+3); 10+s: B fragment s of tile
// t+1; 20+m: A fragment m of tile t+1 (27: into the second A7 set).
constexpr int kW4Items[8][8] = {
    {10, 1, 11, 1, 0, 0, 0, 0}, {12, 1, 13, 1, 0, 0, 0, 0}, {14, 1, 15, 1, 0, 0, 0, 0},
    {16, 1, 17, 1, 0, 0, 0, 0}, {20, 1, 21, 1, 0, 0, 0, 0}, {22, 1, 23, 1, 0, 0, 0, 0},
    {24, 1, 25, 1, 27, 0, 0, 0}, {26, 1, 1, 0, 0, 0, 0, 0}};

constexpr int w4_piece(int blk, int gap) {  // running index of a DMA item (0..15)
  int n = 0;
  for (int b = 0; b < 8; ++b)
    for (int g = 0; g < 8; ++g) {
      if (b == blk && g == gap) return n;
      if (kW4Items[b][g] == 1) ++n;
    }
  return n;
}

// One K-tile t (stage S = SO, tile t+1 in SN = S^1), two barriers:
//   Bar0: B(t+1) landed (vmcnt 16: A(t+1), B(t+2) may still fly); every wave
//         finished reading A(t) from S.A in K-tile t-1 (lgkmcnt 0).
//   blocks 0-3: MFMAs of tile t | read B(t+1) from S^1.B | DMA A(t+2) -> S.A
//   Bar_mid: A(t+1) landed (vmcnt 16: B(t+2), A(t+2) may fly); every wave
//         finished reading B(t+1) from S^1.B.
//   blocks 4-7: MFMAs | read A(t+1) from S^1.A | DMA B(t+3) -> S^1.B
// Each operand half thus gets ~1.5 K-tiles of DMA flight (one K-tile was not
// enough: the same kernel without the DMA wait ran 17 % faster).
template <int SO, int DIAG_NOWAIT = 0, int SCALED = 0>
__device__ __forceinline__ void ktile_w4(const Ctx4& c, const char* smem, int t, f32x4 (&acc)[8][8],
                                         i32x8 (&A)[8], i32x8& A7c, i32x8& A7n, i32x8 (&Bc)[8],
                                         i32x8 (&Bn)[8], int sc) {
  constexpr int SN = STAGE4 - SO;  // stage of tile t+1
  const int ta = t + 2 < c.nk ? t + 2 : c.nk - 1;  // clamped tail DMAs (harmless re-reads)
  const int tb = t + 3 < c.nk ? t + 3 : c.nk - 1;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    if (mi == 0 || mi == 4) {
      if constexpr (DIAG_NOWAIT == 1)  // timing-only diagnostic: never wait for the DMA
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if constexpr (DIAG_NOWAIT == 2)  // timing-only diagnostic: no waits, no barriers
        asm volatile("" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      mfma_f8_acc<SCALED>(acc[mi][ni], Bc[ni], mi == 7 ? A7c : A[mi], sc);
      if constexpr (DIAG_NOWAIT != 3) {  // 3: timing-only, MFMAs + barriers alone
        const int it = kW4Items[mi][ni];
        if (it == 1) {
          const int h = w4_piece(mi, ni);  // 0..7: A of t+2 into S; 8..15: B of t+3 into S^1
          if (h < 8)
            issue_piece(c, SO, ta, h);
          else
            issue_piece(c, SN, tb, h);
        } else if (it >= 10 && it < 20) {
          Bn[it - 10] = frag(smem + (it - 10) * 16 * BK, c.boff[SN / STAGE4]);
        } else if (it == 27) {
          A7n = frag(smem + 7 * 16 * BK, c.aoff[SN / STAGE4]);
        } else if (it >= 20) {
          A[it - 20] = frag(smem + (it - 20) * 16 * BK, c.aoff[SN / STAGE4]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The last K-tile of an unsplit tile with the epilogue folded in: block row
// mi - 1 of C leaves (store_block16 through this wave's own LDS buffer, past
// the two stages) while block row mi's MFMAs run, so the C stores of a tile
// overlap its final MFMAs instead of following them (one tile per CU, e.g.
// 4096^3: the whole kernel is one tile). No fragment reads or DMAs: the
// fragments of the last K-tile are in registers, and no barrier is needed
// (the stages are neither read nor refilled). Block mi's eight MFMAs separate
// block mi - 1's last accumulator write from its AGPR reads.
template <int SCALED, bool NTS>
__device__ __forceinline__ void ktile_w4_last(f32x4 (&acc)[8][8], const i32x8 (&A)[8], const i32x8& A7c,
                                              const i32x8 (&Bc)[8], int sc, char* ebuf, char* Cb,
                                              long long ldc_b, int row0, int col0, int M, int N,
                                              bool interior, float alpha, int lane) {
  // The lane id is re-formed (v_mbcnt of an opaque mask) at every store so
  // hipcc cannot hoist the eight stores' per-lane addresses above the MFMAs,
  // where they would be live at once and spill (as W4S's epilogue).
  (void)lane;
  auto store = [&](int i) {
    unsigned all = ~0u;
    asm volatile("" : "+s"(all));
    const int eln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
    if (interior)
      store_block16<kBF16, false, true, 8, NTS>(ebuf, acc[i], alpha, Cb, ldc_b, row0 + i * 16, col0, M, N,
                                                eln);
    else
      store_block16<kBF16, true, true, 8, NTS>(ebuf, acc[i], alpha, Cb, ldc_b, row0 + i * 16, col0, M, N,
                                               eln);
  };
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) mfma_f8_acc<SCALED>(acc[mi][ni], Bc[ni], mi == 7 ? A7c : A[mi], sc);
    __builtin_amdgcn_sched_barrier(0);
    if (mi >= 1) store(mi - 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  store(7);
}

// SUB: XCD sub-block shape (map_tile); 1 (8x4) and 2 (2x16) are A/B experiments.
// SCALED: see mfma_f8_acc (1 = kFp8W4Scaled, A/B only).
// TRACE: write the tile timeline (common.h tile_trace_write; kFp8W4Trace).
// NTS: non-temporal C stores (common.h store_block16; false: A/B kFp8W4TS).
// FUSED: unsplit tiles store C during their last K-tile (ktile_w4_last;
// false: A/B kFp8W4Unfused).
template <int DIAG_NOWAIT, int SUB = 0, int SCALED = 0, int TRACE = 0, bool NTS = true, bool FUSED = true>
__global__ void __launch_bounds__(NT4, 1) gemm_fp8_w4(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE4 + (FUSED ? 4 * kEpiBuf : 0)];
  TileTrace tr;
  if constexpr (TRACE) tr.t[0] = tile_clock();

  int bz, tm, tn;
  // Split-K (grids that under-fill the CUs): the grid's "batch" is batch x S
  // with the slice innermost, as in gemm_w4.hip; slice s runs K-tiles
  // [s * kt_per, +kt_per) and the slices meet in the epilogue (splitk.h).
  // A tile-range launch (GemmArgs::tile_span) instead maps block b to local
  // tile b % span of the range and slice b / span: a tile's slices share the
  // XCD (b % 8), so their meet stays in one L2.
  int slice = 0;
  long long meet_tile;
  if (a.tile_span > 0) {
    const int local = blockIdx.x % a.tile_span;
    slice = blockIdx.x / a.tile_span;
    map_tile(a, a.tile_base + local, bz, tm, tn, SUB);
    meet_tile = local;
  } else {
    map_tile(a, blockIdx.x, bz, tm, tn, SUB);
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

  Ctx4 c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda = a.lda;
  c.ldb = a.ldb;
  c.nk = a.splitk > 1 ? min(a.kt_per, a.K / BK - kt0) : a.K / BK;
  const long long k0 = (long long)kt0 * BK;  // bytes: fp8 rows are K-contiguous
  const char* Ab = (const char*)a.A + (long long)bz * a.sA + (long long)m0 * a.lda + k0;
  const char* Bb = (const char*)a.B + (long long)bz * a.sB + (long long)n0 * a.ldb + k0;
  c.ra = make_rsrc(Ab, (long long)(a.M - m0 - 1) * a.lda + a.K - k0);
  c.rb = make_rsrc(Bb, (long long)(a.N - n0 - 1) * a.ldb + a.K - k0);
  {
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;  // row of piece 0 (swz(r + 32h) = swz(r))
    c.voffA = (uint32_t)(r * a.lda + ((lc8 ^ swz(r)) * 16));
    c.voffB = (uint32_t)(r * a.ldb + ((lc8 ^ swz(r)) * 16));
    const int sw = swz(l16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint32_t ao = (uint32_t)(st * STAGE4 + (wr * 128 + l16) * BK + (((2 * g + h) ^ sw) * 16));
        uint32_t bo = (uint32_t)(st * STAGE4 + A_BYTES + (wc * 128 + l16) * BK +
                                 (((2 * g + h) ^ sw) * 16));
        asm volatile("" : "+v"(ao), "+v"(bo));  // opaque: keep each as its own base VGPR
        c.aoff[st][h] = ao;
        c.boff[st][h] = bo;
      }
    }
  }
  const int sc = __builtin_amdgcn_readfirstlane(kScaleOne);

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
#pragma unroll
  for (int h = 0; h < 16; ++h) issue_piece(c, 0, 0, h);
#pragma unroll
  for (int h = 8; h < 16; ++h) issue_piece(c, STAGE4, t1, h);
#pragma unroll
  for (int h = 0; h < 8; ++h) issue_piece(c, STAGE4, t1, h);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");  // tile 0 landed everywhere
  i32x8 A[8], A7a, A7b, B0[8], B1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    A[i] = frag(smem + i * 16 * BK, c.aoff[0]);
    B0[i] = frag(smem + i * 16 * BK, c.boff[0]);
  }
  A7a = A[7];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // stage 0.B read by all
  if constexpr (TRACE) tr.t[1] = tile_clock();
#pragma unroll
  for (int h = 8; h < 16; ++h) issue_piece(c, 0, t2, h);
  const bool split = a.splitk > 1;
  constexpr bool kFuse = FUSED && TRACE == 0 && DIAG_NOWAIT == 0;
  const bool fuse = kFuse && !split && (nk & 1) == 0;
  const int nloop = fuse ? nk - 1 : nk;  // fused: the last K-tile is ktile_w4_last
  int t = 0;
  for (; t + 1 < nloop; t += 2) {  // branch-free body: B0/B1 and A7a/A7b swap roles every K-tile
    ktile_w4<0, DIAG_NOWAIT, SCALED>(c, smem, t, acc, A, A7a, A7b, B0, B1, sc);
    ktile_w4<STAGE4, DIAG_NOWAIT, SCALED>(c, smem, t + 1, acc, A, A7b, A7a, B1, B0, sc);
  }
  if (t < nloop) ktile_w4<0, DIAG_NOWAIT, SCALED>(c, smem, t, acc, A, A7a, A7b, B0, B1, sc);  // odd count
  if constexpr (kFuse) {
    if (fuse) {
      // nk even (host: fuse only then): the last K-tile nk-1 is odd and
      // computes from (A7b, B1). Handling both parities here kept both sets
      // live through the stores and made hipcc spill (AGPR copies it places
      // next to the asm MFMAs, which it does not know to wait for).
      char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
      char* ebuf = smem + 2 * STAGE4 + wu * kEpiBuf;
      const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
      ktile_w4_last<SCALED, NTS>(acc, A, A7b, B1, sc, ebuf, Cb, (long long)a.ldc * 2, m0 + wr * 128,
                                 n0 + wc * 128, a.M, a.N, interior, a.alpha, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs landed before the LDS is released
      return;
    }
  }
  // Drain the tail DMAs and give the last MFMAs time to write their AGPRs
  // (asm MFMAs are invisible to hipcc's hazard recognizer).
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if constexpr (TRACE) tr.t[2] = tile_clock();

  // Split-K: only the last slice of a tile to arrive writes C, summing the
  // slices' fp32 slots (unscaled) block row by block row (splitk.h).
  SplitSlots sl;
  if (split && !splitk_meet<8, 8, NT4>(a, smem, meet_tile, slice, acc, sl))
    return;
  // Epilogue through LDS as whole rows (common.h store_block16), masked at
  // M / N; every DMA landed and every fragment read done before any wave
  // writes its staging buffers.
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const float alpha = a.alpha;
  char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
  char* ebuf = smem + 1024 + wu * 2 * kEpiBuf;  // past splitk_meet's ticket word
  const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f32x4 v[8];
    if (!split) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[i][j];
    } else {
      splitk_row<8, 8, NT4>(a, sl, slice, i, acc, v);
    }
    if (interior)
      store_block16<kBF16, false, true, 8, NTS>(ebuf + (i & 1) * kEpiBuf, v, alpha, Cb, (long long)a.ldc * 2,
                                        m0 + wr * 128 + i * 16, n0 + wc * 128, a.M, a.N, lane);
    else
      store_block16<kBF16, true, true, 8, NTS>(ebuf + (i & 1) * kEpiBuf, v, alpha, Cb, (long long)a.ldc * 2,
                                       m0 + wr * 128 + i * 16, n0 + wc * 128, a.M, a.N, lane);
  }
  if constexpr (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr.t[3] = tile_clock();
    tile_trace_write(a, tr, blockIdx.x, tm, tn);
  }
}

// ---- fp8 W4S: the W4 fp8 kernel as one K-tile stream per CU --------------
// gemm_w4.hip's W4S carried over (its comment has the why): the DMA items of
// K-tiles nk .. nk+2 fetch the next tile's K-tiles 0 .. 2, the epilogue
// (alpha, bf16) goes out through its own LDS region without a drain, the
// next tile's first two K-tiles wait vmcnt(16 + 32), the first tile issues
// 32 out-of-range LDS-DMA loads in the stores' place, and every MFMA of
// K-tile 0 (one per accumulator: K = 128 per MFMA) starts from C = 0.
// Interior tiles only (M, N % 256), K % 256 == 0, K >= 512 (K = 512: the K4 form); static tiles
// b, b + G, ... (G = grid, a multiple of 8) on a device the GEMM has to itself.
__device__ __forceinline__ void mfma_f8_zero(f32x4& acc, const i32x8& a, const i32x8& b) {
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, 0" : "=&a"(acc) : "v"(a), "v"(b));
}

template <int N>
__device__ __forceinline__ void wait_vm_lgkm_barrier8() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct Src8 {  // one output tile's operand descriptors (K = 0)
  u32x4 ra, rb;
};

__device__ __forceinline__ Src8 tile_src8(const GemmArgs& a, int bz, int tm, int tn) {
  const int m0 = tm * BM, n0 = tn * BN;
  Src8 s;
  s.ra = make_rsrc((const char*)a.A + (long long)bz * a.sA + (long long)m0 * a.lda,
                   (long long)(a.M - m0 - 1) * a.lda + a.K);
  s.rb = make_rsrc((const char*)a.B + (long long)bz * a.sB + (long long)n0 * a.ldb,
                   (long long)(a.N - n0 - 1) * a.ldb + a.K);
  return s;
}

// ktile_w4 with explicit DMA targets: A of item "t+2" (descriptor raT at K
// byte offset kaT), B of "t+3" (rbT at kbT), wait counts W0 / W1, ZERO.
template <int SO, int W0, int W1, bool ZERO>
__device__ __forceinline__ void ktile_w4s(const Ctx4& c, const char* smem, u32x4 raT, uint32_t kaT,
                                          u32x4 rbT, uint32_t kbT, uint32_t lds0w,
                                          f32x4 (&acc)[8][8], i32x8 (&A)[8], i32x8& A7c,
                                          i32x8& A7n, i32x8 (&Bc)[8], i32x8 (&Bn)[8]) {
  constexpr int SN = STAGE4 - SO;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    if (mi == 0) {
      wait_vm_lgkm_barrier8<W0>();
      __builtin_amdgcn_sched_barrier(0);
    } else if (mi == 4) {
      wait_vm_lgkm_barrier8<W1>();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      if constexpr (ZERO)
        mfma_f8_zero(acc[mi][ni], Bc[ni], mi == 7 ? A7c : A[mi]);
      else
        mfma_f8_acc<0>(acc[mi][ni], Bc[ni], mi == 7 ? A7c : A[mi], 0);
      const int it = kW4Items[mi][ni];
      if (it == 1) {
        const int h = w4_piece(mi, ni);
        // the first two K-tiles of a tile (W0 48): soffsets hipcc may have just
        // restored with v_readlane (common.h dma16_at_pad)
        if (h < 8) {  // A of t+2 into S.A: rows (h*4 + wu)*8 + [0,8)
          if constexpr (W0 == 48)
            dma16_at_pad(raT, c.voffA, kaT + (uint32_t)(h * 32 * c.lda), lds0w, SO + h * 4 * 8 * BK);
          else
            dma16_at(raT, c.voffA, kaT + (uint32_t)(h * 32 * c.lda), lds0w, SO + h * 4 * 8 * BK);
        } else {  // B of t+3 into S^1.B
          if constexpr (W0 == 48)
            dma16_at_pad(rbT, c.voffB, kbT + (uint32_t)((h - 8) * 32 * c.ldb), lds0w,
                         SN + A_BYTES + (h - 8) * 4 * 8 * BK);
          else
            dma16_at(rbT, c.voffB, kbT + (uint32_t)((h - 8) * 32 * c.ldb), lds0w,
                     SN + A_BYTES + (h - 8) * 4 * 8 * BK);
        }
      } else if (it >= 10 && it < 20) {
        Bn[it - 10] = frag(smem + (it - 10) * 16 * BK, c.boff[SN / STAGE4]);
      } else if (it == 27) {
        A7n = frag(smem + 7 * 16 * BK, c.aoff[SN / STAGE4]);
      } else if (it >= 20) {
        A[it - 20] = frag(smem + (it - 20) * 16 * BK, c.aoff[SN / STAGE4]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// K4 (nk == 4, K = 512, shipping; kFp8W4SK4 / kFp8W4SK4TS force it on any
// even nk >= 4 for A/B): with four
// K-tiles the first pair is already the pair whose second K-tile fetches the
// next tile's B(0) (item t + 4 = nk), so its DMA targets go through the same
// selects as the last pair's; nk >= 6 never reaches the next tile there.
template <bool NTS = true, bool K4 = false>  // NTS: non-temporal C stores (false: A/B kFp8W4STS)
__global__ void __launch_bounds__(NT4, 1) gemm_fp8_w4s(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE4 + 4 * kEpiBuf];
  // tile_end > 0: the whole-wave part of a tile-range tail plan
  const int T = a.tile_end > 0 ? a.tile_end : a.tiles_m * a.tiles_n * a.batch;
  const int G = gridDim.x;
  int vb = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wu >> 1, wc = wu & 1;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx4 c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  const uint32_t lds0w = c.lds0 + wu * 8 * BK;  // every piece's per-wave LDS rows
  c.lda = a.lda;
  c.ldb = a.ldb;
  c.nk = a.K / BK;
  {
    const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;
    c.voffA = (uint32_t)(r * a.lda + ((lc8 ^ swz(r)) * 16));
    c.voffB = (uint32_t)(r * a.ldb + ((lc8 ^ swz(r)) * 16));
    const int sw = swz(l16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint32_t ao = (uint32_t)(st * STAGE4 + (wr * 128 + l16) * BK + (((2 * g + h) ^ sw) * 16));
        uint32_t bo = (uint32_t)(st * STAGE4 + A_BYTES + (wc * 128 + l16) * BK +
                                 (((2 * g + h) ^ sw) * 16));
        asm volatile("" : "+v"(ao), "+v"(bo));
        c.aoff[st][h] = ao;
        c.boff[st][h] = bo;
      }
    }
  }
  const int nk = c.nk;
  int bz, tm, tn;
  map_tile(a, vb, bz, tm, tn);
  Src8 cur = tile_src8(a, bz, tm, tn);
  int nvb = vb + G, nbz = bz, ntm = tm, ntn = tn;
  Src8 nxt = cur;
  if (nvb < T) {
    map_tile(a, nvb, nbz, ntm, ntn);
    nxt = tile_src8(a, nbz, ntm, ntn);
  }
  f32x4 acc[8][8];  // started by each tile's K-tile 0 (ZERO)

  // Prologue of the first tile, as gemm_fp8_w4's: A(0), B(0) -> stage 0;
  // B(1), A(1) -> stage 1; fragments of K-tile 0; B(2) -> stage 0.B.
  auto dma_a = [&](const u32x4& r, uint32_t ka, int so, int h) {
    dma16_at(r, c.voffA, ka + (uint32_t)(h * 32 * c.lda), lds0w, so + h * 4 * 8 * BK);
  };
  auto dma_b = [&](const u32x4& r, uint32_t kb, int so, int h) {
    dma16_at(r, c.voffB, kb + (uint32_t)((h - 8) * 32 * c.ldb), lds0w, so + A_BYTES + (h - 8) * 4 * 8 * BK);
  };
#pragma unroll
  for (int h = 0; h < 8; ++h) dma_a(cur.ra, 0u, 0, h);
#pragma unroll
  for (int h = 8; h < 16; ++h) dma_b(cur.rb, 0u, 0, h);
#pragma unroll
  for (int h = 8; h < 16; ++h) dma_b(cur.rb, BK, STAGE4, h);
#pragma unroll
  for (int h = 0; h < 8; ++h) dma_a(cur.ra, BK, STAGE4, h);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  i32x8 A[8], A7a, A7b, B0[8], B1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    A[i] = frag(smem + i * 16 * BK, c.aoff[0]);
    B0[i] = frag(smem + i * 16 * BK, c.boff[0]);
  }
  A7a = A[7];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int h = 8; h < 16; ++h) dma_b(cur.rb, 2 * BK, 0, h);
  char* ebuf = smem + 2 * STAGE4 + wu * kEpiBuf;
  {  // 32 dummy LDS-DMA loads in the place of the epilogue stores (see above)
    u32x4 nul;
    nul.x = 0u;
    nul.y = 0u;
    nul.z = 0u;
    nul.w = 0x00020000u;
    const uint32_t eb = c.lds0 + 2 * STAGE4 + wu * kEpiBuf;
#pragma unroll
    for (int i = 0; i < 32; ++i) dma16_m0(nul, 0u, 0u, eb);
  }
  for (;;) {
    const bool more = nvb < T;
    auto sel = [](uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); };
    // descriptor and K offset of item "kt": this tile, the next, or (last
    // tile) a harmless re-read of this tile's last K-tile
    auto tgt = [&](int kt, const u32x4& rc, const u32x4& rn, u32x4& r, uint32_t& ko) {
      const uint32_t m = (kt < nk || !more) ? ~0u : 0u;
      const int k = kt < nk ? kt : (more ? kt - nk : nk - 1);
      r.x = sel(m, rc.x, rn.x);
      r.y = sel(m, rc.y, rn.y);
      r.z = sel(m, rc.z, rn.z);
      r.w = rc.w;
      ko = (uint32_t)k * BK;
    };
    if constexpr (K4) {
      u32x4 ra, rb;
      uint32_t ka, kb;
      tgt(2, cur.ra, nxt.ra, ra, ka);
      tgt(3, cur.rb, nxt.rb, rb, kb);
      ktile_w4s<0, 48, 48, true>(c, smem, ra, ka, rb, kb, lds0w, acc, A, A7a, A7b, B0, B1);
      tgt(3, cur.ra, nxt.ra, ra, ka);
      tgt(4, cur.rb, nxt.rb, rb, kb);
      ktile_w4s<STAGE4, 48, 16, false>(c, smem, ra, ka, rb, kb, lds0w, acc, A, A7b, A7a, B1, B0);
    } else {
      ktile_w4s<0, 48, 48, true>(c, smem, cur.ra, 2 * BK, cur.rb, 3 * BK, lds0w, acc, A, A7a, A7b, B0, B1);
      ktile_w4s<STAGE4, 48, 16, false>(c, smem, cur.ra, 3 * BK, cur.rb, 4 * BK, lds0w, acc, A, A7b, A7a,
                                       B1, B0);
    }
    int t = 2;
    for (; t + 4 < nk; t += 2) {
      ktile_w4s<0, 16, 16, false>(c, smem, cur.ra, (uint32_t)(t + 2) * BK, cur.rb, (uint32_t)(t + 3) * BK,
                                  lds0w, acc, A, A7a, A7b, B0, B1);
      ktile_w4s<STAGE4, 16, 16, false>(c, smem, cur.ra, (uint32_t)(t + 3) * BK, cur.rb,
                                       (uint32_t)(t + 4) * BK, lds0w, acc, A, A7b, A7a, B1, B0);
    }
    for (; t < nk; t += 2) {
      u32x4 ra, rb;
      uint32_t ka, kb;
      tgt(t + 2, cur.ra, nxt.ra, ra, ka);
      tgt(t + 3, cur.rb, nxt.rb, rb, kb);
      ktile_w4s<0, 16, 16, false>(c, smem, ra, ka, rb, kb, lds0w, acc, A, A7a, A7b, B0, B1);
      tgt(t + 3, cur.ra, nxt.ra, ra, ka);
      tgt(t + 4, cur.rb, nxt.rb, rb, kb);
      ktile_w4s<STAGE4, 16, 16, false>(c, smem, ra, ka, rb, kb, lds0w, acc, A, A7b, A7a, B1, B0);
    }
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
    unsigned all = ~0u;
    asm volatile("" : "+s"(all));  // per tile: lane offsets formed here, not kept live
    const int eln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      store_block16<kBF16, false, true, 8, NTS>(ebuf, acc[i], a.alpha, Cb, (long long)a.ldc * 2,
                                        tm * BM + wr * 128 + i * 16, tn * BN + wc * 128, a.M, a.N, eln);
    __builtin_amdgcn_sched_barrier(0);
    if (!more) break;
    vb = nvb;
    bz = nbz;
    tm = ntm;
    tn = ntn;
    cur = nxt;
    nvb = vb + G;
    if (nvb < T) {
      map_tile(a, nvb, nbz, ntm, ntn);
      nxt = tile_src8(a, nbz, ntm, ntn);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA in flight at exit
}

// ---- fp8 stream-K: tiles [tile_base, +tile_span) as one even share of K-tile
// iterations per workgroup ---------------------------------------------------
// For grids of ~1-2 waves of 256x256 tiles (5120^3: 400 tiles = 1.56 waves)
// neither whole tiles nor a split / refined last wave balance the CUs: half of
// them would still run two whole tiles. Here the L = span x nk K-tile
// iterations of the range (map_tile's order, local tile-major) are cut into G
// = gridDim.x equal contiguous shares (splitk.h sk_begin); workgroup w runs its
// share as segments, one per tile it touches: the W4 K-loop over the
// segment's K-range (c.nk = its K-tiles, descriptors based at its first
// K-tile), then either the plain epilogue (a whole tile) or the stream-K meet
// (splitk.h sk_meet: contributor index = w - first owner; the last to arrive
// sums the slots in K order and stores C). a.splitk = slots per tile (the
// most contributors any tile has, host-computed), a.part / a.flags as split-K.
__global__ void __launch_bounds__(NT4, 1) gemm_fp8_sk(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE4];
  // 32-bit share arithmetic (host: L x G < 2^31), kept in SGPRs: the 64-bit
  // divisions run on the VALU, and their VGPR results pushed the kernel into
  // scratch
  // XCD-local shares: workgroup b runs on XCD b % 8 (dispatch round-robin), and
  // map_tile gives XCD x the tiles of index = x mod 8, grouped so their A / B
  // panels share that XCD's L2. So XCD x's G / 8 workgroups share out only
  // its own tiles (local 8 j + x); one chip-wide share order mixed panels
  // across XCDs and ran at ~half speed (profiles/r4m_fp8_stream_k_ab.jsonl).
  const unsigned nk_all = (unsigned)(a.K / BK);
  const unsigned xcd = blockIdx.x & 7, wi = blockIdx.x >> 3, G = gridDim.x >> 3;
  const unsigned L = ((unsigned)a.tile_span - xcd + 7) / 8 * nk_all;  // this XCD's K-tile iterations
  const unsigned hi = __builtin_amdgcn_readfirstlane((wi + 1) * L / G);
  const int sc = __builtin_amdgcn_readfirstlane(kScaleOne);
  for (unsigned it = __builtin_amdgcn_readfirstlane(wi * L / G); it < hi;) {
    // Per-lane values are formed again in every segment from an opaque thread
    // id: hoisted out of the loop they stayed live across the K-loop and spilled.
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = (int)(tid & 63);
    const int wu = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const int wr = wu >> 1, wc = wu & 1;
    const int l16 = lane & 15, g = lane >> 4;
    const int jx = __builtin_amdgcn_readfirstlane(it / nk_all);  // this XCD's jx-th tile
    const int local = 8 * jx + (int)xcd;
    const int kt0 = __builtin_amdgcn_readfirstlane(it - (unsigned)jx * nk_all);
    const int cnt = __builtin_amdgcn_readfirstlane(min(hi - it, nk_all - (unsigned)kt0));
    it += (unsigned)cnt;
    int bz, tm, tn;
    map_tile(a, a.tile_base + local, bz, tm, tn);
    bz = __builtin_amdgcn_readfirstlane(bz);
    tm = __builtin_amdgcn_readfirstlane(tm);
    tn = __builtin_amdgcn_readfirstlane(tn);
    const int m0 = tm * BM, n0 = tn * BN;

    Ctx4 c;
    c.wu = wu;
    c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
    c.lda = a.lda;
    c.ldb = a.ldb;
    c.nk = cnt;
    const long long k0 = (long long)kt0 * BK;
    const char* Ab = (const char*)a.A + (long long)bz * a.sA + (long long)m0 * a.lda + k0;
    const char* Bb = (const char*)a.B + (long long)bz * a.sB + (long long)n0 * a.ldb + k0;
    c.ra = make_rsrc(Ab, (long long)(a.M - m0 - 1) * a.lda + a.K - k0);
    c.rb = make_rsrc(Bb, (long long)(a.N - n0 - 1) * a.ldb + a.K - k0);
    {
      const int r = wu * 8 + (lane >> 3), lc8 = lane & 7;
      c.voffA = (uint32_t)(r * a.lda + ((lc8 ^ swz(r)) * 16));
      c.voffB = (uint32_t)(r * a.ldb + ((lc8 ^ swz(r)) * 16));
      const int sw = swz(l16);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          uint32_t ao = (uint32_t)(st * STAGE4 + (wr * 128 + l16) * BK + (((2 * g + h) ^ sw) * 16));
          uint32_t bo = (uint32_t)(st * STAGE4 + A_BYTES + (wc * 128 + l16) * BK + (((2 * g + h) ^ sw) * 16));
          asm volatile("" : "+v"(ao), "+v"(bo));
          c.aoff[st][h] = ao;
          c.boff[st][h] = bo;
        }
      }
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // prologue and K-loop: gemm_fp8_w4's, over this segment's cnt K-tiles
    const int nk = c.nk;
    const int t1 = nk > 1 ? 1 : 0, t2 = nk > 2 ? 2 : nk - 1;
#pragma unroll
    for (int h = 0; h < 16; ++h) issue_piece(c, 0, 0, h);
#pragma unroll
    for (int h = 8; h < 16; ++h) issue_piece(c, STAGE4, t1, h);
#pragma unroll
    for (int h = 0; h < 8; ++h) issue_piece(c, STAGE4, t1, h);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    i32x8 A[8], A7a, A7b, B0[8], B1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      A[i] = frag(smem + i * 16 * BK, c.aoff[0]);
      B0[i] = frag(smem + i * 16 * BK, c.boff[0]);
    }
    A7a = A[7];
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int h = 8; h < 16; ++h) issue_piece(c, 0, t2, h);
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      ktile_w4<0>(c, smem, t, acc, A, A7a, A7b, B0, B1, sc);
      ktile_w4<STAGE4>(c, smem, t + 1, acc, A, A7b, A7a, B1, B0, sc);
    }
    if (t < nk) ktile_w4<0>(c, smem, t, acc, A, A7a, A7b, B0, B1, sc);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

    const bool whole = kt0 == 0 && (unsigned)cnt == nk_all;
    SplitSlots sl;
    int slot = 0, S = 1;
    if (!whole) {
      const unsigned tb = (unsigned)jx * nk_all;
      // owner of iteration x: max w with w L / G <= x (splitk.h sk_owner)
      const int first = __builtin_amdgcn_readfirstlane((int)(((tb + 1) * G + L - 1) / L) - 1);
      const int last = __builtin_amdgcn_readfirstlane((int)(((tb + nk_all) * G + L - 1) / L) - 1);
      S = last - first + 1;
      slot = (int)wi - first;
      unsigned tm2 = threadIdx.x;
      asm volatile("" : "+v"(tm2));
      if (!sk_meet<8, 8, NT4>(a, smem, local, slot, S, acc, sl, (int)tm2)) continue;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    char* Cb = (char*)a.C + (long long)bz * a.sC * 2;
    char* ebuf = smem + 1024 + wu * 2 * kEpiBuf;  // past sk_meet's ticket word
    const bool interior = m0 + BM <= a.M && n0 + BN <= a.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f32x4 v[8];
      if (whole) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[i][j];
      } else {
        sk_row<8, 8, NT4>(sl, slot, S, i, acc, v);
      }
      if (interior)
        store_block16<kBF16, false, true, 8, true>(ebuf + (i & 1) * kEpiBuf, v, a.alpha, Cb, (long long)a.ldc * 2,
                                                   m0 + wr * 128 + i * 16, n0 + wc * 128, a.M, a.N, lane);
      else
        store_block16<kBF16, true, true, 8, true>(ebuf + (i & 1) * kEpiBuf, v, a.alpha, Cb, (long long)a.ldc * 2,
                                                  m0 + wr * 128 + i * 16, n0 + wc * 128, a.M, a.N, lane);
    }
    // the next segment's prologue refills the stages this epilogue staged through
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

}  // namespace k8

int fp8_sk_slots(long long span, int nk, long long G) { return sk_max_owners(span, nk, G); }

// nk even and >= 4 (round 6: K = 512 runs the K4 form, below; before, nk >= 6)
bool gemm_fp8_w4s_fits(const GemmArgs& a) {
  const int nk = a.K / k8::BK;
  return a.M % k8::BM == 0 && a.N % k8::BN == 0 && a.K % (2 * k8::BK) == 0 && nk >= 4;
}

bool gemm_fp8_w4s_k4_fits(const GemmArgs& a) {  // the K4 variant: nk even, >= 4
  const int nk = a.K / k8::BK;
  return a.M % k8::BM == 0 && a.N % k8::BN == 0 && a.K % (2 * k8::BK) == 0 && nk >= 4;
}

bool gemm_fp8_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (a.K % 128 != 0 || a.K <= 0 || a.N % 4 != 0 || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 16 || a.ldb % 16 || a.ldc % 4) return false;
  if (a.lda < a.K || a.ldb < a.K) return false;
  if (a.batch > 1 && (a.sA % 16 || a.sB % 16 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 8) return false;
  // 32-bit per-lane DMA offsets: up to 255 rows of A / Bt.
  if ((long long)256 * a.lda >= (1LL << 31) || (long long)256 * a.ldb >= (1LL << 31)) return false;
  return true;
}

hipError_t gemm_fp8_launch(GemmArgs a, int variant, hipStream_t stream) {
  a.tiles_m = (a.M + k8::BM - 1) / k8::BM;
  a.tiles_n = (a.N + k8::BN - 1) / k8::BN;
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const int S = variant == 1 && a.splitk > 1 ? a.splitk : 1;  // split-K: the W4 kernel only
  const long long all_tiles = (long long)a.tiles_m * a.tiles_n * a.batch;
  if (a.tile_span < 0 || a.tile_base < 0 || a.tile_end < 0 || a.tile_end > all_tiles ||
      (a.tile_span > 0 && ((variant != 1 && variant != 3) || (long long)a.tile_base + a.tile_span > all_tiles)) ||
      (a.tile_end > 0 && a.tile_span > 0))
    return hipErrorInvalidValue;
  if (variant == 3) {  // stream-K over a tile range (gemm_fp8_sk): grid pers_grid, a.splitk slots per tile
    const long long L = (long long)a.tile_span * (a.K / k8::BK);
    if (a.tile_span < 8 || a.pers_grid <= 0 || a.pers_grid % 8 || a.tile_span / 8 * (a.K / k8::BK) < a.pers_grid / 8 ||
        L * (a.pers_grid + 1) >= (1LL << 31) ||
        a.splitk < 2 || !a.part || !a.flags ||
        a.tile_span > kMaxSplitTiles || sk_max_owners(a.tile_span, a.K / k8::BK, a.pers_grid) > a.splitk)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(k8::gemm_fp8_sk, dim3((unsigned)a.pers_grid), dim3(k8::NT4), 0, stream, a);
    return hipGetLastError();
  }
  const long long tiles = a.tile_span > 0 ? a.tile_span : a.tile_end > 0 ? a.tile_end : all_tiles;
  if (S > 1) {
    const int nk = a.K / k8::BK;
    a.kt_per = (nk + S - 1) / S;
    if ((S - 1) * a.kt_per >= nk || !a.part || !a.flags || tiles > kMaxSplitTiles)
      return hipErrorInvalidValue;  // every slice must own >= 1 K-tile
  } else {
    a.splitk = 1;
  }
  const long long nblocks = tiles * S;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblocks);
  if (variant == 1) {  // the shipping fp8 kernel (kFp8W4)
    hipLaunchKernelGGL(k8::gemm_fp8_w4<0>, grid, dim3(k8::NT4), 0, stream, a);
    return hipGetLastError();
  }
  if (variant == 2) {  // kFp8W4S: streaming persistent (host: gemm_fp8_w4s_fits, pers_grid % 8 == 0)
    if (!gemm_fp8_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8) return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    // K = 512 (four K-tiles): the K4 form. Measured against fp8 W4, which
    // cannot overlap a tile's C stores with anything (settled, two sessions,
    // profiles/r8d/ab_fp8_k512_summary.jsonl): 16384^2 x 512 1544 vs 1328 TF
    // (hipBLASLt 1553), 8192^2 x 512 1551 vs 1398 (1511), 16384 x 8192 x 512
    // 1567 vs 1418 (1544). From six K-tiles on, the K4 form measured within
    // +-2 % of the plain one either way (r8e), so those keep the plain W4S.
    if (a.K / k8::BK < 6)
      hipLaunchKernelGGL((k8::gemm_fp8_w4s<true, true>), pg, dim3(k8::NT4), 0, stream, a);
    else
      hipLaunchKernelGGL(k8::gemm_fp8_w4s<true>, pg, dim3(k8::NT4), 0, stream, a);
    return hipGetLastError();
  }
#ifdef PDMB_EXPERIMENTS
  if (variant == 9)
    hipLaunchKernelGGL(k8::gemm_fp8_w4<1>, grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 10)
    hipLaunchKernelGGL(k8::gemm_fp8_w4<2>, grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 11)
    hipLaunchKernelGGL(k8::gemm_fp8_w4<3>, grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 12)
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 1>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 13)
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 2>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 14)
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 0, 1>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 15)
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 0, 0, 1>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 16)
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 0, 0, 0, false>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 18)  // kFp8W4Unfused: the epilogue after the last K-tile
    hipLaunchKernelGGL((k8::gemm_fp8_w4<0, 0, 0, 0, true, false>), grid, dim3(k8::NT4), 0, stream, a);
  else if (variant == 17) {
    if (!gemm_fp8_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8) return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    hipLaunchKernelGGL(k8::gemm_fp8_w4s<false>, pg, dim3(k8::NT4), 0, stream, a);
  }
  else if (variant == 21 || variant == 22) {  // fp8 W4S / W4 with mode 3's rounds as supertile 9
    if (a.supertile == 3) a.supertile = 9;
    if (variant == 22) {
      if (S > 1) return hipErrorInvalidValue;
      hipLaunchKernelGGL(k8::gemm_fp8_w4<0>, grid, dim3(k8::NT4), 0, stream, a);
    } else {
      if (!gemm_fp8_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8) return hipErrorInvalidValue;
      const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
      if (a.K / k8::BK < 6)
        hipLaunchKernelGGL((k8::gemm_fp8_w4s<true, true>), pg, dim3(k8::NT4), 0, stream, a);
      else
        hipLaunchKernelGGL(k8::gemm_fp8_w4s<true>, pg, dim3(k8::NT4), 0, stream, a);
    }
  }
  else if (variant == 23) {  // kFp8W4SThin: W4S with the aspect-following thin round
    if (!gemm_fp8_w4s_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8 || S > 1) return hipErrorInvalidValue;
    a.supertile = thin_supertile(a.tiles_m, a.tiles_n);
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (a.K / k8::BK < 6)
      hipLaunchKernelGGL((k8::gemm_fp8_w4s<true, true>), pg, dim3(k8::NT4), 0, stream, a);
    else
      hipLaunchKernelGGL(k8::gemm_fp8_w4s<true>, pg, dim3(k8::NT4), 0, stream, a);
  }
  else if (variant == 19 || variant == 20) {  // kFp8W4SK4 / kFp8W4SK4TS: W4S down to nk == 4
    if (!gemm_fp8_w4s_k4_fits(a) || a.pers_grid <= 0 || a.pers_grid % 8) return hipErrorInvalidValue;
    const dim3 pg((unsigned)(nblocks < a.pers_grid ? nblocks : a.pers_grid));
    if (variant == 19)
      hipLaunchKernelGGL((k8::gemm_fp8_w4s<true, true>), pg, dim3(k8::NT4), 0, stream, a);
    else
      hipLaunchKernelGGL((k8::gemm_fp8_w4s<false, true>), pg, dim3(k8::NT4), 0, stream, a);
  }
  else
    hipLaunchKernelGGL(k8::gemm_fp8_nt, grid, dim3(k8::NTHREADS), 0, stream, a);
#else
  return hipErrorInvalidValue;  // experiment variants are not built
#endif
  return hipGetLastError();
}

}  // namespace pdmb
