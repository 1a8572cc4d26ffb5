// gemm_mfma256.hip — the hot kernel: C = A @ B, row-major NN, bf16/fp16 in,
// fp32 accumulate, bf16/fp16 out, on gfx950 MFMA (v_mfma_f32_16x16x32_*).
//
// Replaces the implicit cuBLAS/hipBLASLt GEMM behind every torch.matmul /
// torch.bmm in the reference (matmul_benchmark.py:46,62; matmul_scaling_
// benchmark.py:79,92,120,142,188,211; backup/matmul_overlap_benchmark.py:...).
//
// Design (MI355X-first, not a CUDA translation):
//  * 256x256 output tile per workgroup, BK = 64, 512 threads = 8 waves laid
//    out 2 (M) x 4 (N); each wave owns 128x64 = 8x4 MFMA 16x16 tiles (128
//    fp32 accumulators / lane). 1 workgroup per CU (128 KiB LDS), 2 waves
//    per SIMD.
//  * Operands reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds), no VGPR
//    staging. The LDS image is lane-linear, so bank-conflict swizzles are
//    applied on the per-lane SOURCE address and the same XOR on the read.
//      A image: [256 rows][64 k] 128-B rows, 16-B chunk c stored at
//               c ^ ((row>>1)&7)  -> ds_read_b128 A fragments conflict-free.
//      B image: two halves (nq = 0/1), each [64 k][128 cols] 256-B rows;
//               32-B unit u stored at u ^ ((k&3) | ((k>>3)&1)<<2)
//               -> ds_read_b64_tr_b16 B fragments (k-strided, NN layout)
//               conflict-free.
//  * MFMA operands are swapped (B fragment as the "A" operand) so that the
//    accumulator holds C^T tiles: each lane owns 4 consecutive output
//    columns of one row -> 8-byte stores in the epilogue.
//  * Ping-pong schedule: each K-tile is 4 phases (one 64x32 quadrant of the
//    wave tile x K=64 = 16 MFMAs). A phase is two barrier-separated slots:
//    R (ds_read fragments + issue one LDS-DMA unit) and C (16 MFMA). Waves
//    4..7 run one slot behind waves 0..3, so on every SIMD one wave does
//    MFMA while its partner reads LDS and issues the next DMA.
//    Four schedules are kept for A/B (kernel ids in api.h); SCHED 3 is the
//    default: 0 = DMA issued in the C slot (the first version), 1 = DMA in
//    the R slot, 2 = 1 + reads balanced to 8 per R slot by prefetching the
//    next tile's A0 fragments in phase 3 into a second A register set,
//    3 = two quadrants (32 MFMAs) per compute slot: 4 barriers per K-tile
//    instead of 8 with the same 96 operand registers.
//    Measured on MI355X, 16384^3 bf16 random data: 1315 / 1370 / 1440 TF
//    (hipBLASLt 1362 on the same data); SCHED 2 without per-cluster
//    s_setprio is a further +0.9 % and SCHED 3 another +1.0 % (1446 TF;
//    scripts/ab_kernels.py). PMC: SCHED 3 lifts MFMA utilisation 73.9 → 77.1 %
//    but the clock falls 1.80 → 1.75 GHz — on random data the chip is
//    power-bound, so schedule gains return only partly as wall time.
//  * LDS-DMA units (A-half = 16 KiB, B-half = 16 KiB) are refilled as soon
//    as the last reader of their previous contents has retired, so every
//    unit has ~5-6 phases of flight time. The wait is a counted
//    s_waitcnt vmcnt(10) once per slot, never vmcnt(0) in the loop;
//    barriers are raw s_barrier (a __syncthreads would drain the DMA).
//  * XCD-aware tile order (common.h: map_tile).
//
// Constraints of this fast path (host checks; otherwise gemm_generic.hip):
//  K % 64 == 0, N % 8 == 0, lda/ldb % 8 == 0, ldc % 4 == 0, 16-B aligned
//  A/B, 8-B aligned C. M and N edges are handled (buffer OOB -> zeros,
//  masked stores).
#include "common.h"

namespace pdmb {
namespace k256 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int A_BYTES = BM * BK * 2;        // 32 KiB
constexpr int BH_BYTES = BK * (BN / 2) * 2;  // 16 KiB per B half
constexpr int STAGE = A_BYTES + 2 * BH_BYTES;
constexpr int LDS_BYTES = 2 * STAGE;  // 128 KiB

#define PDMB_SLOT_BARRIER()                   \
  do {                                        \
    __builtin_amdgcn_sched_barrier(0);        \
    asm volatile("s_barrier" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);        \
  } while (0)

#define PDMB_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

struct Ctx {
  // global side
  const char* Ab;  // A of this batch element, at row m0
  const char* Bb;  // B of this batch element, at col n0
  long long a_bytes;  // bytes from Ab to the end of A's extent
  long long b_bytes;  // bytes from Bb to the end of B's extent
  int lda2, ldb2;     // leading dims in bytes
  int nk;             // K / 64
  // per-lane DMA source offsets
  uint32_t voffA[2][2];  // [mq][row-half]
  uint32_t voffB[2][2];  // [nq][k-half]
  // per-lane LDS read offsets (stage 0, quadrant 0)
  uint32_t aoff[2];  // [ks]
  uint32_t boff[2];  // [ni]
  int wu;            // wave id (uniform)
  uint32_t lds0;     // LDS byte address of smem (uniform)
};

// Issue the two LDS-DMA loads of one unit. TYPE: 0 = A rows of quadrant-row
// mq=0, 1 = B half nq=0, 2 = B half nq=1, 3 = A rows mq=1. Tile index is
// clamped so the (harmless) tail loads re-read the last tile.
template <int TYPE, int STG>
__device__ __forceinline__ void issue_unit(const Ctx& c, char* smem, int tile) {
  tile = tile < c.nk ? tile : c.nk - 1;
  const int k0 = tile * BK;
  if constexpr (TYPE == 0 || TYPE == 3) {
    constexpr int mq = TYPE == 0 ? 0 : 1;
    const long long off = (long long)k0 * 2;
    const u32x4 rs = make_rsrc(c.Ab + off, c.a_bytes - off);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      dma16(rs, c.voffA[mq][h], c.lds0 + STG * STAGE + (h * 128 + mq * 64 + c.wu * 8) * 128);
  } else {
    constexpr int nq = TYPE == 1 ? 0 : 1;
    const long long off = (long long)k0 * c.ldb2;
    const u32x4 rs = make_rsrc(c.Bb + off, c.b_bytes - off);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
      dma16(rs, c.voffB[nq][kh],
            c.lds0 + STG * STAGE + A_BYTES + nq * BH_BYTES + (kh * 32 + c.wu * 4) * 256);
  }
}

// A fragments of quadrant-row mq: 4 m-reps x 2 k-steps of ds_read_b128.
template <int STG, int MQ>
__device__ __forceinline__ void read_a(const Ctx& c, const char* smem, s16x8 (&ra)[4][2]) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const char* p = smem + STG * STAGE + (MQ * 64 + mi * 16) * 128 + c.aoff[ks];
      ra[mi][ks] = *(const lds_s16x8*)p;
    }
}

// B fragments of half nq: 2 n-reps x 2 k-steps x 2 transposed reads.
template <int STG, int NQ>
__device__ __forceinline__ void read_b(const Ctx& c, const char* smem, s16x8 (&rb)[2][2]) {
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const char* p = smem + STG * STAGE + A_BYTES + NQ * BH_BYTES + ks * 32 * 256 + c.boff[ni];
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 256));
      rb[ni][ks] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
}

// XF: experiment flags of the SCHED 2 kernel (A/B only; 0 = shipped default).
//   1: s_setprio(1)/(0) around every MFMA cluster (the SCHED 0/1 style; the
//      default SCHED 2 build has none: +0.9 % at 8k and 16k, A/B in one process);
//   2: static priority (waves 4..7 raised once);  4: XCD sub-block 8 (M) x 4 (N)
//      (-1.5 % at 16k). Inside mma_quadrant, bit 0 set = NO per-cluster priority.
template <int DT, int MQ, int NQ, int XF = 0>
__device__ __forceinline__ void mma_quadrant(f32x4 (&acc)[8][4], const s16x8 (&ra)[4][2],
                                             const s16x8 (&rb)[2][2]) {
  if constexpr (!(XF & 3)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        acc[MQ * 4 + mi][NQ * 2 + ni] =
            mfma16x16x32<DT>(rb[ni][ks], ra[mi][ks], acc[MQ * 4 + mi][NQ * 2 + ni]);
  if constexpr (!(XF & 3)) __builtin_amdgcn_s_setprio(0);
}

#define PDMB_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// Diagnostic build only (STAMP = true, kernel id kMfma256Stamp): per wave,
// the cycles spent waiting in the barrier that closes a read slot (wr) and
// in the one that closes a compute slot (wc). A wave that waits after its
// read slot was faster than its partner's MFMAs; a wave that waits after its
// compute slot was waiting for the readers. Stamps go only to a debug buffer.
struct Stamp {
  unsigned long long wr = 0, wc = 0;
};

__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <bool STAMP>
__device__ __forceinline__ void slot_barrier(unsigned long long& sum) {
  if constexpr (STAMP) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t0 = stamp_now();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = stamp_now();
    __builtin_amdgcn_sched_barrier(0);
    sum += t1 - t0;
  } else {
    PDMB_SLOT_BARRIER();
  }
}

// One K-tile (4 phases) from LDS stage STG. Phase P = 4t+q issues unit P+7.
//
// SCHED 0: the unit's LDS-DMA is issued in the compute slot, ahead of the
//   16 MFMAs (vmcnt 8 after the read slot, 10 after the compute slot).
// SCHED 1: the DMA is issued in the READ slot, right after the fragment
//   reads, so its issue cost overlaps the partner wave's MFMAs instead of
//   delaying this wave's own (cdna_hip_programming.md §5 8-phase template:
//   "ds-load subtile; stage prefetch; barrier; MFMA"). Moving the issue one
//   slot earlier makes two things explicit:
//   WAR — the unit refilled in phase P was last read in the read slot of
//     P-1 (or earlier); every wave waits lgkmcnt(0) before the barrier that
//     closes its read slot, so by the time the group one slot ahead issues
//     the DMA, all reads of the old contents have returned.
//   RAW — after issuing unit P+7 a wave waits vmcnt(10): units <= P+2 have
//     landed, which the read slot of P+1 (one barrier later for the lagging
//     group) needs. Each unit now gets one more slot of flight time.
template <int DT, int STG, int SCHED, bool STAMP = false, int XF = 0>
__device__ __forceinline__ void tile_body(const Ctx& c, char* smem, int t, f32x4 (&acc)[8][4],
                                          s16x8 (&ra)[4][2], s16x8 (&ra2)[4][2],
                                          s16x8 (&rb0)[2][2], s16x8 (&rb1)[2][2], Stamp& st) {
  if constexpr (SCHED == 0) {
    // phase q=0: quadrant (0,0)
    read_a<STG, 0>(c, smem, ra);
    read_b<STG, 0>(c, smem, rb0);
    PDMB_VMCNT(8);
    PDMB_SLOT_BARRIER();
    issue_unit<3, STG ^ 1>(c, smem, t + 1);
    mma_quadrant<DT, 0, 0>(acc, ra, rb0);
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    // phase q=1: quadrant (0,1)
    read_b<STG, 1>(c, smem, rb1);
    PDMB_VMCNT(8);
    PDMB_SLOT_BARRIER();
    issue_unit<0, STG>(c, smem, t + 2);
    mma_quadrant<DT, 0, 1>(acc, ra, rb1);
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    // phase q=2: quadrant (1,1)
    read_a<STG, 1>(c, smem, ra);
    PDMB_VMCNT(8);
    PDMB_SLOT_BARRIER();
    issue_unit<1, STG>(c, smem, t + 2);
    mma_quadrant<DT, 1, 1>(acc, ra, rb1);
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    // phase q=3: quadrant (1,0) — operands already in registers
    PDMB_VMCNT(8);
    PDMB_SLOT_BARRIER();
    issue_unit<2, STG>(c, smem, t + 2);
    mma_quadrant<DT, 1, 0>(acc, ra, rb0);
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
  } else if constexpr (SCHED == 2) {
    // SCHED 1 with the fragment reads balanced over the four read slots
    // (8 reads each): A0 of the NEXT tile is read in phase 3 into a second
    // A register set (ra2 = A0, ra = A1), so phase 0 reads only B0.
    // RAW: phase 3 (P = 4t+3) may read units <= P+1 = 4(t+1)+0 = next A0.
    // WAR: next tile's A0 unit is refilled in phase 4(t+1)+1 > P+1.
    // phase q=0: quadrant (0,0) — A0 already in ra2
    read_b<STG, 0>(c, smem, rb0);
    issue_unit<3, STG ^ 1>(c, smem, t + 1);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 0, 0, (XF ^ 1)>(acc, ra2, rb0);
    slot_barrier<STAMP>(st.wc);
    // phase q=1: quadrant (0,1)
    read_b<STG, 1>(c, smem, rb1);
    issue_unit<0, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 0, 1, (XF ^ 1)>(acc, ra2, rb1);
    slot_barrier<STAMP>(st.wc);
    // phase q=2: quadrant (1,1)
    read_a<STG, 1>(c, smem, ra);
    issue_unit<1, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 1, 1, (XF ^ 1)>(acc, ra, rb1);
    slot_barrier<STAMP>(st.wc);
    // phase q=3: quadrant (1,0); prefetch next tile's A0 fragments
    read_a<STG ^ 1, 0>(c, smem, ra2);
    issue_unit<2, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 1, 0, (XF ^ 1)>(acc, ra, rb0);
    slot_barrier<STAMP>(st.wc);
  } else if constexpr (SCHED == 3) {
    // Two quadrants per compute slot (32 MFMAs): a K-tile is 2 phases, X =
    // quadrants (0,0)+(0,1) from A0,B0,B1 and Y = (1,1)+(1,0) from A1,B1,B0,
    // so there are 4 barriers per K-tile instead of 8. Operand registers stay
    // at SCHED 2's 96 (B0/B1 live across X and Y; A0 of the NEXT tile is
    // prefetched in Y into ra2). Read slots: X reads B0,B1 (16 tr reads), Y
    // reads A1 and next A0 (16 b128). Units (u = 4t + {A0,B0,B1,A1}) are issued
    // two per read slot, 6 ahead: phase P issues u = 2P+6, 2P+7.
    // RAW: phase P reads units <= 2P+2, retired by vmcnt(6) (3 units in flight)
    //   at the end of the previous read slot (one barrier more for the lagging
    //   group, as in SCHED 1/2).
    // WAR: each refilled unit was last read in the read slot of P-1 or earlier
    //   (B1/A1 of t+1 in X(t): last read X(t-1) / Y(t-1); A0/B0 of t+2 in
    //   Y(t): last read Y(t-1) / X(t)), and every read slot ends with lgkmcnt(0).
    // phase X: quadrants (0,0),(0,1)
    read_b<STG, 0>(c, smem, rb0);
    read_b<STG, 1>(c, smem, rb1);
    issue_unit<2, STG ^ 1>(c, smem, t + 1);
    issue_unit<3, STG ^ 1>(c, smem, t + 1);
    PDMB_LGKM0();
    PDMB_VMCNT(6);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 0, 0, (XF ^ 1)>(acc, ra2, rb0);
    mma_quadrant<DT, 0, 1, (XF ^ 1)>(acc, ra2, rb1);
    slot_barrier<STAMP>(st.wc);
    // phase Y: quadrants (1,1),(1,0); prefetch next tile's A0
    read_a<STG, 1>(c, smem, ra);
    read_a<STG ^ 1, 0>(c, smem, ra2);
    issue_unit<0, STG>(c, smem, t + 2);
    issue_unit<1, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(6);
    slot_barrier<STAMP>(st.wr);
    mma_quadrant<DT, 1, 1, (XF ^ 1)>(acc, ra, rb1);
    mma_quadrant<DT, 1, 0, (XF ^ 1)>(acc, ra, rb0);
    slot_barrier<STAMP>(st.wc);
  } else {
    // phase q=0: quadrant (0,0)
    read_b<STG, 0>(c, smem, rb0);
    read_a<STG, 0>(c, smem, ra);
    issue_unit<3, STG ^ 1>(c, smem, t + 1);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    mma_quadrant<DT, 0, 0>(acc, ra, rb0);
    PDMB_SLOT_BARRIER();
    // phase q=1: quadrant (0,1)
    read_b<STG, 1>(c, smem, rb1);
    issue_unit<0, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    mma_quadrant<DT, 0, 1>(acc, ra, rb1);
    PDMB_SLOT_BARRIER();
    // phase q=2: quadrant (1,1)
    read_a<STG, 1>(c, smem, ra);
    issue_unit<1, STG>(c, smem, t + 2);
    PDMB_LGKM0();
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    mma_quadrant<DT, 1, 1>(acc, ra, rb1);
    PDMB_SLOT_BARRIER();
    // phase q=3: quadrant (1,0) — operands already in registers
    issue_unit<2, STG>(c, smem, t + 2);
    PDMB_VMCNT(10);
    PDMB_SLOT_BARRIER();
    mma_quadrant<DT, 1, 0>(acc, ra, rb0);
    PDMB_SLOT_BARRIER();
  }
}

template <int DT, int SCHED, bool STAMP = false, int XF = 0>
__global__ void __launch_bounds__(NTHREADS, 2) gemm256_nn(GemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  int bz, tm, tn;
  map_tile(a, blockIdx.x, bz, tm, tn, (XF & 4) != 0);
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);
  if constexpr ((XF & 2) != 0) {
    if (wu >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int wr = wu >> 2, wc = wu & 3;
  const int l16 = lane & 15, g = lane >> 4;

  Ctx c;
  c.wu = wu;
  c.lds0 = (uint32_t)(size_t)((lds_void*)smem);
  c.lda2 = a.lda * 2;
  c.ldb2 = a.ldb * 2;
  c.nk = a.K / BK;
  c.Ab = (const char*)a.A + ((long long)bz * a.sA + (long long)m0 * a.lda) * 2;
  c.Bb = (const char*)a.B + ((long long)bz * a.sB + n0) * 2;
  // Exact byte extents of the operands (a strided view's last row ends at
  // its N / K, not at its leading dimension), so no DMA can touch memory
  // outside the tensor: rows >= M and the tail of B's last row read zeros.
  c.a_bytes = ((long long)(a.M - m0 - 1) * a.lda + a.K) * 2;
  c.b_bytes = ((long long)(a.kb - 1) * a.ldb + (a.N - n0)) * 2;

  {
    const int lr8 = lane >> 3, lc8 = lane & 7;
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = h * 128 + mq * 64 + wu * 8 + lr8;
        const int sc = lc8 ^ ((r >> 1) & 7);
        c.voffA[mq][h] = (uint32_t)(r * c.lda2 + sc * 16);
      }
    const int lr16 = lane >> 4, lc16 = lane & 15;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int k = kh * 32 + wu * 4 + lr16;
        const int s = (k & 3) | (((k >> 3) & 1) << 2);
        const int u = (lc16 >> 1) ^ s;
        const int p = u * 16 + (lc16 & 1) * 8;
        const int n = (p >> 5) * 64 + nq * 32 + (p & 31);
        c.voffB[nq][kh] = (uint32_t)(k * c.ldb2 + n * 2);
      }
    const int swA = (l16 >> 1) & 7;
    c.aoff[0] = (uint32_t)((wr * 128 + l16) * 128 + ((g ^ swA) * 16));
    c.aoff[1] = (uint32_t)((wr * 128 + l16) * 128 + (((4 + g) ^ swA) * 16));
    const int q4 = l16 >> 2, p4 = l16 & 3;
    const int sB = q4 | ((g & 1) << 2);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      c.boff[ni] = (uint32_t)((8 * g + q4) * 256 + (((wc * 2 + ni) ^ sB) * 32) + p4 * 8);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 ra[4][2], ra2[4][2], rb0[2][2], rb1[2][2];

  // Prologue: units 0..6 = A0,B0,B1,A1 of tile 0 and A0,B0,B1 of tile 1.
  issue_unit<0, 0>(c, smem, 0);
  issue_unit<1, 0>(c, smem, 0);
  issue_unit<2, 0>(c, smem, 0);
  issue_unit<3, 0>(c, smem, 0);
  issue_unit<0, 1>(c, smem, 1);
  issue_unit<1, 1>(c, smem, 1);
  if constexpr (SCHED == 3) {
    PDMB_VMCNT(6);  // units 0..2 landed (for this wave); 3..5 in flight
  } else {
    issue_unit<2, 1>(c, smem, 1);
    PDMB_VMCNT(10);  // units 0,1 landed (for this wave)
  }
  PDMB_SLOT_BARRIER();
  // Stagger: waves 4..7 run one slot behind waves 0..3.
  if (wr == 1) PDMB_SLOT_BARRIER();
  // SCHED 2 reads each tile's A0 fragments one phase early; tile 0's here
  // (units 0,1 were retired by every wave before the prologue barrier).
  if constexpr (SCHED >= 2) read_a<0, 0>(c, smem, ra2);

  const int nk = c.nk;
  Stamp st;
  unsigned long long t_loop0 = 0;
  if constexpr (STAMP) t_loop0 = stamp_now();
  for (int t = 0; t < nk; t += 2) {
    tile_body<DT, 0, SCHED, STAMP, XF>(c, smem, t, acc, ra, ra2, rb0, rb1, st);
    if (t + 1 < nk) tile_body<DT, 1, SCHED, STAMP, XF>(c, smem, t + 1, acc, ra, ra2, rb0, rb1, st);
  }
  if constexpr (STAMP) {
    const unsigned long long t_loop1 = stamp_now();
    if (lane == 0 && a.dbg) {
      unsigned long long* d = a.dbg + ((size_t)blockIdx.x * 8 + wu) * 4;
      d[0] = st.wr;
      d[1] = st.wc;
      d[2] = t_loop1 - t_loop0;
      d[3] = (unsigned long long)nk;
    }
  }
  if (wr == 0) PDMB_SLOT_BARRIER();
  PDMB_VMCNT(0);  // drain the clamped tail DMAs before the LDS is released

  // Epilogue: acc[i][j] holds C^T of a 16x16 tile: lane owns row l16 and
  // columns 4g..4g+3.
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
          v.x = pack2<DT>(acc[i][j].x, acc[i][j].y);
          v.y = pack2<DT>(acc[i][j].z, acc[i][j].w);
          *(u32x2*)(crow + col * 2) = v;
        }
      }
    }
  }
}

}  // namespace k256

// Host launcher. Returns hipErrorInvalidValue if the shape is not supported
// by this kernel (caller falls back to the generic kernel).
bool gemm256_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c) {
  if (dt != kBF16 && dt != kF16) return false;
  if (a.K % 64 != 0 || a.K <= 0 || a.N % 8 != 0 || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 4) return false;
  if (a.batch > 1 && (a.sA % 8 || a.sB % 8 || a.sC % 4)) return false;
  if (align_a % 16 || align_b % 16 || align_c % 8) return false;
  // 32-bit per-lane DMA offsets: 255 rows * lda and 63 rows * ldb.
  if ((long long)256 * a.lda * 2 >= (1LL << 31) || (long long)64 * a.ldb * 2 >= (1LL << 31)) return false;
  return true;
}

hipError_t gemm256_launch(int dt, GemmArgs a, int sched, hipStream_t stream) {
  a.tiles_m = (a.M + k256::BM - 1) / k256::BM;
  a.tiles_n = (a.N + k256::BN - 1) / k256::BN;
  a.supertile = choose_supertile(a.tiles_m, a.tiles_n);
  const long long nblocks = (long long)a.tiles_m * a.tiles_n * a.batch;
  if (nblocks <= 0) return hipSuccess;
  if (nblocks > 0x7fffffffLL) return hipErrorInvalidValue;
  dim3 grid((unsigned)nblocks), block(k256::NTHREADS);
#define PDMB_LAUNCH256(D, S) hipLaunchKernelGGL((k256::gemm256_nn<D, S>), grid, block, 0, stream, a)
  if (sched == 4) {  // SCHED 3: the shipping schedule (kMfma256d)
    if (dt == kBF16) PDMB_LAUNCH256(kBF16, 3);
    else PDMB_LAUNCH256(kF16, 3);
    return hipGetLastError();
  }
#ifdef PDMB_EXPERIMENTS
  if (sched >= 10) {  // SCHED 2 experiment flags (bf16 only, A/B builds)
    if (dt != kBF16) return hipErrorInvalidValue;
    switch (sched - 10) {
      case 1: hipLaunchKernelGGL((k256::gemm256_nn<kBF16, 2, false, 1>), grid, block, 0, stream, a); break;
      case 2: hipLaunchKernelGGL((k256::gemm256_nn<kBF16, 2, false, 2>), grid, block, 0, stream, a); break;
      case 4: hipLaunchKernelGGL((k256::gemm256_nn<kBF16, 2, false, 4>), grid, block, 0, stream, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (sched == 3) {  // diagnostic stamp build of SCHED 2 (bf16 only)
    if (dt != kBF16 || !a.dbg) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k256::gemm256_nn<kBF16, 2, true>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  if (dt == kBF16) {
    if (sched == 2) PDMB_LAUNCH256(kBF16, 2);
    else if (sched == 1) PDMB_LAUNCH256(kBF16, 1);
    else PDMB_LAUNCH256(kBF16, 0);
  } else {
    if (sched == 2) PDMB_LAUNCH256(kF16, 2);
    else if (sched == 1) PDMB_LAUNCH256(kF16, 1);
    else PDMB_LAUNCH256(kF16, 0);
  }
  return hipGetLastError();
#else
  return hipErrorInvalidValue;  // experiment schedules are not built
#endif
#undef PDMB_LAUNCH256
}

}  // namespace pdmb
