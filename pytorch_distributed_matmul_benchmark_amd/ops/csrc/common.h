// Shared types and helpers for the gfx950 (CDNA4 / MI355X) GEMM kernels.
//
// Everything here is written for gfx950 only: wave64, MFMA 16x16x32 for
// 16-bit inputs, MFMA 16x16x4 for exact fp32, LDS-DMA (buffer_load ... lds)
// staging. See docs/ARCHITECTURE.md for the design notes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdmb {

// ---- element / fragment types -------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) s16x8 lds_s16x8;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;

// Data-type tags shared by host and device code. Values are part of the
// binding ABI (ops/gemm.py mirrors them).
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kFP8 = 3 /* OCP e4m3fn in, bf16 out */ };

// One MFMA 16x16x32 step on 16-bit operands (a: 8 elements/lane, b: 8).
template <int DT>
__device__ __forceinline__ f32x4 mfma16x16x32(s16x8 a, s16x8 b, f32x4 c);

template <>
__device__ __forceinline__ f32x4 mfma16x16x32<kBF16>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16x16x32<kF16>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// fp32 -> 16-bit with round-to-nearest-even (hipcc emits v_cvt_pk_bf16_f32 /
// v_cvt_pk_f16_f32 on gfx950; NaN stays NaN).
template <int DT>
__device__ __forceinline__ unsigned int pack2(float lo, float hi);
template <>
__device__ __forceinline__ unsigned int pack2<kBF16>(float lo, float hi) {
  __bf16 l = (__bf16)lo, h = (__bf16)hi;
  return (unsigned int)__builtin_bit_cast(unsigned short, l) |
         ((unsigned int)__builtin_bit_cast(unsigned short, h) << 16);
}
template <>
__device__ __forceinline__ unsigned int pack2<kF16>(float lo, float hi) {
  _Float16 l = (_Float16)lo, h = (_Float16)hi;
  return (unsigned int)__builtin_bit_cast(unsigned short, l) |
         ((unsigned int)__builtin_bit_cast(unsigned short, h) << 16);
}

template <int DT>
__device__ __forceinline__ float to_f32(unsigned short v);
template <>
__device__ __forceinline__ float to_f32<kBF16>(unsigned short v) {
  return __uint_as_float(((unsigned int)v) << 16);
}
template <>
__device__ __forceinline__ float to_f32<kF16>(unsigned short v) {
  return (float)__builtin_bit_cast(_Float16, v);
}

// ---- kernel argument block ----------------------------------------------
// Row-major C[b] = A[b] @ B[b]: A is [M,K] (lda), B is [K,N] (ldb), C is
// [M,N] (ldc); all strides in elements. Batch strides in elements.
struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  int kb;  // rows of B holding data (<= K): rows [kb, K) read as zeros through the B
           // descriptors' extent (the padded path's K tail: only A is copied)
  int lda, ldb, ldc;
  long long sA, sB, sC;
  int batch;
  int tiles_m, tiles_n;  // output tiles per batch element
  int supertile;         // XCD-aware round order: 1 = 16x16 tiles, 2-5 thin rounds (map_tile), 0: grouped
  float alpha;           // fp8 only: C = alpha * (A @ B) (per-tensor scales folded)
  unsigned long long* dbg;  // diagnostic builds only (in-kernel stamps); nullptr otherwise
  // Split-K (W4 only; splitk <= 1 = off): K-tile range [slice * kt_per, +kt_per)
  // per workgroup; the S slices of one output tile meet in `part` (fp32, S
  // tile images: one slot per slice) and `flags` (2 counters per tile, zero between launches).
  int splitk, kt_per;
  float* part;
  unsigned* flags;
  // S == 2: the reducer loads the other slice's block rows one row ahead of
  // their use (splitk.h splitk_load_other); 0 = the row-by-row splitk_row
  // path (A/B switch: PDMB_SPLITK_PREFETCH=0).
  int meet_prefetch;
  // Persistent kernels: per-XCD tile queues (8 tickets + 1 exit counter,
  // zero at launch) and the grid (one workgroup per usable CU).
  unsigned* queue;
  int pers_grid;
  // Tile-range launches of the wave-quantisation tail (fp8 W4 / W4S,
  // gemm_dispatch.cpp tail_plan): tile_end > 0 — the launch covers tiles
  // [0, tile_end) of map_tile's order only (the whole waves); tile_span > 0 —
  // it covers tiles [tile_base, tile_base + tile_span), each split `splitk`
  // ways (block = slice * tile_span + local tile; the meet's tile id is the
  // local index, so the slots and counters cover tile_span tiles).
  int tile_end, tile_base, tile_span;
  // Completion signals (W4 only; sig == nullptr = off; parallel/overlap.py
  // signalled pieces). Output tile rows are grouped into slots of sig_rows
  // tile rows, sig_slots per batch element. A tile's C leaves write-through
  // (sc1), every storing wave drains, then one lane adds 1 to the slot's
  // device counter (relaxed, agent); the tile whose add completes the slot
  // for this launch (counter == sig_epoch x tiles in the slot; counters are
  // never reset, so launch e of one signal set completes at e x tiles) stores
  // sig_epoch into the slot's host-mapped flag (system scope), which a host
  // thread polls before issuing that piece's collective.
  unsigned* sig;
  unsigned* sig_host;
  int sig_rows, sig_slots;
  unsigned sig_epoch;
};

// Slot of output tile (bz, tm) and the counter value that completes it in
// this launch (GemmArgs::sig).
__device__ __forceinline__ void signal_tile(const GemmArgs& a, int bz, int tm) {
  const int pr = tm / a.sig_rows;
  const int slot = bz * a.sig_slots + pr;
  const int rows = min(a.sig_rows, a.tiles_m - pr * a.sig_rows);
  const unsigned target = a.sig_epoch * (unsigned)(rows * a.tiles_n);
  const unsigned old = __hip_atomic_fetch_add(a.sig + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1u == target)
    __hip_atomic_store(a.sig_host + slot, a.sig_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- C epilogue through LDS (W4 bf16/fp16, W4 fp8) --------------------------
// After the K-loop a wave holds 128 columns of 16-row blocks as C^T MFMA
// tiles: for block row i, lane (l16, g) owns row l16 and columns 16j + 4g ..
// +3 of each 16-column block j — 8-byte pieces. Stored directly, every store
// instruction writes 16 rows x 32 B: a 256x256 tile is 4096 partial-line
// write requests, and the 256 CUs, which run in lock-step, issue them at the
// same moment (the tile timeline, scripts/tile_timeline.py: 7-8 us per tile
// at 16k, a third of W4's per-tile fixed cost). Staged through a wave-private
// LDS buffer, each 16-row block leaves as 4 dwordx4 stores of 4 whole 256-B
// rows: a quarter of the requests, all of them whole lines.
// Buffer rows are NB * 32 + 8 bytes (W4: 264): the b64 writes (16 lanes =
// 16 rows, 2 banks each) and the b128 reads (16 B chunks of whole rows)
// are conflict-free for NB = 8 and NB = 4. NB = 6 (the 192-column tiles of
// gemm_tile.hip): rows of NB * 32 + 16 = 208 B, 52 dwords, put the 16 rows'
// b64 writes on 16 distinct 4-bank slots (52 r mod 64, r < 16).
template <int NB>
constexpr int epi_pitch() { return NB * 32 + (NB % 4 ? 16 : 8); }
template <int NB = 8>
constexpr int epi_buf() { return 16 * epi_pitch<NB>(); }
constexpr int kEpiPitch = epi_pitch<8>();
constexpr int kEpiBuf = epi_buf<8>();  // one 16-row block of W4, 4224 B

// Store block row v (v[j] = the fp32 C^T tile j, scaled by `alpha` if
// SCALE) of a wave's 16 x (NB * 16) output at (row0, col0) of C (row stride
// ldc_b bytes) through `buf` (epi_buf<NB>() bytes of LDS owned by this
// wave). MASK: rows >= M are skipped, column chunks are cut at N (N % 4 ==
// 0: a chunk is all, half or none).
// NTS (default): non-temporal C stores (global_store ... nt). C is written
// once and never read back by the kernel; hipBLASLt's fp8 kernels store it
// the same way ("NTD"). Measured vs plain stores (profiles/
// r2_ntstore_ab.jsonl): fp8 W4 4096^3 2538 -> 2760 TF, fp8 W4S 16k +0.6 %,
// bf16 W4S 16384^2 x 2048 +1.1 %, 16k +0.2 %; never slower.
// WT: write-through (sc1) buffer stores instead — a tile whose C another
// kernel reads while this launch still runs (GemmArgs::sig): with every
// storing wave drained, the bytes are in memory when the slot is signalled
// (cdna_hip_programming.md Guideline 16 R1; no release fence).
template <int DT, bool MASK, bool SCALE, int NB = 8, bool NTS = true, bool WT = false>
__device__ __forceinline__ void store_block16(char* buf, const f32x4 (&v)[NB], float alpha, char* C,
                                              long long ldc_b, int row0, int col0, int M, int N,
                                              int lane) {
  constexpr int P = epi_pitch<NB>();
  constexpr int CPR = NB * 2;    // 16-B chunks per row
  constexpr int NR = 16 * CPR / 64;  // read instructions: chunk q = lane + 64 r is row q / CPR
  static_assert(16 * CPR % 64 == 0, "whole 16-row blocks per read round");
  const int l16 = lane & 15, g = lane >> 4;
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* lb = (lds_char*)(lds_void*)buf;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    u32x2 w;
    if constexpr (SCALE) {
      w.x = pack2<DT>(v[j].x * alpha, v[j].y * alpha);
      w.y = pack2<DT>(v[j].z * alpha, v[j].w * alpha);
    } else {
      w.x = pack2<DT>(v[j].x, v[j].y);
      w.y = pack2<DT>(v[j].z, v[j].w);
    }
    *(lds_u32x2*)(lb + l16 * P + (j * 16 + 4 * g) * 2) = w;
  }
  if constexpr (WT) {
    // one descriptor per 16-row block (uniform base; offsets < 16 rows x ldc_b)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        C + (long long)row0 * ldc_b + (long long)col0 * 2, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int q = lane + 64 * r, rl = q / CPR, ch = q % CPR;
      const u32x4 x = *(lds_u32x4_t*)(lb + rl * P + ch * 16);
      const int row = row0 + rl, col = col0 + 8 * ch;
      const int off = rl * (int)ldc_b + ch * 16;
      if (!MASK || (row < M && col + 8 <= N)) {
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 16 /* sc1 */);
      } else if (row < M && col + 4 <= N) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{x.x, x.y}, rs, off, 0, 16);
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int q = lane + 64 * r, rl = q / CPR, ch = q % CPR;
    const u32x4 x = *(lds_u32x4_t*)(lb + rl * P + ch * 16);
    const int row = row0 + rl, col = col0 + 8 * ch;
    char* p = C + (long long)row * ldc_b + (long long)col * 2;
    if constexpr (MASK) {
      if (row < M) {
        if (col + 8 <= N) {
          if constexpr (NTS) __builtin_nontemporal_store(x, (u32x4*)p);
          else *(u32x4*)p = x;
        } else if (col + 4 <= N) {
          *(u32x2*)p = u32x2{x.x, x.y};
        }
      }
    } else {
      if constexpr (NTS) __builtin_nontemporal_store(x, (u32x4*)p);
      else *(u32x4*)p = x;
    }
  }
}

// fp32 C (exact-fp32 kernels): the same whole-row epilogue for f32x4 C^T
// blocks. Buffer rows are NB * 64 + 16 bytes (528 for NB = 8: the b128
// writes of 16 rows at one column land 4 banks apart, conflict-free); each
// read instruction moves 64 / (NB * 4) whole rows; stores are non-temporal.
// MASK: rows >= M skipped, 16-B chunks at or past N dropped (N % 4 == 0).
template <int NB>
constexpr int epi_buf_f32() { return 16 * (NB * 64 + 16); }

// PERM: v[j] holds columns 64 (j >> 2) + 16 g + 4 (j & 3) .. + 3 of the lane's
// row (the b128-B-read mapping of gemm_f32_tile.hip / gemm_f32_w4.hip)
// instead of 16 j + 4 g .. + 3.
template <bool MASK, int NB = 8, bool PERM = false>
__device__ __forceinline__ void store_block16_f32(char* buf, const f32x4 (&v)[NB], char* C, long long ldc_b,
                                                  int row0, int col0, int M, int N, int lane) {
  static_assert(!PERM || NB % 4 == 0, "PERM: groups of 4 column blocks");
  constexpr int P = NB * 64 + 16;
  constexpr int CPR = NB * 4;    // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per read instruction
  const int l16 = lane & 15, g = lane >> 4;
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* lb = (lds_char*)(lds_void*)buf;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    *(__attribute__((address_space(3))) f32x4*)(lb + l16 * P + (PERM ? 64 * (j >> 2) + 16 * g + 4 * (j & 3) : j * 16 + 4 * g) * 4) =
        v[j];
  const int rl = lane / CPR, ch = lane % CPR;
#pragma unroll
  for (int r = 0; r < 16 / RPI; ++r) {
    const u32x4 x = *(lds_u32x4_t*)(lb + (RPI * r + rl) * P + ch * 16);
    const int row = row0 + RPI * r + rl, col = col0 + 4 * ch;
    char* p = C + (long long)row * ldc_b + (long long)col * 4;
    if (!MASK || (row < M && col + 4 <= N)) __builtin_nontemporal_store(x, (u32x4*)p);
  }
}

// ---- Tile timeline trace (diagnostic kernel ids; a.dbg != nullptr) --------
// Per tile 8 u64 at dbg[row * 8] (row = the tile's virtual block): [0] start, [1] first K-tile's
// fragments in registers, [2] K-loop done, [3] C stored and drained
// (vmcnt 0), all s_memrealtime (the chip-wide 100 MHz clock, so stamps of
// different CUs compare); [4] HW_ID (CU / SH / SE), [5] XCC_ID, [6] tm << 32 | tn.
// One lane writes them with vector stores (scripts/tile_timeline.py reads them).
__device__ __forceinline__ unsigned long long tile_clock() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

struct TileTrace {
  unsigned long long t[4];
};

__device__ __forceinline__ void tile_trace_write(const GemmArgs& a, const TileTrace& tr, int row, int tm,
                                                 int tn) {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0 && a.dbg) {
    unsigned long long* d = a.dbg + (size_t)row * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = tr.t[i];
    d[4] = hw;
    d[5] = xcc;
    d[6] = ((unsigned long long)(unsigned)tm << 32) | (unsigned)tn;
    d[7] = 0;
  }
}

// ---- LDS-DMA helpers (shared by the LDS-DMA kernels) ----------------------
// Raw buffer descriptor (gfx950 dword3 = 0x00020000: 32-bit data format,
// raw addressing). Bytes at or beyond num_records read as zero, which
// handles the M / N edges with no masking in the K-loop. num_records is
// clamped with 32-bit scalar logic (SALU has no 64-bit less-than).
__device__ __forceinline__ u32x4 make_rsrc(const char* base, long long bytes) {
  const unsigned long long p = (unsigned long long)base;
  unsigned int hi = (unsigned int)((unsigned long long)bytes >> 32);
  unsigned int lo = (unsigned int)bytes;
  // opaque halves: otherwise hipcc folds the clamp back into a 64-bit compare,
  // which SALU lacks, and keeps its constant in a VGPR pair
  asm("" : "+s"(hi), "+s"(lo));
  const unsigned int nr = (hi & 0x80000000u) ? 0u : (hi ? 0xffffffffu : lo);
  u32x4 r;
  r.x = (unsigned int)p;
  r.y = (unsigned int)(p >> 32) & 0xffffu;
  r.z = nr;
  r.w = 0x00020000u;
  return r;
}

// One LDS-DMA wave-instruction: 64 lanes x 16 B from rsrc+voff into LDS at
// lds_base + lane*16. Written as inline asm on purpose: hipcc (ROCm 7.2)
// otherwise treats every later ds_read_b64_tr_b16 as possibly aliasing the
// in-flight DMA and inserts s_waitcnt vmcnt(0), which drains the pipeline.
// The count is ours to keep: every wait on these is an explicit vmcnt(N).
// M0 is saved/restored around the statement (compiler-reserved register).
__device__ __forceinline__ void dma16(u32x4 rsrc, uint32_t voff, uint32_t lds_base) {
  unsigned int keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_base)
      : "memory");
}

// LDS-DMA with a scalar source offset to M0 = lds0w + OFF, OFF an immediate
// (known once a K-tile's item loop is unrolled): M0 is formed by the one
// SALU add that replaces an s_mov, instead of from ~32 precomputed addresses
// held in SGPRs (W4: 96 -> 67 SGPRs; what made W4S fit). M0 is clobbered.
__device__ __forceinline__ void dma16_at(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds0w,
                                         uint32_t off) {
  asm volatile(
      "s_add_u32 m0, %3, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds0w), "i"(off)
      : "memory", "m0", "scc");
}

// dma16_at with 4 wait states before the load (s_nop 3 for the s_nop 0):
// 5 states from the end of any instruction before the statement. A VALU write
// of an SGPR needs 5 wait states before a VMEM instruction reads it, and
// hipcc, which pads its own loads (s_nop 3 after v_readfirstlane + s_mul),
// cannot see the read inside this asm. In W4S and fp8 W4S it restores a few
// spilled soffsets with v_readlane right before the first K-tiles' pieces of
// a tile (round 6, tests/test_sgpr_vmem_hazard.py); those K-tiles use this.
__device__ __forceinline__ void dma16_at_pad(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds0w,
                                             uint32_t off) {
  asm volatile(
      "s_add_u32 m0, %3, %4\n\t"
      "s_nop 3\n\t"
      "buffer_load_dwordx4 %0, %1, %2 offen lds"
      :
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds0w), "i"(off)
      : "memory", "m0", "scc");
}

// ---- block -> output tile mapping -------------------------------------
// Speed only (never correctness): workgroups are dealt round-robin over the
// 8 XCDs (blocks b and b+8 share an XCD). In super-tile mode every "round"
// of 256 workgroups (one per CU) covers one 16x16-tile super-tile, and each
// XCD's 32 workgroups cover a 4x8 sub-block of it, so an XCD's L2 serves
// 4 A-panels + 8 B-panels per K-step (12 fetches instead of 64) and the
// whole chip touches 32 panels per K-step (shared through Infinity Cache).
// Super-tiles sweep N fastest so A panels stay Infinity-Cache resident.
// Otherwise: grouped order with 16 tile-rows per group (chip-wide locality).
// Thin grids (a row chunk of an overlap GEMM, a ws=8 column shard) keep the
// 32-workgroup XCD blocks with a 256-tile round of another shape, given as
// (XCD grid xm x xn) x (block bm x bn): supertile 2 = 8 x 32 tiles (2x4 of
// 4x8), 3 = 32 x 8 (4x2 of 8x4), 4 = 4 x 64 (1x8 of 4x8), 5 = 64 x 4 (8x1 of
// 8x4). sub: XCD sub-block shape in 16x16 rounds, 0 = 4 (M) x 8 (N),
// 1 = 8 x 4 ("tall"), 2 = 2 x 16 ("wide").
inline int choose_supertile(int tiles_m, int tiles_n) {
  if (tiles_m % 16 == 0 && tiles_n % 16 == 0) return 1;
  if (tiles_m % 8 == 0 && tiles_n % 32 == 0) return 2;
  if (tiles_m % 32 == 0 && tiles_n % 8 == 0) return 3;
  if (tiles_m % 4 == 0 && tiles_n % 64 == 0) return 4;
  if (tiles_m % 64 == 0 && tiles_n % 4 == 0) return 5;
  return 0;
}

#ifdef PDMB_EXPERIMENTS
// Experiments (round 6): the thin round that follows the grid's aspect, in
// place of the 16 x 16 round, for 1-4 rounds of a wide or tall grid
// (kFp8W4SThin / kMfmaW4SThin): wide 4 x 64 then 8 x 32, tall 64 x 4 then 32 x 8.
inline int thin_supertile(int tiles_m, int tiles_n) {
  if (tiles_n > tiles_m) {
    if (tiles_m % 4 == 0 && tiles_n % 64 == 0) return 4;
    if (tiles_m % 8 == 0 && tiles_n % 32 == 0) return 2;
  } else if (tiles_m > tiles_n) {
    if (tiles_m % 64 == 0 && tiles_n % 4 == 0) return 5;
    if (tiles_m % 32 == 0 && tiles_n % 8 == 0) return 3;
  }
  return choose_supertile(tiles_m, tiles_n);
}
#endif

__host__ __device__ __forceinline__ void map_tile(const GemmArgs& a, int b, int& bz, int& tm, int& tn,
                                                  int sub = 0) {
  const int tpb = a.tiles_m * a.tiles_n;
#ifdef PDMB_EXPERIMENTS
  // 9 (experiments, round 6): the 32 x 8 round of mode 3 as an 8 x 1 XCD grid
  // of 4 x 8 blocks (each XCD spans the grid's 8 tile columns: 4 A + 8 B
  // panels per K-step instead of mode 3's 8 A + 4 B)
  const bool thin = (a.supertile >= 2 && a.supertile <= 5) || a.supertile == 9;
#else
  const bool thin = a.supertile >= 2 && a.supertile <= 5;
#endif
  if (thin) {
    const int x = b & 7, j = b >> 3;
    const int round = j >> 5, i = j & 31;
    const int st = a.supertile;
    const int xn = st == 2 ? 4 : st == 3 ? 2 : st == 4 ? 8 : 1;  // XCD grid columns
    const int bn = (st == 2 || st == 4 || st == 9) ? 8 : 4, bm = 32 / bn;  // XCD block
    const int SM = (8 / xn) * bm, SN = xn * bn;                   // round shape in tiles
    const int st_n = a.tiles_n / SN;
    const int st_per_b = (a.tiles_m / SM) * st_n;
    bz = round / st_per_b;
    const int s = round - bz * st_per_b;
    const int sr = s / st_n, sc = s - sr * st_n;
    tm = sr * SM + (x / xn) * bm + i / bn;
    tn = sc * SN + (x % xn) * bn + i % bn;
  } else if (a.supertile) {
    const int j = b >> 3;
    const int round = j >> 5, i = j & 31;
    // supertile 6: mode 1 with the XCD -> block position rotated by one per
    // round, so every XCD visits every position of the 16 x 16 round (A/B)
    const int x = a.supertile == 6 ? ((b & 7) + round) & 7 : b & 7;
    const int st_n = a.tiles_n >> 4, st_m = a.tiles_m >> 4;
    const int st_per_b = st_m * st_n;
    bz = round / st_per_b;
    const int s = round - bz * st_per_b;
#ifdef PDMB_EXPERIMENTS
    int sr = s / st_n, sc = s - sr * st_n;
    // round-order A/Bs (experiments build only; the Infinity Cache reuse of
    // the panels between consecutive rounds, profiles/r8c_*: no effect): 7 =
    // snake (odd super-tile rows sweep N backwards), 8 = the super-tiles
    // sweep M fastest
    if (a.supertile == 7 && (sr & 1)) sc = st_n - 1 - sc;
    if (a.supertile == 8) {
      sc = s / st_m;
      sr = s - sc * st_m;
    }
#else
    (void)st_m;
    const int sr = s / st_n, sc = s - sr * st_n;
#endif
    if (sub == 2) {  // XCD sub-block 2 (M) x 16 (N)
      tm = (sr << 4) + (x << 1) + (i >> 4);
      tn = (sc << 4) + (i & 15);
    } else if (sub == 1) {  // XCD sub-block 8 (M) x 4 (N)
      tm = (sr << 4) + ((x & 1) << 3) + (i >> 2);
      tn = (sc << 4) + ((x >> 1) << 2) + (i & 3);
    } else {     // XCD sub-block 4 (M) x 8 (N)
      tm = (sr << 4) + ((x >> 1) << 2) + (i >> 3);
      tn = (sc << 4) + ((x & 1) << 3) + (i & 7);
    }
  } else {
    bz = b / tpb;
    const int L = b - bz * tpb;
    const int gsz = 16 * a.tiles_n;
    const int grp = L / gsz;
    const int first_m = grp * 16;
    int gm = a.tiles_m - first_m;
    gm = gm < 16 ? gm : 16;
    const int r = L - grp * gsz;
    tm = first_m + r % gm;
    tn = r / gm;
  }
}

}  // namespace pdmb
