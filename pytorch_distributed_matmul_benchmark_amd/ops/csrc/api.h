// Host-side C++ API of the native GEMM library (no torch dependency).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#include <utility>

namespace pdmb {

// Shipping kernels (the public `kernel=` surface of ops/gemm.py).
enum Kernel : int {
  kAuto = 0,      // fastest kernel that supports the problem
  kGeneric = 2,   // gemm_generic.hip (any shape)
  kF32_256s = 7,  // gemm_f32_256.hip: exact-fp32 MFMA, 256x256 LDS-DMA tile, staggered DMA
  kMfma256d = 9,  // gemm_mfma256.hip SCHED 3: 8 waves, 256x256, edge tiles (any M, N % 8)
  kFp8W4 = 16,    // gemm_fp8.hip: e4m3 A x column-major B, 4 waves x 128x128, bf16 out
  kMfmaW4 = 21,   // gemm_w4.hip: bf16/fp16 NN, 4 waves x 128x128, AGPR acc, split-K (M, N % 256)
  kT128 = 26,     // gemm_tile.hip: bf16/fp16 NN, 128x128 tile, 4 waves x 64x64, split-K (M, N % 128)
  kT128x2 = 27,   // gemm_tile.hip 128x128 with a 2-stage ring, 2 workgroups per CU (A/B vs kT128)
  kT256x128 = 28, // gemm_tile.hip: 256x128 tile, 4 waves x 128x64, 3-stage ring (M % 256, N % 128)
  kF32W4 = 29,    // gemm_f32_w4.hip: exact fp32, 4 waves x 128x128, AGPR acc (fp32 auto)
  kMfmaW4S = 36,  // gemm_w4.hip W4S: W4 as one K-tile stream per CU (persistent, static tiles)
  kFp8W4S = 37,   // gemm_fp8.hip: the fp8 W4 kernel as one K-tile stream per CU (interior tiles)
  kFp8T128 = 41,      // gemm_tile.hip fp8: 128x128 tile, 4 waves x 64x64, split-K (M, N % 128)
  kFp8T256x128 = 42,  // gemm_tile.hip fp8: 256x128 tile, 4 waves x 128x64, split-K (M % 256, N % 128)
  kF32T128 = 51,      // gemm_f32_tile.hip: exact fp32, 128x128 tile, 4 waves x 64x64, split-K (any M, N % 4)
  kF32T128x2 = 53,    // kF32T128 on 2 LDS stages, two workgroups per CU (grids of >= 2 tiles per CU)
  kT192 = 60,         // gemm_tile.hip: bf16/fp16 NN, 192x192 tile, 4 waves x 96x96, 3-stage ring, split-K
  kT192x128 = 61,     // gemm_tile.hip: bf16/fp16 NN, 192x128 tile, 4 waves x 96x64, 3-stage ring, split-K
  kFp8T192 = 62,      // gemm_tile.hip fp8: 192x192 tile, 4 waves x 96x96, split-K
  kFp8T192x128 = 63,  // gemm_tile.hip fp8: 192x128 tile, 4 waves x 96x64, split-K
  kF32T64 = 64,       // gemm_f32_tile.hip: exact fp32, 64x128 tile, 4 waves x 32x64, split-K (any M, N % 4)
  kF32T64x2 = 65,     // kF32T64 on 2 LDS stages, two workgroups per CU
  kF32W4L = 66,       // gemm_f32_w4.hip: exact-fp32 W4 on the lean K-loop (one whole wave of 256x256 tiles)
};

// Experiment / diagnostic kernel ids (A/B and timing-only builds) live in
// experiments.h; only a library built with PDMB_EXPERIMENTS=1 accepts them.

// True iff this library was built with the experiment kernels.
bool experiments_built();

// dtype kFP8: A, B are OCP fp8 e4m3, B is COLUMN-major (ldb = distance between
// columns, i.e. B is stored as Bt [N,K]), C is bf16 and C = alpha * (A @ B).
struct Problem {
  int dtype;  // DType
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  int lda, ldb, ldc;
  long long sA, sB, sC;
  int batch;
  float alpha = 1.0f;
  // W4 / T128 split-K: K slices per output tile (0 = auto: split only
  // under-filled grids, see choose_splitk; 1 = off). Ignored by the others.
  int splitk = 0;
  // CUs the launch stream may use (a CU-masked stream: parallel/overlap.py
  // MaskedStream); 0 = every CU of the device. The W4 / T128 planner sizes
  // grids for it (a 256-workgroup wave on 248 CUs is two waves).
  int cus = 0;
  // Caller-owned scratch of at least gemm_workspace_bytes(p, kernel) bytes
  // (padded-path copies, split-K partials), stream-ordered with the launch.
  void* workspace = nullptr;
  size_t workspace_bytes = 0;
  // Completion signals (signal_create; nullptr = off): the launch runs the
  // W4 kernel with per-slot tile counters (common.h GemmArgs::sig) — one
  // slot per sig_rows 256-row tile rows of each batch element — and writes
  // sig_epoch into a slot's host flag once all its tiles are stored. Only W4
  // runs signalled (auto: W4 where it would have chosen W4 / W4S; otherwise
  // hipErrorNotSupported); no tail split, no padded path.
  struct Signal* sig = nullptr;
  int sig_rows = 0;
  unsigned sig_epoch = 0;
  // Rows of B holding data (0: all K). The padded path sets it to the caller's
  // K when it pads only A's K (B read in place, rows past K zero by extent).
  int kb = 0;
};

// Completion-signal set of `slots` slots on `device`: device counters
// (hipMalloc, zeroed once, never reset: launch e of the set completes a slot
// at e x its tile count) and host-mapped fine-grained flags the GPU writes
// and a host thread polls.
struct Signal {
  unsigned* dev = nullptr;       // tile counters
  unsigned* host = nullptr;      // flags, host address
  unsigned* host_dev = nullptr;  // flags, device address of the same memory
  int slots = 0;
  int device = 0;
};
hipError_t signal_create(int device, int slots, Signal** out);
void signal_destroy(Signal* s);
// Host wait until flag[slot] reaches `epoch` (wrap-safe); false on timeout.
bool signal_wait(const Signal* s, int slot, unsigned epoch, double timeout_s);
unsigned signal_flag(const Signal* s, int slot);
// Host store of flag[slot] (release); gate(): a one-wave kernel on `stream`
// that waits until flag[slot] reaches `value` or `timeout_s` pass (reduce.hip).
void signal_set(Signal* s, int slot, unsigned value);
hipError_t gate(const Signal* s, int slot, unsigned value, double timeout_s, hipStream_t stream);
// Tile rows of one completion unit for this problem on W4: the rows of one
// 256-workgroup round of its XCD-aware order (map_tile), so pieces finish in
// order and each piece is a whole number of rounds. 0: cannot be signalled.
int signal_granule(const Problem& p, int kernel);

// Split-K arrival counters are a library resource: one zeroed block per
// (device, stream), created on first use and left zeroed by every launch
// (launches on one stream never overlap). kMaxSplitTiles bounds the tiles of
// one split-K launch.
// Graphs: a split-K launch captured on stream s bakes s's counter block into
// the graph (a stream still capturing with no block yet runs unsplit instead:
// hipMalloc is not capturable). Two replays of graphs captured on the same
// stream, or a replay beside eager split-K launches on that stream, must
// therefore not run concurrently — they would share arrival counters. The
// library's own timing loop (bench_gemm) captures on a private stream and
// replays one graph at a time.
constexpr int kMaxSplitTiles = 4096;

// Kernel an `auto` call runs through zero-padded workspace copies (the
// padded fast path), or -1 if `auto` runs the problem as it is.
int resolve_padded(const Problem& p);

// Scratch bytes `gemm(p, kernel, ...)` needs in p.workspace (0 if none).
size_t gemm_workspace_bytes(const Problem& p, int kernel);

// K slices the W4 / T128 kernel that `kernel` resolves to would use for this
// problem (1 = no split; 0 = neither runs it, or p.splitk is not possible).
int choose_splitk(const Problem& p, int kernel);

// Wave-quantisation tail (gemm_dispatch.cpp tail_plan): {M1, S, 0} when auto
// runs rows [0, M1) as one launch and rows [M1, M) split S ways as a second;
// {0, S, T1} (tile-range form) when it runs the first T1 tiles of its tile
// order as one launch and the rest split S ways; {0, 1, 0}: one launch.
struct TailSplit {
  int m1, S, tiles_dp;
  int sub;  // parts per 256x256 tile of a refined tail's second launch (1: split-K tail)
};
TailSplit tail_split(const Problem& p, int kernel);

// Which kernel `kernel` (kAuto allowed) resolves to for this problem;
// -1 if the requested kernel cannot run it.
int resolve_kernel(const Problem& p, int kernel);

// The planner's whole decision for a problem (shape-only use is fine: the
// operand pointers are only checked for alignment): the kernel, its split-K,
// the cost model's time (us; 0 for kernels it does not price) and the
// wave-quantisation tail plan {tail_m1, tail_S} ({0, 1}: one launch).
struct PlanInfo {
  int kernel, splitk;
  double cost_us;
  int tail_m1, tail_S, tail_tiles_dp, tail_sub;
};
PlanInfo plan_info(const Problem& p, int kernel);

// Enqueue C = A @ B on `stream`. Returns hipSuccess or an error; *used (if
// non-null) receives the kernel that ran. With kAuto, a large problem whose K /
// N / alignment miss the fast kernels runs on them through zero-padded
// workspace copies (gemm_dispatch.cpp "padded fast path").
hipError_t gemm(const Problem& p, int kernel, hipStream_t stream, int* used);

// Native timing loop: `warmup` untimed launches, then `iters` launches
// bracketed by hipEvents on `stream` (optionally captured once into a
// hipGraph and replayed, which removes host launch gaps). Returns the
// total elapsed milliseconds of the timed region in *ms.
hipError_t bench_gemm(const Problem& p, int kernel, int iters, int warmup, bool use_graph,
                      hipStream_t stream, float* ms);

const char* kernel_name(int kernel);

// Comm proxy for overlap experiments (scripts/cu_mask_overlap.py): copy
// `bytes` (multiple of 16) from src to dst with exactly `blocks` 256-thread
// workgroups, the footprint of an RCCL collective's channels.
hipError_t comm_proxy(void* dst, const void* src, size_t bytes, int blocks, hipStream_t stream);

// dst[i] = sum over s < nsrc of srcs[s][i] (fp32 accumulate, sources in index
// order, RNE to the element type; dtype 0 f32, 1 f16, 2 bf16). dst may alias a
// source; 16-B vectors when every pointer is 16-B aligned. The local step of the direct two-shot
// all-reduce (reduce.hip). Sources may be peer-mapped (IPC) addresses.
// max_blocks > 0 caps the grid (a reduce running beside a GEMM).
constexpr int kMaxReduceSrcs = 16;
hipError_t reduce_sum(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t stream,
                      int max_blocks = 0);

// n <= kMaxCopies copies dsts[i] <- srcs[i] (bytes[i] bytes each; zero-length
// entries skipped) in ONE launch, `blocks_per` 256-thread workgroups per copy
// (0: 32). The peer-memory all-gather's pull (parallel/ipc.py): every peer's
// block is read over its own xGMI link at once, from one stream.
constexpr int kMaxCopies = 16;
hipError_t multi_copy(void* const* dsts, const void* const* srcs, const size_t* bytes, int n, int blocks_per,
                      hipStream_t stream);

// Diagnostic builds write per-wave stamps here (device memory; nullptr = off).
void set_debug_buffer(void* p);

// Stream-K slots per tile (the most workgroups any tile of a span-tile range
// is shared by, G workgroups over span x nk K-tiles; gemm_fp8.hip gemm_fp8_sk).
int fp8_sk_slots(long long span, int nk, long long G);

}  // namespace pdmb
