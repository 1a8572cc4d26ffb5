// Kernel selection and the native hipEvent timing loop.
//
// The reference times `iters` back-to-back torch.matmul calls between two
// CUDA events from Python (matmul_benchmark.py:54-68, matmul_scaling_
// benchmark.py:85-99). Here the loop itself is native: no Python and no
// allocator in the timed region, each launch writes a caller-owned output,
// and the launches can be captured once into a hipGraph.
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <thread>
#include <unordered_map>

#include <cstdlib>

#include "api.h"
#include "common.h"
#ifdef PDMB_EXPERIMENTS
#include "experiment_ids.h"
#endif

namespace pdmb {

bool gemm256_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm256_launch(int dt, GemmArgs a, int sched, hipStream_t stream);
hipError_t gemm_generic_launch(int dt, GemmArgs a, bool vec, hipStream_t stream);
bool gemm_f32_256_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm_f32_256_launch(GemmArgs a, int variant, hipStream_t stream);
hipError_t gemm_f32_w4_launch(GemmArgs a, hipStream_t stream, int variant);
bool gemm_f32_w4s_fits(const GemmArgs& a);  // experiments build: kF32W4S
bool gemm_f32_w4l_fits(const GemmArgs& a);
bool gemm_w4s_lean_fits(const GemmArgs& a);  // experiments build: kMfmaW4SLean
bool gemm_f32_tile_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
bool gemm_f32_tile_ln_fits(const GemmArgs& a);
hipError_t gemm_f32_tile_launch(GemmArgs a, hipStream_t stream, int variant);
bool gemm_fp8_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm_fp8_launch(GemmArgs a, int variant, hipStream_t stream);
bool gemm_fp8_w4s_fits(const GemmArgs& a);
bool gemm_fp8_w4s_k4_fits(const GemmArgs& a);
bool gemm_w4_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm_w4_launch(int dt, GemmArgs a, hipStream_t stream, int sub = 0);
bool gemm_tile_supported(int dt, int bm, const GemmArgs& a, size_t align_a, size_t align_b,
                         size_t align_c);
hipError_t gemm_tile_launch(int kernel, int dt, GemmArgs a, hipStream_t stream);

static unsigned long long* g_debug_buffer = nullptr;

// The planner's A/B switches (PDMB_SPLIT3, PDMB_T192, PDMB_TILE_TAIL, ...:
// each names one rule below and the measurement behind it). They are read
// ONLY in a PDMB_EXPERIMENTS=1 build, where scripts/ab_kernels.py flips them
// per call to price a rule against its absence. The shipping build ignores
// the environment: every rule is fixed at its shipped value, so a plan
// depends on the shape, layout, dtype and CU budget alone
// (tests/test_golden_plans_cpu.py pins the reference shapes' plans).
// ab_switch(name) = the variable's integer value, or -1 when it is unset
// (always -1 in the shipping build).
static int ab_switch(const char* name) {
#ifdef PDMB_EXPERIMENTS
  const char* e = std::getenv(name);
  return e && e[0] ? std::atoi(e) : -1;
#else
  (void)name;
  return -1;
#endif
}
static bool ab_off(const char* name) { return ab_switch(name) == 0; }  // "=0 leaves the rule out"

void set_debug_buffer(void* p) { g_debug_buffer = (unsigned long long*)p; }

// The problem's shape / layout fields only (the planner's supports() checks:
// no environment reads, which cost ~0.3 us each and ran once per kernel model
// per plan() call).
static GemmArgs shape_args(const Problem& p) {
  GemmArgs a{};
  a.A = p.A;
  a.B = p.B;
  a.C = p.C;
  a.M = p.M;
  a.N = p.N;
  a.K = p.K;
  a.lda = p.lda;
  a.ldb = p.ldb;
  a.ldc = p.ldc;
  a.sA = p.sA;
  a.sB = p.sB;
  a.sC = p.sC;
  a.batch = p.batch < 1 ? 1 : p.batch;
  a.kb = p.kb > 0 && p.kb < p.K ? p.kb : p.K;
  return a;
}

static GemmArgs to_args(const Problem& p) {
  GemmArgs a{};
  a.A = p.A;
  a.B = p.B;
  a.C = p.C;
  a.M = p.M;
  a.N = p.N;
  a.K = p.K;
  a.lda = p.lda;
  a.ldb = p.ldb;
  a.ldc = p.ldc;
  a.sA = p.sA;
  a.sB = p.sB;
  a.sC = p.sC;
  a.batch = p.batch < 1 ? 1 : p.batch;
  a.kb = p.kb > 0 && p.kb < p.K ? p.kb : p.K;
  a.dbg = g_debug_buffer;
  a.alpha = p.alpha;
  // read per launch, so an in-process A/B can flip it (scripts/ab_kernels.py)
  a.meet_prefetch = ab_off("PDMB_SPLITK_PREFETCH") ? 0 : 1;
  if (p.sig) {
    a.sig = p.sig->dev;
    a.sig_host = p.sig->host_dev;
    a.sig_rows = p.sig_rows;
    const int tm = (p.M + 255) / 256;
    a.sig_slots = p.sig_rows > 0 ? (tm + p.sig_rows - 1) / p.sig_rows : 0;
    a.sig_epoch = p.sig_epoch;
  }
  return a;
}

static bool generic_vec_ok(const Problem& p) {
  const int vec_el = p.dtype == kF32 ? 4 : 8;       // 16-B vectors
  const size_t esz = p.dtype == kF32 ? 4 : 2;
  const size_t va = (size_t)p.A, vb = (size_t)p.B, vc = (size_t)p.C;
  if (va % 16 || vb % 16 || vc % (esz * 4)) return false;
  if (p.lda % vec_el || p.ldb % vec_el || p.ldc % 4) return false;
  if (p.batch > 1 && (p.sA % vec_el || p.sB % vec_el || p.sC % 4)) return false;
  return true;
}

bool experiments_built() {
#ifdef PDMB_EXPERIMENTS
  return true;
#else
  return false;
#endif
}

// Experiment / diagnostic kernels (experiments.h): every id, its resolution,
// workspace, launch and name, compiled only into a PDMB_EXPERIMENTS=1 build;
// the shipping build sees stubs that refuse every non-shipping id.
#ifdef PDMB_EXPERIMENTS
static bool is_experiment(int k);
static bool experiment_is_fp8(int k);
static int experiment_resolve_fp8(const Problem& p, int kernel, bool s_fits);
static int experiment_resolve(const Problem& p, int kernel, bool fast, bool w4, bool t128, bool f32fast);
static size_t experiment_workspace_bytes(const Problem& p, int k);
static hipError_t experiment_launch(const Problem& p, int k, const GemmArgs& a, hipStream_t stream);
static const char* experiment_name(int k);
#else
static bool is_experiment(int) { return false; }
static bool experiment_is_fp8(int) { return false; }
static int experiment_resolve_fp8(const Problem&, int, bool) { return -1; }
static int experiment_resolve(const Problem&, int, bool, bool, bool, bool) { return -1; }
static size_t experiment_workspace_bytes(const Problem&, int) { return 0; }
static hipError_t experiment_launch(const Problem&, int, const GemmArgs&, hipStream_t) {
  return hipErrorInvalidValue;
}
static const char* experiment_name(int) { return "auto"; }
#endif

static bool is_fp8_kernel(int k) {
  return k == kFp8W4 || k == kFp8W4S || k == kFp8T128 || k == kFp8T256x128 || k == kFp8T192 ||
         k == kFp8T192x128 || experiment_is_fp8(k);
}

static int device_cus();
static int fp8_split(const Problem& p);
static bool w4s_fits(const Problem& p);
static bool w4s_auto(const Problem& p);
static bool supports(const Problem& p, int kernel);
struct Plan;
static bool f32w4l_whole_waves(const Problem& p, const GemmArgs& a, const Plan& pl);
static int signal_kernel(const Problem& p, int kernel);

struct Plan {
  int kernel;  // kMfmaW4 | kT128 | -1
  int splitk;
  double cost = 0.0;  // plan_cost (us) of the choice
};
static Plan plan(const Problem& p, int kernel);

// The kernel of the whole-problem plan (resolve_kernel without relabelling a
// refined wave-quantisation tail; tail_plan asks this one).
static int resolve_core(const Problem& p, int kernel) {
  if (is_experiment(kernel) && !experiments_built()) return -1;
  const GemmArgs a = shape_args(p);
  if (p.dtype == kFP8) {  // fp8 kernels only; no generic / padded fallback
    if (!(kernel == kAuto || is_fp8_kernel(kernel)) ||
        !gemm_fp8_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C))
      return -1;
    const bool s_fits = gemm_fp8_w4s_fits(a) && device_cus() % 8 == 0;
    if (kernel == kFp8W4S) return s_fits ? kernel : -1;
    if (kernel == kFp8T128 || kernel == kFp8T256x128 || kernel == kFp8T192 || kernel == kFp8T192x128)
      return supports(p, kernel) ? kernel : -1;
    if (is_experiment(kernel)) return experiment_resolve_fp8(p, kernel, s_fits);
    if (kernel != kAuto) return kernel;
    // the streaming kernel on a device of its own with more than one wave of
    // tiles (bf16's W4S waits for 2 per CU; fp8 measured ahead of W4 from 1.3
    // per CU: 5120^2 x 4096 2592 vs 2546, 4608^2 x 3072 1977 vs 1960 TFLOPS, and
    // behind at exactly one, 4096^3 2700 vs 2797; profiles/r4x_fp8_tail_dp_w4_vs_w4s_ab.jsonl)
    const long long T = (long long)(p.M / 256) * (p.N / 256) * (p.batch < 1 ? 1 : p.batch);
    if (s_fits && p.cus == 0 && T >= 2LL * device_cus()) return kFp8W4S;
    // otherwise the planner: fp8 W4 (edge tiles too) or the fp8 tile family
    const Plan pl = plan(p, kAuto);
    if (pl.kernel == kFp8W4 && pl.splitk <= 1 && s_fits && p.cus == 0 && T > device_cus()) return kFp8W4S;
    return pl.kernel >= 0 ? pl.kernel : kFp8W4;
  }
  if (is_fp8_kernel(kernel)) return -1;
  const bool fast = gemm256_supported(p.dtype, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool w4 = gemm_w4_supported(p.dtype, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool t128 = gemm_tile_supported(p.dtype, 128, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool t256 = gemm_tile_supported(p.dtype, 256, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool t192 = gemm_tile_supported(p.dtype, 192, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool f32fast = p.dtype == kF32 &&
                       gemm_f32_256_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  switch (kernel) {
    // Auto: the 4-wave kernel where the tiles are whole (M, N % 256; +4.5 %
    // over SCHED 3 at 16k, profiles/r1_s4_w4_ab.jsonl), SCHED 3 for edge tiles.
    // Auto: the whole-tile kernels where the tiles are whole (W4 for grids
    // that fill the chip, T128 for under-filled ones: plan()), SCHED 3 for
    // edge tiles.
    case kAuto:
      if (w4 || t128 || t256 || t192) {
        const Plan pl = plan(p, kAuto);
        return pl.kernel == kMfmaW4 && pl.splitk == 1 && w4s_auto(p) ? kMfmaW4S : pl.kernel;
      }
      // fp32: the planner over the exact-fp32 family — f32_t128x2 (two
      // 128x128 workgroups per CU) on grids with >= 2 tiles per CU, f32_256s
      // (8 waves, 256x256), f32_w4 (256x256, split-K) and f32_t128 (128x128,
      // split-K) for grids that under-fill the chip.
      if (fast) return kMfma256d;
      if (!f32fast) return kGeneric;
      {
        const Plan pl = plan(p, kAuto);
        // Whole waves of 256x256 tiles (round 6): the lean W4 K-loop (f32_w4l,
        // 98.3 % MFMA busy, profiles/r8lq_fp32_lean_stream.md) in place of
        // the plan below (f32_t128x2, or f32_256s on one long-K wave).
        if (f32w4l_whole_waves(p, a, pl)) return kF32W4L;
        // Exactly one wave of 256x256 tiles on a long K: the 8-wave f32_256s
        // measured 1.0-1.3 % ahead of f32_t128x2 (1024 x 16384 x 16384 152.1
        // vs 150.1, 4096^2 x 14336 152.3 vs 150.8; profiles/r6f_f32_long_k_arms_ab.jsonl)
        if (pl.kernel == kF32T128x2 && pl.splitk <= 1 && p.cus == 0 && p.K >= 8192 &&
            (long long)(p.M / 256) * (p.N / 256) * (p.batch < 1 ? 1 : p.batch) == device_cus() &&
            p.M % 256 == 0 && p.N % 256 == 0)
          return kF32_256s;
        return pl.kernel >= 0 ? pl.kernel : kF32_256s;
      }
    case kGeneric: return kGeneric;
    case kMfma256d: return fast ? kMfma256d : -1;
    case kMfmaW4: return w4 ? kMfmaW4 : -1;
    case kMfmaW4S: return w4 && w4s_fits(p) ? kMfmaW4S : -1;
    case kT128: return t128 ? kT128 : -1;
    case kT128x2: return t128 ? kT128x2 : -1;  // shares T128's constraints
    case kT256x128: return t256 ? kT256x128 : -1;
    case kT192: return t192 ? kT192 : -1;
    case kT192x128: return t192 ? kT192x128 : -1;
    case kF32_256s: return f32fast ? kF32_256s : -1;
    case kF32W4: return f32fast ? kF32W4 : -1;  // same constraints as f32_256
    case kF32W4L: return f32fast && gemm_f32_w4l_fits(a) && p.splitk <= 1 ? kF32W4L : -1;  // unsplit only
    case kF32T128: return p.dtype == kF32 && supports(p, kF32T128) ? kF32T128 : -1;
    case kF32T128x2: return p.dtype == kF32 && supports(p, kF32T128) ? kF32T128x2 : -1;
    case kF32T64: return p.dtype == kF32 && supports(p, kF32T64) ? kF32T64 : -1;
    case kF32T64x2: return p.dtype == kF32 && supports(p, kF32T64) ? kF32T64x2 : -1;
    default:
      return is_experiment(kernel) ? experiment_resolve(p, kernel, fast, w4, t128, f32fast) : -1;
  }
}

// ---- tile size and split-K (W4 / tile family) ------------------------------
// A grid of T output tiles fills the 256 CUs (1 workgroup / CU) only if T is
// a multiple of 256: the matrix_parallel column shards for the reference's
// default sizes (matmul_scaling_benchmark.py:179-188, :351) have T = 32 / 128
// 256x256 tiles (4k / 8k at ws = 8; 4k at ws = 2 too). Two levers: smaller
// tiles (gemm_tile.hip: T256x128 = 2x, T128 = 4x the workgroups; T128x2 runs
// two of them per CU) and splitting K over S workgroups per tile. The planner
// prices every (kernel, S) in microseconds and takes the cheapest (W4 unless
// another is >= 3 % cheaper):
//   waves = ceil(units / (CUs the stream may use x workgroups per CU))
//   t     = waves * (ceil(nk / S) * kt * boost(busy) + kFixedUs) + meet
//   boost = 0.62 + 0.38 * busy: a K-tile runs faster while part of the chip
//           idles (power headroom: W4's K-tile is 1.16 us at 128 workgroups,
//           1.42 us at 256+)
//   meet  = split-K combine, chip-bandwidth bound: every slice but one
//           writes and the last reads back an fp32 tile slab,
//           T * (S-1) * 2 * BM * BN * 4 B / kSlabBw + kMeetUs.
// kt per K-tile at full occupancy (us, random bf16, profiles/r2_*sweep*.jsonl):
// W4 1.42, T256x128 0.80 (0.80-0.85 on the 2-13-wave grids it competes on,
// profiles/r2_planner_fit.jsonl; 0.87 at 16k, where the chip is power-bound and
// W4 wins anyway), T128 0.46, T128x2 0.86 per pair of co-resident workgroups.
// The fit reproduces the measured times of the shard shapes within ~10 %.
//
// fp8 (one K-tile = 128 e4m3: the same bytes per row and MFMA cycles as a
// bf16 K-tile of 64) is planned over its own models: fp8 W4 (edge tiles too;
// its split stays fp8_split's measured rule) and the fp8 tile family.
//
// Exact fp32 (K-tile = 32; fp32 MFMA is not power-bound — f32_256s runs 95 %
// MFMA busy at 2.38 GHz, profiles/r1_fp32_ablation.md — so no idle-CU boost):
// f32_256s 7.1 us per 256x256 K-tile (150-152 TF at 16k), f32_w4 7.1, f32_t128
// 1.81 per 128x128 K-tile (fit to 4096 x {1024, 2048} x 4096: 237 / 471 us,
// profiles/r3_f32_t128_ab.jsonl), f32_t128x2 3.53 per pair of co-resident
// 128x128 workgroups (4096 x 2048 x 4096 458 us, 8192^3 7241 us:
// profiles/r3_f32_t128x2_ab.jsonl), priced only where it has two workgroups
// on every CU. f32_t128x2 is listed first — the incumbent the 3 % hysteresis
// keeps: on full grids it measured ahead of f32_256s in the same process
// (4096^3 149.7 vs 148.4, 8192^3 151.9 vs 149.5, 16384^3 152.0 vs 150.0 TF;
// profiles/r3i_f32_256p_ab.jsonl; f32_256s 7.05-7.16 us per 256x256 K-tile
// across boxes). The other tiles are listed before f32_w4: they measured
// ahead of the split W4 on every under-filled shard shape (4096 x 2048 x 4096
// 145.8 vs 141.6 TF).
struct KernelModel {
  int kernel, bm, bn, occ;
  double kt;
  int cls;   // 0: bf16 / fp16, 1: fp8, 2: fp32
  int maxS;  // largest split-K (1: the kernel does not split)
  double kt2 = 0.0;  // per K-tile on grids of two or more waves (0: kt)
};
static constexpr KernelModel kModels[] = {
    {kMfmaW4, 256, 256, 1, 1.42, 0, 8},
    {kT256x128, 256, 128, 1, 0.80, 0, 8},
    {kT128, 128, 128, 1, 0.46, 0, 8},
    {kT128x2, 128, 128, 2, 0.86, 0, 8},
    {kFp8W4, 256, 256, 1, 1.30, 1, 4},
    {kFp8T256x128, 256, 128, 1, 0.80, 1, 8},
    {kFp8T128, 128, 128, 1, 0.42, 1, 8},
    {kF32T128x2, 128, 128, 2, 3.53, 2, 8},
    {kF32_256s, 256, 256, 1, 7.1, 2, 1},
    {kF32T128, 128, 128, 1, 1.81, 2, 8},
    {kF32W4, 256, 256, 1, 7.1, 2, 8},
    // round 5: 192-row tiles (first estimated from the T256x128 rate per MFMA,
    // 72 / 48 MFMAs per wave per K-tile against its 64; calibrated on the first
    // A/B, profiles/r7e_t192_ab_*.jsonl: bf16 3072^3 46 us = 48 K-tiles x 0.87
    // + 4, 6144^3 340 us = 4 waves x (96 x 0.84 + 4); fp8 3072^3 23.9 us = 24 x
    // 0.83 + 4; T192x128 2304^2 x 4096 40.9 us = 64 x 0.61 x boost + 4).
    // Listed last: the incumbents keep ties. T192x128 runs slower per K-tile
    // past one wave (profiles/r7j_t192_ab_bf16.jsonl: 1024 x 9216 x 16384 332 us
    // over 2 waves, 2560 x 4608 x 16384 341 us, 2304 x 8192 x 16384 530 us over
    // 3 waves: 0.65-0.67 per K-tile, where it lost 7-8 % to W4 on the first two).
    {kT192, 192, 192, 1, 0.86, 0, 8},
    {kT192x128, 192, 128, 1, 0.60, 0, 8, 0.67},
    {kFp8T192, 192, 192, 1, 0.83, 1, 8},
    {kFp8T192x128, 192, 128, 1, 0.60, 1, 8, 0.67},
    // round 5: the exact-fp32 64x128 tile for shard grids that a 128x128 tile
    // fills only by splitting K (4096 x 512 x 4096: 128 tiles x 2 slices; 256
    // 64x128 tiles run unsplit). 0.92 us per K-tile (half a T128 K-tile's
    // MFMAs at 2 % below its rate: one barrier per 2048 MFMA cycles instead of
    // 4096), fit to 4096 x {512, 1024} x 4096 and 2048 x 1024 x 2048
    // (profiles/r7p_f32_t64_ab.jsonl: 140.6 vs 139.0 TF for f32_t128 x 2 at
    // 4096 x 512 x 4096, 136.2 vs 127.7 at 2048 x 1024 x 2048).
    {kF32T64, 64, 128, 1, 0.92, 2, 8},
    // round 5: f32_t64 on 2 stages, two workgroups per CU: 1.80 us per K-tile
    // of a co-resident pair, 0.95 alone (split slices priced per CU on any
    // grid, f32x2_split_grid); its split arms fit within 0.9-1.3x
    // (profiles/r7ao_f32_t64x2_arms.jsonl). Auto vs PDMB_F32T64X2=0 on 21 small
    // grids it changes: median +6.1 %, -0.5 to +37 % (r7ap_f32_t64x2_auto_ab.jsonl).
    {kF32T64x2, 64, 128, 2, 1.80, 2, 8},
};
static int dt_class(const Problem& p) { return p.dtype == kFP8 ? 1 : p.dtype == kF32 ? 2 : 0; }
static constexpr double kFixedUs = 4.0;   // launch + prologue + epilogue
static constexpr double kMeetUs = 4.0;    // combine latency (poll, serial slab read)
static constexpr double kSlabBw = 4.0e6;  // bytes per us of slab traffic, chip-wide
static constexpr int kMinKt = 4;          // K-tiles per slice, at least

static const KernelModel& model_of(int kernel) {
  for (const KernelModel& m : kModels)
    if (m.kernel == kernel) return m;
  return kModels[0];
}

static long long tiles_of(const Problem& p, int kernel) {  // ceil: fp8 W4 runs edge tiles
  const KernelModel& m = model_of(kernel);
  return (long long)((p.M + m.bm - 1) / m.bm) * ((p.N + m.bn - 1) / m.bn) * (p.batch < 1 ? 1 : p.batch);
}

static int ktiles(const Problem& p) { return p.K / (p.dtype == kFP8 ? 128 : p.dtype == kF32 ? 32 : 64); }

static int device_cus() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!n[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    n[dev] = v;
  }
  return n[dev];
}

// W4S (gemm_w4.hip): an even number (>= 6) of K-tiles and a grid of whole
// 8-XCD rounds. Auto picks it over W4 for >= 2 tiles per CU on a device the
// GEMM has to itself (p.cus == 0): its tiles are assigned statically, so a CU
// held by a concurrent kernel (an RCCL collective of an overlap schedule:
// gemm.shared_device, Problem::cus < 0) would hold back a whole tile
// sequence; there, and on CU-masked streams, the dispatch-balanced W4 runs.
// Measured (profiles/r2_w4s_ab.jsonl): +3.1 % at 16384^2 x 2048, +2.8 % at
// K = 4096, +2.2 % on the 16384 x 2048 x 16384 ws=8 shard, +0.1 % at 16k.
static bool w4s_fits(const Problem& p) {  // interior tiles only (its epilogue is unmasked)
  const int nk = p.K / 64;
  return (p.dtype == kBF16 || p.dtype == kF16) && p.M % 256 == 0 && p.N % 256 == 0 && nk % 2 == 0 &&
         nk >= 6 && device_cus() % 8 == 0;
}
static bool w4s_auto(const Problem& p) {
  return p.cus == 0 && w4s_fits(p) && tiles_of(p, kMfmaW4) >= 2LL * device_cus();
}

// f32_w4l on whole waves of 256x256 tiles, K >= 4096, on a device of its own,
// in place of an unsplit f32_t128x2 / f32_256s plan. Settled, two sessions,
// TFLOPS:
//  * one wave (profiles/r8y/, against the old plan): 4096^3 151.8 vs 150.6,
//    8192 x 2048 x 8192 152.2 vs 151.2, 4096^2 x 16384 152.9 vs 151.8,
//    1024 x 16384^2 152.9 vs 152.0, 2048 x 8192^2 151.9 vs 151.2, 4096^2 x
//    8192 152.4 vs 151.2;
//  * more waves (profiles/r8za/, against f32_t128x2): 8192^3 152.3 vs 151.6,
//    16384^3 152.8 vs 151.9, 16384 x {8192, 4096, 2048} x 16384 152.7 / 152.6 /
//    152.4 vs 151.9 / 151.8 / 151.2, 8192 x 4096 x 8192 151.9 vs 151.0, 12288^3
//    152.2 vs 151.9, 8192^2 x 4096 150.9 vs 151.0, 4096^3 x 2 151.1 vs 150.3.
// +0.5 % median (-0.07 to +0.8 %; r8r measured +2.2 / +2.3 % on two one-wave
// grids against a slower f32_256s arm). That is under the 1 % bar VERDICT r5
// set for planner rules; this one is taken as a kernel replacement, not a
// fitted threshold: bitwise-equal output, fewer instructions per K-tile, no
// grid losing beyond noise. Short K loses (16384^2 x 1024: -1.4 %, r8r), hence
// K >= 4096; partial waves keep f32_t128x2's tail plans.
static bool f32w4l_whole_waves(const Problem& p, const GemmArgs& a, const Plan& pl) {
  if (p.cus != 0 || p.dtype != kF32 || pl.splitk > 1 || (pl.kernel != kF32T128x2 && pl.kernel != kF32_256s))
    return false;
  if (p.M % 256 || p.N % 256 || p.K < 4096 || !gemm_f32_w4l_fits(a)) return false;
  const long long T = (long long)(p.M / 256) * (p.N / 256) * (p.batch < 1 ? 1 : p.batch);
  return T > 0 && T % device_cus() == 0;
}

// f32_t128x2 split into slices on a grid of fewer than two tiles per CU
// (plan_uncached takes it there from 3 slices per CU: PDMB_F32X2SPLIT=0 turns
// that off, A/B, read per call).
static bool t64x2_full_on() {  // PDMB_F32T64X2_FULL=0: f32_t64x2 only on the small grids (A/B)
  return !ab_off("PDMB_F32T64X2_FULL");
}
static constexpr double kF32X2AloneKt = 1.9;
static bool f32x2_split_on() { return !ab_off("PDMB_F32X2SPLIT"); }
static bool f32x2_split_grid(const Problem& p, const KernelModel& m, int S, long long T) {
  if (m.kernel == kF32T64x2) return S > 1;  // any grid (its plans date from this model)
  return m.kernel == kF32T128x2 && S > 1 && T < 2LL * (p.cus > 0 ? p.cus : device_cus()) && f32x2_split_on();
}

static bool split3_small_on() { return !ab_off("PDMB_SPLIT3_SMALL"); }
static constexpr double kSlotLatUs = 4.5;
static bool split_slot_lat_on() { return !ab_off("PDMB_SPLIT_SLOT_LAT"); }

// Model time (us) of `kernel` over T of the problem's tiles (T < 0: all of
// them), each split S ways along K.
static double plan_cost_tiles(const Problem& p, int kernel, int S, long long T) {
  const KernelModel& m = model_of(kernel);
  if (T < 0) T = tiles_of(p, kernel);
  const int nk = ktiles(p);
  const int per = (nk + S - 1) / S;
  const long long slots = (long long)(p.cus > 0 ? p.cus : device_cus()) * m.occ;
  const long long units = T * S;
  const long long waves = (units + slots - 1) / slots;
  const double busy = (double)units / (double)(waves * slots);
  const double boost = m.cls == 2 ? 1.0 : 0.62 + 0.38 * busy;  // power headroom (not fp32)
  const double kt = waves > 1 && m.kt2 > 0 ? m.kt2 : m.kt;
  double t = (double)waves * (per * kt * boost + kFixedUs);
  if (f32x2_split_grid(p, m, S, T)) {
    // Split slices of a grid with fewer tiles than two per CU (round 5): the
    // hardware hands each CU its next slice as one finishes, so a CU runs
    // n = ceil(units / CUs) slices, in pairs at the co-resident rate and the
    // odd one alone (kF32X2AloneKt; alone it measured 1.84-1.85 us per
    // K-tile) — not whole two-per-CU waves. It still overprices the split arms
    // the rule admits by 3-30 % (profiles/r7ad_f32_small_split_arms.jsonl: a
    // slice's meet overlaps its co-resident slice's loop, the slab term does
    // not know), so auto takes them only where they are clearly cheaper.
    const long long cus = p.cus > 0 ? p.cus : device_cus();
    const long long n = (units + cus - 1) / cus;
    const double alone = m.kernel == kF32T64x2 ? kF32X2AloneKt / 2.0 : kF32X2AloneKt;
    t = (double)(n / 2) * (per * kt + kFixedUs) + (double)(n % 2) * (per * alone + kFixedUs);
  }
  if (S > 1) t += (double)T * (S - 1) * 2.0 * m.bm * m.bn * 4.0 / kSlabBw + kMeetUs;
  // bf16 / fp16 / fp8 grids of <= 64 tiles split >= 4 ways into slices of <=
  // 32 K-tiles (round 5): the slab term, sized for the chip's bandwidth, misses
  // the reducer's latency there — every slot past the second costs ~4.5 us
  // (forced arms, profiles/r7ai_bf16_small_arms.jsonl: T128 x 4 ran 6.8-9.5 us
  // over the model on 1024^2 x 8192, 512 x 2048 x 8192, 768^2 x 8192, where
  // x 3 ran 14-17 % faster). Auto vs the term off on 13 grids of 4-64 tiles
  // it changes, settled arms, two sessions: +1 to +20 %, median +4.5 %, bf16 and
  // fp16 alike (profiles/r7aj_*_split_slot_latency_ab.jsonl); fp8, 16 grids it
  // moves off T128 x 4, with the x 3 rule below: all gain, +7 to +40 %
  // (r7am_fp8_small_rules_ab.jsonl).
  // PDMB_SPLIT_SLOT_LAT=0 leaves it out (A/B).
  if (S >= 4 && m.cls != 2 && T <= 64 && per <= 32 && split_slot_lat_on()) t += (S - 2) * kSlotLatUs;
  return t;
}

static double plan_cost(const Problem& p, int kernel, int S) { return plan_cost_tiles(p, kernel, S, -1); }

static bool split_ok(const Problem& p, int kernel, int S) {
  if (kernel == kFp8W4) return S == fp8_split(p);  // its measured rule (fp8_split)
  if (S == 1) return true;
  if (S > model_of(kernel).maxS) return false;
  const int nk = ktiles(p);
  const int per = (nk + S - 1) / S;
  const int min_kt = p.dtype == kF32 ? 8 : kMinKt;  // fp32 K-tiles are 32 deep
  return per >= min_kt && (S - 1) * per < nk && tiles_of(p, kernel) <= kMaxSplitTiles;
}

static bool supports(const Problem& p, int kernel) {
  const GemmArgs a = shape_args(p);
  if (kernel == kMfmaW4) return gemm_w4_supported(p.dtype, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  if (kernel == kFp8W4) return gemm_fp8_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  if (kernel == kF32_256s || kernel == kF32W4)
    return p.dtype == kF32 && gemm_f32_256_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  if (kernel == kF32T128 || kernel == kF32T128x2 || kernel == kF32T64 || kernel == kF32T64x2)
    return p.dtype == kF32 && gemm_f32_tile_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  return gemm_tile_supported(p.dtype, model_of(kernel).bm, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
}

// `kernel`: kAuto (choose), or one of kMfmaW4 / kT256x128 / kT128 / kT128x2
// (choose only the split). p.splitk > 0 fixes the split.
static bool is_t192(int k) { return k == kT192 || k == kT192x128 || k == kFp8T192 || k == kFp8T192x128; }

// ---- planner memo -------------------------------------------------------------
// plan() and tail_plan() are pure functions of the problem's shape and layout,
// the CU budget, the requested kernel and (experiments build only) the A/B
// switches in the environment.
// One GEMM call asks them several times (resolve, split, workspace size,
// launch, and tail_plan's own sub-plans): ~8 us of host time per call at
// 1024^3 on the GPU box's host (profiles/r7w_host_overhead.jsonl). Per-thread
// memo keyed by exactly those inputs; in a PDMB_EXPERIMENTS=1 build the
// environment enters as a hash of every PDMB_* variable (one pass over
// environ), so a switch flipped between calls (scripts/ab_kernels.py arms)
// takes effect at once; the shipping build hashes nothing.
extern "C" char** environ;
static uint64_t pdmb_env_hash() {
#ifndef PDMB_EXPERIMENTS
  return 0;  // the shipping planner reads no environment (ab_switch)
#else
  uint64_t h = 1469598103934665603ull;
  for (char** e = environ; e && *e; ++e) {
    const char* v = *e;
    if (v[0] != 'P' || strncmp(v, "PDMB_", 5) != 0) continue;
    for (; *v; ++v) h = (h ^ (unsigned char)*v) * 1099511628211ull;
    h = (h ^ 0xffu) * 1099511628211ull;
  }
  return h;
#endif
}
struct MemoKey {
  int what, kernel, dtype, M, N, K, lda, ldb, ldc, batch, splitk, cus, kb, sig, dev_cus;
  unsigned align;
  long long sA, sB, sC;
  uint64_t env;
};
static MemoKey memo_key(int what, const Problem& p, int kernel) {
  MemoKey k;
  memset(&k, 0, sizeof(k));  // padding compares equal (memcmp)
  k.what = what;
  k.kernel = kernel;
  k.dtype = p.dtype;
  k.M = p.M;
  k.N = p.N;
  k.K = p.K;
  k.lda = p.lda;
  k.ldb = p.ldb;
  k.ldc = p.ldc;
  k.batch = p.batch;
  k.splitk = p.splitk;
  k.cus = p.cus;
  k.kb = p.kb;
  k.sig = p.sig != nullptr;
  k.dev_cus = device_cus();
  k.align = (unsigned)((uintptr_t)p.A & 255) | ((unsigned)((uintptr_t)p.B & 255) << 8) |
            ((unsigned)((uintptr_t)p.C & 255) << 16);
  k.sA = p.sA;
  k.sB = p.sB;
  k.sC = p.sC;
  k.env = pdmb_env_hash();
  return k;
}
struct MemoKeyHash {
  size_t operator()(const MemoKey& k) const {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(&k);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(k); ++i) h = (h ^ b[i]) * 1099511628211ull;
    return (size_t)h;
  }
};
struct MemoKeyEq {
  bool operator()(const MemoKey& a, const MemoKey& b) const { return memcmp(&a, &b, sizeof(a)) == 0; }
};
template <class V>
using Memo = std::unordered_map<MemoKey, V, MemoKeyHash, MemoKeyEq>;
constexpr size_t kMemoMax = 4096;  // entries per thread and kind; cleared when full

static Plan plan_uncached(const Problem& p, int kernel);
static Plan plan(const Problem& p, int kernel) {
  thread_local Memo<Plan> memo;
  const MemoKey k = memo_key(0, p, kernel);
  auto it = memo.find(k);
  if (it != memo.end()) return it->second;
  if (memo.size() >= kMemoMax) memo.clear();
  const Plan r = plan_uncached(p, kernel);
  memo.emplace(k, r);
  return r;
}

// kAuto without f32_t64x2 on the full grids: the baseline f32_tail_plan
// weighs its split tail against (the tails were measured against those plans).
constexpr int kAutoNoT64x2Full = -7;

static Plan plan_uncached(const Problem& p, int kernel) {
  const bool no_t64x2_full = kernel == kAutoNoT64x2Full;
  if (no_t64x2_full) kernel = kAuto;
  // The launch re-plans the split of the kernel auto resolved to with that
  // kernel fixed (tiled_launch). Auto takes f32_t128x2 on a grid of fewer than
  // two tiles per CU only split >= 3 slices per CU (below), a rule the fixed
  // plan does not apply (an explicit request runs it on any grid): there the
  // fixed plan is auto's own.
  // (f32_t64x2: on every grid — auto takes it only split on the full grids.)
  if (((kernel == kF32T128x2 && f32x2_split_on() && tiles_of(p, kernel) < 2LL * (p.cus > 0 ? p.cus : device_cus())) ||
       kernel == kF32T64x2) &&
      p.splitk == 0 && p.dtype == kF32) {
    const Plan a = plan(p, kAuto);
    if (a.kernel == kernel) return a;
  }
  Plan best{-1, 1};
  double bc = 1e300;
  bool any = false;
  // Pass 0 prices the power-of-two splits; pass 1 the 3- (5-, 6-) way
  // splits, whose cheapest plan then replaces the best of pass 0 only by a
  // clear win (the plans of every grid it does not win stay as they were).
  Plan alt{-1, 1};
  double ac = 1e300;
  static const int kS0[] = {1, 2, 4, 8}, kS1[] = {3, 5, 6};
  // PDMB_SPLIT3=0 (read per call; A/B): auto leaves the 3-way split out
  const bool no3 = ab_off("PDMB_SPLIT3");
  // PDMB_T192=0 (read per call; A/B): auto leaves the 192-row tiles out
  const bool no192 = kernel == kAuto && ab_off("PDMB_T192");
  // PDMB_F32T64=0 (read per call; A/B): auto leaves the 64x128 fp32 tile out
  const bool no64 = kernel == kAuto && ab_off("PDMB_F32T64");
  // PDMB_F32T64X2=0 (read per call; A/B): auto leaves f32_t64x2 out
  const bool t64x2_on = !ab_off("PDMB_F32T64X2");
  for (int pass = 0; pass < 2; ++pass)
  for (const KernelModel& m : kModels) {
    if (kernel != kAuto && kernel != m.kernel) continue;
    if (no192 && is_t192(m.kernel)) continue;
    if (no64 && m.kernel == kF32T64) continue;
    // f32_t64x2 in auto only where the 128x128 tiles number fewer than two per
    // CU (the full grids keep their measured f32_t128x2 / tail plans)
    const bool full_grid = tiles_of(p, kF32T128x2) >= 2LL * (p.cus > 0 ? p.cus : device_cus());
    if (kernel == kAuto && m.kernel == kF32T64x2 && (!t64x2_on || (full_grid && (no_t64x2_full || !t64x2_full_on()))))
      continue;
    if (m.cls != dt_class(p) || !supports(p, m.kernel)) continue;
    any = true;
    const int* Ss = pass ? kS1 : kS0;
    const int nS = pass ? 3 : 4;
    for (int si = 0; si < nS; ++si) {
      const int S = Ss[si];
      // 5- / 6-way (round 5): exact fp32 only — its K-tiles carry 4x the MFMA
      // time of bf16's, so the longer meet pays: fp32 1024 x 256 x 16384 92.8
      // vs 68.2 TF, 512 x 6400 x 16384 136.4 vs 115.8, all six grids tried
      // ahead; on bf16 two of six lost (2560 x 256 x 16384 515 vs 543;
      // profiles/r7u_split56_ab_*.jsonl). PDMB_SPLIT56=0 leaves them out (A/B).
      // 8-way (round 5), the same rule, on the exact-fp32 64x128 tile only:
      // 1024 x 256 x 16384 113.5 vs 95.2 TF at 6 ways, 256 x 512 x 16384 58.8
      // vs 48.2, 1024 x 256 x 8192 91.4 vs 81.2; on the 128x128 tiles it lost
      // (512 x 1024 x 16384 f32_t128 x 8 123.3 vs 131.9 for f32_t64 x 4, 512 x
      // 9216 x 16384 f32_t128x2 x 8 137.6 vs 142.3 at 6 ways;
      // profiles/r7ae_f32_split8_x2split_ab.jsonl, confirmed with settled arms
      // on 5 more f32_t64 grids: +1.5 to +20 %, r7af_f32_planner_confirm_settled.jsonl).
      // PDMB_SPLIT8=0 leaves it out.
      if ((S == 5 || S == 6 || (S == 8 && m.kernel == kF32T64)) && p.splitk != S) {
        if (ab_off(S == 8 ? "PDMB_SPLIT8" : "PDMB_SPLIT56") || m.cls != 2 || (ktiles(p) + S - 1) / S < 32 || m.kernel == kF32W4)
          continue;
      } else if (S > 4 && p.splitk != S) {
        continue;
      }
      // The 3-way split (round 5; profiles/r7r_split3_ab_*.jsonl): 256 / 3
      // slices fill a wave that 2 or 4 leave a quarter empty or over-full
      // (bf16 2560 x 4096 x 16384 1238 vs 1091 TF, fp32 2560 x 256 x 8192 119.5
      // vs 84.3). Auto takes it only with >= 32 K-tiles per slice — its
      // reducer reads two slots per row with no row-ahead prefetch (S == 2 has
      // one): bf16 1024^2 x 4096 (22 K-tiles per slice) ran 25.5 us vs 21.9 at
      // S = 2 — and not on the 256^2 fp32 tile (fp32 2560 x 2048 x 4096 on
      // f32_w4 129.0 vs 132.4 for f32_t128 x 4).
      // (The T128 / 4-stage fp32 reducers now prefetch both other slots at
      // S = 3, splitk_load_others3: +7 % on bf16 2560 x 512 x 8192, but with
      // 22 K-tiles per slice S = 3 still lost to S = 2 on two of three bf16
      // grids, profiles/r7z_split3_prefetch_ab_*.jsonl — the 32 stays.)
      // ... except on grids of <= 36 128^2 tiles, where T128 x 3
      // (whose reducer prefetches both other slots) measured ahead of x 2 with
      // 11-22 K-tiles per slice: 768^2 x 4096 249.4 vs 234.6 TF, 512 x 1024 x
      // 4096 231.4 vs 215.2, 384 x 768 x 4096 132.6 vs 122.1
      // (profiles/r7aj_*_split_slot_latency_ab.jsonl forced arms; at 64 tiles
      // it was mixed, r7ai). Auto vs the rule off on 16 grids it changes, bf16
      // and fp16, settled arms, two sessions: all 32 gain, +0.9 to +13.7 %,
      // median +7.5 % (r7ak_*_split3_small_ab.jsonl). PDMB_SPLIT3_SMALL=0
      // leaves it out (A/B).
      // fp8 T128 (round 5, the same A/B, r7am_fp8_small_rules_ab.jsonl) from 16
      // K-tiles per slice: with 11 it lost (1024 x 256 x 4096 159.4 vs 172.3
      // unsplit); with 22, +4 to +8 % over x 2 on five grids.
      const bool s3small = (m.kernel == kT128 || m.kernel == kFp8T128) && tiles_of(p, m.kernel) <= 36 &&
                           (ktiles(p) + 2) / 3 >= (m.kernel == kFp8T128 ? 16 : 8) && split3_small_on();
      if (S == 3 && p.splitk != 3 &&
          (no3 || ((ktiles(p) + 2) / 3 < 32 && !s3small) || m.kernel == kF32W4))
        continue;
      // f32_t64x2 on the full fp32 grids (round 5): split only — unsplit it lost
      // (3072 x 3584 x 4096 130.1 vs 144.4 TF for f32_t128x2 x 3), split 2 ways it
      // gained on the grids without a split tail (4608^2 x 4096 143.2 vs 127.2,
      // 5120 x 2560 x 8192 143.6 vs 130.4; profiles/r7as_f32_t64x2_full_ab.jsonl).
      // Grids with an fp32 split tail keep it (f32_tail_plan's baseline leaves
      // these plans out: on them t64x2 x 2 measured -1.7 to +0.9 %). The rule as
      // built, auto vs PDMB_F32T64X2_FULL=0 on 16 of the 31 non-tail grids of a
      // 784-grid scan it changes: -2.3 to +19.4 %, median +2.3 %
      // (r7at_f32_t64x2_full_rule_ab.jsonl; the two losses are 3072 x 3584 x
      // 4096 and its transpose, where f32_t128x2 x 3 stays 2 % ahead).
      if (kernel == kAuto && m.kernel == kF32T64x2 && full_grid && S < 2) continue;
      if (p.splitk > 0 && S != p.splitk) continue;
      if (!split_ok(p, m.kernel, S)) continue;
      // auto takes a two-per-CU fp32 tile only on grids whose tiles (not split
      // slices) put two on every CU: alone on a CU its 2-stage ring runs slower
      // than the 4-stage one-per-CU tile, and split into pairs it lost to the
      // 4-stage tile on 4096 x 1024 x 4096 and 2048^3 (142.3 / 138.3 vs 146.5 /
      // 143.8 TF, profiles/r3_f32_t128x2_ab.jsonl). An explicit request runs it
      // on any grid.
      // Round 5: split into >= 3 slices per CU it does run there — a CU's
      // co-resident slices hide each other's prologue, epilogue and meet:
      // 2560 x 2048 x 4096 303.6 us as f32_t128x2 x 4 vs 324.0 for f32_t128 x 4
      // (profiles/r7ad_f32_small_split_arms.jsonl); auto vs PDMB_F32X2SPLIT=0 on
      // 20 grids it changes, settled arms, two sessions: -0.5 to +19 %, median
      // +3.3 % (r7af_f32_planner_confirm_settled.jsonl; priced per CU, see
      // f32x2_split_grid; the launch's re-plan with the kernel fixed returns
      // this plan, see the top). PDMB_F32X2SPLIT=0 leaves it out (A/B).
      if (kernel == kAuto && m.cls == 2 && m.occ > 1 &&
          tiles_of(p, m.kernel) < (long long)(p.cus > 0 ? p.cus : device_cus()) * m.occ &&
          !(f32x2_split_on() && S > 1 &&
            tiles_of(p, m.kernel) * S >= 3LL * (p.cus > 0 ? p.cus : device_cus())))
        continue;
      // f32_t64 only within one wave: past it, it measured 3-4 % behind
      // f32_t128 / f32_t128x2 (2048^3 138.0 vs 143.4, 8192 x 512 x 8192 143.6
      // vs 148.0; profiles/r7p_f32_t64_ab.jsonl), and the fp32 tail plan
      // (f32_tail_plan) prices the multi-wave grids against f32_t128x2.
      if (kernel == kAuto && m.kernel == kF32T64 &&
          tiles_of(p, m.kernel) > (long long)(p.cus > 0 ? p.cus : device_cus()))
        continue;
      const double c = plan_cost(p, m.kernel, S);
      if (pass) {  // the cheapest non-power-of-two plan, compared with pass 0's below
        if (c < ac) {
          ac = c;
          alt = Plan{m.kernel, S, c};
        }
      } else if (c < bc * 0.97) {  // a different choice only for a clear win
        bc = c;
        best = Plan{m.kernel, S, c};
      }
    }
  }
  if (alt.kernel >= 0 && ac < bc * 0.97) best = alt;
  // f32_t64x2 on a full grid is the newcomer there, so it never wins on the
  // hysteresis alone: the best plan without it (the 3-way split included)
  // keeps the grid unless f32_t64x2 is priced strictly cheaper. Round 5 took
  // 3072 x 3584 x 4096 (and its transpose) from f32_t128x2 x 3 (model 671 us)
  // to f32_t64x2 x 2 (687 us) because pass 1 needs a 3 % win, and measured
  // 141.6 vs 144.7 TF (profiles/r7at_f32_t64x2_full_rule_table.txt); the 14
  // grids it gained on are priced cheaper with it and keep it.
  if (kernel == kAuto && !no_t64x2_full && best.kernel == kF32T64x2 && p.splitk == 0 &&
      tiles_of(p, kF32T128x2) >= 2LL * (p.cus > 0 ? p.cus : device_cus())) {
    const Plan base = plan(p, kAutoNoT64x2Full);
    if (base.kernel >= 0 && base.cost <= best.cost) best = base;
  }
  if (best.kernel < 0 && any)  // the requested split is impossible for this K
    for (const KernelModel& m : kModels)
      if ((kernel == kAuto || kernel == m.kernel) && m.cls == dt_class(p) && supports(p, m.kernel))
        return Plan{m.kernel, 0};
  return best;
}

static bool is_tiled(int k) {
  return k == kMfmaW4 || k == kT128 || k == kT128x2 || k == kT256x128 || k == kFp8T128 || k == kFp8T256x128 ||
         k == kF32W4 || k == kF32T128 || k == kF32T128x2 || k == kT192 || k == kT192x128 || k == kFp8T192 ||
         k == kFp8T192x128 || k == kF32T64 || k == kF32T64x2;
}

int choose_splitk(const Problem& p, int kernel) {
  const int k = resolve_kernel(p, kernel);
  if (k == kMfmaW4S || k == kFp8W4S || k == kF32W4L) return 1;
  if (k == kFp8W4) return fp8_split(p);
  if (!is_tiled(k)) return 0;
  return plan(p, k).splitk;
}

// ---- wave-quantisation tail (bf16/fp16 W4, fp8 W4) -----------------------------
// A grid of 256x256 tiles whose last wave is mostly empty (6000^2 x 6144: 576
// tiles = 2.25 waves of 256 CUs) runs as two launches on the stream: the first
// M1 rows (a multiple of 256, tile rows that fill whole waves) unsplit, then
// the remaining tile rows as one split-K wave (splitk.h) that fills the chip
// instead of a quarter of it. Priced with plan_cost against the best
// single-launch plan; taken only for a >= 3 % win. Measured (ms, auto before
// -> tail, hipBLASLt; profiles/r2_tail_split_probe.jsonl): 6000^2 x 6144
// 0.375 -> 0.342 (0.362), 6144^3 0.365 -> 0.339 (0.373), 3000 x 7000 x 5056
// 0.203 -> 0.187 (0.193), 10000^2 x 10048 1.518 -> 1.457 (1.684); 5000^2 x 5056
// has no split that helps and stays one launch. The tail rows keep their
// fixed slice order, so results stay bitwise reproducible run to run.
// fp8: the same plan on fp8 W4 (the first launch fp8 W4S where it has >= 2
// tiles per CU; the tail split by fp8_split's measured rule). Probe (us, one
// launch -> tail, hipBLASLt; profiles/r2_fp8_tail_probe.jsonl): 6144^3 196.9
// -> 175.2 (187.6), 6000^2 x 6144 183.9 -> 177.4 (191.0), 7168^3 278.2 ->
// 269.1 (314.9).
//
// The tile-range form (GemmArgs::tile_end / tile_base / tile_span): the first
// launch covers the first whole waves of map_tile's tile order (tiles_dp =
// k x CUs tiles, W4S or W4, fp8 W4S or W4) and the second the remaining
// tiles, each split S ways, as one wave. Rows cannot always cut the grid at a
// wave boundary (6144^3: 24 x 24 tiles, no row count gives 256 or 512 tiles);
// tiles always can. Priced like the row form, taken when it is the cheaper of
// the two; PDMB_TILE_TAIL=0 disables it, =S forces S (A/B, read per call).
//
// Refined tail (round 4): the remaining (< one wave of) tiles are not split
// along K but cut into the tile family's smaller tiles — 256x128 halves or
// 128x128 quarters (gemm_tile.hip, tile_span over W4's tile order), each
// running the whole K unsplit: no fp32 slabs to write and combine, which for
// fp8 (half a bf16 tile's compute per output byte) costs as much as the
// compute it saves. Priced by the same model; PDMB_TAIL_REFINE=0 disables,
// =2 / =4 forces halves / quarters (A/B, read per call).
//
// Decision order (tail_plan): a refined tail that beats the best single
// launch — a W4 launch, or a tile-family one (bf16 6144 x 4096 x 4096 ran as
// three waves of 256x128 tiles) — is taken outright; otherwise, against a W4
// launch only, the tile-range split-K form and then the row form; the fp8
// stream-K form only when PDMB_STREAMK forces it (measured slower everywhere,
// profiles/r4o_fp8_stream_k_modes_ab.jsonl). The whole-wave launch streams
// (W4S / fp8 W4S) only from two tiles per CU. Exact fp32 has its own split
// form (f32_tail_plan below).
struct TailPlan {
  int m1 = 0;        // rows of the first (unsplit) launch; 0 = one launch (row form)
  int S = 1;         // K slices of the tail launch
  int tiles_dp = 0;  // tile-range form: tiles of the first launch (> 0), rest split S ways
  int sub = 0;       // refined tail: the tile-family kernel of the second launch (S == 1)
  bool sk = false;   // stream-K (fp8): tiles [tiles_dp, T) as even K-tile shares, S slots per tile
  int f32k = 0;      // exact fp32: the split tail's kernel (kF32T128 / kF32T128x2; 128x128 tiles)
  bool active() const { return m1 > 0 || tiles_dp > 0 || sk; }
};

// Exact fp32 (f32_t128x2, two 128x128 workgroups per CU: a wave is 2 x CUs
// tiles): the whole waves as one launch, the remaining tiles split S ways as
// one wave of f32_t128 (one workgroup per CU). Measured (TFLOPS, no tail ->
// tail, hipBLASLt; profiles/r5f_f32_tail_ab.jsonl): 5120^3 137.6 -> 148.1
// (143.3), 3072^3 125.8 -> 141.4 (136.2), 5120^2 x 2048 128.3 -> 144.2
// (132.0), 7168^3 146.2 -> 149.6 (144.9), 9216^3 145.3 -> 150.4 (142.0). Priced against
// the last partial wave as it runs unsplit — lightly loaded CUs, about one
// f32_t128 tile time (plan() prices it as a full two-per-CU wave).
// PDMB_TILE_TAIL=0 disables it (A/B).
static TailPlan f32_tail_plan(const Problem& p) {
  TailPlan best;
  if (ab_off("PDMB_TILE_TAIL")) return best;
  if (!supports(p, kF32T128) || !supports(p, kF32T128x2)) return best;
  const Plan whole = plan(p, kAutoNoT64x2Full);  // the best single launch (possibly split: 5120^3 ran f32_t128 x 2)
  if (whole.kernel != kF32T128x2 && whole.kernel != kF32T128) return best;
  const long long cus = device_cus(), slots2 = 2 * cus;
  const long long T = tiles_of(p, kF32T128x2);
  const long long dp = T / slots2 * slots2, rest = T - dp;
  if (dp == 0 || rest == 0 || rest > cus || rest > kMaxSplitTiles) return best;
  const int nk = ktiles(p);
  const double c1 = plan_cost_tiles(p, kF32T128x2, 1, dp);
  double base = whole.cost;
  if (whole.kernel == kF32T128x2 && whole.splitk <= 1)  // its light last wave
    base = std::min(base, c1 + plan_cost_tiles(p, kF32T128, 1, rest));
  double bc = base * 0.97;
  // the tail on f32_t128 only: a split f32_t128x2 tail (4352^3: 132 tiles x 2)
  // measured 3 % slower than no tail (profiles/r5f_f32_tail_ab.jsonl)
  for (int k : {kF32T128}) {
    const long long slots = cus * model_of(k).occ;
    for (int S : {2, 4, 8}) {
      const int per = (nk + S - 1) / S;
      if (rest * S > slots || per < 8 || (S - 1) * per >= nk) continue;
      const double c = c1 + plan_cost_tiles(p, k, S, rest);
      if (c < bc) {
        bc = c;
        best = TailPlan{};
        best.tiles_dp = (int)dp;
        best.S = S;
        best.f32k = k;
      }
    }
  }
  return best;
}

static int sub_parts(int kernel) { return kernel == kT128 || kernel == kFp8T128 ? 4 : 2; }

static int tail_kernel(const Problem& p) {
  return p.dtype == kFP8 ? kFp8W4 : p.dtype == kF32 ? kF32T128x2 : kMfmaW4;
}

static TailPlan tail_plan_uncached(const Problem& p, int kernel);
static TailPlan tail_plan(const Problem& p, int kernel) {
  thread_local Memo<TailPlan> memo;
  const MemoKey k = memo_key(1, p, kernel);
  auto it = memo.find(k);
  if (it != memo.end()) return it->second;
  if (memo.size() >= kMemoMax) memo.clear();
  const TailPlan r = tail_plan_uncached(p, kernel);
  memo.emplace(k, r);
  return r;
}

static TailPlan tail_plan_uncached(const Problem& p, int kernel) {
  TailPlan best;
  if (kernel != kAuto || p.splitk != 0 || p.cus > 0 || p.sig) return best;
  if (p.dtype == kF32 && p.K > 0) return f32_tail_plan(p);
  if ((p.dtype != kBF16 && p.dtype != kF16 && p.dtype != kFP8) || p.M <= 256 || p.K <= 0) return best;
  const int kw = tail_kernel(p);
  if (resolve_core(p, kAuto) < 0 || !supports(p, kw)) return best;
  const Plan whole = plan(p, kAuto);  // the best single launch (W4 or a smaller tile)
  // A refined tail can also beat a single launch of the tile family (bf16
  // 6144 x 4096 x 4096: 768 256x128 tiles = 3 waves, vs one W4 wave + one wave
  // of 256x128 halves); the split-K forms only ever replace a single W4 launch.
  const bool whole_w4 = whole.kernel == kw && whole.splitk == 1;
  const bool whole_tile = whole.splitk <= 1 && (whole.kernel == kT256x128 || whole.kernel == kT128 ||
                                                whole.kernel == kFp8T256x128 || whole.kernel == kFp8T128 ||
                                                whole.kernel == kT192 || whole.kernel == kT192x128 ||
                                                whole.kernel == kFp8T192 || whole.kernel == kFp8T192x128);
  if (!whole_w4 && !whole_tile) return best;
  const long long slots = device_cus();
  const int tm = (p.M + 255) / 256, tn = (p.N + 255) / 256, batch = p.batch < 1 ? 1 : p.batch;
  double bc = whole.cost * 0.97;
  {  // tile-range form: whole waves, then the rest split S ways
    // PDMB_TILE_TAIL (read per call, A/B): 0 = off; 2 / 4 / 8 = only that S, priced
    // as if free (forced wherever the form is feasible)
    int force = ab_switch("PDMB_TILE_TAIL");
    if (force != 0 && force != 2 && force != 4 && force != 8) force = -1;
    const long long T = (long long)tm * tn * batch;
    const int nk = ktiles(p);
    const int rforce = ab_switch("PDMB_TAIL_REFINE");
    const bool fp8 = p.dtype == kFP8;
    for (long long dp = slots; dp < T && force != 0; dp += slots) {
      const long long rest = T - dp;
      const double c1 = plan_cost_tiles(p, kw, 1, dp);
      if (rest < slots && rforce != 0 && force <= 0) {  // refined: the last partial wave in smaller tiles
        for (int ks : {fp8 ? kFp8T256x128 : kT256x128, fp8 ? kFp8T128 : kT128}) {
          const int R = sub_parts(ks);
          if (rforce > 0 && R != rforce) continue;
          if (!supports(p, ks)) continue;
          const double c = rforce > 0 ? -1.0 : c1 + plan_cost_tiles(p, ks, 1, rest * R);
          if (c < bc) {
            bc = c;
            best = TailPlan{};
            best.tiles_dp = (int)dp;
            best.sub = ks;
          }
        }
      }
      if (rforce > 0 || best.sub || !whole_w4) continue;  // a refined tail that pays beats the split-K forms
      for (int S : {2, 4, 8}) {
        const int per = (nk + S - 1) / S;
        if (rest * S > slots || per < 8 || (S - 1) * per >= nk || rest > kMaxSplitTiles) continue;
        if (force > 0 && S != force) continue;
        const double c = force > 0 ? -1.0 : c1 + plan_cost_tiles(p, kw, S, rest);
        if (c < bc) {
          bc = c;
          best = TailPlan{};
          best.tiles_dp = (int)dp;
          best.S = S;
        }
      }
    }
  }
  // Stream-K (fp8, gemm_fp8_sk; PDMB_STREAMK=1 / 2 force it, read per call — A/B
  // until priced): the last 1-2 waves' tiles as G even shares of K-tiles.
  if (p.dtype == kFP8) {
    const int mode = ab_switch("PDMB_STREAMK");
    if ((mode == 1 || mode == 2) && device_cus() % 8 == 0) {
      const long long T = (long long)tm * tn * batch;
      const int nk = ktiles(p);
      const long long G = slots;
      // 1: whole waves before the last 1-2 waves, those stream-K; 2: only the
      // last partial wave stream-K (the whole waves run in lockstep first)
      long long dp = T > 2 * G ? (T / G - 1) * G : 0;
      if (T - dp >= 2 * G) dp += G;
      if (mode == 2) dp = T / G * G;
      const long long rest = T - dp;
      if (rest >= 8 && rest / 8 * nk >= G / 8 && rest <= kMaxSplitTiles) {
        const int smax = fp8_sk_slots(rest, nk, G);
        if (smax >= 2 && smax <= 8) {
          TailPlan k;
          k.tiles_dp = (int)dp;
          k.S = smax;
          k.sk = true;
          return k;
        }
      }
    }
  }
  // A refined tail that beats the single launch is taken over every split-K
  // form, whatever their model price: in every same-process A/B so far it ran
  // at least as fast (bf16 7168^3: 1474 vs 1429 TFLOPS for the S = 8 tile-range
  // split the model preferred; fp8 6144^3 2976 vs 2608;
  // profiles/r4k_*_refined_tail_ab.jsonl) — the model under-prices the split's
  // slab traffic and short slices.
  if (best.sub || !whole_w4) return best;
  for (int r = 1; r < tm; ++r) {  // r tail tile rows
    Problem a = p, b = p;
    a.M = (tm - r) * 256;
    b.M = p.M - a.M;
    const double c1 = plan_cost(a, kw, 1);
    for (int S : {2, 4}) {
      if ((long long)r * tn * batch * S > slots || !split_ok(b, kw, S)) continue;
      const double c = c1 + plan_cost(b, kw, S);
      if (c < bc) {
        bc = c;
        best = TailPlan{};
        best.m1 = a.M;
        best.S = S;
      }
    }
  }
  return best;
}

static Problem tail_part(const Problem& p, const TailPlan& t) {  // rows [m1, M), split S ways
  const size_t esa = p.dtype == kFP8 ? 1 : 2, esc = 2;  // fp8: e4m3 A, bf16 C
  Problem b = p;
  b.M = p.M - t.m1;
  b.A = (const char*)p.A + (size_t)t.m1 * p.lda * esa;
  b.C = (char*)p.C + (size_t)t.m1 * p.ldc * esc;
  b.splitk = t.S;
  return b;
}

PlanInfo plan_info(const Problem& p, int kernel) {
  PlanInfo r{};
  r.kernel = resolve_kernel(p, kernel);
  r.splitk = r.kernel >= 0 ? choose_splitk(p, kernel) : 0;
  if (is_tiled(r.kernel) || r.kernel == kF32_256s || r.kernel == kFp8W4) {
    const int S = r.splitk > 0 ? r.splitk : 1;
    r.cost_us = plan_cost(p, r.kernel, S);
  }
  const TailPlan t = tail_plan(p, kernel);
  r.tail_m1 = t.m1;
  r.tail_S = t.S;
  r.tail_tiles_dp = t.tiles_dp;
  r.tail_sub = t.sk ? 0 : t.sub ? sub_parts(t.sub) : 1;
  return r;
}

TailSplit tail_split(const Problem& p, int kernel) {
  const TailPlan t = tail_plan(p, kernel);
  return {t.m1, t.S, t.tiles_dp, t.sk ? 0 : t.sub ? sub_parts(t.sub) : 1};
}

// fp8 W4 split-K (gemm_fp8.hip): grids of 256x256 tiles that fill at most
// half the CUs are split 2 or 4 ways along K while every slice keeps >= 16
// K-tiles (128 deep) and the split grid still fits the CUs the stream may
// use; p.splitk > 0 fixes it (1 = never). Measured (profiles/
// r2_fp8_splitk_ab.jsonl): 8192x1024x8192 S=2 2237 vs 1844 TF unsplit;
// slices of 8 K-tiles lose (4096x1024x4096 S=4 787 vs 878; 2048^3 S=2 563
// vs 694): the meet's slot traffic and latency outweigh the extra CUs.
static int fp8_split(const Problem& p) {
  if (p.splitk > 0) return p.splitk;
  const long long T = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256) * (p.batch < 1 ? 1 : p.batch);
  const int nk = p.K / 128;
  const long long cus = p.cus > 0 ? p.cus : device_cus();
  int S = 1;
  for (int s : {2, 4})
    if (T * s <= cus && nk / s >= 16 && T <= kMaxSplitTiles) S = s;
  return S;
}
static size_t fp8_split_bytes(const Problem& p, int S) {
  if (S <= 1) return 0;
  const long long T = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256) * (p.batch < 1 ? 1 : p.batch);
  return (size_t)T * S * 256 * 256 * sizeof(float);
}

static size_t splitk_bytes(const Problem& p, int kernel, int S) {
  if (S <= 1) return 0;
  const KernelModel& m = model_of(kernel);
  return (size_t)tiles_of(p, m.kernel) * S * m.bm * m.bn * sizeof(float);  // one slot per slice
}

// Per-(device, stream) counters, zeroed once on the stream before first use,
// never freed (~32 KiB each): split-K (2 per tile, kMaxSplitTiles tiles),
// then the persistent kernels' work queues (kQueueWords). Every launch leaves
// them zero again, so launches on one stream can share them.
//
// A stream being captured gets a counter set of its own per capture (taken
// from a per-device pool of kCapturePool zeroed sets, allocated by the first
// uncaptured call on that device — hipMalloc is not capturable): each graph
// bakes its own counters into its split-K / queue nodes, so two graphs
// captured on one stream may replay concurrently on different streams, and
// beside eager launches on the capture stream. (One graph replayed on two
// streams at once still shares its set; once the pool is used up, captures
// fall back to the capture stream's own set, the serial-replay contract.)
// Returns nullptr when no set is available (no pool and no stream set yet):
// the caller then runs unsplit, or refuses an explicitly requested split.
static constexpr int kQueueWords = 16;  // 8 XCD ticket counters + exit counter (+ pad)
static constexpr int kCapturePool = 64;
static constexpr size_t kCounterBytes = sizeof(unsigned) * (2 * kMaxSplitTiles + kQueueWords);

struct CounterPool {
  unsigned* base = nullptr;
  int used = 0;
};

static unsigned* stream_counters(hipStream_t s) {
  static std::mutex mu;
  static std::unordered_map<unsigned long long, unsigned*>* map =
      new std::unordered_map<unsigned long long, unsigned*>();  // leaked on purpose
  static std::unordered_map<unsigned long long, unsigned*>* captures =
      new std::unordered_map<unsigned long long, unsigned*>();  // (device, capture id) -> set
  static CounterPool pools[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (hipStreamGetCaptureInfo(s, &st, &cid) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  CounterPool& pool = pools[dev];
  if (st != hipStreamCaptureStatusNone) {
    if (st != hipStreamCaptureStatusActive) return nullptr;
    const unsigned long long key = (cid << 8) ^ (unsigned)dev;
    auto it = captures->find(key);
    if (it != captures->end()) return it->second;
    unsigned* c = nullptr;
    if (pool.base && pool.used < kCapturePool) {
      c = pool.base + (size_t)pool.used++ * (kCounterBytes / sizeof(unsigned));
    } else {  // pool used up: the stream's own set (graphs on it then replay serially)
      auto own = map->find(((unsigned long long)(uintptr_t)s << 8) ^ (unsigned)dev);
      if (own == map->end()) return nullptr;
      c = own->second;
    }
    (*captures)[key] = c;
    return c;
  }
  if (!pool.base) {  // zeroed on this stream: ordered before any capture that could use it
    unsigned* b = nullptr;
    if (hipMalloc(&b, kCounterBytes * kCapturePool) == hipSuccess) {
      if (hipMemsetAsync(b, 0, kCounterBytes * kCapturePool, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess)
        pool.base = b;
      else
        (void)hipFree(b);
    }
  }
  const unsigned long long key = ((unsigned long long)(uintptr_t)s << 8) ^ (unsigned)dev;
  auto it = map->find(key);
  if (it != map->end()) return it->second;
  unsigned* c = nullptr;
  if (hipMalloc(&c, kCounterBytes) != hipSuccess) return nullptr;
  if (hipMemsetAsync(c, 0, kCounterBytes, s) != hipSuccess) {
    (void)hipFree(c);
    return nullptr;
  }
  (*map)[key] = c;
  return c;
}

// Launch W4 or a tile-family kernel (k, already resolved) with its planned split.
static hipError_t tiled_launch(const Problem& p, int k, GemmArgs a, void* part, size_t part_bytes,
                               hipStream_t stream, int sub = 0) {
  int S = plan(p, k).splitk;
  if (S < 1) return hipErrorInvalidValue;  // requested split not possible for this K
  if (S > 1) {
    unsigned* flags = stream_counters(stream);
    if (!flags || part_bytes < splitk_bytes(p, k, S) || !part) {
      if (p.splitk > 1) return hipErrorInvalidValue;  // explicitly requested: no silent change
      S = 1;
    } else {
      a.part = (float*)part;
      a.flags = flags;
    }
  }
  a.splitk = S;
  if ((sub >= 7 && sub <= 11) || (sub >= 13 && sub <= 21) || sub == 23 || sub == 24) {  // W4S (13-16: power diag, 17-21, 24: tile order, 23: lean), unsplit, one
                                                              // workgroup per usable CU (a multiple of 8)
    if (S > 1) {
      sub = 0;
    } else {
      a.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
    }
  }
  if (sub == 5 || sub == 6) {  // persistent W4: unsplit, needs the stream's queue
    unsigned* c = S > 1 ? nullptr : stream_counters(stream);
    if (!c) {
      sub = sub == 6 ? 4 : 0;
    } else {
      a.queue = c + 2 * kMaxSplitTiles;
      a.pers_grid = p.cus > 0 ? p.cus : device_cus();
    }
  }
  if (k == kF32W4) return gemm_f32_w4_launch(a, stream, sub);  // sub: the variant (experiments)
  if (k == kF32T128 || k == kF32T128x2 || k == kF32T64 || k == kF32T64x2) return gemm_f32_tile_launch(a, stream, sub);  // sub: the variant
  return k == kMfmaW4 ? gemm_w4_launch(p.dtype, a, stream, sub) : gemm_tile_launch(k, p.dtype, a, stream);
}

// ---- padded fast path -------------------------------------------------------
// A large problem that misses the LDS-DMA kernels only because K / N are off
// their granule (bf16/fp16: K%64, N%8; fp32: K%32, N%4) or because a leading
// dimension / base is misaligned is copied into zero-padded, aligned
// workspace operands and run on the fast kernel (exact: the padding only adds
// zero products). The copies are O(MK + KN + MN) against O(MNK) of MFMA work.
// The workspace is the caller's (Problem::workspace, sized by
// gemm_workspace_bytes), so concurrent streams and graph captures never share
// or reallocate it.
static constexpr double kPadMinFlops = 2147483648.0;  // 2^31

static int pad_k(int dt) { return dt == kF32 ? 32 : 64; }
static int pad_n(int dt) { return dt == kF32 ? 4 : 8; }
static long long round_up(long long x, long long m) { return (x + m - 1) / m * m; }

// dst[r][c] = (r < rows && c < cols) ? src[r][c] : 0 for r < drows, c < dcols.
// dst rows are 16-B aligned (ldd % VEC == 0); each thread writes one 16-B
// vector. Its VEC source elements come as one 16-B or two 8-B loads when the
// source base and row pitch allow (src_align, uniform over the grid: K = 6100
// bf16 rows are 8-B aligned), else as scalar loads, which coalesce across the
// wave. One pass, no memset.
template <typename T>
__global__ void pad_copy(const T* __restrict__ src, long long lds, int rows, int cols,
                         T* __restrict__ dst, long long ldd, int drows, int dcols, int src_align) {
  constexpr int VEC = 16 / sizeof(T);
  union Vec {
    uint4 u;
    uint2 h[2];
    T e[VEC];
  };
  const int vpr = dcols / VEC;  // vectors per dst row (dcols % VEC == 0)
  const long long total = (long long)drows * vpr;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / vpr), c0 = (int)(i % vpr) * VEC;
    const T* s = src + r * lds + c0;
    Vec v;
    if (src_align >= 8 && r < rows && c0 + VEC <= cols) {
      if (src_align >= 16) {
        v.u = *(const uint4*)s;
      } else {
        v.h[0] = ((const uint2*)s)[0];
        v.h[1] = ((const uint2*)s)[1];
      }
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v.e[e] = (r < rows && c0 + e < cols) ? s[e] : (T)0;
    }
    *(uint4*)(dst + r * ldd + c0) = v.u;
  }
}

// dst[r][c] = src[r][c] for r < rows, c < cols (unpad the result; dst arbitrary).
template <typename T>
__global__ void unpad_copy(const T* __restrict__ src, long long lds, int rows, int cols,
                           T* __restrict__ dst, long long ldd) {
  const long long total = (long long)rows * cols;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    dst[r * ldd + c] = src[r * lds + c];
  }
}

template <typename T>
static hipError_t pad_copy_launch(const void* src, long long lds, int rows, int cols, void* dst,
                                  long long ldd, int drows, int dcols, hipStream_t s) {
  const uintptr_t pitch = (uintptr_t)lds * sizeof(T), base = (uintptr_t)src;
  const int align = (base | pitch) % 16 == 0 ? 16 : (base | pitch) % 8 == 0 ? 8 : 1;
  hipLaunchKernelGGL(pad_copy<T>, dim3(4096), dim3(256), 0, s, (const T*)src, lds, rows, cols,
                     (T*)dst, ldd, drows, dcols, align);
  return hipGetLastError();
}

template <typename T>
static hipError_t unpad_copy_launch(const void* src, long long lds, int rows, int cols, void* dst,
                                    long long ldd, hipStream_t s) {
  hipLaunchKernelGGL(unpad_copy<T>, dim3(4096), dim3(256), 0, s, (const T*)src, lds, rows, cols,
                     (T*)dst, ldd);
  return hipGetLastError();
}

static bool wants_padding(const Problem& p, int kernel) {
  if (p.dtype == kFP8 || p.sig) return false;
  if (kernel != kAuto || p.M <= 0 || p.N <= 0 || p.K <= 0) return false;
  const double flops = 2.0 * p.M * (double)p.N * p.K * (p.batch < 1 ? 1 : p.batch);
  if (flops < kPadMinFlops) return false;
  return resolve_kernel(p, kAuto) == kGeneric;
}

// The zero-padded problem `gemm_padded` runs (operands in the workspace).
// direct_c: only K is padded (N already on its granule) and the caller's C is
// aligned, so the kernel writes C in place — no padded C, no unpad copy
// (for 8192^2 x 1000 bf16 that copy moved 256 MB).
// direct_b: N is on its granule and B's base, row pitch and batch stride meet
// the fast kernels' 16-B alignment, so B is read in place: its rows past K
// read as zeros through the DMA descriptors' extent (Problem::kb = K), and
// only A is copied with zero columns K .. Kp (6000^2 x 6100 bf16: 293 MB of
// copy traffic down to 147 MB). A's own columns past K cannot be left to the
// next row's data: a non-finite value there would turn a 0-weighted product
// into NaN.
struct Padded {
  Problem q;
  size_t a_bytes, b_bytes, c_bytes, a_el, b_el, c_el;
  bool direct_c, direct_b;
};

static Padded padded_problem(const Problem& p, char* w) {
  Padded d{};
  const size_t es = p.dtype == kF32 ? 4 : 2;
  const int batch = p.batch < 1 ? 1 : p.batch;
  const long long Kp = round_up(p.K, pad_k(p.dtype)), Np = round_up(p.N, pad_n(p.dtype));
  d.a_el = (size_t)p.M * Kp;
  d.b_el = (size_t)Kp * Np;
  d.c_el = (size_t)p.M * Np;
  d.direct_c = Np == p.N && (uintptr_t)p.C % 16 == 0 && p.ldc % 8 == 0 && p.ldc >= p.N &&
               (batch == 1 || p.sC % 8 == 0);
  const int vec = (int)(16 / es);  // elements per 16 B
  d.direct_b = Np == p.N && (uintptr_t)p.B % 16 == 0 && p.ldb % vec == 0 && p.ldb >= p.N &&
               (batch == 1 || p.sB % vec == 0 || p.sB == 0);
  d.a_bytes = round_up(d.a_el * es * batch, 256);
  d.b_bytes = d.direct_b ? 0 : round_up(d.b_el * es * batch, 256);
  d.c_bytes = d.direct_c ? 0 : round_up(d.c_el * es * batch, 256);
  Problem& q = d.q;
  q = p;
  q.A = w;
  q.B = w ? w + d.a_bytes : nullptr;
  q.C = w ? w + d.a_bytes + d.b_bytes : nullptr;
  if (!w) {  // sizing only: any 256-B aligned stand-in passes the alignment checks
    q.A = q.B = q.C = (void*)(uintptr_t)256;
  }
  q.K = (int)Kp;
  q.N = (int)Np;
  q.lda = (int)Kp;
  q.ldb = (int)Np;
  q.ldc = (int)Np;
  q.sA = (long long)d.a_el;
  q.sB = (long long)d.b_el;
  q.sC = (long long)d.c_el;
  if (d.direct_c) {
    q.C = p.C;
    q.ldc = p.ldc;
    q.sC = p.sC;
  }
  if (d.direct_b) {
    q.B = p.B;
    q.ldb = p.ldb;
    q.sB = p.sB;
    q.kb = p.K;
  }
  q.batch = batch;
  q.workspace = nullptr;
  q.workspace_bytes = 0;
  return d;
}

int resolve_padded(const Problem& p) {
  if (!wants_padding(p, kAuto)) return -1;
  return resolve_kernel(padded_problem(p, nullptr).q, kAuto);
}

// ---- batched streaming GEMMs: one launch per element -------------------------
// A batched problem that auto runs on W4S / fp8 W4S, with every element alone
// >= 2 tiles per CU, runs as one launch per element on the stream, each
// element planned alone (its wave tail included), all on one workspace
// (stream-ordered). Measured in one process (profiles/r3_batch_seq_ab.jsonl):
// bmm of 4 16k bf16 as one launch 1444 TF, as four launches 1515 TF.
static bool batch_split(const Problem& p, int kernel) {
  if (kernel != kAuto || p.batch <= 1 || p.sig || p.splitk != 0) return false;
  Problem q = p;
  q.batch = 1;
  const int k = resolve_kernel(q, kAuto);
  return k == kMfmaW4S || k == kFp8W4S;
}

static Problem batch_elem(const Problem& p, int b) {
  const size_t esa = p.dtype == kFP8 ? 1 : p.dtype == kF32 ? 4 : 2;  // fp8: e4m3 A / B
  const size_t esc = p.dtype == kF32 ? 4 : 2;                         // fp8: bf16 C
  Problem q = p;
  q.batch = 1;
  q.A = (const char*)p.A + (size_t)b * p.sA * esa;
  q.B = (const char*)p.B + (size_t)b * p.sB * esa;
  q.C = (char*)p.C + (size_t)b * p.sC * esc;
  return q;
}

// Split-K slots of a tail plan's second launch.
static size_t tail_bytes(const Problem& p, const TailPlan& t) {
  if (t.sub) return 0;  // refined: unsplit
  if (t.f32k) return (size_t)(tiles_of(p, kF32T128x2) - t.tiles_dp) * t.S * 128 * 128 * sizeof(float);
  if (t.sk) return (size_t)(tiles_of(p, tail_kernel(p)) - t.tiles_dp) * t.S * 256 * 256 * sizeof(float);
  if (t.tiles_dp > 0) {
    const long long T = tiles_of(p, tail_kernel(p));
    return (size_t)(T - t.tiles_dp) * t.S * 256 * 256 * sizeof(float);
  }
  return splitk_bytes(tail_part(p, t), tail_kernel(p), t.S);
}

size_t gemm_workspace_bytes(const Problem& p, int kernel) {
  if (!wants_padding(p, kernel) && batch_split(p, kernel)) return gemm_workspace_bytes(batch_elem(p, 0), kAuto);
  if (p.sig) {
    const int k = signal_kernel(p, kernel);
    return k < 0 ? 0 : splitk_bytes(p, kMfmaW4, plan(p, kMfmaW4).splitk);
  }
  if (wants_padding(p, kernel)) {
    const Padded d = padded_problem(p, nullptr);
    const size_t copies = d.a_bytes + d.b_bytes + d.c_bytes;
    const int k = resolve_kernel(d.q, kAuto);
    const TailPlan t = tail_plan(d.q, kAuto);
    if (t.active()) return copies + tail_bytes(d.q, t);
    return copies + (is_tiled(k) ? splitk_bytes(d.q, k, plan(d.q, k).splitk) : 0);
  }
  const int k = resolve_kernel(p, kernel);
  const TailPlan t = tail_plan(p, kernel);
  if (t.active()) return tail_bytes(p, t);  // the first launch is unsplit
  if (is_tiled(k)) return splitk_bytes(p, k, plan(p, k).splitk);
  if (k == kFp8W4) return fp8_split_bytes(p, fp8_split(p));
  return is_experiment(k) ? experiment_workspace_bytes(p, k) : 0;
}

// fp8 whole-wave launch of a tail plan: W4S where it streams >= 2 tiles per CU
// (as bf16's rule), else W4. PDMB_TAIL_DP_W4S=1 (A/B, read per call) takes W4S
// wherever it fits, the round-3 rule.
static bool fp8_dp_streams(const GemmArgs& d, long long tiles_dp) {
  if (!gemm_fp8_w4s_fits(d) || device_cus() % 8 != 0) return false;
  if (ab_switch("PDMB_TAIL_DP_W4S") == 1) return true;
  return tiles_dp >= 2LL * device_cus();
}

// Which kernel `kernel` resolves to. Auto whose whole-problem plan is a
// 192-row tile launch but whose refined tail beats it (6144^3: four waves of
// 192x192 tiles vs two W4S waves + 256x128 halves) runs the tail: report its
// first, whole-wave launch, as for a W4 plan.
int resolve_kernel(const Problem& p, int kernel) {
  const int k = resolve_core(p, kernel);
  if (kernel != kAuto || !is_t192(k) || p.K <= 0) return k;
  const TailPlan t = tail_plan(p, kAuto);
  if (!t.active() || !t.sub) return k;
  if (p.dtype == kFP8) return fp8_dp_streams(shape_args(p), t.tiles_dp) ? kFp8W4S : kFp8W4;
  return w4s_fits(p) && t.tiles_dp >= 2LL * device_cus() ? kMfmaW4S : kMfmaW4;
}

// The two launches of a tail plan; false: run the problem as one launch (the
// stream has no split-K counters yet inside a graph capture, or the workspace
// was sized for another plan).
static bool gemm_tail(const Problem& p, const TailPlan& t, hipStream_t stream, hipError_t* e) {
  if (t.sub && t.tiles_dp > 0) {  // refined: whole waves, then the rest in the tile family's tiles
    const int G = (device_cus() / 8) * 8;
    GemmArgs d = to_args(p);
    d.splitk = 1;
    d.tile_end = t.tiles_dp;
    GemmArgs r = to_args(p);
    r.splitk = 1;
    r.tile_base = t.tiles_dp;
    r.tile_span = (int)(tiles_of(p, tail_kernel(p)) - t.tiles_dp);
    if (p.dtype == kFP8) {
      const bool s_fits = fp8_dp_streams(d, t.tiles_dp);
      if (s_fits) d.pers_grid = G;
      *e = gemm_fp8_launch(d, s_fits ? 2 : 1, stream);
    } else {
      const bool s = w4s_fits(p) && t.tiles_dp >= 2LL * device_cus();
      if (s) d.pers_grid = G;
      *e = gemm_w4_launch(p.dtype, d, stream, s ? 7 : 0);
    }
    if (*e == hipSuccess) *e = gemm_tile_launch(t.sub, p.dtype, r, stream);
    return true;
  }
  if (!p.workspace || p.workspace_bytes < tail_bytes(p, t) || !stream_counters(stream)) return false;
  if (t.f32k) {  // exact fp32: whole two-per-CU waves, then the rest split S ways as one wave
    GemmArgs d = to_args(p);
    d.splitk = 1;
    d.tile_end = t.tiles_dp;
    GemmArgs r = to_args(p);
    r.splitk = t.S;
    r.tile_base = t.tiles_dp;
    r.tile_span = (int)(tiles_of(p, kF32T128x2) - t.tiles_dp);
    r.part = (float*)p.workspace;
    r.flags = stream_counters(stream);
    *e = gemm_f32_tile_launch(d, stream, 2);
    if (*e == hipSuccess) *e = gemm_f32_tile_launch(r, stream, t.f32k == kF32T128x2 ? 2 : 0);
    return true;
  }
  if (t.sk) {  // fp8 stream-K: whole waves (if any), then the rest as G even K-tile shares
    const int G = (device_cus() / 8) * 8;
    *e = hipSuccess;
    if (t.tiles_dp > 0) {
      GemmArgs d = to_args(p);
      d.splitk = 1;
      d.tile_end = t.tiles_dp;
      const bool s_fits = fp8_dp_streams(d, t.tiles_dp);
      if (s_fits) d.pers_grid = G;
      *e = gemm_fp8_launch(d, s_fits ? 2 : 1, stream);
    }
    GemmArgs r = to_args(p);
    r.splitk = t.S;
    r.tile_base = t.tiles_dp;
    r.tile_span = (int)(tiles_of(p, tail_kernel(p)) - t.tiles_dp);
    r.part = (float*)p.workspace;
    r.flags = stream_counters(stream);
    r.pers_grid = G;
    if (*e == hipSuccess) *e = gemm_fp8_launch(r, 3, stream);
    return true;
  }
  if (t.tiles_dp > 0) {  // tile-range form (GemmArgs::tile_end / tile_span)
    const int G = (device_cus() / 8) * 8;
    GemmArgs d = to_args(p);
    d.splitk = 1;
    d.tile_end = t.tiles_dp;
    GemmArgs r = to_args(p);
    r.splitk = t.S;
    r.tile_base = t.tiles_dp;
    r.tile_span = (int)(tiles_of(p, tail_kernel(p)) - t.tiles_dp);
    r.part = (float*)p.workspace;
    r.flags = stream_counters(stream);
    if (p.dtype == kFP8) {
      const bool s_fits = fp8_dp_streams(d, t.tiles_dp);
      if (s_fits) d.pers_grid = G;
      *e = gemm_fp8_launch(d, s_fits ? 2 : 1, stream);
      if (*e == hipSuccess) *e = gemm_fp8_launch(r, 1, stream);
      return true;
    }
    // bf16 / fp16: W4S over the whole waves where it streams >= 2 tiles per CU
    const bool s = w4s_fits(p) && t.tiles_dp >= 2LL * device_cus();
    if (s) d.pers_grid = G;
    *e = gemm_w4_launch(p.dtype, d, stream, s ? 7 : 0);
    if (*e == hipSuccess) *e = gemm_w4_launch(p.dtype, r, stream, 0);
    return true;
  }
  const Problem b = tail_part(p, t);
  Problem a = p;
  a.M = t.m1;
  if (p.dtype == kFP8) {  // both launches through the fp8 cases of gemm()
    a.splitk = 1;
    a.workspace = nullptr;
    a.workspace_bytes = 0;
    *e = gemm(a, resolve_kernel(a, kAuto) == kFp8W4S ? kFp8W4S : kFp8W4, stream, nullptr);
    if (*e == hipSuccess) *e = gemm(b, kFp8W4, stream, nullptr);
    return true;
  }
  *e = tiled_launch(a, kMfmaW4, to_args(a), nullptr, 0, stream, w4s_auto(a) ? 7 : 0);
  if (*e == hipSuccess) *e = tiled_launch(b, kMfmaW4, to_args(b), p.workspace, p.workspace_bytes, stream);
  return true;
}

static hipError_t gemm_padded(const Problem& p, hipStream_t stream, int* used) {
  if (!p.workspace || p.workspace_bytes < gemm_workspace_bytes(p, kAuto)) return hipErrorInvalidValue;
  const size_t es = p.dtype == kF32 ? 4 : 2;
  const Padded d = padded_problem(p, (char*)p.workspace);
  const Problem& q = d.q;
  char* Ap = (char*)q.A;
  char* Bp = (char*)q.B;
  char* Cp = (char*)p.workspace + d.a_bytes + d.b_bytes;  // padded C (unless direct_c)
  const int batch = q.batch;
  const int Kp = q.K, Np = q.N;
  const bool f32 = p.dtype == kF32;
  hipError_t e;
  for (int b = 0; b < batch; ++b) {
    const char* A = (const char*)p.A + (size_t)b * p.sA * es;
    const char* B = (const char*)p.B + (size_t)b * p.sB * es;
    char* Ad = Ap + b * d.a_el * es;
    char* Bd = Bp + b * d.b_el * es;
    e = f32 ? pad_copy_launch<float>(A, p.lda, p.M, p.K, Ad, Kp, p.M, Kp, stream)
            : pad_copy_launch<unsigned short>(A, p.lda, p.M, p.K, Ad, Kp, p.M, Kp, stream);
    if (e != hipSuccess) return e;
    if (d.direct_b) continue;  // read in place (rows past K: zeros by extent)
    e = f32 ? pad_copy_launch<float>(B, p.ldb, p.K, p.N, Bd, Np, Kp, Np, stream)
            : pad_copy_launch<unsigned short>(B, p.ldb, p.K, p.N, Bd, Np, Kp, Np, stream);
    if (e != hipSuccess) return e;
  }
  const int k = resolve_kernel(q, kAuto);
  if (used) *used = k;
  if (k == kGeneric || k < 0) return hipErrorInvalidValue;  // cannot happen: q is aligned
  GemmArgs a = to_args(q);
  a.splitk = 0;  // only the tiled kernels below split here (their slots follow the copies)
  char* part = Cp + d.c_bytes;
  const size_t part_bytes = p.workspace_bytes - (d.a_bytes + d.b_bytes + d.c_bytes);
  const TailPlan t = tail_plan(q, kAuto);
  Problem qt = q;  // the tail plan's split slots follow the copies too
  qt.workspace = part;
  qt.workspace_bytes = part_bytes;
  if (!(t.active() && gemm_tail(qt, t, stream, &e)))
    e = k == kF32_256s ? gemm_f32_256_launch(a, 1, stream)
      : is_tiled(k) ? tiled_launch(q, k, a, part, part_bytes, stream)
                     : gemm256_launch(q.dtype, a, 4, stream);
  if (e != hipSuccess) return e;
  if (d.direct_c) return hipSuccess;  // the kernel wrote the caller's C
  for (int b = 0; b < batch; ++b) {
    char* C = (char*)p.C + (size_t)b * p.sC * es;
    const char* Cs = Cp + b * d.c_el * es;
    e = f32 ? unpad_copy_launch<float>(Cs, Np, p.M, p.N, C, p.ldc, stream)
            : unpad_copy_launch<unsigned short>(Cs, Np, p.M, p.N, C, p.ldc, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The kernel a signalled launch runs: W4 where `kernel` resolves to W4 or
// W4S (the persistent W4S leaves no CU to the consumers of the signals and
// drains its stores a tile late), otherwise -1.
static int signal_kernel(const Problem& p, int kernel) {
  Problem q = p;
  q.sig = nullptr;
  const int k = resolve_kernel(q, kernel);
  return (k == kMfmaW4 || k == kMfmaW4S) ? kMfmaW4 : -1;
}

int signal_granule(const Problem& p, int kernel) {
  if (signal_kernel(p, kernel) < 0 || p.K <= 0) return 0;
  const int tm = (p.M + 255) / 256, tn = (p.N + 255) / 256;
  switch (choose_supertile(tm, tn)) {  // rows of one 256-tile round of map_tile's order
    case 1: return 16;
    case 2: return 8;
    case 3: return 32;
    case 4: return 4;
    case 5: return 64;
    default: return 16 * ((256 + 16 * tn - 1) / (16 * tn));  // grouped: whole 16-row groups of a round
  }
}

static hipError_t gemm_signalled(const Problem& p, int kernel, hipStream_t stream, int* used) {
  const int k = signal_kernel(p, kernel);
  if (used) *used = k;
  if (k < 0 || p.dtype == kFP8) return hipErrorNotSupported;
  if (p.sig_rows <= 0 || p.sig_epoch == 0 || !p.sig->dev || !p.sig->host_dev) return hipErrorInvalidValue;
  const int tm = (p.M + 255) / 256;
  const int slots = (tm + p.sig_rows - 1) / p.sig_rows * (p.batch < 1 ? 1 : p.batch);
  if (slots > p.sig->slots) return hipErrorInvalidValue;
  if (p.M == 0 || p.N == 0 || p.batch == 0 || p.K == 0) return hipErrorInvalidValue;
  return tiled_launch(p, kMfmaW4, to_args(p), p.workspace, p.workspace_bytes, stream);
}

hipError_t gemm(const Problem& p, int kernel, hipStream_t stream, int* used) {
  if (p.sig) return gemm_signalled(p, kernel, stream, used);
  if (wants_padding(p, kernel)) return gemm_padded(p, stream, used);
  const int k = resolve_kernel(p, kernel);
  if (used) *used = k;
  if (k < 0) return hipErrorInvalidValue;
  if (p.M == 0 || p.N == 0 || p.batch == 0) return hipSuccess;
  if (p.K > 0 && batch_split(p, kernel)) {
    for (int b = 0; b < p.batch; ++b) {
      const hipError_t e = gemm(batch_elem(p, b), kAuto, stream, nullptr);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (p.K > 0) {
    const TailPlan t = tail_plan(p, kernel);
    hipError_t e = hipSuccess;
    if (t.active() && gemm_tail(p, t, stream, &e)) return e;
  }
  GemmArgs a = to_args(p);
  if (p.K == 0) {
    // C = 0 (empty reduction).
    const size_t esz = p.dtype == kF32 ? 4 : 2;
    for (int b = 0; b < a.batch; ++b) {
      char* c = (char*)p.C + (size_t)b * p.sC * esz;
      hipError_t e = hipMemset2DAsync(c, (size_t)p.ldc * esz, 0, (size_t)p.N * esz, p.M, stream);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // One launch of the whole problem: the whole-problem plan's kernel. (k may be
  // the renamed first launch of a refined tail, resolve_kernel; that tail form
  // needs no workspace and never declines, but if a tail did, the launch here
  // is the plan the planner priced, not the renamed kernel. ADVICE r5.)
  const int kw = resolve_core(p, kernel);
  switch (kw) {
    case kFp8W4: {
      GemmArgs s = a;
      s.splitk = 1;
      const int S = fp8_split(p);
      if (S > 1) {
        unsigned* flags = stream_counters(stream);
        if (flags && p.workspace && p.workspace_bytes >= fp8_split_bytes(p, S)) {
          s.splitk = S;
          s.part = (float*)p.workspace;
          s.flags = flags;
        } else if (p.splitk > 1) {
          return hipErrorInvalidValue;  // explicitly requested: no silent change
        }
      }
      return gemm_fp8_launch(s, 1, stream);
    }
    case kFp8W4S: {
      GemmArgs s = a;
      s.pers_grid = ((p.cus > 0 ? p.cus : device_cus()) / 8) * 8;
      return gemm_fp8_launch(s, 2, stream);
    }
    case kMfma256d: return gemm256_launch(p.dtype, a, 4, stream);
    case kMfmaW4:
    case kT128:
    case kT128x2:
    case kT256x128:
    case kFp8T128:
    case kFp8T256x128:
    case kT192:
    case kT192x128:
    case kFp8T192:
    case kFp8T192x128: return tiled_launch(p, kw, a, p.workspace, p.workspace_bytes, stream);
    case kMfmaW4S: return tiled_launch(p, kMfmaW4, a, p.workspace, p.workspace_bytes, stream, 7);
    case kF32_256s: return gemm_f32_256_launch(a, 1, stream);
    case kF32W4L: {
      GemmArgs s = a;
      s.splitk = 1;
      return gemm_f32_w4_launch(s, stream, 16);
    }
    case kF32W4:
    case kF32T128: return tiled_launch(p, kw, a, p.workspace, p.workspace_bytes, stream);
    case kF32T128x2: return tiled_launch(p, kw, a, p.workspace, p.workspace_bytes, stream, 2);
    case kF32T64: return tiled_launch(p, kw, a, p.workspace, p.workspace_bytes, stream, 3);
    case kF32T64x2: return tiled_launch(p, kw, a, p.workspace, p.workspace_bytes, stream, 4);
    default:
      if (is_experiment(kw)) return experiment_launch(p, kw, a, stream);
      return gemm_generic_launch(p.dtype, a, generic_vec_ok(p), stream);
  }
}

hipError_t bench_gemm(const Problem& p, int kernel, int iters, int warmup, bool use_graph,
                      hipStream_t stream, float* ms) {
  *ms = 0.f;
  hipError_t e;
  for (int i = 0; i < warmup; ++i)
    if ((e = gemm(p, kernel, stream, nullptr)) != hipSuccess) return e;
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
  if (use_graph && iters > 0) {
    // Capture on a private stream so the caller's stream is never in
    // capture mode (other libraries may enqueue on it concurrently).
    hipStream_t cap;
    if ((e = hipStreamCreateWithFlags(&cap, hipStreamNonBlocking)) != hipSuccess) return e;
    // Split-K counters cannot be created inside a capture: make them now.
    (void)stream_counters(cap);
    if ((e = hipStreamSynchronize(cap)) != hipSuccess) return e;
    e = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
      for (int i = 0; i < iters && e == hipSuccess; ++i) e = gemm(p, kernel, cap, nullptr);
      hipError_t e2 = hipStreamEndCapture(cap, &graph);
      if (e == hipSuccess) e = e2;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    hipStreamDestroy(cap);
    if (e != hipSuccess) {
      if (graph) hipGraphDestroy(graph);
      return e;
    }
    // Upload/first replay outside the timed region.
    if ((e = hipGraphUpload(exec, stream)) != hipSuccess) return e;
  }
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventRecord(t0, stream);
  if (exec) {
    e = hipGraphLaunch(exec, stream);
  } else {
    e = hipSuccess;
    for (int i = 0; i < iters && e == hipSuccess; ++i) e = gemm(p, kernel, stream, nullptr);
  }
  hipEventRecord(t1, stream);
  if (e == hipSuccess) e = hipEventSynchronize(t1);
  if (e == hipSuccess) e = hipEventElapsedTime(ms, t0, t1);
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  if (exec) hipGraphExecDestroy(exec);
  if (graph) hipGraphDestroy(graph);
  return e;
}

// ---- completion signals ------------------------------------------------------
hipError_t signal_create(int device, int slots, Signal** out) {
  *out = nullptr;
  if (slots <= 0) return hipErrorInvalidValue;
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return e;
  if ((e = hipSetDevice(device)) != hipSuccess) return e;
  Signal* s = new Signal();
  s->slots = slots;
  s->device = device;
  const size_t bytes = ((size_t)slots * sizeof(unsigned) + 255) / 256 * 256;
  e = hipMalloc(&s->dev, bytes);
  if (e == hipSuccess) e = hipMemset(s->dev, 0, bytes);
  // fine-grained, host-mapped: the GPU's system-scope flag stores land in host memory
  if (e == hipSuccess) e = hipHostMalloc(&s->host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    memset(s->host, 0, bytes);
    e = hipHostGetDevicePointer((void**)&s->host_dev, s->host, 0);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    signal_destroy(s);
    return e;
  }
  *out = s;
  return hipSuccess;
}

void signal_destroy(Signal* s) {
  if (!s) return;
  if (s->dev) (void)hipFree(s->dev);
  if (s->host) (void)hipHostFree(s->host);
  delete s;
}

unsigned signal_flag(const Signal* s, int slot) {
  return __atomic_load_n((volatile unsigned*)s->host + slot, __ATOMIC_ACQUIRE);
}

void signal_set(Signal* s, int slot, unsigned value) {
  if (!s || slot < 0 || slot >= s->slots) return;
  __atomic_store_n((volatile unsigned*)s->host + slot, value, __ATOMIC_RELEASE);
}

// Spins (pause) for the first kSpinUs — a piece's flag usually turns within
// tens of us of the wait starting, and this latency delays that piece's
// collective — then sleeps in growing steps up to kSleepMaxUs, so a rank
// waiting out a long GEMM does not hold a host core next to RCCL's proxy
// threads (8 ranks = 8 cores otherwise).
bool signal_wait(const Signal* s, int slot, unsigned epoch, double timeout_s) {
  if (!s || slot < 0 || slot >= s->slots) return false;
  constexpr double kSpinUs = 200.0;
  constexpr int kSleepMaxUs = 50;
  const auto t0 = std::chrono::steady_clock::now();
  int nap = 2;
  bool napping = false;
  for (unsigned spin = 0;; ++spin) {
    if ((int)(signal_flag(s, slot) - epoch) >= 0) return true;
    if (napping || (spin & 255) == 255) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) return false;
      napping = el * 1e6 > kSpinUs;
    }
    if (napping) {
      std::this_thread::sleep_for(std::chrono::microseconds(nap));
      nap = nap * 2 > kSleepMaxUs ? kSleepMaxUs : nap * 2;
    } else {
      __builtin_ia32_pause();
    }
  }
}

// ---- comm proxy ------------------------------------------------------------
__global__ void __launch_bounds__(256) proxy_copy(uint4* __restrict__ dst,
                                                  const uint4* __restrict__ src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

hipError_t comm_proxy(void* dst, const void* src, size_t bytes, int blocks, hipStream_t stream) {
  if (bytes % 16 || blocks <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(proxy_copy, dim3(blocks), dim3(256), 0, stream, (uint4*)dst, (const uint4*)src,
                     bytes / 16);
  return hipGetLastError();
}

const char* kernel_name(int kernel) {
  switch (kernel) {
    case kGeneric: return "pdmb_generic_nn";
    case kMfma256d: return "pdmb_mfma256d_nn";
    case kF32_256s: return "pdmb_f32_256s_nn";
    case kFp8W4: return "pdmb_fp8_w4_nt";
    case kFp8W4S: return "pdmb_fp8_w4s";
    case kFp8T128: return "pdmb_fp8_t128_nt";
    case kFp8T256x128: return "pdmb_fp8_t256x128_nt";
    case kMfmaW4: return "pdmb_w4_nn";
    case kMfmaW4S: return "pdmb_w4s";
    case kT128: return "pdmb_t128_nn";
    case kT128x2: return "pdmb_t128x2_nn";
    case kT256x128: return "pdmb_t256x128_nn";
    case kT192: return "pdmb_t192_nn";
    case kT192x128: return "pdmb_t192x128_nn";
    case kFp8T192: return "pdmb_fp8_t192_nt";
    case kFp8T192x128: return "pdmb_fp8_t192x128_nt";
    case kF32W4: return "pdmb_f32_w4_nn";
    case kF32W4L: return "pdmb_f32_w4l_nn";
    case kF32T128: return "pdmb_f32_t128_nn";
    case kF32T64: return "pdmb_f32_t64_nn";
    case kF32T64x2: return "pdmb_f32_t64x2_nn";
    case kF32T128x2: return "pdmb_f32_t128x2_nn";
    default: return is_experiment(kernel) ? experiment_name(kernel) : "auto";
  }
}

#ifdef PDMB_EXPERIMENTS
#include "experiments.h"
#endif

}  // namespace pdmb
