// Kernel selection and the native hipEvent timing loop.
//
// The reference times `iters` back-to-back torch.matmul calls between two
// CUDA events from Python (matmul_benchmark.py:54-68, matmul_scaling_
// benchmark.py:85-99). Here the loop itself is native: no Python and no
// allocator in the timed region, each launch writes a caller-owned output,
// and the launches can be captured once into a hipGraph.
#include <stdint.h>

#include "api.h"
#include "common.h"

namespace pdmb {

bool gemm256_supported(int dt, const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm256_launch(int dt, GemmArgs a, int sched, hipStream_t stream);
hipError_t gemm_generic_launch(int dt, GemmArgs a, bool vec, hipStream_t stream);
bool gemm_f32_256_supported(const GemmArgs& a, size_t align_a, size_t align_b, size_t align_c);
hipError_t gemm_f32_256_launch(GemmArgs a, int variant, hipStream_t stream);

static unsigned long long* g_debug_buffer = nullptr;

void set_debug_buffer(void* p) { g_debug_buffer = (unsigned long long*)p; }

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
  a.dbg = g_debug_buffer;
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

int resolve_kernel(const Problem& p, int kernel) {
  const GemmArgs a = to_args(p);
  const bool fast = gemm256_supported(p.dtype, a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  const bool f32fast = p.dtype == kF32 &&
                       gemm_f32_256_supported(a, (size_t)p.A, (size_t)p.B, (size_t)p.C);
  if (kernel == kAuto) return fast ? kMfma256c : (f32fast ? kF32_256s : kGeneric);
  if (kernel == kF32_256) return f32fast ? kF32_256 : -1;
  if (kernel == kF32_256s) return f32fast ? kF32_256s : -1;
  if (kernel == kMfma256) return fast ? kMfma256 : -1;
  if (kernel == kMfma256b) return fast ? kMfma256b : -1;
  if (kernel == kMfma256c) return fast ? kMfma256c : -1;
  if (kernel == kMfma256Stamp) return (fast && p.dtype == kBF16) ? kMfma256Stamp : -1;
  if (kernel == kGeneric) return kGeneric;
  return -1;
}

hipError_t gemm(const Problem& p, int kernel, hipStream_t stream, int* used) {
  const int k = resolve_kernel(p, kernel);
  if (used) *used = k;
  if (k < 0) return hipErrorInvalidValue;
  if (p.M == 0 || p.N == 0 || p.batch == 0) return hipSuccess;
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
  if (k == kMfma256) return gemm256_launch(p.dtype, a, 0, stream);
  if (k == kMfma256b) return gemm256_launch(p.dtype, a, 1, stream);
  if (k == kMfma256c) return gemm256_launch(p.dtype, a, 2, stream);
  if (k == kMfma256Stamp) return gemm256_launch(p.dtype, a, 3, stream);
  if (k == kF32_256) return gemm_f32_256_launch(a, 0, stream);
  if (k == kF32_256s) return gemm_f32_256_launch(a, 1, stream);
  return gemm_generic_launch(p.dtype, a, generic_vec_ok(p), stream);
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

const char* kernel_name(int kernel) {
  switch (kernel) {
    case kMfma256:
      return "pdmb_mfma256_nn";
    case kGeneric:
      return "pdmb_generic_nn";
    case kMfma256b:
      return "pdmb_mfma256b_nn";
    case kMfma256c:
      return "pdmb_mfma256c_nn";
    case kMfma256Stamp:
      return "pdmb_mfma256c_stamp";
    case kF32_256:
      return "pdmb_f32_256_nn";
    case kF32_256s:
      return "pdmb_f32_256s_nn";
    default:
      return "auto";
  }
}

}  // namespace pdmb
