// Python bindings of the native GEMM library (torch tensors in, enqueue on
// the caller's current HIP stream). Built with the host compiler against
// the PyTorch-ROCm headers; the kernels themselves live in the .hip files.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "api.h"

namespace {

int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat:
      return 0;
    case at::kHalf:
      return 1;
    case at::kBFloat16:
      return 2;
    case at::kFloat8_e4m3fn:
      return 3;
    default:
      TORCH_CHECK(false, "pdmb: unsupported dtype ", t,
                  " (float32 / float16 / bfloat16 / float8_e4m3fn only)");
  }
  return -1;
}

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pdmb: ", what, " failed: ", hipGetErrorString(e));
}

// A: [M,K] | [b,M,K], B: [K,N] | [b,K,N] (2-D B broadcasts over the batch),
// C: [M,N] | [b,M,N]; innermost stride must be 1 (leading dims free).
// float8_e4m3fn: B must be column-major (stride(-2) == 1, e.g. Bt.t() of a
// row-major [N,K] Bt) and C is bfloat16.
// Cp == nullptr: a probe-only Problem (kernel_for / splitk_for / ... without
// an `out`): C is taken as a contiguous [batch,] M x N at a 256-B aligned
// stand-in address the planner only checks for alignment — nothing is
// allocated just to ask which kernel would run.
pdmb::Problem make_problem(const at::Tensor& A, const at::Tensor& B, const at::Tensor* Cp,
                           double alpha = 1.0) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && (!Cp || Cp->is_cuda()), "pdmb: tensors must be on the GPU");
  TORCH_CHECK(A.device() == B.device() && (!Cp || A.device() == Cp->device()), "pdmb: device mismatch");
  const bool fp8 = A.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(A.scalar_type() == B.scalar_type() &&
                  (!Cp || Cp->scalar_type() == (fp8 ? at::kBFloat16 : A.scalar_type())),
              "pdmb: dtype mismatch (fp8 operands take a bfloat16 output)");
  TORCH_CHECK(A.dim() == 2 || A.dim() == 3, "pdmb: A must be 2-D or 3-D");
  TORCH_CHECK(B.dim() == 2 || B.dim() == 3, "pdmb: B must be 2-D or 3-D");
  const int64_t cdim = Cp ? Cp->dim() : std::max(A.dim(), B.dim());
  TORCH_CHECK(cdim == std::max(A.dim(), B.dim()), "pdmb: bad output rank");
  const bool batched = cdim == 3;
  const int64_t batch = batched ? (Cp ? Cp->size(0) : (A.dim() == 3 ? A.size(0) : B.size(0))) : 1;
  const int64_t M = A.size(-2), K = A.size(-1), N = B.size(-1);
  TORCH_CHECK(B.size(-2) == K, "pdmb: inner dimensions differ: ", A.sizes(), " @ ", B.sizes());
  TORCH_CHECK(!Cp || (Cp->size(-2) == M && Cp->size(-1) == N), "pdmb: output shape mismatch");
  if (batched) {
    TORCH_CHECK(A.dim() == 2 || A.size(0) == batch, "pdmb: batch mismatch");
    TORCH_CHECK(B.dim() == 2 || B.size(0) == batch, "pdmb: batch mismatch");
  }
  auto inner_ok = [](const at::Tensor& t) {
    return t.size(-1) <= 1 || t.stride(-1) == 1;
  };
  auto colmajor_ok = [](const at::Tensor& t) {
    return t.size(-2) <= 1 || t.stride(-2) == 1;
  };
  TORCH_CHECK(inner_ok(A) && (fp8 ? colmajor_ok(B) : inner_ok(B)) && (!Cp || inner_ok(*Cp)),
              fp8 ? "pdmb: fp8 needs row-major A / C and column-major B"
                  : "pdmb: innermost dim must be contiguous");
  // Leading dimension = the real row stride. A row stride below the row
  // length (expanded / overlapping views) would make the kernels address
  // memory outside the tensor, so it is refused (ops/gemm.py makes such
  // inputs contiguous first; an overlapping `out` is an error).
  auto ld = [](const at::Tensor& t, const char* what) {
    const int64_t rows = t.size(-2), cols = t.size(-1);
    if (rows <= 1) return std::max<int64_t>(cols, 1);
    TORCH_CHECK(t.stride(-2) >= cols, "pdmb: ", what, " row stride ", t.stride(-2),
                " < row length ", cols, " (overlapping or expanded view)");
    return t.stride(-2);
  };
  TORCH_CHECK(!Cp || !batched || Cp->size(0) <= 1 || Cp->stride(0) >= Cp->size(-2) * ld(*Cp, "out"),
              "pdmb: out batch stride overlaps (expanded or aliased output)");
  pdmb::Problem p{};
  p.dtype = dtype_code(A.scalar_type());
  p.A = A.data_ptr();
  p.B = B.data_ptr();
  p.C = Cp ? Cp->data_ptr() : (void*)(uintptr_t)256;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = (int)ld(A, "A");
  if (fp8) {
    TORCH_CHECK(N <= 1 || B.stride(-1) >= K, "pdmb: fp8 B column stride < K (overlapping view)");
    const int64_t lb = std::max<int64_t>(B.stride(-1), std::max<int64_t>(K, 1));
    p.ldb = (int)lb;  // distance between columns (Bt row stride)
  } else {
    p.ldb = (int)ld(B, "B");
  }
  p.alpha = (float)alpha;
  p.ldc = Cp ? (int)ld(*Cp, "out") : (int)std::max<int64_t>(N, 1);
  p.sA = (batched && A.dim() == 3) ? A.stride(0) : 0;
  p.sB = (batched && B.dim() == 3) ? B.stride(0) : 0;
  p.sC = batched ? (Cp ? Cp->stride(0) : M * N) : 0;
  p.batch = (int)batch;
  return p;
}

at::Tensor alloc_out(const at::Tensor& A, const at::Tensor& B) {
  std::vector<int64_t> shape;
  if (A.dim() == 3 || B.dim() == 3) shape.push_back(A.dim() == 3 ? A.size(0) : B.size(0));
  shape.push_back(A.size(-2));
  shape.push_back(B.size(-1));
  const bool fp8 = A.scalar_type() == at::kFloat8_e4m3fn;
  return at::empty(shape, A.options().dtype(fp8 ? at::kBFloat16 : A.scalar_type()));
}

// Scratch for one launch from PyTorch's caching allocator on the launch
// stream (padded copies, split-K partials): stream-ordered reuse, safe under
// concurrent streams and torch.cuda.graph capture, never shared.
at::Tensor workspace_for(pdmb::Problem& p, int kernel, const at::Tensor& like) {
  const size_t need = pdmb::gemm_workspace_bytes(p, kernel);
  if (!need) return at::Tensor();
  at::Tensor ws = at::empty({(int64_t)need}, like.options().dtype(at::kByte));
  p.workspace = ws.data_ptr();
  p.workspace_bytes = need;
  return ws;
}

const at::Tensor* opt(const c10::optional<at::Tensor>& C) { return C.has_value() ? &*C : nullptr; }

pdmb::Signal* as_signal(int64_t h) { return reinterpret_cast<pdmb::Signal*>((uintptr_t)h); }

// sig (a signal_create handle, 0 = none), sig_rows, sig_epoch: the launch
// signals per-slot completion (api.h Problem::sig).
at::Tensor matmul(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> out,
                  int64_t kernel, double alpha, int64_t splitk, int64_t cus, int64_t sig,
                  int64_t sig_rows, int64_t sig_epoch) {
  at::Tensor C = out.has_value() ? *out : alloc_out(A, B);
  pdmb::Problem p = make_problem(A, B, &C, alpha);
  p.splitk = (int)splitk;
  p.cus = (int)cus;
  if (sig) {
    p.sig = as_signal(sig);
    TORCH_CHECK(p.sig->device == A.device().index(), "pdmb: signal set lives on another device");
    p.sig_rows = (int)sig_rows;
    p.sig_epoch = (unsigned)sig_epoch;
  }
  c10::hip::HIPGuard guard(A.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(A.device().index()).stream();
  at::Tensor ws = workspace_for(p, (int)kernel, A);
  int used = -1;
  hipError_t e = pdmb::gemm(p, (int)kernel, s, &used);
  TORCH_CHECK(used >= 0, "pdmb: kernel ", kernel, " cannot run this problem",
              sig ? " signalled (W4 only)" : "");
  check_hip(e, "gemm launch");
  return C;
}

int64_t signal_create(int64_t device, int64_t slots) {
  pdmb::Signal* s = nullptr;
  check_hip(pdmb::signal_create((int)device, (int)slots, &s), "signal_create");
  return (int64_t)(uintptr_t)s;
}

void signal_destroy(int64_t h) { pdmb::signal_destroy(as_signal(h)); }

// Host wait (GIL released) until slot's flag reaches epoch; false on timeout.
bool signal_wait(int64_t h, int64_t slot, int64_t epoch, double timeout_s) {
  TORCH_CHECK(h != 0, "pdmb: null signal set");
  py::gil_scoped_release nogil;
  return pdmb::signal_wait(as_signal(h), (int)slot, (unsigned)epoch, timeout_s);
}

int64_t signal_flag(int64_t h, int64_t slot) {
  TORCH_CHECK(h != 0 && slot >= 0 && slot < as_signal(h)->slots, "pdmb: bad signal slot");
  return (int64_t)pdmb::signal_flag(as_signal(h), (int)slot);
}

void signal_set(int64_t h, int64_t slot, int64_t value) {
  TORCH_CHECK(h != 0 && slot >= 0 && slot < as_signal(h)->slots, "pdmb: bad signal slot");
  pdmb::signal_set(as_signal(h), (int)slot, (unsigned)value);
}

// A one-wave kernel on the current stream that holds it until flag[slot] >=
// value (signal_set from the host) or timeout_s pass.
void gate(int64_t h, int64_t slot, int64_t value, double timeout_s) {
  TORCH_CHECK(h != 0, "pdmb: null signal set");
  pdmb::Signal* s = as_signal(h);
  c10::hip::HIPGuard guard((c10::DeviceIndex)s->device);
  hipStream_t st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)s->device).stream();
  check_hip(pdmb::gate(s, (int)slot, (unsigned)value, timeout_s, st), "gate");
}

// Tile rows per completion unit (0: the problem cannot run signalled).
int64_t signal_granule(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> C, int64_t kernel,
                       int64_t cus) {
  pdmb::Problem p = make_problem(A, B, opt(C));
  p.cus = (int)cus;
  return pdmb::signal_granule(p, (int)kernel);
}

int64_t resolve(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> C, int64_t kernel,
                int64_t cus) {
  pdmb::Problem p = make_problem(A, B, opt(C));
  p.cus = (int)cus;
  return pdmb::resolve_kernel(p, (int)kernel);
}

int64_t resolve_padded(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> C,
                       int64_t cus) {
  pdmb::Problem p = make_problem(A, B, opt(C));
  p.cus = (int)cus;
  return pdmb::resolve_padded(p);
}

// K slices the W4 / T128 kernel would use (1 = no split; 0 if neither runs it).
int64_t splitk_for(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> C, int64_t kernel,
                   int64_t splitk, int64_t cus) {
  pdmb::Problem p = make_problem(A, B, opt(C));
  p.splitk = (int)splitk;
  p.cus = (int)cus;
  return pdmb::choose_splitk(p, (int)kernel);
}

// {M1, S, T1, R}: auto runs rows [0, M1) unsplit and [M1, M) split S ways, or
// (tile-range form) tiles [0, T1) unsplit and the rest split S ways — or, R > 1
// (refined tail), cut into R smaller tiles each; {0, 1, 0, 1}: one launch.
std::tuple<int64_t, int64_t, int64_t, int64_t> tail_split_for(const at::Tensor& A, const at::Tensor& B,
                                                     c10::optional<at::Tensor> C, int64_t kernel,
                                                     int64_t cus) {
  pdmb::Problem p = make_problem(A, B, opt(C));
  p.cus = (int)cus;
  const auto t = pdmb::tail_split(p, (int)kernel);
  return {t.m1, t.S, t.tiles_dp, t.sub};
}

// The planner's decision for a SHAPE (no tensors: contiguous operands at an
// aligned stand-in address, so it runs without a GPU): (kernel id, split-K,
// model cost us, tail M1, tail S, tail T1, tail R). dtype: 0 f32, 1 f16, 2 bf16, 3 fp8.
std::tuple<int64_t, int64_t, double, int64_t, int64_t, int64_t, int64_t> plan_shape(int64_t dtype, int64_t M, int64_t N,
                                                                  int64_t K, int64_t batch,
                                                                  int64_t kernel, int64_t cus) {
  pdmb::Problem p{};
  p.dtype = (int)dtype;
  p.A = p.B = p.C = (void*)(uintptr_t)4096;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = (int)K;
  p.ldb = dtype == 3 ? (int)K : (int)N;  // fp8 B is column-major (Bt [N, K])
  p.ldc = (int)N;
  p.batch = (int)batch;
  p.sA = M * K;
  p.sB = K * N;
  p.sC = M * N;
  p.cus = (int)cus;
  const pdmb::PlanInfo r = pdmb::plan_info(p, (int)kernel);
  return {r.kernel, r.splitk, r.cost_us, r.tail_m1, r.tail_S, r.tail_tiles_dp, r.tail_sub};
}

// Total milliseconds for `iters` timed launches (after `warmup`).
double bench(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t iters,
             int64_t warmup, bool graph, int64_t kernel, int64_t splitk) {
  pdmb::Problem p = make_problem(A, B, &C);
  p.splitk = (int)splitk;
  TORCH_CHECK(pdmb::resolve_kernel(p, (int)kernel) >= 0, "pdmb: kernel cannot run this problem");
  c10::hip::HIPGuard guard(A.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(A.device().index()).stream();
  at::Tensor ws = workspace_for(p, (int)kernel, A);  // lives across every timed launch
  float ms = 0.f;
  check_hip(pdmb::bench_gemm(p, (int)kernel, (int)iters, (int)warmup, graph, s, &ms), "bench_gemm");
  return (double)ms;
}

// A stream whose kernels may use only the CUs NOT in `excluded` (the GEMM
// side of a comm/compute overlap: RCCL's workgroups get those CUs at once
// instead of waiting for GEMM workgroups to retire). Bit i of the HIP CU mask
// is CU i of the device's enumeration; `excluded` are those indices. Returns
// the raw handle (wrap with torch.cuda.ExternalStream; free with
// destroy_stream).
int64_t create_cu_masked_stream(int64_t device, std::vector<int64_t> excluded) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  hipDeviceProp_t prop;
  check_hip(hipGetDeviceProperties(&prop, (int)device), "hipGetDeviceProperties");
  const int ncu = prop.multiProcessorCount;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
  for (int64_t i : excluded) {
    TORCH_CHECK(i >= 0 && i < ncu, "pdmb: CU index ", i, " outside [0, ", ncu, ")");
    mask[i / 32] &= ~(1u << (i % 32));
  }
  hipStream_t s = nullptr;
  check_hip(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()),
            "hipExtStreamCreateWithCUMask");
  return (int64_t)(uintptr_t)s;
}

std::vector<int64_t> stream_cu_mask(int64_t stream, int64_t device) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  hipDeviceProp_t prop;
  check_hip(hipGetDeviceProperties(&prop, (int)device), "hipGetDeviceProperties");
  std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
  check_hip(hipExtStreamGetCUMask((hipStream_t)(uintptr_t)stream, (uint32_t)mask.size(), mask.data()),
            "hipExtStreamGetCUMask");
  return std::vector<int64_t>(mask.begin(), mask.end());
}

void destroy_stream(int64_t stream) {
  check_hip(hipStreamDestroy((hipStream_t)(uintptr_t)stream), "hipStreamDestroy");
}

std::string kernel_name(int64_t k) { return pdmb::kernel_name((int)k); }

// Comm proxy (overlap experiments): copy src -> dst with `blocks` workgroups
// on the current stream.
void comm_proxy(const at::Tensor& dst, const at::Tensor& src, int64_t blocks) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda() && dst.is_contiguous() && src.is_contiguous() &&
                  dst.nbytes() == src.nbytes() && dst.nbytes() % 16 == 0,
              "pdmb: comm_proxy needs equal-size contiguous GPU tensors (bytes % 16 == 0)");
  c10::hip::HIPGuard guard(dst.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(dst.device().index()).stream();
  check_hip(pdmb::comm_proxy(dst.data_ptr(), src.data_ptr(), dst.nbytes(), (int)blocks, s),
            "comm_proxy");
}

// out = sum of srcs (fp32 accumulate, in list order) on the current stream: the
// local step of the direct two-shot all-reduce. out may be one of srcs.
void reduce_sum(const at::Tensor& out, const std::vector<at::Tensor>& srcs) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= pdmb::kMaxReduceSrcs, "pdmb: reduce_sum takes 1..",
              pdmb::kMaxReduceSrcs, " sources");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "pdmb: reduce_sum out must be a contiguous GPU tensor");
  const int dt = dtype_code(out.scalar_type());
  TORCH_CHECK(dt <= 2, "pdmb: reduce_sum takes float32 / float16 / bfloat16");
  std::vector<const void*> ptrs;
  for (const auto& t : srcs) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.device() == out.device() &&
                    t.scalar_type() == out.scalar_type() && t.numel() == out.numel(),
                "pdmb: reduce_sum sources must be contiguous, on out's device, of its dtype and length");
    ptrs.push_back(t.data_ptr());
  }
  c10::hip::HIPGuard guard(out.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(out.device().index()).stream();
  check_hip(pdmb::reduce_sum(out.data_ptr(), ptrs.data(), (int)ptrs.size(), out.numel(), dt, s), "reduce_sum");
}

// ---- xGMI peer memory (parallel/ipc.py IpcGather) --------------------------
// IPC-exportable tensors come from a process-lifetime pool (the "arena"):
// every buffer is its own hipMalloc allocation (so its IPC handle maps exactly
// it, offset 0) and is never freed before exit — when its last torch
// reference goes it returns to the pool and the next ipc_empty of the same
// size and device takes it again. Its IPC handle is made once and cached.
// Why: with buffers freed and re-allocated between benchmark modes, handle
// bytes, buffer addresses and peer mappings are all reused
// (scripts/ipc_handle_probe.py records which), so a mapping or a cache entry
// that outlives its buffer can name memory that is gone
// (docs/ARCHITECTURE.md "IPC fault"). With the pool, one handle always means
// one live buffer, and a peer's mapping of it stays valid for the process.
// PDMB_IPC_ARENA=0 (tests, diagnosis) restores hipFree on release and a
// fresh handle per call.
struct IpcBuf {
  void* p;
  size_t bytes;
  int dev;
  bool in_use;
  std::string handle;  // cached hipIpcMemHandle_t bytes ("" until first export)
};
std::mutex g_ipc_mu;
std::vector<IpcBuf>& ipc_pool() {
  static std::vector<IpcBuf>* v = new std::vector<IpcBuf>();  // never destroyed: the runtime may go first
  return *v;
}
bool ipc_arena() {
  const char* e = std::getenv("PDMB_IPC_ARENA");
  return !(e && std::string(e) == "0");
}

at::Tensor ipc_empty(std::vector<int64_t> shape, at::ScalarType dtype, int64_t device) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  int64_t n = 1;
  for (int64_t d : shape) {
    TORCH_CHECK(d >= 0, "pdmb: ipc_empty: negative dimension");
    n *= d;
  }
  const size_t bytes = std::max<size_t>((size_t)n * c10::elementSize(dtype), 256);
  const int dev = (int)device;
  const bool arena = ipc_arena();
  void* p = nullptr;
  if (arena) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto& b : ipc_pool()) {
      if (!b.in_use && b.bytes == bytes && b.dev == dev) {
        b.in_use = true;
        p = b.p;
        break;
      }
    }
  }
  if (p) {
    // A released buffer returns to the pool when its last torch reference
    // goes, which can be before this device's queued work on it has run
    // (hipFree would have synchronized): drain the device before handing it
    // out again. Setup-time only (ipc_empty is never called in a timed loop).
    check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize (ipc_empty reuse)");
  } else {
    check_hip(hipMalloc(&p, bytes), "hipMalloc (ipc_empty)");
    if (arena) {
      std::lock_guard<std::mutex> lk(g_ipc_mu);
      ipc_pool().push_back({p, bytes, dev, true, std::string()});
    }
  }
  return at::from_blob(
      p, shape,
      [dev, arena](void* q) {
        if (arena) {  // back to the pool: still allocated, still exported, handle unchanged
          std::lock_guard<std::mutex> lk(g_ipc_mu);
          for (auto& b : ipc_pool())
            if (b.p == q) b.in_use = false;
          return;
        }
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(dev);
        (void)hipFree(q);
        (void)hipSetDevice(cur);
      },
      at::TensorOptions().dtype(dtype).device(at::Device(at::kCUDA, (c10::DeviceIndex)device)));
}

// (buffers in the pool, of them in use, bytes held)
std::tuple<int64_t, int64_t, int64_t> ipc_pool_stats() {
  std::lock_guard<std::mutex> lk(g_ipc_mu);
  int64_t used = 0, bytes = 0;
  for (const auto& b : ipc_pool()) {
    used += b.in_use;
    bytes += (int64_t)b.bytes;
  }
  return {(int64_t)ipc_pool().size(), used, bytes};
}

// The IPC handle of an ipc_empty tensor (its data pointer must be the base
// of its allocation); a pooled buffer's handle is made once and reused.
py::bytes ipc_handle(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "pdmb: ipc_handle needs a GPU tensor");
  c10::hip::HIPGuard guard(t.device().index());
  void* base = nullptr;
  size_t size = 0;
  check_hip(hipMemGetAddressRange(&base, &size, t.data_ptr()), "hipMemGetAddressRange");
  TORCH_CHECK(base == t.data_ptr(), "pdmb: ipc_handle: the tensor must start its own allocation "
              "(allocate it with ipc_empty)");
  {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (const auto& b : ipc_pool())
      if (b.p == base && !b.handle.empty()) return py::bytes(b.handle);
  }
  hipIpcMemHandle_t h;
  check_hip(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  std::string hs(reinterpret_cast<const char*>(&h), sizeof(h));
  {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto& b : ipc_pool())
      if (b.p == base) b.handle = hs;
  }
  return py::bytes(hs);
}

// (base, size) of the live allocation or peer mapping that holds `addr` in
// this process (hipMemGetAddressRange); raises if none does — an address of
// a closed mapping or a freed buffer (parallel/ipc.py PDMB_IPC_CHECK=1
// checks every pull's source and destination range against it on the host,
// before the launch).
std::tuple<int64_t, int64_t> ipc_range(int64_t addr, int64_t device) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  void* base = nullptr;
  size_t size = 0;
  const hipError_t e = hipMemGetAddressRange(&base, &size, (void*)(uintptr_t)addr);
  TORCH_CHECK(e == hipSuccess, "pdmb: ipc_range: ", std::hex, "0x", addr, std::dec,
              " is not inside a live allocation or mapping of this process (", hipGetErrorString(e), ")");
  return {(int64_t)(uintptr_t)base, (int64_t)size};
}

// Map a peer's allocation into this process (device `device`); returns the
// local address. Close with ipc_close before the exporter frees it.
int64_t ipc_open(py::bytes handle, int64_t device) {
  const std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "pdmb: ipc_open: bad handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  void* p = nullptr;
  check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return (int64_t)(uintptr_t)p;
}

void ipc_close(int64_t ptr, int64_t device) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  check_hip(hipIpcCloseMemHandle((void*)(uintptr_t)ptr), "hipIpcCloseMemHandle");
}

// dst (contiguous, this device) <- `dst.nbytes()` bytes at a peer address
// (an ipc_open mapping + offset), on the current stream. sdma: the
// hipMemcpyDeviceToDeviceNoCU kind, a DMA-engine copy that takes no CU (a
// plain DeviceToDevice copy runs the runtime's blit kernel on CUs); else the
// plain kind (the runtime picks).
void copy_from_peer(const at::Tensor& dst, int64_t src_addr, bool sdma) {
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "pdmb: copy_from_peer: dst must be a contiguous GPU tensor");
  TORCH_CHECK(src_addr != 0, "pdmb: copy_from_peer: null source");
  c10::hip::HIPGuard guard(dst.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(dst.device().index()).stream();
  check_hip(hipMemcpyAsync(dst.data_ptr(), (const void*)(uintptr_t)src_addr, dst.nbytes(),
                           sdma ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice, s),
            "hipMemcpyAsync (copy_from_peer)");
}

// dsts[i] (contiguous, this device) <- dsts[i].nbytes() bytes at srcs[i] (a
// peer mapping + offset, or a local address), every copy in ONE kernel launch
// on the current stream (reduce.hip multi_copy: all links read at once).
void peer_copy(const std::vector<at::Tensor>& dsts, const std::vector<int64_t>& srcs, int64_t blocks_per) {
  TORCH_CHECK(dsts.size() == srcs.size() && (int)dsts.size() <= pdmb::kMaxCopies,
              "pdmb: peer_copy takes equal-length lists of at most ", pdmb::kMaxCopies);
  if (dsts.empty()) return;
  std::vector<void*> d;
  std::vector<const void*> s;
  std::vector<size_t> b;
  for (size_t i = 0; i < dsts.size(); ++i) {
    TORCH_CHECK(dsts[i].is_cuda() && dsts[i].is_contiguous() && dsts[i].device() == dsts[0].device(),
                "pdmb: peer_copy destinations must be contiguous tensors on one GPU");
    TORCH_CHECK(srcs[i] != 0 || dsts[i].nbytes() == 0, "pdmb: peer_copy: null source");
    d.push_back(dsts[i].data_ptr());
    s.push_back((const void*)(uintptr_t)srcs[i]);
    b.push_back(dsts[i].nbytes());
  }
  c10::hip::HIPGuard guard(dsts[0].device().index());
  hipStream_t st = c10::hip::getCurrentHIPStream(dsts[0].device().index()).stream();
  check_hip(pdmb::multi_copy(d.data(), s.data(), b.data(), (int)d.size(), (int)blocks_per, st), "multi_copy");
}

// out = sum over the sources at raw device addresses (peer mappings + offsets,
// or local; each out.numel() elements of out's dtype), fp32 accumulate in list
// order, on the current stream; blocks > 0 caps the grid.
void reduce_sum_addrs(const at::Tensor& out, const std::vector<int64_t>& addrs, int64_t blocks) {
  TORCH_CHECK(!addrs.empty() && (int)addrs.size() <= pdmb::kMaxReduceSrcs, "pdmb: reduce_sum_addrs takes 1..",
              pdmb::kMaxReduceSrcs, " sources");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "pdmb: reduce_sum_addrs out must be a contiguous GPU tensor");
  const int dt = dtype_code(out.scalar_type());
  TORCH_CHECK(dt <= 2, "pdmb: reduce_sum_addrs takes float32 / float16 / bfloat16");
  std::vector<const void*> ptrs;
  for (int64_t a : addrs) {
    TORCH_CHECK(a != 0, "pdmb: reduce_sum_addrs: null source");
    ptrs.push_back((const void*)(uintptr_t)a);
  }
  c10::hip::HIPGuard guard(out.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(out.device().index()).stream();
  check_hip(pdmb::reduce_sum(out.data_ptr(), ptrs.data(), (int)ptrs.size(), out.numel(), dt, s, (int)blocks),
            "reduce_sum");
}

// Diagnostic: set (or clear, with None) the device buffer the stamp kernel writes.
void set_debug_buffer(c10::optional<at::Tensor> buf) {
  if (buf.has_value()) {
    TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kLong && buf->is_contiguous(),
                "pdmb: debug buffer must be a contiguous int64 GPU tensor");
    pdmb::set_debug_buffer(buf->data_ptr());
  } else {
    pdmb::set_debug_buffer(nullptr);
  }
}

// Diagnostics: a host-mapped, coherent buffer that the stamping kernels of an
// experiments build write with system-scope stores, readable by the host
// WHILE a kernel runs (e.g. one that never finishes: scripts/w4s_hang_probe.py).
int64_t host_stamp_alloc(int64_t bytes) {
  void* p = nullptr;
  check_hip(hipHostMalloc(&p, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  memset(p, 0xff, (size_t)bytes);
  pdmb::set_debug_buffer(p);
  return (int64_t)(uintptr_t)p;
}
void host_stamp_free(int64_t ptr) {  // (clears the debug buffer it set)
  pdmb::set_debug_buffer(nullptr);
  if (ptr) check_hip(hipHostFree((void*)(uintptr_t)ptr), "hipHostFree");
}
std::vector<int64_t> host_stamp_read(int64_t ptr, int64_t n) {
  const volatile long long* q = (const volatile long long*)(uintptr_t)ptr;
  std::vector<int64_t> out((size_t)n);
  for (int64_t i = 0; i < n; ++i) out[(size_t)i] = q[i];
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) native GEMM kernels and timing loop";
  m.def("matmul", &matmul, "C = A @ B on gfx950 MFMA (fp8: C = alpha * A @ B, bf16 out)",
        py::arg("A"), py::arg("B"), py::arg("out") = py::none(), py::arg("kernel") = 0,
        py::arg("alpha") = 1.0, py::arg("splitk") = 0, py::arg("cus") = 0, py::arg("sig") = 0,
        py::arg("sig_rows") = 0, py::arg("sig_epoch") = 0);
  m.def("signal_create", &signal_create, py::arg("device"), py::arg("slots"));
  m.def("signal_destroy", &signal_destroy, py::arg("handle"));
  m.def("signal_wait", &signal_wait, py::arg("handle"), py::arg("slot"), py::arg("epoch"),
        py::arg("timeout_s"));
  m.def("signal_flag", &signal_flag, py::arg("handle"), py::arg("slot"));
  m.def("signal_set", &signal_set, py::arg("handle"), py::arg("slot"), py::arg("value"));
  m.def("gate", &gate, "one-wave kernel holding the current stream until flag[slot] >= value",
        py::arg("handle"), py::arg("slot"), py::arg("value"), py::arg("timeout_s"));
  m.def("signal_granule", &signal_granule, py::arg("A"), py::arg("B"), py::arg("out") = py::none(),
        py::arg("kernel") = 0, py::arg("cus") = 0);
  m.def("resolve", &resolve, "kernel id that would run (or -1)", py::arg("A"), py::arg("B"),
        py::arg("out") = py::none(), py::arg("kernel") = 0, py::arg("cus") = 0);
  m.def("resolve_padded", &resolve_padded, "kernel the padded fast path runs (or -1)",
        py::arg("A"), py::arg("B"), py::arg("out") = py::none(), py::arg("cus") = 0);
  m.def("splitk_for", &splitk_for, "W4 K slices for this problem (0: not W4)", py::arg("A"),
        py::arg("B"), py::arg("out") = py::none(), py::arg("kernel") = 0, py::arg("splitk") = 0,
        py::arg("cus") = 0);
  m.def("tail_split_for", &tail_split_for, "auto's wave-quantisation tail {M1, S, T1, R} ({0, 1, 0, 1}: none)",
        py::arg("A"), py::arg("B"), py::arg("out") = py::none(), py::arg("kernel") = 0,
        py::arg("cus") = 0);
  m.def("bench", &bench, "native hipEvent timing loop; returns total ms", py::arg("A"),
        py::arg("B"), py::arg("out"), py::arg("iters"), py::arg("warmup"),
        py::arg("graph") = false, py::arg("kernel") = 0, py::arg("splitk") = 0);
  m.def("kernel_name", &kernel_name);
  m.def("plan_shape", &plan_shape, py::arg("dtype"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("batch") = 1, py::arg("kernel") = 0, py::arg("cus") = 0);
  m.def("comm_proxy", &comm_proxy, py::arg("dst"), py::arg("src"), py::arg("blocks"));
  m.def("reduce_sum", &reduce_sum, "out = sum(srcs) (fp32 accumulate, list order)", py::arg("out"),
        py::arg("srcs"));
  m.def("ipc_empty", &ipc_empty, "tensor in its own hipMalloc allocation (IPC-exportable)",
        py::arg("shape"), py::arg("dtype"), py::arg("device"));
  m.def("ipc_handle", &ipc_handle, py::arg("t"));
  m.def("ipc_pool_stats", &ipc_pool_stats, "(pooled IPC buffers, in use, bytes)");
  m.def("ipc_range", &ipc_range, "(base, size) of the allocation / mapping holding addr",
        py::arg("addr"), py::arg("device"));
  m.def("ipc_open", &ipc_open, py::arg("handle"), py::arg("device"));
  m.def("ipc_close", &ipc_close, py::arg("ptr"), py::arg("device"));
  m.def("copy_from_peer", &copy_from_peer, py::arg("dst"), py::arg("src_addr"), py::arg("sdma") = true);
  m.def("peer_copy", &peer_copy, "dsts[i] <- bytes at srcs[i], one launch", py::arg("dsts"), py::arg("srcs"),
        py::arg("blocks_per") = 0);
  m.def("reduce_sum_addrs", &reduce_sum_addrs, "out = sum of the sources at raw addresses", py::arg("out"),
        py::arg("addrs"), py::arg("blocks") = 0);
  m.attr("MAX_COPIES") = pdmb::kMaxCopies;
  m.def("set_debug_buffer", &set_debug_buffer, py::arg("buf") = py::none());
  m.def("create_cu_masked_stream", &create_cu_masked_stream, py::arg("device"),
        py::arg("excluded"));
  m.def("stream_cu_mask", &stream_cu_mask, py::arg("stream"), py::arg("device"));
  m.def("destroy_stream", &destroy_stream, py::arg("stream"));
  m.attr("EXPERIMENTS") = pdmb::experiments_built();
  m.def("host_stamp_alloc", &host_stamp_alloc, py::arg("bytes"));
  m.def("host_stamp_read", &host_stamp_read, py::arg("ptr"), py::arg("n"));
  m.def("host_stamp_free", &host_stamp_free, py::arg("ptr"));
  m.attr("MAX_SPLIT_TILES") = pdmb::kMaxSplitTiles;
  m.attr("ARCH") = "gfx950";
}
