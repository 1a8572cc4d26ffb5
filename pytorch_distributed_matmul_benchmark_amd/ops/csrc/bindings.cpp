// Python bindings of the native GEMM library (torch tensors in, enqueue on
// the caller's current HIP stream). Built with the host compiler against
// the PyTorch-ROCm headers; the kernels themselves live in the .hip files.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <string>

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
pdmb::Problem make_problem(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C,
                           double alpha = 1.0) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "pdmb: tensors must be on the GPU");
  TORCH_CHECK(A.device() == B.device() && A.device() == C.device(), "pdmb: device mismatch");
  const bool fp8 = A.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(A.scalar_type() == B.scalar_type() &&
                  C.scalar_type() == (fp8 ? at::kBFloat16 : A.scalar_type()),
              "pdmb: dtype mismatch (fp8 operands take a bfloat16 output)");
  TORCH_CHECK(A.dim() == 2 || A.dim() == 3, "pdmb: A must be 2-D or 3-D");
  TORCH_CHECK(B.dim() == 2 || B.dim() == 3, "pdmb: B must be 2-D or 3-D");
  TORCH_CHECK(C.dim() == std::max(A.dim(), B.dim()), "pdmb: bad output rank");
  const bool batched = C.dim() == 3;
  const int64_t batch = batched ? C.size(0) : 1;
  const int64_t M = A.size(-2), K = A.size(-1), N = B.size(-1);
  TORCH_CHECK(B.size(-2) == K, "pdmb: inner dimensions differ: ", A.sizes(), " @ ", B.sizes());
  TORCH_CHECK(C.size(-2) == M && C.size(-1) == N, "pdmb: output shape mismatch");
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
  TORCH_CHECK(inner_ok(A) && (fp8 ? colmajor_ok(B) : inner_ok(B)) && inner_ok(C),
              fp8 ? "pdmb: fp8 needs row-major A / C and column-major B"
                  : "pdmb: innermost dim must be contiguous");
  auto ld = [](const at::Tensor& t) {
    int64_t l = t.stride(-2);
    return std::max<int64_t>(l, std::max<int64_t>(t.size(-1), 1));
  };
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31) && batch < (1LL << 31),
              "pdmb: dimension too large");
  pdmb::Problem p{};
  p.dtype = dtype_code(A.scalar_type());
  p.A = A.data_ptr();
  p.B = B.data_ptr();
  p.C = C.data_ptr();
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = (int)ld(A);
  if (fp8) {
    const int64_t lb = std::max<int64_t>(B.stride(-1), std::max<int64_t>(K, 1));
    p.ldb = (int)lb;  // distance between columns (Bt row stride)
  } else {
    p.ldb = (int)ld(B);
  }
  p.alpha = (float)alpha;
  p.ldc = (int)ld(C);
  p.sA = (batched && A.dim() == 3) ? A.stride(0) : 0;
  p.sB = (batched && B.dim() == 3) ? B.stride(0) : 0;
  p.sC = batched ? C.stride(0) : 0;
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

at::Tensor matmul(const at::Tensor& A, const at::Tensor& B, c10::optional<at::Tensor> out,
                  int64_t kernel, double alpha) {
  at::Tensor C = out.has_value() ? *out : alloc_out(A, B);
  pdmb::Problem p = make_problem(A, B, C, alpha);
  c10::hip::HIPGuard guard(A.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(A.device().index()).stream();
  int used = -1;
  hipError_t e = pdmb::gemm(p, (int)kernel, s, &used);
  TORCH_CHECK(used >= 0, "pdmb: kernel ", kernel, " cannot run this problem");
  check_hip(e, "gemm launch");
  return C;
}

int64_t resolve(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t kernel) {
  return pdmb::resolve_kernel(make_problem(A, B, C), (int)kernel);
}

// Total milliseconds for `iters` timed launches (after `warmup`).
double bench(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t iters,
             int64_t warmup, bool graph, int64_t kernel) {
  pdmb::Problem p = make_problem(A, B, C);
  TORCH_CHECK(pdmb::resolve_kernel(p, (int)kernel) >= 0, "pdmb: kernel cannot run this problem");
  c10::hip::HIPGuard guard(A.device().index());
  hipStream_t s = c10::hip::getCurrentHIPStream(A.device().index()).stream();
  float ms = 0.f;
  check_hip(pdmb::bench_gemm(p, (int)kernel, (int)iters, (int)warmup, graph, s, &ms), "bench_gemm");
  return (double)ms;
}

std::string kernel_name(int64_t k) { return pdmb::kernel_name((int)k); }

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

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) native GEMM kernels and timing loop";
  m.def("matmul", &matmul, "C = A @ B on gfx950 MFMA (fp8: C = alpha * A @ B, bf16 out)",
        py::arg("A"), py::arg("B"), py::arg("out") = py::none(), py::arg("kernel") = 0,
        py::arg("alpha") = 1.0);
  m.def("resolve", &resolve, "kernel id that would run (or -1)", py::arg("A"), py::arg("B"),
        py::arg("out"), py::arg("kernel") = 0);
  m.def("bench", &bench, "native hipEvent timing loop; returns total ms", py::arg("A"),
        py::arg("B"), py::arg("out"), py::arg("iters"), py::arg("warmup"),
        py::arg("graph") = false, py::arg("kernel") = 0);
  m.def("kernel_name", &kernel_name);
  m.def("set_debug_buffer", &set_debug_buffer, py::arg("buf") = py::none());
  m.attr("KERNEL_AUTO") = (int)pdmb::kAuto;
  m.attr("KERNEL_MFMA256") = (int)pdmb::kMfma256;
  m.attr("KERNEL_GENERIC") = (int)pdmb::kGeneric;
  m.attr("KERNEL_MFMA256B") = (int)pdmb::kMfma256b;
  m.attr("KERNEL_MFMA256C") = (int)pdmb::kMfma256c;
  m.attr("KERNEL_MFMA256_STAMP") = (int)pdmb::kMfma256Stamp;
  m.attr("KERNEL_F32_256") = (int)pdmb::kF32_256;
  m.attr("ARCH") = "gfx950";
}
