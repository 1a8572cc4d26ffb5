// pdmb_bench — Python-free native executor of the benchmark (HIP + RCCL).
//
// The same workloads as matmul_scaling_benchmark.py (independent |
// batch_parallel | matrix_parallel, reference matmul_scaling_benchmark.py:
// 69-238, plus ring_parallel, models/ring_parallel.py) driven entirely from C++: one host thread per GPU in one process,
// RCCL communicators from ncclCommInitAll over xGMI, the gfx950 MFMA GEMM
// library of ops/csrc (pdmb::gemm), hipEvents for timing and, for --overlap,
// the schedule of parallel/overlap.py OverlapPipeline: whole GEMMs into a
// ring of outputs, each output's collective on a high-priority comm stream
// while the next GEMM runs, and with --chunks P > 1 the collective started
// piece by piece as the SAME launch's tiles finish (W4 completion signals,
// api.h pdmb::Signal; the rank's host thread waits for each piece's flag and
// issues its RCCL call at once). No PyTorch, no Python:
// useful to separate framework overhead from kernel/fabric behaviour and as a
// reference implementation of the scaling modes for MI355X nodes.
//
//   pdmb_bench --gpus 8 --mode batch_parallel --overlap --sizes 16384 --check
//
// Output: the reference's result lines (Results for NxN, Average time per
// operation, TFLOPS per GPU, Total system TFLOPS, Actual TFLOPS) and, with
// --json FILE, one JSON record per size.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../ops/csrc/api.h"

namespace {

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess)                                                                \
      throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_));          \
  } while (0)
#define NCCL_OK(x)                                                                       \
  do {                                                                                   \
    ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess)                                                               \
      throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_));         \
  } while (0)

enum Mode { kIndependent, kBatchParallel, kMatrixParallel, kRingParallel };

struct Opts {
  int gpus = 1;
  std::vector<int> sizes{4096, 8192, 16384};
  int iters = 50, warmup = 10;
  int dtype = 2;  // pdmb::DType: 0 f32, 1 f16, 2 bf16, 3 fp8 e4m3 (column-major B, bf16 C)
  Mode mode = kIndependent;
  int batch = 4, chunks = 1, kernel = 0;  // chunks: collective pieces per GEMM (signalled)
  bool overlap = false, check = false;
  bool direct = false;     // --allgather direct: P2P to every peer in one group (own link each)
  bool peer = false;       // --allgather ipc: pull every peer's block from its memory (DMA copies)
  bool direct_ar = false;  // --allreduce direct: two-shot P2P exchange + native reduce_sum
  bool peer_ar = false;    // --allreduce ipc: the two shots as pulls from the peers' memory
  std::string json;
};

const char* mode_name(Mode m) {
  return m == kIndependent      ? "independent"
         : m == kBatchParallel  ? "batch_parallel"
         : m == kMatrixParallel ? "matrix_parallel"
                                : "ring_parallel";
}
const char* dtype_name(int d) {
  return d == 0 ? "float32" : d == 1 ? "float16" : d == 2 ? "bfloat16" : "float8_e4m3fn";
}
// Operand and output element types: fp8 (3) multiplies e4m3 operands into a
// bf16 C (the library's kFP8 contract; B column-major, i.e. stored as Bt).
int out_dtype(int d) { return d == 3 ? 2 : d; }
size_t esize(int d) { return d == 0 ? 4 : d == 3 ? 1 : 2; }
size_t oesize(int d) { return esize(out_dtype(d)); }
ncclDataType_t nccl_type(int d) {
  return d == 0 ? ncclFloat32 : d == 1 ? ncclFloat16 : d == 2 ? ncclBfloat16 : ncclUint8;
}
ncclDataType_t nccl_out_type(int d) { return nccl_type(out_dtype(d)); }
int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// ---- device helpers -------------------------------------------------------
// OCP e4m3fn (gfx950's fp8): bias 7, no infinities, S.1111.111 = NaN.
__host__ __device__ __forceinline__ float e4m3_to_float(unsigned char b) {
  const int e = (b >> 3) & 15, m = b & 7;
  const float mag = e == 0 ? (float)m * 0.001953125f /* 2^-9 */
                           : (1.0f + (float)m * 0.125f) * (float)(1 << e) * 0.0078125f /* 2^-7 */;
  return (b & 0x80) ? -mag : mag;
}

__device__ __forceinline__ float to_float(const void* p, long long i, int dt) {
  if (dt == 0) return ((const float*)p)[i];
  if (dt == 3) return e4m3_to_float(((const unsigned char*)p)[i]);
  const unsigned short v = ((const unsigned short*)p)[i];
  if (dt == 2) return __uint_as_float(((unsigned int)v) << 16);
  return (float)__builtin_bit_cast(_Float16, v);
}

// Uniform [-1, 1) from a counter hash (random, non-zero data: zero-filled
// operands run ~20 % fast on MI355X through DVFS).
__global__ void fill_uniform(void* p, long long n, int dt, unsigned long long seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    unsigned long long x = (unsigned long long)i * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    const float u = (float)(x >> 40) * (1.0f / 8388608.0f) - 1.0f;  // 24 random bits
    if (dt == 3) {  // random e4m3 bits: sign, exponent 1..8 (|v| in [2^-6, 3.75]), mantissa
      const unsigned e = 1u + (unsigned)((x >> 40) & 7u), m = (unsigned)(x >> 44) & 7u;
      ((unsigned char*)p)[i] = (unsigned char)(((x >> 63) << 7) | (e << 3) | m);
      continue;
    }
    if (dt == 0) {
      ((float*)p)[i] = u;
    } else if (dt == 2) {
      __bf16 h = (__bf16)u;
      ((__bf16*)p)[i] = h;
    } else {
      ((_Float16*)p)[i] = (_Float16)u;
    }
  }
}

// out[r][j] = sum_k A[rows[r]][k] * B[k][j] in float64 (the check's reference).
__global__ void ref_rows(const void* A, const void* B, const int* rows, int R, int K, int N, int lda,
                         int ldb, int dt, double* out) {
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (idx >= (long long)R * N) return;
  const int r = (int)(idx / N), j = (int)(idx % N);
  double s = 0.0;
  const long long arow = (long long)rows[r] * lda;
  for (int k = 0; k < K; ++k) {
    const long long bi = dt == 3 ? (long long)j * ldb + k : (long long)k * ldb + j;  // fp8: Bt [N,K]
    s += (double)to_float(A, arow + k, dt) * (double)to_float(B, bi, dt);
  }
  out[idx] = s;
}

// Gather sampled rows of a [M, ld] matrix (N columns) into float64.
__global__ void take_rows(const void* C, const int* rows, int R, int N, int ld, int dt, double* out) {
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (idx >= (long long)R * N) return;
  const int r = (int)(idx / N), j = (int)(idx % N);
  out[idx] = (double)to_float(C, (long long)rows[r] * ld + j, dt);
}

// ---- host helpers ---------------------------------------------------------
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  // Throws if another rank aborted (so no rank waits forever on a dead peer).
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    if (aborted_) throw std::runtime_error("another rank failed");
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen != gen_ || aborted_; });
      if (aborted_) throw std::runtime_error("another rank failed");
    }
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m_);
    aborted_ = true;
    cv_.notify_all();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
  bool aborted_ = false;
};

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  Buf() = default;
  explicit Buf(size_t b) : bytes(b) { HIP_OK(hipMalloc(&p, b ? b : 16)); }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  Buf(Buf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; }
  Buf& operator=(Buf&& o) noexcept {
    if (this != &o) {
      if (p) (void)hipFree(p);
      p = o.p;
      bytes = o.bytes;
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

void fill(void* p, long long n, int dt, unsigned long long seed, hipStream_t s) {
  hipLaunchKernelGGL(fill_uniform, dim3(2048), dim3(256), 0, s, p, n, dt, seed);
  HIP_OK(hipGetLastError());
}

pdmb::Problem problem(int dt, const void* A, const void* B, void* C, int M, int N, int K, int lda,
                      int ldb, int ldc, int batch = 1, long long sA = 0, long long sB = 0,
                      long long sC = 0) {
  pdmb::Problem p{};
  p.dtype = dt;
  p.A = A;
  p.B = B;
  p.C = C;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.sA = sA;
  p.sB = sB;
  p.sC = sC;
  p.batch = batch;
  return p;
}

// Launch scratch (padded copies / split-K partials): one growing buffer per
// stream, owned by the rank that owns the streams (run_rank), so no two rank
// threads share the map and a buffer dies with its rank's streams. Growing
// waits for the stream first; it happens in warm-up only.
struct Scratch {
  std::map<hipStream_t, Buf> m;
  void* get(hipStream_t s, size_t bytes) {
    Buf& b = m[s];
    if (b.bytes < bytes) {
      HIP_OK(hipStreamSynchronize(s));
      b = Buf(bytes);
    }
    return b.p;
  }
};

// --overlap and ring_parallel run collectives beside the GEMMs: the planner
// then keeps to dispatch-balanced kernels (Problem::cus = -1: no persistent
// W4S, whose static tile assignment assumes every CU is its own).
static bool g_shared_device = false;

void gemm(const pdmb::Problem& p0, int kernel, hipStream_t s, Scratch& ws) {
  pdmb::Problem p = p0;
  if (g_shared_device && p.cus == 0) p.cus = -1;
  const size_t need = pdmb::gemm_workspace_bytes(p, kernel);
  if (need) {
    p.workspace = ws.get(s, need);
    p.workspace_bytes = need;
  }
  int used = -1;
  HIP_OK(pdmb::gemm(p, kernel, s, &used));
  if (used < 0) throw std::runtime_error("requested kernel cannot run this problem");
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

struct Result {
  double avg_ms = 0, comp_ms = 0, comm_ms = 0, flops_local = 0, flops_total = 0;
  std::string kernel, error;
  std::vector<double> ref;  // sampled-row float64 reference (this rank's part)
  std::vector<double> got;  // sampled-row output as computed/communicated on this rank
  int shard = 0, local_batch = 1, global_batch = 1, chunks = 1;
};

std::vector<int> sample_rows(int M, int R) {
  std::vector<int> rows;
  unsigned long long x = 0x1234567ull;
  for (int i = 0; i < std::min(M, R); ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    rows.push_back(M <= R ? i : (int)((x >> 33) % (unsigned long long)M));
  }
  return rows;
}

// Sampled rows of A@B (float64) and of C, both copied to the host.
void check_rows(int dt, const void* A, const void* B, const void* C, int M, int N, int K, int lda,
                int ldb, int ldc, hipStream_t s, std::vector<double>& ref, std::vector<double>& got) {
  const std::vector<int> rows = sample_rows(M, 32);
  const int R = (int)rows.size();
  Buf drows(R * sizeof(int)), dref((size_t)R * N * 8), dgot((size_t)R * N * 8);
  HIP_OK(hipMemcpyAsync(drows.p, rows.data(), R * sizeof(int), hipMemcpyHostToDevice, s));
  const long long tot = (long long)R * N;
  hipLaunchKernelGGL(ref_rows, dim3(ceil_div(tot, 256)), dim3(256), 0, s, A, B, drows.as<int>(), R,
                     K, N, lda, ldb, dt, dref.as<double>());
  hipLaunchKernelGGL(take_rows, dim3(ceil_div(tot, 256)), dim3(256), 0, s, C, drows.as<int>(), R, N,
                     ldc, out_dtype(dt), dgot.as<double>());
  HIP_OK(hipGetLastError());
  ref.resize(tot);
  got.resize(tot);
  HIP_OK(hipMemcpyAsync(ref.data(), dref.p, tot * 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(got.data(), dgot.p, tot * 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
}

// ---- the overlap pipeline (parallel/overlap.py OverlapPipeline) -------------
// A ring of R output buffers; unit k computes ring slot k % R on the compute
// stream `st` (one whole GEMM launch), and its rows go through `coll(r, r0,
// r1, piece)` on the comm stream `cs`. The next GEMM into a slot waits only
// for that slot's last collective. pieces > 1: the GEMM runs with completion
// signals and this host thread — after queueing the next unit's GEMM — waits
// for each piece's flag and issues that piece's collective at once.
struct Pipeline {
  struct Slot {
    pdmb::Problem p;
    pdmb::Signal* sig = nullptr;
    unsigned epoch = 0;
    hipEvent_t ready = nullptr, done = nullptr;
    bool used = false;
  };
  std::vector<Slot> slots;
  std::vector<std::pair<int, int>> pieces;  // row ranges [r0, r1)
  int sig_rows = 0, kernel = 0;
  long long k = 0;
  int pending = -1;
  hipStream_t st = nullptr, cs = nullptr;
  Scratch* ws = nullptr;
  std::function<void(int, int, int, int)> coll;

  void init(const std::vector<pdmb::Problem>& ring, int requested, int kern, hipStream_t s,
            hipStream_t c, Scratch& w, int device) {
    st = s;
    cs = c;
    ws = &w;
    kernel = kern;
    const int M = ring[0].M;
    pdmb::Problem q = ring[0];
    q.cus = -1;  // as issued beside collectives
    const int granule = requested > 1 ? pdmb::signal_granule(q, kern) : 0;
    const int tm = ceil_div(M, 256);
    if (granule > 0) {
      const int units = tm / granule;
      int P = 1;
      for (int c : {2, 4, 8})
        if (c <= requested && c <= units) P = c;
      if (P > 1) sig_rows = ceil_div(units, P) * granule;
    }
    const int step = sig_rows > 0 ? sig_rows * 256 : M;
    for (int r0 = 0; r0 < M; r0 += step) pieces.push_back({r0, std::min(M, r0 + step)});
    for (const auto& p : ring) {
      Slot sl;
      sl.p = p;
      HIP_OK(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
      if (sig_rows > 0) HIP_OK(pdmb::signal_create(device, (int)pieces.size(), &sl.sig));
      slots.push_back(sl);
    }
  }
  bool signalled() const { return sig_rows > 0; }
  void issue(int r) {
    Slot& sl = slots[r];
    for (size_t j = 0; j < pieces.size(); ++j) {
      if (signalled()) {
        if (!pdmb::signal_wait(sl.sig, (int)j, sl.epoch, 120.0))
          throw std::runtime_error("GEMM completion signal timed out");
      } else if (j == 0) {
        HIP_OK(hipStreamWaitEvent(cs, sl.ready, 0));
      }
      coll(r, pieces[j].first, pieces[j].second, (int)j);
    }
    HIP_OK(hipEventRecord(sl.done, cs));
    sl.used = true;
  }
  void step(int units) {
    for (int u = 0; u < units; ++u) {
      const int r = (int)(k++ % (long long)slots.size());
      Slot& sl = slots[r];
      if (sl.used) HIP_OK(hipStreamWaitEvent(st, sl.done, 0));  // WAR: the slot's collective is done
      pdmb::Problem p = sl.p;
      if (signalled()) {
        p.sig = sl.sig;
        p.sig_rows = sig_rows;
        p.sig_epoch = ++sl.epoch;
      }
      gemm(p, kernel, st, *ws);
      HIP_OK(hipEventRecord(sl.ready, st));
      if (signalled()) {
        if (pending >= 0) issue(pending);  // the next GEMM is queued before this thread blocks
        pending = r;
      } else {
        issue(r);
      }
    }
  }
  void finish() {
    if (pending >= 0) issue(pending);
    pending = -1;
    for (auto& sl : slots)
      if (sl.used) HIP_OK(hipStreamWaitEvent(st, sl.done, 0));
  }
  int last_slot() const { return (int)((k + (long long)slots.size() - 1) % (long long)slots.size()); }
  ~Pipeline() {
    for (auto& sl : slots) {
      if (sl.ready) (void)hipEventDestroy(sl.ready);
      if (sl.done) (void)hipEventDestroy(sl.done);
      pdmb::signal_destroy(sl.sig);
    }
  }
};

// ---- one rank ---------------------------------------------------------------
// Buffers a rank publishes to its peers (--allgather ipc): every rank thread of
// this process maps every GPU's memory directly (peer access), the
// single-process form of parallel/ipc.py's hipIpc mappings.
struct PeerTable {
  explicit PeerTable(int ws) : src(ws) {}
  std::vector<std::vector<char*>> src;  // [rank] -> its gather sources (ring slots)
};

void run_rank(int rank, const Opts& o, int n, ncclComm_t comm, Barrier& bar, Result& res,
              PeerTable& peers) {
  HIP_OK(hipSetDevice(rank));
  const int ws = o.gpus, dt = o.dtype;
  Scratch scr;  // this rank's launch scratch, freed with its streams
  const size_t es = esize(dt), oes = oesize(dt);  // operand / output element bytes
  hipStream_t st, cs;
  int lo = 0, hi = 0;
  HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithPriority(&cs, hipStreamNonBlocking, hi));
  std::vector<hipEvent_t> ev;
  auto event = [&]() {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    ev.push_back(e);
    return e;
  };
  const double flop = 2.0 * n * (double)n * n;
  // Collectives run at every world size (a 1-rank RCCL communicator still
  // executes the collective kernels), so the 1-GPU run exercises the same path.
  const bool dist = comm != nullptr;

  if (o.mode == kIndependent) {
    Buf A((size_t)n * n * es), B((size_t)n * n * es), C((size_t)n * n * oes);
    fill(A.p, (long long)n * n, dt, 2 * rank + 1, st);
    fill(B.p, (long long)n * n, dt, 2 * rank + 2, st);
    const pdmb::Problem p = problem(dt, A.p, B.p, C.p, n, n, n, n, n, n);
    res.kernel = pdmb::kernel_name(pdmb::resolve_kernel(p, o.kernel));
    for (int i = 0; i < o.warmup; ++i) gemm(p, o.kernel, st, scr);
    HIP_OK(hipStreamSynchronize(st));
    bar.wait();
    hipEvent_t e0 = event(), e1 = event();
    HIP_OK(hipEventRecord(e0, st));
    for (int i = 0; i < o.iters; ++i) gemm(p, o.kernel, st, scr);
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipEventSynchronize(e1));
    res.avg_ms = res.comp_ms = elapsed(e0, e1) / std::max(o.iters, 1);
    res.flops_local = flop;
    res.flops_total = o.mode == kIndependent ? flop * ws : flop;
    if (o.check) check_rows(dt, A.p, B.p, C.p, n, n, n, n, n, n, st, res.ref, res.got);
  } else if (o.mode == kBatchParallel) {
    const int gb = std::max(ceil_div(std::max(o.batch, 1), ws) * ws, ws), lb = gb / ws;
    res.local_batch = lb;
    res.global_batch = gb;
    const size_t mat = (size_t)n * n;
    Buf A(lb * mat * es), B(lb * mat * es), C(lb * mat * oes);
    fill(A.p, (long long)(lb * mat), dt, 2 * rank + 1, st);
    fill(B.p, (long long)(lb * mat), dt, 2 * rank + 2, st);
    const pdmb::Problem p = problem(dt, A.p, B.p, C.p, n, n, n, n, n, n, lb, mat, mat, mat);
    res.kernel = pdmb::kernel_name(pdmb::resolve_kernel(p, o.kernel));
    const bool ov = o.overlap && dist;
    // overlap ring: the batch's own outputs (lb >= 2) or C plus a second buffer (C1/C2)
    Buf C2(ov && lb == 1 ? mat * oes : 0);
    // SUM all-reduce of `count` output elements in place: RCCL, or --allreduce
    // direct (parallel/comm.py all_reduce_direct): chunk p goes straight to
    // rank p and the peers' copies of this rank's chunk land in scratch (one
    // group), reduce_sum adds the ws copies in rank order in fp32 into the
    // chunk, then the reduced chunk goes to every peer (a second group). Every
    // transfer of a group has its own xGMI link on a fully connected node.
    auto ar_chunk = [&](size_t count) { return ((count + ws - 1) / ws + 63) / 64 * 64; };  // 16-B aligned chunks
    const size_t ar_chunk_max = ar_chunk(lb * mat);
    // landing slots for the direct exchange only (the ipc form sums in place)
    Buf ARs(o.direct_ar && ws > 1 ? (size_t)(ws - 1) * ar_chunk_max * oes : 0);
    // --allreduce ipc (parallel/ipc.py IpcGather.all_reduce, kernel engine):
    // the same two shots read straight out of the peers' C / C2 (direct peer
    // access between this process's GPUs) from the comm stream — the chunk's
    // sum reads every rank's copy in place (reduce_sum over peer addresses),
    // the reduced chunks come back in one multi_copy launch — with three
    // one-element all-reduces as stream-ordered barriers (outputs final;
    // chunks reduced; nobody still reading this rank's chunk). No copy streams.
    Buf arflag(o.peer_ar ? 256 : 0);
    peers.src[rank] = {(char*)C.p, (char*)C2.p};
    if (o.peer_ar && ws > 1) {
      for (int d = 0; d < ws; ++d) {
        if (d == rank) continue;
        int can = 0;
        HIP_OK(hipDeviceCanAccessPeer(&can, rank, d));
        if (!can) throw std::runtime_error("--allreduce ipc: no peer access between GPUs");
        const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_OK(e);
        (void)hipGetLastError();
      }
      HIP_OK(hipMemsetAsync(arflag.p, 0, arflag.bytes, st));
    }
    bar.wait();  // every rank's buffers published before anyone pulls
    auto peer_allreduce = [&](void* buf, size_t count, hipStream_t s) {
      const size_t chunk = ar_chunk(count);
      auto lo_of = [&](int r) { return std::min(count, (size_t)r * chunk); };
      auto len_of = [&](int r) { return std::min(count, (size_t)(r + 1) * chunk) - lo_of(r); };
      char* b = (char*)buf;
      const int sid = (b >= (char*)C.p && b < (char*)C.p + C.bytes) ? 0 : 1;
      const size_t off = (size_t)(b - (sid ? (char*)C2.p : (char*)C.p));
      const size_t m = len_of(rank);
      auto barrier = [&]() { NCCL_OK(ncclAllReduce(arflag.p, arflag.p, 1, ncclFloat, ncclSum, comm, s)); };
      barrier();  // B0: every rank's output final
      if (m) {
        std::vector<const void*> srcs(ws);
        for (int r = 0; r < ws; ++r) srcs[r] = peers.src[r][sid] + off + lo_of(rank) * oes;
        HIP_OK(pdmb::reduce_sum(b + lo_of(rank) * oes, srcs.data(), ws, (int64_t)m, out_dtype(dt), s));
      }
      barrier();  // B1: every chunk reduced
      std::vector<void*> dsts;
      std::vector<const void*> srcs;
      std::vector<size_t> lens;
      for (int d = 1; d < ws; ++d) {
        const int from = (rank + d) % ws;
        dsts.push_back(b + lo_of(from) * oes);
        srcs.push_back(peers.src[from][sid] + off + lo_of(from) * oes);
        lens.push_back(len_of(from) * oes);
      }
      HIP_OK(pdmb::multi_copy(dsts.data(), srcs.data(), lens.data(), (int)dsts.size(), 0, s));
      barrier();  // B2: no peer still reads this rank's chunk
    };
    auto allreduce = [&](void* buf, size_t count, hipStream_t s) {
      if (o.peer_ar) {
        if (ws > 1 && count) peer_allreduce(buf, count, s);
        return;
      }
      if (!o.direct_ar) {
        NCCL_OK(ncclAllReduce(buf, buf, count, nccl_out_type(dt), ncclSum, comm, s));
        return;
      }
      if (ws == 1 || count == 0) return;
      const size_t chunk = ar_chunk(count);
      auto lo_of = [&](int r) { return std::min(count, (size_t)r * chunk); };
      auto len_of = [&](int r) { return std::min(count, (size_t)(r + 1) * chunk) - lo_of(r); };
      char* base = (char*)buf;
      const size_t m = len_of(rank);
      auto slot = [&](int d) { return (char*)ARs.p + (size_t)(d - 1) * chunk * oes; };  // from rank - d
      NCCL_OK(ncclGroupStart());
      for (int d = 1; d < ws; ++d) {
        const int to = (rank + d) % ws, from = (rank - d + ws) % ws;
        if (len_of(to)) NCCL_OK(ncclSend(base + lo_of(to) * oes, len_of(to), nccl_out_type(dt), to, comm, s));
        if (m) NCCL_OK(ncclRecv(slot(d), m, nccl_out_type(dt), from, comm, s));
      }
      NCCL_OK(ncclGroupEnd());
      if (m) {
        std::vector<const void*> srcs(ws);
        for (int r = 0; r < ws; ++r)
          srcs[r] = r == rank ? (const void*)(base + lo_of(rank) * oes) : (const void*)slot((rank - r + ws) % ws);
        HIP_OK(pdmb::reduce_sum(base + lo_of(rank) * oes, srcs.data(), ws, (int64_t)m, out_dtype(dt), s));
      }
      NCCL_OK(ncclGroupStart());
      for (int d = 1; d < ws; ++d) {
        const int to = (rank + d) % ws, from = (rank - d + ws) % ws;
        if (m) NCCL_OK(ncclSend(base + lo_of(rank) * oes, m, nccl_out_type(dt), to, comm, s));
        if (len_of(from)) NCCL_OK(ncclRecv(base + lo_of(from) * oes, len_of(from), nccl_out_type(dt), from, comm, s));
      }
      NCCL_OK(ncclGroupEnd());
    };
    Pipeline pipe;
    if (ov) {
      std::vector<pdmb::Problem> ring;
      for (int b = 0; b < lb; ++b)
        ring.push_back(problem(dt, (char*)A.p + b * mat * es, (char*)B.p + b * mat * es,
                               (char*)C.p + b * mat * oes, n, n, n, n, n, n));
      if (lb == 1) ring.push_back(problem(dt, A.p, B.p, C2.p, n, n, n, n, n, n));
      pipe.coll = [&](int r, int r0, int r1, int) {
        char* c = (char*)pipe.slots[r].p.C + (size_t)r0 * n * oes;
        allreduce(c, (size_t)(r1 - r0) * n, cs);
      };
      pipe.init(ring, o.chunks, o.kernel, st, cs, scr, rank);
      res.chunks = (int)pipe.pieces.size();
    }
    auto serial_iter = [&](hipEvent_t em) {
      gemm(p, o.kernel, st, scr);
      if (em) HIP_OK(hipEventRecord(em, st));
      if (dist) allreduce(C.p, lb * mat, st);
    };
    for (int i = 0; i < o.warmup; ++i) {
      if (ov) {
        pipe.step(lb);
        pipe.finish();
      } else {
        serial_iter(nullptr);
      }
    }
    HIP_OK(hipStreamSynchronize(st));
    // compute-only reference time (into a scratch output: the ring keeps its reduced values)
    {
      Buf Cs(mat * oes);
      hipEvent_t c0 = event(), c1 = event();
      HIP_OK(hipEventRecord(c0, st));
      for (int i = 0; i < std::min(o.iters, 10); ++i)
        for (int b = 0; b < lb; ++b)
          gemm(problem(dt, (char*)A.p + b * mat * es, (char*)B.p + b * mat * es, Cs.p, n, n, n, n, n, n),
               o.kernel, st, scr);
      HIP_OK(hipEventRecord(c1, st));
      HIP_OK(hipEventSynchronize(c1));
      res.comp_ms = elapsed(c0, c1) / std::max(1, std::min(o.iters, 10));
    }
    bar.wait();
    if (ov) {
      hipEvent_t e0 = event(), e1 = event();
      HIP_OK(hipEventRecord(e0, st));
      for (int i = 0; i < o.iters; ++i) pipe.step(lb);
      pipe.finish();
      HIP_OK(hipEventRecord(e1, st));
      HIP_OK(hipEventSynchronize(e1));
      res.avg_ms = elapsed(e0, e1) / std::max(o.iters, 1);
      res.comm_ms = std::max(0.0, res.avg_ms - res.comp_ms);
    } else {
      std::vector<hipEvent_t> marks;
      for (int i = 0; i <= o.iters; ++i) marks.push_back(event());
      std::vector<hipEvent_t> mids;
      for (int i = 0; i < o.iters; ++i) mids.push_back(event());
      HIP_OK(hipEventRecord(marks[0], st));
      for (int i = 0; i < o.iters; ++i) {
        serial_iter(mids[i]);
        HIP_OK(hipEventRecord(marks[i + 1], st));
      }
      HIP_OK(hipEventSynchronize(marks[o.iters]));
      double comp = 0, cm = 0;
      for (int i = 0; i < o.iters; ++i) {
        comp += elapsed(marks[i], mids[i]);
        cm += elapsed(mids[i], marks[i + 1]);
      }
      const int it = std::max(o.iters, 1);
      res.comp_ms = comp / it;
      res.comm_ms = cm / it;
      res.avg_ms = res.comp_ms + res.comm_ms;
    }
    res.flops_local = flop * lb;
    res.flops_total = flop * gb;
    if (o.check)  // C[0] = sum over ranks of A_r[0] @ B_r[0]: partial refs are summed on the host
      check_rows(dt, A.p, B.p, ov && lb == 1 ? pipe.slots[pipe.last_slot()].p.C : C.p, n, n, n, n, n,
                 n, st, res.ref, res.got);
  } else if (o.mode == kRingParallel) {
    // All-gather-GEMM over BOTH ring directions (models/ring_parallel.py): A
    // row-sharded in blocks of rp rows, B column-sharded. Each block is cut
    // into a top (ht rows, 256-aligned) and a bottom half; tops travel r -> r+1,
    // bottoms r -> r-1, so every hop drives the links to both neighbours. Hop s
    // multiplies the top of rank (r - s)'s block and the bottom of rank
    // (r + s)'s block while the comm stream moves the next two halves (two
    // ncclSend + two ncclRecv in one group).
    const int shard = ceil_div(ceil_div(n, ws), 8) * 8;
    const int c0 = std::min(rank * shard, n), width = std::max(0, std::min(n, c0 + shard) - c0);
    const int rp = ceil_div(n, ws);
    const int ht = std::min(rp, ceil_div(ceil_div(rp, 2), 256) * 256), hb = rp - ht;
    auto rows_of = [&](int j) { return std::max(0, std::min(n, (j + 1) * rp) - j * rp); };
    res.shard = shard;
    const size_t blk = (size_t)rp * n, blt = (size_t)ht * n, blb = (size_t)hb * n;
    Buf Ag((size_t)n * n * es), Bg((size_t)n * n * es), Bl((size_t)n * shard * es);
    Buf Cl((size_t)n * shard * oes), Al(blk * es), Rt0(blt * es), Rt1(blt * es), Rb0(blb * es),
        Rb1(blb * es);
    fill(Ag.p, (long long)n * n, dt, 1000, st);
    fill(Bg.p, (long long)n * n, dt, 1001, st);
    HIP_OK(hipMemsetAsync(Bl.p, 0, Bl.bytes, st));
    const int ldb = dt == 3 ? n : shard;  // fp8: B column-major, its column shard a row range of Bt
    if (width && dt == 3)
      HIP_OK(hipMemcpyAsync(Bl.p, (char*)Bg.p + (size_t)c0 * n, (size_t)width * n, hipMemcpyDeviceToDevice, st));
    else if (width)
      HIP_OK(hipMemcpy2DAsync(Bl.p, shard * es, (char*)Bg.p + c0 * es, n * es, width * es, n,
                              hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemsetAsync(Al.p, 0, Al.bytes, st));
    if (rows_of(rank))
      HIP_OK(hipMemcpyAsync(Al.p, (char*)Ag.p + (size_t)rank * rp * n * es,
                            (size_t)rows_of(rank) * n * es, hipMemcpyDeviceToDevice, st));
    res.kernel = pdmb::kernel_name(
        pdmb::resolve_kernel(problem(dt, Al.p, Bl.p, Cl.p, ht, shard, n, n, ldb, shard), o.kernel));
    char* Rt[2] = {(char*)Rt0.p, (char*)Rt1.p};
    char* Rb[2] = {(char*)Rb0.p, (char*)Rb1.p};
    std::vector<hipEvent_t> gdone, rdone;
    for (int s = 0; s < ws; ++s) gdone.push_back(event());
    for (int s = 0; s + 1 < ws; ++s) rdone.push_back(event());
    hipEvent_t last = nullptr;  // most recently issued GEMM (across iterations)
    // rows [r0, r1) of block j (held in `a` from its row r0) -> C rows j*rp + r0 ..
    auto part_gemm = [&](const char* a, int j, int r0, int r1) {
      r1 = std::min(r1, rows_of(j));
      if (r1 > r0)
        gemm(problem(dt, a, Bl.p, (char*)Cl.p + ((size_t)j * rp + r0) * shard * oes, r1 - r0, shard,
                     n, n, ldb, shard),
             o.kernel, st, scr);
    };
    auto block_gemm = [&](const char* a, int j) { part_gemm(a, j, 0, rp); };
    auto iter = [&]() {
      char* top = (char*)Al.p;
      char* bot = (char*)Al.p + blt * es;
      for (int s = 0; s < ws; ++s) {
        if (s > 0) HIP_OK(hipStreamWaitEvent(st, rdone[s - 1], 0));
        char* nt = Rt[(s + 1) % 2];
        char* nb = Rb[(s + 1) % 2];
        if (s + 1 < ws) {
          if (last) HIP_OK(hipStreamWaitEvent(cs, last, 0));  // nt / nb's last readers are done
          NCCL_OK(ncclGroupStart());
          NCCL_OK(ncclSend(top, blt, nccl_type(dt), (rank + 1) % ws, comm, cs));
          NCCL_OK(ncclRecv(nt, blt, nccl_type(dt), (rank + ws - 1) % ws, comm, cs));
          if (blb) {
            NCCL_OK(ncclSend(bot, blb, nccl_type(dt), (rank + ws - 1) % ws, comm, cs));
            NCCL_OK(ncclRecv(nb, blb, nccl_type(dt), (rank + 1) % ws, comm, cs));
          }
          NCCL_OK(ncclGroupEnd());
          HIP_OK(hipEventRecord(rdone[s], cs));
        }
        part_gemm(top, (rank - s + ws) % ws, 0, ht);
        part_gemm(bot, (rank + s) % ws, ht, rp);  // bot holds the block's rows ht .. rp
        HIP_OK(hipEventRecord(gdone[s], st));
        last = gdone[s];
        top = nt;
        bot = nb;
      }
    };
    for (int i = 0; i < o.warmup; ++i) iter();
    HIP_OK(hipStreamSynchronize(st));
    {
      hipEvent_t q0 = event(), q1 = event();
      const int k = std::max(1, std::min(o.iters, 10));
      HIP_OK(hipEventRecord(q0, st));
      for (int i = 0; i < k; ++i)
        for (int j = 0; j < ws; ++j) block_gemm((const char*)Al.p, j);
      HIP_OK(hipEventRecord(q1, st));
      HIP_OK(hipEventSynchronize(q1));
      res.comp_ms = elapsed(q0, q1) / k;
    }
    bar.wait();
    hipEvent_t m0 = event(), m1 = event();
    HIP_OK(hipEventRecord(m0, st));
    for (int i = 0; i < o.iters; ++i) iter();
    HIP_OK(hipEventRecord(m1, st));
    HIP_OK(hipEventSynchronize(m1));
    HIP_OK(hipStreamSynchronize(cs));
    res.avg_ms = elapsed(m0, m1) / std::max(o.iters, 1);
    res.comm_ms = std::max(0.0, res.avg_ms - res.comp_ms);
    res.flops_local = 2.0 * n * (double)shard * n;
    res.flops_total = flop;
    // Cl is C[:, S_r] exactly (blocks are contiguous, unpadded): sampled rows vs A @ B_local.
    if (o.check) check_rows(dt, Ag.p, Bl.p, Cl.p, n, shard, n, n, ldb, shard, st, res.ref, res.got);
  } else {  // matrix_parallel: replicated A, padded column shard of one global B
    const int shard = ceil_div(ceil_div(n, ws), 8) * 8;
    const int c0 = std::min(rank * shard, n), width = std::max(0, std::min(n, c0 + shard) - c0);
    res.shard = shard;
    Buf A((size_t)n * n * es), Bg((size_t)n * n * es), Bl((size_t)n * shard * es);
    Buf Cl((size_t)n * shard * oes), G((size_t)ws * n * shard * oes);
    fill(A.p, (long long)n * n, dt, 1000, st);
    fill(Bg.p, (long long)n * n, dt, 1001, st);
    HIP_OK(hipMemsetAsync(Bl.p, 0, Bl.bytes, st));
    // fp8: B is column-major (Bt [N,K]), so a column shard is a row range of Bt
    const int ldb = dt == 3 ? n : shard;
    if (width && dt == 3)
      HIP_OK(hipMemcpyAsync(Bl.p, (char*)Bg.p + (size_t)c0 * n, (size_t)width * n, hipMemcpyDeviceToDevice, st));
    else if (width)
      HIP_OK(hipMemcpy2DAsync(Bl.p, shard * es, (char*)Bg.p + c0 * es, n * es, width * es, n,
                              hipMemcpyDeviceToDevice, st));
    const pdmb::Problem p = problem(dt, A.p, Bl.p, Cl.p, n, shard, n, n, ldb, shard);
    res.kernel = pdmb::kernel_name(pdmb::resolve_kernel(p, o.kernel));
    // All-gather `count` elements per rank from `send` into `recv` (rank-major):
    // RCCL's ring/channel algorithm, or --allgather direct: this rank's block
    // sent straight to every peer and every peer's block received straight
    // into its slot, all in one group (on a fully connected node each
    // transfer has its own xGMI link; no forwarding hops).
    // overlap: a ring of two C_local / gather buffer pairs (gather per piece: [ws * rows, shard])
    Buf Cl2(o.overlap ? Cl.bytes : 0), G2(o.overlap ? G.bytes : 0);
    peers.src[rank] = {(char*)Cl.p, (char*)Cl2.p};
    bar.wait();  // every rank's buffers published before anyone pulls
    // --allgather ipc (parallel/ipc.py IpcGather.all_gather, kernel engine):
    // a one-element all-reduce as a stream-ordered barrier (every peer's block
    // final), then every peer's block (same offset in ITS buffer) and the
    // local one in ONE multi_copy launch — every xGMI link read at once from
    // the comm stream, no copy streams — then a second barrier: once it
    // completes every peer has finished reading this rank's block.
    Buf flag(o.peer ? 256 : 0);
    if (o.peer && ws > 1) {
      for (int d = 0; d < ws; ++d) {
        if (d == rank) continue;
        int can = 0;
        HIP_OK(hipDeviceCanAccessPeer(&can, rank, d));
        if (!can) throw std::runtime_error("--allgather ipc: no peer access between GPUs");
        const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_OK(e);
        (void)hipGetLastError();
      }
      HIP_OK(hipMemsetAsync(flag.p, 0, flag.bytes, st));
    }
    auto pull_gather = [&](const char* send, char* recv, size_t count, hipStream_t s) {
      const size_t bytes = count * oes;
      char* base = o.overlap ? (send >= (char*)Cl2.p && send < (char*)Cl2.p + Cl2.bytes ? (char*)Cl2.p
                                                                                        : (char*)Cl.p)
                             : (char*)Cl.p;
      const int slot = base == (char*)Cl.p ? 0 : 1;
      const size_t off = (size_t)(send - base);
      NCCL_OK(ncclAllReduce(flag.p, flag.p, 1, ncclFloat, ncclSum, comm, s));  // B0: blocks final
      std::vector<void*> dsts;
      std::vector<const void*> srcs;
      std::vector<size_t> lens;
      for (int d = 0; d < ws; ++d) {
        const int from = (rank + d) % ws;
        dsts.push_back(recv + (size_t)from * bytes);
        srcs.push_back(d == 0 ? (const void*)send : (const void*)(peers.src[from][slot] + off));
        lens.push_back(bytes);
      }
      HIP_OK(pdmb::multi_copy(dsts.data(), srcs.data(), lens.data(), (int)dsts.size(), 0, s));
      NCCL_OK(ncclAllReduce(flag.p, flag.p, 1, ncclFloat, ncclSum, comm, s));  // B1: reads done
    };
    auto allgather = [&](const void* send, char* recv, size_t count, hipStream_t s) {
      if (o.peer && ws > 1) {
        pull_gather((const char*)send, recv, count, s);
        return;
      }
      if (!o.direct) {
        NCCL_OK(ncclAllGather(send, recv, count, nccl_out_type(dt), comm, s));
        return;
      }
      const size_t bytes = count * oes;
      HIP_OK(hipMemcpyAsync(recv + (size_t)rank * bytes, send, bytes, hipMemcpyDeviceToDevice, s));
      NCCL_OK(ncclGroupStart());
      for (int d = 1; d < ws; ++d) {
        const int to = (rank + d) % ws, from = (rank - d + ws) % ws;
        NCCL_OK(ncclSend(send, count, nccl_out_type(dt), to, comm, s));
        NCCL_OK(ncclRecv(recv + (size_t)from * bytes, count, nccl_out_type(dt), from, comm, s));
      }
      NCCL_OK(ncclGroupEnd());
    };
    Pipeline pipe;
    std::vector<std::vector<char*>> gbuf;  // [slot][piece]
    if (o.overlap) {
      pipe.init({p, problem(dt, A.p, Bl.p, Cl2.p, n, shard, n, n, ldb, shard)}, o.chunks, o.kernel, st,
                cs, scr, rank);
      for (int r = 0; r < 2; ++r) {
        std::vector<char*> v;
        size_t off = 0;
        for (auto pc : pipe.pieces) {
          v.push_back((char*)(r ? G2.p : G.p) + off);
          off += (size_t)ws * (pc.second - pc.first) * shard * oes;
        }
        gbuf.push_back(v);
      }
      pipe.coll = [&](int r, int r0, int r1, int j) {
        allgather((char*)pipe.slots[r].p.C + (size_t)r0 * shard * oes, gbuf[r][j],
                  (size_t)(r1 - r0) * shard, cs);
      };
      res.chunks = (int)pipe.pieces.size();
    }
    auto iter = [&](hipEvent_t em) {
      if (!o.overlap) {
        gemm(p, o.kernel, st, scr);
        if (em) HIP_OK(hipEventRecord(em, st));
        allgather(Cl.p, (char*)G.p, (size_t)n * shard, st);
        return;
      }
      pipe.step(1);
    };
    for (int i = 0; i < o.warmup; ++i) {
      iter(nullptr);
      if (o.overlap) pipe.finish();
    }
    HIP_OK(hipStreamSynchronize(st));
    {
      // compute-only time; overlap: into the slot the timed loop's last unit will NOT gather
      const pdmb::Problem pc = o.overlap ? pipe.slots[(pipe.k + o.iters) % 2].p : p;
      hipEvent_t q0 = event(), q1 = event();
      HIP_OK(hipEventRecord(q0, st));
      for (int i = 0; i < std::min(o.iters, 10); ++i) gemm(pc, o.kernel, st, scr);
      HIP_OK(hipEventRecord(q1, st));
      HIP_OK(hipEventSynchronize(q1));
      res.comp_ms = elapsed(q0, q1) / std::max(1, std::min(o.iters, 10));
    }
    bar.wait();
    std::vector<hipEvent_t> marks, mids;
    for (int i = 0; i <= o.iters; ++i) marks.push_back(event());
    for (int i = 0; i < o.iters; ++i) mids.push_back(event());
    HIP_OK(hipEventRecord(marks[0], st));
    for (int i = 0; i < o.iters; ++i) {
      iter(o.overlap ? nullptr : mids[i]);
      if (o.overlap && i + 1 == o.iters) pipe.finish();  // the last gathers are in the time
      HIP_OK(hipEventRecord(marks[i + 1], st));
    }
    HIP_OK(hipEventSynchronize(marks[o.iters]));
    const int it = std::max(o.iters, 1);
    res.avg_ms = elapsed(marks[0], marks[o.iters]) / it;
    if (!o.overlap) {
      double comp = 0;
      for (int i = 0; i < o.iters; ++i) comp += elapsed(marks[i], mids[i]);
      res.comp_ms = comp / it;
    }
    res.comm_ms = std::max(0.0, res.avg_ms - res.comp_ms);
    res.flops_local = 2.0 * n * (double)shard * n;
    res.flops_total = flop;
    if (o.check) {
      // This rank's reference: sampled rows of A @ B_local (its shard). The
      // gathered rows of EVERY shard as seen on this rank go to `got`
      // ([ws][rows][shard] order); the host matches got(0)[r] with ref(r).
      std::vector<double> own;
      check_rows(dt, A.p, Bl.p, Cl.p, n, shard, n, n, ldb, shard, st, res.ref, own);
      const std::vector<int> rows = sample_rows(n, 32);
      std::vector<unsigned short> h16;
      std::vector<float> h32;
      res.got.clear();
      const int last = o.overlap ? pipe.last_slot() : 0;
      for (int r = 0; r < ws; ++r)
        for (int row : rows) {
          const char* base = (char*)G.p + ((size_t)r * n + row) * shard * oes;
          if (o.overlap) {
            size_t j = 0;
            while (j + 1 < pipe.pieces.size() && row >= pipe.pieces[j].second) ++j;
            const int r0 = pipe.pieces[j].first, rows_j = pipe.pieces[j].second - r0;
            base = gbuf[last][j] + ((size_t)r * rows_j + (row - r0)) * shard * oes;
          }
          if (dt == 0) {
            h32.resize(shard);
            HIP_OK(hipMemcpy(h32.data(), base, shard * 4, hipMemcpyDeviceToHost));
            for (float v : h32) res.got.push_back(v);
          } else {
            h16.resize(shard);
            HIP_OK(hipMemcpy(h16.data(), base, shard * 2, hipMemcpyDeviceToHost));
            for (unsigned short v : h16) {
              float f;
              if (out_dtype(dt) == 2) {
                unsigned int u = (unsigned int)v << 16;
                std::memcpy(&f, &u, 4);
              } else {
                f = (float)__builtin_bit_cast(_Float16, v);
              }
              res.got.push_back(f);
            }
          }
        }
    }
  }
  HIP_OK(hipDeviceSynchronize());
  bar.wait();  // no rank frees a buffer a peer may still read (--allgather ipc)
  for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(st);
  (void)hipStreamDestroy(cs);
}

double norm_relerr(const std::vector<double>& got, const std::vector<double>& ref) {
  double num = 0, den = 0;
  for (size_t i = 0; i < ref.size() && i < got.size(); ++i) {
    num += (got[i] - ref[i]) * (got[i] - ref[i]);
    den += ref[i] * ref[i];
  }
  return std::sqrt(num / std::max(den, 1e-300));
}

void usage() {
  std::printf(
      "pdmb_bench [--gpus N] [--sizes N ...] [--iterations I] [--warmup W]\n"
      "           [--dtype bfloat16|float16|float32|float8_e4m3fn] [--mode independent|batch_parallel|matrix_parallel|ring_parallel]\n"
      "           [--batch B] [--overlap] [--chunks C] [--allgather rccl|direct|ipc] [--allreduce rccl|direct|ipc]\n"
      "           [--kernel ID]\n"
      "           [--check] [--json FILE]\n");
}

Opts parse(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
      return argv[++i];
    };
    if (a == "--gpus") o.gpus = std::stoi(next());
    else if (a == "--iterations") o.iters = std::stoi(next());
    else if (a == "--warmup") o.warmup = std::stoi(next());
    else if (a == "--batch") o.batch = std::stoi(next());
    else if (a == "--chunks") o.chunks = std::stoi(next());
    else if (a == "--kernel") o.kernel = std::stoi(next());
    else if (a == "--overlap") o.overlap = true;
    else if (a == "--allgather") {
      const std::string g = next();
      o.direct = g == "direct";
      o.peer = g == "ipc";
    }
    else if (a == "--allreduce") {
      const std::string r = next();
      o.direct_ar = r == "direct";
      o.peer_ar = r == "ipc";
    }
    else if (a == "--check") o.check = true;
    else if (a == "--json") o.json = next();
    else if (a == "--dtype") {
      const std::string d = next();
      o.dtype = d == "float32" ? 0 : d == "float16" ? 1 : d == "bfloat16" ? 2 : d == "float8_e4m3fn" ? 3 : -1;
      if (o.dtype < 0) throw std::runtime_error("bad --dtype " + d);
    } else if (a == "--mode") {
      const std::string m = next();
      if (m == "independent") o.mode = kIndependent;
      else if (m == "batch_parallel") o.mode = kBatchParallel;
      else if (m == "matrix_parallel") o.mode = kMatrixParallel;
      else if (m == "ring_parallel") o.mode = kRingParallel;
      else throw std::runtime_error("bad --mode " + m);
    } else if (a == "--sizes") {
      o.sizes.clear();
      while (i + 1 < argc && argv[i + 1][0] != '-') o.sizes.push_back(std::stoi(argv[++i]));
    } else if (a == "-h" || a == "--help") {
      usage();
      std::exit(0);
    } else {
      throw std::runtime_error("unknown argument " + a);
    }
  }
  return o;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  try {
    o = parse(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    usage();
    return 2;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < o.gpus || o.gpus < 1) {
    std::fprintf(stderr, "error: %d GPU(s) requested, %d visible\n", o.gpus, ndev);
    return 2;
  }
  g_shared_device = o.overlap || o.mode == kRingParallel;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  std::printf("pdmb_bench (native HIP + RCCL executor)\n  GPU 0: %s (%s), %d CUs\n", prop.name,
              prop.gcnArchName, prop.multiProcessorCount);
  std::printf("  Mode: %s%s, GPUs: %d, dtype: %s, iterations: %d, warmup: %d\n", mode_name(o.mode),
              o.overlap ? " (overlap)" : "", o.gpus, dtype_name(o.dtype), o.iters, o.warmup);
  std::vector<ncclComm_t> comms(o.gpus, nullptr);
  if (o.mode != kIndependent) {
    std::vector<int> devs(o.gpus);
    for (int i = 0; i < o.gpus; ++i) devs[i] = i;
    try {
      NCCL_OK(ncclCommInitAll(comms.data(), o.gpus, devs.data()));
    } catch (const std::exception& e) {
      std::fprintf(stderr, "error: %s\n", e.what());
      return 1;
    }
  }
  FILE* js = o.json.empty() ? nullptr : std::fopen(o.json.c_str(), "a");
  int failures = 0;
  for (int n : o.sizes) {
    std::printf("\nBenchmarking %dx%d matrix multiplication:\n", n, n);
    std::vector<Result> res(o.gpus);
    Barrier bar(o.gpus);
    PeerTable peers(o.gpus);
    std::vector<std::thread> th;
    for (int r = 0; r < o.gpus; ++r)
      th.emplace_back([&, r] {
        try {
          run_rank(r, o, n, comms[r], bar, res[r], peers);
        } catch (const std::exception& e) {
          res[r].error = e.what();
          bar.abort();
        }
      });
    for (auto& t : th) t.join();
    std::string err;
    for (auto& r : res)
      if (!r.error.empty()) err = r.error;
    if (!err.empty()) {
      std::printf("\n  ERROR: %s\n", err.c_str());
      ++failures;
      continue;  // (a failed rank may leave peers' collectives pending; abort the sweep)
    }
    double avg = 0, mx = 0, comp = 0, cm = 0;
    for (auto& r : res) {
      avg += r.avg_ms / o.gpus;
      mx = std::max(mx, r.avg_ms);
      comp += r.comp_ms / o.gpus;
      cm += r.comm_ms / o.gpus;
    }
    const Result& r0 = res[0];
    const double per_gpu = r0.flops_local / (r0.avg_ms * 1e-3) / 1e12;
    const double node = r0.flops_total / (mx * 1e-3) / 1e12;
    const double actual = r0.flops_total / (avg * 1e-3) / 1e12;
    std::printf("\nResults for %dx%d:\n", n, n);
    std::printf("  - Average time per operation: %.3f ms\n", avg);
    if (o.mode != kIndependent)
      std::printf("  - Compute time: %.3f ms, Comm time: %.3f ms%s\n", comp, cm,
                  o.overlap ? " (overlapped; comm = exposed part)" : "");
    std::printf("  - TFLOPS per GPU: %.2f\n", per_gpu);
    if (o.mode == kBatchParallel)
      std::printf("  - Processing %d total batches across %d GPU(s) (%d per GPU)\n", r0.global_batch,
                  o.gpus, r0.local_batch);
    const bool sharded = o.mode == kMatrixParallel || o.mode == kRingParallel;
    std::printf("  - Total system TFLOPS: %.2f\n", sharded ? actual : per_gpu * o.gpus);
    std::printf("  - Actual TFLOPS (total FLOPs / time): %.2f\n", actual);
    std::printf("  - Node TFLOPS (all FLOPs / slowest rank): %.2f\n", node);
    std::printf("  - Kernel: %s\n", r0.kernel.c_str());
    double relerr = -1;
    if (o.check) {
      if (o.mode == kBatchParallel) {
        std::vector<double> sum(r0.ref.size(), 0.0);
        for (auto& r : res)
          for (size_t i = 0; i < sum.size(); ++i) sum[i] += r.ref[i];
        for (auto& r : res) relerr = std::max(relerr, norm_relerr(r.got, sum));
      } else if (o.mode == kMatrixParallel) {
        const size_t blk = r0.ref.size();
        for (auto& r : res)
          for (int q = 0; q < o.gpus; ++q) {
            std::vector<double> g(r.got.begin() + q * blk, r.got.begin() + (q + 1) * blk);
            relerr = std::max(relerr, norm_relerr(g, res[q].ref));
          }
      } else {
        for (auto& r : res) relerr = std::max(relerr, norm_relerr(r.got, r.ref));
      }
      const double tol = o.dtype == 0 ? 1e-5 : o.dtype == 1 ? 2e-3 : 1e-2;  // fp8: bf16 C
      const bool ok = relerr < tol;
      failures += !ok;
      std::printf("  - Check: max rel. error %.2e (%s)\n", relerr, ok ? "PASS" : "FAIL");
    }
    if (js) {
      std::fprintf(js,
                   "{\"script\": \"pdmb_bench\", \"mode\": \"%s\", \"overlap\": %s, \"n\": %d, "
                   "\"dtype\": \"%s\", \"world_size\": %d, \"iterations\": %d, \"warmup\": %d, "
                   "\"avg_ms\": %.6f, \"max_ms\": %.6f, \"compute_ms\": %.6f, \"comm_ms\": %.6f, "
                   "\"tflops_rank0\": %.3f, \"node_tflops\": %.3f, \"actual_tflops\": %.3f, "
                   "\"kernel\": \"%s\", \"pieces\": %d, \"relerr\": %s}\n",
                   mode_name(o.mode), o.overlap ? "true" : "false", n, dtype_name(o.dtype), o.gpus,
                   o.iters, o.warmup, avg, mx, comp, cm, per_gpu, node, actual, r0.kernel.c_str(),
                   r0.chunks, relerr < 0 ? "null" : std::to_string(relerr).c_str());
      std::fflush(js);
    }
  }
  if (js) std::fclose(js);
  for (auto c : comms)
    if (c) ncclCommDestroy(c);
  std::printf("\nBenchmark completed!\n");
  return failures ? 1 : 0;
}
