// Sum of up to kMaxReduceSrcs equal-length buffers into one (the local step of
// the direct two-shot all-reduce, parallel/comm.py `all_reduce_direct`):
//
//   dst[i] = round(src[0][i] + src[1][i] + ... + src[n-1][i])   (fp32 accumulate)
//
// The sources are summed in index order on every rank, so the rank that owns
// a chunk produces the same bits whichever rank it is, and the all-gather that
// follows hands every rank an identical tensor. dst may alias any source (each
// element is read by the thread that writes it).
//
// Memory-bound (n_src reads + 1 write per element): each lane moves 16-B
// vectors (8 bf16 / fp16, 4 fp32), loads of all sources issued before the
// adds, a grid-stride loop over up to 8 workgroups per CU (or the caller's
// cap); a scalar loop covers lengths that are not a multiple of the vector
// width (and unaligned pointers).
//
// The sources may be peer-mapped addresses (parallel/ipc.py: another GPU's
// buffer opened with hipIpcOpenMemHandle): the peer-memory all-reduce sums
// its chunk straight out of every peer's output, one load stream per xGMI
// link, with no landing copy.
//
// multi_copy (below) is the peer-memory all-gather's pull: up to kMaxCopies
// (dst, src, bytes) copies in ONE launch, blockIdx.y = copy, so every peer's
// link is read at once from one stream (no copy-stream fan-out competing for
// the process's hardware queues).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "api.h"

namespace pdmb {
namespace {

struct SrcList {
  const void* p[kMaxReduceSrcs];
};

__device__ inline float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <int DT>
struct Elem;
template <>
struct Elem<0> {  // fp32
  using T = float;
  __device__ static float load(const T* p, int64_t i) { return p[i]; }
  __device__ static void store(T* p, int64_t i, float v) { p[i] = v; }
};
template <>
struct Elem<1> {  // fp16
  using T = _Float16;
  __device__ static float load(const T* p, int64_t i) { return (float)p[i]; }
  __device__ static void store(T* p, int64_t i, float v) { p[i] = (_Float16)v; }
};
template <>
struct Elem<2> {  // bf16 (stored as raw 16-bit)
  using T = uint16_t;
  __device__ static float load(const T* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ static void store(T* p, int64_t i, float v) { p[i] = f32_to_bf16_rne(v); }
};

// One 16-B vector: 4 dwords holding 4 fp32 or 8 16-bit values.
template <int DT>
__device__ inline void unpack_add(const uint4& v, float* acc) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (DT == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += __uint_as_float(w[j]);
  } else if constexpr (DT == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[2 * j] += __uint_as_float(w[j] << 16);
      acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const _Float16 lo = __builtin_bit_cast(_Float16, (uint16_t)(w[j] & 0xffffu));
      const _Float16 hi = __builtin_bit_cast(_Float16, (uint16_t)(w[j] >> 16));
      acc[2 * j] += (float)lo;
      acc[2 * j + 1] += (float)hi;
    }
  }
}

template <int DT>
__device__ inline uint4 pack(const float* acc) {
  uint32_t w[4];
  if constexpr (DT == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = __float_as_uint(acc[j]);
  } else if constexpr (DT == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)f32_to_bf16_rne(acc[2 * j]) | ((uint32_t)f32_to_bf16_rne(acc[2 * j + 1]) << 16);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint16_t lo = __builtin_bit_cast(uint16_t, (_Float16)acc[2 * j]);
      const uint16_t hi = __builtin_bit_cast(uint16_t, (_Float16)acc[2 * j + 1]);
      w[j] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int DT, int NS>
__global__ __launch_bounds__(256) void reduce_sum_kernel(void* dst, SrcList src, int64_t n, bool vec) {
  using E = Elem<DT>;
  using T = typename E::T;
  constexpr int kVec = 16 / sizeof(T);
  const int64_t nvec = vec ? n / kVec : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    uint4 in[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) in[s] = ((const uint4*)src.p[s])[v];
    float acc[kVec];
#pragma unroll
    for (int j = 0; j < kVec; ++j) acc[j] = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) unpack_add<DT>(in[s], acc);  // index order: same bits on every rank
    ((uint4*)dst)[v] = pack<DT>(acc);
  }
  // tail (n % kVec elements, or all of them when a pointer is not 16-B aligned)
  for (int64_t t = nvec * kVec + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
    float a = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) a += E::load((const T*)src.p[s], t);
    E::store((T*)dst, t, a);
  }
}

template <int DT, int NS>
hipError_t launch_ns(void* dst, const SrcList& src, int64_t n, bool vec, int cap, hipStream_t stream) {
  constexpr int kVec = DT == 0 ? 4 : 8;
  const int64_t nvec = vec ? n / kVec : n;
  int64_t blocks = (nvec + 255) / 256;
  const int64_t hi = cap > 0 ? cap : 2048;  // 8 per CU at most by default; grid-stride beyond
  blocks = blocks < 1 ? 1 : (blocks > hi ? hi : blocks);
  hipLaunchKernelGGL((reduce_sum_kernel<DT, NS>), dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n, vec);
  return hipGetLastError();
}

template <int DT>
hipError_t launch_dt(void* dst, const SrcList& src, int nsrc, int64_t n, bool vec, int cap, hipStream_t stream) {
  switch (nsrc) {
#define PDMB_NS(k) \
  case k:          \
    return launch_ns<DT, k>(dst, src, n, vec, cap, stream);
    PDMB_NS(1) PDMB_NS(2) PDMB_NS(3) PDMB_NS(4) PDMB_NS(5) PDMB_NS(6) PDMB_NS(7) PDMB_NS(8)
    PDMB_NS(9) PDMB_NS(10) PDMB_NS(11) PDMB_NS(12) PDMB_NS(13) PDMB_NS(14) PDMB_NS(15) PDMB_NS(16)
#undef PDMB_NS
    default:
      return hipErrorInvalidValue;
  }
}

struct CopyList {
  char* dst[kMaxCopies];
  const char* src[kMaxCopies];
  int64_t bytes[kMaxCopies];
};

// Copy blockIdx.y: kUnroll 16-B loads per lane in flight before their stores
// (a remote read over xGMI has microseconds of latency: bandwidth per
// workgroup is bytes in flight / latency), grid-stride over blockIdx.x; the
// bytes past the last whole vector (or all, if a pointer is not 16-B
// aligned) one byte per lane.
constexpr int kUnroll = 8;
__global__ __launch_bounds__(256) void multi_copy_kernel(CopyList c) {
  const int j = blockIdx.y;
  char* __restrict__ d = c.dst[j];
  const char* __restrict__ s = c.src[j];
  const int64_t bytes = c.bytes[j];
  const bool vec = ((uintptr_t)d % 16 == 0) && ((uintptr_t)s % 16 == 0);
  const int64_t nvec = vec ? bytes / 16 : 0;
  const int64_t lanes = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* sv = (const uint4*)s;
  uint4* dv = (uint4*)d;
  int64_t v = t0;
  for (; v + (kUnroll - 1) * lanes < nvec; v += kUnroll * lanes) {
    uint4 r[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) r[u] = sv[v + u * lanes];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) dv[v + u * lanes] = r[u];
  }
  for (; v < nvec; v += lanes) dv[v] = sv[v];
  for (int64_t b = nvec * 16 + t0; b < bytes; b += lanes) d[b] = s[b];
}

// One wave whose lane 0 polls a host flag (system-scope atomic loads of
// fine-grained host memory) until it reaches `value` or `ticks` of the
// constant wall clock pass — the stream-blocking gate of the hardware-queue
// test (tests/test_ipc_gpu.py): every wave exits by the deadline.
__global__ __launch_bounds__(64) void gate_kernel(const unsigned* flag, unsigned value, unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (true) {
    const unsigned v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((int)(v - value) >= 0) break;
    if (wall_clock64() - t0 > ticks) break;
    __builtin_amdgcn_s_sleep(127);
  }
}

}  // namespace

hipError_t gate(const Signal* s, int slot, unsigned value, double timeout_s, hipStream_t stream) {
  if (!s || slot < 0 || slot >= s->slots || timeout_s <= 0) return hipErrorInvalidValue;
  int rate_khz = 0;  // wall_clock64 frequency
  hipError_t e = hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, s->device);
  if (e != hipSuccess) return e;
  if (rate_khz <= 0) rate_khz = 100000;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e3 * rate_khz);
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, stream, s->host_dev + slot, value, ticks);
  return hipGetLastError();
}

hipError_t multi_copy(void* const* dsts, const void* const* srcs, const size_t* bytes, int n, int blocks_per,
                      hipStream_t stream) {
  if (n < 0 || n > kMaxCopies) return hipErrorInvalidValue;
  CopyList c{};
  int m = 0;
  size_t most = 0;
  for (int i = 0; i < n; ++i) {
    if (!bytes[i]) continue;
    if (!dsts[i] || !srcs[i]) return hipErrorInvalidValue;
    c.dst[m] = (char*)dsts[i];
    c.src[m] = (const char*)srcs[i];
    c.bytes[m] = (int64_t)bytes[i];
    most = bytes[i] > most ? bytes[i] : most;
    ++m;
  }
  if (!m) return hipSuccess;
  // workgroups per copy: the caller's count, or 32 (a 7-peer gather: 224
  // workgroups), never more than the largest copy has 256-lane vector rounds
  int64_t per = blocks_per > 0 ? blocks_per : 32;
  const int64_t need = ((int64_t)(most / 16) + 255) / 256;
  per = per > need ? (need < 1 ? 1 : need) : per;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)per, (unsigned)m), dim3(256), 0, stream, c);
  return hipGetLastError();
}

hipError_t reduce_sum(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t stream,
                      int max_blocks) {
  if (nsrc < 1 || nsrc > kMaxReduceSrcs || n < 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  SrcList s{};
  bool vec = (uintptr_t)dst % 16 == 0;  // 16-B vectors when every pointer allows
  for (int i = 0; i < nsrc; ++i) {
    if (!srcs[i]) return hipErrorInvalidValue;
    vec = vec && (uintptr_t)srcs[i] % 16 == 0;
    s.p[i] = srcs[i];
  }
  switch (dtype) {
    case 0:
      return launch_dt<0>(dst, s, nsrc, n, vec, max_blocks, stream);
    case 1:
      return launch_dt<1>(dst, s, nsrc, n, vec, max_blocks, stream);
    case 2:
      return launch_dt<2>(dst, s, nsrc, n, vec, max_blocks, stream);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace pdmb
