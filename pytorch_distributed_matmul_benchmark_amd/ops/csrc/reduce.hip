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
// adds, a grid-stride loop over up to 8 workgroups per CU; a scalar loop covers
// lengths that are not a multiple of the vector width (and unaligned pointers).
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
hipError_t launch_ns(void* dst, const SrcList& src, int64_t n, bool vec, hipStream_t stream) {
  constexpr int kVec = DT == 0 ? 4 : 8;
  const int64_t nvec = vec ? n / kVec : n;
  int64_t blocks = (nvec + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);  // 8 per CU at most; grid-stride beyond
  hipLaunchKernelGGL((reduce_sum_kernel<DT, NS>), dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n, vec);
  return hipGetLastError();
}

template <int DT>
hipError_t launch_dt(void* dst, const SrcList& src, int nsrc, int64_t n, bool vec, hipStream_t stream) {
  switch (nsrc) {
#define PDMB_NS(k) \
  case k:          \
    return launch_ns<DT, k>(dst, src, n, vec, stream);
    PDMB_NS(1) PDMB_NS(2) PDMB_NS(3) PDMB_NS(4) PDMB_NS(5) PDMB_NS(6) PDMB_NS(7) PDMB_NS(8)
    PDMB_NS(9) PDMB_NS(10) PDMB_NS(11) PDMB_NS(12) PDMB_NS(13) PDMB_NS(14) PDMB_NS(15) PDMB_NS(16)
#undef PDMB_NS
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t reduce_sum(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t stream) {
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
      return launch_dt<0>(dst, s, nsrc, n, vec, stream);
    case 1:
      return launch_dt<1>(dst, s, nsrc, n, vec, stream);
    case 2:
      return launch_dt<2>(dst, s, nsrc, n, vec, stream);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace pdmb
