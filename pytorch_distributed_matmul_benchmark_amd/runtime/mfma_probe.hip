// mfma_probe — FLOP rate of the two bf16 MFMA shapes on random operands.
//
// Question (round-1 verdict, item 5): the 16k headline is power-bound (W4 at
// ~1.75 GHz, 81 % MFMA busy, profiles/r1_s4_pmc_w4.md). Would a W4 built on
// v_mfma_f32_32x32x16_bf16 (half the operand register reads per FLOP) beat
// the v_mfma_f32_16x16x32_bf16 one? Both kernels here do nothing but MFMAs
// on random bf16 operands held in registers (rotating through 8 operand
// sets so the data toggles as in a GEMM), one wave per SIMD on every CU,
// 64 fp32 accumulators per lane either way. If the 32x32 loop does not beat
// the 16x16 loop here, the W4 variant (same LDS traffic, more accumulator
// traffic per MFMA) cannot beat it in the GEMM.
//
//   mfma_probe [--ms 400] [--rounds 5]   -> one JSON line per (shape, round)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int kSets = 8;

// 16 accumulators of 16x16 (4 fp32 each) = 64 AGPRs; 16 MFMAs per step.
__global__ void __launch_bounds__(256, 1) mfma16(const s16x8* __restrict__ src, float* out, int iters) {
  s16x8 a[kSets], b[kSets];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int s = 0; s < kSets; ++s) {
    a[s] = src[(t * 2 * kSets + 2 * s) % (1 << 20)];
    b[s] = src[(t * 2 * kSets + 2 * s + 1) % (1 << 20)];
  }
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; it += kSets) {  // operand set indices stay compile-time
#pragma unroll
    for (int u = 0; u < kSets; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int s = (i + u) % kSets;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i]) : "v"(a[s]), "v"(b[(s + i) % kSets]));
      }
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  out[t] = r;
}

// 4 accumulators of 32x32 (16 fp32 each) = 64 AGPRs; 8 MFMAs per step = the
// same FLOPs per step as mfma16's 16 (each 32x32x16 is 2x a 16x16x32).
__global__ void __launch_bounds__(256, 1) mfma32(const s16x8* __restrict__ src, float* out, int iters) {
  s16x8 a[kSets], b[kSets];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int s = 0; s < kSets; ++s) {
    a[s] = src[(t * 2 * kSets + 2 * s) % (1 << 20)];
    b[s] = src[(t * 2 * kSets + 2 * s + 1) % (1 << 20)];
  }
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  for (int it = 0; it < iters; it += kSets) {
#pragma unroll
    for (int u = 0; u < kSets; ++u)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int s = (i + u) % kSets;
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i & 3]) : "v"(a[s]), "v"(b[(s + i) % kSets]));
      }
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) r += acc[i][e];
  out[t] = r;
}

__global__ void fill_random(unsigned short* p, int n, unsigned seed) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    // bf16 in [-2, 2): sign, exponent 126..127, random mantissa
    const unsigned sign = (x >> 31) & 1, e = 126 + ((x >> 30) & 1), m = (x >> 8) & 0x7f;
    p[i] = (unsigned short)((sign << 15) | (e << 7) | m);
  }
}

int main(int argc, char** argv) {
  double target_ms = 400.0;
  int rounds = 5;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--ms")) target_ms = atof(argv[i + 1]);
    if (!strcmp(argv[i], "--rounds")) rounds = atoi(argv[i + 1]);
  }
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, 0));
  const int blocks = prop.multiProcessorCount;  // 1 workgroup (4 waves = 1 per SIMD) per CU
  const int threads = 256;
  s16x8* src;
  float* out;
  HIP_OK(hipMalloc(&src, (size_t)(1 << 20) * sizeof(s16x8)));
  HIP_OK(hipMalloc(&out, (size_t)blocks * threads * sizeof(float)));
  hipLaunchKernelGGL(fill_random, dim3(1024), dim3(256), 0, 0, (unsigned short*)src, (1 << 20) * 8,
                     12345u);
  HIP_OK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  // FLOPs per step per wave: 16 x 16x16x32 = 8 x 32x32x16 = 262144
  const double flop_step = 16.0 * 2 * 16 * 16 * 32;
  const double waves = (double)blocks * threads / 64;
  // calibrate iterations to ~target_ms at ~2 PF
  const int iters = (int)(target_ms * 1e-3 * 2.0e15 / (flop_step * waves)) / kSets * kSets;
  for (int r = 0; r < rounds + 1; ++r) {
    for (int shape = 0; shape < 2; ++shape) {
      HIP_OK(hipEventRecord(e0, 0));
      if (shape == 0)
        hipLaunchKernelGGL(mfma16, dim3(blocks), dim3(threads), 0, 0, src, out, iters);
      else
        hipLaunchKernelGGL(mfma32, dim3(blocks), dim3(threads), 0, 0, src, out, iters);
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(e1, 0));
      HIP_OK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      if (r == 0) continue;  // warm-up round (clocks)
      const double tflops = flop_step * waves * iters / (ms * 1e-3) / 1e12;
      printf("{\"shape\": \"%s\", \"round\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"iters\": %d, "
             "\"cus\": %d, \"data\": \"random bf16\"}\n",
             shape == 0 ? "16x16x32" : "32x32x16", r, ms, tflops, iters, blocks);
      fflush(stdout);
    }
  }
  HIP_OK(hipFree(src));
  HIP_OK(hipFree(out));
  return 0;
}
