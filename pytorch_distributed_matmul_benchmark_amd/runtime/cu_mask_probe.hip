// cu_mask_probe — where a CU-masked stream's workgroups actually run.
//
// parallel/overlap.py MaskedStream leaves k CUs out of the GEMM stream's mask
// and assumes mask bit i lands on XCD i % 8 (so the first k bits spread the
// free CUs evenly over the 8 XCDs). This probe checks that assumption on the
// hardware: it creates a stream with the same mask (hipExtStreamCreateWithCUMask),
// launches many one-wave workgroups that each record their XCC_ID and HW_ID
// (CU / SH / SE) with vector stores, and prints, per XCD, how many distinct CUs
// ran workgroups (even spread: 32 - k/8 CUs on every XCD), plus how many
// workgroups did not run on XCD blockIdx % 8 (the kernels' XCD-aware tile maps
// assume they all do).
//
//   cu_mask_probe [--exclude k] [--mode first|block] [--blocks N (default 16 per CU)]
//                 [--lds BYTES] [--threads T] [--spin-us U]
//     first: mask bits 0 .. k-1 off (MaskedStream's choice)
//     block: bits j*(n/k) off for j < k (one every n/k bits)
//     --lds / --threads: each workgroup's dynamic LDS and size — 147968 B and
//       256 threads model W4S (one workgroup per CU: the LDS does not fit two)
//     --spin-us: how long each workgroup holds its CU (default 20 us)
//     --bits b0,b1,...: exactly these mask bits off (which XCD / CU a bit
//       names: with the W4S occupancy and one workgroup per CU, the XCD that
//       lost a CU shows a "late" workgroup)
// Each workgroup also stamps its start / end (wall clock): "late" counts the
// workgroups that started more than half a spin after the first one, i.e.
// that queued behind another workgroup instead of finding a free CU — with
// one workgroup per CU and blocks <= the free CUs, a persistent kernel that
// assumes every workgroup runs at once sees exactly those as a serialized
// second round.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void __launch_bounds__(256) where(unsigned* out, int spin) {
  extern __shared__ char lds[];
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // keep the CU busy so later workgroups spread over the free CUs (or queue)
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) {
    lds[0] = 1;  // the dynamic LDS is allocated (occupancy), touch it once
    out[4 * blockIdx.x] = hw;
    out[4 * blockIdx.x + 1] = xcc;
    out[4 * blockIdx.x + 2] = (unsigned)t0;
    out[4 * blockIdx.x + 3] = (unsigned)wall_clock64();
  }
}

int main(int argc, char** argv) {
  int k = 8, nblocks = 0, lds = 0, threads = 64, spin_us = 20;
  const char* mode = "first";
  std::vector<int> bits;  // --bits b0,b1,...: exactly these mask bits off (mode "bits")
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--exclude")) k = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--mode")) mode = argv[i + 1];
    if (!strcmp(argv[i], "--blocks")) nblocks = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--lds")) lds = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--threads")) threads = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--spin-us")) spin_us = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--bits")) {
      mode = "bits";
      for (const char* q = argv[i + 1]; *q;) {
        bits.push_back(atoi(q));
        while (*q && *q != ',') ++q;
        if (*q == ',') ++q;
      }
      k = (int)bits.size();
    }
  }
  if (threads < 64 || threads > 256 || threads % 64 || lds < 0 || lds > 160 * 1024 || spin_us < 1 ||
      spin_us > 100000) {
    fprintf(stderr, "bad --threads (64..256, multiple of 64) / --lds (<= 160 KiB) / --spin-us\n");
    return 2;
  }
  int clk_khz = 0;
  HIP_OK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  if (clk_khz <= 0) clk_khz = 100000;
  const int spin = (int)((long long)spin_us * clk_khz / 1000);
  if (lds > 64 * 1024) HIP_OK(hipFuncSetAttribute((const void*)where, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, 0));
  const int n = prop.multiProcessorCount;
  std::vector<unsigned> mask((n + 31) / 32, 0);
  for (int i = 0; i < n; ++i) mask[i / 32] |= 1u << (i % 32);
  for (int j = 0; j < k && k > 0; ++j) {
    const int bit = !strcmp(mode, "bits") ? bits[j] : !strcmp(mode, "block") ? j * (n / k) : j;
    if (bit < 0 || bit >= n) {
      fprintf(stderr, "mask bit %d outside [0, %d)\n", bit, n);
      return 2;
    }
    mask[bit / 32] &= ~(1u << (bit % 32));
  }
  hipStream_t s;
  HIP_OK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  const int blocks = nblocks > 0 ? nblocks : n * 16;  // n - k: one per free CU, like W4S
  unsigned* d = nullptr;
  HIP_OK(hipMalloc(&d, sizeof(unsigned) * 4 * blocks));
  HIP_OK(hipMemsetAsync(d, 0xff, sizeof(unsigned) * 4 * blocks, s));
  hipLaunchKernelGGL(where, dim3(blocks), dim3(threads), lds, s, d, spin);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(s));
  std::vector<unsigned> h(4 * blocks);
  HIP_OK(hipMemcpy(h.data(), d, sizeof(unsigned) * 4 * blocks, hipMemcpyDeviceToHost));
  std::set<unsigned> cus[16];
  int per_xcc[16] = {0}, late_xcc[16] = {0};
  int off_residue = 0;  // workgroups NOT on XCD blockIdx % 8 (what map_tile's L2 grouping assumes)
  unsigned first = h[2];
  for (int b = 1; b < blocks; ++b)
    if ((int)(h[4 * b + 2] - first) < 0) first = h[4 * b + 2];
  unsigned last_end = first;
  for (int b = 0; b < blocks; ++b) {
    const unsigned hw = h[4 * b], xcc = h[4 * b + 1] & 0xF;
    off_residue += (int)(xcc != (unsigned)(b % 8));
    // CU id within the XCC: CU_ID [11:8], SH_ID [12], SE_ID [15:13]
    cus[xcc].insert(((hw >> 13) & 0x7) << 5 | ((hw >> 12) & 0x1) << 4 | ((hw >> 8) & 0xF));
    ++per_xcc[xcc];
    late_xcc[xcc] += (int)(h[4 * b + 2] - first > (unsigned)(spin / 2));
    if ((int)(h[4 * b + 3] - last_end) > 0) last_end = h[4 * b + 3];
  }
  int late = 0;
  for (int x = 0; x < 16; ++x) late += late_xcc[x];
  printf("{\"cus\": %d, \"excluded\": %d, \"mode\": \"%s\", \"threads\": %d, \"lds\": %d, "
         "\"spin_us\": %d, \"per_xcd\": [",
         n, k, mode, threads, lds, spin_us);
  for (int x = 0; x < 8; ++x)
    printf("%s{\"xcd\": %d, \"distinct_cus\": %zu, \"workgroups\": %d, \"late\": %d}", x ? ", " : "", x,
           cus[x].size(), per_xcc[x], late_xcc[x]);
  printf("], \"blocks\": %d, \"not_on_xcd_blockidx_mod8\": %d, \"late\": %d, \"span_us\": %.1f}\n", blocks,
         off_residue, late, (double)(last_end - first) * 1000.0 / clk_khz);
  HIP_OK(hipFree(d));
  HIP_OK(hipStreamDestroy(s));
  return 0;
}
