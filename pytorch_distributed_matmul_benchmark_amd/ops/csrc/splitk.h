// In-launch split-K combine shared by the W4 (256x256) and T128 (128x128)
// kernels: the S workgroups of one output tile meet in the epilogue (no
// second kernel, no memset, no fences).
//
// Hand-off (cdna_hip_programming.md Guideline 16, "sc1" form; MI355X_MICROARCH
// § visibility, Valid forms row 1): the first S-1 slices to arrive (arrival
// ticket from the per-tile `arrive` counter) store their fp32 accumulators
// WRITE-THROUGH (buffer_store_dwordx4 ... sc1) into their slice's slot, every
// storing wave drains (s_waitcnt vmcnt(0)), the workgroup meets at a barrier,
// and one lane adds to the tile's `done` counter (relaxed, agent scope). The
// last to arrive polls `done` (relaxed agent loads = sc1, s_sleep between)
// until S-1, then EVERY load of the slots is an sc1 load, so no acquire fence
// is needed and none of the ~3.5 us __threadfence() pairs of round 1's
// version are paid. The last slice sums slot 0 + slot 1 + ... in slice order
// with its own registers in its own place: bitwise reproducible whoever
// arrives last. It never waits for a workgroup that has not started (only for
// slots whose owners already took a ticket, i.e. are resident and past their
// K-loop), so no co-residency is assumed (safe beside RCCL / under a CU mask).
// The last slice re-zeroes both counters, which are therefore zero between
// launches on a stream (launches on one stream never overlap; the counters
// are zeroed once per stream when created, gemm_dispatch.cpp).
//
// Slot layout follows the accumulator registers: f32x4 block b of thread t at
// ((slice * NBLK + b) * NT + t) * 16 B, so every access is a coalesced 1 KiB
// wave access and no index math depends on the MFMA layout.
#pragma once

#include "common.h"

namespace pdmb {

struct SplitSlots {
  __amdgpu_buffer_rsrc_t rs;  // this tile's S slots (valid for the reducer)
  int t;                      // thread index
};

template <int NBLK, int NT>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t splitk_rsrc(const GemmArgs& a, long long tile) {
  constexpr long long slot_floats = (long long)NBLK * NT * 4;
  return __builtin_amdgcn_make_buffer_rsrc(a.part + tile * a.splitk * slot_floats, 0,
                                           (int)(a.splitk * slot_floats * 4), 0x00020000);
}

// Returns true in the workgroup that must write C (the last slice); `out`
// then addresses the slots. `smem` is the kernel's one LDS array (reused for
// the broadcast after a barrier: a second __shared__ object can de-pipeline
// the LDS-DMA loop, cdna_hip_programming.md trap 4(a)).
template <int MB, int NB, int NT>
__device__ __forceinline__ bool splitk_meet(const GemmArgs& a, char* smem, long long tile, int slice,
                                            f32x4 (&acc)[MB][NB], SplitSlots& out) {
  constexpr int NBLK = MB * NB;
  const int S = a.splitk;
  unsigned* arrive = a.flags + 2 * tile;
  unsigned* done = arrive + 1;
  int* bcast = (int*)smem;
  const int t = threadIdx.x;
  __syncthreads();  // every wave is past its last LDS read before smem is reused
  if (t == 0)
    bcast[0] = (int)__hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int ord = bcast[0];
  const __amdgpu_buffer_rsrc_t rs = splitk_rsrc<NBLK, NT>(a, tile);
  if (ord < S - 1) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, acc[i][j]), rs,
            ((slice * NBLK + i * NB + j) * NT + t) * 16, 0, 16 /* sc1: write-through */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
    __syncthreads();
    if (t == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  if (t == 0) {
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(S - 1))
      __builtin_amdgcn_s_sleep(1);
    // Nobody touches this tile's counters again in this launch.
    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Compiler-only ordering: keep the sc1 slot loads below the poll.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  out.rs = rs;
  out.t = t;
  return true;
}

// Block row i of the tile's sum over slices, in slice order (the reducer).
template <int MB, int NB, int NT>
__device__ __forceinline__ void splitk_row(const GemmArgs& a, const SplitSlots& sl, int slice, int i,
                                           const f32x4 (&acc)[MB][NB], f32x4 (&v)[NB]) {
  constexpr int NBLK = MB * NB;
  for (int s = 0; s < a.splitk; ++s) {
    f32x4 q[NB];
    if (s == slice) {
#pragma unroll
      for (int j = 0; j < NB; ++j) q[j] = acc[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j)
        q[j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       sl.rs, ((s * NBLK + i * NB + j) * NT + sl.t) * 16, 0, 16 /* sc1 */));
    }
    if (s == 0) {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = q[j];
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] += q[j];
    }
  }
}

// S == 2 (GemmArgs::meet_prefetch): the reducer's loads of the other slice's
// block row i, issued a row ahead of their use. The slot bytes sit behind an
// L2 miss (written through by a workgroup on another XCD, ~1-2 us away), and
// splitk_row's loads could not leave before the previous row's C stores
// (the compiler cannot reorder buffer loads across global stores), so every
// block row paid that latency in turn. Two slices: acc + other is the slice-
// order sum (fp32 addition commutes), bitwise equal to splitk_row.
template <int MB, int NB, int NT>
__device__ __forceinline__ void splitk_load_other(const SplitSlots& sl, int slice, int i, f32x4 (&q)[NB]) {
  constexpr int NBLK = MB * NB;
  const int s = 1 - slice;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    q[j] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sl.rs, ((s * NBLK + i * NB + j) * NT + sl.t) * 16, 0,
                                                     16 /* sc1 */));
}

// S == 3 (round 5; GemmArgs::meet_prefetch): both other slices' block row i,
// issued a row ahead of their use, q[0] = the lower slot, q[1] = the higher.
// The sum stays in slot order — (x0 + x1) + x2 with this slice's registers in
// its own place — so it is bitwise equal to splitk_row (splitk_sum3).
template <int MB, int NB, int NT>
__device__ __forceinline__ void splitk_load_others3(const SplitSlots& sl, int slice, int i, f32x4 (&q)[2][NB]) {
  constexpr int NBLK = MB * NB;
  const int o0 = slice == 0 ? 1 : 0, o1 = slice == 2 ? 1 : 2;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    q[0][j] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sl.rs, ((o0 * NBLK + i * NB + j) * NT + sl.t) * 16, 0,
                                                     16 /* sc1 */));
    q[1][j] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sl.rs, ((o1 * NBLK + i * NB + j) * NT + sl.t) * 16, 0,
                                                     16 /* sc1 */));
  }
}
template <int NB>
__device__ __forceinline__ void splitk_sum3(int slice, const f32x4 (&own)[NB], const f32x4 (&q)[2][NB],
                                            f32x4 (&v)[NB]) {
#pragma unroll
  for (int j = 0; j < NB; ++j)  // fp32 addition commutes: (own + q0) == (q0 + own) bit for bit
    v[j] = slice == 2 ? (q[0][j] + q[1][j]) + own[j] : (own[j] + q[0][j]) + q[1][j];
}

// ---- stream-K meet (gemm_fp8.hip gemm_fp8_sk) ------------------------------
// The same hand-off with a per-tile contributor count: S workgroups (S <=
// a.splitk, the slots per tile) each carry a K-range of the tile; `slot` is
// the contributor's index in K order. Whoever arrives last sums the slots in
// slot order (its own in its own place): bitwise reproducible. A contributor
// that is not last stores and returns false; its workgroup goes on to its next
// K-range — the last one waits only for contributors that already took a
// ticket (past their K-loop), never for one that has not started. t: the
// thread index (the caller's, formed where it wants it live).
template <int MB, int NB, int NT>
__device__ __forceinline__ bool sk_meet(const GemmArgs& a, char* smem, long long tile, int slot, int S,
                                        f32x4 (&acc)[MB][NB], SplitSlots& out, int t) {
  constexpr int NBLK = MB * NB;
  unsigned* arrive = a.flags + 2 * tile;
  unsigned* done = arrive + 1;
  int* bcast = (int*)smem;
  __syncthreads();  // every wave is past its last LDS read before smem is reused
  if (t == 0)
    bcast[0] = (int)__hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int ord = bcast[0];
  const __amdgpu_buffer_rsrc_t rs = splitk_rsrc<NBLK, NT>(a, tile);
  if (ord < S - 1) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, acc[i][j]), rs,
            ((slot * NBLK + i * NB + j) * NT + t) * 16, 0, 16 /* sc1: write-through */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
    __syncthreads();
    if (t == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // bcast (LDS) is not rewritten before every wave has read it
    return false;
  }
  if (t == 0) {
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(S - 1))
      __builtin_amdgcn_s_sleep(1);
    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  out.rs = rs;
  out.t = t;
  return true;
}

// Block row i of a stream-K tile's sum over its S contributors, in slot order.
template <int MB, int NB, int NT>
__device__ __forceinline__ void sk_row(const SplitSlots& sl, int slot, int S, int i, const f32x4 (&acc)[MB][NB],
                                       f32x4 (&v)[NB]) {
  constexpr int NBLK = MB * NB;
  for (int s = 0; s < S; ++s) {
    f32x4 q[NB];
    if (s == slot) {
#pragma unroll
      for (int j = 0; j < NB; ++j) q[j] = acc[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j)
        q[j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       sl.rs, ((s * NBLK + i * NB + j) * NT + sl.t) * 16, 0, 16 /* sc1 */));
    }
    if (s == 0) {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = q[j];
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] += q[j];
    }
  }
}

// Stream-K partition of L = span x nk K-tile iterations over G workgroups:
// workgroup w runs iterations [w L / G, (w + 1) L / G) (L >= G: every range is
// non-empty). Contributors of local tile t: workgroups first .. last.
__host__ __device__ __forceinline__ long long sk_begin(long long w, long long L, long long G) { return w * L / G; }
__host__ __device__ __forceinline__ int sk_owner(long long x, long long L, long long G) {
  // the workgroup whose range holds iteration x: max w with w L / G <= x
  return (int)(((x + 1) * G + L - 1) / L - 1);
}

// The most contributors any tile of a stream-K range has (slots per tile):
// G workgroups in 8 XCD groups of G / 8, XCD x sharing out the range's tiles
// of index = x mod 8 (gemm_fp8.hip gemm_fp8_sk).
inline int sk_max_owners(long long span, int nk, long long G) {
  int m = 0;
  for (long long x = 0; x < 8; ++x) {
    const long long tx = (span - x + 7) / 8, L = tx * nk, g = G / 8;
    for (long long t = 0; t < tx; ++t) {
      const int c = sk_owner(t * nk + nk - 1, L, g) - sk_owner(t * nk, L, g) + 1;
      m = c > m ? c : m;
    }
  }
  return m;
}

}  // namespace pdmb
