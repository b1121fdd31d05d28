// Shared device helpers for the CDNA4 (gfx950) kernels of this framework.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA set;
// there is no alternate-platform path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdp {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// Full 64-lane butterfly sum.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// LDS barrier that does not wait for global loads still in flight: __syncthreads' fence would
// drain them (vmcnt(0)). The release / acquire fences are workgroup-scope and LDS-only
// ("local" address space), so they order the LDS stores before the barrier and the LDS loads after
// it in the compiler's memory model (a bare s_barrier is not a memory operation to LLVM, so nothing
// would stop an LDS access from being scheduled across it) while lowering to lgkmcnt(0) alone.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Bijective XCD-aware remap of a flat workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"). Blocks are dealt round-robin over the 8 XCDs,
// so consecutive *remapped* ids land on the same XCD and share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace cdp
