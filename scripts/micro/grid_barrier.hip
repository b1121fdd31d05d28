// Micro-benchmark: cost of a device-wide barrier inside one launch vs a kernel boundary (gfx950).
// A: phase 1 (each block writes 4 KB) | grid barrier (agent-scope release/acquire) | phase 2 (each
//    block reads its neighbour's 4 KB) -- one launch.
// B: the same two phases as two launches.
// C: as A, but the exchanged data uses agent-scope relaxed stores / loads and the barrier relaxed
//    agent-scope atomics (no L2 writeback / invalidate).
// Every spin is bounded (gives up after ~1M polls and records the failure).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NT = 256;
constexpr int WORDS = 1024;  // per block

__device__ void grid_sync(unsigned* bar, unsigned nb, unsigned* fail, bool relaxed) {
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned old;
    if (relaxed) old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (old / nb + 1) * nb;
    int polls = 0;
    while (true) {
      unsigned v = relaxed ? __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(v - target) >= 0) break;
      if (++polls > (1 << 20)) { atomicAdd(fail, 1u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void phase1(float* buf, int it) {
  float* b = buf + (size_t)blockIdx.x * WORDS;
  for (int i = threadIdx.x; i < WORDS; i += NT) b[i] = (float)(it + i + blockIdx.x);
}
__global__ __launch_bounds__(NT) void phase2(const float* buf, float* out, int it) {
  const int src = (blockIdx.x + 1) % gridDim.x;
  const float* b = buf + (size_t)src * WORDS;
  float s = 0.f;
  for (int i = threadIdx.x; i < WORDS; i += NT) s += b[i] - (float)(it + i + src);
  if (s != 0.f) atomicAdd(out, 1.f);
}
template <bool RELAXED>
__global__ __launch_bounds__(NT) void fused(float* buf, float* out, unsigned* bar, unsigned* fail, int it) {
  float* b = buf + (size_t)blockIdx.x * WORDS;
  for (int i = threadIdx.x; i < WORDS; i += NT) {
    const float v = (float)(it + i + blockIdx.x);
    if (RELAXED) __hip_atomic_store(b + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else b[i] = v;
  }
  if (RELAXED) __builtin_amdgcn_s_waitcnt(0);
  grid_sync(bar, gridDim.x, fail, RELAXED);
  const int src = (blockIdx.x + 1) % gridDim.x;
  const float* c = buf + (size_t)src * WORDS;
  float s = 0.f;
  for (int i = threadIdx.x; i < WORDS; i += NT) {
    const float v = RELAXED ? __hip_atomic_load(c + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : c[i];
    s += v - (float)(it + i + src);
  }
  if (s != 0.f) atomicAdd(out, 1.f);
}

int main() {
  int nb = 256;
  float *buf, *out;
  unsigned *bar, *fail;
  CK(hipMalloc(&buf, sizeof(float) * WORDS * 1024));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&bar, 4));
  CK(hipMalloc(&fail, 4));
  CK(hipMemset(out, 0, 4));
  CK(hipMemset(bar, 0, 4));
  CK(hipMemset(fail, 0, 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int REPS = 200;
  for (int nbi : {64, 128, 256}) {
    nb = nbi;
    for (int mode = 0; mode < 3; ++mode) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < REPS; ++r) {
        if (mode == 0) {
          hipLaunchKernelGGL(phase1, dim3(nb), dim3(NT), 0, st, buf, r);
          hipLaunchKernelGGL(phase2, dim3(nb), dim3(NT), 0, st, buf, out, r);
        } else if (mode == 1) {
          hipLaunchKernelGGL(fused<false>, dim3(nb), dim3(NT), 0, st, buf, out, bar, fail, r);
        } else {
          hipLaunchKernelGGL(fused<true>, dim3(nb), dim3(NT), 0, st, buf, out, bar, fail, r);
        }
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      float best = 1e9f;
      for (int k = 0; k < 5; ++k) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      float h_out;
      unsigned h_fail;
      CK(hipMemcpy(&h_out, out, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&h_fail, fail, 4, hipMemcpyDeviceToHost));
      printf("blocks %3d  %-28s %7.2f us per rep   mismatches %g  spin-failures %u\n", nb,
             mode == 0 ? "two launches" : mode == 1 ? "one launch, acq/rel barrier" : "one launch, relaxed sc1",
             best * 1e3f / REPS, h_out, h_fail);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
