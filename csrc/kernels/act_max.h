// Producer side of an activation's per-image / per-channel |max| slots (ActMaxOut, kernels.h): the
// f16x2 GEMMs that consume the activation scale each of their rows by its image's (forward, data
// gradient) or its channel's (weight gradient) maximum (x3_common.h).
//
// A kernel that writes an NHWC activation folds |value| on chip -- per image in a thread-local
// running max that moves into a small LDS window when the image changes, per channel in registers
// of the thread's fixed channel quad -- and publishes once per block: one atomicMax per image of the
// window and one per channel (block b into channel copy b % kActCopies). The slots are
// zero-initialised by the host (a memset of the step's slot chunk, ops.cpp), so the value a
// consumer reads is exactly the maximum over everything the producer wrote.
#pragma once
#include "common.h"
#include "kernels.h"

namespace cdp {

constexpr int kImgWin = 16;     // images per block held in LDS (others go straight to global slots)
constexpr int kMaxActC = 2048;  // channels of the largest activation (ResNet-50's 2048)

// Address-space-explicit unsigned max atomics: LDS (ds_max_u32, workgroup scope) and global
// (memory-side, agent scope). Spelling the address space keeps the compiler from merging an LDS
// and a global atomic of one branch into a flat atomic (which gfx950 codegen rejects).
typedef __attribute__((address_space(3))) unsigned lds_u32;
typedef __attribute__((address_space(1))) unsigned glb_u32;
__device__ __forceinline__ void lds_max_u32(unsigned* p, unsigned v) {
  __hip_atomic_fetch_max((lds_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void glb_max_u32(unsigned* p, unsigned v) {
  __hip_atomic_fetch_max((glb_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float absmax4(float4 v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ float4 absmax4(float4 a, float4 v) {
  return make_float4(fmaxf(a.x, fabsf(v.x)), fmaxf(a.y, fabsf(v.y)), fmaxf(a.z, fabsf(v.z)), fmaxf(a.w, fabsf(v.w)));
}

// LDS image window + channel slots of one block. init() zeroes them (call before any add and
// follow by a barrier); publish() after a barrier that follows the last add.
template <int NCH>
struct ActMaxBlock {
  unsigned img[kImgWin];
  unsigned ch[NCH];
  __device__ void init(int tid, int nthreads) {
    for (int j = tid; j < kImgWin + NCH; j += nthreads) (j < kImgWin ? img[j] : ch[j - kImgWin]) = 0u;
  }
  __device__ void add_ch(int c, float v) {
    const unsigned b = __float_as_uint(v);
    if (b) lds_max_u32(&ch[c], b);
  }
  __device__ void add_ch4(int c0, float4 v) {
    add_ch(c0, v.x);
    add_ch(c0 + 1, v.y);
    add_ch(c0 + 2, v.z);
    add_ch(c0 + 3, v.w);
  }
  // channel quad c0..c0+3 of C: into LDS when the table holds C channels, else straight into the
  // block's global channel copy (a layer wider than the table; publish() then gets nch = 0)
  __device__ void add_ch4_any(int c0, float4 v, int C, const ActMaxOut& o, int copy) {
    if (C <= NCH) {
      add_ch4(c0, v);
      return;
    }
    unsigned* dst = o.ch + (long long)copy * C + c0;
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (__float_as_uint(e[j])) glb_max_u32(&dst[j], __float_as_uint(e[j]));
  }
  // global slot publication: img0 = first image of the window, channels [c0, c0 + nch) of C
  __device__ void publish(const ActMaxOut& o, int img0, int N, int c0, int nch, int C, int copy, int tid,
                          int nthreads) {
    for (int j = tid; j < kImgWin; j += nthreads)
      if (img[j] && img0 + j < N) glb_max_u32(&o.img[img0 + j], img[j]);
    unsigned* dst = o.ch + (long long)copy * C + c0;
    for (int c = tid; c < nch; c += nthreads)
      if (ch[c]) glb_max_u32(&dst[c], ch[c]);
  }
};

// A thread's running max of the image it is currently writing.
struct ImgRun {
  int cur = -1;
  float m = 0.f;
  template <int NCH>
  __device__ __forceinline__ void flush(ActMaxBlock<NCH>& s, int img0, const ActMaxOut& o) {
    const unsigned b = __float_as_uint(m);
    if (cur >= 0 && b) {
      const int j = cur - img0;
      if (j >= 0 && j < kImgWin) lds_max_u32(&s.img[j], b);
      else glb_max_u32(&o.img[cur], b);
    }
  }
  template <int NCH>
  __device__ __forceinline__ void add(int img, float v, ActMaxBlock<NCH>& s, int img0, const ActMaxOut& o) {
    if (img != cur) {
      flush(s, img0, o);
      cur = img;
      m = 0.f;
    }
    m = fmaxf(m, v);
  }
};

}  // namespace cdp
