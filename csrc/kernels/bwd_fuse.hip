// Backward-pass reduction fusion for a Conv -> BN -> ReLU [-> MaxPool] chain (VGG,
// /root/reference/src/Part 1/model.py:11-27), gfx950.
//
// After the weight- and data-gradient GEMMs of block L+1 have written their split-K slabs, ONE
// launch finishes both and starts block L's BatchNorm backward:
//   job D (blocks [0, nbd)):  dX = sum_z slab_D[z] (+ addend)  -- the gradient reaching block L's
//        output -- and, from the same registers, block L's BN-backward partial sums per channel:
//        sum dz, sum dz*xhat [, sum xhat], with the pool / ReLU routing recomputed from block L's
//        saved conv output (what bn_bwd_reduce_kernel computes in a launch of its own);
//   job W (blocks [nbd, nbd + nbw)): dW = sum_z slab_W[z]  (what slab_sum4_kernel computes).
// The two jobs are independent memory-bound reductions; sharing a launch removes two dependent
// dispatches per block (~1.6 us floor each under hipGraph, plus their ramp and tail) and the
// second read of dX. Summation orders are fixed, so results are deterministic.
#include "common.h"
#include "kernels.h"

namespace cdp {
namespace {

constexpr int RBD = 32;  // rows per job-D block = rows per BN partial

__device__ __forceinline__ float4 aff_act(float4 y, float4 sc, float4 sh, bool relu) {
  float4 z;
  z.x = fmaf(y.x, sc.x, sh.x);
  z.y = fmaf(y.y, sc.y, sh.y);
  z.z = fmaf(y.z, sc.z, sh.z);
  z.w = fmaf(y.w, sc.w, sh.w);
  if (relu) {
    z.x = fmaxf(z.x, 0.f);
    z.y = fmaxf(z.y, 0.f);
    z.z = fmaxf(z.z, 0.f);
    z.w = fmaxf(z.w, 0.f);
  }
  return z;
}

__device__ __forceinline__ float f4get(const float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4add(float4& v, int j, float a) {
  if (j == 0) v.x += a;
  else if (j == 1) v.y += a;
  else if (j == 2) v.z += a;
  else v.w += a;
}

// One channel of a 2x2 window: sum of the routed gradient and of gradient * xhat over the window
// (first max wins in scan order (0,0),(0,1),(1,0),(1,1), like ATen and bn_bwd_reduce_kernel).
__device__ __forceinline__ void window_sums(float z0, float z1, float z2, float z3, float x0, float x1, float x2,
                                            float x3, float g, bool relu, float& sdz, float& sdx) {
  int arg = 0;
  float mx = z0;
  if (z1 > mx) { mx = z1; arg = 1; }
  if (z2 > mx) { mx = z2; arg = 2; }
  if (z3 > mx) { mx = z3; arg = 3; }
  const float gg = (!relu || mx > 0.f) ? g : 0.f;
  sdz = gg;
  sdx = gg * (arg == 0 ? x0 : arg == 1 ? x1 : arg == 2 ? x2 : x3);
}

__global__ __launch_bounds__(256) void bwd_reduce_kernel(BwdReduceArgs a) {
  __shared__ float4 red[3][256];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  if (b < a.nbd) {
    // ---------------------------------------------------------------- job D
    const int bx = b % a.d_nbx, by = b / a.d_nbx;
    const int cq = tid & 15, rl = tid >> 4;
    const int C = a.d_Nout;
    const int n = bx * 64 + cq * 4;
    const bool nok = n < C;
    const int y0 = by * RBD;
    const long long plane = (long long)a.d_M * C;
    float4 g[RBD / 16];
    // both rows' slab loads in batches of 8 splits (one round trip per batch); out-of-range rows /
    // splits load a valid address and are masked to zero
#pragma unroll
    for (int i = 0; i < RBD / 16; ++i) g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool any = nok && y0 + rl < a.d_M;
    for (int z0 = 0; any && z0 < a.d_S; z0 += 8) {
      float4 t[RBD / 16][8];
#pragma unroll
      for (int i = 0; i < RBD / 16; ++i) {
        const int m = y0 + rl + 16 * i;
        const float* src = a.d_slab + (long long)(m < a.d_M ? m : y0 + rl) * C + n;
#pragma unroll
        for (int k = 0; k < 8; ++k) t[i][k] = ld4(src + (long long)(z0 + k < a.d_S ? z0 + k : 0) * plane);
      }
#pragma unroll
      for (int i = 0; i < RBD / 16; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (z0 + k >= a.d_S) t[i][k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < RBD / 16; ++i) {
        float4& s = g[i];
        s.x += ((t[i][0].x + t[i][1].x) + (t[i][2].x + t[i][3].x)) + ((t[i][4].x + t[i][5].x) + (t[i][6].x + t[i][7].x));
        s.y += ((t[i][0].y + t[i][1].y) + (t[i][2].y + t[i][3].y)) + ((t[i][4].y + t[i][5].y) + (t[i][6].y + t[i][7].y));
        s.z += ((t[i][0].z + t[i][1].z) + (t[i][2].z + t[i][3].z)) + ((t[i][4].z + t[i][5].z) + (t[i][6].z + t[i][7].z));
        s.w += ((t[i][0].w + t[i][1].w) + (t[i][2].w + t[i][3].w)) + ((t[i][4].w + t[i][5].w) + (t[i][6].w + t[i][7].w));
      }
    }
    // (one "slab" that is dX itself, read in place: nothing to write back)
    const bool in_place = a.d_slab == a.d_y && !a.d_addend;
#pragma unroll
    for (int i = 0; i < RBD / 16; ++i) {
      const int m = y0 + rl + 16 * i;
      float4 s = g[i];
      if (m < a.d_M && nok && !in_place) {
        const long long o = (long long)m * C + n;
        if (a.d_addend) {
          const float4 ad = ld4(a.d_addend + o);
          s.x += ad.x; s.y += ad.y; s.z += ad.z; s.w += ad.w;
        }
        st4(a.d_y + o, s);
      }
      g[i] = s;
    }
    if (!a.bn_part) return;
    // block L's BN backward partials over this block's rows (pooled pixels when bn_pool)
    const bool relu = a.bn_relu != 0;
    const int H = a.bn_H, W = a.bn_W;
    const int Ho = a.bn_pool ? H / 2 : H, Wo = a.bn_pool ? W / 2 : W;
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1, a3 = a1;
    if (nok) {
      const float* st = a.bn_stats;
      const float4 mu = ld4(st + n), is = ld4(st + C + n), sc = ld4(st + 2 * C + n), sh = ld4(st + 3 * C + n);
#pragma unroll
      for (int i = 0; i < RBD / 16; ++i) {
        const int m = y0 + rl + 16 * i;
        if (m >= a.d_M) continue;
        if (!a.bn_pool) {
          const float4 yv = ld4(a.bn_y + (long long)m * C + n);
          const float4 z = aff_act(yv, sc, sh, relu);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float dz = (!relu || f4get(z, e) > 0.f) ? f4get(g[i], e) : 0.f;
            const float xh = (f4get(yv, e) - f4get(mu, e)) * f4get(is, e);
            f4add(a1, e, dz);
            f4add(a2, e, dz * xh);
            f4add(a3, e, xh);
          }
        } else {
          const int t = fdiv(m, a.bn_fd_wo);
          const int wo = m - t * Wo;
          const int nn = fdiv(t, a.bn_fd_ho);
          const int ho = t - nn * Ho;
          const float* base = a.bn_y + (((long long)nn * H + 2 * ho) * W + 2 * wo) * C + n;
          const float4 v0 = ld4(base), v1 = ld4(base + C), v2 = ld4(base + (long long)W * C),
                       v3 = ld4(base + (long long)W * C + C);
          const float4 z0 = aff_act(v0, sc, sh, relu), z1 = aff_act(v1, sc, sh, relu), z2 = aff_act(v2, sc, sh, relu),
                       z3 = aff_act(v3, sc, sh, relu);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float m_ = f4get(mu, e), s_ = f4get(is, e);
            const float x0 = (f4get(v0, e) - m_) * s_, x1 = (f4get(v1, e) - m_) * s_, x2 = (f4get(v2, e) - m_) * s_,
                        x3 = (f4get(v3, e) - m_) * s_;
            float sdz, sdx;
            window_sums(f4get(z0, e), f4get(z1, e), f4get(z2, e), f4get(z3, e), x0, x1, x2, x3, f4get(g[i], e), relu,
                        sdz, sdx);
            f4add(a1, e, sdz);
            f4add(a2, e, sdx);
            f4add(a3, e, (x0 + x1) + (x2 + x3));
          }
        }
      }
    }
    red[0][tid] = a1;
    red[1][tid] = a2;
    red[2][tid] = a3;
    __syncthreads();
    if (rl == 0 && nok) {
      float4 s1 = a1, s2 = a2, s3 = a3;
#pragma unroll
      for (int k = 1; k < 16; ++k) {
        const float4 p = red[0][k * 16 + cq], q = red[1][k * 16 + cq], r = red[2][k * 16 + cq];
        s1.x += p.x; s1.y += p.y; s1.z += p.z; s1.w += p.w;
        s2.x += q.x; s2.y += q.y; s2.z += q.z; s2.w += q.w;
        s3.x += r.x; s3.y += r.y; s3.z += r.z; s3.w += r.w;
      }
      const int PS = a.bn_ps;
      float* dst = a.bn_part + ((long long)by * C + n) * PS;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dst[e * PS] = f4get(s1, e);
        dst[e * PS + 1] = f4get(s2, e);
        if (PS == 3) dst[e * PS + 2] = f4get(s3, e);
      }
    }
    return;
  }
  // ------------------------------------------------------------------ job W
  const int bw = b - a.nbd;
  const int CB = a.w_cb, SL = 256 / CB;
  const int cl = tid % CB, sl = tid / CB;
  const long long i = (long long)bw * CB + cl;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < a.w_n4) {
    int z = sl;
    for (; z + 3 * SL < a.w_S; z += 4 * SL) {
      const float4 p = a.w_slab[(long long)z * a.w_n4 + i], q = a.w_slab[(long long)(z + SL) * a.w_n4 + i];
      const float4 r = a.w_slab[(long long)(z + 2 * SL) * a.w_n4 + i], t = a.w_slab[(long long)(z + 3 * SL) * a.w_n4 + i];
      s.x += (p.x + q.x) + (r.x + t.x); s.y += (p.y + q.y) + (r.y + t.y);
      s.z += (p.z + q.z) + (r.z + t.z); s.w += (p.w + q.w) + (r.w + t.w);
    }
    for (; z < a.w_S; z += SL) {
      const float4 p = a.w_slab[(long long)z * a.w_n4 + i];
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
  }
  if (SL > 1) {
    red[0][tid] = s;
    __syncthreads();
    if (sl != 0) return;
    for (int k = 1; k < SL; ++k) {
      const float4 p = red[0][k * CB + cl];
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
  }
  if (i < a.w_n4) a.w_dst[i] = s;
}

}  // namespace

int bwd_reduce_rows_per_part() { return RBD; }

void bwd_reduce_launch(BwdReduceArgs a, hipStream_t st) {
  if (a.bn_part && a.bn_pool) {
    a.bn_fd_wo = make_fastdiv(a.bn_W / 2);
    a.bn_fd_ho = make_fastdiv(a.bn_H / 2);
  }
  a.nbd = 0;
  a.d_nbx = 0;
  if (a.d_slab) {
    a.d_nbx = (a.d_Nout + 63) / 64;
    a.nbd = a.d_nbx * ((a.d_M + RBD - 1) / RBD);
  }
  int nbw = 0;
  if (a.w_slab) {
    // widest column-slot count that still gives >= ~1024 blocks (as slab_sum4_kernel's launcher)
    a.w_cb = (a.w_n4 >= 256LL * 1024 || a.w_S <= 1) ? 256 : (a.w_n4 >= 64LL * 1024 || a.w_S <= 4) ? 64 : 16;
    nbw = (int)((a.w_n4 + a.w_cb - 1) / a.w_cb);
  }
  if (a.nbd + nbw == 0) return;
  hipLaunchKernelGGL(bwd_reduce_kernel, dim3(a.nbd + nbw), dim3(256), 0, st, a);
}

}  // namespace cdp
