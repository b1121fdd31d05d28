// Small fused kernels: softmax cross-entropy (fwd / bwd / accuracy), fused SGD, CIFAR-style
// augmentation, weight transpose for conv data-gradients, stack-mean for the gather/scatter
// strategy, and generic scale / channel-sum helpers. gfx950, wave64.
//
// Reference anchors:
//   CrossEntropyLoss            /root/reference/src/Part 1/main.py:110,39
//   accuracy (max(1), eq, sum)  /root/reference/src/Part 1/main.py:70-71
//   optim.SGD(lr .1, mom .9, wd 1e-4)   /root/reference/src/Part 1/main.py:114-115
//   RandomCrop(32,4)+HFlip+Normalize    /root/reference/src/Part 1/main.py:82-93
//   torch.mean(torch.stack(inputs), 0)  /root/reference/src/Part 2a/main.py:122
#include <algorithm>
#include <stdexcept>

#include "act_max.h"
#include "common.h"
#include "kernels.h"
#include "x3_common.h"

namespace cdp {
namespace {

// ------------------------------------------------------------------ cross-entropy
// One block of 1024 threads. Narrow rows (C <= 64, e.g. CIFAR's 10 classes): one row per thread;
// wide rows (ImageNet's 1000): one row per wave. Per-row loss = logsumexp - logit[target]; the mean
// (fp64 block reduction, deterministic) and the top-1 correct count are written once.
__global__ __launch_bounds__(1024) void xent_fwd_kernel(const float* __restrict__ logits, const long long* __restrict__ tgt,
                                                       int B, int C, float* __restrict__ loss,
                                                       long long* __restrict__ correct, float* __restrict__ sum_out) {
  __shared__ double red[16];
  __shared__ int redc[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double acc = 0.0;
  int nc = 0;
  if (C <= 64) {
    for (int r = tid; r < B; r += 1024) {
      const float* row = logits + (long long)r * C;
      float mx = row[0];
      int am = 0;
      for (int c = 1; c < C; ++c) {
        const float v = row[c];
        if (v > mx) { mx = v; am = c; }
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(row[c] - mx);
      const long long t = tgt[r];
      const bool tok = t >= 0 && t < C;  // out-of-range targets poison the loss instead of reading OOB
      acc += tok ? (double)(logf(se) + mx - row[t]) : (double)NAN;
      nc += (tok && am == (int)t) ? 1 : 0;
    }
  } else if (C <= 1024) {
    // a wave's rows r = wid + 16 k (the loop below's assignment and order) four at a time, every
    // logit of the four loaded before the first is reduced: one memory round trip per four rows
    // (ResNet's 1000 classes: 40 -> a few us per call)
    constexpr int RB = 4, J = 16;
    for (int rb = wid; rb < B; rb += 16 * RB) {
      float v[RB][J];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = rb + 16 * k;
        const float* row = logits + (long long)(r < B ? r : 0) * C;
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int c = lane + 64 * j;
          v[k][j] = (r < B && c < C) ? row[c] : -INFINITY;
        }
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = rb + 16 * k;
        if (r >= B) break;
        float mx = -INFINITY;
        int am = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (v[k][j] > mx) { mx = v[k][j]; am = lane + 64 * j; }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float omx = __shfl_xor(mx, o, kWave);
          const int oam = __shfl_xor(am, o, kWave);
          if (omx > mx || (omx == mx && oam < am)) { mx = omx; am = oam; }
        }
        float se = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (lane + 64 * j < C) se += expf(v[k][j] - mx);
        se = wave_sum(se);
        if (lane == 0) {
          const long long t = tgt[r];
          const bool tok = t >= 0 && t < C;
          acc += tok ? (double)(logf(se) + mx - logits[(long long)r * C + t]) : (double)NAN;
          nc += (tok && am == (int)t) ? 1 : 0;
        }
      }
    }
  } else {
    for (int r = wid; r < B; r += 16) {
      const float* row = logits + (long long)r * C;
      float mx = -INFINITY;
      int am = 0x7fffffff;
      for (int c = lane; c < C; c += 64) {
        const float v = row[c];
        if (v > mx) { mx = v; am = c; }
      }
      // wave argmax: larger value wins, ties -> smaller index (first occurrence)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float omx = __shfl_xor(mx, o, kWave);
        const int oam = __shfl_xor(am, o, kWave);
        if (omx > mx || (omx == mx && oam < am)) { mx = omx; am = oam; }
      }
      float se = 0.f;
      for (int c = lane; c < C; c += 64) se += expf(row[c] - mx);
      se = wave_sum(se);
      if (lane == 0) {
        const long long t = tgt[r];
        const bool tok = t >= 0 && t < C;
        acc += tok ? (double)(logf(se) + mx - row[t]) : (double)NAN;
        nc += (tok && am == (int)t) ? 1 : 0;
      }
    }
  }
  acc = wave_sum_d(acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o, kWave);
  if (lane == 0) {
    red[wid] = acc;
    redc[wid] = nc;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    long long n = 0;
    for (int i = 0; i < 16; ++i) {
      s += red[i];
      n += redc[i];
    }
    if (loss) loss[0] = (float)(s / (double)B);
    if (sum_out) sum_out[0] = (float)s;
    if (correct) correct[0] += n;
  }
}

// dlogits = (softmax - onehot) * gscale[0] / B
__global__ __launch_bounds__(256) void xent_bwd_kernel(const float* __restrict__ logits, const long long* __restrict__ tgt,
                                                      const float* __restrict__ gscale, int B, int C,
                                                      float* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float* row = logits + (long long)r * C;
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, row[c]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += expf(row[c] - mx);
  se = wave_sum(se);
  const float k = gscale[0] / (float)B;
  const float inv = 1.f / se;
  const long long t = tgt[r];
  for (int c = lane; c < C; c += 64) {
    const float sm = expf(row[c] - mx) * inv;
    dlogits[(long long)r * C + c] = (sm - (c == t ? 1.f : 0.f)) * k;
  }
}

// ------------------------------------------------------------------ SGD (torch semantics)
// d_p = g*gs (+wd*p); buf = first ? d_p : buf*m + (1-damp)*d_p; d_p = nesterov ? d_p + m*buf : buf;
// p -= lr*d_p. Op order and fma placement follow ATen's add(alpha) (fmadd) so results match
// torch.optim.SGD to the last ulp on the same inputs.
__device__ __forceinline__ void sgd_one(float& p, float g, float& b, float lr, float m, float damp, float wd, float gs,
                                        bool nesterov, bool first, bool maximize, bool has_mom) {
  float d = g * gs;
  if (maximize) d = -d;
  if (wd != 0.f) d = fmaf(p, wd, d);
  if (has_mom) {
    if (first) b = d;
    else b = fmaf(d, 1.f - damp, b * m);
    d = nesterov ? fmaf(b, m, d) : b;
  }
  p = fmaf(d, -lr, p);
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                                                 long long n, const float* __restrict__ lr_ptr, float lr_host, float m,
                                                 float damp, float wd, float gs, int flags, long long* counter) {
  const bool nesterov = flags & 1, first = flags & 2, maximize = flags & 4, has_mom = flags & 8;
  // a data loader's step counter advanced by the step (one dispatch less per step; the counter is
  // read by this step's augment kernel, which ran before)
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) counter[0] += 1;
  const float lr = lr_ptr ? lr_ptr[0] : lr_host;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float dummy = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = ld4(p + 4 * i);
    const float4 gv = ld4(g + 4 * i);
    float4 bv = has_mom && !first ? ld4(buf + 4 * i) : f4zero();
    sgd_one(pv.x, gv.x, bv.x, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
    sgd_one(pv.y, gv.y, bv.y, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
    sgd_one(pv.z, gv.z, bv.z, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
    sgd_one(pv.w, gv.w, bv.w, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
    st4(p + 4 * i, pv);
    if (has_mom) st4(buf + 4 * i, bv);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    float bb = has_mom && !first ? buf[i] : 0.f;
    float pp = p[i];
    sgd_one(pp, g[i], has_mom ? bb : dummy, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
    p[i] = pp;
    if (has_mom) buf[i] = bb;
  }
}

// ------------------------------------------------------------------ weight maxima
// A 32x32 (co, ci) tile's contribution to its weight's maxima (weight_max_elems layout, kernels.h):
// the per-co partial of its ci block and the per-ci partial of its co block. Threads fold their
// values into s[0..32) (by co) and s[32..64) (by ci) with LDS atomics (zeroed by the caller before a
// barrier); after a barrier the first 64 threads store the 64 partials.
__device__ __forceinline__ void tile_max_add(unsigned* s, int co_local, int ci_local, float v) {
  const unsigned b = __float_as_uint(fabsf(v));
  if (b) {
    lds_max_u32(&s[co_local], b);
    lds_max_u32(&s[32 + ci_local], b);
  }
}
__device__ __forceinline__ void tile_max_store(const unsigned* s, float* __restrict__ wmax, int Co, int Ci, int co0,
                                               int ci0) {
  const int t = threadIdx.x;
  const int nci = (Ci + 31) / 32;
  if (t < 32 && co0 + t < Co) wmax[(long long)(ci0 / 32) * Co + co0 + t] = __uint_as_float(s[t]);
  else if (t >= 32 && t < 64 && ci0 + t - 32 < Ci)
    wmax[(long long)nci * Co + (long long)(co0 / 32) * Ci + ci0 + t - 32] = __uint_as_float(s[t]);
}

// ------------------------------------------------------------------ SGD + next-step weight preparation
// One pass over the parameter arena per step: the optimizer that writes W also emits what the next
// forward / backward GEMMs need from it (weight_prep_kernel's products): the f16x2 |max| partial of
// every 32x32 (co, ci) block and, where asked, W^T [ci][tap][co] (the data-gradient B operand).
// Blocks [0, nblk_w) own one (conv weight, co32, ci32) tile over all taps: load p / g / buf of the
// tile (branch-free buffer loads, TG taps per round trip), update exactly as sgd_kernel (same
// sgd_one), store p / buf in place, then the |max| and the transpose of the NEW p through LDS.
// Blocks [nblk_w, ...) each run sgd_kernel's float4 update over one chunk of the arena that no conv
// weight covers (biases, BatchNorm parameters, the classifier).
__global__ __launch_bounds__(256) void sgd_prep_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ buf, const SgdPrepSeg* __restrict__ segs,
                                                      int nseg, int nblk_w, const SgdPrepChunk* __restrict__ chunks,
                                                      float* __restrict__ part, const float* __restrict__ lr_ptr,
                                                      float lr_host, float m, float damp, float wd, float gs,
                                                      int flags, long long* counter) {
  // taps per group: 3 x 3 float4 in flight per thread keeps the kernel near 64 VGPRs (8 waves per
  // SIMD for this bandwidth-bound pass; a whole 3x3 filter per group held 256 VGPRs, 1 wave per SIMD)
  constexpr int TG = 3;
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) counter[0] += 1;  // as sgd_kernel
  __shared__ float tile[TG][32][33];
  __shared__ unsigned smax[64];
  const bool nesterov = flags & 1, first = flags & 2, maximize = flags & 4, has_mom = flags & 8;
  const float lr = lr_ptr ? lr_ptr[0] : lr_host;
  const int b = blockIdx.x;
  if (b >= nblk_w) {
    const SgdPrepChunk ch = chunks[b - nblk_w];
    for (int i = threadIdx.x; i < ch.n4; i += 256) {
      const long long e = ch.start + 4LL * i;
      float4 pv = ld4(p + e);
      const float4 gv = ld4(g + e);
      float4 bv = has_mom && !first ? ld4(buf + e) : f4zero();
      sgd_one(pv.x, gv.x, bv.x, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
      sgd_one(pv.y, gv.y, bv.y, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
      sgd_one(pv.z, gv.z, bv.z, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
      sgd_one(pv.w, gv.w, bv.w, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
      st4(p + e, pv);
      if (has_mom) st4(buf + e, bv);
    }
    return;
  }
  int si = 0;
  while (si + 1 < nseg && segs[si + 1].blk0 <= b) ++si;
  const SgdPrepSeg sg = segs[si];
  const int Co = sg.co, T = sg.t, Ci = sg.ci;
  float* __restrict__ wt = sg.wt;
  const int local = b - sg.blk0;
  const int nci = (Ci + 31) / 32;
  const int co0 = (local / nci) * 32, ci0 = (local % nci) * 32;
  const unsigned bytes = (unsigned)((long long)Co * T * Ci * 4);
  float* const pw = p + sg.off;
  float* const bw = buf ? buf + sg.off : nullptr;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(pw, bytes);
  const __amdgpu_buffer_rsrc_t gr = make_rsrc(g + sg.off, bytes);
  const __amdgpu_buffer_rsrc_t br = make_rsrc(has_mom && !first ? bw : pw, bytes);
  if (threadIdx.x < 64) smax[threadIdx.x] = 0u;
  __syncthreads();
  if ((Ci & 3) == 0) {
    float4 mx4 = f4zero();  // |max| of the NEW (co, ci .. ci + 3) values over the taps
    // float4 along ci: thread (co row tid / 8, ci quad tid % 8) of the 32 x 32 tile, one (co, tap)
    // row of 32 ci per 8 threads (128 B), every tap of the group; the transpose goes through LDS
    // and leaves as float4 runs of 4 co of W^T [ci][tap][co]
    const int rco = threadIdx.x >> 3, c4 = threadIdx.x & 7;
    const int co = co0 + rco, ci = ci0 + 4 * c4;
    const bool ok = co < Co && ci < Ci;
    for (int t0 = 0; t0 < T; t0 += TG) {
      float4 vp[TG], vg[TG], vb[TG];
      unsigned off[TG];
#pragma unroll
      for (int q = 0; q < TG; ++q) {
        off[q] = (ok && t0 + q < T) ? (unsigned)(((co * T + t0 + q) * Ci + ci) * 4) : kOOB;
        vp[q] = bload4(pr, off[q]);
        vg[q] = bload4(gr, off[q]);
        vb[q] = has_mom && !first ? bload4(br, off[q]) : f4zero();
      }
#pragma unroll
      for (int q = 0; q < TG; ++q) {
        sgd_one(vp[q].x, vg[q].x, vb[q].x, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
        sgd_one(vp[q].y, vg[q].y, vb[q].y, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
        sgd_one(vp[q].z, vg[q].z, vb[q].z, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
        sgd_one(vp[q].w, vg[q].w, vb[q].w, lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
        if (off[q] != kOOB) {
          st4(pw + (off[q] >> 2), vp[q]);
          if (has_mom) st4(bw + (off[q] >> 2), vb[q]);
          mx4 = make_float4(fmaxf(mx4.x, fabsf(vp[q].x)), fmaxf(mx4.y, fabsf(vp[q].y)), fmaxf(mx4.z, fabsf(vp[q].z)),
                            fmaxf(mx4.w, fabsf(vp[q].w)));
        }
      }
      if (wt) {
#pragma unroll
        for (int q = 0; q < TG; ++q) {
          tile[q][rco][4 * c4] = vp[q].x;
          tile[q][rco][4 * c4 + 1] = vp[q].y;
          tile[q][rco][4 * c4 + 2] = vp[q].z;
          tile[q][rco][4 * c4 + 3] = vp[q].w;
        }
        __syncthreads();
        // thread (ci row tid / 8, co quad tid % 8): W^T[ci][tap][co .. co + 3]
        const int rci = threadIdx.x >> 3, q4 = threadIdx.x & 7;
        const int ci_o = ci0 + rci, co_o = co0 + 4 * q4;
#pragma unroll
        for (int q = 0; q < TG; ++q) {
          const int tap = t0 + q;
          if (tap >= T) break;
          if (ci_o < Ci && co_o + 3 < Co) {
            st4(wt + ((long long)ci_o * T + tap) * Co + co_o,
                make_float4(tile[q][4 * q4][rci], tile[q][4 * q4 + 1][rci], tile[q][4 * q4 + 2][rci],
                            tile[q][4 * q4 + 3][rci]));
          } else if (ci_o < Ci) {
            for (int j = 0; j < 4 && co_o + j < Co; ++j)
              wt[((long long)ci_o * T + tap) * Co + co_o + j] = tile[q][4 * q4 + j][rci];
          }
        }
        __syncthreads();
      }
    }
    const float4 z = mx4;  // (this thread's co row rco, ci quad c4)
    tile_max_add(smax, rco, 4 * c4, z.x);
    tile_max_add(smax, rco, 4 * c4 + 1, z.y);
    tile_max_add(smax, rco, 4 * c4 + 2, z.z);
    tile_max_add(smax, rco, 4 * c4 + 3, z.w);
  } else {
    // Ci not a multiple of 4 (an RGB stem's 3 input channels): one element per lane
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    float mco[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t0 = 0; t0 < T; t0 += TG) {
      float vp[TG][4], vg[TG][4], vb[TG][4];
      unsigned off[TG][4];
#pragma unroll
      for (int q = 0; q < TG; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int co = co0 + ty + 8 * jj, ci = ci0 + tx, tap = t0 + q;
          off[q][jj] = (co < Co && ci < Ci && tap < T) ? (unsigned)(((co * T + tap) * Ci + ci) * 4) : kOOB;
          vp[q][jj] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)off[q][jj], 0, 0));
          vg[q][jj] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gr, (int)off[q][jj], 0, 0));
          vb[q][jj] = has_mom && !first
                          ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(br, (int)off[q][jj], 0, 0))
                          : 0.f;
        }
#pragma unroll
      for (int q = 0; q < TG; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          sgd_one(vp[q][jj], vg[q][jj], vb[q][jj], lr, m, damp, wd, gs, nesterov, first, maximize, has_mom);
          if (off[q][jj] != kOOB) {
            pw[off[q][jj] >> 2] = vp[q][jj];
            if (has_mom) bw[off[q][jj] >> 2] = vb[q][jj];
            mco[jj] = fmaxf(mco[jj], fabsf(vp[q][jj]));
          }
        }
      if (wt) {
#pragma unroll
        for (int q = 0; q < TG; ++q)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) tile[q][ty + 8 * jj][tx] = vp[q][jj];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TG; ++q) {
          const int tap = t0 + q;
          if (tap >= T) break;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int ci = ci0 + ty + 8 * jj, co = co0 + tx;
            if (ci < Ci && co < Co) wt[((long long)ci * T + tap) * Co + co] = tile[q][tx][ty + 8 * jj];
          }
        }
        __syncthreads();
      }
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) tile_max_add(smax, ty + 8 * jj, tx, mco[jj]);
  }
  __syncthreads();
  tile_max_store(smax, part + sg.pofs, Co, Ci, co0, ci0);
}

// ------------------------------------------------------------------ augmentation
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// out[b][h][w][c] (NHWC fp32) from uint8 HWC images[idx[b]], with optional RandomCrop(pad) and
// RandomHorizontalFlip(0.5) drawn from a counter-based hash of (seed, *counter, b), then
// ToTensor (/255) and Normalize(mean, std). Padding is zero in uint8 space (torchvision fill=0).
__global__ __launch_bounds__(256) void augment_kernel(const unsigned char* __restrict__ imgs,
                                                     const long long* __restrict__ idx, long long idx_off, int B,
                                                     int H, int W, int C, float m0, float m1, float m2, float is0,
                                                     float is1, float is2, int pad, int flip,
                                                     const long long* __restrict__ counter, unsigned long long seed,
                                                     float* __restrict__ out, long long nbatches,
                                                     const long long* __restrict__ labels,
                                                     long long* __restrict__ labels_out) {
  const int b = blockIdx.y;
  if (b >= B) return;
  const unsigned long long ctr = counter ? (unsigned long long)counter[0] : 0ull;
  // nbatches > 0: the batch offset into idx follows the step counter, so a replayed hipGraph walks
  // the epoch order without a host-side index copy per step
  const long long off = nbatches > 0 ? idx_off + (long long)(ctr % (unsigned long long)nbatches) * B : idx_off;
  const long long src_i = idx ? idx[off + b] : (off + b);
  if (labels_out && blockIdx.x == 0 && threadIdx.x == 0) labels_out[b] = labels[src_i];
  const unsigned long long r = splitmix64(seed ^ splitmix64(ctr * 0x100000001B3ull + (unsigned long long)b));
  const int span = 2 * pad + 1;
  const int oy = pad ? (int)(r % span) - pad : 0;
  const int ox = pad ? (int)((r >> 16) % span) - pad : 0;
  const bool fl = flip && ((r >> 40) & 1);
  const unsigned char* src = imgs + src_i * (long long)H * W * C;
  const float mean[3] = {m0, m1, m2};
  const float istd[3] = {is0, is1, is2};
  const int npix = H * W;
  float* dst = out + (long long)b * npix * C;
  // one thread per output pixel, all its channels (one index decode per pixel, not per element)
  for (int px = blockIdx.x * blockDim.x + threadIdx.x; px < npix; px += gridDim.x * blockDim.x) {
    const int h = px / W, w = px - (px / W) * W;
    const int ww = fl ? (W - 1 - w) : w;  // flip applied after the crop (torchvision order)
    const int sh = h + oy, sw = ww + ox;
    const bool in = (unsigned)sh < (unsigned)H && (unsigned)sw < (unsigned)W;
    const unsigned char* sp = src + (long long)(in ? sh * W + sw : 0) * C;
    for (int c = 0; c < C; ++c) {
      const float v = in ? (float)sp[c] * (1.f / 255.f) : 0.f;
      const int ci = c < 3 ? c : 2;
      dst[(long long)px * C + c] = (v - mean[ci]) * istd[ci];
    }
  }
}

__global__ void counter_inc_kernel(long long* c) { c[0] += 1; }

// dX of a stride-2 conv's sub-pixel parity classes with no filter taps (bit 2 ph + pw of mask):
// zeros, float4 along C (NHWC), one thread per float4 of the classes' pixels
__global__ __launch_bounds__(256) void subpixel_zero_kernel(float* __restrict__ dx, int N, int H, int W, int C4,
                                                            int mask, FastDiv fd_C4, FastDiv fd_W) {
  const long long total = (long long)N * H * W * C4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int pix = (int)(i / C4);  // < 2^31 pixels (launcher)
    const int t = fdiv(pix, fd_W);
    const int w = pix - t * W;
    const int h = t % H;
    if ((mask >> (2 * (h & 1) + (w & 1))) & 1) st4(dx + 4 * i, f4zero());
  }
}

// ------------------------------------------------------------------ weight transpose
// W[co][tap][ci] -> Wt[ci][tap][co]   (tap = kh*KW+kw; conv data-gradient uses Wt as its B^T)
__global__ __launch_bounds__(256) void wtrans_kernel(const float* __restrict__ w, float* __restrict__ wt, int Co,
                                                     int T, int Ci) {
  __shared__ float tile[32][33];
  const int tap = blockIdx.z;
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int j = ty; j < 32; j += 8) {
    const int co = co0 + j, ci = ci0 + tx;
    tile[j][tx] = (co < Co && ci < Ci) ? w[((long long)co * T + tap) * Ci + ci] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int ci = ci0 + j, co = co0 + tx;
    if (ci < Ci && co < Co) wt[((long long)ci * T + tap) * Co + co] = tile[tx][j];
  }
}

// ------------------------------------------------------------------ weight preparation
// One launch for all conv weights of a step (replaces a transpose launch per layer plus the
// |max| pass): block (segment, co32, ci32) walks the T taps of its 32x32 (co, ci) block, writes its
// per-co and per-ci |max| partials (the f16x2 operand scales of the weight's two GEMM roles) and,
// when asked, the tile transposed through LDS.
// Taps go in groups of TG: all of a group's loads are issued before any is used (branch-free: out
// of range elements read 0 through the buffer range check), so a 3x3 filter costs one memory round
// trip per block instead of nine.
__global__ __launch_bounds__(256) void weight_prep_kernel(WeightPrepArgs a, float* __restrict__ part) {
  constexpr int TG = 9;
  __shared__ float tile[TG][32][33];
  __shared__ unsigned smax[64];
  const int b = blockIdx.x;
  int seg = 0;
  while (seg + 1 < a.nseg && a.blk0[seg + 1] <= b) ++seg;
  const int Co = a.co[seg], T = a.t[seg], Ci = a.ci[seg];
  const float* __restrict__ w = a.w[seg];
  float* __restrict__ wt = a.wt[seg];
  const int local = b - a.blk0[seg];
  const int nci = (Ci + 31) / 32;
  const int co0 = (local / nci) * 32, ci0 = (local % nci) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(w, (unsigned)((long long)Co * T * Ci * 4));
  if (threadIdx.x < 64) smax[threadIdx.x] = 0u;
  __syncthreads();
  float mco[4] = {0.f, 0.f, 0.f, 0.f};  // |max| of (co0 + ty + 8 jj, ci0 + tx) over the taps
  for (int t0 = 0; t0 < T; t0 += TG) {
    float v[TG][4];
#pragma unroll
    for (int g = 0; g < TG; ++g)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int co = co0 + ty + 8 * jj, ci = ci0 + tx, tap = t0 + g;
        const unsigned o = (co < Co && ci < Ci && tap < T) ? (unsigned)(((co * T + tap) * Ci + ci) * 4) : kOOB;
        v[g][jj] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wr, (int)o, 0, 0));
      }
#pragma unroll
    for (int g = 0; g < TG; ++g)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mco[jj] = fmaxf(mco[jj], fabsf(v[g][jj]));
    if (wt) {
#pragma unroll
      for (int g = 0; g < TG; ++g)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) tile[g][ty + 8 * jj][tx] = v[g][jj];
      __syncthreads();
#pragma unroll
      for (int g = 0; g < TG; ++g) {
        const int tap = t0 + g;
        if (tap >= T) break;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int ci = ci0 + ty + 8 * jj, co = co0 + tx;
          if (ci < Ci && co < Co) wt[((long long)ci * T + tap) * Co + co] = tile[g][tx][ty + 8 * jj];
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) tile_max_add(smax, ty + 8 * jj, tx, mco[jj]);
  __syncthreads();
  tile_max_store(smax, part + a.pofs[seg], Co, Ci, co0, ci0);
}

// ------------------------------------------------------------------ channel padding
// out[p][0..C4) = (x[p][0..C), 0...) for NHWC pixels p: the RGB stem's 3 -> 4 channel padding in
// one pass (one float4 store per pixel) over a contiguous pixel range per block, plus the padded
// tensor's per-image / per-channel |max| (act_max.h) the f16x2 GEMM scales need.
__global__ __launch_bounds__(256) void pad_c4_kernel(const float* __restrict__ x, int N, long long HW, int C,
                                                     float* __restrict__ out, FastDiv fd_HW, ActMaxOut am) {
  __shared__ ActMaxBlock<4> sam;
  const bool want = am.img != nullptr;
  const long long npix = (long long)N * HW;
  const long long per = (npix + gridDim.x - 1) / gridDim.x;
  const long long p0 = (long long)blockIdx.x * per, p1 = min(npix, p0 + per);
  const int img0 = (int)(min(p0, npix - 1) / HW);
  if (want) {
    sam.init(threadIdx.x, 256);
    __syncthreads();
  }
  ImgRun run;
  float4 cm = f4zero();
  for (long long p = p0 + threadIdx.x; p < p1; p += 256) {
    const float* src = x + p * C;
    float v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = c < C ? src[c] : 0.f;
    const float4 z = make_float4(v[0], v[1], v[2], v[3]);
    st4(out + p * 4, z);
    if (want) {
      run.add(fdiv((int)p, fd_HW), absmax4(z), sam, img0, am);
      cm = absmax4(cm, z);
    }
  }
  if (want) {
    run.flush(sam, img0, am);
    sam.add_ch4(0, cm);
    __syncthreads();
    sam.publish(am, img0, N, 0, 4, 4, blockIdx.x % kActCopies, threadIdx.x, 256);
  }
}

// ------------------------------------------------------------------ stack mean / scale / colsum
struct StackSrcs {
  const float* p[kMaxStackSrcs];
};
__global__ __launch_bounds__(256) void stack_mean_kernel(StackSrcs srcs, int k, long long n, float* __restrict__ dst) {
  const float inv = 1.f / (float)k;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < k; ++j) s += srcs.p[j][i];
    dst[i] = s * inv;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, long long n, float a) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] *= a;
}

// out[c] (+)= sum_r x[r][c]   (Linear bias gradient)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ x, int R, int C, float* __restrict__ out,
                                                     int accumulate) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < C)
    for (int r = rl; r < R; r += 4) s += x[(long long)r * C + c];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < C) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// ------------------------------------------------------------------ narrow Linear (classifier heads)
// O <= 16 outputs (VGG-11's fc1 is 512 -> 10: a 128x128 MFMA tile would be >90% padding).
constexpr int SL_MAXO = 16;

// y[r][o] = x[r] . W[o] + b[o]: one wave per row; each lane keeps its slice of x in registers,
// accumulates all O partial dot products, and the wave reduces them through LDS once.
__global__ __launch_bounds__(256) void small_linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ b, int B, int I, int O,
                                                               float* __restrict__ y) {
  __shared__ float red[4][SL_MAXO][65];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wv;
  float part[SL_MAXO];
#pragma unroll
  for (int o = 0; o < SL_MAXO; ++o) part[o] = 0.f;
  if (r < B) {
    const float* xr = x + (long long)r * I;
    for (int i = lane; i < I; i += 64) {
      const float xv = xr[i];
      // no per-o branch: clamped rows keep every load unconditional (a runtime-predicated load per
      // element makes hipcc wait vmcnt(0) around each one); rows >= O are never stored
#pragma unroll
      for (int o = 0; o < SL_MAXO; ++o) part[o] = fmaf(xv, w[(long long)min(o, O - 1) * I + i], part[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < SL_MAXO; ++o) red[wv][o][lane] = part[o];
  __syncthreads();
  if (r < B && lane < O) {
    float s = 0.f;
    for (int k = 0; k < 64; ++k) s += red[wv][lane][k];
    y[(long long)r * O + lane] = s + (b ? b[lane] : 0.f);
  }
}

// One launch for all three gradients:
//   blocks [0, nbx)          dX[r][i] = sum_o dy[r][o] * W[o][i]       (thread per element)
//   blocks [nbx, nbx + nbw)  dW[o][i] = sum_r dy[r][o] * x[r][i]       (16 columns x 16 row-lanes per
//                            block; every thread accumulates all O outputs of its column)
//   last block               db[o]    = sum_r dy[r][o]
// (dy: global memory, or the block's LDS copy in xent_linear_bwd_kernel)
__device__ __forceinline__ void small_linear_bwd_body(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ w, int B, int I, int O,
                                                      float* __restrict__ dx, float* __restrict__ dw,
                                                      float* __restrict__ db, int nbx, int nbw, int bid) {
  __shared__ float red[16][SL_MAXO][17];
  if (bid < nbx) {
    const long long e = (long long)bid * 256 + threadIdx.x;
    if (e >= (long long)B * I) return;
    const int r = (int)(e / I), i = (int)(e % I);
    float s = 0.f;
    for (int o = 0; o < O; ++o) s = fmaf(dy[(long long)r * O + o], w[(long long)o * I + i], s);
    dx[e] = s;
  } else if (bid < nbx + nbw) {
    const int col = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int i = (bid - nbx) * 16 + col;
    float acc[SL_MAXO];
#pragma unroll
    for (int o = 0; o < SL_MAXO; ++o) acc[o] = 0.f;
    if (i < I) {
      for (int r = rl; r < B; r += 16) {
        const float xv = x[(long long)r * I + i];
#pragma unroll
        for (int o = 0; o < SL_MAXO; ++o) acc[o] = fmaf(dy[(long long)r * O + min(o, O - 1)], xv, acc[o]);
      }
    }
#pragma unroll
    for (int o = 0; o < SL_MAXO; ++o) red[rl][o][col] = acc[o];
    __syncthreads();
    // 256 threads finish 16 columns x O outputs
    const int o = threadIdx.x >> 4;
    if (o < O && i - col + (threadIdx.x & 15) < I) {
      const int c = threadIdx.x & 15;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red[k][o][c];
      dw[(long long)o * I + (bid - nbx) * 16 + c] = s;
    }
  } else if (db) {
    __shared__ float rdb[4][64];
    const int o = threadIdx.x & 63, rl = threadIdx.x >> 6;
    float s = 0.f;
    if (o < O)
      for (int r = rl; r < B; r += 4) s += dy[(long long)r * O + o];
    rdb[rl][o] = s;
    __syncthreads();
    if (rl == 0 && o < O) db[o] = rdb[0][o] + rdb[1][o] + rdb[2][o] + rdb[3][o];
  }
}

__global__ __launch_bounds__(256) void small_linear_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                               const float* __restrict__ w, int B, int I, int O,
                                                               float* __restrict__ dx, float* __restrict__ dw,
                                                               float* __restrict__ db, int nbx, int nbw) {
  small_linear_bwd_body(dy, x, w, B, I, O, dx, dw, db, nbx, nbw, blockIdx.x);
}

// The classifier's backward in one launch (CrossEntropyLoss -> Linear(512, 10), the reference's
// fc1 + criterion, /root/reference/src/Part 1/model.py:40-45 with main.py:39-40,110): every block
// first forms dlogits = (softmax(logits) - onehot(t)) * gscale / B for all B rows in its LDS (one
// thread per row, O <= 16 classes), block 0 also stores it (the loss's gradient autograd passes on),
// then the block does its part of the narrow Linear's gradients:
//   blocks [0, nbx)          16 columns i of dX x 32 rows (16 row lanes x 16 columns), each
//                            dX[r][i] = sum_o dy[r][o] W[o][i] in small_linear_bwd_body's order; with a
//                            BatchNorm link (lk.y != null: the input is the last VGG block's pooled,
//                            1x1 output, so column i is channel i) the block also reduces that block's
//                            BN backward partials from the dX it just formed -- sum dz, sum dz * xhat,
//                            sum xhat over each 2x2 window through max-pool + ReLU, as bn_bwd_reduce --
//                            into part[row chunk][i][0..ps), so the block's backward takes them instead of a
//                            statistics launch of its own (ops/functional.py _BNLink)
//   blocks [nbx, nbx + nbw)  dW, last block db (small_linear_bwd_body)
// Three launches (xent_bwd, small_linear_bwd, bn_bwd_reduce) and two kernel boundaries less per step.
__global__ __launch_bounds__(256) void xent_linear_bwd_kernel(const float* __restrict__ logits,
                                                              const long long* __restrict__ tgt,
                                                              const float* __restrict__ gscale,
                                                              const float* __restrict__ x, const float* __restrict__ w,
                                                              int B, int I, int O, float* __restrict__ dlogits,
                                                              float* __restrict__ dx, float* __restrict__ dw,
                                                              float* __restrict__ db, int nbx, int nbw, XentBnLink lk) {
  __shared__ float sdy[kXentLinMax];
  const float k = gscale[0] / (float)B;
  for (int r = threadIdx.x; r < B; r += 256) {
    const float* row = logits + (long long)r * O;
    float v[SL_MAXO];
    float mx = -INFINITY;
#pragma unroll
    for (int o = 0; o < SL_MAXO; ++o) {
      v[o] = o < O ? row[o] : -INFINITY;
      mx = fmaxf(mx, v[o]);
    }
    float se = 0.f;
#pragma unroll
    for (int o = 0; o < SL_MAXO; ++o)
      if (o < O) se += expf(v[o] - mx);
    const float inv = 1.f / se;
    const long long t = tgt[r];
#pragma unroll
    for (int o = 0; o < SL_MAXO; ++o) {
      if (o >= O) break;
      const float d = (expf(v[o] - mx) * inv - (o == t ? 1.f : 0.f)) * k;
      sdy[r * O + o] = d;
      if (blockIdx.x == 0) dlogits[(long long)r * O + o] = d;
    }
  }
  __syncthreads();
  if ((int)blockIdx.x >= nbx) {
    small_linear_bwd_body(sdy, x, w, B, I, O, nullptr, dw, db, 0, nbw, blockIdx.x - nbx);
    return;
  }
  __shared__ float red[3][16][17];
  const int col = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int ncol = (I + 15) / 16;
  const int chunk = blockIdx.x / ncol;  // rows [32 chunk, 32 chunk + 32): the BN partial index
  const int i = (blockIdx.x - chunk * ncol) * 16 + col;
  const bool ok = i < I;
  const int rend = min(B, kXentLinRows * (chunk + 1));
  float wc[SL_MAXO];
#pragma unroll
  for (int o = 0; o < SL_MAXO; ++o) wc[o] = ok ? w[(long long)min(o, O - 1) * I + i] : 0.f;
  float a1 = 0.f, a2 = 0.f, a3 = 0.f;
  float sc = 0.f, sh = 0.f, mu = 0.f, is = 0.f;
  const bool link = lk.y != nullptr && ok;
  if (link) {
    mu = lk.stats[i];
    is = lk.stats[I + i];
    sc = lk.stats[2 * I + i];
    sh = lk.stats[3 * I + i];
  }
  for (int r = kXentLinRows * chunk + rl; r < rend && ok; r += 16) {
    float s = 0.f;
    for (int o = 0; o < O; ++o) s = fmaf(sdy[r * O + o], wc[o], s);
    dx[(long long)r * I + i] = s;
    if (link) {
      // the block's 2x2 pre-BN window of channel i (lk.H = lk.W = 2) or its single pixel
      const int np = lk.pool ? 4 : 1;
      float yv[4], z[4], d[4];
      for (int p = 0; p < np; ++p) {
        yv[p] = lk.y[((long long)r * np + p) * I + i];  // NHWC, pixels (0,0),(0,1),(1,0),(1,1)
        z[p] = fmaf(yv[p], sc, sh);
        if (lk.relu) z[p] = fmaxf(z[p], 0.f);
      }
      if (lk.pool) {
        int arg = 0;
        float m = z[0];
        if (z[1] > m) { m = z[1]; arg = 1; }
        if (z[2] > m) { m = z[2]; arg = 2; }
        if (z[3] > m) { m = z[3]; arg = 3; }
        const float gg = (!lk.relu || m > 0.f) ? s : 0.f;
        for (int p = 0; p < 4; ++p) d[p] = arg == p ? gg : 0.f;
      } else {
        d[0] = (!lk.relu || z[0] > 0.f) ? s : 0.f;
      }
      for (int p = 0; p < np; ++p) {
        const float xh = (yv[p] - mu) * is;
        a1 += d[p];
        a2 += d[p] * xh;
        a3 += xh;
      }
    }
  }
  if (lk.y == nullptr) return;  // (uniform over the block)
  red[0][rl][col] = a1;
  red[1][rl][col] = a2;
  red[2][rl][col] = a3;
  __syncthreads();
  if (rl < lk.ps && ok) {
    float t = 0.f;
    for (int q = 0; q < 16; ++q) t += red[rl][q][col];
    lk.part[((long long)chunk * I + i) * lk.ps + rl] = t;
  }
}

// global average pool over HW of NHWC -> [N][C]; and its backward (32-bit index decode by
// multiply-shift: the launchers check the sizes)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const float* __restrict__ x, int N, int HW, int C,
                                                          float* __restrict__ y, FastDiv fd_C) {
  const int total = N * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int n = fdiv(i, fd_C);
    const int c = i - n * C;
    float s = 0.f;
    for (int k = 0; k < HW; ++k) s += x[((long long)n * HW + k) * C + c];
    y[i] = s / (float)HW;
  }
}
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ gy, int N, int HW, int C,
                                                          float* __restrict__ gx, FastDiv fd_C, FastDiv fd_HW) {
  const int total = N * HW * C;
  const float inv = 1.f / (float)HW;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int pix = fdiv(i, fd_C);
    const int c = i - pix * C;
    const int n = fdiv(pix, fd_HW);
    gx[i] = gy[n * C + c] * inv;
  }
}

// MaxPool2d(k, s, p) forward on NHWC with int32 argmax (flat h*W+w), and backward (scatter-add).
// Max-pool on NHWC, float4 along C. The argmax is kept as the window-local tap index (uint8,
// first max wins in (dh, dw) scan order like ATen), a quarter of an int32 index map.
// 32-bit indices with multiply-shift division (the launchers check the sizes): the 64-bit divisions
// the index decode took before were ~40 instructions each, four per element, in passes that are
// otherwise bandwidth-bound
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C,
                                                          int k, int s, int pd, int Ho, int Wo, float* __restrict__ y,
                                                          unsigned char* __restrict__ arg, FastDiv fd_C4, FastDiv fd_Wo,
                                                          FastDiv fd_Ho) {
  const int C4 = C >> 2;
  const int total = N * Ho * Wo * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int pix = fdiv(i, fd_C4);
    const int c4 = i - pix * C4;
    const int t = fdiv(pix, fd_Wo);
    const int wo = pix - t * Wo;
    const int n = fdiv(t, fd_Ho);
    const int ho = t - n * Ho;
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int am[4] = {-1, -1, -1, -1};
    const float* base = x + (long long)n * H * W * C + 4 * c4;
    for (int dh = 0; dh < k; ++dh) {
      const int h = ho * s - pd + dh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int w = wo * s - pd + dw;
        if ((unsigned)w >= (unsigned)W) continue;
        const float4 v = ld4(base + ((long long)h * W + w) * C);
        const float vv[4] = {v.x, v.y, v.z, v.w};
        const int tap = dh * k + dw;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (vv[e] > m[e] || am[e] < 0) {
            m[e] = vv[e];
            am[e] = tap;
          }
      }
    }
    st4(y + (long long)pix * C + 4 * c4, make_float4(m[0], m[1], m[2], m[3]));
    *reinterpret_cast<uchar4*>(arg + (long long)pix * C + 4 * c4) =
        make_uchar4((unsigned char)am[0], (unsigned char)am[1], (unsigned char)am[2], (unsigned char)am[3]);
  }
}

// Gather form of the backward (no atomics, no zero fill): every input element sums the gradients
// of the windows that cover it and whose argmax tap is this element.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ gy,
                                                          const unsigned char* __restrict__ arg, int N, int H, int W,
                                                          int C, int k, int s, int pd, int Ho, int Wo,
                                                          float* __restrict__ gx, FastDiv fd_C4, FastDiv fd_W,
                                                          FastDiv fd_H) {
  const int C4 = C >> 2;
  const int total = N * H * W * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int pix = fdiv(i, fd_C4);
    const int c4 = i - pix * C4;
    const int t = fdiv(pix, fd_W);
    const int w = pix - t * W;
    const int n = fdiv(t, fd_H);
    const int h = t - n * H;
    // windows ho with ho*s - pd <= h <= ho*s - pd + k - 1
    const int ho0 = max(0, (h + pd - k + s) / s), ho1 = min(Ho - 1, (h + pd) / s);
    const int wo0 = max(0, (w + pd - k + s) / s), wo1 = min(Wo - 1, (w + pd) / s);
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ho = ho0; ho <= ho1; ++ho)
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int tap = (h - (ho * s - pd)) * k + (w - (wo * s - pd));
        const long long o = (((long long)n * Ho + ho) * Wo + wo) * C + 4 * c4;
        const uchar4 a = *reinterpret_cast<const uchar4*>(arg + o);
        const float4 v = ld4(gy + o);
        if (a.x == tap) g[0] += v.x;
        if (a.y == tap) g[1] += v.y;
        if (a.z == tap) g[2] += v.z;
        if (a.w == tap) g[3] += v.w;
      }
    st4(gx + (long long)pix * C + 4 * c4, make_float4(g[0], g[1], g[2], g[3]));
  }
}

int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}



// sub-filter transpose for the sub-pixel data gradient: wt[ci][a][b][co] = w[co][kh0+2a][kw0+2b][ci]
__global__ __launch_bounds__(256) void wtrans_sub_kernel(const float* __restrict__ w, float* __restrict__ wt, int Co,
                                                         int KH, int KW, int Ci, int kh0, int kw0, int nkw) {
  __shared__ float tile[32][33];
  const int t = blockIdx.z;  // sub-tap a * nkw + b
  const int tap_in = (kh0 + 2 * (t / nkw)) * KW + kw0 + 2 * (t % nkw);
  const int T_in = KH * KW, T_out = gridDim.z;
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int co = co0 + j, ci = ci0 + tx;
    tile[j][tx] = (co < Co && ci < Ci) ? w[((long long)co * T_in + tap_in) * Ci + ci] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int ci = ci0 + j, co = co0 + tx;
    if (ci < Ci && co < Co) wt[((long long)ci * T_out + t) * Co + co] = tile[tx][j];
  }
}
}  // namespace

void xent_fwd_launch(const float* logits, const long long* tgt, int B, int C, float* loss, long long* correct,
                     float* sum_out, hipStream_t st) {
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(1), dim3(1024), 0, st, logits, tgt, B, C, loss, correct, sum_out);
}
void xent_bwd_launch(const float* logits, const long long* tgt, const float* gscale, int B, int C, float* dlogits,
                     hipStream_t st) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, logits, tgt, gscale, B, C, dlogits);
}
void sgd_launch(float* p, const float* g, float* buf, long long n, const float* lr_ptr, float lr, float momentum,
                float dampening, float wd, float grad_scale, bool nesterov, bool first, bool maximize,
                hipStream_t st, long long* counter) {
  const int flags = (nesterov ? 1 : 0) | (first ? 2 : 0) | (maximize ? 4 : 0) | (momentum != 0.f ? 8 : 0);
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, p, g, buf, n, lr_ptr, lr, momentum,
                     dampening, wd, grad_scale, flags, counter);
}
void sgd_prep_launch(float* p, const float* g, float* buf, const SgdPrepSeg* segs, int nseg, int nblk_w,
                     const SgdPrepChunk* chunks, int nchunk, float* wmax, const float* lr_ptr, float lr,
                     float momentum, float dampening, float wd, float grad_scale, bool nesterov, bool first,
                     bool maximize, hipStream_t st, long long* counter) {
  const int flags = (nesterov ? 1 : 0) | (first ? 2 : 0) | (maximize ? 4 : 0) | (momentum != 0.f ? 8 : 0);
  if (nblk_w + nchunk <= 0) return;
  hipLaunchKernelGGL(sgd_prep_kernel, dim3(nblk_w + nchunk), dim3(256), 0, st, p, g, buf, segs, nseg, nblk_w, chunks,
                     wmax, lr_ptr, lr, momentum, dampening, wd, grad_scale, flags, counter);
}
void augment_launch(const unsigned char* imgs, const long long* idx, long long idx_off, int B, int H, int W, int C,
                    const float* mean, const float* inv_std, int pad, bool flip, const long long* counter,
                    unsigned long long seed, float* out, hipStream_t st, long long nbatches,
                    const long long* labels, long long* labels_out) {
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(augment_kernel, grid, dim3(256), 0, st, imgs, idx, idx_off, B, H, W, C, mean[0], mean[1],
                     mean[2], inv_std[0], inv_std[1], inv_std[2], pad, flip ? 1 : 0, counter, seed, out, nbatches,
                     labels, labels_out);
}
void subpixel_zero_launch(float* dx, int N, int H, int W, int C, int mask, hipStream_t st) {
  if ((long long)N * H * W >= (1LL << 31) || (C & 3)) throw std::runtime_error("subpixel_zero: bad shape");
  const long long n4 = (long long)N * H * W * (C / 4);
  hipLaunchKernelGGL(subpixel_zero_kernel, dim3(grid_for(n4)), dim3(256), 0, st, dx, N, H, W, C / 4, mask,
                     make_fastdiv(C / 4), make_fastdiv(W));
}
// Zero-fill as a kernel (act-max slot chunks, ops.cpp alloc_slots): a kernel node of a captured
// graph is ordered like every other kernel of the step
__global__ __launch_bounds__(256) void fill_u32_kernel(unsigned* __restrict__ p, long long n, unsigned v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ __launch_bounds__(256) void fill_u32x4_kernel(uint4* __restrict__ p, long long n4, unsigned v) {
  const uint4 q = make_uint4(v, v, v, v);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
    p[i] = q;
}
void fill_u32_launch(unsigned* p, long long n, unsigned v, hipStream_t st) {
  if (n <= 0) return;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0 && (n & 3) == 0) {  // 16-B stores (slot chunks: 256-B multiples)
    const long long n4 = n / 4, blocks = std::min<long long>(512, (n4 + 255) / 256);
    hipLaunchKernelGGL(fill_u32x4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<uint4*>(p), n4, v);
    return;
  }
  const long long blocks = std::min<long long>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(fill_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, n, v);
}
// Device-to-device copy as a kernel (the root's own block of the grouped gather / scatter): inside a
// captured step a kernel node is ordered like the collectives around it (a captured memset node was
// measured to race, see fill_u32_kernel)
__global__ __launch_bounds__(256) void copy16_kernel(uint4* __restrict__ d, const uint4* __restrict__ s, long long n16) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x)
    d[i] = s[i];
}
__global__ __launch_bounds__(256) void copy1_kernel(unsigned char* __restrict__ d, const unsigned char* __restrict__ s,
                                                    long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    d[i] = s[i];
}
void copy_bytes_launch(void* dst, const void* src, long long bytes, hipStream_t st) {
  if (bytes <= 0) return;
  const bool wide = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | (uintptr_t)bytes) & 15) == 0;
  const long long n = wide ? bytes / 16 : bytes;
  const long long blocks = std::max<long long>(1, std::min<long long>(2048, (n + 255) / 256));
  if (wide)
    hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<uint4*>(dst),
                       static_cast<const uint4*>(src), n);
  else
    hipLaunchKernelGGL(copy1_kernel, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<unsigned char*>(dst),
                       static_cast<const unsigned char*>(src), n);
}
void counter_inc_launch(long long* c, hipStream_t st) {
  hipLaunchKernelGGL(counter_inc_kernel, dim3(1), dim3(1), 0, st, c);
}
void weight_prep_launch(const WeightPrepArgs& a, float* part, hipStream_t st) {
  hipLaunchKernelGGL(weight_prep_kernel, dim3(a.blk0[a.nseg]), dim3(256), 0, st, a, part);
}
void wtrans_launch(const float* w, float* wt, int Co, int T, int Ci, hipStream_t st) {
  dim3 grid((Ci + 31) / 32, (Co + 31) / 32, T);
  hipLaunchKernelGGL(wtrans_kernel, grid, dim3(256), 0, st, w, wt, Co, T, Ci);
}
void pad_c4_launch(const float* x, int N, long long HW, int C, float* out, ActMaxOut am, hipStream_t st) {
  const long long npix = (long long)N * HW;
  const int grid = (int)std::min<long long>(1024, std::max<long long>(1, (npix + 255) / 256));
  hipLaunchKernelGGL(pad_c4_kernel, dim3(grid), dim3(256), 0, st, x, N, HW, C, out, make_fastdiv((int)HW), am);
}
void stack_mean_launch(const float* const* srcs, int k, long long n, float* dst, hipStream_t st) {
  StackSrcs a{};
  for (int j = 0; j < k && j < kMaxStackSrcs; ++j) a.p[j] = srcs[j];
  hipLaunchKernelGGL(stack_mean_kernel, dim3(grid_for(n)), dim3(256), 0, st, a, k < kMaxStackSrcs ? k : kMaxStackSrcs, n,
                     dst);
}
// Test-only post-op (RcclComm::set_test_postop): every wave first idles ~delay_us with s_sleep
// (no memory traffic), then scales. Used to prove that consumers wait on the collective's event.
__global__ __launch_bounds__(256) void delay_scale_kernel(float* __restrict__ x, long long n, float a, int sleeps) {
  for (int i = 0; i < sleeps; ++i) __builtin_amdgcn_s_sleep(127);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] *= a;
}

// One thread writes the GPU's constant-rate wall clock (s_memrealtime, 100 MHz) into ts[idx]:
// a stream-ordered timestamp far cheaper than a timing event (which ends in a release barrier).
__global__ void timestamp_kernel(long long* ts, int idx) { ts[idx] = (long long)wall_clock64(); }

void timestamp_launch(long long* ts, int idx, hipStream_t st) {
  hipLaunchKernelGGL(timestamp_kernel, dim3(1), dim3(1), 0, st, ts, idx);
}

void delay_scale_launch(float* x, long long n, float a, double delay_us, hipStream_t st) {
  // s_sleep 127 ~ 127*64 cycles ~ 3.4 us at 2.4 GHz
  const int sleeps = (int)(delay_us / 3.4) + 1;
  if (a == 1.f) {
    // a pure delay (the modelled all-reduce time): 16 sleeping workgroups, about the CUs an RCCL
    // all-reduce's channels occupy, so the compute stream keeps the rest of the chip
    hipLaunchKernelGGL(delay_scale_kernel, dim3(16), dim3(64), 0, st, x, 0LL, a, sleeps);
    return;
  }
  hipLaunchKernelGGL(delay_scale_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, a, sleeps);
}
void scale_launch(float* x, long long n, float a, hipStream_t st) {
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, a);
}
void colsum_launch(const float* x, int R, int C, float* out, bool accumulate, hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 63) / 64), dim3(256), 0, st, x, R, C, out, accumulate ? 1 : 0);
}
void small_linear_fwd_launch(const float* x, const float* w, const float* b, int B, int I, int O, float* y,
                             hipStream_t st) {
  hipLaunchKernelGGL(small_linear_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, x, w, b, B, I, O, y);
}
void small_linear_bwd_launch(const float* dy, const float* x, const float* w, int B, int I, int O, float* dx, float* dw,
                             float* db, hipStream_t st) {
  const int nbx = dx ? (int)(((long long)B * I + 255) / 256) : 0;
  const int nbw = (I + 15) / 16;
  hipLaunchKernelGGL(small_linear_bwd_kernel, dim3(nbx + nbw + 1), dim3(256), 0, st, dy, x, w, B, I, O, dx, dw, db,
                     nbx, nbw);
}
void xent_linear_bwd_launch(const float* logits, const long long* tgt, const float* gscale, const float* x,
                            const float* w, int B, int I, int O, float* dlogits, float* dx, float* dw, float* db,
                            const XentBnLink& lk, hipStream_t st) {
  if (O > SL_MAXO || (long long)B * O > kXentLinMax) throw std::runtime_error("xent_linear_bwd: classifier too wide");
  if (lk.y && (!dx || lk.ps < 2 || lk.ps > 3)) throw std::runtime_error("xent_linear_bwd: BN link needs dX");
  const int nbx = dx ? ((I + 15) / 16) * xent_lin_chunks(B) : 0;
  const int nbw = (I + 15) / 16;
  hipLaunchKernelGGL(xent_linear_bwd_kernel, dim3(nbx + nbw + 1), dim3(256), 0, st, logits, tgt, gscale, x, w, B, I, O,
                     dlogits, dx, dw, db, nbx, nbw, lk);
}
void avgpool_fwd_launch(const float* x, int N, int HW, int C, float* y, hipStream_t st) {
  if ((long long)N * HW * C >= (1LL << 31)) throw std::runtime_error("avgpool: tensor too large");
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_for((long long)N * C)), dim3(256), 0, st, x, N, HW, C, y,
                     make_fastdiv(C));
}
void avgpool_bwd_launch(const float* gy, int N, int HW, int C, float* gx, hipStream_t st) {
  if ((long long)N * HW * C >= (1LL << 31)) throw std::runtime_error("avgpool: tensor too large");
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long long)N * HW * C)), dim3(256), 0, st, gy, N, HW, C, gx,
                     make_fastdiv(C), make_fastdiv(HW));
}
void maxpool_fwd_launch(const float* x, int N, int H, int W, int C, int k, int s, int p, int Ho, int Wo, float* y,
                        unsigned char* arg, hipStream_t st) {
  if ((long long)N * H * W * (C / 4) >= (1LL << 31)) throw std::runtime_error("maxpool: tensor too large");
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((long long)N * Ho * Wo * (C / 4))), dim3(256), 0, st, x, N,
                     H, W, C, k, s, p, Ho, Wo, y, arg, make_fastdiv(C / 4), make_fastdiv(Wo), make_fastdiv(Ho));
}
void maxpool_bwd_launch(const float* gy, const unsigned char* arg, int N, int H, int W, int C, int k, int s, int p,
                        int Ho, int Wo, float* gx, hipStream_t st) {
  if ((long long)N * H * W * (C / 4) >= (1LL << 31)) throw std::runtime_error("maxpool: tensor too large");
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for((long long)N * H * W * (C / 4))), dim3(256), 0, st, gy, arg,
                     N, H, W, C, k, s, p, Ho, Wo, gx, make_fastdiv(C / 4), make_fastdiv(W), make_fastdiv(H));
}

void wtrans_sub_launch(const float* w, float* wt, int Co, int KH, int KW, int Ci, int kh0, int kw0, int nkh, int nkw,
                       hipStream_t st) {
  dim3 grid((Ci + 31) / 32, (Co + 31) / 32, nkh * nkw);
  hipLaunchKernelGGL(wtrans_sub_kernel, grid, dim3(256), 0, st, w, wt, Co, KH, KW, Ci, kh0, kw0, nkw);
}

}  // namespace cdp
