// Channel-owner fusion of the split-K reduction with the BatchNorm that follows it, for layers
// with few output rows (the deep VGG layers; every layer past the first two at 32 images per GPU),
// gfx950. Reference block: Conv2d -> BatchNorm2d -> ReLU [-> MaxPool2d(2,2)],
// /root/reference/src/Part 1/model.py:11-27.
//
// BatchNorm needs a reduction over all M rows of a channel before anything can be applied, so the
// split-K path takes three dependent launches per layer: the GEMM writes slabs, a row-blocked
// reduction sums them and emits per-row-block statistics partials, and a finalize+apply launch
// merges the partials and writes the activation. A device-wide barrier is not cheaper than a
// launch on MI355X (docs/PERF.md: every block has to write back / invalidate its XCD's L2).
// Here a workgroup instead owns 16 channels for ALL rows (512 threads = 4 channel quads x 128 row
// lanes, up to 16 rows each in registers), so the whole reduction -> statistics -> apply chain is
// block-local: one launch after the GEMM instead of two. Channels are independent, so there is no
// cross-block traffic. (16 channels = 64 B per row and lane group: with one quad per block (16 B
// per row, 64 rows = 64 cache lines per wave instruction) the same launches ran 3x slower.)
//
//   chan_fwd_kernel:  y = sum_z slab[z] + bias (saved for backward); mean / var over the block's
//                     rows (two-pass, fp64 merge); running statistics; out = [pool2](relu(BN(y)));
//                     per-block |max| of out (the next GEMM's f16x2 operand scale).
//   chan_bwd_kernel:  job D -- dX = sum_z slab_D[z] (the gradient at block L's output, written for
//                     autograd), block L's BN backward sums with the pool / ReLU routing recomputed
//                     from block L's saved y, dgamma / dbeta / conv-bias gradient, and
//                     dy = scale * (dz - mean(dz) - xhat * mean(dz * xhat)) with its |max|;
//                     job W -- dW = sum_z slab_W[z] (the block's weight gradient), in the same
//                     launch as bwd_reduce_kernel does.
// Summation orders are fixed, so results are deterministic.
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "x3_common.h"

namespace cdp {
namespace {

constexpr int NT = 512;  // threads per block (8 waves)
constexpr int NW = NT / 64;
constexpr int CQ = 4;         // channel quads per block
constexpr int CB = 4 * CQ;    // channels per block
constexpr int RL = NT / CQ;   // row lanes

__device__ __forceinline__ float4 f4add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float f4c(const float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int j, float a) {
  if (j == 0) v.x = a;
  else if (j == 1) v.y = a;
  else if (j == 2) v.z = a;
  else v.w = a;
}
__device__ __forceinline__ float4 act4(float4 y, float4 sc, float4 sh, bool relu) {
  float4 z = make_float4(fmaf(y.x, sc.x, sh.x), fmaf(y.y, sc.y, sh.y), fmaf(y.z, sc.z, sh.z), fmaf(y.w, sc.w, sh.w));
  if (relu) z = make_float4(fmaxf(z.x, 0.f), fmaxf(z.y, 0.f), fmaxf(z.z, 0.f), fmaxf(z.w, 0.f));
  return z;
}
__device__ __forceinline__ float amax4(float4 z) {
  return fmaxf(fmaxf(fabsf(z.x), fabsf(z.y)), fmaxf(fabsf(z.z), fabsf(z.w)));
}

// Block-wide fp64 sums over the row lanes of K per-thread float4 values: channel quad q = tid % CQ,
// component j of value k -> red[k * CB + 4 q + j] (LDS, visible to every thread on return).
// red: (NW + 1) x K x CB doubles.
template <int K>
__device__ __forceinline__ void block_sum4(const float4 (&v)[K], double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double s = (double)f4c(v[k], j);
#pragma unroll
      for (int o = 32; o >= CQ; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane < CQ) red[K * CB + (wv * K + k) * CB + 4 * lane + j] = s;
    }
  __syncthreads();
  if (threadIdx.x < K * CB) {
    const int k = threadIdx.x / CB, e = threadIdx.x % CB;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[K * CB + (w * K + k) * CB + e];
    red[threadIdx.x] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ float block_max(float am, float* red) {
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
  return m;
}

// Element offset (row * C + n0) of row k (0..RPU-1) of unit u: a 2x2 window (POOL) or one pixel.
template <bool POOL>
__device__ __forceinline__ unsigned unit_row(int u, int k, int H, int W, int Ho, int Wo, int C, int n0) {
  if (!POOL) return (unsigned)u * (unsigned)C + (unsigned)n0;
  const int wo = u % Wo, t = u / Wo, ho = t % Ho, n = t / Ho;
  const int r = (n * H + 2 * ho + (k >> 1)) * W + 2 * wo + (k & 1);
  return (unsigned)r * (unsigned)C + (unsigned)n0;
}

// ------------------------------------------------------------------ forward
// RT = row slots per thread (UPT units of RPU rows); slab loads in batches of ZB splits.
template <int RT, bool POOL>
__global__ __launch_bounds__(NT) void chan_fwd_kernel(ChanFwdArgs a) {
  constexpr int RPU = POOL ? 4 : 1;
  constexpr int UPT = RT / RPU;
  constexpr int ZB = 16 / RT;  // 16 slab loads in flight per lane
  __shared__ double red[(NW + 1) * CB];
  __shared__ float fred[NW];
  __shared__ float s_sc[CB], s_sh[CB];
  const int tid = threadIdx.x;
  const int q = tid % CQ, rl = tid / CQ;
  const int C = a.C, n0 = blockIdx.x * CB + 4 * q;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const int U = a.N * Ho * Wo;
  const int M = a.N * a.H * a.W;
  unsigned off[RT];  // byte offsets of the rows (kOOB for slots past the last unit)
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    const int u = rl + RL * i;
#pragma unroll
    for (int k = 0; k < RPU; ++k)
      off[i * RPU + k] = u < U ? unit_row<POOL>(u, k, a.H, a.W, Ho, Wo, C, n0) * 4u : kOOB;
  }
  // pass 1: y = sum_z slab[z] + bias, split batches of ZB (one round trip each)
  const unsigned plane = (unsigned)M * (unsigned)C * 4u;
  const __amdgpu_buffer_rsrc_t sr = make_rsrc(a.slab, plane * (unsigned)a.S);
  float4 v[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) v[r] = f4zero();
  for (int z0 = 0; z0 < a.S; z0 += ZB) {
    float4 t[ZB][RT];
#pragma unroll
    for (int k = 0; k < ZB; ++k)
#pragma unroll
      for (int r = 0; r < RT; ++r)
        t[k][r] = bload4(sr, (z0 + k < a.S && off[r] != kOOB) ? off[r] + (unsigned)(z0 + k) * plane : kOOB);
#pragma unroll
    for (int k = 0; k < ZB; ++k)
#pragma unroll
      for (int r = 0; r < RT; ++r) v[r] = f4add4(v[r], t[k][r]);
  }
  const float4 bv = a.bias ? ld4(a.bias + n0) : f4zero();
  float4 s = f4zero();
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (off[r] == kOOB) continue;
    v[r] = f4add4(v[r], bv);
    st4(a.y + off[r] / 4u, v[r]);
    s = f4add4(s, v[r]);
  }
  // statistics: mean, then the sum of squared deviations (two passes over registers, fp64 merge)
  {
    const float4 sv[1] = {s};
    block_sum4<1>(sv, red);
  }
  const double invM = 1.0 / (double)M;
  const float4 mf = make_float4((float)(red[4 * q] * invM), (float)(red[4 * q + 1] * invM),
                                (float)(red[4 * q + 2] * invM), (float)(red[4 * q + 3] * invM));
  const double tot = tid < CB ? red[tid] : 0.0;
  __syncthreads();  // red is reused below
  float4 sq = f4zero();
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (off[r] == kOOB) continue;
    const float dx = v[r].x - mf.x, dy = v[r].y - mf.y, dz = v[r].z - mf.z, dw = v[r].w - mf.w;
    sq.x = fmaf(dx, dx, sq.x);
    sq.y = fmaf(dy, dy, sq.y);
    sq.z = fmaf(dz, dz, sq.z);
    sq.w = fmaf(dw, dw, sq.w);
  }
  {
    const float4 qv[1] = {sq};
    block_sum4<1>(qv, red);
  }
  if (tid < CB) {
    const int c = blockIdx.x * CB + tid;
    const double mean = tot * invM;
    // the deviations were taken from the fp32-rounded mean: remove that offset's contribution
    const double dm = mean - (double)(float)mean;
    const double M2 = fmax(0.0, red[tid] - (double)M * dm * dm);
    const double var = M2 * invM;
    const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
    const float g = a.gamma ? a.gamma[c] : 1.f;
    const float bb = a.beta ? a.beta[c] : 0.f;
    const float scale = g * invstd;
    const float shift = bb - (float)mean * scale;
    s_sc[tid] = scale;
    s_sh[tid] = shift;
    a.stats[c] = (float)mean;
    a.stats[C + c] = invstd;
    a.stats[2 * C + c] = scale;
    a.stats[3 * C + c] = shift;
    if (a.running_mean) {
      float f = a.momentum;
      if (f < 0.f) f = 1.f / (float)(a.nbt[0] + 1);  // momentum=None: cumulative average
      const double unb = M > 1 ? M2 / (double)(M - 1) : var;
      a.running_mean[c] = (1.f - f) * a.running_mean[c] + f * (float)mean;
      a.running_var[c] = (1.f - f) * a.running_var[c] + f * (float)unb;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid == 0 && a.nbt) a.nbt[0] += 1;
  // apply: [pool2](relu(y * scale + shift))
  const float4 sc = make_float4(s_sc[4 * q], s_sc[4 * q + 1], s_sc[4 * q + 2], s_sc[4 * q + 3]);
  const float4 sh = make_float4(s_sh[4 * q], s_sh[4 * q + 1], s_sh[4 * q + 2], s_sh[4 * q + 3]);
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    const int u = rl + RL * i;
    if (u >= U) continue;
    float4 z = act4(v[i * RPU], sc, sh, a.relu);
    if (POOL) {
#pragma unroll
      for (int k = 1; k < RPU; ++k) {
        const float4 t = act4(v[i * RPU + k], sc, sh, a.relu);
        z = make_float4(fmaxf(z.x, t.x), fmaxf(z.y, t.y), fmaxf(z.z, t.z), fmaxf(z.w, t.w));
      }
    }
    st4(a.out + (long long)u * C + n0, z);
    am = fmaxf(am, amax4(z));
  }
  if (a.amax_part) {
    am = block_max(am, fred);
    if (tid == 0) a.amax_part[blockIdx.x] = am;
  }
}

// ------------------------------------------------------------------ backward
// dz at the RPU rows of one unit: the gradient g at the unit's (pooled) output routed through
// max-pool (first max wins in scan order (0,0),(0,1),(1,0),(1,1), like ATen) and ReLU (z > 0),
// with z = act(BN(y)) recomputed from the saved y
template <bool POOL>
__device__ __forceinline__ void unit_dz(const float4* yv, float4 g, float4 sc, float4 sh, bool relu,
                                        float4 (&dz)[POOL ? 4 : 1]) {
  if (!POOL) {
    const float4 z = act4(yv[0], sc, sh, relu);
    dz[0] = make_float4((!relu || z.x > 0.f) ? g.x : 0.f, (!relu || z.y > 0.f) ? g.y : 0.f,
                        (!relu || z.z > 0.f) ? g.z : 0.f, (!relu || z.w > 0.f) ? g.w : 0.f);
  } else {
    const float4 z0 = act4(yv[0], sc, sh, relu), z1 = act4(yv[1], sc, sh, relu), z2 = act4(yv[2], sc, sh, relu),
                 z3 = act4(yv[3], sc, sh, relu);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a0 = f4c(z0, e), a1 = f4c(z1, e), a2 = f4c(z2, e), a3 = f4c(z3, e);
      int arg = 0;
      float mx = a0;
      if (a1 > mx) { mx = a1; arg = 1; }
      if (a2 > mx) { mx = a2; arg = 2; }
      if (a3 > mx) { mx = a3; arg = 3; }
      const float gg = (!relu || mx > 0.f) ? f4c(g, e) : 0.f;
      f4set(dz[0], e, arg == 0 ? gg : 0.f);
      f4set(dz[1 % (POOL ? 4 : 1)], e, arg == 1 ? gg : 0.f);
      f4set(dz[2 % (POOL ? 4 : 1)], e, arg == 2 ? gg : 0.f);
      f4set(dz[3 % (POOL ? 4 : 1)], e, arg == 3 ? gg : 0.f);
    }
  }
}

template <int RT, bool POOL>
__device__ __forceinline__ void chan_bwd_d(const ChanBwdArgs& a) {
  constexpr int RPU = POOL ? 4 : 1;
  constexpr int UPT = RT / RPU;
  constexpr int ZB = UPT >= 8 ? 1 : 8 / UPT;
  __shared__ double red[(NW + 1) * 3 * CB];
  __shared__ float fred[NW];
  __shared__ float s_k1[CB], s_k2[CB];
  const int tid = threadIdx.x;
  const int q = tid % CQ, rl = tid / CQ;
  const int C = a.C, n0 = blockIdx.x * CB + 4 * q;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const int U = a.N * Ho * Wo;
  const int M = a.N * a.H * a.W;
  const bool relu = a.relu != 0;
  unsigned yo[RT];  // byte offsets of the y rows
  unsigned go[UPT];  // byte offsets of the dX rows
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    const int u = rl + RL * i;
    go[i] = u < U ? ((unsigned)u * (unsigned)C + (unsigned)n0) * 4u : kOOB;
#pragma unroll
    for (int k = 0; k < RPU; ++k) yo[i * RPU + k] = u < U ? unit_row<POOL>(u, k, a.H, a.W, Ho, Wo, C, n0) * 4u : kOOB;
  }
  // y rows first (independent of the slabs: both round trips overlap)
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(a.y, (unsigned)M * (unsigned)C * 4u);
  float4 yv[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) yv[r] = bload4(yr, yo[r]);
  const unsigned plane = (unsigned)U * (unsigned)C * 4u;
  const __amdgpu_buffer_rsrc_t sr = make_rsrc(a.d_slab, plane * (unsigned)a.d_S);
  float4 g[UPT];
#pragma unroll
  for (int i = 0; i < UPT; ++i) g[i] = f4zero();
  for (int z0 = 0; z0 < a.d_S; z0 += ZB) {
    float4 t[ZB][UPT];
#pragma unroll
    for (int k = 0; k < ZB; ++k)
#pragma unroll
      for (int i = 0; i < UPT; ++i)
        t[k][i] = bload4(sr, (z0 + k < a.d_S && go[i] != kOOB) ? go[i] + (unsigned)(z0 + k) * plane : kOOB);
#pragma unroll
    for (int k = 0; k < ZB; ++k)
#pragma unroll
      for (int i = 0; i < UPT; ++i) g[i] = f4add4(g[i], t[k][i]);
  }
  if (a.d_y != a.d_slab) {  // (d_S == 1 reading dX in place: nothing to write)
#pragma unroll
    for (int i = 0; i < UPT; ++i)
      if (go[i] != kOOB) st4(a.d_y + go[i] / 4u, g[i]);
  }
  const float4 mu = ld4(a.stats + n0), is = ld4(a.stats + C + n0);
  const float4 sc = ld4(a.stats + 2 * C + n0), sh = ld4(a.stats + 3 * C + n0);
  // sums of dz, dz * xhat and xhat (dz recomputed per unit in both passes: no dz array held)
  float4 acc[3] = {f4zero(), f4zero(), f4zero()};
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    if (go[i] == kOOB) continue;
    float4 dz[RPU];
    unit_dz<POOL>(yv + i * RPU, g[i], sc, sh, relu, dz);
#pragma unroll
    for (int k = 0; k < RPU; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (f4c(yv[i * RPU + k], e) - f4c(mu, e)) * f4c(is, e);
        const float d = f4c(dz[k], e);
        f4set(acc[0], e, f4c(acc[0], e) + d);
        f4set(acc[1], e, fmaf(d, xh, f4c(acc[1], e)));
        f4set(acc[2], e, f4c(acc[2], e) + xh);
      }
  }
  block_sum4<3>(acc, red);
  if (tid < CB) {
    const int c = blockIdx.x * CB + tid;
    const double invM = 1.0 / (double)M;
    const double t0 = red[tid], t1 = red[CB + tid], t2 = red[2 * CB + tid];
    s_k1[tid] = (float)t0 * (float)invM;
    s_k2[tid] = (float)t1 * (float)invM;
    if (a.gbeta) a.gbeta[c] = (float)t0;
    if (a.ggamma) a.ggamma[c] = (float)t1;
    // conv-bias gradient sum(dy) = -scale * sum(xhat) * sum(dz * xhat) / M
    if (a.gdb) a.gdb[c] = (float)(-(double)a.stats[2 * C + c] * t2 * t1 * invM);
  }
  __syncthreads();
  const float4 k1 = make_float4(s_k1[4 * q], s_k1[4 * q + 1], s_k1[4 * q + 2], s_k1[4 * q + 3]);
  const float4 k2 = make_float4(s_k2[4 * q], s_k2[4 * q + 1], s_k2[4 * q + 2], s_k2[4 * q + 3]);
  // re-read after the barrier: the compiler must then recompute dz / xhat here instead of keeping
  // the first pass's values live across the reduction (which spilled at 16 rows per thread)
  const float4 mu2 = ld4(a.stats + n0), is2 = ld4(a.stats + C + n0);
  const float4 sc2 = ld4(a.stats + 2 * C + n0), sh2 = ld4(a.stats + 3 * C + n0);
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    if (go[i] == kOOB) continue;
    float4 dz[RPU];
    unit_dz<POOL>(yv + i * RPU, g[i], sc2, sh2, relu, dz);
#pragma unroll
    for (int k = 0; k < RPU; ++k) {
      float4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (f4c(yv[i * RPU + k], e) - f4c(mu2, e)) * f4c(is2, e);
        f4set(o, e, f4c(sc2, e) * (f4c(dz[k], e) - f4c(k1, e) - xh * f4c(k2, e)));
      }
      st4(a.dy + yo[i * RPU + k] / 4u, o);
      am = fmaxf(am, amax4(o));
    }
  }
  if (a.amax_part) {
    am = block_max(am, fred);
    if (tid == 0) a.amax_part[blockIdx.x] = am;
  }
}

__device__ __forceinline__ void chan_bwd_w(const ChanBwdArgs& a, int bw) {
  __shared__ float4 wred[NT];
  const int tid = threadIdx.x;
  const int wcb = a.w_cb, SL = NT / wcb;
  const int cl = tid % wcb, sl = tid / wcb;
  const long long i = (long long)bw * wcb + cl;
  float4 s = f4zero();
  if (i < a.w_n4) {
    int z = sl;
    for (; z + 3 * SL < a.w_S; z += 4 * SL) {
      const float4 p = a.w_slab[(long long)z * a.w_n4 + i], q = a.w_slab[(long long)(z + SL) * a.w_n4 + i];
      const float4 r = a.w_slab[(long long)(z + 2 * SL) * a.w_n4 + i], t = a.w_slab[(long long)(z + 3 * SL) * a.w_n4 + i];
      s.x += (p.x + q.x) + (r.x + t.x); s.y += (p.y + q.y) + (r.y + t.y);
      s.z += (p.z + q.z) + (r.z + t.z); s.w += (p.w + q.w) + (r.w + t.w);
    }
    for (; z < a.w_S; z += SL) s = f4add4(s, a.w_slab[(long long)z * a.w_n4 + i]);
  }
  if (SL > 1) {
    wred[tid] = s;
    __syncthreads();
    if (sl != 0) return;
    for (int k = 1; k < SL; ++k) s = f4add4(s, wred[k * wcb + cl]);
  }
  if (i < a.w_n4) a.w_dst[i] = s;
}

template <int RT, bool POOL>
__global__ __launch_bounds__(NT) void chan_bwd_kernel(ChanBwdArgs a) {
  if ((int)blockIdx.x < a.nbd) chan_bwd_d<RT, POOL>(a);
  else chan_bwd_w(a, (int)blockIdx.x - a.nbd);
}

// rows held per thread for `units` units of rpu rows: 1, 2, 4, 8 or 16 (0: too many)
int chan_rt(long long units, int rpu) {
  const long long upt = (units + RL - 1) / RL;
  long long rt = upt * rpu;
  int p = 1;
  while (p < rt) p <<= 1;
  return p <= 16 ? p : 0;
}

// read per call so one process can compare both paths (CDP_CHAN=0 disables the fusion)
long long chan_max_rows() {
  const char* off = std::getenv("CDP_CHAN");
  if (off && off[0] == '0') return 0;
  const char* e = std::getenv("CDP_CHAN_MAXROWS");
  return e ? std::atoll(e) : 2048LL;
}

}  // namespace

// Rows held per lane above which the fusion loses to the two-launch path (measured on MI355X,
// VGG-11 at 32 images per GPU, eager rocprofv3, us per layer, fused vs reduction + finalize/apply):
// forward 9.7 vs 11.5 at 1 row per lane, 15.2 vs 11.5 at 4, 26-30 vs ~12 at 16; backward 9.8 vs
// 16.7 at 1, 11.4-15.8 vs 16.7 at 4, 31-33 vs 16.7 at 16. A block's rows are a serial chain of
// split-K load batches, and 16 channels per block leave few blocks for the larger maps.
int chan_rt_limit(bool bwd) {
  const char* e = std::getenv(bwd ? "CDP_CHAN_BWD_RT" : "CDP_CHAN_FWD_RT");
  return e ? std::atoi(e) : (bwd ? 4 : 1);
}

bool chan_fwd_ok(int N, int H, int W, int C, bool pool, bool bwd) {
  const long long M = (long long)N * H * W;
  if ((C % CB) != 0 || M > chan_max_rows() || M < 1) return false;
  if (pool && ((H & 1) || (W & 1))) return false;
  const long long units = pool ? M / 4 : M;
  const int rt = chan_rt(units, pool ? 4 : 1);
  return rt != 0 && rt <= chan_rt_limit(bwd) && M * C * 16LL < (1LL << 31);
}

int chan_amax_parts(int C) { return C / CB; }

void chan_fwd_launch(const ChanFwdArgs& a, hipStream_t st) {
  const long long M = (long long)a.N * a.H * a.W;
  const int rt = chan_rt(a.pool ? M / 4 : M, a.pool ? 4 : 1);
  const dim3 grid(a.C / CB), blk(NT);
  if (a.pool) {
    if (rt <= 4) hipLaunchKernelGGL((chan_fwd_kernel<4, true>), grid, blk, 0, st, a);
    else if (rt == 8) hipLaunchKernelGGL((chan_fwd_kernel<8, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((chan_fwd_kernel<16, true>), grid, blk, 0, st, a);
  } else {
    if (rt == 1) hipLaunchKernelGGL((chan_fwd_kernel<1, false>), grid, blk, 0, st, a);
    else if (rt == 2) hipLaunchKernelGGL((chan_fwd_kernel<2, false>), grid, blk, 0, st, a);
    else if (rt == 4) hipLaunchKernelGGL((chan_fwd_kernel<4, false>), grid, blk, 0, st, a);
    else if (rt == 8) hipLaunchKernelGGL((chan_fwd_kernel<8, false>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((chan_fwd_kernel<16, false>), grid, blk, 0, st, a);
  }
}

void chan_bwd_launch(ChanBwdArgs a, hipStream_t st) {
  const long long M = (long long)a.N * a.H * a.W;
  const int rt = chan_rt(a.pool ? M / 4 : M, a.pool ? 4 : 1);
  a.nbd = a.C / CB;
  int nbw = 0;
  if (a.w_slab) {
    a.w_cb = (a.w_n4 >= 256LL * 1024 || a.w_S <= 1) ? 512 : (a.w_n4 >= 64LL * 1024 || a.w_S <= 4) ? 128 : 32;
    nbw = (int)((a.w_n4 + a.w_cb - 1) / a.w_cb);
  }
  const dim3 grid(a.nbd + nbw), blk(NT);
  if (a.pool) {
    if (rt <= 4) hipLaunchKernelGGL((chan_bwd_kernel<4, true>), grid, blk, 0, st, a);
    else if (rt == 8) hipLaunchKernelGGL((chan_bwd_kernel<8, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((chan_bwd_kernel<16, true>), grid, blk, 0, st, a);
  } else {
    if (rt == 1) hipLaunchKernelGGL((chan_bwd_kernel<1, false>), grid, blk, 0, st, a);
    else if (rt == 2) hipLaunchKernelGGL((chan_bwd_kernel<2, false>), grid, blk, 0, st, a);
    else if (rt == 4) hipLaunchKernelGGL((chan_bwd_kernel<4, false>), grid, blk, 0, st, a);
    else if (rt == 8) hipLaunchKernelGGL((chan_bwd_kernel<8, false>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((chan_bwd_kernel<16, false>), grid, blk, 0, st, a);
  }
}

}  // namespace cdp
