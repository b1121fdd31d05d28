// BatchNorm2d (+ReLU)(+MaxPool2d 2x2/2) forward and backward on NHWC fp32, gfx950.
//
// Reference layer stack: Conv2d -> BatchNorm2d -> ReLU(inplace) [-> MaxPool2d(2,2)] built by
// _make_layers at /root/reference/src/Part 1/model.py:11-27. Training-mode BN uses batch
// statistics (biased variance) and updates running_mean / running_var (unbiased) with
// momentum 0.1 and num_batches_tracked; eval mode uses the running statistics.
//
// Data flow per block (forward):
//   conv epilogue -> per-tile (mean, M2) partials  ->  bn_finalize (Chan merge, fp64)  ->
//   bn_act_fwd: z = relu(y*scale + shift), optional 2x2 max -> next layer input
// Backward recomputes z and the pool argmax from the saved conv output y (nothing else is
// stored):  bn_bwd_reduce (sum dz, sum dz*xhat per channel)  ->  chan_finalize  ->
//   bn_bwd_apply: dy = scale*(dz - mean(dz) - xhat*mean(dz*xhat)), plus partial sum(dy) for the
//   conv bias gradient.
// All element kernels move float4 along C (C % 4 == 0).
#include <algorithm>
#include <cstdlib>

#include "act_max.h"
#include "common.h"
#include "kernels.h"
#include "x3_common.h"

namespace cdp {
namespace {

// ------------------------------------------------------------------ finalize (train)
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ part, int nparts, int rpp, int M,
                                                          int C, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, long long* nbt, float momentum,
                                                          float eps, float* __restrict__ stats) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  // this thread's partials (b = tid + 256 k) are loaded in one batch and kept in registers for
  // both passes: one memory round trip instead of one per partial and pass (nparts <= 2048; more
  // fall back to a second, looped batch)
  // (buffer loads: the partials past nparts read 0 with no branch around the loads)
  constexpr int KB = 8;
  float pm[KB], pq[KB];
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)nparts * (unsigned)C * 8u);
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int b = tid + 256 * k;
    const unsigned o = b < nparts ? (unsigned)(b * C + c) * 8u : kOOB;
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(pr, (int)o, 0, 0);
    pm[k] = __uint_as_float(v[0]);
    pq[k] = __uint_as_float(v[1]);
  }
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int b = tid + 256 * k;
    if (b < nparts) s += (double)min(rpp, M - b * rpp) * (double)pm[k];
  }
  for (int b = tid + 256 * KB; b < nparts; b += 256)
    s += (double)min(rpp, M - b * rpp) * (double)part[((long long)b * C + c) * 2];
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / (double)M;
  __syncthreads();
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int b = tid + 256 * k;
    if (b < nparts) {
      const double d = (double)pm[k] - mean;
      q += (double)pq[k] + (double)min(rpp, M - b * rpp) * d * d;
    }
  }
  for (int b = tid + 256 * KB; b < nparts; b += 256) {
    const int cnt = min(rpp, M - b * rpp);
    const double d = (double)part[((long long)b * C + c) * 2] - mean;
    q += (double)part[((long long)b * C + c) * 2 + 1] + (double)cnt * d * d;
  }
  q = wave_sum_d(q);
  if ((tid & 63) == 0) red[tid >> 6] = q;
  __syncthreads();
  if (tid == 0) {
    const double m2 = red[0] + red[1] + red[2] + red[3];
    const double var = m2 / (double)M;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f;
    const float bb = beta ? beta[c] : 0.f;
    const float scale = g * invstd;
    // stats layout: [mean | invstd | scale | shift] x C
    stats[c] = (float)mean;
    stats[C + c] = invstd;
    stats[2 * C + c] = scale;
    stats[3 * C + c] = bb - (float)mean * scale;
    if (running_mean) {
      float f = momentum;
      if (f < 0.f) f = 1.f / (float)(nbt[0] + 1);  // momentum=None: cumulative average
      const double unb = M > 1 ? m2 / (double)(M - 1) : var;
      running_mean[c] = (1.f - f) * running_mean[c] + f * (float)mean;
      running_var[c] = (1.f - f) * running_var[c] + f * (float)unb;
    }
    if (c == 0 && nbt) nbt[0] += 1;
  }
}

// eval mode: scale/shift from running stats
__global__ void bn_eval_stats_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                     float eps, float* stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  stats[c] = rm[c];
  stats[C + c] = invstd;
  stats[2 * C + c] = g * invstd;
  stats[3 * C + c] = b - rm[c] * g * invstd;
}

__device__ __forceinline__ float4 affine_act(float4 y, float4 sc, float4 sh, bool relu) {
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

// Finalize + apply in one launch for layers with few statistics partials (nparts <= 128, the
// deep VGG layers): block = 64 channels x one chunk of output rows. Every block merges its 64
// channels' partials itself (fp64, the formulas of bn_finalize_kernel); the chunk-0 blocks publish
// stats and the running statistics; then the block applies [pool2](relu(y*scale + shift)) to its
// rows. Saves a dependent launch per layer; the redundant merge reads <= 64 KB per block from L2.
constexpr int FIN_MAXP = 128;      // backward fused finalize (bn_bwd_fin_apply) and 64-channel forward blocks
constexpr int FIN_MAXP16 = 512;    // forward, 16-channel blocks (16 merge threads per channel)
// A fused-finalize block's row r (pooled window or pixel) of y: the 2x2 window's four pixels (pool)
// or the pixel in v[0], channels n0..n0+3.
constexpr int kFinRPT = 4;  // rows per thread loaded before the statistics merge
// (pooled) pixel index -> (n, ho, wo) by multiply-shift division (32-bit indices: the launchers'
// tensors stay below 2^31 pooled pixels); 64-bit '/' and '%' here cost ~40 instructions each per row
struct PoolDiv {
  FastDiv wo, ho;
};
inline PoolDiv make_pooldiv(int Wo, int Ho) { return PoolDiv{make_fastdiv(Wo), make_fastdiv(Ho)}; }
__device__ __forceinline__ void pool_decode(int r, int Wo, int Ho, const PoolDiv& pd, int& n, int& ho, int& wo) {
  const int t = fdiv(r, pd.wo);
  wo = r - t * Wo;
  n = fdiv(t, pd.ho);
  ho = t - n * Ho;
}
__device__ __forceinline__ long long fin_row_off(long long r, int pool, int H, int W, int Ho, int Wo, int C, int n0,
                                                 const PoolDiv& pd) {
  if (!pool) return r * C + n0;
  int n, ho, wo;
  pool_decode((int)r, Wo, Ho, pd, n, ho, wo);
  return (((long long)n * H + 2 * ho) * W + 2 * wo) * C + n0;
}
__device__ __forceinline__ void fin_load_row(const float* __restrict__ y, float4 (&v)[4], long long r, int pool, int H,
                                             int W, int Ho, int Wo, int C, int n0, const PoolDiv& pd) {
  const float* b = y + fin_row_off(r, pool, H, W, Ho, Wo, C, n0, pd);
  v[0] = ld4(b);
  if (pool) {
    v[1] = ld4(b + C);
    v[2] = ld4(b + (long long)W * C);
    v[3] = ld4(b + (long long)W * C + C);
  }
}
// rows ra, ra + rs, ... (the first kFinRPT of this thread); rows past r1 load row 0 (unused)
__device__ __forceinline__ void fin_prefetch(const float* __restrict__ y, float4 (&pv)[kFinRPT][4], long long ra,
                                             long long r1, int pool, int H, int W, int Ho, int Wo, int C, int n0,
                                             const PoolDiv& pd, int rs = 16) {
#pragma unroll
  for (int i = 0; i < kFinRPT; ++i) {
    const long long r = ra + rs * i;
    fin_load_row(y, pv[i], r < r1 ? r : 0, pool, H, W, Ho, Wo, C, n0, pd);
  }
}
// CG channels per block: 64 (4 merge threads per channel) or 16 (16 merge threads per channel: a
// quarter of the merge work per thread, 4x the blocks repeating it)
template <int CG, bool POOL>
__global__ __launch_bounds__(256) void bn_fin_act_kernel(const float* __restrict__ part, int nparts, int rpp, int M,
                                                         int C, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* running_mean,
                                                         float* running_var, long long* nbt, float momentum,
                                                         float eps, float* __restrict__ stats,
                                                         const float* __restrict__ y, float* __restrict__ out, int N,
                                                         int H, int W, int relu, int chunks, FastDiv fd_HWo,
                                                         ActMaxOut am, PoolDiv pd) {
  constexpr int pool = POOL ? 1 : 0;  // (as bn_bwd_reduce_kernel)
  constexpr int TQ = 256 / CG;  // merge threads per channel
  constexpr int CQ = CG / 4;    // phase 2: channel quads x RL row lanes
  constexpr int RL = 256 / CQ;
  __shared__ double red[TQ][CG];
  __shared__ float s_sc[CG], s_sh[CG];
  __shared__ ActMaxBlock<CG> sam;  // per-image / per-channel |max| of the block's output
  const int ngroups = C / CG;
  const int cg = blockIdx.x % ngroups, chunk = blockIdx.x / ngroups;
  const int tid = threadIdx.x;
  const int ch = tid % CG, q = tid / CG;
  const int c = cg * CG + ch;
  const bool want = am.img != nullptr;
  if (want) sam.init(tid, 256);  // (the merge's barriers below order it before every add)
  // phase-2 geometry, and this thread's first kFinRPT rows of y loaded before the merge: the y
  // round trip overlaps the partials' instead of following it
  const int cq = tid % CQ, rl = tid / CQ;
  const int n0 = cg * CG + 4 * cq;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const long long rows = (long long)N * Ho * Wo;
  const long long per = (rows + chunks - 1) / chunks;
  const long long r0 = (long long)chunk * per, r1 = min(rows, r0 + per);
  const int img0 = fdiv((int)min(r0, rows - 1), fd_HWo);
  float4 pv[kFinRPT][4];
  fin_prefetch(y, pv, r0 + rl, r1, pool, H, W, Ho, Wo, C, n0, pd, RL);
  // phase 1: thread (ch, q) merges partials b = q + TQ k -- one batch of buffer loads
  // (only the batches of 8 loads that hold partials are issued: kp = ceil(nparts / TQ) rounded up to 8)
  constexpr int KP = (CG == 16 ? FIN_MAXP16 : FIN_MAXP) / TQ;
  const int kp = (((nparts + TQ - 1) / TQ) + 7) & ~7;
  float pm[KP], pq[KP];
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)nparts * (unsigned)C * 8u);
#pragma unroll
  for (int k0 = 0; k0 < KP; k0 += 8) {
    if (k0 >= kp) break;
#pragma unroll
    for (int k = k0; k < k0 + 8; ++k) {
      const int b = q + TQ * k;
      const unsigned o = b < nparts ? (unsigned)(b * C + c) * 8u : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(pr, (int)o, 0, 0);
      pm[k] = __uint_as_float(v[0]);
      pq[k] = __uint_as_float(v[1]);
    }
  }
  double sm = 0.0;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int b = q + TQ * k;
    if (b < nparts) sm += (double)min(rpp, M - b * rpp) * (double)pm[k];
  }
  red[q][ch] = sm;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int t = 0; t < TQ; ++t) tot += red[t][ch];
  const double mean = tot / (double)M;
  __syncthreads();
  double sq = 0.0;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int b = q + TQ * k;
    if (b < nparts) {
      const double d = (double)pm[k] - mean;
      sq += (double)pq[k] + (double)min(rpp, M - b * rpp) * d * d;
    }
  }
  red[q][ch] = sq;
  __syncthreads();
  if (q == 0) {
    double m2 = 0.0;
#pragma unroll
    for (int t = 0; t < TQ; ++t) m2 += red[t][ch];
    const double var = m2 / (double)M;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f;
    const float bb = beta ? beta[c] : 0.f;
    const float scale = g * invstd;
    const float shift = bb - (float)mean * scale;
    s_sc[ch] = scale;
    s_sh[ch] = shift;
    if (chunk == 0) {
      stats[c] = (float)mean;
      stats[C + c] = invstd;
      stats[2 * C + c] = scale;
      stats[3 * C + c] = shift;
      if (running_mean) {
        float f = momentum;
        if (f < 0.f) f = 1.f / (float)(nbt[0] + 1);  // momentum=None: cumulative average
        const double unb = M > 1 ? m2 / (double)(M - 1) : var;
        running_mean[c] = (1.f - f) * running_mean[c] + f * (float)mean;
        running_var[c] = (1.f - f) * running_var[c] + f * (float)unb;
      }
      if (c == 0 && nbt) nbt[0] += 1;
    }
  }
  __syncthreads();
  // phase 2: this chunk's output rows, 16 channel quads x 16 row lanes
  const float4 sc = make_float4(s_sc[4 * cq], s_sc[4 * cq + 1], s_sc[4 * cq + 2], s_sc[4 * cq + 3]);
  const float4 sh = make_float4(s_sh[4 * cq], s_sh[4 * cq + 1], s_sh[4 * cq + 2], s_sh[4 * cq + 3]);
  ImgRun run;
  float4 cm = f4zero();
  auto emit = [&](long long r, const float4 (&v)[4]) {
    float4 z = affine_act(v[0], sc, sh, relu);
    if (pool) {
      const float4 z1 = affine_act(v[1], sc, sh, relu), z2 = affine_act(v[2], sc, sh, relu),
                   z3 = affine_act(v[3], sc, sh, relu);
      z.x = fmaxf(fmaxf(z.x, z1.x), fmaxf(z2.x, z3.x));
      z.y = fmaxf(fmaxf(z.y, z1.y), fmaxf(z2.y, z3.y));
      z.z = fmaxf(fmaxf(z.z, z1.z), fmaxf(z2.z, z3.z));
      z.w = fmaxf(fmaxf(z.w, z1.w), fmaxf(z2.w, z3.w));
    }
    st4(out + r * C + n0, z);
    if (want) {
      run.add(fdiv((int)r, fd_HWo), absmax4(z), sam, img0, am);
      cm = absmax4(cm, z);
    }
  };
#pragma unroll
  for (int i = 0; i < kFinRPT; ++i)
    if (r0 + rl + RL * i < r1) emit(r0 + rl + RL * i, pv[i]);
  for (long long r = r0 + rl + RL * kFinRPT; r < r1; r += RL) {
    float4 v[4];
    fin_load_row(y, v, r, pool, H, W, Ho, Wo, C, n0, pd);
    emit(r, v);
  }
  if (want) {
    run.flush(sam, img0, am);
    sam.add_ch4(4 * cq, cm);
    __syncthreads();
    sam.publish(am, img0, N, cg * CG, CG, C, blockIdx.x % kActCopies, tid, 256);
  }
}

// ------------------------------------------------------------------ forward apply
// out = [pool2](relu(y*scale+shift)) (+ residual before relu when res != null). Block b writes the
// contiguous float4 range [b * per, (b + 1) * per) of out (per a multiple of 256 and of C / 4 when
// qmode != 0, so a thread's channel quad is fixed: qmode 1 = one quad (C / 4 divides 256), 2 = two
// alternating quads (C / 4 == 512), 0 = any C, per-element LDS channel maxima), and folds the
// per-image / per-channel |max| of what it writes into am (act_max.h).
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                                         const float* __restrict__ res, float* __restrict__ out,
                                                         int N, int H, int W, int C, int pool, int relu, int per,
                                                         int qmode, FastDiv fd_C4, FastDiv fd_HWo, ActMaxOut am,
                                                         unsigned char* __restrict__ rmask,
                                                         const float* __restrict__ res_y,
                                                         const float* __restrict__ res_st, PoolDiv pd) {
  __shared__ ActMaxBlock<kMaxActC> sam;
  const int C4 = C >> 2;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const int total = N * Ho * Wo * C4;
  const float* scale = stats + 2 * C;
  const float* shift = stats + 3 * C;
  const int tid = threadIdx.x;
  const int i0 = blockIdx.x * per, i1 = min(total, i0 + per);
  const bool want = am.img != nullptr;
  const int img0 = fdiv(fdiv(min(i0, total - 1), fd_C4), fd_HWo);
  if (want) {
    sam.init(tid, 256);
    __syncthreads();
  }
  ImgRun run;
  float4 cm[2] = {f4zero(), f4zero()};
  // store one output float4 (element i, k-th of this thread) and fold it into the block's maxima
  auto finish = [&](int i, int pix, int c4, float4 z, int k) {
    if (rmask)  // the ReLU's pass mask for the backward (1 byte per float4 instead of re-reading out)
      rmask[i] = (unsigned char)((z.x > 0.f ? 1 : 0) | (z.y > 0.f ? 2 : 0) | (z.z > 0.f ? 4 : 0) | (z.w > 0.f ? 8 : 0));
    st4(out + (long long)pix * C + 4 * c4, z);
    if (want) {
      run.add(fdiv(pix, fd_HWo), absmax4(z), sam, img0, am);
      if (qmode == 1 || (qmode == 2 && !(k & 1))) cm[0] = absmax4(cm[0], z);
      else if (qmode == 2) cm[1] = absmax4(cm[1], z);
      else sam.add_ch4_any(4 * c4, make_float4(fabsf(z.x), fabsf(z.y), fabsf(z.z), fabsf(z.w)), C, am,
                           blockIdx.x % kActCopies);
    }
  };
  if (!pool) {
    // kU elements per thread loaded before any is used: one element's load -> apply -> store chain
    // per iteration leaves a wave with one or two requests in flight (4.2 TB/s on ResNet-50's passes)
    constexpr int kU = 4;
    int k = 0;
    for (int ib = i0 + tid; ib < i1; ib += 256 * kU, k += kU) {
      float4 yv[kU], rv[kU];
      int pv[kU], cv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = min(ib + 256 * u, i1 - 1);  // past the end: reload the last element, unused
        pv[u] = fdiv(i, fd_C4);
        cv[u] = i - pv[u] * C4;
        const long long off = (long long)pv[u] * C + 4 * cv[u];
        yv[u] = ld4(y + off);
        rv[u] = res ? ld4(res + off) : res_y ? ld4(res_y + off) : f4zero();
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (ib + 256 * u >= i1) break;
        const int c4 = cv[u];
        float4 z = affine_act(yv[u], ld4(scale + 4 * c4), ld4(shift + 4 * c4), false);
        // res_y: the downsample branch's BatchNorm, applied here instead of materialized
        if (res || res_y) {
          const float4 r = res ? rv[u]
                               : affine_act(rv[u], ld4(res_st + 2 * C + 4 * c4), ld4(res_st + 3 * C + 4 * c4), false);
          z.x += r.x; z.y += r.y; z.z += r.z; z.w += r.w;
        }
        if (relu) {
          z.x = fmaxf(z.x, 0.f); z.y = fmaxf(z.y, 0.f); z.z = fmaxf(z.z, 0.f); z.w = fmaxf(z.w, 0.f);
        }
        finish(ib + 256 * u, pv[u], c4, z, k + u);
      }
    }
  } else {
    int k = 0;
    for (int i = i0 + tid; i < i1; i += 256, ++k) {
      const int pix = fdiv(i, fd_C4);
      const int c4 = i - pix * C4;
      const float4 sc = ld4(scale + 4 * c4), sh = ld4(shift + 4 * c4);
      int n, ho, wo;
      pool_decode(pix, Wo, Ho, pd, n, ho, wo);
      const float* base = y + (((long long)n * H + 2 * ho) * W + 2 * wo) * C + 4 * c4;
      const float4 z0 = affine_act(ld4(base), sc, sh, relu);
      const float4 z1 = affine_act(ld4(base + C), sc, sh, relu);
      const float4 z2 = affine_act(ld4(base + (long long)W * C), sc, sh, relu);
      const float4 z3 = affine_act(ld4(base + (long long)W * C + C), sc, sh, relu);
      float4 z;
      z.x = fmaxf(fmaxf(z0.x, z1.x), fmaxf(z2.x, z3.x));
      z.y = fmaxf(fmaxf(z0.y, z1.y), fmaxf(z2.y, z3.y));
      z.z = fmaxf(fmaxf(z0.z, z1.z), fmaxf(z2.z, z3.z));
      z.w = fmaxf(fmaxf(z0.w, z1.w), fmaxf(z2.w, z3.w));
      finish(i, pix, c4, z, k);
    }
  }
  if (want) {  // per-image / per-channel |max| of this block's output (the consumer GEMMs' scales)
    run.flush(sam, img0, am);
    if (qmode == 1 && i0 + tid < i1) sam.add_ch4(4 * (tid % C4), cm[0]);
    if (qmode == 2) {
      if (i0 + tid < i1) sam.add_ch4(4 * tid, cm[0]);
      if (i0 + tid + 256 < i1) sam.add_ch4(4 * (tid + 256), cm[1]);
    }
    __syncthreads();
    sam.publish(am, img0, N, 0, C <= kMaxActC ? C : 0, C, blockIdx.x % kActCopies, tid, 256);
  }
}

// ------------------------------------------------------------------ backward helpers
// For one channel component of a 2x2 window: the gradient reaching each element through
// max-pool (first max wins, scanning (0,0),(0,1),(1,0),(1,1) like ATen) and ReLU (z > 0).
__device__ __forceinline__ void pool_relu_grad(float z0, float z1, float z2, float z3, float g, bool relu, float& d0,
                                               float& d1, float& d2, float& d3) {
  int arg = 0;
  float mx = z0;
  if (z1 > mx) { mx = z1; arg = 1; }
  if (z2 > mx) { mx = z2; arg = 2; }
  if (z3 > mx) { mx = z3; arg = 3; }
  const float gg = (!relu || mx > 0.f) ? g : 0.f;
  d0 = arg == 0 ? gg : 0.f;
  d1 = arg == 1 ? gg : 0.f;
  d2 = arg == 2 ? gg : 0.f;
  d3 = arg == 3 ? gg : 0.f;
}

#define F4GET(v, j) ((j) == 0 ? (v).x : (j) == 1 ? (v).y : (j) == 2 ? (v).z : (v).w)

// the post-ReLU output's sign pattern of one float4 from its residual mask byte (bn_act_fwd_kernel)
__device__ __forceinline__ float4 mask_f4(unsigned char m) {
  return make_float4((float)(m & 1), (float)((m >> 1) & 1), (float)((m >> 2) & 1), (float)((m >> 3) & 1));
}

// Per (block, channel) partial sums of dz and dz*xhat, where dz is the gradient at the BN output,
// and (PS == 3) of xhat itself, from which chan_finalize derives the conv-bias gradient
// sum(dy) = -scale * sum(xhat) * sum(dz*xhat) / M without a second pass over dy.
// Block = 256 threads; for C4 <= 256 threads split as ppb pixel lanes x C4 channel quads.
// POOL is a template parameter: the pooled branch's four pixels per thread need ~130 VGPRs, which
// the unpooled instantiation (most of ResNet's BN passes) would otherwise carry at half the occupancy.
template <int PS, bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ y, const float* __restrict__ gout,
                                                            const float* __restrict__ stats, float* __restrict__ part,
                                                            int N, int H, int W, int C, int relu,
                                                            const float* __restrict__ zout,
                                                            const unsigned char* __restrict__ rmask, PoolDiv pd) {
  __shared__ float4 red1[256], red2[256], red3[PS == 3 ? 256 : 1];
  constexpr int pool = POOL ? 1 : 0;
  const int C4 = C >> 2;
  const int tid = threadIdx.x;
  const int cq_per_thread = (C4 + 255) / 256;  // 1 or 2
  const int lanes_c = C4 < 256 ? C4 : 256;
  const int ppb = 256 / lanes_c;               // pixel lanes per block
  const int cq0 = tid % lanes_c;
  const int pl = tid / lanes_c;
  const bool active = pl < ppb;
  const float* mean = stats;
  const float* invstd = stats + C;
  const float* scale = stats + 2 * C;
  const float* shift = stats + 3 * C;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const long long npix = (long long)N * Ho * Wo;  // output (pooled) pixels
  for (int j = 0; j < cq_per_thread; ++j) {
    const int cq = cq0 + j * 256;
    float4 a1 = f4zero(), a2 = f4zero(), a3 = f4zero();
    if (active && cq < C4) {
      const float4 sc = ld4(scale + 4 * cq), sh = ld4(shift + 4 * cq);
      const float4 mu = ld4(mean + 4 * cq), is = ld4(invstd + 4 * cq);
      for (long long px = (long long)blockIdx.x * ppb + pl; px < npix; px += (long long)gridDim.x * ppb) {
        const float4 g = ld4(gout + px * C + 4 * cq);
        if (!pool) {
          const float4 yv = ld4(y + px * C + 4 * cq);
          const float4 z = rmask ? mask_f4(rmask[px * C4 + cq])
                                 : zout ? ld4(zout + px * C + 4 * cq) : affine_act(yv, sc, sh, relu);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float dz = (!relu || F4GET(z, e) > 0.f) ? F4GET(g, e) : 0.f;
            const float xh = (F4GET(yv, e) - F4GET(mu, e)) * F4GET(is, e);
            if (e == 0) { a1.x += dz; a2.x += dz * xh; a3.x += xh; }
            if (e == 1) { a1.y += dz; a2.y += dz * xh; a3.y += xh; }
            if (e == 2) { a1.z += dz; a2.z += dz * xh; a3.z += xh; }
            if (e == 3) { a1.w += dz; a2.w += dz * xh; a3.w += xh; }
          }
        } else {
          int n, ho, wo;
          pool_decode((int)px, Wo, Ho, pd, n, ho, wo);
          const float* base = y + (((long long)n * H + 2 * ho) * W + 2 * wo) * C + 4 * cq;
          const float4 y0 = ld4(base), y1 = ld4(base + C), y2 = ld4(base + (long long)W * C),
                       y3 = ld4(base + (long long)W * C + C);
          const float4 z0 = affine_act(y0, sc, sh, relu), z1 = affine_act(y1, sc, sh, relu),
                       z2 = affine_act(y2, sc, sh, relu), z3 = affine_act(y3, sc, sh, relu);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float d0, d1, d2, d3;
            pool_relu_grad(F4GET(z0, e), F4GET(z1, e), F4GET(z2, e), F4GET(z3, e), F4GET(g, e), relu, d0, d1, d2,
                           d3);
            const float m = F4GET(mu, e), s = F4GET(is, e);
            const float sdz = d0 + d1 + d2 + d3;
            const float x0 = (F4GET(y0, e) - m) * s, x1 = (F4GET(y1, e) - m) * s, x2 = (F4GET(y2, e) - m) * s,
                        x3 = (F4GET(y3, e) - m) * s;
            const float sdx = d0 * x0 + d1 * x1 + d2 * x2 + d3 * x3;
            const float sx = (x0 + x1) + (x2 + x3);
            if (e == 0) { a1.x += sdz; a2.x += sdx; a3.x += sx; }
            if (e == 1) { a1.y += sdz; a2.y += sdx; a3.y += sx; }
            if (e == 2) { a1.z += sdz; a2.z += sdx; a3.z += sx; }
            if (e == 3) { a1.w += sdz; a2.w += sdx; a3.w += sx; }
          }
        }
      }
    }
    red1[tid] = a1;
    red2[tid] = a2;
    if constexpr (PS == 3) red3[tid] = a3;
    __syncthreads();
    if (pl == 0 && cq < C4) {
      float4 s1 = a1, s2 = a2, s3 = a3;
      for (int k = 1; k < ppb; ++k) {
        const float4 b1 = red1[k * lanes_c + cq0], b2 = red2[k * lanes_c + cq0];
        s1.x += b1.x; s1.y += b1.y; s1.z += b1.z; s1.w += b1.w;
        s2.x += b2.x; s2.y += b2.y; s2.z += b2.z; s2.w += b2.w;
        if constexpr (PS == 3) {
          const float4 b3 = red3[k * lanes_c + cq0];
          s3.x += b3.x; s3.y += b3.y; s3.z += b3.z; s3.w += b3.w;
        }
      }
      float* dst = part + ((long long)blockIdx.x * C + 4 * cq) * PS;
      dst[0] = s1.x; dst[1] = s2.x;
      dst[PS] = s1.y; dst[PS + 1] = s2.y;
      dst[2 * PS] = s1.z; dst[2 * PS + 1] = s2.z;
      dst[3 * PS] = s1.w; dst[3 * PS + 1] = s2.w;
      if constexpr (PS == 3) {
        dst[2] = s3.x; dst[5] = s3.y; dst[8] = s3.z; dst[11] = s3.w;
      }
    }
    __syncthreads();
  }
}

// Sum per-block partials (PS floats per (block, channel); fp64 accumulation, deterministic order):
// out[c] = sum_b part[b][c][0], out[C+c] = sum_b part[b][c][1]. Optionally also writes them into
// two gradient slots (accumulating if requested), and the conv-bias gradient db = sum_m dy_m:
//   dbmode 1 (training BN, PS == 3):  sum_m scale*(dz - S0/M - xhat*S1/M) = -scale * S2 * S1 / M
//   dbmode 2 (eval BN, dy = scale*dz): scale * S0
// so the bias gradient needs neither per-block partials of dy nor a launch of its own.
__global__ __launch_bounds__(256) void chan_finalize_kernel(const float* __restrict__ part, int nparts, int C, int PS,
                                                            float* __restrict__ out, float* g0, float* g1,
                                                            int accumulate, float* __restrict__ gdb,
                                                            const float* __restrict__ scale, double invM,
                                                            int dbmode) {
  __shared__ double r0[4], r1[4], r2[4];
  const int c = blockIdx.x;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  // all of this thread's partials in one batch of loads (nparts <= 1024), then the sums; the
  // summation order per thread is unchanged (b ascending), so results are as before
  constexpr int KB = 4;
  float v0[KB], v1[KB], v2[KB];
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)nparts * (unsigned)C * (unsigned)PS * 4u);
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int b = threadIdx.x + 256 * k;
    const unsigned o = b < nparts ? (unsigned)((b * C + c) * PS) * 4u : kOOB;
    v0[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)o, 0, 0));
    v1[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 4u), 0, 0));
    v2[k] = PS == 3 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 8u), 0, 0)) : 0.f;
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    s0 += (double)v0[k];
    s1 += (double)v1[k];
    s2 += (double)v2[k];
  }
  for (int b = threadIdx.x + 256 * KB; b < nparts; b += 256) {
    const float* q = part + ((long long)b * C + c) * PS;
    s0 += (double)q[0];
    s1 += (double)q[1];
    if (PS == 3) s2 += (double)q[2];
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  if (PS == 3) s2 = wave_sum_d(s2);
  if ((threadIdx.x & 63) == 0) {
    r0[threadIdx.x >> 6] = s0;
    r1[threadIdx.x >> 6] = s1;
    r2[threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double d0 = r0[0] + r0[1] + r0[2] + r0[3];
    const double d1 = r1[0] + r1[1] + r1[2] + r1[3];
    const double d2 = r2[0] + r2[1] + r2[2] + r2[3];
    const float t0 = (float)d0, t1 = (float)d1;
    if (out) {
      out[c] = dbmode == 2 ? 0.f : t0;  // eval-mode BN has no batch-statistics terms
      out[C + c] = dbmode == 2 ? 0.f : t1;
    }
    if (g0) g0[c] = accumulate ? g0[c] + t0 : t0;
    if (g1) g1[c] = accumulate ? g1[c] + t1 : t1;
    if (dbmode) {
      const float db = dbmode == 1 ? (float)(-(double)scale[c] * d2 * d1 * invM) : (float)((double)scale[c] * d0);
      gdb[c] = accumulate ? gdb[c] + db : db;
    }
  }
}

// dy = scale*(dz - sum(dz)/M - xhat*sum(dz*xhat)/M), full resolution; partial sum(dy) per
// (block, channel) for the conv bias gradient. Each thread handles one pooled window (pool) or
// one pixel; for odd H/W under pooling the uncovered border gets dz = 0. Block b walks the
// contiguous (pooled) pixel range [b * per, (b + 1) * per), per = ceil(npix / gridDim.x), and folds
// the per-image / per-channel |max| of the dy it writes into am (act_max.h).
// (POOL: as bn_bwd_reduce_kernel)
template <bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ y, const float* __restrict__ gout,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ sums, float* __restrict__ dy,
                                                           float* __restrict__ dbias_part, int N, int H, int W,
                                                           int C, int relu, const float* __restrict__ zout,
                                                           float* __restrict__ dres, FastDiv fd_IMG, FastDiv fd_HW,
                                                           ActMaxOut am, const unsigned char* __restrict__ rmask,
                                                           PoolDiv pd) {
  __shared__ float4 red[256];
  __shared__ ActMaxBlock<kMaxActC> sam;
  constexpr int pool = POOL ? 1 : 0;
  const bool want = am.img != nullptr;
  if (want) {
    sam.init(threadIdx.x, 256);
    __syncthreads();
  }
  ImgRun run;  // fd_IMG: (pooled) pixels per image; fd_HW: full-resolution pixels per image
  const int C4 = C >> 2;
  const int tid = threadIdx.x;
  const int cq_per_thread = (C4 + 255) / 256;
  const int lanes_c = C4 < 256 ? C4 : 256;
  const int ppb = 256 / lanes_c;
  const int cq0 = tid % lanes_c;
  const int pl = tid / lanes_c;
  const bool active = pl < ppb;
  const float* mean = stats;
  const float* invstd = stats + C;
  const float* scale = stats + 2 * C;
  const float* shift = stats + 3 * C;
  const long long Mtot = (long long)N * H * W;
  const float invM = 1.f / (float)Mtot;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const long long npix = pool ? (long long)N * Ho * Wo : Mtot;
  const long long pper = (npix + gridDim.x - 1) / gridDim.x;
  const long long p0 = (long long)blockIdx.x * pper, p1 = min(npix, p0 + pper);
  const int img0 = fdiv((int)min(p0, npix - 1), fd_IMG);
  for (int j = 0; j < cq_per_thread; ++j) {
    const int cq = cq0 + j * 256;
    float4 acc = f4zero();
    float4 cm = f4zero();  // this channel quad's |max| of dy
    if (active && cq < C4) {
      const float4 sc = ld4(scale + 4 * cq), sh = ld4(shift + 4 * cq);
      const float4 mu = ld4(mean + 4 * cq), is = ld4(invstd + 4 * cq);
      const float4 s1 = ld4(sums + 4 * cq), s2 = ld4(sums + C + 4 * cq);
      float4 k1, k2;  // dy = sc*(dz - k1 - xhat*k2)
      k1.x = s1.x * invM; k1.y = s1.y * invM; k1.z = s1.z * invM; k1.w = s1.w * invM;
      k2.x = s2.x * invM; k2.y = s2.y * invM; k2.z = s2.z * invM; k2.w = s2.w * invM;
      int img = 0;  // image of the pixel being emitted
      auto emit = [&](long long off, float4 yv, float4 dz) {
        float4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (F4GET(yv, e) - F4GET(mu, e)) * F4GET(is, e);
          const float v = F4GET(sc, e) * (F4GET(dz, e) - F4GET(k1, e) - xh * F4GET(k2, e));
          if (e == 0) o.x = v;
          if (e == 1) o.y = v;
          if (e == 2) o.z = v;
          if (e == 3) o.w = v;
        }
        st4(dy + off, o);
        acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
        if (want) {
          run.add(img, absmax4(o), sam, img0, am);
          cm = absmax4(cm, o);
        }
      };
      for (long long px = p0 + pl; px < p1; px += ppb) {
        img = fdiv((int)px, fd_IMG);
        const float4 g = ld4(gout + px * C + 4 * cq);
        if (!pool) {
          const float4 yv = ld4(y + px * C + 4 * cq);
          const float4 z = rmask ? mask_f4(rmask[px * C4 + cq])
                                 : zout ? ld4(zout + px * C + 4 * cq) : affine_act(yv, sc, sh, relu);
          float4 dz;
          dz.x = (!relu || z.x > 0.f) ? g.x : 0.f;
          dz.y = (!relu || z.y > 0.f) ? g.y : 0.f;
          dz.z = (!relu || z.z > 0.f) ? g.z : 0.f;
          dz.w = (!relu || z.w > 0.f) ? g.w : 0.f;
          if (dres) st4(dres + px * C + 4 * cq, dz);
          emit(px * C + 4 * cq, yv, dz);
        } else {
          int n, ho, wo;
          pool_decode((int)px, Wo, Ho, pd, n, ho, wo);
          const long long o0 = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + 4 * cq;
          const long long o1 = o0 + C, o2 = o0 + (long long)W * C, o3 = o2 + C;
          const float4 y0 = ld4(y + o0), y1 = ld4(y + o1), y2 = ld4(y + o2), y3 = ld4(y + o3);
          const float4 z0 = affine_act(y0, sc, sh, relu), z1 = affine_act(y1, sc, sh, relu),
                       z2 = affine_act(y2, sc, sh, relu), z3 = affine_act(y3, sc, sh, relu);
          float4 d0, d1, d2, d3;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float a, b, c, d;
            pool_relu_grad(F4GET(z0, e), F4GET(z1, e), F4GET(z2, e), F4GET(z3, e), F4GET(g, e), relu, a, b, c, d);
            if (e == 0) { d0.x = a; d1.x = b; d2.x = c; d3.x = d; }
            if (e == 1) { d0.y = a; d1.y = b; d2.y = c; d3.y = d; }
            if (e == 2) { d0.z = a; d1.z = b; d2.z = c; d3.z = d; }
            if (e == 3) { d0.w = a; d1.w = b; d2.w = c; d3.w = d; }
          }
          emit(o0, y0, d0);
          emit(o1, y1, d1);
          emit(o2, y2, d2);
          emit(o3, y3, d3);
        }
      }
      // odd-size border under pooling: rows/cols not covered by any window get dz = 0
      if (pool && ((H & 1) || (W & 1))) {
        const long long nb = (long long)N * H * W;
        for (long long px = (long long)blockIdx.x * ppb + pl; px < nb; px += (long long)gridDim.x * ppb) {
          const int w = (int)(px % W);
          const int h = (int)((px / W) % H);
          if (h < 2 * Ho && w < 2 * Wo) continue;
          img = fdiv((int)px, fd_HW);
          emit(px * C + 4 * cq, ld4(y + px * C + 4 * cq), f4zero());
        }
      }
      if (want) sam.add_ch4_any(4 * cq, cm, C, am, blockIdx.x % kActCopies);
    }
    red[tid] = acc;
    __syncthreads();
    if (dbias_part && pl == 0 && cq < C4) {
      float4 s = acc;
      for (int k = 1; k < ppb; ++k) {
        const float4 b = red[k * lanes_c + cq0];
        s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
      }
      float* dst = dbias_part + ((long long)blockIdx.x * C + 4 * cq) * 2;
      dst[0] = s.x; dst[1] = 0.f; dst[2] = s.y; dst[3] = 0.f;
      dst[4] = s.z; dst[5] = 0.f; dst[6] = s.w; dst[7] = 0.f;
    }
    __syncthreads();
  }
  if (want) {
    run.flush(sam, img0, am);
    __syncthreads();
    sam.publish(am, img0, N, 0, C <= kMaxActC ? C : 0, C, blockIdx.x % kActCopies, tid, 256);
  }
}

// Backward twin of bn_fin_act_kernel for layers with few statistics partials (nparts <= 128: the
// deep VGG layers, whose partials come from the consumer block's bwd_reduce_kernel): block = 64
// channels x one chunk of output rows. Every block merges its channels' partials itself (fp64, as
// chan_finalize_kernel); the chunk-0 blocks publish dgamma, dbeta and the conv-bias gradient; then
// the block writes dy = scale*(dz - sum(dz)/M - xhat*sum(dz*xhat)/M) for its rows, with the
// pool / ReLU routing recomputed from y. Training mode only (no residual, even map under pooling).
template <bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_fin_apply_kernel(
    const float* __restrict__ part, int nparts, int PS, const float* __restrict__ y,
    const float* __restrict__ gout, const float* __restrict__ stats, float* __restrict__ dy, float* gbeta,
    float* ggamma, float* gdb, int N, int H, int W, int C, int relu, int chunks, FastDiv fd_HWo,
    ActMaxOut am, PoolDiv pd) {
  constexpr int pool = POOL ? 1 : 0;
  __shared__ double red[3][4][64];
  __shared__ float s_k1[64], s_k2[64];
  __shared__ ActMaxBlock<64> sam;  // per-image / per-channel |max| of the block's dy
  const int ngroups = C >> 6;
  const int cg = blockIdx.x % ngroups, chunk = blockIdx.x / ngroups;
  const int tid = threadIdx.x;
  const int ch = tid & 63, q = tid >> 6;
  const int c = cg * 64 + ch;
  const long long Mtot = (long long)N * H * W;
  const bool want = am.img != nullptr;
  if (want) sam.init(tid, 256);  // (the merge's barriers below order it before every add)
  // phase-2 geometry, and this thread's first kFinRPT rows of y and of gout loaded before the
  // merge (their round trip overlaps the partials')
  const int cq = tid & 15, rl = tid >> 4;
  const int n0 = cg * 64 + 4 * cq;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const long long rows = (long long)N * Ho * Wo;
  const long long per = (rows + chunks - 1) / chunks;
  const long long r0 = (long long)chunk * per, r1 = min(rows, r0 + per);
  const int img0 = fdiv((int)min(r0, rows - 1), fd_HWo);
  float4 pv[kFinRPT][4], pg[kFinRPT];
  fin_prefetch(y, pv, r0 + rl, r1, pool, H, W, Ho, Wo, C, n0, pd);
#pragma unroll
  for (int i = 0; i < kFinRPT; ++i) {
    const long long r = r0 + rl + 16 * i;
    pg[i] = ld4(gout + (r < r1 ? r : 0) * C + n0);
  }
  // phase 1: thread (ch, q) sums partials b = q + 4k (one batch of buffer loads, ascending b)
  // all of this thread's partials in one round trip (issued in groups of 8 up to kp = ceil(nparts /
  // 4) rounded up to 8; a group loop that summed before loading the next took one round trip per
  // group: 4 for nparts = 128)
  constexpr int KP = FIN_MAXP / 4;
  const int kp = (((nparts + 3) >> 2) + 7) & ~7;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)nparts * (unsigned)C * (unsigned)PS * 4u);
  float v0[KP], v1[KP], v2[KP];
#pragma unroll
  for (int k0 = 0; k0 < KP; k0 += 8) {
    if (k0 >= kp) break;
#pragma unroll
    for (int k = k0; k < k0 + 8; ++k) {
      const int b = q + 4 * k;
      const unsigned o = b < nparts ? (unsigned)((b * C + c) * PS) * 4u : kOOB;
      v0[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)o, 0, 0));
      v1[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 4u), 0, 0));
      v2[k] = PS == 3 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 8u), 0, 0)) : 0.f;
    }
  }
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    if (q + 4 * k < nparts) {
      s0 += (double)v0[k];
      s1 += (double)v1[k];
      s2 += (double)v2[k];
    }
  }
  red[0][q][ch] = s0;
  red[1][q][ch] = s1;
  red[2][q][ch] = s2;
  __syncthreads();
  if (q == 0) {
    const double d0 = (red[0][0][ch] + red[0][1][ch]) + (red[0][2][ch] + red[0][3][ch]);
    const double d1 = (red[1][0][ch] + red[1][1][ch]) + (red[1][2][ch] + red[1][3][ch]);
    const double d2 = (red[2][0][ch] + red[2][1][ch]) + (red[2][2][ch] + red[2][3][ch]);
    const float t0 = (float)d0, t1 = (float)d1;
    const float invM = 1.f / (float)Mtot;
    s_k1[ch] = t0 * invM;
    s_k2[ch] = t1 * invM;
    if (chunk == 0) {
      if (gbeta) gbeta[c] = t0;
      if (ggamma) ggamma[c] = t1;
      if (gdb) gdb[c] = (float)(-(double)stats[2 * C + c] * d2 * d1 * (1.0 / (double)Mtot));
    }
  }
  __syncthreads();
  // phase 2: this chunk's rows (pooled windows or pixels), 16 channel quads x 16 row lanes
  const float4 sc = ld4(stats + 2 * C + n0), sh = ld4(stats + 3 * C + n0);
  const float4 mu = ld4(stats + n0), is = ld4(stats + C + n0);
  const float4 k1 = make_float4(s_k1[4 * cq], s_k1[4 * cq + 1], s_k1[4 * cq + 2], s_k1[4 * cq + 3]);
  const float4 k2 = make_float4(s_k2[4 * cq], s_k2[4 * cq + 1], s_k2[4 * cq + 2], s_k2[4 * cq + 3]);
  ImgRun run;
  float4 cm = f4zero();
  int img = 0;  // image of the row being emitted
  auto emit = [&](long long off, float4 yv, float4 dz) {
    float4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (F4GET(yv, e) - F4GET(mu, e)) * F4GET(is, e);
      const float v = F4GET(sc, e) * (F4GET(dz, e) - F4GET(k1, e) - xh * F4GET(k2, e));
      if (e == 0) o.x = v;
      if (e == 1) o.y = v;
      if (e == 2) o.z = v;
      if (e == 3) o.w = v;
    }
    st4(dy + off, o);
    if (want) {
      run.add(img, absmax4(o), sam, img0, am);
      cm = absmax4(cm, o);
    }
  };
  auto row = [&](long long r, const float4 (&v)[4], float4 g) {
    img = fdiv((int)r, fd_HWo);
    if (!pool) {
      const float4 yv = v[0];
      const float4 z = affine_act(yv, sc, sh, relu);
      float4 dz;
      dz.x = (!relu || z.x > 0.f) ? g.x : 0.f;
      dz.y = (!relu || z.y > 0.f) ? g.y : 0.f;
      dz.z = (!relu || z.z > 0.f) ? g.z : 0.f;
      dz.w = (!relu || z.w > 0.f) ? g.w : 0.f;
      emit(r * C + n0, yv, dz);
    } else {
      const long long o0 = fin_row_off(r, pool, H, W, Ho, Wo, C, n0, pd);
      const long long o1 = o0 + C, o2 = o0 + (long long)W * C, o3 = o2 + C;
      const float4 y0 = v[0], y1 = v[1], y2 = v[2], y3 = v[3];
      const float4 z0 = affine_act(y0, sc, sh, relu), z1 = affine_act(y1, sc, sh, relu),
                   z2 = affine_act(y2, sc, sh, relu), z3 = affine_act(y3, sc, sh, relu);
      float4 d0, d1, d2, d3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a, b, cc, d;
        pool_relu_grad(F4GET(z0, e), F4GET(z1, e), F4GET(z2, e), F4GET(z3, e), F4GET(g, e), relu, a, b, cc, d);
        if (e == 0) { d0.x = a; d1.x = b; d2.x = cc; d3.x = d; }
        if (e == 1) { d0.y = a; d1.y = b; d2.y = cc; d3.y = d; }
        if (e == 2) { d0.z = a; d1.z = b; d2.z = cc; d3.z = d; }
        if (e == 3) { d0.w = a; d1.w = b; d2.w = cc; d3.w = d; }
      }
      emit(o0, y0, d0);
      emit(o1, y1, d1);
      emit(o2, y2, d2);
      emit(o3, y3, d3);
    }
  };
#pragma unroll
  for (int i = 0; i < kFinRPT; ++i)
    if (r0 + rl + 16 * i < r1) row(r0 + rl + 16 * i, pv[i], pg[i]);
  for (long long r = r0 + rl + 16 * kFinRPT; r < r1; r += 16) {
    float4 v[4];
    fin_load_row(y, v, r, pool, H, W, Ho, Wo, C, n0, pd);
    row(r, v, ld4(gout + r * C + n0));
  }
  if (want) {
    run.flush(sam, img0, am);
    sam.add_ch4(4 * cq, cm);
    __syncthreads();
    sam.publish(am, img0, N, cg * 64, 64, C, blockIdx.x % kActCopies, tid, 256);
  }
}

// chan_finalize with 8 channels per block and 32 partial lanes: a wave's load covers 8 partial rows
// x 8 adjacent channels (<= 2 cache lines per row) instead of 64 rows x one channel (a line per
// partial and channel), all of a thread's partials in one batch of loads up to 1024 partials.
// Taken for wide layers with many partials (C >= 256, 513-1024 partials: ResNet-50's large
// BatchNorms, 15.97 -> 15.82 ms/step at 64 images, three interleaved pairs); with fewer partials
// or channels (every VGG-11 layer) it measured slower than one block per channel (1.343 -> 1.385
// ms at 256 images when taken everywhere).
__global__ __launch_bounds__(256) void chan_finalize8_kernel(const float* __restrict__ part, int nparts, int C, int PS,
                                                             float* __restrict__ out, float* g0, float* g1,
                                                             int accumulate, float* __restrict__ gdb,
                                                             const float* __restrict__ scale, double invM,
                                                             int dbmode) {
  __shared__ double red[3][32][8];
  const int ch = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + ch;
  const bool cok = c < C;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  constexpr int KB = 32;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)nparts * (unsigned)C * (unsigned)PS * 4u);
  for (int b0 = pl; b0 < nparts; b0 += 32 * KB) {
    float v0[KB], v1[KB], v2[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int b = b0 + 32 * k;
      const unsigned o = (b < nparts && cok) ? (unsigned)((b * C + c) * PS) * 4u : kOOB;
      v0[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)o, 0, 0));
      v1[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 4u), 0, 0));
      v2[k] = PS == 3 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, (int)(o + 8u), 0, 0)) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      s0 += (double)v0[k];
      s1 += (double)v1[k];
      s2 += (double)v2[k];
    }
  }
  red[0][pl][ch] = s0;
  red[1][pl][ch] = s1;
  red[2][pl][ch] = s2;
  __syncthreads();
  if (threadIdx.x < 8) {
    const int cc = blockIdx.x * 8 + threadIdx.x;
    if (cc >= C) return;
    double d0 = 0.0, d1 = 0.0, d2 = 0.0;
    for (int q = 0; q < 32; ++q) {
      d0 += red[0][q][threadIdx.x];
      d1 += red[1][q][threadIdx.x];
      d2 += red[2][q][threadIdx.x];
    }
    const float t0 = (float)d0, t1 = (float)d1;
    if (out) {
      out[cc] = dbmode == 2 ? 0.f : t0;  // eval-mode BN has no batch-statistics terms
      out[C + cc] = dbmode == 2 ? 0.f : t1;
    }
    if (g0) g0[cc] = accumulate ? g0[cc] + t0 : t0;
    if (g1) g1[cc] = accumulate ? g1[cc] + t1 : t1;
    if (dbmode) {
      const float db = dbmode == 1 ? (float)(-(double)scale[cc] * d2 * d1 * invM) : (float)((double)scale[cc] * d0);
      gdb[cc] = accumulate ? gdb[cc] + db : db;
    }
  }
}

int act_grid(long long work_items) {
  long long b = (work_items + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

int bn_bwd_grid(int N, int H, int W, int C, bool pool) {
  const int C4 = C / 4;
  const int lanes_c = C4 < 256 ? C4 : 256;
  const int ppb = 256 / lanes_c;
  const long long npix = (long long)N * (pool ? (H / 2) * (W / 2) : H * W);
  long long b = (npix + ppb - 1) / ppb;
  // ~2 pixels per thread lane, <= 1024 partial rows (one batch of loads in chan_finalize), and
  // never fewer workgroups than CUs while there are rows for them. Every pixel a lane handles is
  // one dependent memory round trip (the loop is not software-pipelined): at ~8 per lane the
  // small deep-layer passes were latency-bound (deep VGG layers otherwise ran 16-128 workgroups,
  // ~11 us per kernel)
  const long long rows = b;
  b = (b + 1) / 2;
  if (b < 256) b = rows < 256 ? rows : 256;
  // <= 1024 workgroups (2048 measured slower: the extra partial rows cost more in the finalize)
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

void bn_finalize_launch(const float* part, int nparts, int rpp, int M, int C, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                        float* stats, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, part, nparts, rpp, M, C, gamma, beta,
                     running_mean, running_var, nbt, momentum, eps, stats);
}

void bn_eval_stats_launch(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                          float* stats, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, rm, rv, eps,
                     stats);
}

// Timing experiment only (wrong numbers): CDP_EXP_SKIP_BN_APPLY=2 makes the fused finalize + apply
// kernels merge one statistics partial instead of all of them, same grid and block shape -- the
// ceiling of finalizing in the producer, which would leave the apply kernels 2 floats per channel.
static int exp_merge_parts(int nparts) {
  static const bool on = [] {
    const char* e = std::getenv("CDP_EXP_SKIP_BN_APPLY");
    return e && e[0] == '2';
  }();
  return on ? 1 : nparts;
}

// (up to 512 partials: 16-channel blocks above 32 partials, 32 M2-merge loads per thread)
bool bn_fin_act_ok(int nparts, int C, bool residual) { return !residual && nparts <= FIN_MAXP16 && (C % 64) == 0; }

// channels per fused-finalize block: 16 above 32 partials, else 64 (a 64-channel block merges at
// most FIN_MAXP partials, so past that the 16-channel blocks are the only correct choice)
static int fin_cg(int nparts) { return nparts > 32 ? 16 : 64; }

int bn_fin_act_grid(int N, int H, int W, int C, bool pool, int nparts) {
  const long long rows = (long long)N * (pool ? (H / 2) * (W / 2) : H * W);
  const int cg = nparts > 0 ? fin_cg(nparts) : 64;
  const int ngroups = C / cg;
  const int rl = 1024 / cg;  // row lanes per block
  // >= one row per row lane, <= 512 blocks (each repeats the partial merge)
  long long chunks = std::max<long long>(1, std::min<long long>((rows + rl - 1) / rl, 512 / ngroups));
  return (int)(chunks * ngroups);
}

static int out_pixels_per_image(int H, int W, bool pool) { return pool ? (H / 2) * (W / 2) : H * W; }

void bn_fin_act_launch(const float* part, int nparts, int rpp, int C, const float* gamma, const float* beta,
                       float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                       float* stats, const float* y, float* out, int N, int H, int W, bool pool, bool relu,
                       ActMaxOut am, hipStream_t st) {
  const int grid = bn_fin_act_grid(N, H, W, C, pool, nparts);
  const int M = N * H * W;
  const int cg = fin_cg(nparts);
  auto k = cg == 64 ? (pool ? bn_fin_act_kernel<64, true> : bn_fin_act_kernel<64, false>)
                    : (pool ? bn_fin_act_kernel<16, true> : bn_fin_act_kernel<16, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, part,
                     exp_merge_parts(nparts), rpp, M, C, gamma, beta, running_mean, running_var, nbt, momentum, eps, stats, y, out, N,
                     H, W, relu ? 1 : 0, grid / (C / cg),
                     make_fastdiv(out_pixels_per_image(H, W, pool)), am, make_pooldiv(W / 2, H / 2));
}

bool bn_bwd_fin_apply_ok(int nparts, int C, int H, int W, bool pool) {
  return nparts <= FIN_MAXP && (C % 64) == 0 && !(pool && ((H & 1) || (W & 1)));
}

void bn_bwd_fin_apply_launch(const float* part, int nparts, int ps, const float* y, const float* gout,
                             const float* stats, float* dy, float* gbeta, float* ggamma, float* gdb, int N, int H,
                             int W, int C, bool pool, bool relu, ActMaxOut am, hipStream_t st) {
  const int grid = bn_fin_act_grid(N, H, W, C, pool);
  hipLaunchKernelGGL(pool ? bn_bwd_fin_apply_kernel<true> : bn_bwd_fin_apply_kernel<false>, dim3(grid), dim3(256), 0,
                     st, part, exp_merge_parts(nparts), ps, y, gout, stats, dy, gbeta, ggamma, gdb, N, H, W, C,
                     relu ? 1 : 0, grid / (C / 64),
                     make_fastdiv(out_pixels_per_image(H, W, pool)), am, make_pooldiv(W / 2, H / 2));
}

int bn_act_grid(int N, int H, int W, int C, bool pool) {
  return act_grid((long long)N * out_pixels_per_image(H, W, pool) * (C / 4));
}

void bn_act_fwd_launch(const float* y, const float* stats, const float* res, float* out, int N, int H, int W, int C,
                       bool pool, bool relu, hipStream_t st, ActMaxOut am, unsigned char* rmask, const float* res_y,
                       const float* res_st) {
  const int C4 = C / 4;
  const long long total = (long long)N * out_pixels_per_image(H, W, pool) * C4;
  // contiguous per-block ranges, whole multiples of 256 float4 (and of C4: fixed channel quads)
  const int qmode = (C4 <= 256 && (256 % C4) == 0) ? 1 : C4 == 512 ? 2 : 0;
  const long long unit = qmode == 2 ? 512 : 256;
  const long long blocks = bn_act_grid(N, H, W, C, pool);
  const long long per = std::max(unit, ((total + blocks - 1) / blocks + unit - 1) / unit * unit);
  hipLaunchKernelGGL(bn_act_fwd_kernel, dim3((unsigned)((total + per - 1) / per)), dim3(256), 0, st, y, stats, res,
                     out, N, H, W, C, pool ? 1 : 0, relu ? 1 : 0, (int)per, qmode, make_fastdiv(C4),
                     make_fastdiv(out_pixels_per_image(H, W, pool)), am, pool ? nullptr : rmask, res_y, res_st,
                     make_pooldiv(W / 2, H / 2));
}

void bn_bwd_reduce_launch(const float* y, const float* gout, const float* stats, float* part, int nblocks, int N,
                          int H, int W, int C, bool pool, bool relu, const float* zout, hipStream_t st,
                          bool with_xsum, const unsigned char* rmask) {
  auto k = with_xsum ? (pool ? bn_bwd_reduce_kernel<3, true> : bn_bwd_reduce_kernel<3, false>)
                     : (pool ? bn_bwd_reduce_kernel<2, true> : bn_bwd_reduce_kernel<2, false>);
  hipLaunchKernelGGL(k, dim3(nblocks), dim3(256), 0, st, y, gout, stats, part, N, H, W, C, relu ? 1 : 0, zout, rmask,
                     make_pooldiv(W / 2, H / 2));
}

void chan_finalize_launch(const float* part, int nparts, int C, float* out, float* g0, float* g1, bool accumulate,
                          hipStream_t st, int ps, float* gdb, const float* scale, long long M, int dbmode) {
  if (C >= 256 && nparts > 512 && nparts <= 1024)
    hipLaunchKernelGGL(chan_finalize8_kernel, dim3((C + 7) / 8), dim3(256), 0, st, part, nparts, C, ps, out, g0, g1,
                       accumulate ? 1 : 0, gdb, scale, M > 0 ? 1.0 / (double)M : 0.0, dbmode);
  else
    hipLaunchKernelGGL(chan_finalize_kernel, dim3(C), dim3(256), 0, st, part, nparts, C, ps, out, g0, g1,
                       accumulate ? 1 : 0, gdb, scale, M > 0 ? 1.0 / (double)M : 0.0, dbmode);
}

void bn_bwd_apply_launch(const float* y, const float* gout, const float* stats, const float* sums, float* dy,
                         float* dbias_part, int nblocks, int N, int H, int W, int C, bool pool, bool relu,
                         const float* zout, float* dres, hipStream_t st, ActMaxOut am, const unsigned char* rmask) {
  hipLaunchKernelGGL(pool ? bn_bwd_apply_kernel<true> : bn_bwd_apply_kernel<false>, dim3(nblocks), dim3(256), 0, st,
                     y, gout, stats, sums, dy, dbias_part, N, H, W, C, relu ? 1 : 0, zout, dres, make_fastdiv(out_pixels_per_image(H, W, pool)),
                     make_fastdiv(H * W), am, rmask, make_pooldiv(W / 2, H / 2));
}

}  // namespace cdp
