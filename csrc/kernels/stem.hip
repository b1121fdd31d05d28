// RGB stem of the CIFAR networks (VGG layer 0): 3x3 conv, stride 1, pad 1, Cin <= 4 input
// channels read straight from the NHWC input (K laid out as 9 taps x 4 channels in registers, the
// missing channels as zeros: no padded copies of x or W), Cout = 64 -- the layer with K = 27
// that the generic GEMM tiles serve badly (one or two K-steps per tile, half of them padding;
// SURVEY.md §2.4).
//
// Both kernels use the exact fp32 MFMA (v_mfma_f32_32x32x2f32 / 16x16x4f32): the stem has < 1 %
// of the step's FLOPs, so fp32-input matrix cores cost nothing here and need no operand scaling.
//
//   stem_fwd_kernel    y = conv(x) + b, plus the per-256-row BatchNorm partials (mean, M2) that
//                      bn_finalize merges -- one pass, y written once.
//   stem_wgrad_kernel  dW partials with the BatchNorm/ReLU/max-pool backward applied on the fly:
//                      dy = scale * (route(gout) - S0/M - xhat * S1/M) is never written to memory
//                      (for VGG-11 at B=256 that is a 67 MB write + read saved per step).
//
// Reference anchor: the first Conv2d(3, 64, 3, padding=1) + BatchNorm2d + ReLU + MaxPool2d(2) of
// /root/reference/src/Part 1/model.py:14-25.
#include "common.h"
#include "kernels.h"
#include "x3_common.h"

#include <algorithm>

namespace cdp {

namespace {


// ---------------------------------------------------------------------------------- y tile
// The 256-pixel x 64-channel conv tile: 4 waves of 64 pixels x 64 channels (2 x 2 tiles of 32 x 32). K = 9 taps x
// 4 channels = 36 = 18 MFMA steps of k = 2; per tap a lane feeds two channels of its pixel (k even /
// odd half of the wave).
//
// B operand image: wl[co][k], k = 4 tap + c over the raw [Co][9][Cin] weights, channels >= Cin zero.
// Step 1 issues this thread's 9 weight loads, step 2 (after the x loads are in flight) stores them.
__device__ __forceinline__ void stem_w_issue(const float* __restrict__ w, int Cin, float (&wv9)[9]) {
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(w, (unsigned)(64 * 9 * Cin * 4));
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int e = tid + 256 * q, co = e / 36, k = e - co * 36, tap = k >> 2, c = k & 3;
    const unsigned o = c < Cin ? (unsigned)((co * 9 * Cin + tap * Cin + c) * 4) : kOOB;
    wv9[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wr, (int)o, 0, 0));
  }
}
__device__ __forceinline__ void stem_w_store(const float (&wv9)[9], float (*wl)[37]) {
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int e = threadIdx.x + 256 * q, co = e / 36, k = e - co * 36;
    wl[co][k] = wv9[q];
  }
}
// x operand of this wave's 64 pixels m0w .. m0w + 63 (buffer loads: padding taps, channels >= Cin
// and pixels >= M read 0 -- no branches around the loads)
__device__ __forceinline__ void stem_x_issue(__amdgpu_buffer_rsrc_t xr, int m0w, int M, int H, int W, int Cin,
                                             float (&lo)[9][2], float (&hi)[9][2]) {
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  int pn[2], pp[2], pq[2];
  bool pok[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int m = m0w + 32 * a + i;
    pok[a] = m < M;
    const int mm = pok[a] ? m : 0;
    pn[a] = mm / (H * W);
    const int r = mm - pn[a] * H * W;
    pp[a] = r / W;
    pq[a] = r - pp[a] * W;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int kh = t / 3, kw = t - 3 * (t / 3);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int ih = pp[a] + kh - 1, iw = pq[a] + kw - 1;
      const bool ok = pok[a] && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const unsigned o = ok ? (unsigned)((((pn[a] * H + ih) * W + iw) * Cin) * 4) : kOOB;
      lo[t][a] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)(h < Cin ? o + 4u * h : kOOB), 0, 0));
      hi[t][a] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(xr, (int)(2 + h < Cin ? o + 4u * (2 + h) : kOOB), 0, 0));
    }
  }
}
// acc[a][b][r] = y[m0w + 32 a + (r & 3) + 8 (r >> 2) + 4 h][32 b + i] (conv + bias)
__device__ __forceinline__ void stem_y_mfma(const float (&lo)[9][2], const float (&hi)[9][2], const float (*wl)[37],
                                            const float* __restrict__ bias, f32x16 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float bv = bias ? bias[32 * b + i] : 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = bv;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(lo[t][a], wl[32 * b + i][4 * t + h], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(hi[t][a], wl[32 * b + i][4 * t + 2 + h], acc[a][b], 0, 0, 0);
      }
}
// ---------------------------------------------------------------------------------- forward
// y = conv(x) + b (when y != nullptr) and the per-256-row BatchNorm partials (mean, M2).
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ y,
                                                       float* __restrict__ part, int N, int H, int W, int Cin) {
  constexpr int Co = 64;  // one block column: row stride and output offsets are compile-time
  __shared__ float red[4][64];
  __shared__ float wl[64][37];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int M = N * H * W;
  const int m0 = blockIdx.x * 256 + wv * 64;

  // loads in one batch (one memory latency): weights, then the 36 x values
  float wv9[9];
  stem_w_issue(w, Cin, wv9);
  float lo[9][2], hi[9][2];
  stem_x_issue(make_rsrc(x, (unsigned)((long long)M * Cin * 4)), m0, M, H, W, Cin, lo, hi);
  stem_w_store(wv9, wl);
  lds_barrier();
  f32x16 acc[2][2];
  stem_y_mfma(lo, hi, wl, bias, acc);

  // epilogue: BN partials, then the y stores last -- a barrier after them would make every wave
  // wait for its stores to reach memory (the stats' barriers come first instead)
  const bool full = (int)blockIdx.x * 256 + 256 <= M;
  if (part) {
    const int cnt = min(256, M - (int)blockIdx.x * 256);
    float csum[2] = {0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
          csum[b] += m < M ? acc[a][b][r] : 0.f;
        }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      csum[b] += __shfl_xor(csum[b], 32, 64);
      if (h == 0) red[wv][32 * b + i] = csum[b];
    }
    __syncthreads();
    float mean[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int c = 32 * b + i;
      mean[b] = (red[0][c] + red[1][c] + red[2][c] + red[3][c]) / (float)cnt;
    }
    __syncthreads();
    float cm2[2] = {0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float d = acc[a][b][r] - mean[b];
          cm2[b] += m < M ? d * d : 0.f;
        }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      cm2[b] += __shfl_xor(cm2[b], 32, 64);
      if (h == 0) red[wv][32 * b + i] = cm2[b];
    }
    __syncthreads();
    if (wv == 0 && h == 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int c = 32 * b + i;
        float* dst = part + ((long long)blockIdx.x * Co + c) * 2;
        dst[0] = mean[b];
        dst[1] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
      }
    }
  }
  // y (lane: column i of each 32-wide tile, 16 rows): one base address per lane, the 64 stores at
  // compile-time offsets
  float* yb = y + (long long)(m0 + 4 * h) * Co + i;
  if (full) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) yb[(32 * a + (r & 3) + 8 * (r >> 2)) * Co + 32 * b] = acc[a][b][r];
  } else {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h < M)
            yb[(32 * a + (r & 3) + 8 * (r >> 2)) * Co + 32 * b] = acc[a][b][r];
  }
}

// ---------------------------------------------------------------------------------- weight grad
// v_mfma_f32_16x16x4f32 with its k = 4 spread over 4 max-pool windows: lane l = (i = l % 16,
// j = l / 16) owns window j of the wave's current group of 4, and the 4 pixels of every window go
// through 4 successive MFMA steps (step p: k-slot j = pixel p of window j). A lane thus holds
// its window's whole 2 x 2 patch and routes the pool gradient without any cross-lane exchange.
// Rows and columns are permuted so every operand is one wide load per lane:
//   A tile ct, row r  <-> channel co = 4 r + ct  (lane i holds channels 4i..4i+3: one float4 of y / gout)
//   B tile c,  col t  <-> tap t (< 9), input channel c (lane i = tap i: its Cin values are contiguous)
// C[co][tap, c] += dy[px][co] * x[px shifted by tap][c]; the permutation is undone when the block
// writes its partial [Co = 64][36] (k = 4 tap + c, the slab reduction keeps the first Cin of 4).
template <int CIN>
__global__ __launch_bounds__(256, 2) void stem_wgrad_kernel(const float* __restrict__ y, const float* __restrict__ gout,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ sums,
                                                            const float* __restrict__ x, float* __restrict__ slab,
                                                            int N, int H, int W) {
  constexpr int C = 64;
  __shared__ float red[4][C][36];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, j = lane >> 4;
  const int Ho = H >> 1, Wo = W >> 1;
  const int nwin = N * Ho * Wo;
  const float invM = 1.f / (float)(N * H * W);

  float sc[4], sh[4], mu[4], is[4], k1[4], k2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 4 * i + e;
    mu[e] = stats[c];
    is[e] = stats[C + c];
    sc[e] = stats[2 * C + c];
    sh[e] = stats[3 * C + c];
    k1[e] = sums[c] * invM;
    k2[e] = sums[C + c] * invM;
  }
  const bool tap_ok = i < 9;
  const int tkh = i / 3 - 1, tkw = i - 3 * (i / 3) - 1;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, (unsigned)((long long)N * H * W * CIN * 4));

  f32x4 acc[4][CIN];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int c = 0; c < CIN; ++c) acc[ct][c] = f32x4{};

  // each wave takes groups of 4 windows, U groups per iteration (all loads issued up front)
  constexpr int U = 2;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  for (int g0 = gw; 4 * g0 < nwin; g0 += U * nw) {
    float4 yv[U][4], gv[U];
    float xv[U][4][CIN];
    bool wok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int win = 4 * (g0 + u * nw) + j;
      wok[u] = win < nwin;
      const int wn = wok[u] ? win : 0;
      const int n = wn / (Ho * Wo);
      const int r = wn - n * Ho * Wo;
      const int ho = r / Wo, wo = r - (r / Wo) * Wo;
      gv[u] = *reinterpret_cast<const float4*>(gout + (long long)wn * C + 4 * i);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int ph = 2 * ho + (p >> 1), pw = 2 * wo + (p & 1);
        yv[u][p] = *reinterpret_cast<const float4*>(y + (((long long)n * H + ph) * W + pw) * C + 4 * i);
        const int ih = ph + tkh, iw = pw + tkw;
        const bool ok = wok[u] && tap_ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const unsigned o = ok ? (unsigned)(((n * H + ih) * W + iw) * CIN * 4) : kOOB;
#pragma unroll
        for (int c = 0; c < CIN; ++c)
          xv[u][p][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)(o + 4u * c), 0, 0));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // pool routing of the window (same as bn_bwd_apply: first max wins), then dy per pixel
      float dyv[4][4];  // [pixel][channel e]
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float yy[4], z[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          yy[p] = e == 0 ? yv[u][p].x : e == 1 ? yv[u][p].y : e == 2 ? yv[u][p].z : yv[u][p].w;
          z[p] = fmaxf(fmaf(yy[p], sc[e], sh[e]), 0.f);
        }
        const float gg = e == 0 ? gv[u].x : e == 1 ? gv[u].y : e == 2 ? gv[u].z : gv[u].w;
        int arg = 0;
        float mx = z[0];
        if (z[1] > mx) { mx = z[1]; arg = 1; }
        if (z[2] > mx) { mx = z[2]; arg = 2; }
        if (z[3] > mx) { mx = z[3]; arg = 3; }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float dz = (arg == p && mx > 0.f) ? gg : 0.f;
          const float xh = (yy[p] - mu[e]) * is[e];
          dyv[p][e] = wok[u] ? sc[e] * (dz - k1[e] - xh * k2[e]) : 0.f;
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int c = 0; c < CIN; ++c)
            acc[ct][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(dyv[p][ct], xv[u][p][c], acc[ct][c], 0, 0, 0);
    }
  }
  // D layout: lane l holds rows 4 (l / 16) + v (channel co = 4 row + ct), column l % 16 (tap)
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (i < 9) {
#pragma unroll
        for (int v = 0; v < 4; ++v) red[wv][4 * (4 * j + v) + ct][4 * i + c] = c < CIN ? acc[ct][c < CIN ? c : 0][v] : 0.f;
      }
    }
  __syncthreads();
  float* dst = slab + (long long)blockIdx.x * C * 36;
  for (int e = tid; e < C * 36; e += 256) {
    const int co = e / 36, k = e - co * 36;
    dst[e] = (red[0][co][k] + red[1][co][k]) + (red[2][co][k] + red[3][co][k]);
  }
}


}  // namespace

bool stem_ok(int Cin, int KH, int KW, int stride, int pad, int Co) {
  return Cin >= 1 && Cin <= 4 && KH == 3 && KW == 3 && stride == 1 && pad == 1 && Co == 64;
}

void stem_fwd_launch(const float* x, const float* w, const float* bias, float* y, float* part, int N, int H, int W,
                     int Cin, int Co, hipStream_t st) {
  const long long M = (long long)N * H * W;
  (void)Co;  // == 64 (stem_ok)
  hipLaunchKernelGGL(stem_fwd_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, x, w, bias, y, part, N, H,
                     W, Cin);
}

int stem_wgrad_blocks(int N, int H, int W) {
  const long long nwin = (long long)N * (H / 2) * (W / 2);
  long long b = (nwin + 63) / 64;  // >= 16 windows per wave (4 groups of 4)
  if (b > 1024) b = 1024;
  return (int)std::max<long long>(1, b);
}

void stem_wgrad_launch(const float* y, const float* gout, const float* stats, const float* sums, const float* x,
                       float* slab, int nblk, int N, int H, int W, int Cin, hipStream_t st) {
  if (Cin == 3)
    hipLaunchKernelGGL(stem_wgrad_kernel<3>, dim3(nblk), dim3(256), 0, st, y, gout, stats, sums, x, slab, N, H, W);
  else if (Cin == 4)
    hipLaunchKernelGGL(stem_wgrad_kernel<4>, dim3(nblk), dim3(256), 0, st, y, gout, stats, sums, x, slab, N, H, W);
  else if (Cin == 2)
    hipLaunchKernelGGL(stem_wgrad_kernel<2>, dim3(nblk), dim3(256), 0, st, y, gout, stats, sums, x, slab, N, H, W);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<1>, dim3(nblk), dim3(256), 0, st, y, gout, stats, sums, x, slab, N, H, W);
}

}  // namespace cdp
