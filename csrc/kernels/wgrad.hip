// Convolution weight-gradient on fp32-input MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
//   dW[co][(kh,kw,c)] = sum_m dY[m][co] * Xcol[m][(kh,kw,c)]     m = (n, p, q)
//
// This is the autograd weight-gradient of nn.Conv2d used by every reference stage
// (/root/reference/src/Part 1/main.py:40 `loss.backward()`), with the long reduction over
// N*P*Q split across workgroups (split-K) into fp32 slabs that a second kernel sums straight into
// the flat gradient arena (optionally accumulating, for gradient accumulation).
//
// Tile: 128 (co) x 128 (k) x 32 (m), 256 threads = 2x2 waves of 64x64. Both operands are staged
// m-major ([m][co] and [m][k]) exactly as they sit in memory, so no transpose is needed: an MFMA
// operand lane (i, h) reads row m = 2s + h, column i -- 32 consecutive floats per half-wave,
// conflict-free ds_read_b32.
#include <cstdlib>
#include <type_traits>

#include <algorithm>

#include "act_max.h"
#include "common.h"
#include "kernels.h"
#include "x3_common.h"
#include "wgrad_x3_body.h"

namespace cdp {
namespace {

using namespace x3wgrad;

// BM (co) x BN (k) x 32 (m) tile, 256 threads = 2x2 waves of (BM/2)x(BN/2).
template <int BM, int BN, bool FAST>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradParams p) {
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int STAGE = WBK * (LDA + LDB);
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int CPR_A = BM / 4, RPP_A = 256 / CPR_A, NP_A = WBK / RPP_A;  // float4 per row, rows/pass, passes
  constexpr int CPR_B = BN / 4, RPP_B = 256 / CPR_B, NP_B = WBK / RPP_B;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int ntn = (p.Kdim + BN - 1) / BN;
  const int ntm = (p.Cout + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // tile (tm, tn) fastest, split slowest: blocks of one split share the dY/X row window in L2
  const int tile = bid % (ntm * ntn);
  const int split = bid / (ntm * ntn);
  const int tm_idx = tile / ntn, tn_idx = tile % ntn;
  const int co0 = tm_idx * BM, r0 = tn_idx * BN;
  const int mt_total = (p.M + WBK - 1) / WBK;
  const int kt_begin = (int)(((long long)split * mt_total) / p.splits);
  const int kt_end = (int)(((long long)(split + 1) * mt_total) / p.splits);
  const int PQ = p.P * p.Q;

  float4 ra[NP_A], rb[NP_B];
  const int ca = tid % CPR_A, cb = tid % CPR_B;
  const int co = co0 + ca * 4;
  // per-thread B column decode (fixed for the whole kernel): k = r0 + 4*cb .. +3
  const int kcol = r0 + cb * 4;
  int b_kh = 0, b_kw = 0, b_c = 0;
  const bool b_kok = kcol < p.Kdim;
  if (FAST && b_kok) {
    const int tap = fdiv(kcol, p.fd_C);
    b_c = kcol - tap * p.C;
    b_kh = fdiv(tap, p.fd_KW);
    b_kw = tap - b_kh * p.KW;
  }

  auto load_tile = [&](int kt) {
    const int mb = kt * WBK;
#pragma unroll
    for (int i = 0; i < NP_A; ++i) {
      const int m = mb + tid / CPR_A + RPP_A * i;
      const bool mok = m < p.M;
      if (FAST) {
        ra[i] = (mok && co < p.Cout) ? ld4(p.dy + (long long)m * p.Cout + co) : f4zero();
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = (mok && co + j < p.Cout) ? p.dy[(long long)m * p.Cout + co + j] : 0.f;
        ra[i] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
#pragma unroll
    for (int i = 0; i < NP_B; ++i) {
      const int m = mb + tid / CPR_B + RPP_B * i;
      const bool mok = m < p.M;
      const int mm = mok ? m : 0;
      const int n = fdiv(mm, p.fd_PQ);
      const int rem = mm - n * PQ;
      const int pp = fdiv(rem, p.fd_Q), qq = rem - pp * p.Q;
      const int ih0 = pp * p.stride - p.pad, iw0 = qq * p.stride - p.pad;
      const float* xb = p.x + (long long)n * p.H * p.W * p.C;
      if (FAST) {
        const int ih = ih0 + b_kh, iw = iw0 + b_kw;
        const bool ok = mok && b_kok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        rb[i] = ok ? ld4(xb + ((long long)ih * p.W + iw) * p.C + b_c) : f4zero();
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = kcol + j;
          float v = 0.f;
          if (mok && k < p.Kdim) {
            const int tap = fdiv(k, p.fd_C);
            const int c = k - tap * p.C;
            const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
            const int ih = ih0 + kh, iw = iw0 + kw;
            if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
              v = xb[((long long)ih * p.W + iw) * p.C + c];
          }
          e[j] = v;
        }
        rb[i] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  };
  auto store_tile = [&](float* st) {
#pragma unroll
    for (int i = 0; i < NP_A; ++i) st4(st + (tid / CPR_A + RPP_A * i) * LDA + ca * 4, ra[i]);
#pragma unroll
    for (int i = 0; i < NP_B; ++i) st4(st + WBK * LDA + (tid / CPR_B + RPP_B * i) * LDB + cb * 4, rb[i]);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int l32 = lane & 31, hh = lane >> 5;
  if (kt_begin < kt_end) {
    load_tile(kt_begin);
    store_tile(smem);
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const int cur = (kt - kt_begin) & 1;
      const bool more = kt + 1 < kt_end;
      if (more) load_tile(kt + 1);
      const float* As = smem + cur * STAGE;
      const float* Bs = As + WBK * LDA;
#pragma unroll
      for (int s = 0; s < WBK / 2; ++s) {
        const int row = 2 * s + hh;
        float af[TM], bf[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = As[row * LDA + wm * (BM / 2) + a * 32 + l32];
#pragma unroll
        for (int b = 0; b < TN; ++b) bf[b] = Bs[row * LDB + wn * (BN / 2) + b * 32 + l32];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a], bf[b], acc[a][b], 0, 0, 0);
      }
      if (more) store_tile(smem + (cur ^ 1) * STAGE);
      __syncthreads();
    }
  }

  float* out = p.out + (long long)split * p.Cout * p.Kdim;
  const bool full = co0 + BM <= p.Cout && r0 + BN <= p.Kdim;
  auto store = [&](auto pred) {  // unpredicated stores for in-bounds tiles
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int k = r0 + wn * (BN / 2) + b * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = co0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (!decltype(pred)::value || (c < p.Cout && k < p.Kdim)) out[(long long)c * p.Kdim + k] = acc[a][b][r];
        }
      }
  };
  if (full) store(std::false_type{});
  else store(std::true_type{});
}

template <int BM, int BN, bool FAST, int NP = 3, bool PIPE = false>
__global__ __launch_bounds__(wg_threads<BM>(), BM >= 256 ? 1 : 2) void wgrad_x3_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[wgrad_x3_smem_elems<BM, BN, NP, PIPE>()];
  wgrad_x3_body<BM, BN, FAST, NP, PIPE>(p, smem, blockIdx.x, gridDim.x);
}

// dst[r][c] = (accumulate ? dst : 0) + sum_z slab[z][r][c]  over rows x src_cols, keeping the first
// dst_cols of each row (dst_cols < src_cols strips channel padding). Block = CB column slots x SL
// split lanes; the SL partial sums meet in LDS, so short slabs with many splits still spread over
// many workgroups.
template <int CB>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int S, long long n_src,
                                                       int src_cols, int dst_cols, float* __restrict__ dst,
                                                       int accumulate) {
  constexpr int SL = 256 / CB;
  __shared__ float red[SL][CB];
  const int cl = threadIdx.x % CB, sl = threadIdx.x / CB;
  const long long i = (long long)blockIdx.x * CB + cl;
  float s = 0.f;
  if (i < n_src) {
    int z = sl;
    for (; z + 3 * SL < S; z += 4 * SL) {
      const float a = slab[(long long)z * n_src + i], b = slab[(long long)(z + SL) * n_src + i];
      const float c = slab[(long long)(z + 2 * SL) * n_src + i], d = slab[(long long)(z + 3 * SL) * n_src + i];
      s += (a + b) + (c + d);
    }
    for (; z < S; z += SL) s += slab[(long long)z * n_src + i];
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && i < n_src) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < SL; ++k) t += red[k][cl];
    const long long r = i / src_cols;
    const int c = (int)(i - r * src_cols);
    if (c < dst_cols) {
      float* d = dst + r * dst_cols + c;
      *d = accumulate ? *d + t : t;
    }
  }
}

// Unstrided float4 form: dst[i] = (accumulate ? dst[i] : 0) + sum_z slab[z][i] for n % 4 == 0.
// CB float4 column slots x SL = 256 / CB split lanes per block; every thread keeps up to four
// independent 16-B loads in flight. CB is chosen at launch so the grid has >= ~1024 blocks.
template <int CB>
__global__ __launch_bounds__(256) void slab_sum4_kernel(const float4* __restrict__ slab, int S, long long n4,
                                                        float4* __restrict__ dst, int accumulate) {
  constexpr int SL = 256 / CB;
  __shared__ float4 red[SL > 1 ? SL : 1][CB];
  const int cl = threadIdx.x % CB, sl = threadIdx.x / CB;
  const long long i = (long long)blockIdx.x * CB + cl;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int z = sl;
    for (; z + 3 * SL < S; z += 4 * SL) {
      const float4 a = slab[(long long)z * n4 + i], b = slab[(long long)(z + SL) * n4 + i];
      const float4 c = slab[(long long)(z + 2 * SL) * n4 + i], d = slab[(long long)(z + 3 * SL) * n4 + i];
      s.x += (a.x + b.x) + (c.x + d.x);
      s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z);
      s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; z < S; z += SL) {
      const float4 a = slab[(long long)z * n4 + i];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  if constexpr (SL > 1) {
    red[sl][cl] = s;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < SL; ++k) {
      const float4 b = red[k][cl];
      s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
    }
  }
  if (i < n4) {
    if (accumulate) {
      const float4 o = dst[i];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    dst[i] = s;
  }
}

}  // namespace

template <int BM, int BN>
void wgrad_launch_t(const WgradParams& p, bool x3, hipStream_t st, int np) {
  const int ntn = (p.Kdim + BN - 1) / BN;
  const int ntm = (p.Cout + BM - 1) / BM;
  const bool fast = (p.C % 4) == 0 && (p.Cout % 4) == 0;
  dim3 grid(ntm * ntn * p.splits);
  if (x3) {
    if (np == 1) {
      if (fast) hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, true, 1>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, false, 1>), grid, dim3(256), 0, st, p);
    } else if (np == 2) {
      if (fast)
        hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, true, 2, true>), grid, dim3(wg_threads<BM>()), 0, st, p);
      else hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, false, 2>), grid, dim3(256), 0, st, p);
    } else if (fast) hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((wgrad_x3_kernel<BM, BN, false>), grid, dim3(256), 0, st, p);
  } else {
    if (fast) hipLaunchKernelGGL((wgrad_kernel<BM, BN, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((wgrad_kernel<BM, BN, false>), grid, dim3(256), 0, st, p);
  }
}

void wgrad_launch(const WgradParams& p, int bm, int bn, bool x3, hipStream_t st, int np) {
  if (bm == 256 && bn == 128 && x3 && np == 2 && (p.C % 4) == 0 && (p.Cout % 4) == 0) {
    // host plan only picks 256 for the pipelined f16x2 path (plan_wgrad)
    hipLaunchKernelGGL((wgrad_x3_kernel<256, 128, true, 2, true>), dim3(((p.Cout + 255) / 256) * ((p.Kdim + 127) / 128) * p.splits),
                       dim3(512), 0, st, p);
    return;
  }
  if (bm == 128 && bn == 128) wgrad_launch_t<128, 128>(p, x3, st, np);
  else if (bm == 128) wgrad_launch_t<128, 64>(p, x3, st, np);
  else if (bn == 128) wgrad_launch_t<64, 128>(p, x3, st, np);
  else wgrad_launch_t<64, 64>(p, x3, st, np);
}

// ---------------------------------------------------------------- standalone act max
namespace {
// Per-image / per-channel |max| of an NHWC activation [N][HW][C] (act_max.h) for operands no fused
// producer measured (user inputs, a classifier's input, tests). Block b reads the contiguous range
// [b * per, (b + 1) * per) of float4s (VEC, C % 4 == 0; per a multiple of 256 and of C / 4 when
// qmode != 0, as in bn_act_fwd_kernel) or of floats.
template <bool VEC>
__global__ __launch_bounds__(256) void act_max_kernel(const float* __restrict__ x, int N, int C, int total, int per,
                                                      int qmode, FastDiv fd_U, FastDiv fd_HW, ActMaxOut am) {
  __shared__ ActMaxBlock<kMaxActC> sam;
  const int tid = threadIdx.x;
  const int U = VEC ? C / 4 : C;  // units (float4 or float) per pixel
  const int i0 = blockIdx.x * per, i1 = min(total, i0 + per);
  const int img0 = fdiv(fdiv(min(i0, total - 1), fd_U), fd_HW);
  const bool lds_ch = C <= kMaxActC;
  sam.init(tid, 256);
  __syncthreads();
  ImgRun run;
  float4 cm[2] = {f4zero(), f4zero()};
  int k = 0;
  for (int i = i0 + tid; i < i1; i += 256, ++k) {
    const int pix = fdiv(i, fd_U);
    const int u = i - pix * U;
    const int img = fdiv(pix, fd_HW);
    if constexpr (VEC) {
      const float4 v = ld4(x + 4LL * i);
      run.add(img, absmax4(v), sam, img0, am);
      if (qmode == 1 || (qmode == 2 && !(k & 1))) cm[0] = absmax4(cm[0], v);
      else if (qmode == 2) cm[1] = absmax4(cm[1], v);
      else if (lds_ch) sam.add_ch4(4 * u, make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)));
      else {
        const float e[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
        for (int j = 0; j < 4; ++j)
          if (__float_as_uint(e[j])) glb_max_u32(&am.ch[4 * u + j], __float_as_uint(e[j]));
      }
    } else {
      const float v = fabsf(x[i]);
      run.add(img, v, sam, img0, am);
      if (lds_ch) sam.add_ch(u, v);
      else if (__float_as_uint(v)) glb_max_u32(&am.ch[u], __float_as_uint(v));
    }
  }
  run.flush(sam, img0, am);
  if (VEC && qmode == 1 && i0 + tid < i1) sam.add_ch4(4 * (tid % U), cm[0]);
  if (VEC && qmode == 2) {
    if (i0 + tid < i1) sam.add_ch4(4 * tid, cm[0]);
    if (i0 + tid + 256 < i1) sam.add_ch4(4 * (tid + 256), cm[1]);
  }
  __syncthreads();
  sam.publish(am, img0, N, 0, lds_ch ? C : 0, C, blockIdx.x % kActCopies, tid, 256);
}
}  // namespace

void act_max_launch(const float* x, int N, long long HW, int C, ActMaxOut o, hipStream_t st) {
  const bool vec = (C % 4) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int U = vec ? C / 4 : C;
  const long long total = (long long)N * HW * U;
  if (total <= 0) return;
  const int qmode = !vec ? 0 : (U <= 256 && (256 % U) == 0) ? 1 : U == 512 ? 2 : 0;
  const long long unit = qmode == 2 ? 512 : 256;
  const long long blocks = std::min<long long>(1024, std::max<long long>(1, (total + 255) / 256));
  const long long per = std::max(unit, ((total + blocks - 1) / blocks + unit - 1) / unit * unit);
  const dim3 grid((unsigned)((total + per - 1) / per));
  if (vec)
    hipLaunchKernelGGL(act_max_kernel<true>, grid, dim3(256), 0, st, x, N, C, (int)total, (int)per, qmode,
                       make_fastdiv(U), make_fastdiv((int)HW), o);
  else
    hipLaunchKernelGGL(act_max_kernel<false>, grid, dim3(256), 0, st, x, N, C, (int)total, (int)per, 0,
                       make_fastdiv(U), make_fastdiv((int)HW), o);
}

void slab_sum_launch(const float* slab, int S, long long n, float* dst, bool accumulate, hipStream_t st) {
  slab_sum_strided_launch(slab, S, n, 1, 1, dst, accumulate, st);
}

void slab_sum_strided_launch(const float* slab, int S, long long n_src, int src_cols, int dst_cols, float* dst,
                             bool accumulate, hipStream_t st) {
  const bool vec = src_cols == dst_cols && n_src % 4 == 0 && (reinterpret_cast<uintptr_t>(slab) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  if (vec) {
    const long long n4 = n_src / 4;
    const float4* s4 = reinterpret_cast<const float4*>(slab);
    float4* d4 = reinterpret_cast<float4*>(dst);
    const int acc = accumulate ? 1 : 0;
    // widest column slot count that still gives >= 1024 blocks (more split lanes when n is short)
    if (n4 >= 256LL * 1024 || S <= 1)
      hipLaunchKernelGGL(slab_sum4_kernel<256>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, s4, S, n4, d4,
                         acc);
    else if (n4 >= 64LL * 1024 || S <= 4)
      hipLaunchKernelGGL(slab_sum4_kernel<64>, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, s4, S, n4, d4,
                         acc);
    else
      hipLaunchKernelGGL(slab_sum4_kernel<16>, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st, s4, S, n4, d4,
                         acc);
    return;
  }
  if (S >= 16 && n_src < (1 << 18)) {
    hipLaunchKernelGGL(slab_sum_kernel<16>, dim3((unsigned)((n_src + 15) / 16)), dim3(256), 0, st, slab, S, n_src,
                       src_cols, dst_cols, dst, accumulate ? 1 : 0);
  } else {
    hipLaunchKernelGGL(slab_sum_kernel<64>, dim3((unsigned)((n_src + 63) / 64)), dim3(256), 0, st, slab, S, n_src,
                       src_cols, dst_cols, dst, accumulate ? 1 : 0);
  }
}

}  // namespace cdp
