// Implicit-GEMM convolution on fp32-input MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
// One kernel family serves:
//   * conv forward          rows m = (n, p, q) output pixels, K = (kh, kw, c), N = Cout
//   * conv data-gradient     rows m = (n, ih, iw) input pixels, K = (kh, kw, cout), N = Cin,
//                            gathered "transposed" from dY with the pre-transposed weight
//   * Linear forward         a 1x1 conv over [B,1,1,I]
//
// Reference semantics: nn.Conv2d(k=3,s=1,p=1,bias=True) at /root/reference/src/Part 1/model.py:18-23
// (and the strided / 1x1 / 7x7 convs of the ResNet-50 config). The reference runs them through
// ATen/oneDNN on CPU; here they are one LDS-tiled MFMA kernel with the bias add and the per-block
// BatchNorm statistics (mean, M2 -- Chan's parallel form) fused into the epilogue, so the
// following BatchNorm never re-reads the conv output for its statistics.
//
// Tile: BM x BN x 32, 256 threads = 4 waves as 2x2, each wave (BM/2)x(BN/2) built from 32x32
// MFMA tiles. Operands are staged global -> registers -> LDS (double buffered, one barrier per
// K-tile); the gather needs per-lane zero-padding, which LDS-DMA cannot express. Rows of both LDS
// tiles are K-contiguous with a 16-byte pad (36 floats) so the ds_read_b128 fragment reads are
// bank-conflict free (MI355X_MICROARCH.md §LDS, ds_read_b128 lane groups). The MFMA K index is
// permuted: lanes 0-31 consume k = s, lanes 32-63 consume k = 16 + s at step s, so each lane
// reads 4 consecutive k per ds_read_b128.
#include "common.h"
#include "kernels.h"
#include "conv_epilogue.h"

namespace cdp {

namespace {

constexpr int BK = 32;
constexpr int LDK = BK + 4;

// MODE 0: C % 32 == 0 (a K-tile lies in one filter tap: one decode per tile)
// MODE 1: C % 4 == 0  (float4 gathers, per-float4 tap decode; e.g. the channel-padded RGB stem)
// MODE 2: anything   (scalar gathers)
template <int BM, int BN, int MODE, bool DGRAD>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvGemmParams p) {
  constexpr int TM = BM / 64;  // 32-row MFMA tiles per wave
  constexpr int TN = BN / 64;  // 32-col MFMA tiles per wave
  constexpr int STAGE = (BM + BN) * LDK;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  static_assert(2 * STAGE >= epi_lds_floats<BM, BN>(), "epilogue scratch");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int ntn = (p.Nout + BN - 1) / BN;
  const int total = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, total);
  // order: tn fastest, then split, then tm -> blocks sharing an A slice are adjacent
  const int tn_idx = bid % ntn;
  const int rest = bid / ntn;
  const int split = rest % p.splits;
  const int tm_idx = rest / p.splits;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;

  const int kt_begin = (int)(((long long)split * p.ktiles) / p.splits);
  const int kt_end = (int)(((long long)(split + 1) * p.ktiles) / p.splits);

  const int PQ = p.P * p.Q;

  // ---------------- per-thread gather setup ----------------
  // vector modes: each thread owns BM/32 A rows (row = tid/8 + 32*i) and one float4 column (tid%8).
  // scalar mode: each thread owns one A row and CPT consecutive scalar columns.
  constexpr bool VEC = MODE != 2;
  constexpr int A_LD = VEC ? BM / 32 : 1;
  constexpr int B_LD = VEC ? BN / 32 : 1;
  constexpr int TPR_A = 256 / BM;            // generic: threads per A row
  constexpr int CPT_A = BK / TPR_A;          // generic: columns per thread (A)
  constexpr int TPR_B = 256 / BN;
  constexpr int CPT_B = BK / TPR_B;

  const float* a_base[A_LD];
  int a_h[A_LD], a_w[A_LD];
  bool a_ok[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int row = VEC ? ((tid >> 3) + 32 * i) : (tid / TPR_A);
    const int m = m0 + row;
    a_ok[i] = m < p.M;
    const int mm = a_ok[i] ? m : 0;
    const int n = fdiv(mm, p.fd_PQ);
    const int rem = mm - n * PQ;
    const int pp = fdiv(rem, p.fd_Q);
    const int qq = rem - pp * p.Q;
    a_base[i] = p.x + (long long)n * p.H * p.W * p.C;
    if (DGRAD) {
      a_h[i] = pp + p.pad;  // oh*stride = ih + pad - kh
      a_w[i] = qq + p.pad;
    } else {
      a_h[i] = pp * p.stride - p.pad;
      a_w[i] = qq * p.stride - p.pad;
    }
  }

  float4 ra[VEC ? A_LD : 1];
  float4 rb[VEC ? B_LD : 1];
  float sa[VEC ? 1 : CPT_A];
  float sb[VEC ? 1 : CPT_B];

  auto pix_ok = [&](int i, int kh, int kw, int& ih, int& iw) -> bool {
    if (DGRAD) {
      int oh = a_h[i] - kh, ow = a_w[i] - kw;
      if (oh < 0 || ow < 0) return false;
      if (p.stride != 1) {
        if ((oh % p.stride) | (ow % p.stride)) return false;
        oh /= p.stride;
        ow /= p.stride;
      }
      ih = oh;
      iw = ow;
      return oh < p.H && ow < p.W;
    } else {
      ih = a_h[i] + kh;
      iw = a_w[i] + kw;
      return (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    }
  };

  auto load_tile = [&](int kt) {
    const int r0 = kt * BK;
    if (MODE == 1) {
      const int r = r0 + (tid & 7) * 4;
      const bool rok = r < p.Kdim;
      const int tap = fdiv(r, p.fd_C);
      const int c = r - tap * p.C;
      const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        int ih, iw;
        const bool ok = rok && a_ok[i] && pix_ok(i, kh, kw, ih, iw);
        ra[i] = ok ? ld4(a_base[i] + ((long long)ih * p.W + iw) * p.C + c) : f4zero();
      }
#pragma unroll
      for (int i = 0; i < B_LD; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        rb[i] = (rok && n < p.Nout) ? ld4(p.w + (long long)n * p.Kdim + r) : f4zero();
      }
    } else if (MODE == 0) {
      const int tap = fdiv(r0, p.fd_C);
      const int c0 = r0 - tap * p.C + (tid & 7) * 4;
      const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        int ih, iw;
        const bool ok = a_ok[i] && pix_ok(i, kh, kw, ih, iw);
        ra[i] = ok ? ld4(a_base[i] + ((long long)ih * p.W + iw) * p.C + c0) : f4zero();
      }
#pragma unroll
      for (int i = 0; i < B_LD; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        rb[i] = (n < p.Nout) ? ld4(p.w + (long long)n * p.Kdim + r0 + (tid & 7) * 4) : f4zero();
      }
    } else {
      const int cbase = (tid % TPR_A) * CPT_A;
#pragma unroll
      for (int j = 0; j < CPT_A; ++j) {
        const int r = r0 + cbase + j;
        float v = 0.f;
        if (a_ok[0] && r < p.Kdim) {
          const int tap = fdiv(r, p.fd_C);
          const int c = r - tap * p.C;
          const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
          int ih, iw;
          if (pix_ok(0, kh, kw, ih, iw)) v = a_base[0][((long long)ih * p.W + iw) * p.C + c];
        }
        sa[j] = v;
      }
      const int nrow = n0 + tid / TPR_B;
      const int cb = (tid % TPR_B) * CPT_B;
#pragma unroll
      for (int j = 0; j < CPT_B; ++j) {
        const int r = r0 + cb + j;
        sb[j] = (nrow < p.Nout && r < p.Kdim) ? p.w[(long long)nrow * p.Kdim + r] : 0.f;
      }
    }
  };

  auto store_tile = [&](float* st) {
    float* As = st;
    float* Bs = st + BM * LDK;
    if (VEC) {
#pragma unroll
      for (int i = 0; i < A_LD; ++i) st4(As + ((tid >> 3) + 32 * i) * LDK + (tid & 7) * 4, ra[i]);
#pragma unroll
      for (int i = 0; i < B_LD; ++i) st4(Bs + ((tid >> 3) + 32 * i) * LDK + (tid & 7) * 4, rb[i]);
    } else {
      const int arow = tid / TPR_A, acb = (tid % TPR_A) * CPT_A;
#pragma unroll
      for (int j = 0; j < CPT_A; ++j) As[arow * LDK + acb + j] = sa[j];
      const int brow = tid / TPR_B, bcb = (tid % TPR_B) * CPT_B;
#pragma unroll
      for (int j = 0; j < CPT_B; ++j) Bs[brow * LDK + bcb + j] = sb[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int koff = (lane >> 5) * 16;
  const int l32 = lane & 31;

  if (kt_begin < kt_end) {
    load_tile(kt_begin);
    store_tile(smem);
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const int cur = (kt - kt_begin) & 1;
      const bool more = kt + 1 < kt_end;
      if (more) load_tile(kt + 1);
      const float* As = smem + cur * STAGE;
      const float* Bs = As + BM * LDK;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        float4 af[TM], bf[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = ld4(As + (wm * (BM / 2) + a * 32 + l32) * LDK + koff + s4 * 4);
#pragma unroll
        for (int b = 0; b < TN; ++b) bf[b] = ld4(Bs + (wn * (BN / 2) + b * 32 + l32) * LDK + koff + s4 * 4);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].x, bf[b].x, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].y, bf[b].y, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].z, bf[b].z, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].w, bf[b].w, acc[a][b], 0, 0, 0);
          }
      }
      if (more) store_tile(smem + (cur ^ 1) * STAGE);
      __syncthreads();
    }
  }

  conv_epilogue<BM, BN>(p, acc, smem, m0, n0, tm_idx, split);
}

// Sum split-K slabs, add bias, store, and emit BatchNorm partials over RB-row groups.
// Thread = one output column of a 64-column strip; 4 row lanes x RB/4 rows.
constexpr int RB = 32;
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int S, int M, int Nout,
                                                            const float* __restrict__ bias, float* y,
                                                            float* __restrict__ part, RowRemap rr,
                                                            const float* addend) {
  __shared__ float red[4][64];
  const int col = threadIdx.x & 63;
  const int rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + col;
  const int y0 = blockIdx.y * RB;
  const bool nok = n < Nout;
  const float bv = (bias && nok) ? bias[n] : 0.f;
  float v[RB / 4];
  const long long plane = (long long)M * Nout;
#pragma unroll
  for (int i = 0; i < RB / 4; ++i) {
    const int m = y0 + rl + 4 * i;
    float s = 0.f;
    if (m < M && nok) {
      const float* src = slab + (long long)m * Nout + n;
      for (int z = 0; z < S; ++z) s += src[z * plane];
      s += bv;
      const long long o = remap_row(rr, m) * Nout + n;
      if (addend) s += addend[o];
      y[o] = s;
    }
    v[i] = s;
  }
  if (!part) return;
  const int cnt = min(RB, M - y0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < RB / 4; ++i) s += (y0 + rl + 4 * i < M) ? v[i] : 0.f;
  red[rl][col] = s;
  __syncthreads();
  const float mean = (red[0][col] + red[1][col] + red[2][col] + red[3][col]) / (float)cnt;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int i = 0; i < RB / 4; ++i) {
    const float d = v[i] - mean;
    s += (y0 + rl + 4 * i < M) ? d * d : 0.f;
  }
  red[rl][col] = s;
  __syncthreads();
  if (rl == 0 && nok) {
    float* dst = part + ((long long)blockIdx.y * Nout + n) * 2;
    dst[0] = mean;
    dst[1] = red[0][col] + red[1][col] + red[2][col] + red[3][col];
  }
}

// float4 variant (Nout % 4 == 0): block = 16 column quads (64 columns) x 16 row lanes, RB rows;
// every thread keeps 2 rows x 4 columns in registers and issues its S slab loads back to back.
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* __restrict__ slab, int S, int M, int Nout,
                                                             const float* __restrict__ bias, float* y,
                                                             float* __restrict__ part, RowRemap rr,
                                                            const float* addend) {
  __shared__ float4 red[16][16];
  const int cq = threadIdx.x & 15;
  const int rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + cq * 4;
  const int y0 = blockIdx.y * RB;
  const bool nok = n < Nout;
  const float4 bv = (bias && nok) ? ld4(bias + n) : f4zero();
  const long long plane = (long long)M * Nout;
  float4 v[RB / 16];
  // all rows' slab loads in batches of 8 splits (one memory round trip per batch, not one per 4
  // splits and row): out-of-range rows / splits load a valid address and are masked to zero
  float4 acc[RB / 16];
#pragma unroll
  for (int i = 0; i < RB / 16; ++i) acc[i] = f4zero();
  const bool any = nok && y0 + rl < M;
  for (int z0 = 0; any && z0 < S; z0 += 8) {
    float4 t[RB / 16][8];
#pragma unroll
    for (int i = 0; i < RB / 16; ++i) {
      const int m = y0 + rl + 16 * i;
      const float* src = slab + (long long)(m < M ? m : y0 + rl) * Nout + n;
#pragma unroll
      for (int k = 0; k < 8; ++k) t[i][k] = ld4(src + (long long)(z0 + k < S ? z0 + k : 0) * plane);
    }
#pragma unroll
    for (int i = 0; i < RB / 16; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (z0 + k >= S) t[i][k] = f4zero();
#pragma unroll
    for (int i = 0; i < RB / 16; ++i) {
      float4& a = acc[i];
      a.x += ((t[i][0].x + t[i][1].x) + (t[i][2].x + t[i][3].x)) + ((t[i][4].x + t[i][5].x) + (t[i][6].x + t[i][7].x));
      a.y += ((t[i][0].y + t[i][1].y) + (t[i][2].y + t[i][3].y)) + ((t[i][4].y + t[i][5].y) + (t[i][6].y + t[i][7].y));
      a.z += ((t[i][0].z + t[i][1].z) + (t[i][2].z + t[i][3].z)) + ((t[i][4].z + t[i][5].z) + (t[i][6].z + t[i][7].z));
      a.w += ((t[i][0].w + t[i][1].w) + (t[i][2].w + t[i][3].w)) + ((t[i][4].w + t[i][5].w) + (t[i][6].w + t[i][7].w));
    }
  }
#pragma unroll
  for (int i = 0; i < RB / 16; ++i) {
    const int m = y0 + rl + 16 * i;
    float4 s = acc[i];
    if (m < M && nok) {
      s.x += bv.x; s.y += bv.y; s.z += bv.z; s.w += bv.w;
      const long long o = remap_row(rr, m) * Nout + n;
      if (addend) {
        const float4 ad = ld4(addend + o);
        s.x += ad.x; s.y += ad.y; s.z += ad.z; s.w += ad.w;
      }
      st4(y + o, s);
    }
    v[i] = s;
  }
  if (!part) return;
  const int cnt = min(RB, M - y0);
  float4 t = f4zero();
#pragma unroll
  for (int i = 0; i < RB / 16; ++i)
    if (y0 + rl + 16 * i < M) { t.x += v[i].x; t.y += v[i].y; t.z += v[i].z; t.w += v[i].w; }
  red[rl][cq] = t;
  __syncthreads();
  float4 mean = f4zero();
#pragma unroll
  for (int k = 0; k < 16; ++k) { mean.x += red[k][cq].x; mean.y += red[k][cq].y; mean.z += red[k][cq].z; mean.w += red[k][cq].w; }
  const float ic = 1.f / (float)cnt;
  mean.x *= ic; mean.y *= ic; mean.z *= ic; mean.w *= ic;
  __syncthreads();
  t = f4zero();
#pragma unroll
  for (int i = 0; i < RB / 16; ++i)
    if (y0 + rl + 16 * i < M) {
      const float a = v[i].x - mean.x, b = v[i].y - mean.y, c = v[i].z - mean.z, d = v[i].w - mean.w;
      t.x += a * a; t.y += b * b; t.z += c * c; t.w += d * d;
    }
  red[rl][cq] = t;
  __syncthreads();
  if (rl == 0 && nok) {
    float4 q = f4zero();
#pragma unroll
    for (int k = 0; k < 16; ++k) { q.x += red[k][cq].x; q.y += red[k][cq].y; q.z += red[k][cq].z; q.w += red[k][cq].w; }
    float* dst = part + ((long long)blockIdx.y * Nout + n) * 2;
    dst[0] = mean.x; dst[1] = q.x; dst[2] = mean.y; dst[3] = q.y;
    dst[4] = mean.z; dst[5] = q.z; dst[6] = mean.w; dst[7] = q.w;
  }
}

template <int BM, int BN, int MODE, bool DGRAD>
void launch_igemm(const ConvGemmParams& p, int ntiles, hipStream_t st) {
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, MODE, DGRAD>), dim3(ntiles * p.splits), dim3(256), 0, st, p);
}

template <int MODE, bool DGRAD>
void dispatch_tile(const ConvGemmParams& p, int bm, int bn, hipStream_t st) {
  const int ntm = (p.M + bm - 1) / bm, ntn = (p.Nout + bn - 1) / bn;
  const int nt = ntm * ntn;
  if (bm == 128 && bn == 128) launch_igemm<128, 128, MODE, DGRAD>(p, nt, st);
  else if (bm == 128 && bn == 64) launch_igemm<128, 64, MODE, DGRAD>(p, nt, st);
  else if (bm == 64 && bn == 128) launch_igemm<64, 128, MODE, DGRAD>(p, nt, st);
  else launch_igemm<64, 64, MODE, DGRAD>(p, nt, st);
}

}  // namespace

int conv_igemm_rows_per_part(int bm) { return bm; }
int splitk_rows_per_part() { return RB; }

void conv_igemm_launch(const ConvGemmParams& p, int bm, int bn, bool dgrad, hipStream_t st) {
  if ((p.C % BK) == 0 && (p.Kdim % BK) == 0) {
    if (dgrad) dispatch_tile<0, true>(p, bm, bn, st);
    else dispatch_tile<0, false>(p, bm, bn, st);
  } else if ((p.C % 4) == 0 && (p.Kdim % 4) == 0) {
    if (dgrad) dispatch_tile<1, true>(p, bm, bn, st);
    else dispatch_tile<1, false>(p, bm, bn, st);
  } else {
    if (dgrad) dispatch_tile<2, true>(p, bm, bn, st);
    else dispatch_tile<2, false>(p, bm, bn, st);
  }
}

void splitk_reduce_launch(const float* slab, int S, int M, int Nout, const float* bias, float* y, float* part,
                          hipStream_t st, const RowRemap* rr, const float* addend) {
  dim3 grid((Nout + 63) / 64, (M + RB - 1) / RB);
  const RowRemap r = rr ? *rr : RowRemap{};
  if ((Nout & 3) == 0)
    hipLaunchKernelGGL(splitk_reduce4_kernel, grid, dim3(256), 0, st, slab, S, M, Nout, bias, y, part, r, addend);
  else hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, slab, S, M, Nout, bias, y, part, r, addend);
}

}  // namespace cdp
