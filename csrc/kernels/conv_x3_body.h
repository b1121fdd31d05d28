// Implicit-GEMM convolution at fp32 accuracy on the 16-bit matrix cores (gfx950): the kernel body
// shared by conv_x3.hip (its own launches) and bwd_pair.hip (data gradient beside the weight
// gradient in one launch). See conv_x3.hip for the numerics and the pipeline.
#pragma once
#include <type_traits>

#include "common.h"
#include "conv_epilogue.h"
#include "kernels.h"
#include "x3_common.h"

namespace cdp {
namespace x3conv {

constexpr int BK = 32;
constexpr int LDH = BK;  // bf16 per LDS row (64 B, 16-B chunks XOR-swizzled, see chunk_pos)

// 16-B chunk c (0..3) of LDS row r lives at chunk position c ^ f((r >> 2) & 3), f(q) = -q mod 4:
// the 8-lane groups of the ds_write_b128 stores (two rows x four chunks) and the 16-lane groups
// of the ds_read_b128 fragment reads hit distinct banks, both for the 32x32x16 operand (16 rows,
// one chunk) and for the 16x16x32 operand (8 rows x 2 chunks).
__device__ __forceinline__ int chunk_pos(int r, int c) { return c ^ ((-(r >> 2)) & 3); }

// Split 8 consecutive-k fp32 values into three bf16x8 planes (as 4 packed pairs each).
__device__ __forceinline__ void split8(const float (&v)[8], u32x4& s0, u32x4& s1, u32x4& s2) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned a, b, c;
    split_pair(v[2 * j], v[2 * j + 1], a, b, c);
    s0[j] = a;
    s1[j] = b;
    s2[j] = c;
  }
}

// Split 8 consecutive-k fp32 values of an operand scaled by s into two fp16x8 planes (f16x2).
__device__ __forceinline__ void split8h(const float (&v)[8], float s, u32x4& s0, u32x4& s1) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned a, b;
    split_pair_h(v[2 * j], v[2 * j + 1], s, a, b);
    s0[j] = a;
    s1[j] = b;
  }
}

// NP = 16-bit planes per operand: 3 = fp32-accurate bf16 split (six products), 2 = f16x2
// (power-of-two-scaled operands as two fp16 terms, three products on v_mfma_f32_32x32x16_f16, see
// x3_common.h), 1 = plain bf16 operands with fp32 accumulation (one product; the non-parity fast
// mode, CDP_CONV_GEMM=bf16).
// 8 consecutive-k fp32 values rounded to bf16 (one plane)
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = pack_bf16x2(f32x2{v[2 * j], v[2 * j + 1]});
  return r;
}

// LDS of one workgroup (bf16 elements): two stages of NP planes of A and B, at least the epilogue's
// scratch (conv_epilogue.h; only the one-plane 64 x 64 tile needs more than its stages), then
// (f16x2) the reciprocal row scales of both operands, BM + BN floats that alias nothing
template <int BM, int BN, int NP>
constexpr int conv_x3_scales_at() {
  return 2 * NP * (BM + BN) * LDH > 2 * epi_lds_floats<BM, BN>() ? 2 * NP * (BM + BN) * LDH
                                                                  : 2 * epi_lds_floats<BM, BN>();
}
template <int BM, int BN, int NP>
constexpr int conv_x3_smem_elems() {
  return conv_x3_scales_at<BM, BN, NP>() + (NP == 2 ? 2 * (BM + BN) : 0);
}

// The kernel body as a device function: `smem` holds conv_x3_smem_elems() bf16 (the caller's one
// LDS array), `vbid` / `nvb` are this workgroup's id and the count of workgroups running this
// GEMM (a launch may carry other work beside it: bwd_pair.hip).
template <int BM, int BN, int MODE, bool DGRAD, int NP = 3>
__device__ __forceinline__ void conv_x3_body(const ConvGemmParams& p, __bf16* __restrict__ smem, int vbid, int nvb) {
  static_assert(NP >= 1 && NP <= 3, "planes");
  constexpr unsigned ES = 2u;  // log2 bytes per element of the (fp32) global operands
  constexpr int WM = waves_m<BM>();  // waves along M (2 x WM waves)
  constexpr int NT = WM * 128;       // threads
  constexpr int RS = NT / 4;         // rows covered by one pass of the loaders
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / 64;
  constexpr int A_LD = BM / RS;  // A rows per thread (row = tid/4 + RS i), 8 consecutive k each
  constexpr int B_LD = BN / RS;
  static_assert(A_LD >= 1 && B_LD >= 1, "tile too narrow for the loader");
  constexpr int PA = BM * LDH, PB = BN * LDH;
  constexpr int STAGE = NP * (PA + PB);  // bf16 per stage: A planes [NP][BM][LDH], B planes [NP][BN][LDH]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int ntn = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(vbid, nvb);
  const int tn_idx = bid % ntn;
  const int rest = bid / ntn;
  const int split = rest % p.splits;
  const int tm_idx = rest / p.splits;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int kt_begin = (int)(((long long)split * p.ktiles) / p.splits);
  const int kt_end = (int)(((long long)(split + 1) * p.ktiles) / p.splits);
  const int PQ = p.P * p.Q;
  const int HWC = p.H * p.W * p.C;

  const int kq = (tid & 3) * 8;  // this thread's 8 consecutive k within the tile
  const int rrow = tid >> 2;     // + RS i

  // buffers (host guarantees < 2 GiB each): out-of-range offsets read as zero
  const unsigned xplane = ((unsigned)p.N * (unsigned)HWC) << ES;
  const unsigned wplane = ((unsigned)p.Nout * (unsigned)p.Kdim) << ES;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, xplane);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, wplane);

  // per A row: spatial anchor and element offset of (n, anchor, kq)
  int a_h[A_LD], a_w[A_LD], a_n[A_LD], a_off[A_LD];
  unsigned a_io[A_LD];  // f16x2: byte offset of the row's image slot (p.a_img), kOOB past M
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + rrow + RS * i;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    const int n = fdiv(mm, p.fd_PQ);
    a_io[i] = ok ? (unsigned)n * 4u : kOOB;
    const int rem = mm - mul24(n, PQ);
    const int pp = fdiv(rem, p.fd_Q);
    const int qq = rem - mul24(pp, p.Q);
    if (DGRAD) {
      a_h[i] = pp + p.pad;  // oh*stride = ih + pad - kh
      a_w[i] = qq + p.pad_w;  // column pad (differs from pad in sub-pixel class launches)
    } else {
      a_h[i] = mul24(pp, p.stride) - p.pad;
      a_w[i] = mul24(qq, p.stride) - p.pad;
    }
    if (!ok) a_h[i] = -(1 << 22);  // fails every bounds test below
    a_n[i] = mul24(n, HWC);
    a_off[i] = a_n[i] + mul24(mul24(a_h[i], p.W) + a_w[i], p.C) + kq;
  }
  // per B row: byte offset of (row, kq); rows past Nout read zeros
  unsigned b_off[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int n = n0 + rrow + RS * i;
    b_off[i] = n < p.Nout ? (unsigned)(mul24(n, p.Kdim) + kq) << ES : kOOB;
  }

  // f16x2: one power-of-two scale per GEMM row of each operand (x3_common.h) -- A rows by their
  // image (p.a_img), B rows from the weight's per-row partials (p.b_row; the four threads that load
  // a B row split its partials and meet by two shuffles). The loads go out here and are waited for
  // after the first tiles' loads are issued.
  constexpr int BQ = 4;  // B-row partials per thread in the first batch (16 per row)
  float sa_r[NP == 2 ? A_LD : 1], sb_r[NP == 2 ? B_LD : 1];
  unsigned am_a[NP == 2 ? A_LD : 1];
  float am_b[NP == 2 ? B_LD : 1][BQ];
  const __amdgpu_buffer_rsrc_t brow = make_rsrc(p.b_row, (unsigned)p.b_np * (unsigned)p.b_stride * 4u);
  if constexpr (NP == 2) {
    const __amdgpu_buffer_rsrc_t ir = make_rsrc(p.a_img, (unsigned)p.N * 4u);
#pragma unroll
    for (int i = 0; i < A_LD; ++i) am_a[i] = __builtin_amdgcn_raw_buffer_load_b32(ir, (int)a_io[i], 0, 0);
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int n = n0 + rrow + RS * i;
#pragma unroll
      for (int j = 0; j < BQ; ++j) {
        const int q = (tid & 3) + 4 * j;
        const unsigned o = (n < p.Nout && q < p.b_np) ? (unsigned)(q * p.b_stride + n) * 4u : kOOB;
        am_b[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brow, (int)o, 0, 0));
      }
    }
  }
  auto finish_scales = [&]() {
    if constexpr (NP == 2) {
#pragma unroll
      for (int i = 0; i < A_LD; ++i) sa_r[i] = pow2_scale(__uint_as_float(am_a[i]));
#pragma unroll
      for (int i = 0; i < B_LD; ++i) {
        const int n = n0 + rrow + RS * i;
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < BQ; ++j) m = fmaxf(m, am_b[i][j]);
        for (int q = (tid & 3) + 4 * BQ; q < p.b_np; q += 4) {  // wide weights (Ci or Co > 512)
          const unsigned o = n < p.Nout ? (unsigned)(q * p.b_stride + n) * 4u : kOOB;
          m = fmaxf(m, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brow, (int)o, 0, 0)));
        }
        m = fmaxf(m, __shfl_xor(m, 1, kWave));
        m = fmaxf(m, __shfl_xor(m, 2, kWave));
        sb_r[i] = pow2_scale(m);
      }
    }
  };

  // byte offset of A row i at filter tap (kh, kw), channel offset c (relative to kq); OOB if padded
  auto a_voff = [&](int i, int kh, int kw, int c) -> unsigned {
    if (DGRAD) {
      int oh = a_h[i] - kh, ow = a_w[i] - kw;
      if (p.stride == 1) {
        const bool ok = (unsigned)oh < (unsigned)p.H && (unsigned)ow < (unsigned)p.W;
        return ok ? (unsigned)(a_off[i] - mul24(mul24(kh, p.W) + kw, p.C) + c) << ES : kOOB;
      }
      bool ok = oh >= 0 && ow >= 0 && ((oh | ow) & (p.stride - 1)) == 0;  // stride is 2 (power of two)
      oh >>= 1;
      ow >>= 1;
      ok = ok && oh < p.H && ow < p.W;
      return ok ? (unsigned)(a_n[i] + mul24(mul24(oh, p.W) + ow, p.C) + kq + c) << ES : kOOB;
    } else {
      const int ih = a_h[i] + kh, iw = a_w[i] + kw;
      const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      return ok ? (unsigned)(a_off[i] + mul24(mul24(kh, p.W) + kw, p.C) + c) << ES : kOOB;
    }
  };

  // register ping-pong: fp32 tiles (8 k per row)
  float va0[A_LD][8], va1[A_LD][8];
  float vb0[B_LD][8], vb1[B_LD][8];

  auto put4 = [](float (&d)[8], int off, float4 v) {
    d[off] = v.x;
    d[off + 1] = v.y;
    d[off + 2] = v.z;
    d[off + 3] = v.w;
  };

  // valid == false: every offset is past the buffers, so the loads return zeros without touching
  // memory. Issuing them unconditionally (no branch around the prefetch) lets the compiler wait
  // with vmcnt(#newer loads) for the older tile instead of vmcnt(0) at a control-flow merge,
  // which would have drained the prefetch of the next tile.
  auto load_tile = [&](int kt, auto& va, auto& vb, bool valid) {
    const int r0 = kt * BK;
    if (MODE == 0) {
      // the whole K-tile lies in one filter tap (C % 32 == 0): tap decode is wave-uniform
      const int tap = fdiv(r0, p.fd_C);
      const int c0 = r0 - tap * p.C;
      const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const unsigned o = valid ? a_voff(i, kh, kw, c0) : kOOB;
        put4(va[i], 0, bload4(xr, o));
        put4(va[i], 4, bload4(xr, o + 16u));
      }
    } else if (MODE == 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = r0 + kq + 4 * h;
        const bool rok = valid && r < p.Kdim;
        const int tap = fdiv(rok ? r : 0, p.fd_C);
        const int c = r - tap * p.C;
        const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
          const unsigned o = rok ? a_voff(i, kh, kw, c - kq) : kOOB;
          put4(va[i], 4 * h, bload4(xr, o));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = r0 + kq + j;
        const bool rok = valid && r < p.Kdim;
        const int tap = fdiv(rok ? r : 0, p.fd_C);
        const int c = r - tap * p.C;
        const int kh = fdiv(tap, p.fd_KW), kw = tap - kh * p.KW;
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
          const unsigned o = rok ? a_voff(i, kh, kw, c - kq) : kOOB;
          va[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, (int)o, 0, 0));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const unsigned o = valid ? b_off[i] + ((unsigned)r0 << ES) : kOOB;
      if (MODE == 0) {
        put4(vb[i], 0, bload4(wr, o));
        put4(vb[i], 4, bload4(wr, o + 16u));
      } else if (MODE == 1) {
        // Kdim % 4 == 0: a float4 is either inside the row or wholly past its end
        put4(vb[i], 0, bload4(wr, r0 + kq < p.Kdim ? o : kOOB));
        put4(vb[i], 4, bload4(wr, r0 + kq + 4 < p.Kdim ? o + 16u : kOOB));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          vb[i][j] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(wr, (int)(r0 + kq + j < p.Kdim ? o + 4u * j : kOOB), 0, 0));
      }
    }
  };

  auto store_tile = [&](const auto& va, const auto& vb, __bf16* st) {
    const int cp = chunk_pos(rrow, tid & 3) * 8;  // rrow + RS i has the same (row >> 2) & 3
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      __bf16* d = st + (rrow + RS * i) * LDH + cp;
      if constexpr (NP == 1) {
        *reinterpret_cast<u32x4*>(d) = pack8(va[i]);
      } else if constexpr (NP == 2) {
        u32x4 s0, s1;
        split8h(va[i], sa_r[i], s0, s1);
        *reinterpret_cast<u32x4*>(d) = s0;
        *reinterpret_cast<u32x4*>(d + PA) = s1;
      } else {
        u32x4 s0, s1, s2;
        split8(va[i], s0, s1, s2);
        *reinterpret_cast<u32x4*>(d) = s0;
        *reinterpret_cast<u32x4*>(d + PA) = s1;
        *reinterpret_cast<u32x4*>(d + 2 * PA) = s2;
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      __bf16* d = st + NP * PA + (rrow + RS * i) * LDH + cp;
      if constexpr (NP == 1) {
        *reinterpret_cast<u32x4*>(d) = pack8(vb[i]);
      } else if constexpr (NP == 2) {
        u32x4 s0, s1;
        split8h(vb[i], sb_r[i], s0, s1);
        *reinterpret_cast<u32x4*>(d) = s0;
        *reinterpret_cast<u32x4*>(d + PB) = s1;
      } else {
        u32x4 s0, s1, s2;
        split8(vb[i], s0, s1, s2);
        *reinterpret_cast<u32x4*>(d) = s0;
        *reinterpret_cast<u32x4*>(d + PB) = s1;
        *reinterpret_cast<u32x4*>(d + 2 * PB) = s2;
      }
    }
  };

  // accumulators: 32x32x16 tiles (TM x TN)
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int l32 = lane & 31;
  const int hh = lane >> 5;

  // MFMAs over one LDS stage: the split products per output tile and 32-deep K-tile, as two
  // 32x32x16 steps
  auto compute = [&](const __bf16* st) {
    if constexpr (NP == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 af[TM][2], bf[TN][2];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int r = wm * (BM / WM) + a * 32 + l32;
          const __bf16* src = st + r * LDH + chunk_pos(r, 2 * s + hh) * 8;
#pragma unroll
          for (int q = 0; q < 2; ++q) af[a][q] = *reinterpret_cast<const f16x8*>(src + q * PA);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int r = wn * (BN / 2) + b * 32 + l32;
          const __bf16* src = st + NP * PA + r * LDH + chunk_pos(r, 2 * s + hh) * 8;
#pragma unroll
          for (int q = 0; q < 2; ++q) bf[b][q] = *reinterpret_cast<const f16x8*>(src + q * PB);
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            f32x16 c = acc[a][b];
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][1], bf[b][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][0], bf[b][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][0], bf[b][0], c, 0, 0, 0);
            acc[a][b] = c;
          }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[TM][3], bf[TN][3];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int r = wm * (BM / WM) + a * 32 + l32;
          const __bf16* src = st + r * LDH + chunk_pos(r, 2 * s + hh) * 8;
#pragma unroll
          for (int q = 0; q < NP; ++q) af[a][q] = *reinterpret_cast<const bf16x8*>(src + q * PA);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int r = wn * (BN / 2) + b * 32 + l32;
          const __bf16* src = st + NP * PA + r * LDH + chunk_pos(r, 2 * s + hh) * 8;
#pragma unroll
          for (int q = 0; q < NP; ++q) bf[b][q] = *reinterpret_cast<const bf16x8*>(src + q * PB);
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            f32x16 c = acc[a][b];
            if constexpr (NP == 1) {
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bf[b][0], c, 0, 0, 0);
              continue;
            }
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][2], bf[b][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][1], bf[b][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bf[b][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][1], bf[b][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bf[b][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][0], bf[b][0], c, 0, 0, 0);
            acc[a][b] = c;
          }
      }
    }
  };

  // Software pipeline, one barrier per K-tile: while the MFMAs consume stage t&1, tile t+1
  // (loaded into registers one iteration earlier) is split into stage (t+1)&1 and tile t+2 is
  // being fetched into the other register set.
  // f16x2: each row's reciprocal scale goes to its own LDS slot now, so the epilogue reads them
  // without a barrier of its own (the main loop's first barrier publishes them; a tile-less
  // split slice has one below). The threads with kq == 0 hold the scales of their loader rows.
  float* s_ia = reinterpret_cast<float*>(smem + conv_x3_scales_at<BM, BN, NP>());
  float* s_ib = s_ia + BM;
  auto publish_scales = [&]() {
    if constexpr (NP == 2) {
      if ((tid & 3) == 0) {
#pragma unroll
        for (int i = 0; i < A_LD; ++i) s_ia[rrow + RS * i] = 1.f / sa_r[i];
#pragma unroll
        for (int i = 0; i < B_LD; ++i) s_ib[rrow + RS * i] = 1.f / sb_r[i];
      }
    }
  };
  if (kt_begin < kt_end) {
    load_tile(kt_begin, va0, vb0, true);
    load_tile(kt_begin + 1, va1, vb1, kt_begin + 1 < kt_end);
    finish_scales();
    publish_scales();
    store_tile(va0, vb0, smem);
    __syncthreads();
    int kt = kt_begin;
    for (; kt + 1 < kt_end; kt += 2) {
      load_tile(kt + 2, va0, vb0, kt + 2 < kt_end);
      compute(smem);
      store_tile(va1, vb1, smem + STAGE);
      __syncthreads();
      load_tile(kt + 3, va1, vb1, kt + 3 < kt_end);
      compute(smem + STAGE);
      // unconditional (past the last tile it stores stale registers into a stage nothing reads),
      // so the split can interleave with the MFMAs above
      store_tile(va0, vb0, smem);
      __syncthreads();
    }
    if (kt < kt_end) compute(smem);  // odd tile count: the last tile sits in stage 0
  } else {  // no K-tiles: the (zero) accumulators still get unscaled
    finish_scales();
    publish_scales();
    __syncthreads();
  }

  if constexpr (NP == 2) {
    // undo the row scales (exact: powers of two); a lane's accumulators span 16 x TM rows and TN
    // columns, their reciprocals published before the main loop's first barrier
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const float ib = s_ib[wn * (BN / 2) + b * 32 + l32];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[a][b][r] = acc[a][b][r] * s_ia[wm * (BM / WM) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh] * ib;
    }
  }
  conv_epilogue<BM, BN>(p, acc, reinterpret_cast<float*>(smem), m0, n0, tm_idx, split);
}

}  // namespace x3conv
}  // namespace cdp
