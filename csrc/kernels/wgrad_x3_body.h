// fp32-accurate convolution weight gradient on the 16-bit matrix cores (gfx950): the kernel body
// shared by wgrad.hip (its own launches) and bwd_pair.hip (weight gradient beside the data
// gradient in one launch).
#pragma once
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "x3_common.h"

namespace cdp {
namespace x3wgrad {

constexpr int WBK = 32;

// ---------------------------------------------------------------------------------------------
// fp32-accurate weight gradient on the bf16 MFMA (v_mfma_f32_32x32x16_bf16): both operands are
// split into three bf16 terms and the six products of order >= 2^-16 are accumulated (see
// conv_x3.hip for the error analysis). The MFMA needs 8 consecutive reduction (m) indices per
// lane, so the tiles are transposed on their way into LDS: a thread gathers RPT consecutive m
// rows x 4 columns (float4 per row, coalesced along the channels), splits them and writes, per
// column and plane, its RPT m-values as one 8- or 4-byte LDS store into a [col][m] image (80-B
// row pitch). Lanes of a store group differ in m first, so the stores are conflict free; the
// fragment reads are the conflict-free ds_read_b128 pattern of conv_x3.hip.
constexpr int XLD = WBK + 8;  // bf16 per LDS row

// v[r] = row m+r of this thread's 4 columns; write, per column and plane, the RPT m-values
// (packed bf16 pairs) into the [col][m] image at dst. sc[c]: column c's f16x2 scale (NP == 2).
template <int RPT, int NP>
__device__ __forceinline__ void split_store_cols(const float4 (&v)[RPT], __bf16* dst, int plane, const float (&sc)[4]) {
  // (component access by constant index only: a pointer walk over `v` makes the compiler
  // promote the register array to LDS scratch)
  auto comp = [](const float4& q, int c) { return c == 0 ? q.x : c == 1 ? q.y : c == 2 ? q.z : q.w; };
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    unsigned h0[RPT / 2], h1[RPT / 2], h2[RPT / 2];
#pragma unroll
    for (int r = 0; r < RPT / 2; ++r) {
      if constexpr (NP == 1) h0[r] = pack_bf16x2(f32x2{comp(v[2 * r], c), comp(v[2 * r + 1], c)});
      else if constexpr (NP == 2) split_pair_h(comp(v[2 * r], c), comp(v[2 * r + 1], c), sc[c], h0[r], h1[r]);
      else split_pair(comp(v[2 * r], c), comp(v[2 * r + 1], c), h0[r], h1[r], h2[r]);
    }
    __bf16* d = dst + c * XLD;
    if constexpr (NP == 1) {
      if constexpr (RPT == 4) *reinterpret_cast<uint2*>(d) = make_uint2(h0[0], h0[1]);
      else *reinterpret_cast<unsigned*>(d) = h0[0];
    } else if constexpr (NP == 2) {
      if constexpr (RPT == 4) {
        *reinterpret_cast<uint2*>(d) = make_uint2(h0[0], h0[1]);
        *reinterpret_cast<uint2*>(d + plane) = make_uint2(h1[0], h1[1]);
      } else {
        *reinterpret_cast<unsigned*>(d) = h0[0];
        *reinterpret_cast<unsigned*>(d + plane) = h1[0];
      }
    } else if constexpr (RPT == 4) {
      *reinterpret_cast<uint2*>(d) = make_uint2(h0[0], h0[1]);
      *reinterpret_cast<uint2*>(d + plane) = make_uint2(h1[0], h1[1]);
      *reinterpret_cast<uint2*>(d + 2 * plane) = make_uint2(h2[0], h2[1]);
    } else {
      *reinterpret_cast<unsigned*>(d) = h0[0];
      *reinterpret_cast<unsigned*>(d + plane) = h1[0];
      *reinterpret_cast<unsigned*>(d + 2 * plane) = h2[0];
    }
  }
}

// NP = 3: split-bf16 (six products); 2: f16x2 (scaled operands, two fp16 terms, three products on
// v_mfma_f32_32x32x16_f16, see x3_common.h); 1: plain bf16 operands (non-parity mode)
// PIPE: two LDS stages and two register sets, one barrier per K-tile (tile t+1 is split into the
// other stage while the MFMAs consume tile t, tile t+2 in flight); else one stage, register
// prefetch of t+1 only, two barriers per K-tile.
// BM = 256 (f16x2 only): 512 threads = 4 (co) x 2 (k) waves of 64x64, one workgroup per CU.
template <int BM>
constexpr int wg_threads() { return BM >= 256 ? 512 : 256; }

// LDS of one workgroup (bf16 elements)
template <int BM, int BN, int NP, bool PIPE>
constexpr int wgrad_x3_smem_elems() { return (PIPE ? 2 : 1) * NP * (BM + BN) * XLD; }

// The kernel body as a device function (see conv_x3_body): `smem` holds wgrad_x3_smem_elems() bf16,
// `vbid` / `nvb` are this workgroup's id and the count of workgroups running this GEMM.
template <int BM, int BN, bool FAST, int NP = 3, bool PIPE = false>
__device__ __forceinline__ void wgrad_x3_body(const WgradParams& p, __bf16* __restrict__ smem, int vbid, int nvb) {
  constexpr int NT = wg_threads<BM>();
  constexpr int WMW = NT / 128;  // waves along co (x 2 along k)
  constexpr int TM = BM / WMW / 32, TN = BN / 64;
  constexpr int PA = BM * XLD, PB = BN * XLD;
  // m rows per thread, 4 columns (one float4) each: 4 for 128-wide / 256-wide tiles, 2 for 64
  constexpr int RPT_A = BM * WBK / (NT * 4), RPT_B = BN * WBK / (NT * 4);
  static_assert(RPT_B >= 2, "tile too narrow for the loader");
  constexpr int MQ_A = WBK / RPT_A, MQ_B = WBK / RPT_B;  // m groups per tile (8 or 16)
  constexpr int STAGE = NP * (PA + PB);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int ntn = (p.Kdim + BN - 1) / BN;
  const int ntm = (p.Cout + BM - 1) / BM;
  const int bid = xcd_remap(vbid, nvb);
  const int tile = bid % (ntm * ntn);
  const int split = bid / (ntm * ntn);
  const int tm_idx = tile / ntn, tn_idx = tile % ntn;
  const int co0 = tm_idx * BM, r0 = tn_idx * BN;
  const int mt_total = (p.M + WBK - 1) / WBK;
  const int kt_begin = (int)(((long long)split * mt_total) / p.splits);
  const int kt_end = (int)(((long long)(split + 1) * mt_total) / p.splits);
  const int PQ = p.P * p.Q;
  const int HWC = p.H * p.W * p.C;

  // A (dY^T): thread -> m group (fastest) and 4-column group
  const int a_mq = tid % MQ_A, a_cg = tid / MQ_A;
  const int co = co0 + a_cg * 4;
  // B (Xcol): same shape over the k columns
  const int b_mq = tid % MQ_B, b_cg = tid / MQ_B;
  const int kcol = r0 + b_cg * 4;
  int b_kh = 0, b_kw = 0, b_c = 0;
  const bool b_kok = kcol < p.Kdim;
  if (FAST && b_kok) {
    const int tap = fdiv(kcol, p.fd_C);
    b_c = kcol - tap * p.C;
    b_kh = fdiv(tap, p.fd_KW);
    b_kw = tap - b_kh * p.KW;
  }
  // FAST path buffers (host keeps both < 2 GiB): dY rows are addressed relative to the tile's
  // first row through a per-tile descriptor, so these offsets are loop invariant
  unsigned a_off[RPT_A];
#pragma unroll
  for (int i = 0; i < RPT_A; ++i)
    a_off[i] = co < p.Cout ? (unsigned)(mul24(a_mq * RPT_A + i, p.Cout) + co) * 4u : kOOB;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, (unsigned)p.N * (unsigned)HWC * 4u);
  // f16x2: one power-of-two scale per output row co (dY's channel co) and per output column
  // (tap, ci) (x's channel ci), from the producers' per-channel maxima (x3_common.h). Thread t
  // reduces the kActCopies copies of row t of the BM + BN rows and columns: loads issued here,
  // waited for after the first tiles' loads; the scales meet in LDS (stage 1 of the pipelined
  // kernel, or stage 0 behind a second barrier), and every thread keeps the 4 of its A columns
  // (sa4) and of its B columns (sb4).
  float sa4[4] = {1.f, 1.f, 1.f, 1.f}, sb4[4] = {1.f, 1.f, 1.f, 1.f};
  unsigned chm[NP == 2 ? kActCopies : 1];
  if constexpr (NP == 2) {
    static_assert(BM + BN <= NT, "one scale row per thread");
    const int j = tid;
    unsigned base = kOOB, stride = 0;
    const unsigned* src = p.dy_ch;
    unsigned nrow = (unsigned)p.Cout;
    if (j < BM) {
      if (co0 + j < p.Cout) base = (unsigned)(co0 + j) * 4u;
      stride = (unsigned)p.Cout * 4u;
    } else if (j < BM + BN) {
      const int k = r0 + j - BM;
      src = p.x_ch;
      nrow = (unsigned)p.C;
      if (k < p.Kdim) base = (unsigned)(k - fdiv(k, p.fd_C) * p.C) * 4u;
      stride = (unsigned)p.C * 4u;
    }
    const __amdgpu_buffer_rsrc_t cr = make_rsrc(src, (unsigned)kActCopies * nrow * 4u);
#pragma unroll
    for (int q = 0; q < kActCopies; ++q)
      chm[q] = __builtin_amdgcn_raw_buffer_load_b32(cr, (int)(base == kOOB ? kOOB : base + q * stride), 0, 0);
  }
  auto finish_scales = [&]() {
    if constexpr (NP == 2) {
      float* scr = reinterpret_cast<float*>(smem + (PIPE ? STAGE : 0));
      unsigned m = 0u;
#pragma unroll
      for (int q = 0; q < kActCopies; ++q) m = max(m, chm[q]);
      if (tid < BM + BN) scr[tid] = pow2_scale(__uint_as_float(m));
      lds_barrier();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sa4[c] = scr[a_cg * 4 + c];
        sb4[c] = scr[BM + b_cg * 4 + c];
      }
      if constexpr (!PIPE) lds_barrier();  // stage 0 is the first tile's destination
    }
  };

  float4 ra[RPT_A], rb[RPT_B], ra1[RPT_A], rb1[RPT_B];
  // valid == false (FAST only): zero-size / out-of-range buffers, so the loads return zeros without
  // touching memory and can be issued without a branch (see conv_x3.hip)
  auto load_tile = [&](int kt, float4 (&ra)[RPT_A], float4 (&rb)[RPT_B], bool valid = true) {
    const int mb = kt * WBK;
    if (FAST) {
      const __amdgpu_buffer_rsrc_t dr = make_rsrc(p.dy + (long long)(valid ? mb : 0) * p.Cout,
                                                  valid ? (unsigned)(p.M - mb) * (unsigned)p.Cout * 4u : 0u);
#pragma unroll
      for (int i = 0; i < RPT_A; ++i) ra[i] = bload4(dr, a_off[i]);
#pragma unroll
      for (int i = 0; i < RPT_B; ++i) {
        const int m = mb + b_mq * RPT_B + i;
        const int mm = m < p.M ? m : 0;
        const int n = fdiv(mm, p.fd_PQ);
        const int rem = mm - mul24(n, PQ);
        const int pp = fdiv(rem, p.fd_Q), qq = rem - mul24(pp, p.Q);
        const int ih = mul24(pp, p.stride) - p.pad + b_kh, iw = mul24(qq, p.stride) - p.pad + b_kw;
        const bool ok = valid && m < p.M && b_kok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        rb[i] = bload4(xr, ok ? (unsigned)(mul24(n, HWC) + mul24(mul24(ih, p.W) + iw, p.C) + b_c) * 4u : kOOB);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < RPT_A; ++i) {
      const int m = mb + a_mq * RPT_A + i;
      const bool mok = m < p.M;
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = (mok && co + j < p.Cout) ? p.dy[(long long)m * p.Cout + co + j] : 0.f;
      ra[i] = make_float4(e[0], e[1], e[2], e[3]);
    }
#pragma unroll
    for (int i = 0; i < RPT_B; ++i) {
      const int m = mb + b_mq * RPT_B + i;
      const bool mok = m < p.M;
      const int mm = mok ? m : 0;
      const int n = fdiv(mm, p.fd_PQ);
      const int rem = mm - n * PQ;
      const int pp = fdiv(rem, p.fd_Q), qq = rem - pp * p.Q;
      const int ih0 = pp * p.stride - p.pad, iw0 = qq * p.stride - p.pad;
      const float* xb = p.x + (long long)n * p.H * p.W * p.C;
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
  };
  auto store_tile = [&](const float4 (&ra)[RPT_A], const float4 (&rb)[RPT_B], __bf16* st) {
    split_store_cols<RPT_A, NP>(ra, st + (a_cg * 4) * XLD + a_mq * RPT_A, PA, sa4);
    split_store_cols<RPT_B, NP>(rb, st + NP * PA + (b_cg * 4) * XLD + b_mq * RPT_B, PB, sb4);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int l32 = lane & 31, hh = lane >> 5;
  const int koff = hh * 8;
  auto compute = [&](const __bf16* As) {
    const __bf16* Bs = As + NP * PA;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (NP == 2) {
          f16x8 af[TM][2], bf[TN][2];
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            const __bf16* src = As + (wm * (BM / WMW) + a * 32 + l32) * XLD + s * 16 + koff;
#pragma unroll
            for (int q = 0; q < 2; ++q) af[a][q] = *reinterpret_cast<const f16x8*>(src + q * PA);
          }
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const __bf16* src = Bs + (wn * (BN / 2) + b * 32 + l32) * XLD + s * 16 + koff;
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
          continue;
        }
        bf16x8 af[TM][3], bf[TN][3];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const __bf16* src = As + (wm * (BM / WMW) + a * 32 + l32) * XLD + s * 16 + koff;
#pragma unroll
          for (int q = 0; q < NP; ++q) af[a][q] = *reinterpret_cast<const bf16x8*>(src + q * PA);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const __bf16* src = Bs + (wn * (BN / 2) + b * 32 + l32) * XLD + s * 16 + koff;
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
  };
  if constexpr (PIPE) {
    if (kt_begin < kt_end) {
      static_assert(!PIPE || FAST, "the pipelined kernel issues branch-free FAST loads");
      load_tile(kt_begin, ra, rb);
      load_tile(kt_begin + 1, ra1, rb1, kt_begin + 1 < kt_end);
      finish_scales();
      store_tile(ra, rb, smem);
      __syncthreads();
      int kt = kt_begin;
      for (; kt + 1 < kt_end; kt += 2) {
        load_tile(kt + 2, ra, rb, kt + 2 < kt_end);
        compute(smem);
        store_tile(ra1, rb1, smem + STAGE);
        __syncthreads();
        load_tile(kt + 3, ra1, rb1, kt + 3 < kt_end);
        compute(smem + STAGE);
        store_tile(ra, rb, smem);  // past the last tile: stale registers into a stage nothing reads
        __syncthreads();
      }
      if (kt < kt_end) compute(smem);
    } else {
      finish_scales();
    }
  } else if (kt_begin < kt_end) {
    load_tile(kt_begin, ra, rb);
    finish_scales();
    store_tile(ra, rb, smem);
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const bool more = kt + 1 < kt_end;
      if (more) load_tile(kt + 1, ra, rb);
      compute(smem);
      __syncthreads();
      if (more) {
        store_tile(ra, rb, smem);
        __syncthreads();
      }
    }
  } else {
    finish_scales();
  }

  if constexpr (NP == 2) {
    // undo the row / column scales (exact: powers of two): the reciprocals meet in LDS (free now),
    // written by the threads of the first m group of every A / B column group
    float* s_ia = reinterpret_cast<float*>(smem);
    float* s_ib = s_ia + BM;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (a_mq == 0) s_ia[a_cg * 4 + c] = 1.f / sa4[c];
      if (b_mq == 0) s_ib[b_cg * 4 + c] = 1.f / sb4[c];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const float ib = s_ib[wn * (BN / 2) + b * 32 + l32];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[a][b][r] = acc[a][b][r] * s_ia[wm * (BM / WMW) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh] * ib;
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
          const int c = co0 + wm * (BM / WMW) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (!decltype(pred)::value || (c < p.Cout && k < p.Kdim)) out[(long long)c * p.Kdim + k] = acc[a][b][r];
        }
      }
  };
  if (full) store(std::false_type{});
  else store(std::true_type{});
}

}  // namespace x3wgrad
}  // namespace cdp
