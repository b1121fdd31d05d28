// Shared epilogue of the implicit-GEMM conv kernels (fp32-MFMA and split-bf16 variants).
//
// The accumulator tile layout is the same for v_mfma_f32_32x32x2_f32 and
// v_mfma_f32_32x32x16_bf16 (C/D map is dtype-independent on gfx950): lane l holds column
// l&31 and rows (r&3) + 8*(r>>2) + 4*(l>>5) of each 32x32 tile.
//
// splits > 1: store the raw partial tile into its split-K slab.
// splits == 1: add bias, store, and (when p.part) emit per-block BatchNorm partials
// (mean_b, M2_b per column, two exact passes over the registers) so the following
// BatchNorm never re-reads the conv output for its statistics.
#pragma once
#include <cstdint>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace cdp {

// Wave grid: WM x 2 waves (WM = 4 for BM = 256, else 2), each owning (BM/WM) x (BN/2).
template <int BM>
constexpr int waves_m() { return BM >= 256 ? 4 : 2; }

// Wide stores: the accumulator layout gives a lane one column, so a plain epilogue writes a 32 x 32
// sub-tile with 16 four-byte store instructions per lane. For the small-K GEMMs (ResNet's 1x1
// convolutions, K = 64..256) that store stream, not HBM, bounds the kernel (200704 x 256 x 64: 2.2
// TB/s written, a fill of the same bytes 6.8). A full tile instead goes through LDS one 32 x 32
// sub-tile per wave and leaves as 16-B row segments: 4 store instructions. Staging area per wave
// (row stride kStageLd floats: the two half-waves' rows of one ds_write land 32 banks apart), past
// the statistics scratch (2 x WM x BN floats) and the f16x2 row-scale arrays (BM + BN floats).
constexpr int kStageLd = 40;
template <int BM, int BN>
constexpr int epi_stage_base() { return (2 * waves_m<BM>() * BN + BM + BN + 3) & ~3; }
template <int BM, int BN>
constexpr int epi_lds_floats() { return epi_stage_base<BM, BN>() + waves_m<BM>() * 2 * 32 * kStageLd; }

// Store the wave's accumulators (full tile) to dst[rowmap(m) * ld + n] with 16-B stores.
template <int BM, int BN, class RowMap>
__device__ __forceinline__ void wide_store(const f32x16 (&acc)[BM / waves_m<BM>() / 32][BN / 64], float* red,
                                           float* __restrict__ dst, long long ld, int m0, int n0, RowMap rowmap) {
  constexpr int WM = waves_m<BM>();
  constexpr int TM = BM / WM / 32, TN = BN / 64;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int l32 = lane & 31;
  const int hh = lane >> 5;
  float* st = red + epi_stage_base<BM, BN>() + wid * 32 * kStageLd;
  const int rq = lane >> 3, cq = (lane & 7) * 4;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[((r & 3) + 8 * (r >> 2) + 4 * hh) * kStageLd + l32] = acc[a][b][r];
      // one wave's private area: LDS runs a wave's operations in order, the wait keeps the
      // compiler from moving the reads above the writes
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int mb = m0 + wm * (BM / WM) + a * 32;
      const int n = n0 + wn * (BN / 2) + b * 32 + cq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rq + 8 * i;
        const float4 v = *reinterpret_cast<const float4*>(st + row * kStageLd + cq);
        *reinterpret_cast<float4*>(dst + rowmap(mb + row) * ld + n) = v;
      }
      asm volatile("" ::: "memory");  // the next sub-tile's writes stay behind these reads
    }
}

template <int BM, int BN>
__device__ __forceinline__ void conv_tile_stats(const ConvGemmParams& p,
                                                const f32x16 (&acc)[BM / waves_m<BM>() / 32][BN / 64], float* red,
                                                int m0, int n0, int tm_idx);

template <int BM, int BN>
__device__ __forceinline__ void conv_epilogue(const ConvGemmParams& p,
                                              f32x16 (&acc)[BM / waves_m<BM>() / 32][BN / 64], float* red, int m0,
                                              int n0, int tm_idx, int split) {
  constexpr int WM = waves_m<BM>();
  constexpr int TM = BM / WM / 32, TN = BN / 64;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int l32 = lane & 31;
  const int hh = lane >> 5;
  // whole tile in bounds (the common case): unpredicated stores, no per-element exec branches
  const bool full = m0 + BM <= p.M && n0 + BN <= p.Nout;
  const bool wide = !p.narrow && (p.Nout & 3) == 0 && ((reinterpret_cast<uintptr_t>(p.y) & 15) == 0);
  if (p.splits > 1) {
    float* out = p.y + (long long)split * p.M * p.Nout;
    auto slab_store = [&](auto pred) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int n = n0 + wn * (BN / 2) + b * 32 + l32;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * (BM / WM) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (!decltype(pred)::value || (m < p.M && n < p.Nout)) out[(long long)m * p.Nout + n] = acc[a][b][r];
          }
        }
    };
    if (full && wide) {
      __syncthreads();  // the staging area aliases the operand LDS the last K-tile may still read
      wide_store<BM, BN>(acc, red, out, p.Nout, m0, n0, [](int m) { return (long long)m; });
    } else if (full) {
      slab_store(std::false_type{});
    } else {
      slab_store(std::true_type{});
    }
    return;
  }

  // (measured and rejected: the addend loaded as 16-B rows through LDS, like the stores -- ResNet-50
  // 14.87 -> 15.35 ms, the extra barrier and 64 more VGPRs in the data-gradient kernels)
  if (p.addend) {  // y += addend (may alias y): every load is issued before any store
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wn * (BN / 2) + b * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * (BM / WM) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          // branch-free (clamped address + select) so all loads issue before the first wait
          const bool ok = m < p.M && n < p.Nout;
          const float av = p.addend[ok ? remap_row(p.rr, m) * p.Nout + n : 0];
          acc[a][b][r] += ok ? av : 0.f;
        }
      }
  }
  float bias_v[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int n = n0 + wn * (BN / 2) + b * 32 + l32;
    bias_v[b] = (p.bias && n < p.Nout) ? p.bias[n] : 0.f;
  }
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] += bias_v[b];
  // the output stores go last: a barrier behind them (the statistics' ones) would make every wave
  // wait for its stores to reach memory first
  auto out_store = [&](auto pred) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wn * (BN / 2) + b * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * (BM / WM) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (!decltype(pred)::value || (m < p.M && n < p.Nout)) p.y[remap_row(p.rr, m) * p.Nout + n] = acc[a][b][r];
        }
      }
  };
  if (p.part) conv_tile_stats<BM, BN>(p, acc, red, m0, n0, tm_idx);  // ends past a barrier
  else if (full && wide) __syncthreads();  // the staging area aliases the operand LDS
  if (full && wide) wide_store<BM, BN>(acc, red, p.y, p.Nout, m0, n0, [&](int m) { return remap_row(p.rr, m); });
  else if (full) out_store(std::false_type{});
  else out_store(std::true_type{});
}

// BN partials (mean, M2) of the tile's columns over its valid rows -> p.part[tm_idx]. Each wave
// reduces its own rows exactly (two passes over its registers: sum, then squares about the wave's
// mean), the WM waves of a column meet once in LDS, and the first wave row merges their
// (count, mean, M2) triples with Chan's formula -- one barrier after the aliasing one. Replaced a
// block-wide two-pass version with four barriers: same-box hipGraph step, VGG-11 at 256 images
// 1.351-1.355 -> 1.304-1.306 ms (four interleaved pairs), 32 images 0.5143-0.5155 -> 0.5103-0.5120,
// ResNet-50 unchanged; the first step's loss agrees to 1.4e-6.
template <int BM, int BN>
__device__ __forceinline__ void conv_tile_stats(const ConvGemmParams& p,
                                                const f32x16 (&acc)[BM / waves_m<BM>() / 32][BN / 64], float* red,
                                                int m0, int n0, int tm_idx) {
  constexpr int WM = waves_m<BM>();
  constexpr int TM = BM / WM / 32, TN = BN / 64;
  constexpr int WR = BM / WM;  // rows per wave
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int l32 = lane & 31;
  const int hh = lane >> 5;
  __syncthreads();  // `red` aliases the operand LDS
  const int wrow0 = m0 + wm * WR;
  const int nw = max(0, min(WR, p.M - wrow0));  // this wave's valid rows
  const float inv_nw = nw > 0 ? 1.f / (float)nw : 0.f;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wrow0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        s += (m < p.M) ? acc[a][b][r] : 0.f;
      }
    s += __shfl_xor(s, 32, kWave);
    const float mean_w = s * inv_nw;
    float q = 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wrow0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float d = acc[a][b][r] - mean_w;
        q += (m < p.M) ? d * d : 0.f;
      }
    q += __shfl_xor(q, 32, kWave);
    if (hh == 0) {
      const int c = wn * (BN / 2) + b * 32 + l32;
      red[(wm * BN + c) * 2] = mean_w;
      red[(wm * BN + c) * 2 + 1] = q;
    }
  }
  __syncthreads();
  if (wm == 0 && hh == 0) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int c = wn * (BN / 2) + b * 32 + l32;
      const int n = n0 + c;
      if (n < p.Nout) {
        float cnt = (float)min(WR, p.M - m0), mean = red[c * 2], m2 = red[c * 2 + 1];
#pragma unroll
        for (int w = 1; w < WM; ++w) {
          const float nb = (float)max(0, min(WR, p.M - (m0 + w * WR)));
          if (nb > 0.f) {
            const float mb = red[(w * BN + c) * 2], qb = red[(w * BN + c) * 2 + 1];
            const float tot = cnt + nb, delta = mb - mean;
            mean = fmaf(delta, nb / tot, mean);
            m2 += qb + delta * delta * (cnt * nb / tot);
            cnt = tot;
          }
        }
        float* dst = p.part + ((long long)tm_idx * p.Nout + n) * 2;
        dst[0] = mean;
        dst[1] = m2;
      }
    }
  }
}

}  // namespace cdp
