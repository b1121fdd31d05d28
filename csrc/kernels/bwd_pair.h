// A conv block's two gradient GEMMs in ONE launch (gfx950): the data gradient dX = dY * W^T
// (conv_x3_body, transposed gather) and the weight gradient dW = dY^T * Xcol (wgrad_x3_body) both
// read dY and are independent, so the workgroups of one launch are split between them: blocks
// [0, nd) run the data-gradient tiles, [nd, nd + nw) the weight-gradient tiles.
//
// Why one launch: at the reference's strong-scaling batches (32-64 images per GPU,
// /root/reference/src/Part 2a/main.py:22) each of the two grids of a deep VGG layer is a few dozen
// to a few hundred workgroups on a 256-CU chip; run back to back they leave CUs idle twice, side by
// side they fill the chip once and save a dependent dispatch (VGG-11, 32 images per GPU: 0.70 ->
// 0.64 ms per step; 256 images: 1.41 -> 1.40 ms). Two streams were measured 2x slower: under hipGraph
// every fork/join costs more than the overlap returns (docs/PERF.md). Both bodies are f16x2 tiles
// with the same workgroup size (512 threads for the 256x128 pair, 256 for the others); the LDS array
// is the larger of the two images.
#pragma once
#include "conv_x3_body.h"
#include "wgrad_x3_body.h"

namespace cdp {
namespace pair_detail {

using namespace x3conv;
using namespace x3wgrad;

template <int DBM, int DBN, int WBM, int WBN>
struct PairCfg {
  static constexpr int kThreads = waves_m<DBM>() * 128;
  static_assert(kThreads == wg_threads<WBM>(), "both bodies must run the same workgroup size");
  static constexpr int kSmem = conv_x3_smem_elems<DBM, DBN, 2>() > wgrad_x3_smem_elems<WBM, WBN, 2, true>()
                                   ? conv_x3_smem_elems<DBM, DBN, 2>()
                                   : wgrad_x3_smem_elems<WBM, WBN, 2, true>();
};

template <int DBM, int DBN, int WBM, int WBN>
__global__ __launch_bounds__(waves_m<DBM>() * 128, DBM >= 256 ? 1 : 2) void bwd_pair_kernel(
    ConvGemmParams pd, WgradParams pw, int nd, int nw) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[PairCfg<DBM, DBN, WBM, WBN>::kSmem];
  const int b = blockIdx.x;
  if (b < nd) conv_x3_body<DBM, DBN, 0, true, 2>(pd, smem, b, nd);
  else wgrad_x3_body<WBM, WBN, true, 2, true>(pw, smem, b - nd, nw);
}

template <int DBM, int DBN, int WBM, int WBN>
void launch_pair(const ConvGemmParams& pd, const WgradParams& pw, hipStream_t st) {
  const int nd = ((pd.M + DBM - 1) / DBM) * ((pd.Nout + DBN - 1) / DBN) * pd.splits;
  const int nw = ((pw.Cout + WBM - 1) / WBM) * ((pw.Kdim + WBN - 1) / WBN) * pw.splits;
  hipLaunchKernelGGL((bwd_pair_kernel<DBM, DBN, WBM, WBN>), dim3(nd + nw), dim3(PairCfg<DBM, DBN, WBM, WBN>::kThreads),
                     0, st, pd, pw, nd, nw);
}

// one translation unit per data-gradient tile (parallel builds): the four weight-gradient tiles of
// a 256-thread pair
template <int DBM, int DBN>
bool launch_pair_d(int wbm, int wbn, const ConvGemmParams& pd, const WgradParams& pw, hipStream_t st);
template <>
bool launch_pair_d<128, 128>(int, int, const ConvGemmParams&, const WgradParams&, hipStream_t);
template <>
bool launch_pair_d<128, 64>(int, int, const ConvGemmParams&, const WgradParams&, hipStream_t);
template <>
bool launch_pair_d<64, 128>(int, int, const ConvGemmParams&, const WgradParams&, hipStream_t);
template <>
bool launch_pair_d<64, 64>(int, int, const ConvGemmParams&, const WgradParams&, hipStream_t);

}  // namespace pair_detail
}  // namespace cdp

#define CDP_PAIR_TU(DBM, DBN)                                                                              \
  namespace cdp {                                                                                          \
  namespace pair_detail {                                                                                  \
  template <>                                                                                              \
  bool launch_pair_d<DBM, DBN>(int wbm, int wbn, const ConvGemmParams& pd, const WgradParams& pw,          \
                               hipStream_t st) {                                                           \
    if (wbm == 128 && wbn == 128) launch_pair<DBM, DBN, 128, 128>(pd, pw, st);                             \
    else if (wbm == 128 && wbn == 64) launch_pair<DBM, DBN, 128, 64>(pd, pw, st);                          \
    else if (wbm == 64 && wbn == 128) launch_pair<DBM, DBN, 64, 128>(pd, pw, st);                          \
    else if (wbm == 64 && wbn == 64) launch_pair<DBM, DBN, 64, 64>(pd, pw, st);                            \
    else return false;                                                                                     \
    return true;                                                                                           \
  }                                                                                                        \
  }                                                                                                        \
  }
