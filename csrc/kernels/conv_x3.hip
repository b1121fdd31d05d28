// Implicit-GEMM convolution at fp32 accuracy on the bf16 matrix cores (gfx950).
//
// gfx950 has no reduced-precision fp32 MFMA (no xf32) and its exact fp32-input MFMA
// (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate. This kernel keeps fp32 numerics while
// using v_mfma_f32_32x32x16_bf16: every fp32 operand is split into three bf16 terms,
//     a = a0 + a1 + a2,   a0 = rn(a), a1 = rn(a - a0), a2 = rn(a - a0 - a1)
// (each subtraction is exact, and three 8-bit significands cover fp32's 24 bits, so the split is
// exact up to underflow), and the product is formed from the six terms of order >= 2^-16:
//     a*b ~= a0b0 + (a0b1 + a1b0) + (a0b2 + a1b1 + a2b0)
// accumulated in fp32 by the MFMA. The dropped terms are <= 2^-23 |ab| -- the size of one fp32
// rounding -- so the result matches an fp32 GEMM to within the accumulation error of the fp32
// MFMA itself (tests/test_kernels_gpu.py::test_x3_gemm_accuracy measures both against fp64).
// Six bf16 MFMAs cost 6*32 = 192 cycles per 32x32x16 step versus 8*64 = 512 for eight fp32
// MFMAs: 2.67x the MFMA throughput.
//
// Same GEMM mapping as conv_igemm.hip (forward / transposed-gather data gradient, MODE 0/1/2
// gathers, identical epilogue). Pipeline (one barrier per K-tile): operands are gathered
// global -> registers through buffer loads whose range check supplies the zero padding; two
// register sets and two LDS stages let the split + store of tile t+1 (v_cvt_pk_bf16_f32,
// v_pk_add_f32) interleave with the MFMAs of tile t while tile t+2 is in flight. LDS rows are
// 64 B with XOR-swizzled 16-B chunks (chunk_pos), conflict free for the ds_write_b128 stores and
// the ds_read_b128 fragment reads. 96 KB of LDS for 128x128 (one workgroup per CU, the MFMA
// pipe kept busy by the in-wave interleave), 72 KB for 64x128.
#include "conv_x3_body.h"

namespace cdp {

namespace {

using namespace x3conv;

template <int BM, int BN, int MODE, bool DGRAD, int NP = 3>
__global__ __launch_bounds__(waves_m<BM>() * 128, (NP == 2 && BM + BN <= 256) ? 2 : (BM + BN >= 256) ? 1 : 2) void
conv_x3_kernel(ConvGemmParams p) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[conv_x3_smem_elems<BM, BN, NP>()];
  conv_x3_body<BM, BN, MODE, DGRAD, NP>(p, smem, blockIdx.x, gridDim.x);
}

template <int BM, int BN, int MODE, bool DGRAD>
void launch_x3(const ConvGemmParams& p, int ntiles, int np, hipStream_t st) {
  const dim3 blk(waves_m<BM>() * 128), grd(ntiles * p.splits);
  if (np == 1) hipLaunchKernelGGL((conv_x3_kernel<BM, BN, MODE, DGRAD, 1>), grd, blk, 0, st, p);
  else if (np == 2) hipLaunchKernelGGL((conv_x3_kernel<BM, BN, MODE, DGRAD, 2>), grd, blk, 0, st, p);
  else hipLaunchKernelGGL((conv_x3_kernel<BM, BN, MODE, DGRAD, 3>), grd, blk, 0, st, p);
}

template <int MODE, bool DGRAD>
void dispatch_x3(const ConvGemmParams& p, int bm, int bn, int np, hipStream_t st) {
  const int ntm = (p.M + bm - 1) / bm, ntn = (p.Nout + bn - 1) / bn;
  const int nt = ntm * ntn;
  if (bm == 256) launch_x3<256, 128, MODE, DGRAD>(p, nt, np, st);
  else if (bm == 128 && bn == 128) launch_x3<128, 128, MODE, DGRAD>(p, nt, np, st);
  else if (bm == 128 && bn == 64) launch_x3<128, 64, MODE, DGRAD>(p, nt, np, st);
  else if (bm == 64 && bn == 128) launch_x3<64, 128, MODE, DGRAD>(p, nt, np, st);
  else launch_x3<64, 64, MODE, DGRAD>(p, nt, np, st);
}

}  // namespace

void conv_x3_launch(const ConvGemmParams& p, int bm, int bn, bool dgrad, hipStream_t st, int np) {
  if ((p.C % BK) == 0 && (p.Kdim % BK) == 0) {
    if (dgrad) dispatch_x3<0, true>(p, bm, bn, np, st);
    else dispatch_x3<0, false>(p, bm, bn, np, st);
  } else if ((p.C % 4) == 0 && (p.Kdim % 4) == 0) {
    if (dgrad) dispatch_x3<1, true>(p, bm, bn, np, st);
    else dispatch_x3<1, false>(p, bm, bn, np, st);
  } else {
    if (dgrad) dispatch_x3<2, true>(p, bm, bn, np, st);
    else dispatch_x3<2, false>(p, bm, bn, np, st);
  }
}

}  // namespace cdp
