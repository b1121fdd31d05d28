// Host-side launch API of the gfx950 kernels. Every launcher is asynchronous on the given
// stream, allocates nothing and never synchronises, so any sequence of them can be captured
// into a hipGraph (cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>

namespace cdp {

// Exact division by a runtime-invariant divisor for dividends in [0, 2^31):
// q = umulhi(n, mul) >> shift with mul = ceil(2^(31+l) / d), l = ceil(log2 d) (the CUTLASS
// FastDivmod construction). Turns the ~30-instruction integer divide of the implicit-GEMM
// gathers into two VALU ops.
struct FastDiv {
  unsigned d, mul, shift;
};

inline FastDiv make_fastdiv(int d) {
  FastDiv f{(unsigned)d, 0u, 0u};
  if (d <= 1) return f;
  unsigned l = 0;
  while ((1ull << l) < (unsigned long long)d) ++l;
  const unsigned long long p = 31ull + l;
  f.mul = (unsigned)(((1ull << p) + (unsigned long long)d - 1ull) / (unsigned long long)d);
  f.shift = (unsigned)(p - 32ull);
  return f;
}

#if defined(__HIPCC__)
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return f.d == 1u ? n : (int)(__umulhi((unsigned)n, f.mul) >> f.shift);
}
#endif

// Output-row remap of a sub-pixel data-gradient launch: GEMM row m = (n, i, j) over a P x Q class
// grid lands in dX row (n, 2i + ph, 2j + pw) of an H x W image.
struct RowRemap {
  int on, H, W, ph, pw, P, Q;
  FastDiv fd_PQ, fd_Q;
};

#if defined(__HIPCC__)
__device__ __forceinline__ long long remap_row(const RowRemap& r, int m) {
  if (!r.on) return m;
  const int n = fdiv(m, r.fd_PQ);
  const int rem = m - n * r.P * r.Q;
  const int i = fdiv(rem, r.fd_Q);
  const int j = rem - i * r.Q;
  return ((long long)n * r.H + 2 * i + r.ph) * r.W + 2 * j + r.pw;
}
#endif

struct ConvGemmParams {
  const float* x;     // gather source, NHWC [N][H][W][C]
  const float* w;     // B^T rows [Nout][Kdim], Kdim ordered (kh, kw, c)
  float* y;           // [M][Nout] output, or split-K slab base [splits][M][Nout]
  const float* bias;  // [Nout] or nullptr (ignored when splits > 1)
  float* part;        // BN partials [ceil(M/BM)][Nout][2] (mean, M2) or nullptr
  int N, H, W, C;     // source dims
  int P, Q;           // GEMM-row spatial dims: rows m = (n, p, q)
  int KH, KW, stride, pad;
  int Nout, M, Kdim, ktiles, splits;
  FastDiv fd_PQ, fd_Q, fd_C, fd_KW;
  int pad_w;    // data gradient, sub-pixel class launches only: column pad (pad is the row pad)
  RowRemap rr;  // sub-pixel class launches: scatter output rows into dX
  const float* addend;  // optional: y += addend (same layout as y; may alias y)
  // f16x2 engine: the operand scales are powers of two per GEMM ROW of each operand, so they
  // factor out of every output exactly (x3_common.h):
  //   A (gathered x / dY): one scale per image, from a_img[n] = max |A| over image n (float bits,
  //     an activation's per-image slots, ActMaxOut); GEMM row m belongs to image m / (P*Q)
  //   B (W rows co, or W^T rows ci): one scale per row, max over b_np partials
  //     b_row[q * b_stride + n] (a weight's per-co / per-ci maxima, weight_prep)
  const unsigned* a_img;
  const float* b_row;
  int b_np, b_stride;
  int narrow;  // 1: four-byte epilogue stores (the A/B of conv_epilogue.h's wide stores, CDP_WIDE_STORES=0)
};

struct WgradParams {
  const float* dy;  // [M][Cout]
  const float* x;   // NHWC [N][H][W][C]
  float* out;       // slab base [splits][Cout][Kdim]
  int N, H, W, C, P, Q, KH, KW, stride, pad;
  int Cout, Kdim, M, splits;
  FastDiv fd_PQ, fd_Q, fd_C, fd_KW;
  // f16x2 engine: per-channel maxima (float bits, kActCopies copies each, ActMaxOut) of dY
  // ([copies][Cout]: one scale per output row co) and of x ([copies][C]: one scale per column
  // (tap, ci), by its channel ci)
  const unsigned* dy_ch;
  const unsigned* x_ch;
};

// ---- per-image / per-channel |max| of an activation (the f16x2 operand scales) ---------------
// A producer kernel of an NHWC activation [N][HW][C] (BatchNorm apply, channel padding, the
// standalone pass) reduces |value| per image and per channel on chip and publishes the maxima with
// one atomicMax per (block, image) and per (block, channel) into zero-initialised slots: the
// activation's "act max" tensor, int32 [N + kActCopies * C] = img[N] then ch[kActCopies][C] (float
// bits; for non-negative floats the unsigned order is the float order). Block b adds its channel
// maxima into copy b % kActCopies, so no more than 1/kActCopies of a grid's blocks meet on one
// address; consumers take the max over the copies.
constexpr int kActCopies = 8;
struct ActMaxOut {
  unsigned* img;  // [N] or nullptr (no maxima wanted)
  unsigned* ch;   // [kActCopies][C]
};
inline long long act_max_elems(long long N, long long C) { return N + kActCopies * C; }
// A conv weight [Co][T][Ci]'s maxima, float [nci * Co + nco * Ci] (nco = ceil(Co / 32), nci =
// ceil(Ci / 32)): per-co partials [nci][Co] (max over a 32-wide ci block and all taps), then per-ci
// partials [nco][Ci]; written by weight_prep_kernel / sgd_prep_kernel with plain stores.
inline long long weight_max_elems(long long Co, long long Ci) {
  return ((Ci + 31) / 32) * Co + ((Co + 31) / 32) * Ci;
}

// conv_igemm.hip (exact fp32-input MFMA)
void conv_igemm_launch(const ConvGemmParams& p, int bm, int bn, bool dgrad, hipStream_t st);
// conv_x3.hip (fp32-accurate 3-term bf16 split on the bf16 MFMA)
// np = operand planes: 3 = split-bf16 (six products), 2 = f16x2 (power-of-two-scaled operands,
// two fp16 terms, three products; needs p.a_img / p.b_row), 1 = operands rounded to bf16, one
// product per MAC (the non-parity fast mode)
void conv_x3_launch(const ConvGemmParams& p, int bm, int bn, bool dgrad, hipStream_t st, int np = 3);
void splitk_reduce_launch(const float* slab, int S, int M, int Nout, const float* bias, float* y, float* part,
                          hipStream_t st, const RowRemap* rr = nullptr, const float* addend = nullptr);
int splitk_rows_per_part();

// wgrad.hip
// x3: the split engines on the 16-bit MFMA (np as for conv_x3_launch); otherwise the exact
// fp32-input MFMA
void wgrad_launch(const WgradParams& p, int bm, int bn, bool x3, hipStream_t st, int np = 3);
// standalone act max of an NHWC activation [N][HW][C] (C % 4 == 0 or any C with the scalar path):
// per-image and per-channel |max| into zeroed slots o (see ActMaxOut), for operands without a
// fused producer
void act_max_launch(const float* x, int N, long long HW, int C, ActMaxOut o, hipStream_t st);
// Per-step weight preparation of a model's conv weights in one launch: for every segment (a
// channels_last weight [Co][T][Ci]) its maxima (weight_max_elems floats at part + pofs[s], the
// f16x2 operand scales; one block per 32x32 (co, ci) tile) and, when wt[s] != nullptr, the
// data-gradient operand W^T [Ci][T][Co].
constexpr int kMaxAmaxSegs = 64;
struct WeightPrepArgs {
  const float* w[kMaxAmaxSegs];
  float* wt[kMaxAmaxSegs];
  int co[kMaxAmaxSegs], t[kMaxAmaxSegs], ci[kMaxAmaxSegs];
  int blk0[kMaxAmaxSegs + 1];
  long long pofs[kMaxAmaxSegs];
  int nseg;
};
void weight_prep_launch(const WeightPrepArgs& a, float* part, hipStream_t st);
// SGD over an arena range fused with the next step's weight preparation (sgd_prep_kernel): one
// descriptor per conv weight (element offset in the range, W^T destination or null, shape, first
// block, offset of its maxima in the plan's buffer) and one per float4 chunk of the range outside
// every conv weight
struct SgdPrepSeg {
  long long off;
  float* wt;
  int co, t, ci, blk0;
  long long pofs;
};
struct SgdPrepChunk {
  long long start;
  int n4, pad;
};
constexpr int kSgdPrepChunk4 = 1024;  // float4 per rest chunk (one workgroup)
void sgd_prep_launch(float* p, const float* g, float* buf, const SgdPrepSeg* segs, int nseg, int nblk_w,
                     const SgdPrepChunk* chunks, int nchunk, float* wmax, const float* lr_ptr, float lr,
                     float momentum, float dampening, float wd, float grad_scale, bool nesterov, bool first,
                     bool maximize, hipStream_t st, long long* counter = nullptr);
void slab_sum_launch(const float* slab, int S, long long n, float* dst, bool accumulate, hipStream_t st);
void slab_sum_strided_launch(const float* slab, int S, long long n_src, int src_cols, int dst_cols, float* dst,
                             bool accumulate, hipStream_t st);

// stem.hip: 3x3 / stride 1 / pad 1 convs with Cin <= 4 and 64 outputs (exact fp32 MFMA)
bool stem_ok(int Cin, int KH, int KW, int stride, int pad, int Co);
void stem_fwd_launch(const float* x, const float* w, const float* bias, float* y, float* part, int N, int H, int W,
                     int Cin, int Co, hipStream_t st);
int stem_wgrad_blocks(int N, int H, int W);
// dW partials [nblk][64][36] with the pool(2x2)/ReLU/BatchNorm(training) backward applied on the fly;
// Co = 64, even H and W
void stem_wgrad_launch(const float* y, const float* gout, const float* stats, const float* sums, const float* x,
                       float* slab, int nblk, int N, int H, int W, int Cin, hipStream_t st);

// bwd_pair.hip: a block's data-gradient GEMM (MODE 0 transposed gather) and weight-gradient GEMM in
// one launch, when both are f16x2 tiles of one workgroup size (bwd_pair_ok)
bool bwd_pair_ok(const ConvGemmParams& pd, int bm, int bn, const WgradParams& pw, int wbm, int wbn, int np);
void bwd_pair_launch(const ConvGemmParams& pd, int bm, int bn, const WgradParams& pw, int wbm, int wbn,
                     hipStream_t st);

// bwd_fuse.hip: one launch that finishes a block's two gradient GEMMs' split-K slabs and starts the
// previous block's BatchNorm backward (see the file header).
struct BwdReduceArgs {
  // job D: y[m][n] = sum_z d_slab[z][m][n] (+ d_addend), [d_M][d_Nout], d_Nout % 4 == 0
  const float* d_slab;
  float* d_y;
  const float* d_addend;
  int d_S, d_M, d_Nout;
  // optional: BN-backward partials [ceil(d_M / rows_per_part)][d_Nout][bn_ps] of the BN whose
  // (pooled) output d_y is the gradient of; bn_y = its saved conv output [N][bn_H][bn_W][d_Nout]
  const float* bn_y;
  const float* bn_stats;
  float* bn_part;
  int bn_H, bn_W, bn_pool, bn_relu, bn_ps;
  FastDiv bn_fd_wo, bn_fd_ho;  // pooled width / height divisors (set by bwd_reduce_launch)
  // job W: w_dst[i] = sum_z w_slab[z][i] over w_n4 float4s
  const float4* w_slab;
  float4* w_dst;
  int w_S;
  long long w_n4;
  // set by the launcher
  int nbd, d_nbx, w_cb;
};
void bwd_reduce_launch(BwdReduceArgs a, hipStream_t st);
int bwd_reduce_rows_per_part();

// bn.hip
int bn_bwd_grid(int N, int H, int W, int C, bool pool);
void bn_finalize_launch(const float* part, int nparts, int rpp, int M, int C, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                        float* stats, hipStream_t st);
void bn_eval_stats_launch(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                          float* stats, hipStream_t st);
// Every BN apply kernel below takes an ActMaxOut `am` (am.img == nullptr: none wanted): the
// per-image / per-channel |max| of the tensor it writes (out / dy), for the consumer GEMMs' f16x2
// operand scales.
// finalize + apply in one launch (training, no residual, nparts <= 128, C % 64 == 0)
bool bn_fin_act_ok(int nparts, int C, bool residual);
int bn_fin_act_grid(int N, int H, int W, int C, bool pool, int nparts = 0);  // nparts 0: 64-channel blocks
void bn_fin_act_launch(const float* part, int nparts, int rpp, int C, const float* gamma, const float* beta,
                       float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                       float* stats, const float* y, float* out, int N, int H, int W, bool pool, bool relu,
                       ActMaxOut am, hipStream_t st);
// backward twin (training, no residual, nparts <= 128, C % 64 == 0, even map under pooling):
// finalize the statistics partials (dbeta, dgamma, conv-bias gradient when gdb) and write dy in one
// launch
bool bn_bwd_fin_apply_ok(int nparts, int C, int H, int W, bool pool);
void bn_bwd_fin_apply_launch(const float* part, int nparts, int ps, const float* y, const float* gout,
                             const float* stats, float* dy, float* gbeta, float* ggamma, float* gdb, int N, int H,
                             int W, int C, bool pool, bool relu, ActMaxOut am, hipStream_t st);
int bn_act_grid(int N, int H, int W, int C, bool pool);
// rmask (residual + ReLU blocks): one byte per float4 of the output, bit e = (output channel 4q+e > 0),
// at the float4's index (pixel * C/4 + q). The backward reads it instead of the 16x larger output.
// res_y / res_st: the residual as a raw conv output and its BN stats block, normalized on the fly
// (res_y * scale + shift, no activation) instead of a materialized `res`
void bn_act_fwd_launch(const float* y, const float* stats, const float* res, float* out, int N, int H, int W, int C,
                       bool pool, bool relu, hipStream_t st, ActMaxOut am = ActMaxOut{nullptr, nullptr},
                       unsigned char* rmask = nullptr, const float* res_y = nullptr, const float* res_st = nullptr);
void bn_bwd_reduce_launch(const float* y, const float* gout, const float* stats, float* part, int nblocks, int N,
                          int H, int W, int C, bool pool, bool relu, const float* zout, hipStream_t st,
                          bool with_xsum = false, const unsigned char* rmask = nullptr);
void chan_finalize_launch(const float* part, int nparts, int C, float* out, float* g0, float* g1, bool accumulate,
                          hipStream_t st, int ps = 2, float* gdb = nullptr, const float* scale = nullptr,
                          long long M = 0, int dbmode = 0);
void bn_bwd_apply_launch(const float* y, const float* gout, const float* stats, const float* sums, float* dy,
                         float* dbias_part, int nblocks, int N, int H, int W, int C, bool pool, bool relu,
                         const float* zout, float* dres, hipStream_t st, ActMaxOut am = ActMaxOut{nullptr, nullptr},
                         const unsigned char* rmask = nullptr);

// misc.hip
void xent_fwd_launch(const float* logits, const long long* tgt, int B, int C, float* loss, long long* correct,
                     float* sum_out, hipStream_t st);
void xent_bwd_launch(const float* logits, const long long* tgt, const float* gscale, int B, int C, float* dlogits,
                     hipStream_t st);
// counter (optional): a step counter the kernel advances by one (DeviceLoader.advance_with)
void sgd_launch(float* p, const float* g, float* buf, long long n, const float* lr_ptr, float lr, float momentum,
                float dampening, float wd, float grad_scale, bool nesterov, bool first, bool maximize,
                hipStream_t st, long long* counter = nullptr);
// nbatches > 0: batch offset idx_off + (counter % nbatches) * B; labels_out[b] = labels[idx[...]] when given
void augment_launch(const unsigned char* imgs, const long long* idx, long long idx_off, int B, int H, int W, int C,
                    const float* mean, const float* inv_std, int pad, bool flip, const long long* counter,
                    unsigned long long seed, float* out, hipStream_t st, long long nbatches = 0,
                    const long long* labels = nullptr, long long* labels_out = nullptr);
// zeros into the NHWC dX pixels of the sub-pixel parity classes set in mask (bit 2 ph + pw)
// dst[0 .. bytes) = src[0 .. bytes) as a kernel (16-B accesses when both pointers and bytes allow)
void copy_bytes_launch(void* dst, const void* src, long long bytes, hipStream_t st);
// p[0 .. n) = v as a kernel
void fill_u32_launch(unsigned* p, long long n, unsigned v, hipStream_t st);
void subpixel_zero_launch(float* dx, int N, int H, int W, int C, int mask, hipStream_t st);
void counter_inc_launch(long long* c, hipStream_t st);
void wtrans_launch(const float* w, float* wt, int Co, int T, int Ci, hipStream_t st);
// sub-filter transpose: wt[ci][a][b][co] = w[co][kh0 + 2a][kw0 + 2b][ci] (a < nkh, b < nkw)
void wtrans_sub_launch(const float* w, float* wt, int Co, int KH, int KW, int Ci, int kh0, int kw0, int nkh, int nkw,
                       hipStream_t st);
// NHWC channel padding C (<= 4) -> 4 with zeros, N images of HW pixels; am (optional): the padded
// tensor's act max (per image / per channel, see ActMaxOut)
void pad_c4_launch(const float* x, int N, long long HW, int C, float* out, ActMaxOut am, hipStream_t st);
// dst = mean of k <= kMaxStackSrcs tensors; srcs is a HOST array (the pointers travel in the kernel
// arguments: no pointer-table upload, so nothing can race with a host buffer's lifetime)
constexpr int kMaxStackSrcs = 128;
void stack_mean_launch(const float* const* srcs, int k, long long n, float* dst, hipStream_t st);
void scale_launch(float* x, long long n, float a, hipStream_t st);
void delay_scale_launch(float* x, long long n, float a, double delay_us, hipStream_t st);
// ts[idx] = the GPU wall clock (100 MHz) when the stream reaches this point
void timestamp_launch(long long* ts, int idx, hipStream_t st);
void colsum_launch(const float* x, int R, int C, float* out, bool accumulate, hipStream_t st);
void small_linear_fwd_launch(const float* x, const float* w, const float* b, int B, int I, int O, float* y,
                             hipStream_t st);
void small_linear_bwd_launch(const float* dy, const float* x, const float* w, int B, int I, int O, float* dx, float* dw,
                             float* db, hipStream_t st);
// CrossEntropy backward + narrow Linear backward in one launch (B * O <= kXentLinMax, O <= 16),
// optionally with the BN backward partials of the block that produced the Linear's input
// (y != nullptr: that block's pre-BN output [B][pool ? 2x2 : 1x1][C = I] NHWC, stats [4][C],
// part [1][C][ps] out)
constexpr int kXentLinMax = 8192;
constexpr int kXentLinRows = 32;  // dX rows per block (and per BN partial)
inline int xent_lin_chunks(int B) { return (B + kXentLinRows - 1) / kXentLinRows; }
struct XentBnLink {
  const float* y;
  const float* stats;
  float* part;
  int pool, relu, ps;
};
void xent_linear_bwd_launch(const float* logits, const long long* tgt, const float* gscale, const float* x,
                            const float* w, int B, int I, int O, float* dlogits, float* dx, float* dw, float* db,
                            const XentBnLink& lk, hipStream_t st);
void avgpool_fwd_launch(const float* x, int N, int HW, int C, float* y, hipStream_t st);
void avgpool_bwd_launch(const float* gy, int N, int HW, int C, float* gx, hipStream_t st);
// NHWC, C % 4 == 0; arg = window-local argmax tap (uint8, k*k <= 255)
void maxpool_fwd_launch(const float* x, int N, int H, int W, int C, int k, int s, int p, int Ho, int Wo, float* y,
                        unsigned char* arg, hipStream_t st);
void maxpool_bwd_launch(const float* gy, const unsigned char* arg, int N, int H, int W, int C, int k, int s, int p,
                        int Ho, int Wo, float* gx, hipStream_t st);

}  // namespace cdp
