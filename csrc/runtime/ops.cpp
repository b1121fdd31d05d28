// Torch-facing wrappers around the gfx950 kernels: shape checks, workspace allocation through
// PyTorch's caching allocator (graph-capture safe), tile / split-K selection, and the fused
// Conv -> BatchNorm -> ReLU [-> MaxPool] block used by the VGG model family
// (/root/reference/src/Part 1/model.py:11-27).
//
// Layout contract: activations are logical NCHW tensors in channels_last memory format (physical
// NHWC); conv weights are logical [Co, Ci, KH, KW] in channels_last format (physical OHWI =
// GEMM B^T rows). Outputs follow the same contract, so every op is a drop-in for its torch.nn
// counterpart on channels_last tensors.
#include "ops.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <tuple>
#include <string>
#include <unordered_map>

#include "../kernels/kernels.h"

namespace cdp {

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}

at::Tensor nhwc(const at::Tensor& t) {
  if (t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast)) return t;
  return t.contiguous(at::MemoryFormat::ChannelsLast);
}

const float* fptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
float* fptr_mut(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

struct GemmPlan {
  int bm, bn, splits, ktiles;
};

int num_cus() {
  static int cus = [] {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    return prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  }();
  return cus;
}

// Conv GEMM engine:
//   3 = f16x2 (default): power-of-two-scaled operands as two fp16 terms, three products on the
//       fp16 MFMA (conv_x3.hip / wgrad.hip with NP = 2, see x3_common.h); its error against fp64
//       is at or below the exact fp32 MFMA's on every conv shape class (tests/test_kernels_gpu.py)
//   1 = x3: 3-term bf16 split, six products on the bf16 MFMA (same kernels, NP = 3), as accurate
//   0 = exact fp32-input MFMA (conv_igemm.hip)
//   2 = plain bf16 operands with fp32 accumulation (one product per MAC: the non-parity fast mode)
// CDP_CONV_GEMM=f16x2|x3|f32|bf16 selects at start-up; set_conv_gemm at run time.
int& conv_gemm_mode() {
  static int m = [] {
    const char* e = std::getenv("CDP_CONV_GEMM");
    if (e && std::string(e) == "f32") return 0;
    if (e && std::string(e) == "bf16") return 2;
    if (e && std::string(e) == "x3") return 1;
    return 3;
  }();
  return m;
}
bool x3_family() { return conv_gemm_mode() != 0; }
bool f16x2_mode() { return conv_gemm_mode() == 3; }
// 16-bit operand planes of the split kernels for the current engine
int split_planes() { return conv_gemm_mode() == 2 ? 1 : conv_gemm_mode() == 3 ? 2 : 3; }

// ---------------------------------------------------------------- act max slots
// An activation's per-image / per-channel |max| slots (ActMaxOut, kernels.h) must start at zero:
// its producer atomically maxes into them. They are views into chunks of device memory zeroed by
// ONE fill kernel per chunk, not per producer:
//  * eager: a ring of chunks; the current chunk is bumped through, and a chunk is re-zeroed and
//    reused only once no slot view of it is alive (its storage is then held by the ring alone);
//  * inside a hipGraph capture: every capture takes fresh chunks (from the graph's memory pool,
//    kept alive with it) whose zero-fill kernel is captured, so each replay re-zeroes them before its
//    producers run.
// Everything is ordered on the current stream, like the caching allocator's reuse; a chunk taken up
// on another stream than its last allocating stream (its memset and producers) first makes the new
// stream wait for that one. Readers are assumed to run on the allocating stream, or to be ordered
// before its next work (the consumer GEMMs of this runtime run on the producer's stream); a caller
// reading slots on another stream must keep the slot tensor alive until that read has completed.
constexpr long long kSlotChunk = 1LL << 16;     // int32 slots per eager chunk (256 KB)
constexpr long long kCapSlotChunk = 1LL << 18;  // ... per captured chunk (1 MB: one fill node for a VGG-11 step)
struct SlotPool {
  std::vector<at::Tensor> ring;
  std::vector<long long> used;
  std::vector<hipStream_t> last;  // stream of each chunk's latest memset / allocation
  hipEvent_t ev = nullptr;
  int cur = -1;
  unsigned long long cap_id = 0;
  at::Tensor cap_cur;
  long long cap_used = 0;
  long long cap_total = 0, cap_hint = 0;  // slots taken by the current / largest earlier capture
  // a capture's chunks stay referenced until that capture has ended: freed earlier, their blocks
  // could be handed to a later allocation of the SAME capture (the graph's private pool) while the
  // captured memset and producers still address them. Once the capture is over, the pool keeps the
  // blocks for the graph's lifetime, so the references are dropped when the next
  // capture starts (not at an eager call: one on another stream cannot tell whether the capture is
  // still running) -- at most one capture's chunks are held, however often the step is re-captured.
  std::vector<std::pair<unsigned long long, at::Tensor>> cap_keep;
};

std::atomic<long long>& slot_memsets() {
  static std::atomic<long long> n{0};
  return n;
}

template <class Fresh>
at::Tensor alloc_slots_impl(SlotPool& P, long long n, const at::TensorOptions& opts, hipStream_t st,
                            hipStreamCaptureStatus cs, unsigned long long id, Fresh& fresh);

at::Tensor alloc_slots(long long n, const at::Tensor& like, hipStream_t st) {
  static std::mutex mu;
  static std::unordered_map<int, SlotPool> pools;
  std::lock_guard<std::mutex> lk(mu);
  n = (n + 63) / 64 * 64;  // 256-B aligned views
  SlotPool& P = pools[like.get_device()];
  const at::TensorOptions opts = like.options().dtype(at::kInt);
  // Chunks are zeroed by a KERNEL, not hipMemsetAsync: a captured memset node was measured to race
  // with the step's first producers when other work ran between replays (the replayed step drifted
  // from its eager twin; with the fill kernel it is bitwise equal, scripts/diag/replay_vs_eager.py)
  auto fresh = [&](long long size) {
    at::Tensor b = at::empty({size}, opts);
    fill_u32_launch(reinterpret_cast<unsigned*>(b.data_ptr<int>()), size, 0u, st);
    slot_memsets().fetch_add(1, std::memory_order_relaxed);
    return b;
  };
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  TORCH_CHECK(hipStreamGetCaptureInfo(st, &cs, &id) == hipSuccess, "act max slots: capture query failed");
  static const bool trace = [] {
    const char* e = std::getenv("CDP_SLOT_TRACE");
    return e && e[0] == '1';
  }();
  if (trace) {
    at::Tensor v = alloc_slots_impl(P, n, opts, st, cs, id, fresh);
    std::fprintf(stderr, "[slots] cap=%d id=%llu st=%p ptr=%p n=%lld\n", (int)cs, id, (void*)st, v.data_ptr(), n);
    return v;
  }
  return alloc_slots_impl(P, n, opts, st, cs, id, fresh);
}

template <class Fresh>
at::Tensor alloc_slots_impl(SlotPool& P, long long n, const at::TensorOptions& opts, hipStream_t st,
                            hipStreamCaptureStatus cs, unsigned long long id, Fresh& fresh) {
  if (cs == hipStreamCaptureStatusActive && id != P.cap_id && !P.cap_keep.empty()) {
    P.cap_keep.clear();  // a new capture: the earlier ones have ended (their pools keep the blocks)
    P.cap_cur = at::Tensor();
  }
  if (cs == hipStreamCaptureStatusActive) {
    // a capture's first chunk is sized by the largest earlier capture (a re-captured step takes one
    // chunk, i.e. one captured memset of just its slots; ResNet-50 took eight 256 KB ones)
    if (id != P.cap_id) {
      P.cap_hint = std::max(P.cap_hint, P.cap_total);
      P.cap_total = 0;
    }
    if (id != P.cap_id || !P.cap_cur.defined() || P.cap_used + n > P.cap_cur.numel()) {
      P.cap_cur = fresh(std::max(std::max(kCapSlotChunk, n), id != P.cap_id ? P.cap_hint : 0LL));
      P.cap_keep.emplace_back(id, P.cap_cur);
      P.cap_used = 0;
      P.cap_id = id;
    }
    P.cap_total += n;
    at::Tensor v = P.cap_cur.narrow(0, P.cap_used, n);
    P.cap_used += n;
    return v;
  }
  TORCH_CHECK(cs == hipStreamCaptureStatusNone, "act max slots: stream capture invalidated");
  // st waits for whatever chunk i's last stream has enqueued (no-op on the same stream)
  auto order_after = [&](int i) {
    const hipStream_t prev = P.last[i];
    if (prev != st) {
      if (!P.ev) TORCH_CHECK(hipEventCreateWithFlags(&P.ev, hipEventDisableTiming) == hipSuccess, "act max slots: event");
      TORCH_CHECK(hipEventRecord(P.ev, prev) == hipSuccess && hipStreamWaitEvent(st, P.ev, 0) == hipSuccess,
                  "act max slots: cross-stream ordering failed");
      P.last[i] = st;
    }
  };
  if (P.cur < 0 || P.used[P.cur] + n > P.ring[P.cur].numel()) {
    int pick = -1;
    for (size_t i = 0; i < P.ring.size(); ++i)
      if ((int)i != P.cur && P.ring[i].storage().use_count() == 1 && P.ring[i].numel() >= n) {
        pick = (int)i;
        break;
      }
    if (pick < 0) {
      P.ring.push_back(fresh(std::max(kSlotChunk, n)));
      P.used.push_back(0);
      P.last.push_back(st);
      pick = (int)P.ring.size() - 1;
    } else {
      order_after(pick);  // the chunk's last readers finish before the re-zeroing
      fill_u32_launch(reinterpret_cast<unsigned*>(P.ring[pick].data_ptr<int>()), P.ring[pick].numel(), 0u, st);
      slot_memsets().fetch_add(1, std::memory_order_relaxed);
      P.used[pick] = 0;
    }
    P.cur = pick;
  } else {
    order_after(P.cur);  // the chunk's memset precedes the new producer
  }
  at::Tensor v = P.ring[P.cur].narrow(0, P.used[P.cur], n);
  P.used[P.cur] += n;
  return v;
}

// (images, channels, pixels per image) of an activation operand: NHWC 4-D or [rows, features] 2-D
struct ActShape {
  long long N, C, HW;
};
ActShape act_shape(const at::Tensor& t) {
  TORCH_CHECK(t.dim() == 4 || t.dim() == 2, "act max: 4-D NHWC or 2-D tensors only");
  const long long N = t.size(0), C = t.size(1);
  return {N, C, N * C > 0 ? t.numel() / (N * C) : 0};
}
ActMaxOut act_out(const at::Tensor& s, long long N) {
  unsigned* b = reinterpret_cast<unsigned*>(s.data_ptr<int>());
  return ActMaxOut{b, b + N};
}
// Fresh zeroed act max slots for an activation of `like`'s images / channels (f16x2 engine only).
at::Tensor new_act_max(long long N, long long C, const at::Tensor& like, hipStream_t st) {
  return alloc_slots(act_max_elems(N, C), like, st);
}

// The act max of an f16x2 GEMM activation operand t (NHWC channels_last 4-D or contiguous 2-D):
// its producer's when the caller has it, else a standalone pass. Undefined outside the f16x2 engine.
at::Tensor act_max(const at::Tensor& t, const c10::optional<at::Tensor>& given, hipStream_t st) {
  if (!f16x2_mode()) return at::Tensor();
  const ActShape s = act_shape(t);
  if (given.has_value() && given->defined()) {
    TORCH_CHECK(given->scalar_type() == at::kInt && given->numel() >= act_max_elems(s.N, s.C),
                "act max of a [", s.N, ", ", s.C, ", ...] operand must be int32 with >= ", act_max_elems(s.N, s.C),
                " slots (per image, then ", kActCopies, " x per channel)");
    return *given;
  }
  // per-image / per-channel maxima do not depend on the memory layout: measure a dense NHWC view
  const at::Tensor u = t.dim() == 2 ? t.contiguous() : nhwc(t);
  at::Tensor slots = new_act_max(s.N, s.C, u, st);
  act_max_launch(u.data_ptr<float>(), (int)s.N, s.HW, (int)s.C, act_out(slots, s.N), st);
  return slots;
}
}  // namespace

std::vector<std::vector<at::Tensor>> weight_prep_impl(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t,
                                                      const at::Tensor* amax_into,
                                                      const std::vector<c10::optional<at::Tensor>>* wt_into);

namespace {
// A conv weight's maxima (weight_max_elems floats; 2-D [O, I] weights as [O, I, 1, 1]): given or
// measured here (weight_prep without the transpose). Undefined outside the f16x2 engine.
at::Tensor weight_max(const at::Tensor& w, const c10::optional<at::Tensor>& given) {
  if (!f16x2_mode()) return at::Tensor();
  const long long Co = w.size(0), Ci = w.size(1);
  if (given.has_value() && given->defined()) {
    TORCH_CHECK(given->scalar_type() == at::kFloat && given->numel() == weight_max_elems(Co, Ci),
                "weight max of a [", Co, ", ", Ci, ", ...] weight must be ", weight_max_elems(Co, Ci), " floats");
    return *given;
  }
  const at::Tensor w4 = w.dim() == 2 ? w.reshape({Co, Ci, 1, 1}) : w;
  return weight_prep_impl({w4}, {false}, nullptr, nullptr)[0][0];
}
}  // namespace

int64_t act_max_memsets() { return slot_memsets().load(std::memory_order_relaxed); }
int64_t act_max_copies() { return kActCopies; }

// The act max of a tensor by the standalone pass (tests; the f16x2 engine only, else undefined).
at::Tensor act_max_of(const at::Tensor& t) {
  check_f32_cuda(t, "act_max input");
  const at::Tensor u = t.dim() == 4 ? nhwc(t) : t.contiguous();
  return act_max(u, c10::nullopt, cur_stream());
}

// Per-step preparation of a model's conv weights in one launch per 64 weights: {maxima per weight
// (f16x2 engine: weight_max_elems floats each, the per-co / per-ci |max| partials; empty list
// otherwise), W^T [Ci][KH*KW*Co] per weight with want_t[i] (undefined tensor otherwise)}. The
// transposes are the data-gradient B operand, so backward no longer transposes every weight in its
// own launch.
// With `into` (maxima + W^T tensors from sgd_prep_plan), the products are written into those
// buffers instead of fresh ones (refreshing a fused-step plan after the weights were edited).
std::vector<std::vector<at::Tensor>> weight_prep_impl(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t,
                                                      const at::Tensor* amax_into,
                                                      const std::vector<c10::optional<at::Tensor>>* wt_into) {
  TORCH_CHECK(ts.size() == want_t.size(), "weight_prep: one want_t flag per weight");
  std::vector<at::Tensor> amax, wts;
  hipStream_t st = cur_stream();
  long long into_off = 0;
  for (size_t s0 = 0; s0 < ts.size(); s0 += kMaxAmaxSegs) {
    const size_t ns = std::min<size_t>(kMaxAmaxSegs, ts.size() - s0);
    WeightPrepArgs a{};
    a.nseg = (int)ns;
    std::vector<at::Tensor> keep;
    int tot = 0;
    long long ptot = 0;
    for (size_t i = 0; i < ns; ++i) {
      const at::Tensor& t0 = ts[s0 + i];
      check_f32_cuda(t0, "weight_prep input");
      TORCH_CHECK(t0.dim() == 4, "weight_prep expects conv weights [Co, Ci, KH, KW]");
      const at::Tensor t = nhwc(t0);
      keep.push_back(t);
      const int Co = t.size(0), Ci = t.size(1), T = t.size(2) * t.size(3);
      a.w[i] = t.data_ptr<float>();
      a.co[i] = Co;
      a.t[i] = T;
      a.ci[i] = Ci;
      at::Tensor wt;
      if (want_t[s0 + i]) {
        if (wt_into) {
          TORCH_CHECK((*wt_into)[s0 + i].has_value() && (*wt_into)[s0 + i]->numel() == (long long)Ci * T * Co,
                      "weight_prep_into: missing / mis-sized W^T buffer");
          wt = *(*wt_into)[s0 + i];
        } else {
          wt = at::empty({Ci, (long long)T * Co}, t.options());
        }
      }
      a.wt[i] = wt.defined() ? wt.data_ptr<float>() : nullptr;
      wts.push_back(wt);
      a.blk0[i] = tot;
      a.pofs[i] = ptot;
      tot += ((Co + 31) / 32) * ((Ci + 31) / 32);
      ptot += weight_max_elems(Co, Ci);
    }
    a.blk0[ns] = tot;
    at::Tensor part;
    if (amax_into) {
      TORCH_CHECK(amax_into->numel() >= into_off + ptot, "weight_prep_into: maxima buffer too small");
      part = amax_into->narrow(0, into_off, ptot);
      into_off += ptot;
    } else {
      part = at::empty({ptot}, ts[s0].options());
    }
    weight_prep_launch(a, part.data_ptr<float>(), st);
    if (f16x2_mode())
      for (size_t i = 0; i < ns; ++i) {
        const long long end = i + 1 < ns ? a.pofs[i + 1] : ptot;
        amax.push_back(part.narrow(0, a.pofs[i], end - a.pofs[i]));
      }
  }
  return {amax, wts};
}

std::vector<std::vector<at::Tensor>> weight_prep(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t) {
  return weight_prep_impl(ts, want_t, nullptr, nullptr);
}

void weight_prep_into(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t, const at::Tensor& amax,
                      const std::vector<c10::optional<at::Tensor>>& wts) {
  TORCH_CHECK(wts.size() == ts.size(), "weight_prep_into: one W^T slot per weight");
  weight_prep_impl(ts, want_t, &amax, &wts);
}

namespace {

// f16x2 operand scales of a conv GEMM (kernels.h): A rows by the gathered operand's images (act
// max `a` of p.N images x p.C channels), B rows from the weight's maxima `wm` of a [Co, Ci, ...]
// weight -- its per-co partials for the forward (B = W), its per-ci partials for the data gradient
// (B = W^T).
void set_scales(ConvGemmParams& p, const at::Tensor& a, const at::Tensor& wm, bool dgrad, long long Co, long long Ci) {
  if (!a.defined() || !wm.defined()) return;
  TORCH_CHECK(a.numel() >= act_max_elems(p.N, p.C), "conv GEMM: act max smaller than its operand's");
  TORCH_CHECK(wm.numel() == weight_max_elems(Co, Ci), "conv GEMM: weight maxima of a different shape");
  p.a_img = reinterpret_cast<const unsigned*>(a.data_ptr<int>());
  const long long nco = (Co + 31) / 32, nci = (Ci + 31) / 32;
  if (!dgrad) {
    p.b_row = wm.data_ptr<float>();
    p.b_np = (int)nci;
    p.b_stride = (int)Co;
  } else {
    p.b_row = wm.data_ptr<float>() + nci * Co;
    p.b_np = (int)nco;
    p.b_stride = (int)Ci;
  }
}
// weight gradient: dY's per-channel maxima scale the output rows (co), x's the columns (tap, ci)
void set_scales(WgradParams& p, const at::Tensor& dy, const at::Tensor& x) {
  if (!dy.defined() || !x.defined()) return;
  TORCH_CHECK(dy.numel() >= act_max_elems(p.N, p.Cout) && x.numel() >= act_max_elems(p.N, p.C),
              "weight gradient: act max smaller than its operand's");
  p.dy_ch = reinterpret_cast<const unsigned*>(dy.data_ptr<int>()) + p.N;
  p.x_ch = reinterpret_cast<const unsigned*>(x.data_ptr<int>()) + p.N;
}

// The x3 kernels address through 32-bit buffer offsets and 24-bit index multiplies; shapes past
// those limits (or a strided data-gradient other than stride 2) take the exact fp32 kernels.
constexpr long long kBuf = 1LL << 31;
constexpr long long kIdx = 1LL << 23;
bool x3_ok(const ConvGemmParams& p, bool dgrad) {
  const long long hwc = (long long)p.H * p.W * p.C;
  return (long long)p.N * hwc * 4 < kBuf && (long long)p.Nout * p.Kdim * 4 < kBuf && hwc < kIdx &&
         (long long)p.P * p.Q < kIdx && p.Kdim < kIdx && (!dgrad || p.stride == 1 || p.stride == 2);
}
bool x3_ok(const WgradParams& p) {
  const long long hwc = (long long)p.H * p.W * p.C;
  return (long long)p.N * hwc * 4 < kBuf && (long long)p.M * p.Cout * 4 < kBuf && hwc < kIdx &&
         (long long)p.P * p.Q < kIdx;
}

// ---------------------------------------------------------------- GEMM launch log
// CDP_GEMM_LOG=1: every conv / weight-gradient GEMM launch appends (kind, M, N, K, bm, bn, splits)
// in enqueue order, so a profile's GEMM dispatches can be labelled with their shapes
// (scripts/pmc_resnet_layers.py joins it with rocprofv3's kernel trace and counters).
struct GemmLogRec {
  std::string kind;
  long long M, N, K;
  int bm, bn, splits;
};
static std::mutex& gemm_log_mu() {
  static std::mutex m;
  return m;
}
static std::vector<GemmLogRec>& gemm_log_vec() {
  static std::vector<GemmLogRec> v;
  return v;
}
static bool gemm_log_on() {
  static const bool on = [] {
    const char* e = std::getenv("CDP_GEMM_LOG");
    return e && e[0] == '1';
  }();
  return on;
}
static void gemm_log_add(const char* kind, long long M, long long N, long long K, int bm, int bn, int splits) {
  if (!gemm_log_on()) return;
  std::lock_guard<std::mutex> g(gemm_log_mu());
  gemm_log_vec().push_back({kind, M, N, K, bm, bn, splits});
}
std::vector<std::tuple<std::string, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>> gemm_log_snapshot(bool clear) {
  std::lock_guard<std::mutex> g(gemm_log_mu());
  std::vector<std::tuple<std::string, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>> out;
  for (const auto& r : gemm_log_vec()) out.emplace_back(r.kind, r.M, r.N, r.K, r.bm, r.bn, r.splits);
  if (clear) gemm_log_vec().clear();
  return out;
}
static void wgrad_launch_logged(const WgradParams& p, int bm, int bn, bool x3, hipStream_t st, int np) {
  gemm_log_add("wgrad", p.Cout, p.Kdim, (long long)p.M, bm, bn, p.splits);
  wgrad_launch(p, bm, bn, x3, st, np);
}

// CDP_WIDE_STORES=0: the conv GEMM epilogues store four bytes per lane (conv_epilogue.h)
static bool narrow_stores() {
  static const bool on = [] {
    const char* e = std::getenv("CDP_WIDE_STORES");
    return e && e[0] == '0';
  }();
  return on;
}

void conv_launch(const ConvGemmParams& p0, int bm, int bn, bool dgrad, hipStream_t st) {
  gemm_log_add(dgrad ? "dgrad" : "fwd", p0.M, p0.Nout, p0.Kdim, bm, bn, p0.splits);
  ConvGemmParams p = p0;
  p.narrow = narrow_stores();
  if (x3_family() && x3_ok(p, dgrad)) {
    TORCH_CHECK(!f16x2_mode() || (p.a_img && p.b_row), "f16x2 conv GEMM launched without operand maxima");
    conv_x3_launch(p, bm, bn, dgrad, st, split_planes());
  }
  else conv_igemm_launch(p, bm, bn, dgrad, st);
}

// Launch a conv GEMM with g.splits split-K slices. p.y / p.bias / p.addend / p.part / p.rr describe
// the final output; split slices meet through an fp32 slab and the reduction kernel, which also
// applies bias / addend / the sub-pixel row scatter and emits the BN partials (then per
// splitk_rows_per_part() rows). Returns the rows per BN partial.
//
// Measured and rejected (round 2): an in-kernel fixup (last-arriving split of a tile sums the
// slabs) is 3-10x slower on MI355X -- cross-XCD visibility of the partials needs either a full L2
// writeback/invalidate per workgroup or write-through stores, both far costlier than one extra
// launch (docs/PERF.md).
// Split-K reductions a block's backward defers into one bwd_reduce launch (bwd_fuse.hip): the
// weight gradient's slab sum (w_*) and the data gradient's split-K reduction (d_*).
struct DeferredReduce {
  at::Tensor w_slab;
  float* w_dst = nullptr;
  int w_S = 0;
  long long w_n = 0;
  at::Tensor d_slab;
  const float* d_src = nullptr;  // d_slab's data, or (d_S == 1) the finished dX read back in place
  float* d_y = nullptr;
  const float* d_addend = nullptr;
  int d_S = 0, d_M = 0, d_Nout = 0;
  bool d_on = false;
};

// A weight-gradient GEMM held back so the data-gradient GEMM of the same block can run beside it in
// one launch (bwd_pair.hip); `after` is the work that must follow it (its slab reduction), if any.
struct PendingWgrad {
  bool set = false;
  WgradParams p{};
  int bm = 0, bn = 0;
  std::function<void()> after;
  // owners of every buffer p points into (dy / x may be channels_last copies and their |max|
  // partials measured in wgrad_impl): without them the caching allocator could hand a freed block
  // to dX before the held launch reads it
  std::vector<at::Tensor> keep;
  void run_after() {
    set = false;
    if (after) after();
    after = nullptr;
    keep.clear();
  }
  // launch it alone (no data-gradient GEMM took it)
  void flush(hipStream_t st) {
    if (!set) return;
    wgrad_launch_logged(p, bm, bn, true, st, 2);
    run_after();
  }
};

// CDP_BWD_PAIR=0: the two gradient GEMMs of a block as two launches
bool bwd_pair_enabled() {
  const char* e = std::getenv("CDP_BWD_PAIR");
  return !(e && e[0] == '0');
}

bool bwd_fuse_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CDP_BWD_FUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// alloc_part(rows_per_part), when given, returns the BN partial buffer for that layout.
// defer, when given, takes over a plain split-K reduction (no bias / BN partials / row scatter):
// the GEMM is enqueued and the reduction left to the caller's bwd_reduce launch.
// The conv GEMM launch, or -- a pending weight gradient of the same block given and both GEMMs
// being f16x2 256x128 tiles -- both GEMMs in one bwd_pair launch.
std::atomic<long long>& pair_counter() {
  static std::atomic<long long> n{0};
  return n;
}

void conv_launch_or_pair(const ConvGemmParams& p, const GemmPlan& g, bool dgrad, hipStream_t st,
                         PendingWgrad* pending) {
  if (pending && pending->set && dgrad && f16x2_mode() && x3_ok(p, true) && p.a_img && p.b_row &&
      bwd_pair_ok(p, g.bm, g.bn, pending->p, pending->bm, pending->bn, split_planes())) {
    gemm_log_add("pair_dgrad", p.M, p.Nout, p.Kdim, g.bm, g.bn, p.splits);
    gemm_log_add("pair_wgrad", pending->p.Cout, pending->p.Kdim, (long long)pending->p.M, pending->bm, pending->bn,
                 pending->p.splits);
    ConvGemmParams q = p;
    q.narrow = narrow_stores();
    bwd_pair_launch(q, g.bm, g.bn, pending->p, pending->bm, pending->bn, st);
    pair_counter().fetch_add(1, std::memory_order_relaxed);
    pending->run_after();
    return;
  }
  conv_launch(p, g.bm, g.bn, dgrad, st);
}

int conv_gemm_splitk(ConvGemmParams p, const GemmPlan& g, bool dgrad, hipStream_t st, at::TensorOptions opts,
                     std::vector<at::Tensor>& keep, const std::function<float*(int)>& alloc_part = nullptr,
                     DeferredReduce* defer = nullptr, PendingWgrad* pending = nullptr) {
  p.splits = g.splits;
  if (g.splits == 1) {
    if (alloc_part) p.part = alloc_part(g.bm);
    conv_launch_or_pair(p, g, dgrad, st, pending);
    if (defer && !alloc_part && !p.part && !p.bias && !p.rr.on && !p.addend && (p.Nout % 4) == 0) {
      // no split-K slab, but the block's bwd_reduce launch still runs the previous block's BN
      // statistics pass over dX (one "slab": dX itself, rewritten unchanged; the addend is already in)
      defer->d_on = true;
      defer->d_src = p.y;
      defer->d_y = p.y;
      defer->d_addend = nullptr;
      defer->d_S = 1;
      defer->d_M = p.M;
      defer->d_Nout = p.Nout;
    }
    return g.bm;
  }
  at::Tensor slab = at::empty({g.splits, (long long)p.M, p.Nout}, opts);
  keep.push_back(slab);
  if (defer && !alloc_part && !p.part && !p.bias && !p.rr.on && (p.Nout % 4) == 0) {
    defer->d_slab = slab;
    defer->d_src = slab.data_ptr<float>();
    defer->d_on = true;
    defer->d_y = p.y;
    defer->d_addend = p.addend;
    defer->d_S = g.splits;
    defer->d_M = p.M;
    defer->d_Nout = p.Nout;
    p.y = slab.data_ptr<float>();
    p.addend = nullptr;
    conv_launch_or_pair(p, g, dgrad, st, pending);
    return splitk_rows_per_part();
  }
  float* y = p.y;
  const float* bias = p.bias;
  const float* addend = p.addend;
  float* part = alloc_part ? alloc_part(splitk_rows_per_part()) : p.part;
  RowRemap rr = p.rr;
  p.y = slab.data_ptr<float>();
  p.bias = nullptr;
  p.addend = nullptr;
  p.part = nullptr;
  p.rr.on = 0;  // slabs are class-local; the reduction scatters
  conv_launch_or_pair(p, g, dgrad, st, pending);
  splitk_reduce_launch(slab.data_ptr<float>(), g.splits, p.M, p.Nout, bias, y, part, st, rr.on ? &rr : nullptr,
                       addend);
  return splitk_rows_per_part();
}

// Workgroups each kernel keeps resident per CU (min of the LDS and VGPR limits of the build).
int conv_blocks_per_cu(int bm, int bn) {
  if (f16x2_mode()) return (bm + bn) >= 384 ? 1 : (bm + bn) >= 256 ? 2 : 3;  // 2 x 2 x (bm+bn) x 64 B
  if (x3_family()) return (bm + bn) >= 256 ? 1 : (bm + bn) >= 192 ? 2 : 3;  // 2 x 3 x (bm+bn) x 64 B
  return std::max(1, std::min(4, (160 * 1024) / (2 * (bm + bn) * 36 * 4)));
}
// Split-K cost model constants (MFMA rate per engine, fp32-equivalent; slab round-trip bandwidth).
// Round 2 swept the rate x0.6-x1.6 and the slab bandwidth 2-8 TB/s: every VGG-11 layer's plan and
// the step stayed within +-2 % (docs/PERF.md), so they are fixed.
double conv_mfma_rate() {
  const int m = conv_gemm_mode();
  return m == 1 ? 250.0e12 : m == 2 ? 800.0e12 : m == 3 ? 450.0e12 : 120.0e12;
}
double slab_bw() { return 4.0e12; }
int wgrad_blocks_per_cu(int bm, int bn) {
  // f16x2 (two-stage pipeline): 2 stages x 2 planes x (bm+bn) x 80 B of LDS, 214 / 153 / 110 VGPRs
  // (128x128 / 128x64 / 64x64)
  if (f16x2_mode()) return bm >= 256 ? 1 : (bm + bn) >= 192 ? 2 : 3;
  if (x3_family()) return (bm + bn) >= 256 ? 2 : (bm + bn) >= 192 ? 3 : 5;
  return std::max(1, std::min(4, (160 * 1024) / (2 * 32 * (bm + bn + 8) * 4)));
}

// Split-K factor that best fills whole waves of resident workgroups: a grid just over one wave
// (e.g. 540 blocks on 512 slots) costs almost two waves of time, so quantisation dominates.
int choose_splits(long long tiles, int ktiles, int slots, int min_kt, double flops, double slab_bytes_per_split,
                  double rate = 120.0e12) {
  if (tiles >= slots) return 1;
  const int smax = std::max(1, ktiles / std::max(1, min_kt));
  // modelled time: MFMA work at `rate` scaled by wave-quantisation efficiency, plus the fp32
  // split-K slab round trip (write + read) at ~4 TB/s
  auto cost = [&](int s) {
    const long long blocks = tiles * s;
    const long long waves = (blocks + slots - 1) / slots;
    const double eff = (double)blocks / (double)(waves * slots);
    const double slab = s > 1 ? 2.0 * s * slab_bytes_per_split / slab_bw() : 0.0;
    return flops / (rate * eff) + slab;
  };
  int best = 1;
  double best_t = cost(1);
  for (int w = 1; w <= 4; ++w) {
    const int s = (int)std::min<long long>(smax, (long long)w * slots / tiles);
    if (s < 1) continue;
    const double t = cost(s);
    if (t < best_t * 0.98) {
      best = s;
      best_t = t;
    }
  }
  return best;
}

// Plan override for tuning sweeps (scripts/sweep_gemm.py): when set, every conv GEMM / weight-gradient
// GEMM planned afterwards uses this tile and split count (0 = keep the planner's choice).
struct PlanOverride {
  int bm = 0, bn = 0, splits = 0;
};
PlanOverride& conv_override() {
  static PlanOverride o;
  return o;
}
PlanOverride& wgrad_override() {
  static PlanOverride o;
  return o;
}

// ---- f16x2 planner: a cost model fitted to measurements
// A tile / split-K sweep of the VGG-11 conv GEMMs (forward, data and weight gradient, each with its
// split-K reduction; 32 / 64 / 128 / 256 images per GPU; 5,240 timed configurations) on MI355X
// (scripts/sweep_gemm.py -> profiles/tuning/vgg11_gemm_sweep_r3.json) was fitted by
// scripts/fit_plan_model.py to
//   t = t0 + rounds * (a0 + kps * max(l0 + l1 (bm + bn), k bm bn / rho, k (bm + bn) / beta))
//       + [splits > 1] (r0 + r1 * splits * P * Q * 4e-6)                                    (us)
// for a P x Q output tiled bm x bn, reduction R split `splits` ways (kps K-tiles of 32 per block);
// a CU holds nb = ceil(blocks / CUs) blocks, k = min(nb, residency) at a time, in rounds of the
// residency. The three per-K-tile terms are a latency floor, the CU's MAC rate and its operand-load
// rate, the last two shared by co-resident blocks. The planner takes the modelled argmin over every
// tile and split count; its choices come within 3.4 % (conv) / 1.1 % (weight gradient) of the
// measured best over the sweep, against 13 % for the previous heuristic (which preferred 256x128
// tiles with up to 16 splits everywhere: 2x slower at 32 images per GPU on the deep layers).
struct GemmCostModel {
  double t0, a0, l0, l1, rho, beta, r0, r1;
};
constexpr GemmCostModel kConvCost{9.934, 3.163e-06, 1.698e-07, 0.002637, 3.041e4, 558.2, 0.05613, 0.3461};
constexpr GemmCostModel kWgradCost{8.188, 1.54e-05, 0.1129, 0.003117, 2.541e4, 367.8, 2.707, 0.345};

double model_time(const GemmCostModel& m, int residency, long long P, long long Q, long long R, int bm, int bn,
                  int s) {
  const long long tiles = ((P + bm - 1) / bm) * ((Q + bn - 1) / bn);
  const long long blocks = tiles * s;
  const long long kt = (R + 31) / 32, kps = (kt + s - 1) / s;
  const long long nb = (blocks + num_cus() - 1) / num_cus();
  const long long k = std::min<long long>(nb, residency);
  const long long rounds = (nb + residency - 1) / residency;
  const double per = m.a0 + (double)kps * std::max({m.l0 + m.l1 * (bm + bn), (double)(k * bm * bn) / m.rho,
                                                     (double)(k * (bm + bn)) / m.beta});
  return m.t0 + (double)rounds * per + (s > 1 ? m.r0 + m.r1 * (double)s * (double)P * (double)Q * 4e-6 : 0.0);
}

// The model decides only where it predicts a clear gain over the previous heuristic's plan (which was
// tuned in the full training step at 256 images per GPU, where its 256x128 tiles also pair the two
// gradient GEMMs of a block in one launch): its plan must model at most gain x the heuristic's time,
// gain = 0.95 for GEMMs under 3.2 GFLOP (the model is accurate there: few blocks, latency-bound) and
// 0.85 above (it overrates 128x128 tiles at large M; its log-space fit is dominated by the many
// small configurations). Measured in the bench step, VGG-11 ms/step at 32 / 64 / 128 / 256 images
// per GPU: heuristic 0.638 / 0.757 / 0.970 / 1.409 (one box); model everywhere 0.551 / 0.698 /
// 0.985 / 1.454 (same box); a single threshold of 0.95 / 0.87 / 0.80 (another box):
// 0.552 / 0.731 / 0.981 / 1.377, 0.588 / 0.733 / 0.967 / 1.366, 0.616 / 0.743 / 0.987 / 1.363.
double model_gain(double flops) { return flops < 3.2e9 ? 0.95 : 0.85; }

bool model_planner_on() { return f16x2_mode(); }

struct PlanKey {
  int kind, mode;
  long long a, b, c;
  bool operator==(const PlanKey& o) const {
    return kind == o.kind && mode == o.mode && a == o.a && b == o.b && c == o.c;
  }
};
struct PlanKeyHash {
  size_t operator()(const PlanKey& k) const {
    size_t h = std::hash<long long>()(k.a) * 1000003u ^ std::hash<long long>()(k.b) * 10007u ^
               std::hash<long long>()(k.c) * 101u;
    return h ^ (size_t)(k.kind * 31 + k.mode);
  }
};

// argmin of the model over the f16x2 tiles and split counts (each block keeps >= 2 K-tiles);
// returns {bm, bn, splits}
std::array<int, 3> model_plan(bool wgrad, long long P, long long Q, long long R) {
  static std::unordered_map<PlanKey, std::array<int, 3>, PlanKeyHash> cache;
  static std::mutex mu;
  const PlanKey key{wgrad ? 1 : 0, conv_gemm_mode(), P, Q, R};
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  static const int tiles[5][2] = {{256, 128}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
  const long long kt = (R + 31) / 32;
  const int smax = (int)std::max<long long>(1, std::min<long long>(wgrad ? 1024 : 64, kt / 2));
  std::array<int, 3> best{128, 64, 1};
  double best_t = 1e30;
  for (const auto& t : tiles) {
    const int bm = t[0], bn = t[1];
    if (bm == 256 && wgrad && (Q % 128) != 0) continue;  // 256-row weight-gradient tiles: 128-wide k only
    const int res = wgrad ? wgrad_blocks_per_cu(bm, bn) : conv_blocks_per_cu(bm, bn);
    for (int s = 1; s <= smax; ++s) {
      const double tm = model_time(wgrad ? kWgradCost : kConvCost, res, P, Q, R, bm, bn, s);
      if (tm < best_t) {
        best_t = tm;
        best = {bm, bn, s};
      }
    }
  }
  std::lock_guard<std::mutex> g(mu);
  cache[key] = best;
  return best;
}

// Plans measured inside the training block where they beat the fitted model's plan: the data- and
// weight-gradient GEMMs timed together in their paired launch (one grid: its wave quantisation and
// CU residency are shared, so the best pair is not the pair of the best single launches), the
// forward with its split-K reduction and BN pass (scripts/sweep_pair.py, hipGraph-timed,
// profiles/tuning/). kind: 0 forward, 1 data gradient, 2 weight gradient; mode: conv_gemm_mode().
struct TunedPlan {
  int kind, mode;
  long long M;
  int N, K, bm, bn, splits;
};
const std::vector<TunedPlan>& tuned_plans() {
  // {kind, mode, M, N, K, bm, bn, splits}: VGG-11 blocks at the reference's strong-scaling batches
  // (32 / 64 / 128 images per GPU) and the headline batch (256); block time planner -> tuned (us,
  // medians of alternating re-timings, scripts/sweep_pair.py, profiles/tuning/vgg11_pair_sweep_r4.md)
  static const std::vector<TunedPlan> t = {
      // 32 images, block 1 (64->128 @16): 76.9 -> 74.7; re-swept on the round-6 tree 80.6 -> 78.4
      // (profiles/tuning/vgg11_pair_sweep_r6.md)
      {1, 3, 8192, 64, 1152, 64, 64, 1},
      {2, 3, 8192, 128, 576, 128, 64, 12},
      // 32 images, block 2 (128->256 @8): 77.3 -> 75.7 (scripts/verify_plans.py, 5 alternations)
      {1, 3, 2048, 128, 2304, 64, 64, 4},
      {2, 3, 2048, 256, 1152, 128, 64, 6},
      // 32 images, block 3 (256->256 @8): backward 98.5 -> 93.2, forward 37.6 -> 36.0
      {1, 3, 2048, 256, 2304, 64, 128, 4},
      {2, 3, 2048, 256, 2304, 128, 128, 6},
      {0, 3, 2048, 256, 2304, 64, 128, 8},
      // 32 images, block 4 (256->512 @4): 77.7 -> 72.3
      {1, 3, 512, 256, 4608, 64, 64, 6},
      // 32 images, block 5 (512->512 @4): 98.3 -> 89.9
      {1, 3, 512, 512, 4608, 128, 128, 6},
      // 32 images, blocks 6-7 (512->512 @2): 64.9 -> 62.9
      {1, 3, 128, 512, 4608, 64, 128, 12},
      // 128 images, block 1 (64->128 @16): backward 143.9 -> 128.7, forward 49.4 -> 47.9
      {1, 3, 32768, 64, 1152, 128, 64, 1},
      {2, 3, 32768, 128, 576, 128, 64, 24},
      {0, 3, 32768, 128, 576, 128, 64, 1},
      // 128 images, block 2 (128->256 @8): 133.7 -> 125.2
      {1, 3, 8192, 128, 2304, 256, 128, 3},
      {2, 3, 8192, 256, 1152, 256, 128, 12},
      // 128 images, block 4 (256->512 @4): 127.7 -> 117.0
      {1, 3, 2048, 256, 4608, 256, 128, 6},
      {2, 3, 2048, 512, 2304, 256, 128, 4},
      // 128 images, blocks 6-7 forward (512->512 @2): 35.7 -> 34.7
      {0, 3, 512, 512, 4608, 64, 128, 8},
      // 64 images, block 1: backward 100.9 -> 92.1
      {1, 3, 16384, 64, 1152, 64, 64, 1},
      {2, 3, 16384, 128, 576, 128, 64, 24},
      // 64 images, block 2: backward 101.7 -> 95.7, forward 40.5 -> 35.0
      {1, 3, 4096, 128, 2304, 64, 128, 3},
      {2, 3, 4096, 256, 1152, 128, 128, 12},
      {0, 3, 4096, 256, 1152, 64, 64, 1},
      // 64 images, block 3: backward 124.8 -> 115.2
      {1, 3, 4096, 256, 2304, 256, 128, 3},
      {2, 3, 4096, 256, 2304, 256, 128, 8},
      // 64 images, block 4: backward 99.5 -> 92.7, forward 35.9 -> 34.5
      {1, 3, 1024, 256, 4608, 64, 128, 6},
      {2, 3, 1024, 512, 2304, 64, 64, 1},
      {0, 3, 1024, 512, 2304, 64, 128, 4},
      // 64 images, blocks 6-7: backward 78.0 -> 72.2, forward 30.3 -> 29.6
      {1, 3, 256, 512, 4608, 64, 128, 6},
      {0, 3, 256, 512, 4608, 64, 128, 16},
      // ResNet-50, 64 images at 224x224 (scripts/sweep_resnet.py, per GEMM, >= 4 % faster):
      // forward 256->512 1x1/2 @56 82.9 -> 76.6, 256->128 1x1 @56 94.1 -> 87.5, 128->512 1x1 @28
      // 61.7 -> 57.2, 1024->256 1x1 @14 37.8 -> 35.8, 64->64 1x1 @56 28.1 -> 26.9
      {0, 3, 50176, 512, 256, 128, 128, 1},
      {0, 3, 200704, 128, 256, 128, 128, 1},
      {0, 3, 50176, 512, 128, 64, 128, 1},
      {0, 3, 12544, 256, 1024, 64, 128, 1},
      {0, 3, 200704, 64, 64, 64, 64, 1},
      // round 6, after the LDS-staged 16-B epilogue stores: forward 64->256 1x1 @56 83.1 -> 73.5,
      // data gradients 64->64 1x1 @56 22.6 -> 21.4 and 64->256 1x1 @56 45.6 -> 44.5
      {0, 3, 200704, 256, 64, 128, 128, 1},
      {1, 3, 200704, 64, 64, 64, 64, 1},
      {1, 3, 200704, 64, 256, 64, 64, 1},
      // data gradients of 256->64 @56 70.4 -> 65.9, 256->128 @56 111.7 -> 105.4, 512->128 @28
      // 54.8 -> 48.9, 512->256 @28 77.5 -> 69.5, 256->1024 @14 36.7 -> 34.2 (all 1x1)
      {1, 3, 200704, 256, 64, 128, 128, 1},
      {1, 3, 200704, 256, 128, 128, 128, 1},
      {1, 3, 50176, 512, 128, 64, 128, 1},
      {1, 3, 50176, 512, 256, 128, 128, 1},
      {1, 3, 12544, 256, 1024, 64, 128, 1},
      // weight gradient of 512->128 1x1 @28: 42.5 -> 39.3
      {2, 3, 50176, 128, 512, 128, 128, 64},
      // 256 images, blocks 2 and 3: data gradient over 2 / 1 splits (190.6 -> 186.8, 266.6 -> 260.9)
      {1, 3, 16384, 128, 2304, 256, 128, 2},
      {1, 3, 16384, 256, 2304, 256, 128, 1},
      // 256 images, block 4 (256->512 @4): 173.4 -> 166.7
      {1, 3, 4096, 256, 4608, 256, 128, 3},
      {2, 3, 4096, 512, 2304, 256, 128, 4},
      // 256 images, blocks 6-7 (512->512 @2): 122.2 -> 111.4, 120.8 -> 110.4
      {1, 3, 1024, 512, 4608, 256, 128, 6},
      {2, 3, 1024, 512, 4608, 256, 128, 2},
  };
  return t;
}
bool tuned_off() {
  static const bool off = [] {
    const char* e = std::getenv("CDP_TUNED_PLANS");
    return e && e[0] == '0';
  }();
  return off;
}
const TunedPlan* tuned_plan(int kind, long long M, int N, int K) {
  if (tuned_off()) return nullptr;
  const int mode = conv_gemm_mode();
  for (const auto& t : tuned_plans())
    if (t.kind == kind && t.mode == mode && t.M == M && t.N == N && t.K == K) return &t;
  return nullptr;
}

GemmPlan plan_gemm(long long M, int Nout, int Kdim, int kind = 0) {
  GemmPlan g;
  g.ktiles = (Kdim + 31) / 32;
  g.bn = (Nout % 128 == 0) ? 128 : 64;
  const int target = 2 * num_cus();
  long long tiles128 = ((M + 127) / 128) * ((Nout + g.bn - 1) / g.bn);
  g.bm = (tiles128 >= target || M > 4096) ? 128 : 64;
  // x3 engine: 8-wave 256x128 tiles (two waves per SIMD next to the software pipeline); measured
  // on VGG-11 B=256 they beat 128x128 / 64x128 on every layer, split-K making up the grid
  // (127.5k vs 124.5k img/s with 256 only for M >= 8192)
  if (x3_family() && g.bn == 128) g.bm = 256;
  const long long tiles = ((M + g.bm - 1) / g.bm) * ((Nout + g.bn - 1) / g.bn);
  const int slots = conv_blocks_per_cu(g.bm, g.bn) * num_cus();
  g.splits = std::min(16, choose_splits(tiles, g.ktiles, slots, 4, 2.0 * M * Nout * Kdim, 4.0 * M * Nout,
                                        conv_mfma_rate()));
  if (model_planner_on()) {
    const auto m = model_plan(false, M, Nout, Kdim);
    const double t_model = model_time(kConvCost, conv_blocks_per_cu(m[0], m[1]), M, Nout, Kdim, m[0], m[1], m[2]);
    const double t_heur = model_time(kConvCost, conv_blocks_per_cu(g.bm, g.bn), M, Nout, Kdim, g.bm, g.bn, g.splits);
    if (t_model <= model_gain(2.0 * M * Nout * Kdim) * t_heur) {
      g.bm = m[0];
      g.bn = m[1];
      g.splits = m[2];
    }
  }
  if (const TunedPlan* t = tuned_plan(kind, M, Nout, Kdim)) {
    g.bm = t->bm;
    g.bn = t->bn;
    g.splits = std::max(1, std::min(t->splits, g.ktiles));
  }
  const PlanOverride& o = conv_override();
  if (o.bm) g.bm = o.bm;
  if (o.bn) g.bn = o.bn;
  if (o.splits) g.splits = std::max(1, std::min(o.splits, g.ktiles));
  if (g.bm == 256 && !x3_family()) g.bm = 128;
  if (g.bm == 256) g.bn = 128;  // the only 256-row conv tile (dispatch_x3)
  return g;
}

struct WgradPlan {
  int bm, bn, splits;
};

WgradPlan plan_wgrad(int Cout, int Kdim, long long M) {
  WgradPlan w;
  w.bm = Cout >= 128 ? 128 : 64;
  // 128-wide k tiles also when Kdim is an odd multiple of 64 and >= 512 (e.g. 576 = 9 x 64: 4.5
  // tiles, the last one half padding). Measured on VGG-11 layer 1 (B=256): 70.7 -> 61.9 us.
  w.bn = (Kdim % 128 == 0 || Kdim >= 512) ? 128 : 64;
  // 256x128 f16x2 tiles, 8 waves, one workgroup per CU. Measured on MI355X, VGG-11 B=256:
  // 156.0k -> 161.7k img/s (the x gather and split are shared by four co waves instead of two)
  if (f16x2_mode() && Cout >= 256 && Cout % 4 == 0 && w.bn == 128) w.bm = 256;
  const long long tiles = (long long)((Cout + w.bm - 1) / w.bm) * ((Kdim + w.bn - 1) / w.bn);
  const int mt = (int)std::min<long long>((M + 31) / 32, 1 << 30);
  const int slots = wgrad_blocks_per_cu(w.bm, w.bn) * num_cus();
  w.splits = std::min(1024, choose_splits(tiles, mt, slots, 4, 2.0 * M * Cout * Kdim, 4.0 * Cout * Kdim,
                                          conv_mfma_rate()));
  if (model_planner_on() && (Cout % 4) == 0) {
    const auto m = model_plan(true, Cout, Kdim, M);
    const double t_model = model_time(kWgradCost, wgrad_blocks_per_cu(m[0], m[1]), Cout, Kdim, M, m[0], m[1], m[2]);
    const double t_heur = model_time(kWgradCost, wgrad_blocks_per_cu(w.bm, w.bn), Cout, Kdim, M, w.bm, w.bn, w.splits);
    if (t_model <= model_gain(2.0 * M * Cout * Kdim) * t_heur) {
      w.bm = m[0];
      w.bn = m[1];
      w.splits = m[2];
    }
  }
  if (const TunedPlan* t = tuned_plan(2, M, Cout, Kdim)) {
    w.bm = t->bm;
    w.bn = t->bn;
    w.splits = std::max(1, std::min(t->splits, mt));
  }
  const PlanOverride& o = wgrad_override();
  if (o.bm) w.bm = o.bm;
  if (o.bn) w.bn = o.bn;
  if (o.splits) w.splits = std::max(1, std::min(o.splits, mt));
  if (w.bm == 256 && !(f16x2_mode() && w.bn == 128 && Cout % 4 == 0)) w.bm = 128;  // 256 rows: f16x2 256x128 only
  return w;
}

template <class P>
void set_divs(P& p) {
  p.fd_PQ = make_fastdiv(p.P * p.Q);
  p.fd_Q = make_fastdiv(p.Q);
  p.fd_C = make_fastdiv(p.C);
  p.fd_KW = make_fastdiv(p.KW);
}

// Zero-pad the channel dim of a channels_last 4-D tensor up to a multiple of 4 (RGB stems:
// 3 -> 4) so the float4 gather paths apply. C < 4 is one kernel that can also emit the padded
// tensor's act max (f16x2 operand scales) into *amax.
at::Tensor pad_channels4(const at::Tensor& t, at::Tensor* amax = nullptr) {
  const int64_t C = t.size(1), C4 = (C + 3) / 4 * 4;
  at::Tensor o = at::empty({t.size(0), C4, t.size(2), t.size(3)}, t.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (C < 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast)) {
    hipStream_t st = cur_stream();
    ActMaxOut am{nullptr, nullptr};
    if (amax) {
      *amax = new_act_max(t.size(0), 4, t, st);
      am = act_out(*amax, t.size(0));
    }
    pad_c4_launch(t.data_ptr<float>(), (int)t.size(0), t.size(2) * t.size(3), (int)C, o.data_ptr<float>(), am, st);
    return o;
  }
  o.zero_();
  o.narrow(1, 0, C).copy_(t);
  return o;
}

}  // namespace

// paired gradient launches (bwd_pair) issued by this process so far (tests check the pair is taken)
int64_t pair_launches() { return pair_counter().load(std::memory_order_relaxed); }

void set_gemm_override(const std::string& kind, int64_t bm, int64_t bn, int64_t splits) {
  TORCH_CHECK(kind == "conv" || kind == "wgrad", "set_gemm_override: kind must be 'conv' or 'wgrad'");
  TORCH_CHECK(bm == 0 || bm == 64 || bm == 128 || bm == 256, "bm must be 0, 64, 128 or 256");
  TORCH_CHECK(bn == 0 || bn == 64 || bn == 128, "bn must be 0, 64 or 128");
  TORCH_CHECK(bm != 256 || bn == 128, "256-row tiles are 256x128");
  PlanOverride& o = kind == "conv" ? conv_override() : wgrad_override();
  o.bm = (int)bm;
  o.bn = (int)bn;
  o.splits = (int)splits;
}

std::vector<int64_t> plan_info(const std::string& kind, int64_t M, int64_t N, int64_t K) {
  if (kind == "conv" || kind == "dgrad") {
    const GemmPlan g = plan_gemm(M, (int)N, (int)K, kind == "dgrad" ? 1 : 0);
    return {g.bm, g.bn, g.splits};
  }
  TORCH_CHECK(kind == "wgrad", "plan_info: kind must be 'conv', 'dgrad' or 'wgrad'");
  const WgradPlan w = plan_wgrad((int)N, (int)K, M);  // N = Cout, K = Kdim, M = reduction rows
  return {w.bm, w.bn, w.splits};
}

void set_conv_gemm(const std::string& mode) {
  TORCH_CHECK(mode == "x3" || mode == "f32" || mode == "bf16" || mode == "f16x2",
              "conv gemm engine must be 'x3', 'f16x2', 'f32' or 'bf16', got ", mode);
  conv_gemm_mode() = mode == "x3" ? 1 : mode == "bf16" ? 2 : mode == "f16x2" ? 3 : 0;
}
std::string get_conv_gemm() {
  const int m = conv_gemm_mode();
  return m == 1 ? "x3" : m == 2 ? "bf16" : m == 3 ? "f16x2" : "f32";
}

// ---------------------------------------------------------------- conv forward
// Returns y (channels_last [N, Cout, P, Q]). When `part` is requested the per-tile BatchNorm
// partials are returned in a second tensor [nparts, Cout, 2] together with rows-per-part.
std::vector<at::Tensor> conv2d_fwd(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& bias,
                                   int64_t stride, int64_t pad, bool want_stats, const c10::optional<at::Tensor>& x_amax,
                                   const c10::optional<at::Tensor>& w_amax) {
  check_f32_cuda(x_, "x");
  check_f32_cuda(w_, "weight");
  TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4, "conv2d_fwd expects 4-D input and weight");
  const at::Tensor x = nhwc(x_);
  const at::Tensor w = nhwc(w_);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Co = w.size(0), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(w.size(1) == C, "weight in-channels mismatch: ", w.size(1), " vs ", C);
  const int P = (H + 2 * pad - KH) / stride + 1;
  const int Q = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty conv output");
  const long long M = (long long)N * P * Q;
  TORCH_CHECK(M < (1LL << 31), "conv rows overflow int32");
  const int Kdim = KH * KW * C;
  auto opts = x.options();
  at::Tensor y = at::empty({N, Co, P, Q}, opts.memory_format(at::MemoryFormat::ChannelsLast));
  GemmPlan g = plan_gemm(M, Co, Kdim);
  ConvGemmParams p{};
  p.x = x.data_ptr<float>();
  p.w = w.data_ptr<float>();
  p.N = N; p.H = H; p.W = W; p.C = C; p.P = P; p.Q = Q;
  p.KH = KH; p.KW = KW; p.stride = (int)stride; p.pad = (int)pad;
  p.Nout = Co; p.M = (int)M; p.Kdim = Kdim; p.ktiles = g.ktiles; p.splits = g.splits;
  set_divs(p);
  at::Tensor part, rpp;
  hipStream_t st = cur_stream();
  const at::Tensor xa = act_max(x, x_amax, st), wa = weight_max(w, w_amax);
  set_scales(p, xa, wa, false, Co, C);
  p.y = y.data_ptr<float>();
  p.bias = fptr(bias);
  // BN partials: one per BM-row tile (splits == 1) or per reduction row block (split-K)
  std::function<float*(int)> alloc_part;
  if (want_stats)
    alloc_part = [&](int rows_pp) {
      part = at::empty({(M + rows_pp - 1) / rows_pp, Co, 2}, opts);
      return part.data_ptr<float>();
    };
  std::vector<at::Tensor> keep;
  const int rb = conv_gemm_splitk(p, g, false, st, opts, keep, alloc_part);
  if (want_stats) rpp = at::full({1}, rb, opts.dtype(at::kInt).device(at::kCPU));
  if (want_stats) return {y, part, rpp};
  return {y};
}

// CDP_SUBPIXEL_ZERO=0: the tap-less sub-pixel classes as K-less GEMM launches (A/B)
static bool subpixel_zero_enabled() {
  const char* e = std::getenv("CDP_SUBPIXEL_ZERO");
  return !(e && e[0] == '0');
}

// ---------------------------------------------------------------- conv data gradient
// Stride-2 data gradient by sub-pixel decomposition: the input pixels of parity class (ph, pw)
// receive gradient only from the filter taps kh = kh0 + 2a, kw = kw0 + 2b, kh0 = (ph + pad) % 2,
// through dY[(ih + pad - kh) / 2]. Each class is therefore a dense stride-1 correlation of dY with
// a quarter-size sub-filter over a quarter of the rows: 4 GEMMs doing 1/4 of the work of the
// masked full-resolution gather (which spends 3/4 of its MACs on taps that cannot contribute).
// Classes without taps (e.g. the odd pixels of a 1x1 stride-2 conv: three of the four) receive no
// gradient: with an addend, dX is the addend itself (accumulated in place) and those pixels are
// already final; without one, a single fill pass writes their zeros (subpixel_zero_launch: one
// bandwidth-bound launch instead of three K-less GEMM launches, whose epilogues wrote at ~2 TB/s).
// Returns false when a shape is outside the x3 kernels' addressing limits.
bool conv2d_dgrad_subpixel(const at::Tensor& dy, const at::Tensor& w, at::Tensor& dx, int pad, hipStream_t st,
                           const float* addend, const at::Tensor& dya, const at::Tensor& wa) {
  const int N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  const int Co = w.size(0), KH = w.size(2), KW = w.size(3);
  const int P = dy.size(2), Q = dy.size(3);
  if (Co % 32 != 0) return false;
  std::vector<at::Tensor> keep;  // sub-filters / slabs stay alive until the launches are enqueued
  // pass 1: every class within the kernels' addressing limits (decided before any launch)
  int empty_mask = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      const int Hc = (H - ph + 1) / 2, Wc = (W - pw + 1) / 2;
      if (Hc <= 0 || Wc <= 0) continue;
      const int kh0 = (ph + pad) % 2, kw0 = (pw + pad) % 2;
      const int nkh = kh0 < KH ? (KH - kh0 + 1) / 2 : 0, nkw = kw0 < KW ? (KW - kw0 + 1) / 2 : 0;
      if (nkh * nkw == 0) empty_mask |= 1 << (2 * ph + pw);
    }
  if (empty_mask && !addend && (C % 4) == 0 && !subpixel_zero_enabled()) empty_mask = 0;
  if (empty_mask && (addend || (C % 4) == 0)) {
    if (!addend) subpixel_zero_launch(dx.data_ptr<float>(), N, H, W, C, empty_mask, st);
  } else {
    empty_mask = 0;  // (C % 4 != 0 without an addend: the K-less GEMM launches write the zeros)
  }
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      const int Hc = (H - ph + 1) / 2, Wc = (W - pw + 1) / 2;
      if (Hc <= 0 || Wc <= 0) continue;
      const int kh0 = (ph + pad) % 2, kw0 = (pw + pad) % 2;
      const int nkh = kh0 < KH ? (KH - kh0 + 1) / 2 : 0, nkw = kw0 < KW ? (KW - kw0 + 1) / 2 : 0;
      const long long Mc = (long long)N * Hc * Wc;
      const int Kc = nkh * nkw * Co;
      if (Kc == 0 && (empty_mask >> (2 * ph + pw) & 1)) continue;  // written above / already the addend
      ConvGemmParams p{};
      p.N = N; p.H = P; p.W = Q; p.C = Co; p.P = Hc; p.Q = Wc;
      p.KH = std::max(nkh, 1); p.KW = std::max(nkw, 1); p.stride = 1;
      p.pad = (ph + pad - kh0) / 2;  // oh = i + pad - a
      p.pad_w = (pw + pad - kw0) / 2;
      p.Nout = C; p.M = (int)Mc; p.Kdim = Kc;
      set_divs(p);
      p.rr = RowRemap{1, H, W, ph, pw, Hc, Wc, make_fastdiv(Hc * Wc), make_fastdiv(Wc)};
      p.x = dy.data_ptr<float>();
      // rows (n, i, j) keep dY's image n; a sub-filter's per-ci |max| is bounded by the whole filter's
      set_scales(p, dya, wa, true, Co, C);
      if (!x3_ok(p, true)) return false;
      at::Tensor wt;
      if (Kc > 0) {
        wt = at::empty({C, Kc}, dy.options());
        wtrans_sub_launch(w.data_ptr<float>(), wt.data_ptr<float>(), Co, KH, KW, C, kh0, kw0, nkh, nkw, st);
        keep.push_back(wt);
        p.w = wt.data_ptr<float>();
      } else {
        p.w = w.data_ptr<float>();  // never read: no K-tiles
      }
      GemmPlan g = plan_gemm(Mc, C, std::max(Kc, 32), 1);
      p.ktiles = (Kc + 31) / 32;
      if (Kc == 0) g.splits = 1;
      p.y = dx.data_ptr<float>();
      p.addend = addend;
      conv_gemm_splitk(p, g, true, st, dy.options(), keep);
    }
  return true;
}

// dX[N, C, H, W] from dY[N, Co, P, Q] and W[Co, C, KH, KW] (any stride / padding).
at::Tensor dgrad_impl(const at::Tensor& dy_, const at::Tensor& w_, std::vector<int64_t> in_shape, int64_t stride,
                      int64_t pad, const c10::optional<at::Tensor>& addend, const c10::optional<at::Tensor>& dy_amax,
                      const c10::optional<at::Tensor>& w_amax, const c10::optional<at::Tensor>& w_t,
                      DeferredReduce* defer, PendingWgrad* pending = nullptr) {
  check_f32_cuda(dy_, "grad_output");
  check_f32_cuda(w_, "weight");
  const at::Tensor dy = nhwc(dy_);
  const at::Tensor w = nhwc(w_);
  const int N = in_shape[0], C = in_shape[1], H = in_shape[2], W = in_shape[3];
  const int Co = w.size(0), KH = w.size(2), KW = w.size(3);
  const int P = dy.size(2), Q = dy.size(3);
  TORCH_CHECK(dy.size(1) == Co && dy.size(0) == N, "dgrad shape mismatch");
  auto opts = dy.options();
  hipStream_t st = cur_stream();
  // dx = dgrad (+ addend, accumulated in the GEMM epilogue and written over the addend in place)
  const bool has_add = addend.has_value() && addend->defined();
  if (has_add)
    TORCH_CHECK(addend->scalar_type() == at::kFloat && addend->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    addend->size(0) == N && addend->size(1) == C && addend->size(2) == H && addend->size(3) == W,
                "dgrad addend must be a channels_last fp32 tensor of the input's shape");
  const float* addp = has_add ? addend->data_ptr<float>() : nullptr;
  const at::Tensor dya = act_max(dy, dy_amax, st), wa = weight_max(w, w_amax);  // W^T rows: W's per-ci maxima
  if (stride == 2 && x3_family()) {
    at::Tensor dx = has_add ? *addend : at::empty({N, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast));
    if (conv2d_dgrad_subpixel(dy, w, dx, (int)pad, st, addp, dya, wa)) return dx;
  }
  // Wt[ci][tap][co] = W[co][tap][ci]: from the step's weight_prep when given, else transposed here
  at::Tensor wt;
  if (w_t.has_value() && w_t->defined()) {
    wt = *w_t;
    TORCH_CHECK(wt.is_contiguous() && wt.numel() == (long long)C * KH * KW * Co, "dgrad: w_t must be [Ci, KH*KW*Co]");
  } else {
    wt = at::empty({C, KH * KW * Co}, opts);
    wtrans_launch(w.data_ptr<float>(), wt.data_ptr<float>(), Co, KH * KW, C, st);
  }
  at::Tensor dx = has_add ? *addend : at::empty({N, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast));
  const long long M = (long long)N * H * W;
  const int Kdim = KH * KW * Co;
  GemmPlan g = plan_gemm(M, C, Kdim, 1);
  ConvGemmParams p{};
  p.x = dy.data_ptr<float>();
  p.w = wt.data_ptr<float>();
  p.N = N; p.H = P; p.W = Q; p.C = Co; p.P = H; p.Q = W;
  p.KH = KH; p.KW = KW; p.stride = (int)stride; p.pad = (int)pad; p.pad_w = (int)pad;
  p.Nout = C; p.M = (int)M; p.Kdim = Kdim; p.ktiles = g.ktiles; p.splits = g.splits;
  set_divs(p);
  set_scales(p, dya, wa, true, Co, C);
  p.y = dx.data_ptr<float>();
  p.addend = addp;
  std::vector<at::Tensor> keep;
  conv_gemm_splitk(p, g, true, st, opts, keep, nullptr, defer, pending);
  return dx;
}

at::Tensor conv2d_dgrad(const at::Tensor& dy, const at::Tensor& w, std::vector<int64_t> in_shape, int64_t stride,
                        int64_t pad, const c10::optional<at::Tensor>& addend, const c10::optional<at::Tensor>& dy_amax,
                        const c10::optional<at::Tensor>& w_amax, const c10::optional<at::Tensor>& w_t) {
  return dgrad_impl(dy, w, in_shape, stride, pad, addend, dy_amax, w_amax, w_t, nullptr);
}

// ---------------------------------------------------------------- conv weight gradient
// dW (channels_last [Co, C, KH, KW]); written into `out` when given (accumulating if asked).
at::Tensor conv2d_wgrad(const at::Tensor& dy_, const at::Tensor& x_, std::vector<int64_t> w_shape, int64_t stride,
                        int64_t pad, const c10::optional<at::Tensor>& out, bool accumulate,
                        const c10::optional<at::Tensor>& dy_amax, const c10::optional<at::Tensor>& x_amax) {
  return conv2d_wgrad_keep(dy_, x_, w_shape, stride, pad, out, accumulate, -1, dy_amax, x_amax);
}

// keep_c >= 0: x carries zero-padded channels; only the first keep_c input channels of dW are
// written (the strip is fused into the split-K slab reduction).
at::Tensor wgrad_impl(const at::Tensor& dy_, const at::Tensor& x_, std::vector<int64_t> w_shape, int64_t stride,
                      int64_t pad, const c10::optional<at::Tensor>& out, bool accumulate, int64_t keep_c,
                      const c10::optional<at::Tensor>& dy_amax, const c10::optional<at::Tensor>& x_amax,
                      DeferredReduce* defer, PendingWgrad* pending = nullptr) {
  check_f32_cuda(dy_, "grad_output");
  check_f32_cuda(x_, "input");
  const at::Tensor dy = nhwc(dy_);
  const at::Tensor x = nhwc(x_);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Co = w_shape[0], KH = w_shape[2], KW = w_shape[3];
  const int P = dy.size(2), Q = dy.size(3);
  const long long M = (long long)N * P * Q;
  const int Kdim = KH * KW * C;
  const int Ckeep = keep_c >= 0 ? (int)keep_c : C;
  auto opts = x.options();
  at::Tensor dw;
  if (out.has_value() && out->defined()) {
    dw = *out;
    TORCH_CHECK(dw.is_contiguous(at::MemoryFormat::ChannelsLast) && dw.numel() == (long long)Co * KH * KW * Ckeep,
                "wgrad out must be channels_last contiguous");
  } else {
    dw = at::empty({Co, Ckeep, KH, KW}, opts.memory_format(at::MemoryFormat::ChannelsLast));
    accumulate = false;
  }
  hipStream_t st = cur_stream();
  WgradParams p{};
  p.dy = dy.data_ptr<float>();
  p.x = x.data_ptr<float>();
  p.N = N; p.H = H; p.W = W; p.C = C; p.P = P; p.Q = Q;
  p.KH = KH; p.KW = KW; p.stride = (int)stride; p.pad = (int)pad;
  p.Cout = Co; p.Kdim = Kdim; p.M = (int)M;
  const WgradPlan wp = plan_wgrad(Co, Kdim, M);
  p.splits = wp.splits;
  set_divs(p);
  const at::Tensor dya = act_max(dy, dy_amax, st), xa = act_max(x, x_amax, st);
  set_scales(p, dya, xa);
  // the GEMM launch, held back in `pending` when it can run beside the block's data gradient
  const bool hold = pending && f16x2_mode() && x3_ok(p) && (C % 4) == 0 && (Co % 4) == 0 && p.dy_ch && p.x_ch;
  auto launch = [&](std::function<void()> after) {
    if (hold) {
      pending->set = true;
      pending->p = p;
      pending->bm = wp.bm;
      pending->bn = wp.bn;
      pending->after = std::move(after);
      pending->keep = {dy, x, dya, xa};
      return;
    }
    wgrad_launch_logged(p, wp.bm, wp.bn, x3_family() && x3_ok(p), st, split_planes());
    if (after) after();
  };
  if (p.splits == 1 && !accumulate && Ckeep == C) {
    p.out = dw.data_ptr<float>();
    launch(nullptr);
  } else {
    at::Tensor slab = at::empty({p.splits, Co, Kdim}, opts);
    p.out = slab.data_ptr<float>();
    const long long n = (long long)Co * Kdim;
    if (defer && !accumulate && Ckeep == C && (n % 4) == 0 &&
        (reinterpret_cast<uintptr_t>(dw.data_ptr<float>()) & 15) == 0) {
      defer->w_slab = slab;
      defer->w_dst = dw.data_ptr<float>();
      defer->w_S = p.splits;
      defer->w_n = n;
      launch(nullptr);
    } else {
      float* dst = dw.data_ptr<float>();
      const int S = p.splits;
      launch([slab, S, n, C, Ckeep, dst, accumulate, st] {
        slab_sum_strided_launch(slab.data_ptr<float>(), S, n, C, Ckeep, dst, accumulate, st);
      });
    }
  }
  return dw;
}

at::Tensor conv2d_wgrad_keep(const at::Tensor& dy, const at::Tensor& x, std::vector<int64_t> w_shape, int64_t stride,
                             int64_t pad, const c10::optional<at::Tensor>& out, bool accumulate, int64_t keep_c,
                             const c10::optional<at::Tensor>& dy_amax, const c10::optional<at::Tensor>& x_amax) {
  return wgrad_impl(dy, x, w_shape, stride, pad, out, accumulate, keep_c, dy_amax, x_amax, nullptr);
}

// ---------------------------------------------------------------- RGB stem (stem.hip)
bool stem_enabled() { return true; }
static bool bn_fin_enabled(bool bwd);

// Training-mode conv + BN + act [+ pool] of a Cin <= 4 stem; same outputs as conv_bn_act_fwd with
// x saved unpadded (xsave = x) and no f16x2 maxima for x / W (the stem kernels need none).
std::vector<at::Tensor> stem_bn_act_fwd(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& b,
                                        const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                                        const c10::optional<at::Tensor>& running_mean,
                                        const c10::optional<at::Tensor>& running_var,
                                        const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                        double eps, bool pool, bool relu) {
  check_f32_cuda(x_, "x");
  check_f32_cuda(w_, "weight");
  const at::Tensor x = nhwc(x_), w = nhwc(w_);
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  TORCH_CHECK(w.size(1) == Cin, "stem weight in-channels mismatch");
  auto opts = x.options();
  hipStream_t st = cur_stream();
  at::Tensor y = at::empty({N, Co, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast));
  const long long M = (long long)N * H * W;
  const int nparts = (int)((M + 255) / 256);
  at::Tensor part = at::empty({nparts, Co, 2}, opts);
  gemm_log_add("stem_fwd", (long long)N * H * W, Co, 9LL * Cin, 256, 64, 1);
  stem_fwd_launch(x.data_ptr<float>(), w.data_ptr<float>(), fptr(b), y.data_ptr<float>(),
                  part.data_ptr<float>(), N, H, W, Cin, Co, st);
  at::Tensor stats = at::empty({4, Co}, opts);
  long long* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined())
    nbt = reinterpret_cast<long long*>(num_batches_tracked->data_ptr<int64_t>());
  // up to 128 images (<= 512 partials of 256 rows) finalize and apply in one launch, as the
  // deeper blocks do (one dispatch fewer at the strong-scaling batches)
  const bool fused = bn_fin_enabled(false) && bn_fin_act_ok(nparts, Co, false);
  if (!fused)
    bn_finalize_launch(part.data_ptr<float>(), nparts, 256, (int)M, Co, fptr(gamma), fptr(beta),
                       fptr_mut(running_mean), fptr_mut(running_var), nbt, (float)momentum, (float)eps,
                       stats.data_ptr<float>(), st);
  at::Tensor out = at::empty({N, Co, pool ? H / 2 : H, pool ? W / 2 : W},
                             opts.memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor out_amax;  // the output's act max: the next conv's operand scales (f16x2)
  ActMaxOut am{nullptr, nullptr};
  if (f16x2_mode()) {
    out_amax = new_act_max(N, Co, out, st);
    am = act_out(out_amax, N);
  }
  if (fused)
    bn_fin_act_launch(part.data_ptr<float>(), nparts, 256, Co, fptr(gamma), fptr(beta), fptr_mut(running_mean),
                      fptr_mut(running_var), nbt, (float)momentum, (float)eps, stats.data_ptr<float>(),
                      y.data_ptr<float>(), out.data_ptr<float>(), N, H, W, pool, relu, am, st);
  else
    bn_act_fwd_launch(y.data_ptr<float>(), stats.data_ptr<float>(), nullptr, out.data_ptr<float>(), N, H, W, Co, pool,
                      relu, st, am);
  return {out, y, stats, x, out_amax, at::Tensor(), at::Tensor(), at::Tensor()};
}

// ---------------------------------------------------------------- fused block forward
// out = [maxpool2](act(BN(conv3x3(x) + b) [+ residual])), training or eval BatchNorm.
// Returns {out, y (conv output), stats [4, C] = (mean, invstd, scale, shift)}.
// One-launch BN finalize + apply for the layers with few statistics partials: forward
// bn_fin_act and backward bn_bwd_fin_apply (both default; CDP_BN_FIN_ACT=0 / CDP_BN_BWD_FIN=0
// select finalize-then-apply). Both load their first rows of y (and gout) before merging the
// partials, so the two round trips overlap. Same-box A/B on MI355X, VGG-11 hipGraph step: forward
// 1.399 vs 1.407 ms at 256 images per GPU (fused 0.6 % faster, two boxes agree); backward 1.409 vs
// 1.404 ms at 256 images (within noise) and 0.632 vs 0.641 ms at 32 images (1.3 % faster, where
// every deep layer qualifies). Read per call so a test can compare both paths in one process.
// CDP_EXP_SKIP_BN_APPLY=1: TIMING EXPERIMENT ONLY, numerically wrong -- the fused finalize + apply
// launches of the small layers are skipped (their outputs stay uninitialised), which bounds what
// moving BatchNorm into the consumer GEMMs could save (docs/PERF.md, round 5)
static bool exp_skip_bn_apply() {
  const char* e = std::getenv("CDP_EXP_SKIP_BN_APPLY");
  return e && e[0] == '1';
}
static bool bn_fin_enabled(bool bwd = false) {
  const char* e = std::getenv(bwd ? "CDP_BN_BWD_FIN" : "CDP_BN_FIN_ACT");
  return !(e && e[0] == '0');
}
// CDP_BN_*=1 (set explicitly): take the fused path wherever it applies, whatever the batch (tests)
static bool bn_fin_forced(bool bwd = false) {
  const char* e = std::getenv(bwd ? "CDP_BN_BWD_FIN" : "CDP_BN_FIN_ACT");
  return e && e[0] == '1';
}

std::vector<at::Tensor> conv_bn_act_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                        const c10::optional<at::Tensor>& gamma,
                                        const c10::optional<at::Tensor>& beta,
                                        const c10::optional<at::Tensor>& running_mean,
                                        const c10::optional<at::Tensor>& running_var,
                                        const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                        double eps, bool training, int64_t stride, int64_t pad, bool pool, bool relu,
                                        const c10::optional<at::Tensor>& residual,
                                        const c10::optional<at::Tensor>& x_amax,
                                        const c10::optional<at::Tensor>& w_amax,
                                        const c10::optional<at::Tensor>& res_y,
                                        const c10::optional<at::Tensor>& res_stats, bool defer_apply) {
  // RGB stem (3x3 / stride 1 / pad 1, Cin <= 4, training BN): one exact-fp32 MFMA kernel reading
  // the raw NHWC input, no channel padding, no operand scales (stem.hip)
  const bool lazy_res = res_y.has_value() && res_y->defined();
  if (stem_enabled() && stem_ok((int)x.size(1), (int)w.size(2), (int)w.size(3), stride, pad, (int)w.size(0)) &&
      training && !(residual.has_value() && residual->defined()) && !lazy_res && !defer_apply)
    return stem_bn_act_fwd(x, w, b, gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, pool,
                           relu);
  // other stems: zero-pad 3 -> 4 channels so the float4 gather path runs (the padded input is what
  // backward needs, so it is returned for saving)
  const bool padc = (x.size(1) % 4) != 0;
  at::Tensor pad_amax;  // the padding pass measures x on the way (f16x2)
  const at::Tensor xin = padc ? pad_channels4(nhwc(x), f16x2_mode() ? &pad_amax : nullptr) : x;
  const at::Tensor win = padc ? pad_channels4(nhwc(w)) : w;
  // f16x2 operand maxima: x's from its producer when given; W's once per step, reused by backward
  // (zero channel padding does not change a maximum; a given x act max of the unpadded tensor is
  // not used for the padded one, whose channel count differs)
  const at::Tensor xa = act_max(xin, pad_amax.defined() ? c10::optional<at::Tensor>(pad_amax)
                                     : padc ? c10::optional<at::Tensor>() : x_amax,
                                cur_stream());
  const at::Tensor wa = weight_max(win, padc ? c10::optional<at::Tensor>() : w_amax);
  std::vector<at::Tensor> r = conv2d_fwd(xin, win, b, stride, pad, training, xa, wa);
  at::Tensor y = r[0];
  const int N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  TORCH_CHECK(C % 4 == 0, "BatchNorm channel count must be a multiple of 4");
  auto opts = y.options();
  at::Tensor stats = at::empty({4, C}, opts);
  hipStream_t st = cur_stream();
  const bool has_res = (residual.has_value() && residual->defined()) || lazy_res;
  TORCH_CHECK(!(lazy_res && residual.has_value() && residual->defined()), "conv_bn_act_fwd: residual or res_y, not both");
  // few statistics partials (the deep layers): finalize and apply in one launch (bn_fin_act_kernel)
  bool fused_fin = false;
  int nparts = 0, rpp = 0;
  long long* nbt = nullptr;
  if (training) {
    nparts = r[1].size(0);
    rpp = r[2].item<int>();
    if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
      TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong, "num_batches_tracked must be int64");
      nbt = reinterpret_cast<long long*>(num_batches_tracked->data_ptr<int64_t>());
    }
    fused_fin = bn_fin_enabled() && bn_fin_act_ok(nparts, C, has_res) && !defer_apply;
    if (!fused_fin)
      bn_finalize_launch(r[1].data_ptr<float>(), nparts, rpp, N * H * W, C, fptr(gamma), fptr(beta),
                         fptr_mut(running_mean), fptr_mut(running_var), nbt, (float)momentum, (float)eps,
                         stats.data_ptr<float>(), st);
  } else {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "eval BatchNorm needs running stats");
    bn_eval_stats_launch(C, fptr(gamma), fptr(beta), running_mean->data_ptr<float>(), running_var->data_ptr<float>(),
                         (float)eps, stats.data_ptr<float>(), st);
  }
  if (defer_apply) {
    // statistics only: the consumer applies this BatchNorm itself (a downsample branch, added inside
    // the residual block's apply pass through res_y / res_stats). `out` is a shape-only placeholder
    // for autograd (one element, expanded): nothing may read it.
    TORCH_CHECK(!pool && !relu && !has_res, "conv_bn_act_fwd: defer_apply is for a plain BatchNorm (no pool, "
                                            "activation or residual)");
    at::Tensor ph = at::empty({1}, opts).expand({N, C, H, W});
    return {ph, y, stats, xin, at::Tensor(), xa, wa, at::Tensor()};
  }
  at::Tensor res, ry, rst;
  if (has_res) {
    TORCH_CHECK(!pool, "residual + pool not supported");
    if (lazy_res) {
      ry = nhwc(*res_y);
      TORCH_CHECK(res_stats.has_value() && res_stats->defined() && res_stats->numel() == 4 * C &&
                      res_stats->is_contiguous() && ry.size(0) == N && ry.size(1) == C && ry.size(2) == H &&
                      ry.size(3) == W,
                  "conv_bn_act_fwd: res_y must match the output and res_stats be its [4, C] stats block");
      rst = *res_stats;
    } else {
      res = nhwc(*residual);
    }
  }
  at::Tensor out = at::empty({N, C, pool ? H / 2 : H, pool ? W / 2 : W},
                             opts.memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor out_amax;  // the output's act max: the next conv's operand scales (f16x2)
  ActMaxOut am{nullptr, nullptr};
  if (f16x2_mode()) {
    out_amax = new_act_max(N, C, out, st);
    am = act_out(out_amax, N);
  }
  if (fused_fin && exp_skip_bn_apply()) {
    // timing experiment only (wrong numbers): no finalize + apply launch at all -- the ceiling of
    // what applying BatchNorm in the consumer GEMM's operand load could save
  } else if (fused_fin)
    bn_fin_act_launch(r[1].data_ptr<float>(), nparts, rpp, C, fptr(gamma), fptr(beta), fptr_mut(running_mean),
                      fptr_mut(running_var), nbt, (float)momentum, (float)eps, stats.data_ptr<float>(),
                      y.data_ptr<float>(), out.data_ptr<float>(), N, H, W, pool, relu, am, st);
  // a residual block's ReLU pass mask (1 byte per float4): its backward reads this, not `out`
  at::Tensor rmask;
  static const bool mask_on = [] {
    const char* e = std::getenv("CDP_RES_MASK");
    return !(e && e[0] == '0');
  }();
  if (mask_on && has_res && relu && !fused_fin)
    rmask = at::empty({(long long)N * H * W * (C / 4)}, opts.dtype(at::kByte));
  if (!(fused_fin && exp_skip_bn_apply()) && !fused_fin)
    bn_act_fwd_launch(y.data_ptr<float>(), stats.data_ptr<float>(), res.defined() ? res.data_ptr<float>() : nullptr,
                      out.data_ptr<float>(), N, H, W, C, pool, relu, st, am,
                      rmask.defined() ? rmask.data_ptr<uint8_t>() : nullptr, ry.defined() ? ry.data_ptr<float>() : nullptr,
                      rst.defined() ? rst.data_ptr<float>() : nullptr);
  return {out, y, stats, xin, out_amax, xa, wa, rmask};
}

// ---------------------------------------------------------------- fused block backward
// Returns {dx (undefined when !need_dx), dw, db, dgamma, dbeta, dresidual (when zout given),
// prev_part, dy's act max (f16x2)}.
std::vector<at::Tensor> conv_bn_act_bwd(const at::Tensor& gout_, const at::Tensor& x, const at::Tensor& w,
                                        const at::Tensor& y, const at::Tensor& stats, int64_t stride, int64_t pad,
                                        bool pool, bool relu, bool need_dx, bool has_bias,
                                        const c10::optional<at::Tensor>& zout_, bool training,
                                        const c10::optional<at::Tensor>& dw_out,
                                        const c10::optional<at::Tensor>& db_out,
                                        const c10::optional<at::Tensor>& dgamma_out,
                                        const c10::optional<at::Tensor>& dbeta_out,
                                        const c10::optional<at::Tensor>& dx_addend,
                                        const c10::optional<at::Tensor>& x_amax,
                                        const c10::optional<at::Tensor>& w_amax,
                                        const c10::optional<at::Tensor>& w_t,
                                        const c10::optional<at::Tensor>& part_in,
                                        const c10::optional<at::Tensor>& prev_y,
                                        const c10::optional<at::Tensor>& prev_stats, bool prev_pool, bool prev_relu,
                                        int64_t prev_ps, const c10::optional<at::Tensor>& bias) {
  check_f32_cuda(gout_, "grad_output");
  const at::Tensor gout = nhwc(gout_);
  const int N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  auto opts = y.options();
  hipStream_t st = cur_stream();
  auto slot = [&](const c10::optional<at::Tensor>& o, std::initializer_list<int64_t> shape, bool cl) {
    if (o.has_value() && o->defined()) return *o;
    return cl ? at::empty(shape, opts.memory_format(at::MemoryFormat::ChannelsLast)) : at::empty(shape, opts);
  };
  // the residual block's ReLU: its pass mask (uint8, conv_bn_act_fwd's 8th output) or its output
  at::Tensor zout;
  const unsigned char* rmask = nullptr;
  if (zout_.has_value() && zout_->defined()) {
    if (zout_->scalar_type() == at::kByte) {
      zout = *zout_;
      TORCH_CHECK(zout.is_cuda() && zout.is_contiguous() && zout.numel() == (long long)N * H * W * (C / 4),
                  "conv_bn_act_bwd: the residual ReLU mask must hold one byte per float4 of the output");
      rmask = zout.data_ptr<uint8_t>();
    } else {
      zout = nhwc(*zout_);
    }
  }
  const float* zout_f = zout.defined() && !rmask ? zout.data_ptr<float>() : nullptr;
  const int nblk = bn_bwd_grid(N, H, W, C, pool);
  // The conv-bias gradient sum(dy) comes out of the finalize of the statistics reduction
  // (chan_finalize dbmode): in training mode from one extra partial, sum(xhat); in eval mode as
  // scale * sum(dz). Only a pooled odd-size map (border pixels outside every window, which the
  // reduction does not visit) takes the separate partial-sum pass over dy.
  const bool odd_pool = pool && ((H & 1) || (W & 1));
  const bool fused_db = has_bias && !odd_pool;
  const int ps = fused_db && training ? 3 : 2;
  // the statistics reduction: from the consumer block's fused backward reduction when it made it
  // (part_in, see prev_* below), else a launch of its own
  at::Tensor part;
  if (part_in.has_value() && part_in->defined()) {
    part = *part_in;
    TORCH_CHECK(part.dim() == 3 && part.size(1) == C && part.size(2) == ps && !zout.defined(),
                "conv_bn_act_bwd: part_in must be [nparts, C, ", ps, "] (no residual)");
  } else {
    part = at::empty({nblk, C, ps}, opts);
    bn_bwd_reduce_launch(y.data_ptr<float>(), gout.data_ptr<float>(), stats.data_ptr<float>(),
                         part.data_ptr<float>(), nblk, N, H, W, C, pool, relu, zout_f, st, ps == 3, rmask);
  }
  const int nparts = (int)part.size(0);
  at::Tensor sums = at::empty({2, C}, opts);
  // gradients go straight into the caller's slots (flat-arena views) when provided
  at::Tensor dgamma = slot(dgamma_out, {C}, false), dbeta = slot(dbeta_out, {C}, false);
  at::Tensor db;
  if (has_bias) db = slot(db_out, {C}, false);
  // eval-mode BatchNorm is a fixed affine map: dy = scale * dz (no batch-statistics terms)
  const int dbmode = fused_db ? (training ? 1 : 2) : 0;
  // RGB stem without an input gradient (VGG layer 0): the weight-gradient kernel applies the
  // BN / ReLU / pool backward on the fly, so dy is never materialised (stem.hip)
  const int cin = (int)x.size(1);
  const bool stem_path = stem_enabled() && !need_dx && training && pool && relu && !zout.defined() && fused_db &&
                         C == 64 && stem_ok(cin, (int)w.size(2), (int)w.size(3), stride, pad, C) &&
                         cin == (int)w.size(1) && (H % 2) == 0 && (W % 2) == 0;
  // few statistics partials (the deep layers): finalize and apply in one launch (bn_bwd_fin_apply_kernel),
  // at <= 64 images per GPU. Same-box A/B, hipGraph step, fused vs chan_finalize + bn_bwd_apply
  // (three interleaved pairs each, round 4): 32 images 0.5394 vs 0.5444 ms (fused 0.9 % faster),
  // 64 images 0.7135 vs 0.7134 (tie), 128 images 0.9478 vs 0.9458, 256 images 1.3444 vs 1.3411
  // (the two-launch path 0.2 % faster: its 1024-block apply outruns the fused kernel's
  // <= 512 blocks that each repeat the partial merge)
  const bool fused_fin = bn_fin_enabled(true) && training && !stem_path && !zout.defined() && (!has_bias || fused_db) &&
                         bn_bwd_fin_apply_ok(nparts, C, H, W, pool) && (N <= 64 || bn_fin_forced(true));
  if (!fused_fin)
    chan_finalize_launch(part.data_ptr<float>(), nparts, C, sums.data_ptr<float>(), dbeta.data_ptr<float>(),
                         dgamma.data_ptr<float>(), false, st, ps, fused_db ? db.data_ptr<float>() : nullptr,
                         stats.data_ptr<float>() + 2 * C, (long long)N * H * W, dbmode);
  if (!training && dbmode != 2) sums.zero_();
  if (stem_path) {
    const at::Tensor xin = nhwc(x);
    const int nb = stem_wgrad_blocks(N, H, W);
    at::Tensor slab = at::empty({nb, C, 36}, opts);
    gemm_log_add("stem_wgrad", C, 9LL * cin, (long long)N * H * W, 64, 36, nb);
    stem_wgrad_launch(y.data_ptr<float>(), gout.data_ptr<float>(), stats.data_ptr<float>(), sums.data_ptr<float>(),
                      xin.data_ptr<float>(), slab.data_ptr<float>(), nb, N, H, W, cin, st);
    at::Tensor dw = dw_out.has_value() && dw_out->defined()
                        ? *dw_out
                        : at::empty({C, cin, w.size(2), w.size(3)}, opts.memory_format(at::MemoryFormat::ChannelsLast));
    TORCH_CHECK(dw.is_contiguous(at::MemoryFormat::ChannelsLast), "stem dW slot must be channels_last");
    slab_sum_strided_launch(slab.data_ptr<float>(), nb, (long long)C * 36, 4, cin, dw.data_ptr<float>(), false, st);
    return {at::Tensor(), dw, db, dgamma, dbeta, at::Tensor(), at::Tensor(), at::Tensor()};
  }
  at::Tensor dy = at::empty({N, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor dbpart;
  const bool sep_db = has_bias && !fused_db;
  if (sep_db) dbpart = at::empty({nblk, C, 2}, opts);
  at::Tensor dres;
  if (zout.defined()) dres = at::empty({N, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor dy_amax;  // dy's act max: operand scales of both gradient GEMMs (f16x2)
  ActMaxOut am{nullptr, nullptr};
  if (f16x2_mode()) {
    dy_amax = new_act_max(N, C, dy, st);
    am = act_out(dy_amax, N);
  }
  if (fused_fin && exp_skip_bn_apply()) {
    // timing experiment only (wrong numbers), as in conv_bn_act_fwd
  } else if (fused_fin)
    bn_bwd_fin_apply_launch(part.data_ptr<float>(), nparts, ps, y.data_ptr<float>(), gout.data_ptr<float>(),
                            stats.data_ptr<float>(), dy.data_ptr<float>(), dbeta.data_ptr<float>(),
                            dgamma.data_ptr<float>(), has_bias ? db.data_ptr<float>() : nullptr, N, H, W, C, pool,
                            relu, am, st);
  else
    bn_bwd_apply_launch(y.data_ptr<float>(), gout.data_ptr<float>(), stats.data_ptr<float>(),
                        sums.data_ptr<float>(), dy.data_ptr<float>(), sep_db ? dbpart.data_ptr<float>() : nullptr,
                        nblk, N, H, W, C, pool, relu, zout_f,
                        dres.defined() ? dres.data_ptr<float>() : nullptr, st, am, rmask);
  const c10::optional<at::Tensor> dya = dy_amax.defined() ? c10::optional<at::Tensor>(dy_amax) : c10::nullopt;
  if (sep_db)
    chan_finalize_launch(dbpart.data_ptr<float>(), nblk, C, nullptr, db.data_ptr<float>(), nullptr, false, st);
  // x may carry zero-padded channels (RGB stem, see conv_bn_act_fwd)
  const bool padc = x.size(1) != w.size(1);
  // (running the weight gradient on a side stream beside the data gradient was measured 2x slower
  // on MI355X: two full-occupancy GEMM grids compete instead of overlapping; docs/PERF.md)
  at::Tensor dx, dw;
  // both GEMMs' split-K reductions (and, given prev_*, the previous block's BN statistics
  // reduction) in one bwd_reduce launch after the two GEMMs (bwd_fuse.hip)
  // Only with a previous BN to serve: on its own the merge of the two reductions buys nothing (the
  // weight-gradient slab then waits in HBM behind the data-gradient GEMM; ResNet-50 B=64 measured
  // 0.4 % slower with it)
  DeferredReduce dr;
  const bool has_prev = prev_y.has_value() && prev_y->defined() && prev_stats.has_value() && prev_stats->defined();
  DeferredReduce* defer = (bwd_fuse_enabled() && !padc && has_prev) ? &dr : nullptr;
  // the weight gradient waits for the data gradient so both GEMMs can share one launch (bwd_pair)
  PendingWgrad pend;
  PendingWgrad* pp = (need_dx && !padc && stride == 1 && bwd_pair_enabled()) ? &pend : nullptr;
  dw = wgrad_impl(dy, x, {w.size(0), x.size(1), w.size(2), w.size(3)}, stride, pad, dw_out, false,
                  padc ? w.size(1) : -1, dya, x_amax, defer, pp);
  if (need_dx) {
    if (padc) {
      at::Tensor dx4 = conv2d_dgrad(dy, pad_channels4(nhwc(w)), {x.size(0), x.size(1), x.size(2), x.size(3)}, stride,
                                    pad, c10::nullopt, dya, w_amax);
      dx = dx4.narrow(1, 0, w.size(1)).contiguous(at::MemoryFormat::ChannelsLast);
      if (dx_addend.has_value() && dx_addend->defined()) dx.add_(*dx_addend);
    } else {
      // residual-branch gradient (dx_addend) is accumulated by the data-gradient GEMM's epilogue
      dx = dgrad_impl(dy, w, {x.size(0), x.size(1), x.size(2), x.size(3)}, stride, pad, dx_addend, dya, w_amax, w_t,
                      defer, pp);
    }
  }
  pend.flush(st);  // no data-gradient GEMM took it: launch the weight gradient alone
  at::Tensor prev_part;
  if (dr.w_slab.defined() || dr.d_on) {
    BwdReduceArgs a{};
    if (dr.d_on) {
      a.d_slab = dr.d_src;
      a.d_y = dr.d_y;
      a.d_addend = dr.d_addend;
      a.d_S = dr.d_S;
      a.d_M = dr.d_M;
      a.d_Nout = dr.d_Nout;
      // the previous block's BN statistics reduction over this dX (its gradient at the BN output)
      if (has_prev && !(dx_addend.has_value() && dx_addend->defined())) {
        const at::Tensor py = nhwc(*prev_y);
        const int pH = py.size(2), pW = py.size(3);
        TORCH_CHECK(py.size(0) == x.size(0) && py.size(1) == x.size(1) &&
                        (prev_pool ? (pH / 2 == x.size(2) && pW / 2 == x.size(3))
                                   : (pH == x.size(2) && pW == x.size(3))) &&
                        (prev_ps == 2 || prev_ps == 3) && prev_stats->numel() == 4 * py.size(1),
                    "conv_bn_act_bwd: prev_y / prev_stats do not describe the BN that produced x");
        prev_part = at::empty({(dr.d_M + bwd_reduce_rows_per_part() - 1) / bwd_reduce_rows_per_part(), x.size(1),
                               prev_ps}, opts);
        a.bn_y = py.data_ptr<float>();
        a.bn_stats = prev_stats->data_ptr<float>();
        a.bn_part = prev_part.data_ptr<float>();
        a.bn_H = pH;
        a.bn_W = pW;
        a.bn_pool = prev_pool ? 1 : 0;
        a.bn_relu = prev_relu ? 1 : 0;
        a.bn_ps = (int)prev_ps;
      }
    }
    if (dr.w_slab.defined()) {
      a.w_slab = reinterpret_cast<const float4*>(dr.w_slab.data_ptr<float>());
      a.w_dst = reinterpret_cast<float4*>(dr.w_dst);
      a.w_S = dr.w_S;
      a.w_n4 = dr.w_n / 4;
    }
    bwd_reduce_launch(a, st);
  }
  return {dx, dw, db, dgamma, dbeta, dres, prev_part, dy_amax};
}

// ---------------------------------------------------------------- linear
// y[B, O] = x[B, I] @ W[O, I]^T + b  (1x1 implicit GEMM)
at::Tensor linear_fwd(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& b) {
  check_f32_cuda(x_, "input");
  check_f32_cuda(w_, "weight");
  const at::Tensor x = x_.contiguous(), w = w_.contiguous();
  const int B = x.size(0), I = x.size(1), O = w.size(0);
  TORCH_CHECK(w.size(1) == I, "linear shape mismatch");
  at::Tensor y = at::empty({B, O}, x.options());
  if (O <= 16) {
    small_linear_fwd_launch(x.data_ptr<float>(), w.data_ptr<float>(), fptr(b), B, I, O, y.data_ptr<float>(),
                            cur_stream());
    return y;
  }
  GemmPlan g = plan_gemm(B, O, I);
  ConvGemmParams p{};
  p.x = x.data_ptr<float>();
  p.w = w.data_ptr<float>();
  p.N = B; p.H = 1; p.W = 1; p.C = I; p.P = 1; p.Q = 1; p.KH = 1; p.KW = 1; p.stride = 1; p.pad = 0;
  p.Nout = O; p.M = B; p.Kdim = I; p.ktiles = g.ktiles; p.splits = g.splits;
  set_divs(p);
  hipStream_t st = cur_stream();
  set_scales(p, act_max(x, c10::nullopt, st), weight_max(w, c10::nullopt), false, O, I);
  if (g.splits == 1) {
    p.y = y.data_ptr<float>();
    p.bias = fptr(b);
    conv_launch(p, g.bm, g.bn, false, st);
  } else {
    at::Tensor slab = at::empty({g.splits, B, O}, x.options());
    p.y = slab.data_ptr<float>();
    conv_launch(p, g.bm, g.bn, false, st);
    splitk_reduce_launch(slab.data_ptr<float>(), g.splits, B, O, fptr(b), y.data_ptr<float>(), nullptr, st);
  }
  return y;
}

// {dx, dw, db}
std::vector<at::Tensor> linear_bwd(const at::Tensor& gy_, const at::Tensor& x_, const at::Tensor& w_, bool need_dx,
                                   bool has_bias, const c10::optional<at::Tensor>& dw_out,
                                   const c10::optional<at::Tensor>& db_out) {
  const at::Tensor gy = gy_.contiguous(), x = x_.contiguous(), w = w_.contiguous();
  const int B = x.size(0), I = x.size(1), O = w.size(0);
  hipStream_t st = cur_stream();
  if (O <= 16) {
    at::Tensor dx = need_dx ? at::empty({B, I}, x.options()) : at::Tensor();
    at::Tensor dw = (dw_out.has_value() && dw_out->defined()) ? *dw_out : at::empty({O, I}, x.options());
    at::Tensor db;
    if (has_bias) db = (db_out.has_value() && db_out->defined()) ? *db_out : at::empty({O}, x.options());
    small_linear_bwd_launch(gy.data_ptr<float>(), x.data_ptr<float>(), w.data_ptr<float>(), B, I, O,
                            need_dx ? dx.data_ptr<float>() : nullptr, dw.data_ptr<float>(),
                            has_bias ? db.data_ptr<float>() : nullptr, st);
    return {dx, dw, db};
  }
  at::Tensor dx;
  if (need_dx) {
    // dx[B, I] = gy[B, O] @ W[O, I]  ->  B^T = W^T [I][O]
    at::Tensor wt = at::empty({I, O}, x.options());
    wtrans_launch(w.data_ptr<float>(), wt.data_ptr<float>(), O, 1, I, st);
    dx = linear_fwd(gy, wt, c10::nullopt);
  }
  // dW[O, I] = gy^T x  (1x1 wgrad over B rows)
  at::Tensor dw = (dw_out.has_value() && dw_out->defined()) ? *dw_out : at::empty({O, I}, x.options());
  TORCH_CHECK(dw.is_contiguous() && dw.numel() == (int64_t)O * I, "linear dW slot must be contiguous [O, I]");
  WgradParams p{};
  p.dy = gy.data_ptr<float>();
  p.x = x.data_ptr<float>();
  p.N = B; p.H = 1; p.W = 1; p.C = I; p.P = 1; p.Q = 1; p.KH = 1; p.KW = 1; p.stride = 1; p.pad = 0;
  p.Cout = O; p.Kdim = I; p.M = B;
  const WgradPlan wp = plan_wgrad(O, I, B);
  p.splits = wp.splits;
  set_divs(p);
  set_scales(p, act_max(gy, c10::nullopt, st), act_max(x, c10::nullopt, st));
  if (p.splits == 1) {
    p.out = dw.data_ptr<float>();
    wgrad_launch_logged(p, wp.bm, wp.bn, x3_family() && x3_ok(p), st, split_planes());
  } else {
    at::Tensor slab = at::empty({p.splits, O, I}, x.options());
    p.out = slab.data_ptr<float>();
    wgrad_launch_logged(p, wp.bm, wp.bn, x3_family() && x3_ok(p), st, split_planes());
    slab_sum_launch(slab.data_ptr<float>(), p.splits, (long long)O * I, dw.data_ptr<float>(), false, st);
  }
  at::Tensor db;
  if (has_bias) {
    db = (db_out.has_value() && db_out->defined()) ? *db_out : at::empty({O}, x.options());
    colsum_launch(gy.data_ptr<float>(), B, O, db.data_ptr<float>(), false, st);
  }
  return {dx, dw, db};
}

// ---------------------------------------------------------------- cross entropy
// {loss (0-dim), correct (int64 [1], accumulated in place when given)}
at::Tensor xent_fwd(const at::Tensor& logits_, const at::Tensor& target, const c10::optional<at::Tensor>& correct) {
  check_f32_cuda(logits_, "logits");
  TORCH_CHECK(target.scalar_type() == at::kLong, "target must be int64");
  const at::Tensor logits = logits_.contiguous();
  const at::Tensor tgt = target.contiguous();
  const int B = logits.size(0), C = logits.size(1);
  at::Tensor loss = at::empty({}, logits.options());
  long long* cp = nullptr;
  if (correct.has_value() && correct->defined()) cp = reinterpret_cast<long long*>(correct->data_ptr<int64_t>());
  xent_fwd_launch(logits.data_ptr<float>(), reinterpret_cast<const long long*>(tgt.data_ptr<int64_t>()), B, C, loss.data_ptr<float>(), cp, nullptr,
                  cur_stream());
  return loss;
}

at::Tensor xent_bwd(const at::Tensor& gloss, const at::Tensor& logits_, const at::Tensor& target) {
  const at::Tensor logits = logits_.contiguous();
  const at::Tensor g = gloss.to(at::kFloat).contiguous();
  const int B = logits.size(0), C = logits.size(1);
  at::Tensor d = at::empty_like(logits);
  xent_bwd_launch(logits.data_ptr<float>(), reinterpret_cast<const long long*>(target.contiguous().data_ptr<int64_t>()), g.data_ptr<float>(), B, C,
                  d.data_ptr<float>(), cur_stream());
  return d;
}

// {dlogits, dx, dw, db}: the softmax cross-entropy gradient and, in the same launch, the narrow
// Linear's three gradients from it (ops/functional.py fuses them when the loss directly consumes
// the classifier's logits)
std::vector<at::Tensor> xent_linear_bwd(const at::Tensor& gloss, const at::Tensor& logits_, const at::Tensor& target,
                                        const at::Tensor& x_, const at::Tensor& w_, bool need_dx, bool has_bias,
                                        const c10::optional<at::Tensor>& dw_out, const c10::optional<at::Tensor>& db_out,
                                        const c10::optional<at::Tensor>& link_y,
                                        const c10::optional<at::Tensor>& link_stats, bool link_pool, bool link_relu,
                                        int64_t link_ps) {
  const at::Tensor logits = logits_.contiguous(), x = x_.contiguous(), w = w_.contiguous();
  const at::Tensor g = gloss.to(at::kFloat).contiguous();
  const at::Tensor tgt = target.contiguous();
  check_f32_cuda(logits, "logits");
  check_f32_cuda(x, "input");
  const int B = x.size(0), I = x.size(1), O = w.size(0);
  TORCH_CHECK(logits.size(0) == B && logits.size(1) == O && w.size(1) == I, "xent_linear_bwd: shape mismatch");
  TORCH_CHECK(O <= 16 && (long long)B * O <= kXentLinMax, "xent_linear_bwd: classifier too wide");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.numel() == B, "xent_linear_bwd: int64 target per row");
  at::Tensor dl = at::empty_like(logits);
  at::Tensor dx = need_dx ? at::empty({B, I}, x.options()) : at::Tensor();
  at::Tensor dw = (dw_out.has_value() && dw_out->defined()) ? *dw_out : at::empty({O, I}, x.options());
  TORCH_CHECK(dw.is_contiguous() && dw.numel() == (int64_t)O * I, "linear dW slot must be contiguous [O, I]");
  at::Tensor db;
  if (has_bias) db = (db_out.has_value() && db_out->defined()) ? *db_out : at::empty({O}, x.options());
  XentBnLink lk{nullptr, nullptr, nullptr, 0, 0, 2};
  at::Tensor part;
  if (link_y.has_value() && link_y->defined()) {
    // the block that produced x: pre-BN output y [B, C = I, 2, 2] (pooled to 1x1) or [B, I, 1, 1]
    const at::Tensor& yb = *link_y;
    check_f32_cuda(yb, "link y");
    const int hw = link_pool ? 2 : 1;
    TORCH_CHECK(need_dx && yb.dim() == 4 && yb.size(0) == B && yb.size(1) == I && yb.size(2) == hw &&
                    yb.size(3) == hw && yb.is_contiguous(at::MemoryFormat::ChannelsLast),
                "xent_linear_bwd: BN link needs the block's channels_last [B, I, ", hw, ", ", hw, "] output");
    TORCH_CHECK(link_stats.has_value() && link_stats->is_cuda() && link_stats->numel() == 4LL * I &&
                    link_stats->is_contiguous() && (link_ps == 2 || link_ps == 3),
                "xent_linear_bwd: BN link stats [4, C] and ps in {2, 3}");
    part = at::empty({xent_lin_chunks(B), I, link_ps}, x.options());
    lk = XentBnLink{yb.data_ptr<float>(), link_stats->data_ptr<float>(), part.data_ptr<float>(), link_pool ? 1 : 0,
                    link_relu ? 1 : 0, (int)link_ps};
  }
  xent_linear_bwd_launch(logits.data_ptr<float>(), reinterpret_cast<const long long*>(tgt.data_ptr<int64_t>()),
                         g.data_ptr<float>(), x.data_ptr<float>(), w.data_ptr<float>(), B, I, O, dl.data_ptr<float>(),
                         need_dx ? dx.data_ptr<float>() : nullptr, dw.data_ptr<float>(),
                         has_bias ? db.data_ptr<float>() : nullptr, lk, cur_stream());
  return {dl, dx, dw, db, part};
}

// ---------------------------------------------------------------- SGD over a flat arena
long long* counter_ptr(const c10::optional<at::Tensor>& c) {
  if (!(c.has_value() && c->defined())) return nullptr;
  TORCH_CHECK(c->is_cuda() && c->scalar_type() == at::kLong && c->numel() >= 1, "step counter must be a device int64");
  return reinterpret_cast<long long*>(c->data_ptr<int64_t>());
}

void sgd_step(at::Tensor p, const at::Tensor& g, c10::optional<at::Tensor> buf, const c10::optional<at::Tensor>& lr_t,
              double lr, double momentum, double dampening, double wd, double grad_scale, bool nesterov, bool first,
              bool maximize, const c10::optional<at::Tensor>& counter) {
  check_f32_cuda(p, "param");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && p.numel() == g.numel(), "sgd: flat contiguous tensors required");
  float* bp = nullptr;
  if (momentum != 0.0) {
    TORCH_CHECK(buf.has_value() && buf->numel() == p.numel(), "sgd: momentum buffer required");
    bp = buf->data_ptr<float>();
  }
  sgd_launch(p.data_ptr<float>(), g.data_ptr<float>(), bp, p.numel(), fptr(lr_t), (float)lr, (float)momentum,
             (float)dampening, (float)wd, (float)grad_scale, nesterov, first, maximize, cur_stream(),
             counter_ptr(counter));
}

// ---------------------------------------------------------------- SGD + next-step weight preparation
// Plan of the fused optimizer step over the flat range [s, e) of `flat` (an arena's parameter
// storage): one segment per conv weight (a channels_last view inside the range), the W^T
// destinations where want_t, and float4 chunks for everything else in the range. Returns
// {descriptor (device bytes), meta (cpu int64: nseg, nblk_w, nchunk), weight maxima (device;
// weight_max_elems floats per weight, back to back, as weight_prep lays them out), W^T per weight
// (undefined where not wanted)}. Built once per arena layout, outside any capture.
// With amax_out / amax_offsets the maxima go to caller-owned storage at the given float offsets
// (one per weight): the per-bucket plans of an overlapped optimizer step share ONE maxima tensor,
// laid out as the forward expects, and each writes only its own weights' part of it.
std::vector<at::Tensor> sgd_prep_plan(const at::Tensor& flat, int64_t s, int64_t e, const std::vector<at::Tensor>& ws,
                                      const std::vector<bool>& want_t, const c10::optional<at::Tensor>& amax_out,
                                      const std::vector<int64_t>& amax_offsets) {
  check_f32_cuda(flat, "arena");
  TORCH_CHECK(ws.size() == want_t.size() && !ws.empty(), "sgd_prep_plan: one want_t flag per weight");
  const bool ext = amax_out.has_value() && amax_out->defined();
  TORCH_CHECK(!ext || amax_offsets.size() == ws.size(), "sgd_prep_plan: one maxima offset per weight");
  if (ext) check_f32_cuda(*amax_out, "amax_out");
  TORCH_CHECK(0 <= s && s < e && e <= flat.numel() && (s % 4) == 0, "sgd_prep_plan: bad range");
  const float* base = flat.data_ptr<float>() + s;
  std::vector<SgdPrepSeg> segs;
  std::vector<std::pair<long long, long long>> covered;
  std::vector<at::Tensor> outs;
  int blk = 0;
  long long ptot = 0;
  for (size_t i = 0; i < ws.size(); ++i) {
    const at::Tensor& w = ws[i];
    check_f32_cuda(w, "sgd_prep weight");
    TORCH_CHECK(w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "sgd_prep_plan: conv weights must be channels_last [Co, Ci, KH, KW]");
    const long long off = w.data_ptr<float>() - base;
    TORCH_CHECK(off >= 0 && off + w.numel() <= e - s && (off % 4) == 0, "sgd_prep_plan: weight outside the range");
    const int Co = w.size(0), Ci = w.size(1), T = w.size(2) * w.size(3);
    TORCH_CHECK((long long)Co * T * Ci * 4 < (1LL << 31), "sgd_prep_plan: weight too large");
    at::Tensor wt;
    if (want_t[i]) wt = at::empty({Ci, (long long)T * Co}, flat.options());
    outs.push_back(wt);
    long long pofs = ptot;
    if (ext) {
      pofs = amax_offsets[i];
      TORCH_CHECK(pofs >= 0 && pofs + weight_max_elems(Co, Ci) <= amax_out->numel(),
                  "sgd_prep_plan: maxima offset outside amax_out");
    }
    segs.push_back(SgdPrepSeg{off, wt.defined() ? wt.data_ptr<float>() : nullptr, Co, T, Ci, blk, pofs});
    blk += ((Co + 31) / 32) * ((Ci + 31) / 32);
    ptot += weight_max_elems(Co, Ci);
    covered.push_back({off, off + (w.numel() + 3) / 4 * 4});
  }
  std::sort(covered.begin(), covered.end());
  std::vector<SgdPrepChunk> chunks;
  long long cur = 0;
  auto add_gap = [&](long long a, long long b) {
    for (long long x = a; x < b; x += 4LL * kSgdPrepChunk4)
      chunks.push_back(SgdPrepChunk{x, (int)(std::min<long long>(b - x, 4LL * kSgdPrepChunk4) / 4), 0});
  };
  for (const auto& c : covered) {
    TORCH_CHECK(c.first >= cur, "sgd_prep_plan: overlapping weights");
    add_gap(cur, c.first);
    cur = c.second;
  }
  TORCH_CHECK(((e - s) % 4) == 0, "sgd_prep_plan: range must be whole float4s");
  add_gap(cur, e - s);
  const size_t seg_bytes = segs.size() * sizeof(SgdPrepSeg);
  const size_t bytes = seg_bytes + chunks.size() * sizeof(SgdPrepChunk);
  at::Tensor host = at::empty({(long long)std::max<size_t>(bytes, 16)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr<uint8_t>(), segs.data(), seg_bytes);
  if (!chunks.empty()) std::memcpy(host.data_ptr<uint8_t>() + seg_bytes, chunks.data(), bytes - seg_bytes);
  at::Tensor desc = host.to(flat.device());
  at::Tensor meta = at::tensor({(int64_t)segs.size(), (int64_t)blk, (int64_t)chunks.size()}, at::kLong);
  at::Tensor amax = ext ? *amax_out : at::empty({std::max(ptot, 1LL)}, flat.options());
  std::vector<at::Tensor> r = {desc, meta, amax};
  for (auto& t : outs) r.push_back(t);
  return r;
}

void sgd_step_prep(at::Tensor p, const at::Tensor& g, c10::optional<at::Tensor> buf, const c10::optional<at::Tensor>& lr_t,
                   double lr, double momentum, double dampening, double wd, double grad_scale, bool nesterov, bool first,
                   bool maximize, const at::Tensor& desc, const at::Tensor& meta, at::Tensor amax,
                   const c10::optional<at::Tensor>& counter) {
  check_f32_cuda(p, "param");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && p.numel() == g.numel(), "sgd: flat contiguous tensors required");
  float* bp = nullptr;
  if (momentum != 0.0) {
    TORCH_CHECK(buf.has_value() && buf->numel() == p.numel(), "sgd: momentum buffer required");
    bp = buf->data_ptr<float>();
  }
  TORCH_CHECK(meta.device().is_cpu() && meta.numel() == 3 && desc.is_cuda(), "sgd_step_prep: plan from sgd_prep_plan");
  const int64_t* mt = meta.data_ptr<int64_t>();
  const int nseg = (int)mt[0], nblk = (int)mt[1], nchunk = (int)mt[2];
  TORCH_CHECK(desc.numel() >= (int64_t)(nseg * sizeof(SgdPrepSeg) + nchunk * sizeof(SgdPrepChunk)),
              "sgd_step_prep: descriptor smaller than the plan");
  const uint8_t* d = desc.data_ptr<uint8_t>();
  sgd_prep_launch(p.data_ptr<float>(), g.data_ptr<float>(), bp, reinterpret_cast<const SgdPrepSeg*>(d), nseg, nblk,
                  reinterpret_cast<const SgdPrepChunk*>(d + nseg * sizeof(SgdPrepSeg)), nchunk,
                  amax.data_ptr<float>(), fptr(lr_t), (float)lr, (float)momentum, (float)dampening, (float)wd,
                  (float)grad_scale, nesterov, first, maximize, cur_stream(), counter_ptr(counter));
}

// ---------------------------------------------------------------- data augmentation
at::Tensor augment(const at::Tensor& images, const c10::optional<at::Tensor>& indices, int64_t idx_offset, int64_t batch,
                   std::vector<double> mean, std::vector<double> std_, int64_t pad, bool flip,
                   const c10::optional<at::Tensor>& counter, int64_t seed, c10::optional<at::Tensor> out,
                   int64_t nbatches, const c10::optional<at::Tensor>& labels,
                   const c10::optional<at::Tensor>& labels_out) {
  TORCH_CHECK(images.is_cuda() && images.scalar_type() == at::kByte && images.dim() == 4,
              "images must be uint8 [N, H, W, C] on the GPU");
  const int H = images.size(1), W = images.size(2), C = images.size(3);
  at::Tensor o;
  if (out.has_value() && out->defined()) o = *out;
  else
    o = at::empty({batch, C, H, W}, images.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
  float m[3], is[3];
  for (int i = 0; i < 3; ++i) {
    m[i] = (float)mean[std::min<size_t>(i, mean.size() - 1)];
    is[i] = (float)(1.0 / std_[std::min<size_t>(i, std_.size() - 1)]);
  }
  TORCH_CHECK(o.is_cuda() && o.device() == images.device() && o.scalar_type() == at::kFloat && o.numel() >= batch * C * H * W,
              "augment: out must be a float32 tensor on the images' device holding the batch");
  const long long* ip = nullptr;
  if (indices.has_value() && indices->defined()) {
    TORCH_CHECK(indices->device() == images.device() && indices->scalar_type() == at::kLong && indices->is_contiguous(),
                "augment: indices must be a contiguous int64 tensor on the images' device");
    // the kernel reads idx[idx_offset + (counter % nbatches) * batch + b] for b < batch
    TORCH_CHECK(idx_offset >= 0 && idx_offset + std::max<int64_t>(nbatches, 1) * batch <= indices->numel(),
                "augment: idx_offset + max(nbatches, 1) * batch = ", idx_offset + std::max<int64_t>(nbatches, 1) * batch,
                " exceeds the ", indices->numel(), " indices");
    ip = reinterpret_cast<const long long*>(indices->data_ptr<int64_t>());
  } else {
    TORCH_CHECK(idx_offset >= 0 && idx_offset + std::max<int64_t>(nbatches, 1) * batch <= images.size(0),
                "augment: the batch range exceeds the ", images.size(0), " images");
  }
  const long long* cp = nullptr;
  if (counter.has_value() && counter->defined()) cp = reinterpret_cast<const long long*>(counter->data_ptr<int64_t>());
  TORCH_CHECK(nbatches == 0 || cp, "counter-driven batch offsets need the counter");
  const long long* lp = nullptr;
  long long* lo = nullptr;
  if (labels_out.has_value() && labels_out->defined()) {
    TORCH_CHECK(labels.has_value() && labels->defined() && labels->scalar_type() == at::kLong &&
                    labels_out->scalar_type() == at::kLong && labels_out->numel() >= batch,
                "labels / labels_out must be int64, labels_out holding the batch");
    TORCH_CHECK(labels->device() == images.device() && labels_out->device() == images.device() &&
                    labels->numel() >= images.size(0) && labels->is_contiguous() && labels_out->is_contiguous(),
                "augment: labels (one per image) and labels_out must be contiguous on the images' device");
    lp = reinterpret_cast<const long long*>(labels->data_ptr<int64_t>());
    lo = reinterpret_cast<long long*>(labels_out->data_ptr<int64_t>());
  }
  augment_launch(images.data_ptr<uint8_t>(), ip, idx_offset, (int)batch, H, W, C, m, is, (int)pad, flip, cp,
                 (unsigned long long)seed, o.data_ptr<float>(), cur_stream(), nbatches, lp, lo);
  return o;
}

void counter_inc(at::Tensor c) { counter_inc_launch(reinterpret_cast<long long*>(c.data_ptr<int64_t>()), cur_stream()); }

// ---------------------------------------------------------------- misc
void stack_mean(const std::vector<at::Tensor>& srcs, at::Tensor dst) {
  TORCH_CHECK(!srcs.empty(), "stack_mean: empty list");
  const int k = srcs.size();
  TORCH_CHECK(k <= kMaxStackSrcs, "stack_mean: at most ", kMaxStackSrcs, " tensors");
  // The pointers go in the kernel arguments. (They used to be uploaded as a device table by a
  // non-blocking copy from a temporary pageable host tensor, freed when the statement ended: now
  // and then the copy read reused host memory and the mean read a stale buffer -- the gather /
  // scatter strategy was not reproducible run to run.)
  std::vector<const float*> ptrs(k);
  for (int i = 0; i < k; ++i) {
    TORCH_CHECK(srcs[i].is_contiguous() && srcs[i].numel() == dst.numel() && srcs[i].device() == dst.device(),
                "stack_mean: shape / device mismatch");
    ptrs[i] = srcs[i].data_ptr<float>();
  }
  stack_mean_launch(ptrs.data(), k, dst.numel(), dst.data_ptr<float>(), cur_stream());
}

// one workgroup idles ~us microseconds on the current stream (no memory traffic): lets the host
// enqueue a whole phase ahead of the GPU, so events recorded in it time the GPU's own execution
void gpu_sleep(double us) { delay_scale_launch(nullptr, 0, 1.f, us, cur_stream()); }

// frequency of the clock gpu_timestamp reads (kHz)
int64_t gpu_wall_clock_khz() {
  int dev = 0, khz = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  return khz;
}

// ts[idx] = the GPU's wall clock when the current stream reaches this point
void gpu_timestamp(at::Tensor ts, int64_t idx) {
  TORCH_CHECK(ts.is_cuda() && ts.scalar_type() == at::kLong && idx >= 0 && idx < ts.numel(),
              "gpu_timestamp: device int64 buffer and an index inside it");
  timestamp_launch(reinterpret_cast<long long*>(ts.data_ptr<int64_t>()), (int)idx, cur_stream());
}

void scale_(at::Tensor x, double a) {
  TORCH_CHECK(x.is_contiguous(), "scale_: contiguous tensor required");
  scale_launch(x.data_ptr<float>(), x.numel(), (float)a, cur_stream());
}

std::vector<at::Tensor> maxpool2d_fwd(const at::Tensor& x_, int64_t k, int64_t s, int64_t p) {
  const at::Tensor x = nhwc(x_);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 4 == 0 && k * k <= 255, "maxpool2d: needs C % 4 == 0 and k*k <= 255");
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  at::Tensor y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor arg = at::empty({N, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  maxpool_fwd_launch(x.data_ptr<float>(), N, H, W, C, k, s, p, Ho, Wo, y.data_ptr<float>(), arg.data_ptr<uint8_t>(),
                     cur_stream());
  return {y, arg};
}

at::Tensor maxpool2d_bwd(const at::Tensor& gy_, const at::Tensor& arg, std::vector<int64_t> in_shape, int64_t k,
                         int64_t s, int64_t p) {
  const at::Tensor gy = nhwc(gy_);
  const int N = in_shape[0], C = in_shape[1], H = in_shape[2], W = in_shape[3];
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool2d_bwd: arg must be the uint8 channels_last map of maxpool2d_fwd");
  at::Tensor gx = at::empty({N, C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  maxpool_bwd_launch(gy.data_ptr<float>(), arg.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)s, (int)p, gy.size(2),
                     gy.size(3), gx.data_ptr<float>(), cur_stream());
  return gx;
}

at::Tensor avgpool_fwd(const at::Tensor& x_) {
  const at::Tensor x = nhwc(x_);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  at::Tensor y = at::empty({N, C}, x.options());
  avgpool_fwd_launch(x.data_ptr<float>(), N, H * W, C, y.data_ptr<float>(), cur_stream());
  return y;
}

at::Tensor avgpool_bwd(const at::Tensor& gy_, std::vector<int64_t> in_shape) {
  const at::Tensor gy = gy_.contiguous();
  const int N = in_shape[0], C = in_shape[1], H = in_shape[2], W = in_shape[3];
  at::Tensor gx = at::empty({N, C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  avgpool_bwd_launch(gy.data_ptr<float>(), N, H * W, C, gx.data_ptr<float>(), cur_stream());
  return gx;
}


std::vector<std::tuple<std::string, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>> gemm_log(bool clear) {
  return gemm_log_snapshot(clear);
}

}  // namespace cdp
