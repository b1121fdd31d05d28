// Native bucketed gradient reducer (the engine behind both the `bucketed_overlap` strategy and the
// DistributedDataParallel wrapper). It replaces the PyTorch C++ Reducer that the reference's Part 3
// gets implicitly from `DDP(model)` (/root/reference/src/Part 3/main.py:61).
//
// Design (MI355X-first, not a translation of torch's Reducer):
//  * gradients live in ONE flat fp32 arena; every parameter's .grad is a view into it and every
//    bucket is a contiguous arena range, so the all-reduce runs in place with zero copies;
//  * autograd post-hooks on the AccumulateGrad nodes (C++, no Python/GIL on the hot path) count
//    readiness per bucket; a bucket is launched the moment it is complete, strictly in bucket order
//    so every rank issues the same collective sequence;
//  * launches go to the RCCL communicator's own stream (ordered after the compute
//    stream by an event), so the all-reduce of late-layer buckets overlaps the rest of backward;
//    the end-of-backward callback makes the compute stream wait on the last bucket only (buckets
//    complete in order on one stream);
//  * ncclAvg performs the 1/world_size averaging inside the collective; the c10d path (gloo on CPU,
//    used by the CPU test-suite) uses SUM + an in-place scale;
//  * the observed ready order of the first iteration is recorded so the Python side can rebuild the
//    arena layout / bucket plan in true gradient-ready order (identically on all ranks).
#include "reducer.h"

#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/accumulate_grad.h>
#include <torch/csrc/autograd/variable.h>

#include <rocprofiler-sdk-roctx/roctx.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

#include "../kernels/kernels.h"
#include "ops.h"
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

namespace cdp {

namespace {
struct ReadyHook : public torch::autograd::FunctionPostHook {
  ReadyHook(Reducer* r, size_t i) : reducer(r), index(i) {}
  torch::autograd::variable_list operator()(const torch::autograd::variable_list& outputs,
                                            const torch::autograd::variable_list& /*inputs*/) override {
    reducer->mark_ready(index);
    return outputs;
  }
  Reducer* reducer;
  size_t index;
};
}  // namespace

Reducer::Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views, std::vector<at::Tensor> bucket_views,
                 std::vector<int64_t> bucket_starts, std::shared_ptr<RcclComm> rccl,
                 c10::intrusive_ptr<c10d::ProcessGroup> pg, bool find_unused, bool average)
    : params_(std::move(params)),
      grad_views_(std::move(grad_views)),
      bucket_views_(std::move(bucket_views)),
      rccl_(std::move(rccl)),
      pg_(std::move(pg)),
      find_unused_(find_unused),
      average_(average) {
  TORCH_CHECK(params_.size() == grad_views_.size(), "params / grad views mismatch");
  TORCH_CHECK(rccl_ || pg_, "Reducer needs an RCCL communicator or a process group");
  const size_t nb = bucket_views_.size();
  TORCH_CHECK(bucket_starts.size() == nb + 1, "bucket_starts must have num_buckets + 1 entries");
  // bucket b covers parameter indices [bucket_starts[b], bucket_starts[b+1]) (any order of ranges)
  bucket_of_.assign(params_.size(), -1);
  bucket_size_.assign(nb, 0);
  for (size_t b = 0; b < nb; ++b) {
    const int64_t lo = std::min(bucket_starts[b], bucket_starts[b + 1]);
    const int64_t hi = std::max(bucket_starts[b], bucket_starts[b + 1]);
    for (int64_t i = lo; i < hi; ++i) {
      TORCH_CHECK(bucket_of_[i] < 0, "parameter ", i, " assigned to two buckets");
      bucket_of_[i] = (int)b;
      bucket_size_[b]++;
    }
  }
  for (size_t i = 0; i < params_.size(); ++i) TORCH_CHECK(bucket_of_[i] >= 0, "parameter ", i, " has no bucket");
  world_ = rccl_ ? rccl_->size() : pg_->getSize();
  const char* rx = std::getenv("CDP_ROCTX");
  roctx_ = rx && std::strcmp(rx, "1") == 0;
  pending_.assign(nb, 0);
  works_.resize(nb);
  pg_works_.resize(nb);
  ready_flag_.assign(params_.size(), 0);
  // install autograd hooks
  for (size_t i = 0; i < params_.size(); ++i) {
    auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
    TORCH_CHECK(acc, "parameter ", i, " does not require grad");
    hook_keys_.push_back(acc->add_post_hook(std::make_unique<ReadyHook>(this, i)));
    accumulators_.push_back(acc);
  }
}

Reducer::~Reducer() { remove_hooks(); }

namespace {
// One step stream (and its join event) per device for the process, shared by every reducer: a
// reducer is re-created when the caller switches streams (rebind_if_stream_changed, e.g. at the start
// of a hipGraph capture), and destroying or synchronizing a stream there would invalidate the capture
// (and, as for the communicator's stream, a stream must outlive every buffer used on it).
std::pair<hipStream_t, hipEvent_t> device_step_stream(int dev) {
  static std::mutex mu;
  static std::unordered_map<int, std::pair<hipStream_t, hipEvent_t>> m;
  std::lock_guard<std::mutex> g(mu);
  auto it = m.find(dev);
  if (it != m.end()) return it->second;
  hipStream_t s = nullptr;
  hipEvent_t e = nullptr;
  TORCH_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, 0) == hipSuccess &&
                  hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess,
              "reducer: step stream creation failed");
  m[dev] = {s, e};
  return m[dev];
}
}  // namespace

void Reducer::set_bucket_step(int64_t b, at::Tensor p, at::Tensor g, c10::optional<at::Tensor> buf,
                              c10::optional<at::Tensor> lr_t, double lr, double momentum, double dampening, double wd,
                              bool nesterov, bool first, bool maximize, c10::optional<at::Tensor> desc,
                              c10::optional<at::Tensor> meta, c10::optional<at::Tensor> amax,
                              c10::optional<at::Tensor> counter) {
  std::lock_guard<std::mutex> gl(mu_);
  TORCH_CHECK(rccl_, "overlapped optimizer step: needs the RCCL communicator (stream-ordered collectives)");
  TORCH_CHECK(b >= 0 && b < (int64_t)bucket_views_.size(), "set_bucket_step: bad bucket ", b);
  TORCH_CHECK(g.data_ptr() == bucket_views_[b].data_ptr() && g.numel() == bucket_views_[b].numel(),
              "set_bucket_step: the gradient range must be bucket ", b, "'s own arena range");
  TORCH_CHECK(p.is_cuda() && p.numel() == g.numel() && p.is_contiguous(), "set_bucket_step: parameter range");
  TORCH_CHECK(!desc.has_value() || (meta.has_value() && amax.has_value()), "set_bucket_step: incomplete prep plan");
  if (steps_.size() != bucket_views_.size()) steps_.assign(bucket_views_.size(), BucketStep{});
  BucketStep& s = steps_[b];
  s.set = true;
  s.p = std::move(p);
  s.g = std::move(g);
  s.buf = std::move(buf);
  s.lr_t = std::move(lr_t);
  s.lr = lr;
  s.momentum = momentum;
  s.dampening = dampening;
  s.wd = wd;
  s.nesterov = nesterov;
  s.first = first;
  s.maximize = maximize;
  s.desc = std::move(desc);
  s.meta = std::move(meta);
  s.amax = std::move(amax);
  s.counter = std::move(counter);
}

// The SGD of bucket b on the step stream, ordered after b's all-reduce (its completion event). The
// parameters of b are no longer read by this backward: a bucket is launched only after every one of
// its gradients is ready, i.e. after the backward kernels of those layers (data gradient included,
// both are enqueued before autograd accumulates the weight gradient) were enqueued on the compute
// stream, and the all-reduce is ordered after them.
void Reducer::run_step(int b) {
  BucketStep& s = steps_[b];
  const int dev = s.p.get_device();
  if (!step_stream_) std::tie(step_stream_, step_done_) = device_step_stream(dev);
  TORCH_CHECK(hipStreamWaitEvent(step_stream_, works_[b]->event(), 0) == hipSuccess, "reducer: step stream wait");
  {
    c10::hip::HIPStreamGuard guard(c10::hip::getStreamFromExternal(step_stream_, (c10::DeviceIndex)dev));
    if (roctx_) {
      char name[48];
      std::snprintf(name, sizeof(name), "cdp.bucket_step[%d]", b);
      roctxRangePushA(name);
    }
    if (s.desc.has_value())
      sgd_step_prep(s.p, s.g, s.buf, s.lr_t, s.lr, s.momentum, s.dampening, s.wd, 1.0, s.nesterov, s.first, s.maximize,
                    *s.desc, *s.meta, *s.amax, s.counter);
    else
      sgd_step(s.p, s.g, s.buf, s.lr_t, s.lr, s.momentum, s.dampening, s.wd, 1.0, s.nesterov, s.first, s.maximize,
               s.counter);
    if (roctx_) roctxRangePop();
  }
  if (trace_) log_event("s", (int64_t)b);
  ++stepped_now_;
}

void Reducer::log_event(const char* kind, int64_t idx) {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  trace_log_.emplace_back(kind, idx, (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec);
}

void Reducer::remove_hooks() {
  for (size_t i = 0; i < accumulators_.size(); ++i) accumulators_[i]->del_post_hook(hook_keys_[i]);
  accumulators_.clear();
  hook_keys_.clear();
}

void Reducer::reset_state() {
  for (size_t b = 0; b < pending_.size(); ++b) pending_[b] = bucket_size_[b];
  std::fill(ready_flag_.begin(), ready_flag_.end(), 0);
  next_launch_ = 0;
  callback_queued_ = false;
  stepped_now_ = 0;
  for (auto& w : works_) w.reset();
  for (auto& w : pg_works_) w.reset();
}

void Reducer::prepare_for_backward(const std::vector<at::Tensor>& outputs) {
  std::lock_guard<std::mutex> g(mu_);
  TORCH_CHECK(!armed_ || next_launch_ == 0,
              "Expected to have finished reduction in the prior iteration before starting a new one. Some "
              "parameters did not receive gradients; pass find_unused_parameters=True or make sure every output "
              "participates in the loss.");
  reset_state();
  armed_ = true;
  if (!find_unused_) return;
  // Traverse the autograd graph from the outputs; parameters whose AccumulateGrad node is not
  // reachable will never fire their hook this iteration, so mark them ready right away.
  std::unordered_set<torch::autograd::Node*> seen;
  std::vector<torch::autograd::Node*> stack;
  for (const auto& o : outputs) {
    if (!o.defined() || !o.requires_grad()) continue;
    auto fn = o.grad_fn();
    if (fn && seen.insert(fn.get()).second) stack.push_back(fn.get());
  }
  while (!stack.empty()) {
    auto* n = stack.back();
    stack.pop_back();
    for (const auto& e : n->next_edges()) {
      auto* nn = e.function.get();
      if (nn && seen.insert(nn).second) stack.push_back(nn);
    }
  }
  unused_.clear();
  for (size_t i = 0; i < params_.size(); ++i)
    if (!seen.count(accumulators_[i].get())) unused_.push_back(i);
  for (size_t i : unused_) mark_ready_locked(i, /*from_hook=*/false);
}

void Reducer::mark_ready(size_t i) {
  std::lock_guard<std::mutex> g(mu_);
  if (!armed_) return;  // e.g. inside no_sync(), or a backward not preceded by a wrapped forward
  mark_ready_locked(i, /*from_hook=*/true);
}

void Reducer::mark_ready_locked(size_t i, bool from_hook) {
  if (ready_flag_[i]) return;  // reentrant / repeated backward through the same param
  ready_flag_[i] = 1;
  if (from_hook) {
    // keep .grad a view of the arena (it may have been replaced, e.g. by zero_grad(set_to_none=True))
    at::Tensor& gref = params_[i].mutable_grad();
    const at::Tensor& view = grad_views_[i];
    if (!gref.defined()) {
      view.zero_();
      gref = view;
    } else if (!gref.is_same(view) && gref.data_ptr() != view.data_ptr()) {
      view.copy_(gref);
      gref = view;
    }
    if (record_order_) order_.push_back((int64_t)i);
    if (trace_) log_event("h", (int64_t)i);
    if (!callback_queued_) {
      callback_queued_ = true;
      torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
    }
  } else {
    at::Tensor& gref = params_[i].mutable_grad();
    if (!gref.defined()) {
      grad_views_[i].zero_();
      gref = grad_views_[i];
    }
  }
  const int b = bucket_of_[i];
  if (--pending_[b] == 0 && !defer_) {
    while (next_launch_ < (int)pending_.size() && pending_[next_launch_] == 0) launch(next_launch_++);
  }
}

void Reducer::launch(int b) {
  at::Tensor& v = bucket_views_[b];
  if (trace_) log_event("l", (int64_t)b);
  if (roctx_) {
    char name[48];
    std::snprintf(name, sizeof(name), "cdp.bucket_allreduce[%d]", b);
    roctxRangePushA(name);
  }
  if (rccl_) {
    works_[b] = rccl_->all_reduce(v, average_ ? "avg" : "sum", /*async=*/true);
    if (b < (int)steps_.size() && steps_[b].set) run_step(b);
  } else {
    std::vector<at::Tensor> ts{v};
    pg_works_[b] = pg_->allreduce(ts);
  }
  if (roctx_) roctxRangePop();
  ++launched_total_;
}

int64_t Reducer::join_post_broadcast() {
  std::lock_guard<std::mutex> g(mu_);
  const int64_t n = (int64_t)post_works_.size();
  for (auto& w : post_works_) w->wait();  // orders the current stream after the broadcast
  post_works_.clear();
  return n;
}

void Reducer::finalize() {
  std::lock_guard<std::mutex> g(mu_);
  if (!armed_) return;
  if (trace_) log_event("f", -1);
  // Parameters whose hook never fired (e.g. reached from an output that stays out of the loss)
  // are marked ready FIRST, so the launch loop below counts every bucket -- also in the deferred
  // (calibration) iteration, where marking launches nothing by itself.
  std::string missing;
  for (size_t i = 0; i < params_.size(); ++i)
    if (!ready_flag_[i]) {
      if (find_unused_) mark_ready_locked(i, false);
      else missing += std::to_string(i) + " ";
    }
  if (!missing.empty()) {
    armed_ = false;
    TORCH_CHECK(false,
                "DistributedDataParallel: parameters with indices [ ", missing,
                "] did not receive gradients in this iteration. Enable find_unused_parameters=True or make sure "
                "all forward outputs participate in the loss.");
  }
  if (defer_) {
    // the timed calibration backward: the bucket launches wait for the GPU to finish it. A
    // collective enqueued while the GPU still runs the backward (the host is ahead of it) was
    // measured to stretch that backward ~6x on MI355X, even at one rank with no RCCL kernel
    // (scripts/diag/queue_prio.py: 0.36 -> 1.9-2.3 ms at 32 images), and it is the
    // compute-only timeline the bucket planner needs
    if (!bucket_views_.empty() && bucket_views_[0].is_cuda())
      TORCH_CHECK(hipStreamSynchronize(c10::hip::getCurrentHIPStream().stream()) == hipSuccess,
                  "reducer: stream synchronize failed");
  }
  while (next_launch_ < (int)pending_.size() && pending_[next_launch_] == 0) launch(next_launch_++);
  TORCH_CHECK(next_launch_ == (int)pending_.size(), "reducer: ", (int)pending_.size() - next_launch_,
              " bucket(s) left unlaunched at the end of backward");
  if (rccl_) {
    // all buckets run in order on the communicator stream: waiting on the last one covers them all
    if (!works_.empty() && works_.back()) works_.back()->wait();
    // the buffer broadcast behind the last bucket: nothing on the compute stream waits for it here
    // (a previous backward's broadcasts nobody joined: the compute stream waits for them first)
    for (auto& w : post_works_) w->wait();
    post_works_.clear();
    for (auto& t : post_bcast_) post_works_.push_back(rccl_->broadcast(t, 0, /*async=*/true));
    post_issued_ += (int64_t)post_bcast_.size();
    if (stepped_now_ > 0) {
      // ... and the bucket steps in order on the step stream: the compute stream (the next forward
      // reads the stepped weights) waits for the last one
      const hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
      TORCH_CHECK(hipEventRecord(step_done_, step_stream_) == hipSuccess &&
                      hipStreamWaitEvent(cur, step_done_, 0) == hipSuccess,
                  "reducer: step stream join failed");
    }
  } else {
    for (size_t b = 0; b < pg_works_.size(); ++b) {
      if (!pg_works_[b]) continue;
      pg_works_[b]->wait();
      if (average_ && world_ > 1) {
        at::Tensor& v = bucket_views_[b];
        if (v.is_cuda())
          scale_launch(v.data_ptr<float>(), v.numel(), 1.f / (float)world_, c10::hip::getCurrentHIPStream().stream());
        else
          v.div_((double)world_);
      }
    }
  }
  if (record_order_) {
    record_order_ = false;
    have_order_ = true;
  }
  ++iterations_;
  armed_ = false;
  next_launch_ = 0;
  stepped_last_ = stepped_now_;
  steps_.clear();  // registered per backward
}

std::vector<int64_t> Reducer::ready_order() const {
  std::lock_guard<std::mutex> g(mu_);
  return have_order_ ? order_ : std::vector<int64_t>{};
}

}  // namespace cdp
