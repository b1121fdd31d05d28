#pragma once
#include <ATen/ATen.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "rccl_comm.h"

namespace cdp {

class Reducer {
 public:
  // params[i] / grad_views[i]: parameter i and its arena-backed gradient view.
  // bucket_views[b]: flat arena range of bucket b (launch order), covering parameter indices
  // [bucket_starts[b], bucket_starts[b+1]) (either direction).
  Reducer(std::vector<at::Tensor> params, std::vector<at::Tensor> grad_views, std::vector<at::Tensor> bucket_views,
          std::vector<int64_t> bucket_starts, std::shared_ptr<RcclComm> rccl, c10::intrusive_ptr<c10d::ProcessGroup> pg,
          bool find_unused, bool average);
  ~Reducer();

  void prepare_for_backward(const std::vector<at::Tensor>& outputs);
  void mark_ready(size_t i);
  void finalize();
  void remove_hooks();
  std::vector<int64_t> ready_order() const;
  int64_t iterations() const { return iterations_; }
  int64_t launched_total() const { return launched_total_; }
  int num_buckets() const { return (int)bucket_views_.size(); }
  // Event log for overlap tests/tracing: ('h', param index) when a gradient-ready hook fires,
  // ('l', bucket) when a bucket collective is launched, ('f', -1) at the end-of-backward callback;
  // each with its host CLOCK_MONOTONIC time in ns (same clock as Python's time.monotonic_ns()).
  void set_trace(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    trace_ = on;
    trace_log_.clear();
  }
  std::vector<std::tuple<std::string, int64_t, int64_t>> trace_log() const {
    std::lock_guard<std::mutex> g(mu_);
    return trace_log_;
  }
  // defer: hold every bucket's launch until the end-of-backward callback (the reducer's timed
  // calibration backward, so its ready timeline is the compute's own, free of comm interference)
  void set_defer(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    defer_ = on;
  }
  void disarm() {
    std::lock_guard<std::mutex> g(mu_);
    armed_ = false;
    steps_.clear();
    post_works_.clear();  // a failed capture's broadcasts never ran
    post_issued_ = 0;
  }
  // Overlapped optimizer step (opt-in, RCCL path): the SGD of bucket b's arena range is enqueued on
  // the reducer's own step stream right behind b's all-reduce, so it runs while later buckets are
  // still being reduced (and backward still computes), instead of after the last one. Registered
  // per backward (the hyperparameters / first-step flag of that iteration); the end-of-backward
  // callback orders the compute stream after the last bucket's step and drops the registrations.
  void set_bucket_step(int64_t b, at::Tensor p, at::Tensor g, c10::optional<at::Tensor> buf,
                       c10::optional<at::Tensor> lr_t, double lr, double momentum, double dampening, double wd,
                       bool nesterov, bool first, bool maximize, c10::optional<at::Tensor> desc,
                       c10::optional<at::Tensor> meta, c10::optional<at::Tensor> amax, c10::optional<at::Tensor> counter);
  void clear_bucket_steps() {
    std::lock_guard<std::mutex> g(mu_);
    steps_.clear();
  }
  // buckets whose step ran in the last completed backward
  int64_t stepped_buckets() const { return stepped_last_; }
  // Early buffer broadcast (opt-in, RCCL path): rank 0's module buffers are broadcast on the comm
  // stream right behind the last bucket at the end of every synced backward, instead of at the start
  // of the next forward; the compute stream does not wait for them there. join_post_broadcast()
  // makes the current stream wait for the pending broadcasts (the optimizer step's end or the next
  // forward calls it) and returns how many it joined. An empty list turns it off.
  void set_post_broadcast(std::vector<at::Tensor> ts) {
    std::lock_guard<std::mutex> g(mu_);
    post_bcast_ = std::move(ts);
  }
  int64_t join_post_broadcast();
  // broadcasts issued by the backwards since the last call (the next forward skips its own then)
  int64_t take_post_issued() {
    std::lock_guard<std::mutex> g(mu_);
    const int64_t n = post_issued_;
    post_issued_ = 0;
    return n;
  }

 private:
  void reset_state();
  void mark_ready_locked(size_t i, bool from_hook);
  void launch(int b);
  void run_step(int b);

  struct BucketStep {
    bool set = false;
    at::Tensor p, g;
    c10::optional<at::Tensor> buf, lr_t, desc, meta, amax, counter;
    double lr = 0, momentum = 0, dampening = 0, wd = 0;
    bool nesterov = false, first = false, maximize = false;
  };
  std::vector<BucketStep> steps_;
  std::vector<at::Tensor> post_bcast_;
  std::vector<std::shared_ptr<RcclWork>> post_works_;
  int64_t post_issued_ = 0;
  hipStream_t step_stream_ = nullptr;
  hipEvent_t step_done_ = nullptr;
  int64_t stepped_now_ = 0, stepped_last_ = 0;

  std::vector<at::Tensor> params_, grad_views_, bucket_views_;
  std::shared_ptr<RcclComm> rccl_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  bool find_unused_, average_;
  int world_ = 1;
  std::vector<int> bucket_of_, bucket_size_, pending_;
  std::vector<char> ready_flag_;
  std::vector<std::shared_ptr<RcclWork>> works_;
  std::vector<c10::intrusive_ptr<c10d::Work>> pg_works_;
  std::vector<std::shared_ptr<torch::autograd::Node>> accumulators_;
  std::vector<uintptr_t> hook_keys_;
  std::vector<size_t> unused_;
  std::vector<int64_t> order_;
  mutable std::mutex mu_;
  int next_launch_ = 0;
  bool armed_ = false, callback_queued_ = false, record_order_ = true, have_order_ = false;
  int64_t iterations_ = 0, launched_total_ = 0;
  bool trace_ = false;
  bool defer_ = false;
  bool roctx_ = false;  // CDP_ROCTX=1: roctx range per bucket launch (rocprofv3 --marker-trace)
  std::vector<std::tuple<std::string, int64_t, int64_t>> trace_log_;  // (kind, index, CLOCK_MONOTONIC ns)
  void log_event(const char* kind, int64_t idx);
};

}  // namespace cdp
