// Native RCCL communicator: one per process/GPU, its own normal-priority comm stream, stream-ordered
// collectives, and a watchdog thread that aborts the communicator when a collective outlives
// its timeout (the reference has no failure detection at all: a dead rank hangs gloo forever,
// SURVEY.md §5.3).
#pragma once
#include <ATen/ATen.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace cdp {

class RcclComm;

// A pooled HIP event, returned to its communicator's pool when the last owner drops it.
// Holds only a weak reference so the watchdog's pending list never owns the communicator.
struct PooledEvent {
  PooledEvent(std::weak_ptr<RcclComm> c, hipEvent_t e) : comm(std::move(c)), ev(e) {}
  ~PooledEvent();
  std::weak_ptr<RcclComm> comm;
  hipEvent_t ev;
};

// Completion handle of an asynchronous collective.
class RcclWork {
 public:
  RcclWork(std::shared_ptr<RcclComm> comm, std::shared_ptr<PooledEvent> done, std::vector<at::Tensor> keep)
      : comm_(std::move(comm)), done_(std::move(done)), keep_(std::move(keep)) {}
  // Make the caller's current stream wait for the collective (no host block).
  void wait();
  // Block the host until the collective finished (raises on communicator failure / timeout).
  void synchronize();
  bool is_completed();
  // the completion event (recorded on the communicator stream after the collective)
  hipEvent_t event() const { return done_->ev; }

 private:
  std::shared_ptr<RcclComm> comm_;
  std::shared_ptr<PooledEvent> done_;
  std::vector<at::Tensor> keep_;  // keeps the buffers alive until the work is dropped
};

class RcclComm : public std::enable_shared_from_this<RcclComm> {
 public:
  static std::string unique_id();
  RcclComm(const std::string& uid, int rank, int world, int device, double timeout_s);
  ~RcclComm();

  int rank() const { return rank_; }
  int size() const { return world_; }
  int device() const { return device_; }
  int count();  // ranks in the communicator as RCCL sees them (ncclCommCount)
  hipStream_t stream() const { return stream_; }
  const std::string& stream_kind() const { return stream_kind_; }
  bool healthy() const { return !failed_.load(); }
  std::string error() const;
  void abort(const std::string& why);
  void set_timeout(double s) { timeout_s_ = s; }
  double timeout() const { return timeout_s_.load(); }
  // collectives enqueued while the caller's stream was being captured into a hipGraph (they run
  // at every replay), and collectives enqueued eagerly
  long long captured_collectives() const { return n_captured_.load(); }
  long long eager_collectives() const { return n_eager_.load(); }
  void shutdown();

  std::shared_ptr<RcclWork> all_reduce(at::Tensor t, const std::string& op, bool async);
  std::shared_ptr<RcclWork> broadcast(at::Tensor t, int root, bool async);
  std::shared_ptr<RcclWork> reduce(at::Tensor t, int root, const std::string& op, bool async);
  std::shared_ptr<RcclWork> all_gather(at::Tensor out, at::Tensor in, bool async);
  std::shared_ptr<RcclWork> reduce_scatter(at::Tensor out, at::Tensor in, const std::string& op, bool async);
  std::shared_ptr<RcclWork> gather(at::Tensor t, std::vector<at::Tensor> outs, int root, bool async);
  std::shared_ptr<RcclWork> scatter(at::Tensor t, std::vector<at::Tensor> ins, int root, bool async);
  std::shared_ptr<RcclWork> all_to_all(at::Tensor out, at::Tensor in, bool async);
  std::shared_ptr<RcclWork> send(at::Tensor t, int peer, bool async);
  std::shared_ptr<RcclWork> recv(at::Tensor t, int peer, bool async);
  void barrier();

  // Test hook (CDP_REDUCER_TEST_POSTOP): after every all_reduce, enqueue on the communicator
  // stream a ~delay_us spin followed by x *= scale, *inside* the collective's completion event.
  // A consumer that is not correctly ordered after the collective then reads unscaled data.
  void set_test_postop(double delay_us, double scale) {
    postop_delay_us_ = delay_us;
    postop_scale_ = scale;
  }
  // Modelled-xGMI variant (one GPU standing in for a W-rank node): every all_reduce's post-op
  // spins alpha_us + 2 (W - 1) / W * bytes / (GBps * 1e3) us -- a ring all-reduce's time at that
  // per-link bandwidth -- so bucket timelines and overlap can be measured without peers.
  void set_test_postop_model(double alpha_us, double gbps, int w) {
    postop_alpha_us_ = alpha_us;
    postop_gbps_ = gbps;
    postop_w_ = w;
    postop_scale_ = 1.0;
  }

  hipEvent_t get_event();
  void put_event(hipEvent_t e);
  void check() const;

 private:
  hipStream_t begin();  // order the comm stream after the current stream; returns current stream
  std::shared_ptr<RcclWork> end(hipStream_t cur, bool async, std::vector<at::Tensor> keep, const char* what);
  void watchdog_loop();

  // Atomic: the watchdog's abort() and shutdown() hand the comm off with exchange(nullptr), so
  // exactly one of them frees it, and collectives (which re-check failed_ under mu_) never see
  // a freed comm.
  std::atomic<ncclComm_t> comm_{nullptr};
  double postop_delay_us_ = 0.0, postop_scale_ = 1.0;
  double postop_alpha_us_ = 0.0, postop_gbps_ = 0.0;
  int postop_w_ = 0;
  int rank_, world_, device_;
  hipStream_t stream_ = nullptr;
  std::string stream_kind_;
  hipEvent_t start_ev_ = nullptr;
  std::mutex mu_;
  std::mutex ev_mu_;
  std::vector<hipEvent_t> free_events_;

  struct Pending {
    std::shared_ptr<PooledEvent> ev;
    std::chrono::steady_clock::time_point t0;
    std::string what;
  };
  std::mutex wd_mu_;
  std::deque<Pending> pending_;
  std::thread wd_thread_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> failed_{false};
  std::atomic<long long> n_captured_{0}, n_eager_{0};
  std::atomic<double> timeout_s_;
  mutable std::mutex err_mu_;
  std::string err_;
};

}  // namespace cdp
