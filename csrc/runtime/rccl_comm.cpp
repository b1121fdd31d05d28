// RCCL communicator (see rccl_comm.h). Collective call sites in the reference that this replaces:
//   dist.gather / dist.scatter          /root/reference/src/Part 2a/main.py:121-127
//   dist.all_reduce(SUM)                /root/reference/src/Part 2b/main.py:118
//   DDP broadcast / bucket all-reduce   /root/reference/src/Part 3/main.py:61 (inside torch's Reducer)
// Ordering model: every collective is issued on this communicator's own stream after an event
// recorded on the caller's current stream; synchronous calls make the current stream wait on the
// completion event, asynchronous ones hand that event back as an RcclWork. Nothing blocks the
// host except barrier()/synchronize(), so the calls are hipGraph-capturable.
#include "rccl_comm.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstring>
#include <map>
#include <mutex>

#include "../kernels/kernels.h"
#include <sstream>

namespace cdp {

namespace {

#define RCCL_CHECK(cmd)                                                                     \
  do {                                                                                      \
    ncclResult_t r_ = (cmd);                                                                \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", ncclGetErrorString(r_), " at " #cmd);     \
  } while (0)
#define HIP_CHECK(cmd)                                                                      \
  do {                                                                                      \
    hipError_t e_ = (cmd);                                                                  \
    TORCH_CHECK(e_ == hipSuccess, "HIP error ", hipGetErrorString(e_), " at " #cmd);        \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t);
  }
}

ncclRedOp_t to_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod" || op == "product") return ncclProd;
  TORCH_CHECK(false, "unsupported reduce op: ", op);
}

void check_tensor(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "RCCL collectives need GPU tensors");
  TORCH_CHECK(t.is_contiguous() || t.is_contiguous(at::MemoryFormat::ChannelsLast),
              "RCCL collectives need dense tensors");
}

// The communicator's stream lives as long as the process (one per device and priority, reused by
// later communicators): asynchronous collectives recordStream() their buffers on it, so the caching
// allocator records an event on this stream whenever such a buffer is freed -- possibly after the
// communicator is gone (e.g. a gradient arena collected at interpreter exit), which on a destroyed
// stream crashes inside the HIP runtime. PyTorch's own pool streams are never destroyed either.
hipStream_t process_stream(int device, int priority) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  std::lock_guard<std::mutex> g(mu);
  auto it = streams.find({device, priority});
  if (it != streams.end()) return it->second;
  hipStream_t s = nullptr;
  HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  streams[{device, priority}] = s;
  return s;
}

}  // namespace

PooledEvent::~PooledEvent() {
  if (auto c = comm.lock()) c->put_event(ev);
  else hipEventDestroy(ev);
}

void RcclWork::wait() {
  comm_->check();
  HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), done_->ev, 0));
}

void RcclWork::synchronize() {
  // poll so a watchdog abort surfaces as an error instead of a hang
  while (true) {
    hipError_t e = hipEventQuery(done_->ev);
    if (e == hipSuccess) break;
    TORCH_CHECK(e == hipErrorNotReady, "HIP error while waiting for RCCL work: ", hipGetErrorString(e));
    comm_->check();
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  comm_->check();
}

bool RcclWork::is_completed() { return hipEventQuery(done_->ev) == hipSuccess; }

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device, double timeout_s)
    : rank_(rank), world_(world), device_(device), timeout_s_(timeout_s) {
  TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  HIP_CHECK(hipSetDevice(device));
  // The comm stream is the communicator's own non-blocking stream at NORMAL priority (0): private
  // (PyTorch's pool never hands it to anyone else, unlike a pool stream, which torch.cuda.Stream()
  // returns again after 32 calls) and placed the same way every time. Measured on MI355X
  // (profiles/comm_stream_priority_r5.md, VGG-11 at 32 images, one rank):
  //  * eager DDP backward span: own normal-priority stream 414-422 us, PyTorch pool stream 420-441,
  //    a stream at the device's LEAST priority (+1 on ROCm) 2173-2392 us with compute dispatches
  //    40-57 us apart -- the round-4 slowdown: its "own" stream was created at that least priority;
  //  * captured DDP step (RCCL kernel + post-op per bucket): 0.552-0.555 / 0.559-0.565 / 0.553-0.555 ms;
  //  * every side stream kind ran on its own hardware queue (rocprofv3 Queue_Id 2, compute on 1).
  // CDP_COMM_STREAM = own (default) | pool | low selects the stream for such A/B runs. (A CU-masked
  // stream kind was dropped: it brought no gain and its diagnostic run crashed at process exit.)
  const char* kind = std::getenv("CDP_COMM_STREAM");
  stream_kind_ = kind && *kind ? kind : "own";
  if (stream_kind_ == "own" || stream_kind_ == "low") {
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    stream_ = process_stream(device, stream_kind_ == "low" ? lo : 0);
  } else {
    TORCH_CHECK(stream_kind_ == "pool", "CDP_COMM_STREAM must be own, pool or low");
    stream_ = c10::hip::getStreamFromPool(/*isHighPriority=*/false, (c10::DeviceIndex)device).stream();
  }
  HIP_CHECK(hipEventCreateWithFlags(&start_ev_, hipEventDisableTiming));
  ncclComm_t c = nullptr;
  RCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  comm_.store(c);
  wd_thread_ = std::thread([this] { watchdog_loop(); });
}

void RcclComm::shutdown() {
  if (stop_.exchange(true)) return;
  if (wd_thread_.joinable()) {
    if (wd_thread_.get_id() == std::this_thread::get_id()) wd_thread_.detach();
    else wd_thread_.join();
  }
  {
    std::lock_guard<std::mutex> g(wd_mu_);
    pending_.clear();
  }
  std::lock_guard<std::mutex> g(mu_);  // no collective is mid-enqueue while the comm is torn down
  if (ncclComm_t c = comm_.exchange(nullptr)) {
    if (failed_.load()) ncclCommAbort(c);
    else ncclCommDestroy(c);
  }
}

RcclComm::~RcclComm() {
  shutdown();
  {
    std::lock_guard<std::mutex> g(ev_mu_);
    for (auto e : free_events_) hipEventDestroy(e);
    free_events_.clear();
  }
  if (start_ev_) hipEventDestroy(start_ev_);
  // (the stream is the process's, see process_stream; a pool stream belongs to PyTorch)
}

std::string RcclComm::error() const {
  std::lock_guard<std::mutex> g(err_mu_);
  return err_;
}

void RcclComm::check() const {
  if (failed_.load()) TORCH_CHECK(false, "RCCL communicator failed: ", error());
}

void RcclComm::abort(const std::string& why) {
  {
    std::lock_guard<std::mutex> g(err_mu_);
    if (err_.empty()) err_ = why;
  }
  if (failed_.exchange(true)) return;  // first caller only
  // From here on every collective fails its check() under mu_ before touching comm_. Wait (bounded)
  // for a collective that is mid-enqueue to leave RCCL, so the comm is not freed under it. If the
  // holder stays inside RCCL (blocked on a dead peer, e.g. p2p connection setup), abort anyway:
  // ncclCommAbort is what unblocks it, and it re-checks failed_ on return.
  std::unique_lock<std::mutex> g(mu_, std::defer_lock);
  const auto t0 = std::chrono::steady_clock::now();
  while (!g.try_lock() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  if (ncclComm_t c = comm_.exchange(nullptr)) ncclCommAbort(c);
}

hipEvent_t RcclComm::get_event() {
  std::lock_guard<std::mutex> g(ev_mu_);
  if (!free_events_.empty()) {
    hipEvent_t e = free_events_.back();
    free_events_.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

void RcclComm::put_event(hipEvent_t e) {
  std::lock_guard<std::mutex> g(ev_mu_);
  free_events_.push_back(e);
}

hipStream_t RcclComm::begin() {
  check();
  TORCH_CHECK(comm_ != nullptr, "RCCL communicator is shut down");
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  // the caller's work must not BE the comm stream (e.g. a PyTorch pool stream handed out again by
  // torch.cuda.Stream()): the wait below would then order it behind itself, and unrelated work
  // would queue behind the collectives
  TORCH_CHECK(cur != stream_, "RCCL communicator: the current stream is the communicator's own stream (",
              stream_kind_, "); run compute on another stream");
  HIP_CHECK(hipEventRecord(start_ev_, cur));
  HIP_CHECK(hipStreamWaitEvent(stream_, start_ev_, 0));
  return cur;
}

std::shared_ptr<RcclWork> RcclComm::end(hipStream_t cur, bool async, std::vector<at::Tensor> keep, const char* what) {
  auto ev = std::make_shared<PooledEvent>(weak_from_this(), get_event());
  HIP_CHECK(hipEventRecord(ev->ev, stream_));
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(cur, &cs);
  const bool captured = cs != hipStreamCaptureStatusNone;
  (captured ? n_captured_ : n_eager_).fetch_add(1);
  if (!async) {
    HIP_CHECK(hipStreamWaitEvent(cur, ev->ev, 0));
  } else if (!captured) {
    // the caching allocator must not recycle these blocks before the comm stream is done
    auto s = c10::hip::getStreamFromExternal(stream_, device_);
    for (auto& t : keep) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), s);
  }
  if (!captured) {
    std::lock_guard<std::mutex> g(wd_mu_);
    pending_.push_back({ev, std::chrono::steady_clock::now(), what});
  }
  return std::make_shared<RcclWork>(shared_from_this(), ev, async ? std::move(keep) : std::vector<at::Tensor>{});
}

void RcclComm::watchdog_loop() {
  hipSetDevice(device_);
  // This thread only polls events. Opt it out of global-mode capture checks: otherwise a
  // hipEventQuery here while the main thread captures a hipGraph (torch.cuda.graph uses the
  // global mode) would invalidate that capture.
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  hipThreadExchangeStreamCaptureMode(&mode);
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    std::string timed_out;
    {
      std::lock_guard<std::mutex> g(wd_mu_);
      while (!pending_.empty()) {
        auto& p = pending_.front();
        hipError_t e = hipEventQuery(p.ev->ev);
        if (e == hipSuccess) {
          pending_.pop_front();
          continue;
        }
        const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - p.t0).count();
        if (age > timeout_s_.load()) {
          std::ostringstream os;
          os << "collective '" << p.what << "' on rank " << rank_ << " did not complete within " << timeout_s_.load()
             << " s (a peer rank is dead or stuck)";
          timed_out = os.str();
        }
        break;
      }
    }
    ncclComm_t c = comm_.load();  // only this thread and shutdown() (which joined it) free the comm
    if (c && !failed_.load()) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        timed_out = std::string("asynchronous RCCL error: ") + ncclGetErrorString(ae);
    }
    if (!timed_out.empty()) {
      abort(timed_out);
      std::lock_guard<std::mutex> g(wd_mu_);
      pending_.clear();
    }
  }
}

std::shared_ptr<RcclWork> RcclComm::all_reduce(at::Tensor t, const std::string& op, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  // one rank: an in-place all-reduce (and broadcast / reduce below) is the identity, so no RCCL
  // kernel is issued (the stream ordering and the work object stay). At world size 1 RCCL's
  // kernels were measured to hold back the compute stream's dispatches for ~50 us each
  // (scripts/diag/ready_timing.py); the test post-op keeps the collective so its ordering tests run.
  const bool model = postop_w_ > 1 && postop_gbps_ > 0.0;
  const bool postop = postop_delay_us_ > 0.0 || postop_scale_ != 1.0 || model;
  if (world_ > 1 || postop)
    RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_op(op), comm_, stream_));
  if (postop) {
    TORCH_CHECK(t.scalar_type() == at::kFloat, "test post-op needs fp32 tensors");
    double delay = postop_delay_us_;
    if (model)
      delay = postop_alpha_us_ + 2.0 * (postop_w_ - 1) / postop_w_ * (double)t.numel() * 4.0 / (postop_gbps_ * 1e3);
    delay_scale_launch(t.data_ptr<float>(), t.numel(), (float)postop_scale_, delay, stream_);
  }
  return end(cur, async, {t}, "all_reduce");
}

std::shared_ptr<RcclWork> RcclComm::broadcast(at::Tensor t, int root, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  if (world_ > 1)
    RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
  // modelled-xGMI test mode (set_test_postop_model): a pipelined broadcast costs about
  // alpha + bytes / B; the pure delay kernel touches no data (any dtype)
  if (postop_w_ > 1 && postop_gbps_ > 0.0)
    delay_scale_launch(nullptr, 0, 1.f, postop_alpha_us_ + (double)t.nbytes() / (postop_gbps_ * 1e3), stream_);
  return end(cur, async, {t}, "broadcast");
}

std::shared_ptr<RcclWork> RcclComm::reduce(at::Tensor t, int root, const std::string& op, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  if (world_ > 1)
    RCCL_CHECK(ncclReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_op(op), root, comm_,
                          stream_));
  return end(cur, async, {t}, "reduce");
}

std::shared_ptr<RcclWork> RcclComm::all_gather(at::Tensor out, at::Tensor in, bool async) {
  check_tensor(out);
  check_tensor(in);
  TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: output must hold world_size inputs");
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  RCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, stream_));
  return end(cur, async, {out, in}, "all_gather");
}

std::shared_ptr<RcclWork> RcclComm::reduce_scatter(at::Tensor out, at::Tensor in, const std::string& op, bool async) {
  check_tensor(out);
  check_tensor(in);
  TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: input must hold world_size outputs");
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  RCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()), to_op(op), comm_,
                               stream_));
  return end(cur, async, {out, in}, "reduce_scatter");
}

// Reference-faithful gather (Part 2a): grouped point-to-point receives on the root.
std::shared_ptr<RcclWork> RcclComm::gather(at::Tensor t, std::vector<at::Tensor> outs, int root, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  const size_t bytes = t.numel() * t.element_size();
  std::vector<at::Tensor> keep{t};
  RCCL_CHECK(ncclGroupStart());
  if (rank_ == root) {
    TORCH_CHECK((int)outs.size() == world_, "gather: root needs world_size output tensors");
    for (int r = 0; r < world_; ++r) {
      check_tensor(outs[r]);
      TORCH_CHECK(outs[r].numel() == t.numel(), "gather: output size mismatch");
      keep.push_back(outs[r]);
      if (r == root) copy_bytes_launch(outs[r].data_ptr(), t.data_ptr(), (long long)bytes, stream_);
      else RCCL_CHECK(ncclRecv(outs[r].data_ptr(), t.numel(), to_nccl(t.scalar_type()), r, comm_, stream_));
    }
  } else {
    RCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
  }
  RCCL_CHECK(ncclGroupEnd());
  return end(cur, async, keep, "gather");
}

std::shared_ptr<RcclWork> RcclComm::scatter(at::Tensor t, std::vector<at::Tensor> ins, int root, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  const size_t bytes = t.numel() * t.element_size();
  std::vector<at::Tensor> keep{t};
  RCCL_CHECK(ncclGroupStart());
  if (rank_ == root) {
    TORCH_CHECK((int)ins.size() == world_, "scatter: root needs world_size input tensors");
    for (int r = 0; r < world_; ++r) {
      check_tensor(ins[r]);
      TORCH_CHECK(ins[r].numel() == t.numel(), "scatter: input size mismatch");
      keep.push_back(ins[r]);
      if (r == root) copy_bytes_launch(t.data_ptr(), ins[r].data_ptr(), (long long)bytes, stream_);
      else RCCL_CHECK(ncclSend(ins[r].data_ptr(), t.numel(), to_nccl(t.scalar_type()), r, comm_, stream_));
    }
  } else {
    RCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
  }
  RCCL_CHECK(ncclGroupEnd());
  return end(cur, async, keep, "scatter");
}

std::shared_ptr<RcclWork> RcclComm::all_to_all(at::Tensor out, at::Tensor in, bool async) {
  check_tensor(out);
  check_tensor(in);
  TORCH_CHECK(in.numel() == out.numel() && in.numel() % world_ == 0, "all_to_all: equal, divisible sizes required");
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  const int64_t chunk = in.numel() / world_;
  const size_t esz = in.element_size();
  RCCL_CHECK(ncclGroupStart());
  for (int r = 0; r < world_; ++r) {
    RCCL_CHECK(ncclSend(static_cast<char*>(in.data_ptr()) + r * chunk * esz, chunk, to_nccl(in.scalar_type()), r,
                        comm_, stream_));
    RCCL_CHECK(ncclRecv(static_cast<char*>(out.data_ptr()) + r * chunk * esz, chunk, to_nccl(in.scalar_type()), r,
                        comm_, stream_));
  }
  RCCL_CHECK(ncclGroupEnd());
  return end(cur, async, {out, in}, "all_to_all");
}

std::shared_ptr<RcclWork> RcclComm::send(at::Tensor t, int peer, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  RCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
  return end(cur, async, {t}, "send");
}

std::shared_ptr<RcclWork> RcclComm::recv(at::Tensor t, int peer, bool async) {
  check_tensor(t);
  std::lock_guard<std::mutex> g(mu_);
  hipStream_t cur = begin();
  RCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
  return end(cur, async, {t}, "recv");
}

int RcclComm::count() {
  std::lock_guard<std::mutex> g(mu_);
  check();
  ncclComm_t c = comm_.load();
  TORCH_CHECK(c != nullptr, "RCCL communicator is shut down");
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  return n;
}

void RcclComm::barrier() {
  at::Tensor t = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
  auto w = all_reduce(t, "sum", true);
  w->synchronize();
}

}  // namespace cdp
