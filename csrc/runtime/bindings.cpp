// Python bindings of the native runtime: kernels (ops.cpp), RCCL communicator, bucketed reducer.
#include <torch/csrc/utils/pybind.h>
#include <torch/extension.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include "ops.h"
#include "rccl_comm.h"
#include "reducer.h"

namespace py = pybind11;
using namespace cdp;

namespace {
// Diagnostics (CDP_SEGV_BT=1 at import): print the native stack of a SIGSEGV to stderr, then die
// with the default action. Host-side only; no debugger attaches to the GPU process.
void segv_backtrace(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "[cdp] native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  if (const char* bt = std::getenv("CDP_SEGV_BT"); bt && bt[0] == '1') signal(SIGSEGV, segv_backtrace);
  m.doc() = "cs744_distributed_data_parallel_amd native runtime (gfx950 kernels, RCCL comm, reducer)";
  m.attr("ARCH") = "gfx950";

  // -------------------------------------------------------------- kernels
  m.def("set_conv_gemm", &set_conv_gemm, py::arg("mode"),
        "select the conv GEMM engine: x3 (3-term bf16 split), f16x2 (scaled 2-term fp16 split), f32 (exact fp32 "
        "MFMA) or bf16 (bf16 operands, non-parity)");
  m.def("get_conv_gemm", &get_conv_gemm);
  m.def("set_gemm_override", &set_gemm_override, py::arg("kind"), py::arg("bm") = 0, py::arg("bn") = 0,
        py::arg("splits") = 0, "force the tile / split-K plan of later GEMMs (tuning sweeps; zeros restore the planner)");
  m.def("pair_launches", &pair_launches, "paired data/weight-gradient launches issued so far");
  m.def("plan_info", &plan_info, py::arg("kind"), py::arg("M"), py::arg("N"), py::arg("K"));
  m.def("clear_hip_error", [] { return std::string(hipGetErrorName(hipGetLastError())); },
        "reset the thread's last HIP error (e.g. after an invalidated stream capture) and return its name");
  m.def("conv2d_fwd", &conv2d_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"), py::arg("pad"),
        py::arg("want_stats") = false, py::arg("x_amax") = py::none(), py::arg("w_amax") = py::none());
  m.def("conv2d_dgrad", &conv2d_dgrad, py::arg("dy"), py::arg("w"), py::arg("in_shape"), py::arg("stride"),
        py::arg("pad"), py::arg("addend") = py::none(), py::arg("dy_amax") = py::none(), py::arg("w_amax") = py::none(),
        py::arg("w_t") = py::none());
  m.def("conv2d_wgrad", &conv2d_wgrad, py::arg("dy"), py::arg("x"), py::arg("w_shape"), py::arg("stride"),
        py::arg("pad"), py::arg("out") = py::none(), py::arg("accumulate") = false, py::arg("dy_amax") = py::none(),
        py::arg("x_amax") = py::none());
  m.def("conv_bn_act_fwd", &conv_bn_act_fwd, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("gamma"),
        py::arg("beta"), py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches_tracked"),
        py::arg("momentum"), py::arg("eps"), py::arg("training"), py::arg("stride"), py::arg("pad"), py::arg("pool"),
        py::arg("relu"), py::arg("residual"), py::arg("x_amax") = py::none(), py::arg("w_amax") = py::none(),
        py::arg("res_y") = py::none(), py::arg("res_stats") = py::none(), py::arg("defer_apply") = false,
        "fused conv + BN [+ residual] [+ ReLU] [+ 2x2 max-pool] forward; returns (out, y, stats, x_saved, out_amax, "
        "x_amax, w_amax, relu_mask). defer_apply: statistics only, out a shape-only placeholder; res_y / res_stats: "
        "the residual as such a deferred branch's raw output and stats, normalized inside this block's apply pass");
  m.def("act_max", &act_max_of, py::arg("t"),
        "f16x2 engine: an activation's per-image / per-channel |max| slots by the standalone pass (int32 [N + "
        "copies * C], float bits; undefined tensor for other engines)");
  m.def("act_max_memsets", &act_max_memsets, "slot-chunk memsets issued so far (tests)");
  m.def("act_max_copies", &act_max_copies, "per-channel slot copies of an act max");
  m.def("conv_bn_act_bwd", &conv_bn_act_bwd, py::arg("gout"), py::arg("x"), py::arg("w"), py::arg("y"),
        py::arg("stats"), py::arg("stride"), py::arg("pad"), py::arg("pool"), py::arg("relu"), py::arg("need_dx"),
        py::arg("has_bias"), py::arg("zout") = py::none(), py::arg("training") = true, py::arg("dw_out") = py::none(),
        py::arg("db_out") = py::none(), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        py::arg("dx_addend") = py::none(), py::arg("x_amax") = py::none(), py::arg("w_amax") = py::none(),
        py::arg("w_t") = py::none(), py::arg("part_in") = py::none(), py::arg("prev_y") = py::none(),
        py::arg("prev_stats") = py::none(), py::arg("prev_pool") = false, py::arg("prev_relu") = false,
        py::arg("prev_ps") = 2, py::arg("bias") = py::none(),
        "fused block backward; returns (dx, dw, db, dgamma, dbeta, dres, prev_part, dy_amax). prev_* describe the BN whose "
        "output is x: its statistics reduction is then fused into this block's data-gradient reduction and returned "
        "as prev_part (undefined when not fused), which that block's backward takes as part_in");
  m.def("weight_prep_into", &weight_prep_into, py::arg("weights"), py::arg("want_t"), py::arg("amax"), py::arg("wts"),
        "weight_prep writing into existing buffers (a fused-step plan's)");
  m.def("weight_prep", &weight_prep, py::arg("weights"), py::arg("want_t"),
        "one launch per step: conv weights' |max| partials (f16x2; else empty) and W^T [Ci, KH*KW*Co] per weight "
        "with want_t (the data-gradient operand)");
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_bwd", &linear_bwd, py::arg("gy"), py::arg("x"), py::arg("w"), py::arg("need_dx"),
        py::arg("has_bias"), py::arg("dw_out") = py::none(), py::arg("db_out") = py::none());
  m.def("xent_fwd", &xent_fwd, py::arg("logits"), py::arg("target"), py::arg("correct") = py::none());
  m.def("xent_bwd", &xent_bwd);
  m.def("gemm_log", &gemm_log, py::arg("clear") = false,
        "CDP_GEMM_LOG=1: (kind, M, N, K, bm, bn, splits) of every conv / weight-gradient GEMM launch so far");
  m.def("xent_linear_bwd", &xent_linear_bwd, py::arg("gloss"), py::arg("logits"), py::arg("target"), py::arg("x"),
        py::arg("w"), py::arg("need_dx"), py::arg("has_bias"), py::arg("dw_out") = py::none(),
        py::arg("db_out") = py::none(), py::arg("link_y") = py::none(), py::arg("link_stats") = py::none(),
        py::arg("link_pool") = false, py::arg("link_relu") = false, py::arg("link_ps") = 2,
        "CrossEntropy backward + narrow Linear backward in one launch (+ the BN backward partials of the block "
        "that produced the Linear's input, link_*): {dlogits, dx, dw, db, part}");
  m.def("sgd_step", &sgd_step, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr_t"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("grad_scale"), py::arg("nesterov"),
        py::arg("first"), py::arg("maximize"), py::arg("counter") = py::none());
  m.def("sgd_prep_plan", &sgd_prep_plan, py::arg("flat"), py::arg("start"), py::arg("end"), py::arg("weights"),
        py::arg("want_t"), py::arg("amax_out") = py::none(), py::arg("amax_offsets") = std::vector<int64_t>{},
        "plan of the fused SGD + weight-preparation step over an arena range");
  m.def("sgd_step_prep", &sgd_step_prep, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr_t"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("grad_scale"), py::arg("nesterov"),
        py::arg("first"), py::arg("maximize"), py::arg("desc"), py::arg("meta"), py::arg("amax"),
        py::arg("counter") = py::none(),
        "SGD over an arena range that also emits the next step's weight |max| / W^T");
  m.def("augment", &augment, py::arg("images"), py::arg("indices"), py::arg("idx_offset"), py::arg("batch"),
        py::arg("mean"), py::arg("std"), py::arg("pad"), py::arg("flip"), py::arg("counter"), py::arg("seed"),
        py::arg("out") = py::none(), py::arg("nbatches") = 0, py::arg("labels") = py::none(),
        py::arg("labels_out") = py::none(),
        "gather + RandomCrop + flip + normalize one batch (NHWC fp32); nbatches > 0 takes the batch offset from "
        "the step counter; labels_out receives the batch's labels");
  m.def("counter_inc", &counter_inc);
  m.def("stack_mean", &stack_mean);
  m.def("scale_", &scale_);
  m.def("gpu_sleep", &gpu_sleep, py::arg("us"), "idle one workgroup ~us on the current stream");
  m.def("gpu_wall_clock_khz", &gpu_wall_clock_khz);
  m.def("gpu_timestamp", &gpu_timestamp, py::arg("ts"), py::arg("idx"), "ts[idx] = GPU wall clock (100 MHz)");
  m.def("create_stream",
        [](int priority, bool nonblocking, bool cu_mask) {
          hipStream_t st = nullptr;
          if (cu_mask) {
            uint32_t mask[8];
            for (auto& w : mask) w = 0xffffffffu;  // every CU: a stream on a queue of its own
            TORCH_CHECK(hipExtStreamCreateWithCUMask(&st, 8, mask) == hipSuccess, "hipExtStreamCreateWithCUMask failed");
          } else {
            TORCH_CHECK(hipStreamCreateWithPriority(&st, nonblocking ? hipStreamNonBlocking : hipStreamDefault,
                                                    priority) == hipSuccess,
                        "hipStreamCreateWithPriority failed");
          }
          return reinterpret_cast<intptr_t>(st);
        },
        py::arg("priority") = 0, py::arg("nonblocking") = true, py::arg("cu_mask") = false,
        "diagnostics: a raw HIP stream for torch.cuda.ExternalStream; the caller destroys it with "
        "destroy_stream before the process exits (HIP's own teardown must not meet a live CU-masked queue)");
  m.def("destroy_stream", [](intptr_t s) {
    hipStream_t st = reinterpret_cast<hipStream_t>(s);
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess && hipStreamDestroy(st) == hipSuccess,
                "hipStreamDestroy failed");
  });
  m.def("stream_priority_range", [] {
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    return std::vector<int>{lo, hi};
  });
  m.def("maxpool2d_fwd", &maxpool2d_fwd);
  m.def("maxpool2d_bwd", &maxpool2d_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);

  // -------------------------------------------------------------- RCCL
  py::class_<RcclWork, std::shared_ptr<RcclWork>>(m, "RcclWork")
      .def("wait", &RcclWork::wait)
      .def("synchronize", &RcclWork::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("is_completed", &RcclWork::is_completed);

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("unique_id", [] { return py::bytes(RcclComm::unique_id()); })
      .def(py::init([](py::bytes uid, int rank, int world, int device, double timeout) {
             std::string id = uid;  // copy while holding the GIL
             py::gil_scoped_release nogil;
             return std::make_shared<RcclComm>(id, rank, world, device, timeout);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("timeout") = 1800.0)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("stream_ptr", [](RcclComm& c) { return reinterpret_cast<intptr_t>(c.stream()); })
      .def_property_readonly("stream_kind", &RcclComm::stream_kind)
      .def("count", &RcclComm::count)
      .def("healthy", &RcclComm::healthy)
      .def("error", &RcclComm::error)
      .def("abort", &RcclComm::abort)
      .def("shutdown", &RcclComm::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("set_timeout", &RcclComm::set_timeout)
      .def("set_test_postop", &RcclComm::set_test_postop, py::arg("delay_us"), py::arg("scale"),
           "test hook: delay + scale after every all_reduce, inside its completion event")
      .def("set_test_postop_model", &RcclComm::set_test_postop_model, py::arg("alpha_us"), py::arg("gbps"),
           py::arg("world"), "test hook: modelled ring all-reduce time after every all_reduce (one-GPU stand-in)")
      .def("timeout", &RcclComm::timeout)
      .def("captured_collectives", &RcclComm::captured_collectives)
      .def("eager_collectives", &RcclComm::eager_collectives)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("async_op") = false)
      .def("broadcast", &RcclComm::broadcast, py::arg("t"), py::arg("root") = 0, py::arg("async_op") = false)
      .def("reduce", &RcclComm::reduce, py::arg("t"), py::arg("root") = 0, py::arg("op") = "sum",
           py::arg("async_op") = false)
      .def("all_gather", &RcclComm::all_gather, py::arg("out"), py::arg("inp"), py::arg("async_op") = false)
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum",
           py::arg("async_op") = false)
      .def("gather", &RcclComm::gather, py::arg("t"), py::arg("outs"), py::arg("root") = 0,
           py::arg("async_op") = false)
      .def("scatter", &RcclComm::scatter, py::arg("t"), py::arg("ins"), py::arg("root") = 0,
           py::arg("async_op") = false)
      .def("all_to_all", &RcclComm::all_to_all, py::arg("out"), py::arg("inp"), py::arg("async_op") = false)
      .def("send", &RcclComm::send, py::arg("t"), py::arg("peer"), py::arg("async_op") = false)
      .def("recv", &RcclComm::recv, py::arg("t"), py::arg("peer"), py::arg("async_op") = false)
      .def("barrier", &RcclComm::barrier, py::call_guard<py::gil_scoped_release>());

  // -------------------------------------------------------------- reducer
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init<std::vector<at::Tensor>, std::vector<at::Tensor>, std::vector<at::Tensor>, std::vector<int64_t>,
                    std::shared_ptr<RcclComm>, c10::intrusive_ptr<c10d::ProcessGroup>, bool, bool>(),
           py::arg("params"), py::arg("grad_views"), py::arg("bucket_views"), py::arg("bucket_starts"),
           py::arg("rccl"), py::arg("pg"), py::arg("find_unused"), py::arg("average"))
      .def("prepare_for_backward", &Reducer::prepare_for_backward)
      .def("remove_hooks", &Reducer::remove_hooks)
      .def("ready_order", &Reducer::ready_order)
      .def("disarm", &Reducer::disarm)
      .def("set_defer", &Reducer::set_defer)
      .def("set_trace", &Reducer::set_trace)
      .def("trace_log", &Reducer::trace_log)
      .def_property_readonly("iterations", &Reducer::iterations)
      .def_property_readonly("launched_total", &Reducer::launched_total)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def("set_bucket_step", &Reducer::set_bucket_step, py::arg("bucket"), py::arg("p"), py::arg("g"), py::arg("buf"),
           py::arg("lr_t"), py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("nesterov"),
           py::arg("first"), py::arg("maximize"), py::arg("desc") = py::none(), py::arg("meta") = py::none(),
           py::arg("amax") = py::none(), py::arg("counter") = py::none(),
           "SGD over bucket b's arena range, run on the reducer's step stream as soon as b's all-reduce completes "
           "(held for the next backward only)")
      .def("clear_bucket_steps", &Reducer::clear_bucket_steps)
      .def("set_post_broadcast", &Reducer::set_post_broadcast, py::arg("tensors"))
      .def("join_post_broadcast", &Reducer::join_post_broadcast)
      .def("take_post_issued", &Reducer::take_post_issued)
      .def_property_readonly("stepped_buckets", &Reducer::stepped_buckets);
}
