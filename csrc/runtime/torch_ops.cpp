// The gfx950 kernels as PyTorch custom ops: torch.ops.cdp.*
//
// Schema-registered (TORCH_LIBRARY) so the ops are visible to the dispatcher, to TorchScript and
// to torch.compile graphs as opaque calls; the GPU implementations are the same entry points the
// Python autograd Functions use (ops.cpp), and cdp::conv2d / cdp::linear carry C++ autograd
// formulas (Autograd dispatch key), so
//     y = torch.ops.cdp.conv2d(x, w, b, 1, 1); y.sum().backward()
// runs the implicit-GEMM forward, data-gradient and weight-gradient kernels.
//
// Reference anchors: nn.Conv2d(k=3, s=1, p=1) (/root/reference/src/Part 1/model.py:18-23),
// nn.Linear(512, 10) (:40), CrossEntropyLoss (/root/reference/src/Part 1/main.py:110).
#include <torch/autograd.h>
#include <torch/library.h>

#include "../kernels/kernels.h"
#include "ops.h"

namespace cdp {
namespace {

at::Tensor conv2d_cuda(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b, int64_t stride,
                       int64_t pad) {
  return conv2d_fwd(x, w, b, stride, pad, false)[0];
}

at::Tensor conv2d_dgrad_cuda(const at::Tensor& dy, const at::Tensor& w, at::IntArrayRef in_shape, int64_t stride,
                             int64_t pad) {
  return conv2d_dgrad(dy, w, in_shape.vec(), stride, pad, c10::nullopt);
}

at::Tensor conv2d_wgrad_cuda(const at::Tensor& dy, const at::Tensor& x, at::IntArrayRef w_shape, int64_t stride,
                             int64_t pad) {
  return conv2d_wgrad(dy, x, w_shape.vec(), stride, pad, c10::nullopt, false);
}

at::Tensor linear_cuda(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b) {
  return linear_fwd(x, w, b);
}

at::Tensor cross_entropy_cuda(const at::Tensor& logits, const at::Tensor& target) {
  return xent_fwd(logits, target, c10::nullopt);
}

std::tuple<at::Tensor, at::Tensor> max_pool2d_cuda(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  auto r = maxpool2d_fwd(x, k, s, p);
  return {r[0], r[1]};
}

// ---------------------------------------------------------------- autograd formulas
class Conv2dFn : public torch::autograd::Function<Conv2dFn> {
 public:
  static at::Tensor forward(torch::autograd::AutogradContext* ctx, const at::Tensor& x, const at::Tensor& w,
                            const c10::optional<at::Tensor>& b, int64_t stride, int64_t pad) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->save_for_backward({x, w});
    ctx->saved_data["stride"] = stride;
    ctx->saved_data["pad"] = pad;
    ctx->saved_data["has_bias"] = b.has_value() && b->defined();
    static auto op = c10::Dispatcher::singleton().findSchemaOrThrow("cdp::conv2d", "").typed<decltype(conv2d_cuda)>();
    return op.call(x, w, b, stride, pad);
  }

  static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::variable_list gy) {
    auto saved = ctx->get_saved_variables();
    const at::Tensor &x = saved[0], &w = saved[1];
    const int64_t stride = ctx->saved_data["stride"].toInt(), pad = ctx->saved_data["pad"].toInt();
    const at::Tensor dy = gy[0].contiguous(at::MemoryFormat::ChannelsLast);
    at::Tensor dx = conv2d_dgrad(dy, w, x.sizes().vec(), stride, pad, c10::nullopt);
    at::Tensor dw = conv2d_wgrad(dy, x, w.sizes().vec(), stride, pad, c10::nullopt, false);
    at::Tensor db;
    if (ctx->saved_data["has_bias"].toBool()) db = dy.sum({0, 2, 3});
    return {dx, dw, db, at::Tensor(), at::Tensor()};
  }
};

at::Tensor conv2d_autograd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                           int64_t stride, int64_t pad) {
  return Conv2dFn::apply(x, w, b, stride, pad);
}

class LinearFn : public torch::autograd::Function<LinearFn> {
 public:
  static at::Tensor forward(torch::autograd::AutogradContext* ctx, const at::Tensor& x, const at::Tensor& w,
                            const c10::optional<at::Tensor>& b) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->save_for_backward({x, w});
    ctx->saved_data["has_bias"] = b.has_value() && b->defined();
    return linear_fwd(x, w, b);
  }

  static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::variable_list gy) {
    auto saved = ctx->get_saved_variables();
    const bool has_bias = ctx->saved_data["has_bias"].toBool();
    auto r = linear_bwd(gy[0].contiguous(), saved[0], saved[1], true, has_bias, c10::nullopt, c10::nullopt);
    return {r[0], r[1], has_bias ? r[2] : at::Tensor()};
  }
};

at::Tensor linear_autograd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b) {
  return LinearFn::apply(x, w, b);
}

}  // namespace

TORCH_LIBRARY(cdp, m) {
  m.def("conv2d(Tensor x, Tensor w, Tensor? bias, int stride, int pad) -> Tensor");
  m.def("conv2d_dgrad(Tensor dy, Tensor w, int[] in_shape, int stride, int pad) -> Tensor");
  m.def("conv2d_wgrad(Tensor dy, Tensor x, int[] w_shape, int stride, int pad) -> Tensor");
  m.def("linear(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("cross_entropy(Tensor logits, Tensor target) -> Tensor");
  m.def("max_pool2d(Tensor x, int k, int s, int p) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(cdp, CUDA, m) {
  m.impl("conv2d", &conv2d_cuda);
  m.impl("conv2d_dgrad", &conv2d_dgrad_cuda);
  m.impl("conv2d_wgrad", &conv2d_wgrad_cuda);
  m.impl("linear", &linear_cuda);
  m.impl("cross_entropy", &cross_entropy_cuda);
  m.impl("max_pool2d", &max_pool2d_cuda);
}

TORCH_LIBRARY_IMPL(cdp, Autograd, m) {
  m.impl("conv2d", &conv2d_autograd);
  m.impl("linear", &linear_autograd);
}

}  // namespace cdp
