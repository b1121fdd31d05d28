#pragma once
#include <ATen/ATen.h>
#include <c10/util/Optional.h>

#include <string>
#include <tuple>
#include <vector>

namespace cdp {

void set_conv_gemm(const std::string& mode);
// tuning sweeps: force the tile / split-K plan of later conv ('conv') or weight-gradient ('wgrad')
// GEMMs (0 = planner's choice); plan_info returns the planner's {bm, bn, splits}
int64_t pair_launches();
void set_gemm_override(const std::string& kind, int64_t bm, int64_t bn, int64_t splits);
std::vector<int64_t> plan_info(const std::string& kind, int64_t M, int64_t N, int64_t K);
std::string get_conv_gemm();
std::vector<at::Tensor> conv2d_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                   int64_t stride, int64_t pad, bool want_stats,
                                   const c10::optional<at::Tensor>& x_amax = c10::nullopt,
                                   const c10::optional<at::Tensor>& w_amax = c10::nullopt);
at::Tensor conv2d_dgrad(const at::Tensor& dy, const at::Tensor& w, std::vector<int64_t> in_shape, int64_t stride,
                        int64_t pad, const c10::optional<at::Tensor>& addend,
                        const c10::optional<at::Tensor>& dy_amax = c10::nullopt,
                        const c10::optional<at::Tensor>& w_amax = c10::nullopt,
                        const c10::optional<at::Tensor>& w_t = c10::nullopt);
at::Tensor conv2d_wgrad(const at::Tensor& dy, const at::Tensor& x, std::vector<int64_t> w_shape, int64_t stride,
                        int64_t pad, const c10::optional<at::Tensor>& out, bool accumulate,
                        const c10::optional<at::Tensor>& dy_amax = c10::nullopt,
                        const c10::optional<at::Tensor>& x_amax = c10::nullopt);
at::Tensor conv2d_wgrad_keep(const at::Tensor& dy, const at::Tensor& x, std::vector<int64_t> w_shape, int64_t stride,
                             int64_t pad, const c10::optional<at::Tensor>& out, bool accumulate, int64_t keep_c,
                             const c10::optional<at::Tensor>& dy_amax = c10::nullopt,
                             const c10::optional<at::Tensor>& x_amax = c10::nullopt);
std::vector<at::Tensor> conv_bn_act_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                        const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                                        const c10::optional<at::Tensor>& running_mean,
                                        const c10::optional<at::Tensor>& running_var,
                                        const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                        double eps, bool training, int64_t stride, int64_t pad, bool pool, bool relu,
                                        const c10::optional<at::Tensor>& residual,
                                        const c10::optional<at::Tensor>& x_amax = c10::nullopt,
                                        const c10::optional<at::Tensor>& w_amax = c10::nullopt,
                                        const c10::optional<at::Tensor>& res_y = c10::nullopt,
                                        const c10::optional<at::Tensor>& res_stats = c10::nullopt,
                                        bool defer_apply = false);
at::Tensor act_max_of(const at::Tensor& t);
int64_t act_max_memsets();
int64_t act_max_copies();
std::vector<std::vector<at::Tensor>> weight_prep(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t);
void weight_prep_into(const std::vector<at::Tensor>& ts, const std::vector<bool>& want_t, const at::Tensor& amax,
                      const std::vector<c10::optional<at::Tensor>>& wts);
std::vector<at::Tensor> conv_bn_act_bwd(const at::Tensor& gout, const at::Tensor& x, const at::Tensor& w,
                                        const at::Tensor& y, const at::Tensor& stats, int64_t stride, int64_t pad,
                                        bool pool, bool relu, bool need_dx, bool has_bias,
                                        const c10::optional<at::Tensor>& zout, bool training,
                                        const c10::optional<at::Tensor>& dw_out,
                                        const c10::optional<at::Tensor>& db_out,
                                        const c10::optional<at::Tensor>& dgamma_out,
                                        const c10::optional<at::Tensor>& dbeta_out,
                                        const c10::optional<at::Tensor>& dx_addend,
                                        const c10::optional<at::Tensor>& x_amax = c10::nullopt,
                                        const c10::optional<at::Tensor>& w_amax = c10::nullopt,
                                        const c10::optional<at::Tensor>& w_t = c10::nullopt,
                                        const c10::optional<at::Tensor>& part_in = c10::nullopt,
                                        const c10::optional<at::Tensor>& prev_y = c10::nullopt,
                                        const c10::optional<at::Tensor>& prev_stats = c10::nullopt,
                                        bool prev_pool = false, bool prev_relu = false, int64_t prev_ps = 2,
                                        const c10::optional<at::Tensor>& bias = c10::nullopt);
at::Tensor linear_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b);
std::vector<at::Tensor> linear_bwd(const at::Tensor& gy, const at::Tensor& x, const at::Tensor& w, bool need_dx,
                                   bool has_bias, const c10::optional<at::Tensor>& dw_out,
                                   const c10::optional<at::Tensor>& db_out);
at::Tensor xent_fwd(const at::Tensor& logits, const at::Tensor& target, const c10::optional<at::Tensor>& correct);
at::Tensor xent_bwd(const at::Tensor& gloss, const at::Tensor& logits, const at::Tensor& target);
std::vector<at::Tensor> xent_linear_bwd(const at::Tensor& gloss, const at::Tensor& logits, const at::Tensor& target,
                                        const at::Tensor& x, const at::Tensor& w, bool need_dx, bool has_bias,
                                        const c10::optional<at::Tensor>& dw_out, const c10::optional<at::Tensor>& db_out,
                                        const c10::optional<at::Tensor>& link_y = c10::nullopt,
                                        const c10::optional<at::Tensor>& link_stats = c10::nullopt,
                                        bool link_pool = false, bool link_relu = false, int64_t link_ps = 2);
std::vector<at::Tensor> sgd_prep_plan(const at::Tensor& flat, int64_t s, int64_t e, const std::vector<at::Tensor>& ws,
                                      const std::vector<bool>& want_t,
                                      const c10::optional<at::Tensor>& amax_out = c10::nullopt,
                                      const std::vector<int64_t>& amax_offsets = {});
void sgd_step_prep(at::Tensor p, const at::Tensor& g, c10::optional<at::Tensor> buf, const c10::optional<at::Tensor>& lr_t,
                   double lr, double momentum, double dampening, double wd, double grad_scale, bool nesterov, bool first,
                   bool maximize, const at::Tensor& desc, const at::Tensor& meta, at::Tensor amax,
                   const c10::optional<at::Tensor>& counter);
void sgd_step(at::Tensor p, const at::Tensor& g, c10::optional<at::Tensor> buf, const c10::optional<at::Tensor>& lr_t,
              double lr, double momentum, double dampening, double wd, double grad_scale, bool nesterov, bool first,
              bool maximize, const c10::optional<at::Tensor>& counter);
at::Tensor augment(const at::Tensor& images, const c10::optional<at::Tensor>& indices, int64_t idx_offset, int64_t batch,
                   std::vector<double> mean, std::vector<double> std_, int64_t pad, bool flip,
                   const c10::optional<at::Tensor>& counter, int64_t seed, c10::optional<at::Tensor> out,
                   int64_t nbatches = 0, const c10::optional<at::Tensor>& labels = c10::nullopt,
                   const c10::optional<at::Tensor>& labels_out = c10::nullopt);
void counter_inc(at::Tensor c);
void stack_mean(const std::vector<at::Tensor>& srcs, at::Tensor dst);
void gpu_sleep(double us);
void gpu_timestamp(at::Tensor ts, int64_t idx);
int64_t gpu_wall_clock_khz();
void scale_(at::Tensor x, double a);
std::vector<at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t p);
at::Tensor maxpool2d_bwd(const at::Tensor& gy, const at::Tensor& arg, std::vector<int64_t> in_shape, int64_t k,
                         int64_t s, int64_t p);
at::Tensor avgpool_fwd(const at::Tensor& x);
at::Tensor avgpool_bwd(const at::Tensor& gy, std::vector<int64_t> in_shape);

// CDP_GEMM_LOG=1: the GEMM launches so far as (kind, M, N, K, bm, bn, splits), in enqueue order
std::vector<std::tuple<std::string, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>> gemm_log(bool clear);

}  // namespace cdp
