// Python bindings of the pgdist native library (_pgdist_C).
//
// Deliberately torch-header-free: every device buffer crosses the boundary as a
// raw address (tensor.data_ptr()) and the HIP stream as its handle
// (torch.cuda.current_stream().cuda_stream).  Shape/dtype validation lives in
// the typed Python wrappers (pgdist/ops/kernels.py) that call these entry points,
// so this translation unit compiles in seconds and has no ABI coupling to a
// particular PyTorch build.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>

#include <pybind11/stl.h>

#include "runtime/comm.h"
#include "runtime/plan.h"
#include "runtime/runtime.h"

namespace py = pybind11;
typedef unsigned short bf16_t;
typedef uintptr_t P;

// ---- kernel launchers (defined in kernels/*.hip) ----
void launch_bn_fwd_finalize(const float *, int, int, float, const float *, const float *, float,
                            float, float *, float *, long long *, float *, float *, float *, float *,
                            hipStream_t);
void launch_bn_bwd_finalize(const float *, int, int, float, const float *, const float *,
                            const float *, float *, float *, float *, hipStream_t);
void launch_bn_apply(const bf16_t *, const bf16_t *, const float *, const float *, bf16_t *,
                     long long, int, bool, hipStream_t);
void launch_adam_flat(float *, const float *, float *, float *, bf16_t *, long long, const float *,
                      float, float, float, float, float, const unsigned *, const float *, const float *, int,
                      double *, hipStream_t);
void launch_f32_to_bf16(const float *, bf16_t *, long long, hipStream_t);
int dw_fwd_num_partials(int, int, int, int, int);
void dw_set_geom_mode(int);
int dw_geom_mode();
void dw_set_tall_rows(int);
void pw_f8_set_mx(int);
int pw_f8_mx();
void dw_set_small_dgrad(int);
int dw_small_dgrad();
int dw_tall_rows();
int bn_rep();
void bn_fin_arm(const void *desc);
void bn_lz_arm(const void *desc);
void launch_bn_finalize_batch(const void *tab, int n, int maxC, hipStream_t st);
std::string bn_fin_pack(float *, int *, int, int, float, int, const float *, const float *, float, float, float *,
                        float *, long long *, float *, float *, float *, float *, float *, float *, float *);
void bn_set_rep(int rep);
void conv_set_glds(int mode);
int conv_get_glds();
int dw_dgrad_num_partials(int, int, int, int, int);
int dw_wgrad_num_partials(int, int, int, int, int);
void launch_dw_fwd(const bf16_t *, const float *, const float *, int, const bf16_t *, bf16_t *,
                   float *, int, int, int, int, int, hipStream_t);
void launch_dw_dgrad(const bf16_t *, const bf16_t *, const float *, const bf16_t *, const bf16_t *,
                     const float *, const float *, bf16_t *, float *, int, int, int, int, int,
                     float *, hipStream_t);
long long dw_dgrad_wgrad_workspace_floats(int, int, int, int, int);
void launch_dw_wgrad(const bf16_t *, const bf16_t *, const float *, const bf16_t *, const float *,
                     const float *, float *, float *, int, int, int, int, int, hipStream_t);
int pw_gemm_num_partials(int, int, int);
void pwt_trace_set(void *);
void pwb_trace_set(void *);
void pwg_trace_set(void *);
bool pw_bwd_supported(int, int, int);
void pw_bwd_set_min_m(int);
int pw_bwd_num_partials(int, int, int);
long long pw_bwd_wgrad_workspace_floats(int, int, int);
void launch_pw_bwd(int, const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                   const bf16_t *, bf16_t *, const bf16_t *, const float *, const float *, const bf16_t *,
                   const bf16_t *, const bf16_t *, float *, float *, float *, int, int, int, hipStream_t);
bool pw_bwd_recompute_supported(int, int, int);
void launch_wt_transpose(const bf16_t *, bf16_t *, const int *, int, hipStream_t);
void launch_pw_gemm_f8(int, const bf16_t *, const float *, const float *, const uint8_t *, int, const float *,
                       float, bf16_t *, float *, int, int, int, hipStream_t);
void launch_w8_quant(const float *, uint8_t *, float *, const int *, int, hipStream_t);
void launch_pw_gemm(int, int, const bf16_t *, const bf16_t *, const float *, const float *,
                    const float *, const bf16_t *, bf16_t *, const bf16_t *, const float *,
                    const float *, const bf16_t *, float *, int, int, int, bf16_t *, hipStream_t);
long long pw_wgrad_workspace_floats(int, int, int);
void launch_pw_wgrad(const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                     const bf16_t *, const float *, const float *, int, float *, float *, int, int,
                     int, hipStream_t);
long long stem_wgrad_workspace_floats(int, int);
void launch_stem_wgrad(const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                       const bf16_t *, float *, float *, int, int, int, int, hipStream_t);
int stem_fwd_num_partials(int, int, int);
bool launch_stem_fwd(const bf16_t *, const bf16_t *, bf16_t *, float *, int, int, int, int, hipStream_t);
void launch_head(const bf16_t *, const float *, const float *, const float *, const float *,
                 const long long *, int, int, int, int, float, unsigned long long, const float *,
                 int, float, float *, float *, float *, float *, float *, bf16_t *, float *, float *,
                 float *, hipStream_t);
void launch_augment(const unsigned char *, const long long *, const long long *, int, int, int,
                    int, int, const float *, unsigned long long, const float *, long long, bf16_t *,
                    long long *, float *, hipStream_t);
void launch_step_begin(float *, float *, long long, hipStream_t);
int colsum_rows(int);
void launch_wgrad_reduce(float *, int, long long, float *, hipStream_t, bool = false);
void wgrad_reduce_defer(bool on);
void wgrad_reduce_flush(hipStream_t st);
long long bn_part_floats(int, int);
void register_side_stream(hipStream_t);
void launch_reduce_metrics(const float *, const float *, int, double *, hipStream_t);
// ---- dense convolutions (ResNet-50), kernels/conv.hip ----
int conv_fwd_num_partials(int, int, int, int, int, int);
int conv_dgrad_num_partials(int, int, int, int, int, int, int, int);
void launch_conv_fwd(int, const bf16_t *, const float *, const float *, const bf16_t *, bf16_t *, float *, int,
                     int, int, int, int, int, int, int, int, hipStream_t);
void launch_conv_fold_w(const bf16_t *, const float *, const float *, const float *, const float *, bf16_t *, float *,
                        int, int, hipStream_t);
void launch_conv_dgrad_fold(const bf16_t *, const bf16_t *, const bf16_t *, const float *, bf16_t *, const bf16_t *,
                            const float *, const float *, float *, int, int, int, int, int, hipStream_t);
void launch_conv_dgrad(int, const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                       const bf16_t *, bf16_t *, const bf16_t *, const float *, const float *, const bf16_t *,
                       const bf16_t *, const bf16_t *, float *, float *, int, int, int, int, int, int, int, int,
                       int, const uint8_t *, hipStream_t);
long long conv_wgrad_workspace_floats(int, int, int, int, int, int, int, int, int);
void launch_conv_wgrad(const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                       const bf16_t *, const float *, const float *, int, float *, float *, int, int, int, int,
                       int, int, int, int, int, hipStream_t);
void launch_conv_wt(const bf16_t *, bf16_t *, const int *, int, hipStream_t);
void launch_bn_mat(int, const bf16_t *, const bf16_t *, const float *, const float *, const float *, bf16_t *, int, int,
                   hipStream_t);
void launch_res_out(const bf16_t *, const float *, const float *, const bf16_t *, const float *, const float *,
                    bf16_t *, long long, int, const void *, const void *, uint8_t *, hipStream_t);
void launch_maxpool_fwd(const bf16_t *, const float *, const float *, bf16_t *, uint8_t *, int, int, int, int,
                        hipStream_t);
int maxpool_bwd_num_partials(int, int, int);
void launch_maxpool_bwd(const bf16_t *, const uint8_t *, const bf16_t *, const float *, const float *, bf16_t *,
                        float *, int, int, int, int, hipStream_t);
void launch_avgpool(const bf16_t *, float *, int, int, int, hipStream_t);
void launch_head_bwd(const float *, const bf16_t *, const bf16_t *, bf16_t *, float *, int, int, int, hipStream_t);
void launch_softmax_ce(const float *, const long long *, int, int, float, float *, float *, float *, hipStream_t);
long long fc_gemm_workspace_floats(int, int, int);
void launch_fc_gemm(const float *, long long, long long, const float *, long long, long long, const float *, float *,
                    int, int, int, float *, hipStream_t);
void launch_col_sum(const float *, int, int, float *, hipStream_t);
void launch_image_prep(const uint8_t *, const long long *, const long long *, int, int, int, unsigned long long,
                       const float *, bf16_t *, long long *, int, hipStream_t);
void launch_stem_w_s2d(const bf16_t *, bf16_t *, int, hipStream_t);
void launch_s2d_image(const bf16_t *, bf16_t *, int, int, int, hipStream_t);
void launch_conv_fwd_s2d(const bf16_t *, const bf16_t *, bf16_t *, float *, int, int, int, hipStream_t);
long long conv_wgrad_s2d_workspace_floats(int, int, int);
void launch_conv_wgrad_s2d(const bf16_t *, const bf16_t *, const float *, const float *, const float *,
                           const bf16_t *, float *, float *, int, int, int, hipStream_t);

template <typename T>
static T *ptr(P p) { return reinterpret_cast<T *>(p); }
static hipStream_t S(P s) { return reinterpret_cast<hipStream_t>(s); }

static std::string last_error() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? std::string() : std::string(hipGetErrorString(e));
}

PYBIND11_MODULE(_pgdist_C, m) {
  m.doc() = "pgdist native library: gfx950 HIP kernels + C++ runtime";
  m.attr("arch") = "gfx950";
  m.def("last_error", &last_error);
  m.def("colsum_rows", &colsum_rows, "rows of level-1 scratch a wgrad reduction over R partial rows needs");
  m.def("register_side_stream", [](P s) { register_side_stream(S(s)); },
        "give reductions launched on this stream their own arrival counters");
  m.def("bn_part_floats", &bn_part_floats, "floats of workspace a BN finalize over P partial rows needs");

  // ---- BatchNorm ----
  m.def("bn_fwd_finalize", [](P part, int Pn, int C, float count, P gamma, P beta, float eps,
                              float mom, P rm, P rv, P nbt, P mean, P rstd, P scale, P shift, P s) {
    pgdist_rt::run_op([=] {
      launch_bn_fwd_finalize(ptr<float>(part), Pn, C, count, ptr<float>(gamma), ptr<float>(beta), eps,
                             mom, ptr<float>(rm), ptr<float>(rv), ptr<long long>(nbt), ptr<float>(mean),
                             ptr<float>(rstd), ptr<float>(scale), ptr<float>(shift), S(s));
    });
  });
  m.def("bn_bwd_finalize", [](P part, int Pn, int C, float count, P mean, P rstd, P gamma, P coef,
                              P dgamma, P dbeta, P s) {
    pgdist_rt::run_op([=] {
      launch_bn_bwd_finalize(ptr<float>(part), Pn, C, count, ptr<float>(mean), ptr<float>(rstd),
                             ptr<float>(gamma), ptr<float>(coef), ptr<float>(dgamma), ptr<float>(dbeta),
                             S(s));
    });
  });
  m.def("bn_apply", [](P y, P res, P scale, P shift, P out, long long M, int C, bool relu6, P s) {
    pgdist_rt::run_op([=] {
      launch_bn_apply(ptr<bf16_t>(y), ptr<bf16_t>(res), ptr<float>(scale), ptr<float>(shift),
                      ptr<bf16_t>(out), M, C, relu6, S(s));
    });
  });
  // ---- optimizer ----
  m.def("adam_flat", [](P p, P g, P mm, P v, P pb, long long n, P hyper, float b1, float b2,
                        float eps, float wd, float gscale, P skip, P loss, P correct, int B, P acc, P s) {
    pgdist_rt::run_op([=] {
      launch_adam_flat(ptr<float>(p), ptr<float>(g), ptr<float>(mm), ptr<float>(v), ptr<bf16_t>(pb),
                       n, ptr<float>(hyper), b1, b2, eps, wd, gscale, ptr<unsigned>(skip), ptr<float>(loss),
                       ptr<float>(correct), B, ptr<double>(acc), S(s));
    });
  });
  m.def("f32_to_bf16", [](P x, P y, long long n, P s) {
    pgdist_rt::run_op([=] {
      launch_f32_to_bf16(ptr<float>(x), ptr<bf16_t>(y), n, S(s));
    });
  });
  m.def("step_begin", [](P hyper, P zero, long long n, P s) {
    pgdist_rt::run_op([=] { launch_step_begin(ptr<float>(hyper), ptr<float>(zero), n, S(s)); });
  });
  m.def("reduce_metrics", [](P loss, P correct, int B, P acc, P s) {
    pgdist_rt::run_op([=] {
      launch_reduce_metrics(ptr<float>(loss), ptr<float>(correct), B, ptr<double>(acc), S(s));
    });
  });
  // ---- depthwise ----
  m.def("dw_fwd_num_partials", &dw_fwd_num_partials);
  m.def("dw_set_geom_mode", &dw_set_geom_mode);
  m.def("dw_geom_mode", &dw_geom_mode);
  m.def("dw_set_tall_rows", &dw_set_tall_rows);
  m.def("pw_f8_set_mx", &pw_f8_set_mx);
  m.def("pw_f8_mx", &pw_f8_mx);
  m.def("dw_set_small_dgrad", &dw_set_small_dgrad);
  m.def("dw_small_dgrad", &dw_small_dgrad);
  m.def("dw_tall_rows", &dw_tall_rows);
  m.def("bn_rep", &bn_rep, "replica rows of the atomic BN-statistics accumulators");
  m.def("bn_fin_arm", [](P d) { pgdist_rt::run_op([=] { bn_fin_arm(reinterpret_cast<const void *>(d)); }); },
        "arm a device BnFin descriptor for the next BN-statistics producer launch (finalize fused in its tail)");
  m.def("bn_lz_arm", [](P d) { pgdist_rt::run_op([=] { bn_lz_arm(reinterpret_cast<const void *>(d)); }); },
        "arm a device BnFin descriptor for the next BN-parameter consumer launch (lazy finalize in its prologue)");
  m.def("bn_finalize_batch", [](P tab, int n, int maxC, P s) {
    pgdist_rt::run_op([=] { launch_bn_finalize_batch(reinterpret_cast<const void *>(tab), n, maxC, S(s)); });
  }, "finalize every BN of a device table of BnFin descriptor pointers in one launch");
  m.def("bn_fin_pack", [](P acc, P ctr, int rows, int C, float count, int bwd, P gamma, P beta, float eps,
                          float mom, P rm, P rv, P nbt, P mean, P rstd, P scale, P shift, P coef, P dgamma,
                          P dbeta) {
    return py::bytes(bn_fin_pack(ptr<float>(acc), ptr<int>(ctr), rows, C, count, bwd, ptr<float>(gamma),
                                 ptr<float>(beta), eps, mom, ptr<float>(rm), ptr<float>(rv), ptr<long long>(nbt),
                                 ptr<float>(mean), ptr<float>(rstd), ptr<float>(scale), ptr<float>(shift),
                                 ptr<float>(coef), ptr<float>(dgamma), ptr<float>(dbeta)));
  });
  m.def("conv_set_glds", &conv_set_glds, "dense conv staging: 0 register-staged, 2/3 LDS-DMA buffers");
  m.def("conv_get_glds", &conv_get_glds);
  m.def("bn_set_rep", &bn_set_rep, "set the replica rows (large = one row per workgroup: deterministic)");
  m.def("dw_dgrad_num_partials", &dw_dgrad_num_partials);
  m.def("dw_wgrad_num_partials", &dw_wgrad_num_partials);
  m.def("dw_fwd", [](P x, P is, P it, int act, P w, P y, P part, int B, int H, int W, int C,
                     int stride, P s) {
    pgdist_rt::run_op([=] {
      launch_dw_fwd(ptr<bf16_t>(x), ptr<float>(is), ptr<float>(it), act, ptr<bf16_t>(w), ptr<bf16_t>(y),
                    ptr<float>(part), B, H, W, C, stride, S(s));
    });
  });
  m.def("dw_dgrad", [](P g, P ys, P coef, P w, P yp, P ps, P pt, P gout, P part, int B, int H,
                       int W, int C, int stride, P wpart, P s) {
    pgdist_rt::run_op([=] {
      launch_dw_dgrad(ptr<bf16_t>(g), ptr<bf16_t>(ys), ptr<float>(coef), ptr<bf16_t>(w),
                      ptr<bf16_t>(yp), ptr<float>(ps), ptr<float>(pt), ptr<bf16_t>(gout),
                      ptr<float>(part), B, H, W, C, stride, ptr<float>(wpart), S(s));
    });
  });
  m.def("dw_dgrad_wgrad_workspace_floats", &dw_dgrad_wgrad_workspace_floats);
  m.def("dw_wgrad", [](P g, P ys, P coef, P yp, P ps, P pt, P part, P grad, int B, int H, int W,
                       int C, int stride, P s) {
    pgdist_rt::run_op([=] {
      launch_dw_wgrad(ptr<bf16_t>(g), ptr<bf16_t>(ys), ptr<float>(coef), ptr<bf16_t>(yp),
                      ptr<float>(ps), ptr<float>(pt), ptr<float>(part), ptr<float>(grad), B, H, W, C,
                      stride, S(s));
    });
  });
  // ---- pointwise ----
  m.def("pw_gemm_num_partials", &pw_gemm_num_partials);
  m.def("pwt_trace_set", [](P ts) { pwt_trace_set(reinterpret_cast<void *>(ts)); },
        "phase trace buffer of pw_tile ([grid][8] uint64 wall-clock stamps; 0: off; PGDIST_PWT_TRACE builds)");
  m.def("pwb_trace_set", [](P ts) { pwb_trace_set(reinterpret_cast<void *>(ts)); },
        "phase-sum buffer of pw_bwd_fused ([grid][8] uint64; 0: off; PGDIST_PWT_TRACE builds)");
  m.def("pwg_trace_set", [](P ts) { pwg_trace_set(reinterpret_cast<void *>(ts)); },
        "phase trace buffer of pw_wgrad ([grid][8] uint64; 0: off; PGDIST_PWT_TRACE builds)");
  m.def("pw_gemm", [](int pro, int epi, P A, P A2, P pa, P pb, P pc, P W, P out, P Yt, P es, P et,
                      P R, P part, int M, int N, int K, P Aout, P s) {
    pgdist_rt::run_op([=] {
      launch_pw_gemm(pro, epi, ptr<bf16_t>(A), ptr<bf16_t>(A2), ptr<float>(pa), ptr<float>(pb),
                     ptr<float>(pc), ptr<bf16_t>(W), ptr<bf16_t>(out), ptr<bf16_t>(Yt), ptr<float>(es),
                     ptr<float>(et), ptr<bf16_t>(R), ptr<float>(part), M, N, K, ptr<bf16_t>(Aout), S(s));
    });
  });
  m.def("pw_gemm_f8", [](int pro, P A, P pa, P pb, P W8, int ldw8, P wsc, float asc, P out, P part, int M,
                         int N, int K, P s) {
    pgdist_rt::run_op([=] {
      launch_pw_gemm_f8(pro, ptr<bf16_t>(A), ptr<float>(pa), ptr<float>(pb), ptr<uint8_t>(W8), ldw8,
                        ptr<float>(wsc), asc, ptr<bf16_t>(out), ptr<float>(part), M, N, K, S(s));
    });
  });
  m.def("w8_quant", [](P src, P dst, P wsc, P tab, int n, P s) {
    pgdist_rt::run_op([=] {
      launch_w8_quant(ptr<float>(src), ptr<uint8_t>(dst), ptr<float>(wsc), ptr<int>(tab), n, S(s));
    });
  });
  m.def("wt_transpose", [](P src, P dst, P tab, int n, P s) {
    pgdist_rt::run_op([=] {
      launch_wt_transpose(ptr<bf16_t>(src), ptr<bf16_t>(dst), ptr<int>(tab), n, S(s));
    });
  });
  m.def("pw_bwd_supported", &pw_bwd_supported);
  m.def("pw_bwd_set_min_m", &pw_bwd_set_min_m);
  m.def("pw_bwd_num_partials", &pw_bwd_num_partials);
  m.def("pw_bwd_wgrad_workspace_floats", &pw_bwd_wgrad_workspace_floats);
  m.def("pw_bwd_recompute_supported", &pw_bwd_recompute_supported);
  m.def("pw_bwd", [](int epi, P G, P Y, P ca, P cb, P cc, P WT, P out, P Yt, P es, P et, P R, P X, P We,
                     P part, P wpart, P grad, int M, int Kg, int Ng, P s) {
    pgdist_rt::run_op([=] {
      launch_pw_bwd(epi, ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ca), ptr<float>(cb), ptr<float>(cc),
                    ptr<bf16_t>(WT), ptr<bf16_t>(out), ptr<bf16_t>(Yt), ptr<float>(es), ptr<float>(et),
                    ptr<bf16_t>(R), ptr<bf16_t>(X), ptr<bf16_t>(We), ptr<float>(part), ptr<float>(wpart),
                    ptr<float>(grad), M, Kg, Ng, S(s));
    });
  });
  m.def("wgrad_reduce_defer", [](bool on) { pgdist_rt::run_op([=] { wgrad_reduce_defer(on); }); },
        "while on, weight-gradient split reductions are recorded instead of launched");
  m.def("wgrad_reduce_flush", [](P s) { pgdist_rt::run_op([=] { wgrad_reduce_flush(S(s)); }); },
        "launch every recorded weight-gradient reduction (multi-segment launches) on the stream");
  m.def("wgrad_reduce", [](P part, int nsplit, long long n, P grad, P s) {
    pgdist_rt::run_op([=] {
      launch_wgrad_reduce(ptr<float>(part), nsplit, n, ptr<float>(grad), S(s));
    });
  }, "grad[n] = sum of the S split rows of part[S][n] (deterministic, one launch)");
  m.def("pw_wgrad_workspace_floats", &pw_wgrad_workspace_floats);
  m.def("pw_wgrad", [](P G, P Y, P ga, P gb, P gc, P X, P xs, P xt, int xact, P part, P grad, int M,
                       int N, int K, P s) {
    pgdist_rt::run_op([=] {
      launch_pw_wgrad(ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ga), ptr<float>(gb), ptr<float>(gc),
                      ptr<bf16_t>(X), ptr<float>(xs), ptr<float>(xt), xact, ptr<float>(part),
                      ptr<float>(grad), M, N, K, S(s));
    });
  });
  // ---- stem ----
  m.def("stem_fwd_num_partials", &stem_fwd_num_partials);
  m.def("stem_fwd", [](P img, P w, P y, P part, int B, int H, int W, int px, P s) {
    if (px != 0 && px != 1 && px != 2 && px != 4) throw std::invalid_argument("stem_fwd: px must be 0, 1, 2 or 4");
    pgdist_rt::run_op([=] {
      (void)launch_stem_fwd(ptr<bf16_t>(img), ptr<bf16_t>(w), ptr<bf16_t>(y), ptr<float>(part), B, H, W, px, S(s));
    });
  });
  m.def("stem_wgrad_workspace_floats", &stem_wgrad_workspace_floats);
  m.def("stem_wgrad", [](P G, P Y, P ga, P gb, P gc, P img, P part, P grad, int B, int H, int W,
                         int O, P s) {
    pgdist_rt::run_op([=] {
      launch_stem_wgrad(ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ga), ptr<float>(gb), ptr<float>(gc),
                        ptr<bf16_t>(img), ptr<float>(part), ptr<float>(grad), B, H, W, O, S(s));
    });
  });
  // ---- head ----
  m.def("head", [](P y, P sc, P sh, P Wl, P bl, P labels, int B, int HW, int C, int NC, float p,
                   unsigned long long seed, P hyper, int train, float loss_scale, P logits, P loss,
                   P correct, P dlogits, P pd, P g, P part, P dW, P db, P s) {
    pgdist_rt::run_op([=] {
      launch_head(ptr<bf16_t>(y), ptr<float>(sc), ptr<float>(sh), ptr<float>(Wl), ptr<float>(bl),
                  ptr<long long>(labels), B, HW, C, NC, p, seed, ptr<float>(hyper), train, loss_scale,
                  ptr<float>(logits), ptr<float>(loss), ptr<float>(correct), ptr<float>(dlogits),
                  ptr<float>(pd), ptr<bf16_t>(g), ptr<float>(part), ptr<float>(dW), ptr<float>(db), S(s));
    });
  });
  // ---- data ----
  m.def("augment", [](P src, P idx, P labels_src, int nsrc, int B, int out_hw, int train,
                      int double_resize, P params, unsigned long long seed, P hyper, long long epoch_ctr,
                      P out, P labels_out, P params_out, P s) {
    pgdist_rt::run_op([=] {
      launch_augment(ptr<unsigned char>(src), ptr<long long>(idx), ptr<long long>(labels_src), nsrc, B,
                     out_hw, train, double_resize, ptr<float>(params), seed, ptr<float>(hyper),
                     epoch_ctr, ptr<bf16_t>(out), ptr<long long>(labels_out), ptr<float>(params_out), S(s));
    });
  });

  // ---- dense convolutions (ResNet-50) ----
  m.def("conv_fwd_num_partials", &conv_fwd_num_partials);
  m.def("conv_dgrad_num_partials", &conv_dgrad_num_partials);
  m.def("conv_fwd", [](int pro, P x, P pa, P pb, P w, P y, P part, int Nb, int H, int W, int Ci, int N, int R,
                       int Sk, int st, int pad, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_fwd(pro, ptr<bf16_t>(x), ptr<float>(pa), ptr<float>(pb), ptr<bf16_t>(w), ptr<bf16_t>(y),
                      ptr<float>(part), Nb, H, W, Ci, N, R, Sk, st, pad, S(s));
    });
  });
  m.def("conv_dgrad", [](int epi, P G, P Y, P ga, P gb, P gc, P wt, P dx, P Yt, P es, P et, P Rg, P X, P Yt2,
                         P part, P part2, int Nb, int H, int W, int Cin, int Cout, int R, int Sk, int st, int pad,
                         P Xm, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_dgrad(epi, ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ga), ptr<float>(gb), ptr<float>(gc),
                        ptr<bf16_t>(wt), ptr<bf16_t>(dx), ptr<bf16_t>(Yt), ptr<float>(es), ptr<float>(et),
                        ptr<bf16_t>(Rg), ptr<bf16_t>(X), ptr<bf16_t>(Yt2), ptr<float>(part), ptr<float>(part2), Nb,
                        H, W, Cin, Cout, R, Sk, st, pad, ptr<uint8_t>(Xm), S(s));
    });
  });
  m.def("conv_fold_w", [](P wt, P a, P b, P c, P mu, P w2, P fbias, int Cin, int Cout, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_fold_w(ptr<bf16_t>(wt), ptr<float>(a), ptr<float>(b), ptr<float>(c), ptr<float>(mu),
                         ptr<bf16_t>(w2), ptr<float>(fbias), Cin, Cout, S(s));
    });
  });
  m.def("conv_dgrad_fold", [](P G, P Y, P w2, P fbias, P dx, P Yt, P es, P et, P part, int Nb, int H, int W, int Cin,
                              int Cout, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_dgrad_fold(ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<bf16_t>(w2), ptr<float>(fbias), ptr<bf16_t>(dx),
                             ptr<bf16_t>(Yt), ptr<float>(es), ptr<float>(et), ptr<float>(part), Nb, H, W, Cin, Cout,
                             S(s));
    });
  });
  m.def("conv_wgrad_workspace_floats", &conv_wgrad_workspace_floats);
  m.def("conv_wgrad", [](P G, P Y, P ga, P gb, P gc, P x, P xs, P xt, int xpro, P ws, P grad, int Nb, int H,
                         int W, int Ci, int N, int R, int Sk, int st, int pad, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_wgrad(ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ga), ptr<float>(gb), ptr<float>(gc),
                        ptr<bf16_t>(x), ptr<float>(xs), ptr<float>(xt), xpro, ptr<float>(ws), ptr<float>(grad), Nb,
                        H, W, Ci, N, R, Sk, st, pad, S(s));
    });
  });
  m.def("bn_mat", [](int mode, P G, P Y, P a, P b, P c, P out, int M, int C, P s) {
    pgdist_rt::run_op([=] {
      launch_bn_mat(mode, ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(a), ptr<float>(b), ptr<float>(c),
                    ptr<bf16_t>(out), M, C, S(s));
    });
  });
  m.def("conv_wt", [](P src, P dst, P tab, int n, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_wt(ptr<bf16_t>(src), ptr<bf16_t>(dst), ptr<int>(tab), n, S(s));
    });
  });
  m.def("res_out", [](P y, P sc, P sh, P r, P rs, P rt, P out, long long M, int C, P lz, P lz2, P mask, P s) {
    pgdist_rt::run_op([=] {
      launch_res_out(ptr<bf16_t>(y), ptr<float>(sc), ptr<float>(sh), ptr<bf16_t>(r), ptr<float>(rs),
                     ptr<float>(rt), ptr<bf16_t>(out), M, C, ptr<void>(lz), ptr<void>(lz2), ptr<uint8_t>(mask), S(s));
    });
  });
  m.def("maxpool_fwd", [](P y, P sc, P sh, P out, P idx, int Nb, int H, int W, int C, P s) {
    pgdist_rt::run_op([=] {
      launch_maxpool_fwd(ptr<bf16_t>(y), ptr<float>(sc), ptr<float>(sh), ptr<bf16_t>(out), ptr<uint8_t>(idx), Nb,
                         H, W, C, S(s));
    });
  });
  m.def("maxpool_bwd_num_partials", &maxpool_bwd_num_partials);
  m.def("maxpool_bwd", [](P gp, P idx, P y, P sc, P sh, P g, P part, int Nb, int H, int W, int C, P s) {
    pgdist_rt::run_op([=] {
      launch_maxpool_bwd(ptr<bf16_t>(gp), ptr<uint8_t>(idx), ptr<bf16_t>(y), ptr<float>(sc), ptr<float>(sh),
                         ptr<bf16_t>(g), ptr<float>(part), Nb, H, W, C, S(s));
    });
  });
  m.def("avgpool", [](P x, P out, int Nb, int HW, int C, P s) {
    pgdist_rt::run_op([=] {
      launch_avgpool(ptr<bf16_t>(x), ptr<float>(out), Nb, HW, C, S(s));
    });
  });
  m.def("head_bwd", [](P dpool, P x, P y, P G, P part, int Nb, int HW, int C, P s) {
    pgdist_rt::run_op([=] {
      launch_head_bwd(ptr<float>(dpool), ptr<bf16_t>(x), ptr<bf16_t>(y), ptr<bf16_t>(G), ptr<float>(part), Nb,
                      HW, C, S(s));
    });
  });
  m.def("softmax_ce", [](P logits, P labels, int B, int NC, float scale, P loss, P correct, P dlogits, P s) {
    pgdist_rt::run_op([=] {
      launch_softmax_ce(ptr<float>(logits), ptr<long long>(labels), B, NC, scale, ptr<float>(loss),
                        ptr<float>(correct), ptr<float>(dlogits), S(s));
    });
  });
  m.def("fc_gemm_workspace_floats", &fc_gemm_workspace_floats);
  m.def("fc_gemm", [](P A, long long sam, long long sak, P B, long long sbk, long long sbn, P bias, P C, int M, int N,
                      int K, P ws, P s) {
    pgdist_rt::run_op([=] {
      launch_fc_gemm(ptr<float>(A), sam, sak, ptr<float>(B), sbk, sbn, ptr<float>(bias), ptr<float>(C), M, N, K,
                     ptr<float>(ws), S(s));
    });
  });
  m.def("col_sum", [](P X, int M, int N, P out, P s) {
    pgdist_rt::run_op([=] { launch_col_sum(ptr<float>(X), M, N, ptr<float>(out), S(s)); });
  });
  m.def("image_prep", [](P src, P idx, P lab_src, int B, int H, int W, unsigned long long seed, P hyper, P out,
                         P lab_out, int s2d, P s) {
    pgdist_rt::run_op([=] {
      launch_image_prep(ptr<uint8_t>(src), ptr<long long>(idx), ptr<long long>(lab_src), B, H, W, seed,
                        ptr<float>(hyper), ptr<bf16_t>(out), ptr<long long>(lab_out), s2d, S(s));
    });
  });
  // space-to-depth ResNet stem (kernels/conv.hip)
  m.def("stem_w_s2d", [](P w, P w2, int N, P s) {
    pgdist_rt::run_op([=] { launch_stem_w_s2d(ptr<bf16_t>(w), ptr<bf16_t>(w2), N, S(s)); });
  });
  m.def("s2d_image", [](P img, P x2, int B, int H, int W, P s) {
    pgdist_rt::run_op([=] { launch_s2d_image(ptr<bf16_t>(img), ptr<bf16_t>(x2), B, H, W, S(s)); });
  });
  m.def("conv_fwd_s2d", [](P x2, P w2, P y, P part, int Nb, int H2, int N, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_fwd_s2d(ptr<bf16_t>(x2), ptr<bf16_t>(w2), ptr<bf16_t>(y), ptr<float>(part), Nb, H2, N, S(s));
    });
  });
  m.def("conv_wgrad_s2d_workspace_floats", &conv_wgrad_s2d_workspace_floats);
  m.def("conv_wgrad_s2d", [](P G, P Y, P ga, P gb, P gc, P x2, P ws, P grad, int Nb, int H2, int N, P s) {
    pgdist_rt::run_op([=] {
      launch_conv_wgrad_s2d(ptr<bf16_t>(G), ptr<bf16_t>(Y), ptr<float>(ga), ptr<float>(gb), ptr<float>(gc),
                            ptr<bf16_t>(x2), ptr<float>(ws), ptr<float>(grad), Nb, H2, N, S(s));
    });
  });

  // ---- launch plans (runtime/plan.h) ----
  m.def("plan_record_begin", &pgdist_rt::plan_record_begin);
  m.def("plan_record_end", &pgdist_rt::plan_record_end);
  m.def("plan_record_abort", &pgdist_rt::plan_record_abort);
  m.def("plan_recording", &pgdist_rt::plan_recording);
  m.def("plan_replay", &pgdist_rt::plan_replay, "re-issue a recorded step (GIL held: Python ops run inline)");
  m.def("plan_free", &pgdist_rt::plan_free);
  m.def("plan_size", &pgdist_rt::plan_size);
  m.def("plan_recording_size", &pgdist_rt::plan_recording_size);
  m.def("plan_time_ops", &pgdist_rt::plan_time_ops, py::call_guard<py::gil_scoped_release>(),
        "isolated wall time (us) of each op range of a recorded plan (diagnostics; re-runs the ops)");
  m.def("plan_py", [](py::function fn) {
    fn();
    if (pgdist_rt::plan_recording()) {
      // the Python callable is kept alive by the plan; plans are never destroyed after the
      // interpreter finalises (plan.cpp), and plan_free runs with the GIL held
      auto h = std::make_shared<py::object>(std::move(fn));
      pgdist_rt::plan_append([h] { (*h)(); });
    }
  }, "run a Python callable now and, while recording, as a plan op (replayed with the GIL held)");
  m.def("stream_wait", [](P waiter, P signaler) { pgdist_rt::stream_wait(S(waiter), S(signaler)); },
        "waiter waits for the work enqueued so far on signaler (recordable)");
  m.def("memset_async", [](P p, int value, long long bytes, P s) {
    pgdist_rt::memset_async(ptr<void>(p), value, (size_t)bytes, S(s));
  });

  // ---- native communicator (runtime/comm.h): RCCL + P2P xGMI collectives ----
  m.def("rccl_available", &pgdist_rt::rccl_available);
  m.def("rccl_version", &pgdist_rt::rccl_version);
  m.def("comm_unique_id", []() { return py::bytes(pgdist_rt::comm_unique_id()); });
  m.def("comm_create", [](int rank, int world, int device, py::bytes uid, long long region, int blocks, int nlocal,
                          double timeout_s) {
    std::string u = uid;
    py::gil_scoped_release nogil;   // ncclCommInitRank blocks until every rank has joined
    return pgdist_rt::comm_create(rank, world, device, u, region, blocks, nlocal, timeout_s);
  });
  m.def("comm_p2p_handle", [](int id) { return py::bytes(pgdist_rt::comm_p2p_handle(id)); });
  m.def("comm_p2p_open", [](int id, std::vector<py::bytes> hs) {
    std::vector<std::string> v(hs.begin(), hs.end());
    pgdist_rt::comm_p2p_open(id, v);
  });
  m.def("comm_p2p_ready", &pgdist_rt::comm_p2p_ready);
  m.def("comm_stream", &pgdist_rt::comm_stream);
  m.def("comm_blocks", &pgdist_rt::comm_blocks);
  m.def("comm_set_timeout", &pgdist_rt::comm_set_timeout);
  m.def("comm_region_bytes", &pgdist_rt::comm_region_bytes);
  m.def("comm_allreduce", &pgdist_rt::comm_allreduce, "in-place fp32 sum over ranks (recordable)");
  m.def("comm_broadcast", &pgdist_rt::comm_broadcast, "fp32 broadcast from root (recordable)");
  m.def("comm_allreduce_f64", &pgdist_rt::comm_allreduce_f64, "RCCL fp64 all-reduce (recordable)");
  m.def("comm_join", &pgdist_rt::comm_join, "waiter stream waits for the collectives issued so far");
  m.def("comm_time_allreduce", &pgdist_rt::comm_time_allreduce, py::call_guard<py::gil_scoped_release>());
  m.def("comm_error", &pgdist_rt::comm_error, py::call_guard<py::gil_scoped_release>());
  m.def("comm_error_string", &pgdist_rt::comm_error_string);
  m.def("comm_poison", &pgdist_rt::comm_poison, py::call_guard<py::gil_scoped_release>());
  m.def("comm_clear_error", &pgdist_rt::comm_clear_error, py::call_guard<py::gil_scoped_release>());
  m.def("comm_rccl_ranks", &pgdist_rt::comm_rccl_ranks);
  m.def("comm_set_watchdog", &pgdist_rt::comm_set_watchdog, py::call_guard<py::gil_scoped_release>());
  m.def("comm_watchdog", &pgdist_rt::comm_watchdog);
  m.def("comm_inject_stall", &pgdist_rt::comm_inject_stall);
  m.def("comm_error_word", &pgdist_rt::comm_error_word);
  m.def("comm_error_async", &pgdist_rt::comm_error_async);
  m.def("comm_destroy", &pgdist_rt::comm_destroy, py::call_guard<py::gil_scoped_release>());


  // ---- native runtime (host) ----
  m.def("read_cifar10_bin", &pgdist_rt::read_cifar10_bin, py::arg("paths"), py::arg("num_threads") = 4,
        "Read CIFAR-10 binary batches -> (uint8 NHWC [N,32,32,3], int64 labels [N])");
  m.def("shard_indices", &pgdist_rt::shard_indices, py::arg("perm"), py::arg("num_replicas"),
        py::arg("rank"), py::arg("drop_last") = false,
        "DistributedSampler index math on a given permutation (pad by wrap-around, stride by rank)");
}
