// BatchNorm (training mode) for the fused NHWC pipeline.
//
// BN statistics are never computed by a standalone pass over the activation:
// every producer kernel (stem / depthwise / pointwise conv) writes per-workgroup
// partial sums  [P][2][C]  (sum, sum-of-squares) from its epilogue, and the
// consumer applies  z = relu6(y*scale + shift)  in its prologue.  These kernels
// are the tiny per-channel "finalize" steps in between, plus the elementwise
// materialisation of block outputs (BN + residual) — reference semantics:
// torchvision BatchNorm2d(eps=1e-5, momentum=0.1) inside MobileNetV2
// (SURVEY.md §2.6 "BatchNorm2d (train)", §2.8).
#include "../common.h"

// ---------------------------------------------------------------------------
// forward finalize: partial (sum, sumsq) -> mean, rstd, scale, shift (+ running stats)
// grid: ceil(C/64) blocks of 256 threads (64 channels x 4 partial stripes)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(
    const float *__restrict__ part, int P, int C, float count,
    const float *__restrict__ gamma, const float *__restrict__ beta, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var, long long *__restrict__ nbt,
    float *__restrict__ mean_out, float *__restrict__ rstd_out, float *__restrict__ scale_out,
    float *__restrict__ shift_out) {
  __shared__ double sh[2][4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int p = ty; p < P; p += 4) {
      s += (double)part[(size_t)p * 2 * C + c];
      q += (double)part[(size_t)p * 2 * C + C + c];
    }
  }
  sh[0][ty][tx] = s;
  sh[1][ty][tx] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    s = sh[0][0][tx] + sh[0][1][tx] + sh[0][2][tx] + sh[0][3][tx];
    q = sh[1][0][tx] + sh[1][1][tx] + sh[1][2][tx] + sh[1][3][tx];
    const double n = (double)count;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    mean_out[c] = (float)mean;
    rstd_out[c] = rstd;
    scale_out[c] = g * rstd;
    shift_out[c] = b - (float)mean * g * rstd;
    if (running_mean) {
      const double unbiased = n > 1.0 ? var * n / (n - 1.0) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// ---------------------------------------------------------------------------
// backward finalize: partial (sum g, sum g*y) -> dy = alpha*g + beta*y + gamma_c
// coef layout [3][C] = alpha, beta, gamma_c ; writes dgamma/dbeta (fp32 grads)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    const float *__restrict__ part, int P, int C, float count, const float *__restrict__ mean,
    const float *__restrict__ rstd, const float *__restrict__ gamma, float *__restrict__ coef,
    float *__restrict__ dgamma, float *__restrict__ dbeta) {
  __shared__ double sh[2][4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  double sg = 0.0, sgy = 0.0;
  if (c < C) {
    for (int p = ty; p < P; p += 4) {
      sg += (double)part[(size_t)p * 2 * C + c];
      sgy += (double)part[(size_t)p * 2 * C + C + c];
    }
  }
  sh[0][ty][tx] = sg;
  sh[1][ty][tx] = sgy;
  __syncthreads();
  if (ty == 0 && c < C) {
    sg = sh[0][0][tx] + sh[0][1][tx] + sh[0][2][tx] + sh[0][3][tx];
    sgy = sh[1][0][tx] + sh[1][1][tx] + sh[1][2][tx] + sh[1][3][tx];
    const double n = (double)count, mu = mean[c], rs = rstd[c];
    const double g = gamma ? gamma[c] : 1.0;
    const double sgx = (sgy - mu * sg) * rs;  // sum g * xhat
    if (dgamma) dgamma[c] = (float)sgx;
    if (dbeta) dbeta[c] = (float)sg;
    const double a = g * rs;
    coef[c] = (float)a;
    coef[C + c] = (float)(-a * rs * sgx / n);
    coef[2 * C + c] = (float)(-a * sg / n + a * rs * mu * sgx / n);
  }
}

// ---------------------------------------------------------------------------
// materialise out = act(y*scale+shift) (+ res)    [M][C] bf16, C % 8 == 0
// ---------------------------------------------------------------------------
template <bool RELU6, bool RES>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t *__restrict__ y,
                                                      const bf16_t *__restrict__ res,
                                                      const float *__restrict__ scale,
                                                      const float *__restrict__ shift,
                                                      bf16_t *__restrict__ out, long long n8, int C8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % C8) * 8;
    float v[8], r[8];
    unpack8(ldg16(y + i * 8), v);
    if constexpr (RES) unpack8(ldg16(res + i * 8), r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float a = fmaf(v[k], scale[c0 + k], shift[c0 + k]);
      if constexpr (RELU6) a = relu6f(a);
      if constexpr (RES) a += r[k];
      v[k] = a;
    }
    stg16(out + i * 8, pack8(v));
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
void launch_colsum(const float *src, int R, long long n, float *dst, int &rows_out, hipStream_t st);

// part: [P][2][C] followed by scratch for the level-1 fold (colsum_rows(P) * 2C floats)
void launch_bn_fwd_finalize(const float *part, int P, int C, float count, const float *gamma,
                            const float *beta, float eps, float momentum, float *rmean,
                            float *rvar, long long *nbt, float *mean, float *rstd, float *scale,
                            float *shift, hipStream_t st) {
  int rows = P;
  float *tmp = const_cast<float *>(part) + (size_t)P * 2 * C;
  launch_colsum(part, P, 2LL * C, tmp, rows, st);
  if (rows != P) { part = tmp; P = rows; }
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, st, part, P, C,
                     count, gamma, beta, eps, momentum, rmean, rvar, nbt, mean, rstd, scale, shift);
}

void launch_bn_bwd_finalize(const float *part, int P, int C, float count, const float *mean,
                            const float *rstd, const float *gamma, float *coef, float *dgamma,
                            float *dbeta, hipStream_t st) {
  int rows = P;
  float *tmp = const_cast<float *>(part) + (size_t)P * 2 * C;
  launch_colsum(part, P, 2LL * C, tmp, rows, st);
  if (rows != P) { part = tmp; P = rows; }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, st, part, P, C,
                     count, mean, rstd, gamma, coef, dgamma, dbeta);
}

void launch_bn_apply(const bf16_t *y, const bf16_t *res, const float *scale, const float *shift,
                     bf16_t *out, long long M, int C, bool relu6, hipStream_t st) {
  const long long n8 = M * (C / 8);
  int grid = (int)((n8 + 255) / 256);
  if (grid > 8192) grid = 8192;
  const int C8 = C / 8;
  if (relu6) {
    if (res) hipLaunchKernelGGL((bn_apply_kernel<true, true>), dim3(grid), dim3(256), 0, st, y, res, scale, shift, out, n8, C8);
    else hipLaunchKernelGGL((bn_apply_kernel<true, false>), dim3(grid), dim3(256), 0, st, y, res, scale, shift, out, n8, C8);
  } else {
    if (res) hipLaunchKernelGGL((bn_apply_kernel<false, true>), dim3(grid), dim3(256), 0, st, y, res, scale, shift, out, n8, C8);
    else hipLaunchKernelGGL((bn_apply_kernel<false, false>), dim3(grid), dim3(256), 0, st, y, res, scale, shift, out, n8, C8);
  }
}
