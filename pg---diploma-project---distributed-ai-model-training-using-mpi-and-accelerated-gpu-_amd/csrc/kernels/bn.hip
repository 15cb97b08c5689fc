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
#include "../bnfin.h"

#include <stdexcept>
#include <string>

// ---------------------------------------------------------------------------
// Reduction of the [P][2][C] partials (one launch, reduce.h): grid (ceil(C/16) channel
// blocks, nch row chunks), 256 threads = 32 columns ({sum, sumsq} x 16 channels) x 8
// row stripes, fp64 accumulation.  The last workgroup of each channel block gets the
// totals in fin[0..15] (stat 0) / fin[16..31] (stat 1) and runs the finalize.
// ---------------------------------------------------------------------------
namespace {
constexpr int kBnMinRows = 16;
constexpr int kBnOneMax = 1024;   // single-phase (no hand-off) up to this many partial rows

// blockDim.x = 32 * NS threads: 32 columns x NS row stripes (NS = 8 for the two-level
// launch, 32 for the single-workgroup-per-channel-block launch used when P <= 1024)
PG_DEVICE bool bn_reduce(const float *__restrict__ part, int P, int C, int rch, int nch, double *lvl1,
                         int *ctr, double (&sh)[32][32], double (&fin)[32], int &flag) {
  const int tid = threadIdx.x, col = tid & 31, stripe = tid >> 5, NS = blockDim.x >> 5;
  const int c = blockIdx.x * 16 + (col & 15), stat = col >> 4;
  const int r0 = blockIdx.y * rch, r1 = min(P, r0 + rch);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;   // 4 loads in flight per thread, fixed order
  if (c < C) {
    const float *src = part + stat * C + c;
    const size_t ld = (size_t)2 * C;
    int r = r0 + stripe;
    for (; r + 3 * NS < r1; r += 4 * NS) {
      a0 += (double)src[r * ld];
      a1 += (double)src[(r + NS) * ld];
      a2 += (double)src[(r + 2 * NS) * ld];
      a3 += (double)src[(r + 3 * NS) * ld];
    }
    for (; r < r1; r += NS) a0 += (double)src[r * ld];
  }
  sh[stripe][col] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  const size_t row = (size_t)gridDim.x * 32;
  if (tid < 32) {
    double s = 0.0;
    for (int k = 0; k < NS; ++k) s += sh[k][tid];
    if (nch == 1) fin[tid] = s;
    else st_sc1(lvl1 + blockIdx.y * row + blockIdx.x * 32 + tid, s);
  }
  if (nch == 1) {
    __syncthreads();
    return true;
  }
  if (!arrive_last(ctr, nch, &flag)) return false;
  double b = 0.0;
  for (int k = stripe; k < nch; k += NS) b += ld_sc1(lvl1 + k * row + blockIdx.x * 32 + col);
  sh[stripe][col] = b;
  __syncthreads();
  if (tid < 32) {
    double s = 0.0;
    for (int k = 0; k < NS; ++k) s += sh[k][tid];
    fin[tid] = s;
  }
  __syncthreads();
  return true;
}
}  // namespace

// forward: partial (sum, sumsq) -> mean, rstd, scale, shift (+ running stats, unbiased var)
__global__ __launch_bounds__(1024) void bn_fwd_finalize_kernel(
    const float *__restrict__ part, int P, int C, int rch, int nch, double *lvl1, int *ctr, float count,
    const float *__restrict__ gamma, const float *__restrict__ beta, float eps, float momentum,
    float *__restrict__ running_mean, float *__restrict__ running_var, long long *__restrict__ nbt,
    float *__restrict__ mean_out, float *__restrict__ rstd_out, float *__restrict__ scale_out,
    float *__restrict__ shift_out) {
  __shared__ double sh[32][32];
  __shared__ double fin[32];
  __shared__ int flag;
  if (!bn_reduce(part, P, C, rch, nch, lvl1, ctr, sh, fin, flag)) return;
  const int tid = threadIdx.x, c = blockIdx.x * 16 + tid;
  if (tid < 16 && c < C)
    bn_fwd_channel(c, fin[tid], fin[16 + tid], (double)count, gamma, beta, eps, momentum, running_mean,
                   running_var, mean_out, rstd_out, scale_out, shift_out);
  if (nbt && blockIdx.x == 0 && tid == 0) nbt[0] += 1;
}

// backward: partial (sum g, sum g*y) -> dy = alpha*g + beta*y + gamma_c ; coef [3][C], dgamma/dbeta
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    const float *__restrict__ part, int P, int C, int rch, int nch, double *lvl1, int *ctr, float count,
    const float *__restrict__ mean, const float *__restrict__ rstd, const float *__restrict__ gamma,
    float *__restrict__ coef, float *__restrict__ dgamma, float *__restrict__ dbeta) {
  __shared__ double sh[32][32];
  __shared__ double fin[32];
  __shared__ int flag;
  if (!bn_reduce(part, P, C, rch, nch, lvl1, ctr, sh, fin, flag)) return;
  const int tid = threadIdx.x, c = blockIdx.x * 16 + tid;
  if (tid < 16 && c < C)
    bn_bwd_channel(c, C, fin[tid], fin[16 + tid], (double)count, mean, rstd, gamma, coef, dgamma, dbeta);
}

// Finalize of an accumulator with P <= kBnRep rows (the atomic replica rows of the MobileNetV2
// producers): one thread per channel, all 2 x kBnRep row loads issued before the first use
// (rows beyond P re-read row 0 and are weighted 0), 128-thread workgroups — a few workgroups
// instead of C/16 1024-thread ones.
template <bool BWD>
__global__ __launch_bounds__(128) void bn_finalize_small_kernel(
    const float *__restrict__ part, int P, int C, float count, const float *__restrict__ gamma,
    const float *__restrict__ beta, float eps, float momentum, float *__restrict__ rmean, float *__restrict__ rvar,
    long long *__restrict__ nbt, float *__restrict__ mean, float *__restrict__ rstd, float *__restrict__ scale,
    float *__restrict__ shift, float *__restrict__ coef, float *__restrict__ dgamma, float *__restrict__ dbeta) {
  const int c = blockIdx.x * 128 + threadIdx.x;
  if (c < C) {
    // every load of the thread is issued up front (one memory latency, not a chain of them)
    const float g = gamma ? gamma[c] : 1.f;
    const float b = (!BWD && beta) ? beta[c] : 0.f;
    const float rm0 = (!BWD && rmean) ? rmean[c] : 0.f, rv0 = (!BWD && rmean) ? rvar[c] : 0.f;
    const float mu = BWD ? mean[c] : 0.f, rs = BWD ? rstd[c] : 0.f;
    float v[2 * kBnRep];
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const int rr = r < P ? r : 0;
      v[2 * r] = part[(size_t)(2 * rr) * C + c];
      v[2 * r + 1] = part[(size_t)(2 * rr + 1) * C + c];
    }
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const double m = r < P ? 1.0 : 0.0;
      s0 += m * (double)v[2 * r];
      s1 += m * (double)v[2 * r + 1];
    }
    const double n = (double)count;
    if (BWD) {
      const double sgx = (s1 - (double)mu * s0) * rs;   // sum g * xhat
      if (dgamma) dgamma[c] = (float)sgx;
      if (dbeta) dbeta[c] = (float)s0;
      const double a = (double)g * rs;
      coef[c] = (float)a;
      coef[C + c] = (float)(-a * rs * sgx / n);
      coef[2 * C + c] = (float)(-a * s0 / n + a * rs * (double)mu * sgx / n);
    } else {
      const double m = s0 / n;
      double var = s1 / n - m * m;
      if (var < 0.0) var = 0.0;
      const float r = (float)(1.0 / sqrt(var + (double)eps));
      mean[c] = (float)m;
      rstd[c] = r;
      scale[c] = g * r;
      shift[c] = b - (float)m * g * r;
      if (rmean) {
        const double unbiased = n > 1.0 ? var * n / (n - 1.0) : var;
        rmean[c] = (1.f - momentum) * rm0 + momentum * (float)m;
        rvar[c] = (1.f - momentum) * rv0 + momentum * (float)unbiased;
      }
    }
  }
  if (!BWD && nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// ---------------------------------------------------------------------------
// materialise out = act(y*scale+shift) (+ res)    [M][C] bf16, C % 8 == 0
// LZ: scale / shift computed per workgroup from the producer's replica rows (bn_lazy) into LDS
// ---------------------------------------------------------------------------
template <bool RELU6, bool RES, bool LZ>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t *__restrict__ y,
                                                      const bf16_t *__restrict__ res,
                                                      const float *__restrict__ scale,
                                                      const float *__restrict__ shift,
                                                      bf16_t *__restrict__ out, long long n8, int C8,
                                                      const BnFin *lz) {
  extern __shared__ float sp[];   // LZ: [2][C]
  if constexpr (LZ) {   // batched: 4 chunks of 256 channels per memory latency (bnfin.h)
    bn_stage_params<2, 4>(lz, nullptr, nullptr, nullptr, C8 * 8, C8 * 8, sp);
    __syncthreads();
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % C8) * 8;
    float v[8], r[8];
    unpack8(ldg16(y + i * 8), v);
    if constexpr (RES) unpack8(ldg16(res + i * 8), r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float a;
      if constexpr (LZ) a = fmaf(v[k], sp[c0 + k], sp[C8 * 8 + c0 + k]);
      else a = fmaf(v[k], scale[c0 + k], shift[c0 + k]);
      if constexpr (RELU6) a = relu6f(a);
      if constexpr (RES) a += r[k];
      v[k] = a;
    }
    stg16(out + i * 8, pack8(v));
  }
}

// Batched finalize over a table of descriptors (grid: channel blocks x BNs): the side outputs
// of BNs whose consumers finalized lazily (forward: mean / rstd / scale / shift / running
// statistics of every BN of the forward in ONE launch at its end; backward: coef / dgamma /
// dbeta), same values as bn_finalize_small_kernel.
__global__ __launch_bounds__(128) void bn_finalize_batch_kernel(const BnFin *const *__restrict__ tab) {
  const BnFin *d = tab[blockIdx.y];
  const int c = blockIdx.x * 128 + threadIdx.x;
  if (c < d->C) {
    const int C = d->C, rows = d->rows;
    float v[2 * kBnRep];
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const int rr = r < rows ? r : 0;
      v[2 * r] = d->acc[(size_t)(2 * rr) * C + c];
      v[2 * r + 1] = d->acc[(size_t)(2 * rr + 1) * C + c];
    }
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const double m = r < rows ? 1.0 : 0.0;
      s0 += m * (double)v[2 * r];
      s1 += m * (double)v[2 * r + 1];
    }
    if (d->bwd)
      bn_bwd_channel(c, C, s0, s1, (double)d->count, d->mean, d->rstd, d->gamma, d->coef, d->dgamma, d->dbeta);
    else
      bn_fwd_channel(c, s0, s1, (double)d->count, d->gamma, d->beta, d->eps, d->momentum, d->rmean, d->rvar,
                     d->mean, d->rstd, d->scale, d->shift);
  }
  if (!d->bwd && d->nbt && blockIdx.x == 0 && threadIdx.x == 0) d->nbt[0] += 1;
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
int g_bn_rep = kBnRep;

// fused finalize descriptor armed for the next producer launch (see bnfin.h)
static const BnFin *g_bn_fin = nullptr;
void bn_fin_arm(const void *desc) { g_bn_fin = static_cast<const BnFin *>(desc); }
const BnFin *take_bn_fin() {
  const BnFin *d = g_bn_fin;
  g_bn_fin = nullptr;
  return d;
}
// lazy-finalize descriptor armed for the next consumer launch (see bnfin.h bn_lazy)
static const BnFin *g_bn_lz = nullptr;
void bn_lz_arm(const void *desc) { g_bn_lz = static_cast<const BnFin *>(desc); }
const BnFin *take_bn_lz() {
  const BnFin *d = g_bn_lz;
  g_bn_lz = nullptr;
  return d;
}
// error recovery (plan.cpp): no descriptor stays armed for an unrelated later launch
void bn_disarm() {
  g_bn_fin = nullptr;
  g_bn_lz = nullptr;
}
void launch_bn_finalize_batch(const void *tab, int n, int maxC, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(bn_finalize_batch_kernel, dim3((maxC + 127) / 128, n), dim3(128), 0, st,
                     static_cast<const BnFin *const *>(tab));
}
// the descriptor as bytes (the caller copies them to device memory once)
std::string bn_fin_pack(float *acc, int *ctr, int rows, int C, float count, int bwd, const float *gamma,
                        const float *beta, float eps, float momentum, float *rmean, float *rvar, long long *nbt,
                        float *mean, float *rstd, float *scale, float *shift, float *coef, float *dgamma,
                        float *dbeta) {
  if (rows < 1 || rows > kBnRep || C < 1) throw std::invalid_argument("bn_fin_pack: rows in [1, kBnRep], C >= 1");
  if (!acc || !ctr || (bwd ? !(mean && rstd && coef) : !(mean && rstd && scale && shift)))
    throw std::invalid_argument("bn_fin_pack: missing buffer");
  const BnFin d{acc, ctr, rows, C, count, bwd, gamma, beta, eps, momentum, rmean, rvar, nbt,
                mean, rstd, scale, shift, coef, dgamma, dbeta};
  return std::string(reinterpret_cast<const char *>(&d), sizeof d);
}
int bn_rep() { return g_bn_rep; }
void bn_set_rep(int rep) {
  if (rep < 1) throw std::invalid_argument("bn_set_rep: rep must be >= 1");
  g_bn_rep = rep;
}

// part: [P][2][C] followed by the level-1 scratch (bn_part_floats(P, C) floats in total)
long long bn_part_floats(int P, int C) {
  const int nch = red_nch(P, kBnMinRows);
  const long long lvl1 = nch > 1 ? (long long)nch * ((C + 15) / 16) * 32 * 2 : 0;   // doubles -> floats
  return (long long)P * 2 * C + lvl1 + 4;
}

namespace {
double *bn_lvl1(const float *part, int P, int C) {
  // 8-B aligned scratch right after the partials (P * 2C floats, C even)
  return reinterpret_cast<double *>(const_cast<float *>(part) + (size_t)P * 2 * C);
}
}  // namespace

void launch_bn_fwd_finalize(const float *part, int P, int C, float count, const float *gamma,
                            const float *beta, float eps, float momentum, float *rmean,
                            float *rvar, long long *nbt, float *mean, float *rstd, float *scale,
                            float *shift, hipStream_t st) {
  if (P <= kBnRep) {
    hipLaunchKernelGGL(bn_finalize_small_kernel<false>, dim3((C + 127) / 128), dim3(128), 0, st, part, P, C, count,
                       gamma, beta, eps, momentum, rmean, rvar, nbt, mean, rstd, scale, shift, nullptr, nullptr,
                       nullptr);
    return;
  }
  // P <= 1024: one 1024-thread workgroup per 16 channels reads all rows (no hand-off)
  const bool one = P <= kBnOneMax;
  const int rch = one ? P : red_rch(P, kBnMinRows), nch = one ? 1 : red_nch(P, kBnMinRows);
  const int nb = (C + 15) / 16;
  int *ctr = nch > 1 ? reduce_counters(nb, st) : nullptr;
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(nb, nch), dim3(one ? 1024 : 256), 0, st, part, P, C, rch, nch,
                     bn_lvl1(part, P, C), ctr, count, gamma, beta, eps, momentum, rmean, rvar, nbt, mean,
                     rstd, scale, shift);
}

void launch_bn_bwd_finalize(const float *part, int P, int C, float count, const float *mean,
                            const float *rstd, const float *gamma, float *coef, float *dgamma,
                            float *dbeta, hipStream_t st) {
  if (P <= kBnRep) {
    hipLaunchKernelGGL(bn_finalize_small_kernel<true>, dim3((C + 127) / 128), dim3(128), 0, st, part, P, C, count,
                       gamma, nullptr, 0.f, 0.f, nullptr, nullptr, nullptr, const_cast<float *>(mean),
                       const_cast<float *>(rstd), nullptr, nullptr, coef, dgamma, dbeta);
    return;
  }
  const bool one = P <= kBnOneMax;
  const int rch = one ? P : red_rch(P, kBnMinRows), nch = one ? 1 : red_nch(P, kBnMinRows);
  const int nb = (C + 15) / 16;
  int *ctr = nch > 1 ? reduce_counters(nb, st) : nullptr;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(nb, nch), dim3(one ? 1024 : 256), 0, st, part, P, C, rch, nch,
                     bn_lvl1(part, P, C), ctr, count, mean, rstd, gamma, coef, dgamma, dbeta);
}

void launch_bn_apply(const bf16_t *y, const bf16_t *res, const float *scale, const float *shift,
                     bf16_t *out, long long M, int C, bool relu6, hipStream_t st) {
  const BnFin *lz = take_bn_lz();
  const long long n8 = M * (C / 8);
  int grid = (int)((n8 + 255) / 256);
  // lazy: every workgroup finalizes all C channels, so fewer (grid-stride) workgroups
  const int cap = lz ? 2048 : 8192;
  if (grid > cap) grid = cap;
  const int C8 = C / 8;
  const size_t lds = lz ? (size_t)2 * C * sizeof(float) : 0;
#define BNA(R6, RS)                                                                                            \
  if (lz) hipLaunchKernelGGL((bn_apply_kernel<R6, RS, true>), dim3(grid), dim3(256), lds, st, y, res, scale,    \
                             shift, out, n8, C8, lz);                                                           \
  else hipLaunchKernelGGL((bn_apply_kernel<R6, RS, false>), dim3(grid), dim3(256), 0, st, y, res, scale, shift, \
                          out, n8, C8, lz);
  if (relu6) {
    if (res) { BNA(true, true) } else { BNA(true, false) }
  } else {
    if (res) { BNA(false, true) } else { BNA(false, false) }
  }
#undef BNA
}
