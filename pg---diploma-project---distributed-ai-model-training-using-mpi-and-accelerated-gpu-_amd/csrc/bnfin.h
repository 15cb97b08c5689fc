// BatchNorm finalize fused into the tail of the kernel that produces the statistics.
//
// Every producer of BN statistics (stem, 1x1 GEMMs, depthwise fwd / dgrad, head backward)
// adds its per-workgroup partial sums into min(P, bn_rep) replica rows of a zeroed
// accumulator with float atomics (common.h bn_part_add).  Instead of a separate finalize
// launch (a dependent kernel boundary on each side of a ~2 us kernel, 104 per training
// step), the LAST workgroup of the producer to arrive reduces the replica rows and writes
// the finalized per-channel vectors (forward: mean, rstd, scale, shift, running stats;
// backward: the dgrad coefficients and dgamma / dbeta) before the producer ends.
//
// Hand-off (MI355X_MICROARCH.md "inter-workgroup visibility"): float atomics execute at the
// memory side; every wave waits vmcnt(0) for its own atomics, a workgroup barrier, then one
// lane adds to the arrival counter (agent scope, returning); the workgroup whose add returns
// nwg-1 is last, re-arms the counter and reads the rows with agent-scope (sc1) loads.
//
// Deterministic mode (ops.kernels.set_deterministic) keeps the separate fixed-order finalize
// launches: the host then passes no descriptor.
#pragma once
#include "reduce.h"

struct BnFin {
  float *acc;        // [rows][2][C] accumulator the producer adds to (zeroed before it runs)
  int *ctr;          // arrival counter: 0 between launches, re-armed by the last arriver
  int rows, C;
  float count;       // elements per channel
  int bwd;           // 0: forward statistics (sum y, sum y^2); 1: backward (sum g, sum g*y)
  const float *gamma, *beta;
  float eps, momentum;
  float *rmean, *rvar;
  long long *nbt;
  float *mean, *rstd, *scale, *shift;   // forward outputs; the backward reads mean / rstd
  float *coef, *dgamma, *dbeta;         // backward outputs (coef [3][C])
};

// forward: totals (sum, sum of squares) of channel c -> mean, rstd, scale, shift, running stats
PG_DEVICE void bn_fwd_channel(int c, double s0, double s1, double n, const float *gamma, const float *beta,
                              float eps, float momentum, float *rmean, float *rvar, float *mean_out,
                              float *rstd_out, float *scale_out, float *shift_out) {
  const double mean = s0 / n;
  double var = s1 / n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  scale_out[c] = g * rstd;
  shift_out[c] = b - (float)mean * g * rstd;
  if (rmean) {
    const double unbiased = n > 1.0 ? var * n / (n - 1.0) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
  }
}

// backward: totals (sum g, sum g*y) of channel c -> dy = a*g + b*y + c coefficients, dgamma, dbeta
PG_DEVICE void bn_bwd_channel(int c, int C, double sg, double sgy, double n, const float *mean,
                              const float *rstd, const float *gamma, float *coef, float *dgamma, float *dbeta) {
  const double mu = mean[c], rs = rstd[c];
  const double g = gamma ? gamma[c] : 1.0;
  const double sgx = (sgy - mu * sg) * rs;  // sum g * xhat
  if (dgamma) dgamma[c] = (float)sgx;
  if (dbeta) dbeta[c] = (float)sg;
  const double a = g * rs;
  coef[c] = (float)a;
  coef[C + c] = (float)(-a * rs * sgx / n);
  coef[2 * C + c] = (float)(-a * sg / n + a * rs * mu * sgx / n);
}

// global-address-space views (the descriptor's pointers are generic: without the cast the
// counter add and the sc1 loads would be flat_* instructions)
typedef __attribute__((address_space(1))) int g_int;
PG_DEVICE float ld_sc1_global(const float *p) {
  return __uint_as_float(__hip_atomic_load((const __attribute__((address_space(1))) unsigned int *)p,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Called by EVERY thread of EVERY workgroup of the producer, after its last bn_part_add and
// with no early exit before it (fin is kernel-uniform; nullptr: nothing to do).
PG_DEVICE void bn_fin_tail(const BnFin *fin) {
  if (fin == nullptr) return;
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's atomics have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nwg = (int)(gridDim.x * gridDim.y * gridDim.z);
    g_int *ctr = (g_int *)fin->ctr;
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == nwg - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  const int C = fin->C, rows = fin->rows;
  const double n = (double)fin->count;
  const float *acc = fin->acc;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    // all 2 x kBnRep loads issued before the first use (rows beyond `rows` re-read row 0 and
    // are weighted 0): one memory latency per channel instead of one per row
    float v[2 * kBnRep];
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const int rr = r < rows ? r : 0;
      v[2 * r] = ld_sc1_global(acc + (size_t)(2 * rr) * C + c);
      v[2 * r + 1] = ld_sc1_global(acc + (size_t)(2 * rr + 1) * C + c);
    }
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < kBnRep; ++r) {
      const double m = r < rows ? 1.0 : 0.0;
      s0 += m * (double)v[2 * r];
      s1 += m * (double)v[2 * r + 1];
    }
    if (fin->bwd)
      bn_bwd_channel(c, C, s0, s1, n, fin->mean, fin->rstd, fin->gamma, fin->coef, fin->dgamma, fin->dbeta);
    else
      bn_fwd_channel(c, s0, s1, n, fin->gamma, fin->beta, fin->eps, fin->momentum, fin->rmean, fin->rvar,
                     fin->mean, fin->rstd, fin->scale, fin->shift);
  }
  if (!fin->bwd && fin->nbt && threadIdx.x == 0) fin->nbt[0] += 1;
}

// host: the descriptor armed for the next producer launch (bn_fin_arm), taken (and cleared)
// by that launcher; nullptr when none is armed
const BnFin *take_bn_fin();

// ---------------------------------------------------------------------------
// Lazy (consumer-side) finalize.  A kernel that consumes a BN's per-channel parameters
// (forward: scale / shift of the BN-apply prologue; backward: the dgrad coefficients a, b, c)
// computes the ones it needs itself from the producer's replica rows instead of waiting for
// a separate finalize launch between the two kernels: the rows were written by an EARLIER
// kernel, so plain loads see them (kernel-boundary visibility, no hand-off inside the grid).
// Redundant work per workgroup: 2 x kBnRep (+2..4) loads per needed channel, issued together.
// The side outputs (mean / rstd / running statistics; dgamma / dbeta) are written off the
// critical path by the regular finalize kernels (a batched forward finalize at the end of
// the forward, the backward ones on the weight-gradient side stream); the backward form
// reads mean / rstd, which that forward finalize wrote.  Bitwise the values of
// bn_finalize_small_kernel (same accumulation order and rounding).
// ---------------------------------------------------------------------------
PG_DEVICE void bn_lazy(const BnFin *d, int c, float &o0, float &o1, float &o2) {
  const int C = d->C, rows = d->rows;
  const float *acc = d->acc;
  const float g = d->gamma ? d->gamma[c] : 1.f;
  const float b = (!d->bwd && d->beta) ? d->beta[c] : 0.f;
  const float mu = d->bwd ? d->mean[c] : 0.f, rs = d->bwd ? d->rstd[c] : 0.f;
  float v[2 * kBnRep];
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const int rr = r < rows ? r : 0;
    v[2 * r] = acc[(size_t)(2 * rr) * C + c];
    v[2 * r + 1] = acc[(size_t)(2 * rr + 1) * C + c];
  }
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const double m = r < rows ? 1.0 : 0.0;
    s0 += m * (double)v[2 * r];
    s1 += m * (double)v[2 * r + 1];
  }
  const double n = (double)d->count;
  if (d->bwd) {
    const double sgx = (s1 - (double)mu * s0) * rs;
    const double a = (double)g * rs;
    o0 = (float)a;
    o1 = (float)(-a * rs * sgx / n);
    o2 = (float)(-a * s0 / n + a * rs * (double)mu * sgx / n);
  } else {
    const double m = s0 / n;
    double var = s1 / n - m * m;
    if (var < 0.0) var = 0.0;
    const float r = (float)(1.0 / sqrt(var + (double)d->eps));
    o0 = g * r;
    o1 = b - (float)m * g * r;
    o2 = 0.f;
  }
}

// The prologue parameters of a consumer with K channels staged into LDS: P[j * Kp + i] for
// i < Kp (zero past K), j < NPAR.  Lazy (lz != nullptr): computed from the producer's replica
// rows (bn_lazy); else copied from the materialised p0 / p1 / p2.  Thread t handles channels
// t, t + 256, ... (blockDim 256) in batches of MAXIT chunks, every load of a batch issued
// before its first use (clamped indices past K): one memory latency per batch instead of one
// per 256-channel chunk.
template <int NPAR, int MAXIT>
PG_DEVICE void bn_stage_batch(const BnFin *lz, const float *p0, const float *p1, const float *p2, int K, int Kp,
                              float *P, int base) {
  const int tid = threadIdx.x;
  const int nit = (Kp - base - tid + 255) / 256;   // chunks of this batch this thread writes
  if (lz) {
    const int C = lz->C, rows = lz->rows;
    const float *acc = lz->acc;
    const bool bwd = lz->bwd;
    float v[MAXIT][2 * kBnRep], g[MAXIT], x0[MAXIT], x1[MAXIT];
#pragma unroll
    for (int u = 0; u < MAXIT; ++u) {
      const int c = min(base + tid + u * 256, K - 1);
#pragma unroll
      for (int r = 0; r < kBnRep; ++r) {
        const int rr = r < rows ? r : 0;
        v[u][2 * r] = acc[(size_t)(2 * rr) * C + c];
        v[u][2 * r + 1] = acc[(size_t)(2 * rr + 1) * C + c];
      }
      g[u] = lz->gamma ? lz->gamma[c] : 1.f;
      x0[u] = bwd ? lz->mean[c] : (lz->beta ? lz->beta[c] : 0.f);
      x1[u] = bwd ? lz->rstd[c] : 0.f;
    }
    const double n = (double)lz->count;
#pragma unroll
    for (int u = 0; u < MAXIT; ++u) {
      if (u >= nit) break;
      const int i = base + tid + u * 256;
      float o0 = 0.f, o1 = 0.f, o2 = 0.f;
      if (i < K) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int r = 0; r < kBnRep; ++r) {
          const double m = r < rows ? 1.0 : 0.0;
          s0 += m * (double)v[u][2 * r];
          s1 += m * (double)v[u][2 * r + 1];
        }
        if (bwd) {   // same arithmetic as bn_lazy
          const float mu = x0[u], rs = x1[u];
          const double sgx = (s1 - (double)mu * s0) * rs;
          const double a = (double)g[u] * rs;
          o0 = (float)a;
          o1 = (float)(-a * rs * sgx / n);
          o2 = (float)(-a * s0 / n + a * rs * (double)mu * sgx / n);
        } else {
          const double m = s0 / n;
          double var = s1 / n - m * m;
          if (var < 0.0) var = 0.0;
          const float r = (float)(1.0 / sqrt(var + (double)lz->eps));
          o0 = g[u] * r;
          o1 = x0[u] - (float)m * g[u] * r;
        }
      }
      P[i] = o0;
      P[Kp + i] = o1;
      if constexpr (NPAR == 3) P[2 * Kp + i] = o2;
    }
  } else {
    float a[MAXIT], b[MAXIT], c[MAXIT];
#pragma unroll
    for (int u = 0; u < MAXIT; ++u) {
      const int ci = min(base + tid + u * 256, K - 1);
      a[u] = p0[ci];
      b[u] = p1[ci];
      c[u] = NPAR == 3 ? p2[ci] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < MAXIT; ++u) {
      if (u >= nit) break;
      const int i = base + tid + u * 256;
      const bool ok = i < K;
      P[i] = ok ? a[u] : 0.f;
      P[Kp + i] = ok ? b[u] : 0.f;
      if constexpr (NPAR == 3) P[2 * Kp + i] = ok ? c[u] : 0.f;
    }
  }
}

template <int NPAR, int MAXIT = 5>
PG_DEVICE void bn_stage_params(const BnFin *lz, const float *p0, const float *p1, const float *p2, int K,
                               int Kp, float *P) {
  for (int base = 0; base < Kp; base += MAXIT * 256) bn_stage_batch<NPAR, MAXIT>(lz, p0, p1, p2, K, Kp, P, base);
}

// host: the lazy descriptor armed for the next consumer launch (bn_lz_arm); nullptr: the
// consumer reads materialised parameters
const BnFin *take_bn_lz();
