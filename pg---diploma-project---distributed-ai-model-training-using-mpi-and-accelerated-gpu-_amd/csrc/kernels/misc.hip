// Small step-bookkeeping kernels kept on the device so a whole training step
// (and its metrics) can be captured in one hipGraph and replayed without any
// host synchronisation.  The reference pays two .item() device->host syncs per
// batch for its running loss/accuracy (cifar10_mpi_mobilenet_224.py:182-185);
// here the per-image loss/correct vectors written by the head kernel are
// folded into fp64 device accumulators and read once per epoch.
#include "../common.h"

// hyper[1] = optimizer step / RNG step counter
__global__ void step_begin_kernel(float *hyper) {
  if (threadIdx.x == 0) hyper[1] += 1.f;
}

// acc[0] += sum loss, acc[1] += sum correct, acc[2] += B
__global__ __launch_bounds__(256) void reduce_metrics_kernel(const float *__restrict__ loss,
                                                            const float *__restrict__ correct, int B,
                                                            double *__restrict__ acc) {
  __shared__ double sh[2][256];
  double l = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < B; i += 256) {
    l += loss[i];
    c += correct[i];
  }
  sh[0][threadIdx.x] = l;
  sh[1][threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + s];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    acc[0] += sh[0][0];
    acc[1] += sh[1][0];
    acc[2] += (double)B;
  }
}

void launch_step_begin(float *hyper, hipStream_t st) {
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(64), 0, st, hyper);
}

void launch_reduce_metrics(const float *loss, const float *correct, int B, double *acc,
                           hipStream_t st) {
  hipLaunchKernelGGL(reduce_metrics_kernel, dim3(1), dim3(256), 0, st, loss, correct, B, acc);
}

// ---------------------------------------------------------------------------
// Deterministic column reduction, level 1:  dst[q][i] = sum_{r in chunk q} src[r][i].
// Producers emit per-workgroup partial rows (BN statistics, weight-gradient
// split-K slabs); a sequential per-thread loop over thousands of rows is
// latency-bound (tens of us), so rows are first folded in chunks by a 2-D grid
// (columns x row-chunks) and consumers read <= 32 rows.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void colsum_kernel(const float *__restrict__ src, int R, long long n,
                                                    int rch, float *__restrict__ dst) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int r0 = blockIdx.y * rch, r1 = min(R, r0 + rch);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int r = r0;
  for (; r + 3 < r1; r += 4) {
    a0 += src[(size_t)r * n + i];
    a1 += src[(size_t)(r + 1) * n + i];
    a2 += src[(size_t)(r + 2) * n + i];
    a3 += src[(size_t)(r + 3) * n + i];
  }
  for (; r < r1; ++r) a0 += src[(size_t)r * n + i];
  dst[(size_t)blockIdx.y * n + i] = (a0 + a1) + (a2 + a3);
}

// rows_out = number of rows the consumer must read: R (no-op) or ceil(R / rch) in dst
void launch_colsum(const float *src, int R, long long n, float *dst, int &rows_out, hipStream_t st) {
  if (R <= 32) {
    rows_out = R;
    return;
  }
  const int rch = (R + 31) / 32;
  rows_out = (R + rch - 1) / rch;
  dim3 grid((unsigned)((n + 255) / 256), rows_out);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, st, src, R, n, rch, dst);
}

int colsum_rows(int R) {
  if (R <= 32) return 0;
  const int rch = (R + 31) / 32;
  return (R + rch - 1) / rch;
}
