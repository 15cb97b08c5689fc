// Small step-bookkeeping kernels kept on the device so a whole training step
// (and its metrics) can be captured in one hipGraph and replayed without any
// host synchronisation.  The reference pays two .item() device->host syncs per
// batch for its running loss/accuracy (cifar10_mpi_mobilenet_224.py:182-185);
// here the per-image loss/correct vectors written by the head kernel are
// folded into fp64 device accumulators and read once per epoch.
#include "../common.h"

// hyper[1] = optimizer step / RNG step counter; zero[0, n) = 0: the step's BatchNorm statistics
// arena, cleared in the same launch instead of a separate fill at the head of every step
__global__ __launch_bounds__(256) void step_begin_kernel(float *hyper, float *zero, long long n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) hyper[1] += 1.f;
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += gridDim.x * 256LL)
    reinterpret_cast<float4 *>(zero)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) zero[n4 * 4 + threadIdx.x] = 0.f;
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

void launch_step_begin(float *hyper, float *zero, long long n, hipStream_t st) {
  long long grid = ((n >> 2) + 255) / 256;
  grid = grid < 1 ? 1 : (grid > 512 ? 512 : grid);
  hipLaunchKernelGGL(step_begin_kernel, dim3((unsigned)grid), dim3(256), 0, st, hyper, zero, n);
}

void launch_reduce_metrics(const float *loss, const float *correct, int B, double *acc,
                           hipStream_t st) {
  hipLaunchKernelGGL(reduce_metrics_kernel, dim3(1), dim3(256), 0, st, loss, correct, B, acc);
}
