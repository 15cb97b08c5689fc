// Fused multi-tensor Adam over ONE flat fp32 parameter buffer.
//
// Reference: optim.Adam(params, lr=1e-4) with torch defaults (betas 0.9/0.999,
// eps 1e-8, no weight decay, no amsgrad) stepped once per batch
// (cifar10_serial_mobilenet_224.py:76,105; cifar10_mpi_mobilenet_224.py:148,180).
//
// All 158 parameter tensors live in one flat buffer, so the whole optimizer is a
// single launch: it reads grad (scaled by 1/world_size — the DDP average is
// folded in here instead of a separate divide pass), updates m, v, the fp32
// master weights, and writes the bf16 shadow copy the conv kernels read.
// lr and the step counter are read from DEVICE memory so the launch can be
// captured in a hipGraph and replayed while StepLR changes lr.
// `skip`: the data-parallel communicator's error word (comm_error_word) or null; while it is
// nonzero (a gradient collective failed or the communicator was poisoned) the update is
// skipped, so un-reduced gradients never reach the replicas' weights.
#include "../common.h"

__global__ __launch_bounds__(256) void adam_flat_kernel(
    float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
    float *__restrict__ v, bf16_t *__restrict__ pb, long long n4, const float *__restrict__ hyper,
    float beta1, float beta2, float eps, float weight_decay, float grad_scale,
    const unsigned *__restrict__ skip, const float *__restrict__ loss,
    const float *__restrict__ correct, int B, double *__restrict__ acc) {
  // the step's metrics (acc[0] += sum loss, acc[1] += sum correct, acc[2] += B) in the last
  // workgroup, instead of a separate reduce_metrics launch after the update
  if (acc && blockIdx.x == gridDim.x - 1) {
    __shared__ double sh[2][4];
    double l = 0.0, c = 0.0;
    for (int i = threadIdx.x; i < B; i += 256) {
      l += loss[i];
      c += correct[i];
    }
    for (int o = 32; o > 0; o >>= 1) {
      l += __shfl_down(l, o);
      c += __shfl_down(c, o);
    }
    if ((threadIdx.x & 63) == 0) {
      sh[0][threadIdx.x >> 6] = l;
      sh[1][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      acc[0] += sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
      acc[1] += sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
      acc[2] += (double)B;
    }
  }
  if (skip && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  // hyper[0] = lr, hyper[1] = step (already incremented for this update)
  const float lr = hyper[0];
  const float t = hyper[1];
  const float bc1 = 1.f - powf(beta1, t);
  const float bc2 = 1.f - powf(beta2, t);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 pv = reinterpret_cast<float4 *>(p)[i];
    float4 gv = reinterpret_cast<const float4 *>(g)[i];
    float4 mv = reinterpret_cast<float4 *>(m)[i];
    float4 vv = reinterpret_cast<float4 *>(v)[i];
    float pp[4] = {pv.x, pv.y, pv.z, pv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float mm[4] = {mv.x, mv.y, mv.z, mv.w}, ww[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gg[k] * grad_scale;
      if (weight_decay != 0.f) gk = fmaf(weight_decay, pp[k], gk);
      mm[k] = fmaf(beta1, mm[k], (1.f - beta1) * gk);
      ww[k] = fmaf(beta2, ww[k], (1.f - beta2) * gk * gk);
      const float denom = sqrtf(ww[k]) / bc2_sqrt + eps;
      pp[k] = pp[k] - step_size * mm[k] / denom;
    }
    reinterpret_cast<float4 *>(p)[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    reinterpret_cast<float4 *>(m)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    reinterpret_cast<float4 *>(v)[i] = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if (pb) {
      uint2 o;
      o.x = pack2(pp[0], pp[1]);
      o.y = pack2(pp[2], pp[3]);
      reinterpret_cast<uint2 *>(pb)[i] = o;
    }
  }
}

// fp32 -> bf16 shadow refresh (after load / broadcast of the master weights)
__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float *__restrict__ x,
                                                         bf16_t *__restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

void launch_adam_flat(float *p, const float *g, float *m, float *v, bf16_t *pb, long long n,
                      const float *hyper, float beta1, float beta2, float eps, float wd,
                      float grad_scale, const unsigned *skip, const float *loss,
                      const float *correct, int B, double *acc, hipStream_t st) {
  const long long n4 = n / 4;  // caller pads the flat buffer to a multiple of 4
  int grid = (int)((n4 + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(adam_flat_kernel, dim3(grid), dim3(256), 0, st, p, g, m, v, pb, n4, hyper,
                     beta1, beta2, eps, wd, grad_scale, skip, loss, correct, B, acc);
}

void launch_f32_to_bf16(const float *x, bf16_t *y, long long n, hipStream_t st) {
  int grid = (int)((n + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid), dim3(256), 0, st, x, y, n);
}
