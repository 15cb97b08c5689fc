// Stem convolution: 3x3 stride 2 pad 1, 3 -> 32 channels, NHWC bf16.
//
// Reference op: features[0] Conv2d(3, 32, 3, 2, 1) of MobileNetV2 on the
// 224x224 normalised image (SURVEY.md §2.6 "Stem conv 3x3 s2").  The input is
// the output of the GPU augmentation kernel: NHWC with 4 channels (channel 3 is
// an always-zero pad so each pixel is one aligned 8-byte load).
//
// Forward: four threads per output pixel, each computing 8 of the 32 channels
// (27 taps x 8 FMAs, weights broadcast from LDS), storing one 16-B vector and
// accumulating the BN0 partial sums.  The weight gradient is the im2col MFMA kernel in pwconv.hip
// (launch_stem_wgrad).  No input gradient is needed.
#include "../common.h"

namespace {
constexpr int kCo = 32;
}

__global__ __launch_bounds__(256) void stem_fwd_kernel(const bf16_t *__restrict__ img,
                                                      const bf16_t *__restrict__ w,  // [32][3][3][3]
                                                      bf16_t *__restrict__ y, float *__restrict__ part,
                                                      int B, int H, int W, int Ho, int Wo) {
  // thread = (output pixel, group of 8 output channels): 4 threads per pixel, so
  // accumulators + BN partials stay in ~40 VGPRs and each thread stores one 16-B vector
  __shared__ __attribute__((aligned(16))) float ws[27][kCo];  // [c*9+tap][o]
  __shared__ float red[64][kCo];
  const int tid = threadIdx.x;
  for (int i = tid; i < 27 * kCo; i += 256) {
    const int o = i / 27, r = i % 27;  // torch layout index o*27 + c*9 + tap
    ws[r][o] = bf2f(w[i]);
  }
  __syncthreads();
  const int og = tid & 3, o0 = og * 8;
  float s0[8], s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
  const long long npix = (long long)B * Ho * Wo;
  for (long long pix = blockIdx.x * 64ll + (tid >> 2); pix < npix; pix += (long long)gridDim.x * 64) {
    const int b = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix % (Ho * Wo));
    const int oh = rem / Wo, ow = rem % Wo;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ih = oh * 2 - 1 + tap / 3, iw = ow * 2 - 1 + tap % 3;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
      const uint2 u = *reinterpret_cast<const uint2 *>(img + (((size_t)b * H + ih) * W + iw) * 4);
      const float x[3] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                          __uint_as_float(u.y << 16)};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float4 wa = *reinterpret_cast<const float4 *>(&ws[c * 9 + tap][o0]);
        const float4 wb = *reinterpret_cast<const float4 *>(&ws[c * 9 + tap][o0 + 4]);
        acc[0] = fmaf(x[c], wa.x, acc[0]);
        acc[1] = fmaf(x[c], wa.y, acc[1]);
        acc[2] = fmaf(x[c], wa.z, acc[2]);
        acc[3] = fmaf(x[c], wa.w, acc[3]);
        acc[4] = fmaf(x[c], wb.x, acc[4]);
        acc[5] = fmaf(x[c], wb.y, acc[5]);
        acc[6] = fmaf(x[c], wb.z, acc[6]);
        acc[7] = fmaf(x[c], wb.w, acc[7]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0[j] += acc[j];
      s1[j] = fmaf(acc[j], acc[j], s1[j]);
    }
    stg16(y + pix * kCo + o0, pack8(acc));
  }
  // block reduction over the 64 pixel slots sharing a channel group
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid >> 2][o0 + j] = s == 0 ? s0[j] : s1[j];
    __syncthreads();
    if (tid < kCo) {
      float a = 0.f;
      for (int r = 0; r < 64; ++r) a += red[r][tid];
      part[((size_t)blockIdx.x * 2 + s) * kCo + tid] = a;
    }
    __syncthreads();
  }
}

int stem_fwd_num_partials(int B, int H, int W) {
  const long long npix = (long long)B * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  long long g = (npix + 64 * 8 - 1) / (64 * 8);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_stem_fwd(const bf16_t *img, const bf16_t *w, bf16_t *y, float *part, int B, int H,
                     int W, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int grid = stem_fwd_num_partials(B, H, W);
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo);
}
