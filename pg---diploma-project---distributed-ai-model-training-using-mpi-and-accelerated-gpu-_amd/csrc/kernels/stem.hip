// Stem convolution: 3x3 stride 2 pad 1, 3 -> 32 channels, NHWC bf16.
//
// Reference op: features[0] Conv2d(3, 32, 3, 2, 1) of MobileNetV2 on the
// 224x224 normalised image (SURVEY.md §2.6 "Stem conv 3x3 s2").  The input is
// the output of the GPU augmentation kernel: NHWC with 4 channels (channel 3 is
// an always-zero pad so each pixel is one aligned 8-byte load).
//
// Forward: one thread per output pixel computes all 32 channels (27 taps x 32
// FMAs, weights broadcast from LDS), stores 64 B, and accumulates the BN0
// partial sums.  The weight gradient is the im2col MFMA kernel in pwconv.hip
// (launch_stem_wgrad).  No input gradient is needed.
#include "../common.h"

namespace {
constexpr int kCo = 32;
}

__global__ __launch_bounds__(256) void stem_fwd_kernel(const bf16_t *__restrict__ img,
                                                      const bf16_t *__restrict__ w,  // [32][3][3][3]
                                                      bf16_t *__restrict__ y, float *__restrict__ part,
                                                      int B, int H, int W, int Ho, int Wo) {
  __shared__ __attribute__((aligned(16))) float ws[27][kCo];  // [c*9+tap][o]
  __shared__ float red[8][kCo];
  const int tid = threadIdx.x;
  for (int i = tid; i < 27 * kCo; i += 256) {
    const int o = i / 27, r = i % 27;  // torch layout index o*27 + c*9 + tap
    ws[r][o] = bf2f(w[i]);
  }
  __syncthreads();
  float s0[kCo], s1[kCo];
#pragma unroll
  for (int o = 0; o < kCo; ++o) s0[o] = s1[o] = 0.f;
  const long long npix = (long long)B * Ho * Wo;
  for (long long pix = blockIdx.x * 256ll + tid; pix < npix; pix += (long long)gridDim.x * 256) {
    const int b = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix % (Ho * Wo));
    const int oh = rem / Wo, ow = rem % Wo;
    float acc[kCo];
#pragma unroll
    for (int o = 0; o < kCo; ++o) acc[o] = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ih = oh * 2 - 1 + tap / 3, iw = ow * 2 - 1 + tap % 3;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
      const uint2 u = *reinterpret_cast<const uint2 *>(img + (((size_t)b * H + ih) * W + iw) * 4);
      const float x[3] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                          __uint_as_float(u.y << 16)};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float4 *wr = reinterpret_cast<const float4 *>(ws[c * 9 + tap]);
#pragma unroll
        for (int o4 = 0; o4 < kCo / 4; ++o4) {
          const float4 wv = wr[o4];
          acc[o4 * 4 + 0] = fmaf(x[c], wv.x, acc[o4 * 4 + 0]);
          acc[o4 * 4 + 1] = fmaf(x[c], wv.y, acc[o4 * 4 + 1]);
          acc[o4 * 4 + 2] = fmaf(x[c], wv.z, acc[o4 * 4 + 2]);
          acc[o4 * 4 + 3] = fmaf(x[c], wv.w, acc[o4 * 4 + 3]);
        }
      }
    }
    uint4 *dst = reinterpret_cast<uint4 *>(y + pix * kCo);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = acc[q * 8 + j];
        s0[q * 8 + j] += v[j];
        s1[q * 8 + j] = fmaf(v[j], v[j], s1[q * 8 + j]);
      }
      dst[q] = pack8(v);
    }
  }
  // block reduction: wave shuffle then LDS across the 4 waves
  const int lane = tid & 63, wave = tid >> 6;
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int o = 0; o < kCo; ++o) {
      const float v = wave_sum(s == 0 ? s0[o] : s1[o]);
      if (lane == 0) red[s * 4 + wave][o] = v;
    }
  }
  __syncthreads();
  if (tid < 2 * kCo) {
    const int s = tid / kCo, o = tid % kCo;
    part[((size_t)blockIdx.x * 2 + s) * kCo + o] =
        red[s * 4 + 0][o] + red[s * 4 + 1][o] + red[s * 4 + 2][o] + red[s * 4 + 3][o];
  }
}

int stem_fwd_num_partials(int B, int H, int W) {
  const long long npix = (long long)B * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  long long g = (npix + 256 * 8 - 1) / (256 * 8);
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
