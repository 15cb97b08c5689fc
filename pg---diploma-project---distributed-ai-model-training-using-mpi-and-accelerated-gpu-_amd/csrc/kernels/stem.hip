// Stem convolution: 3x3 stride 2 pad 1, 3 -> 32 channels, NHWC bf16.
//
// Reference op: features[0] Conv2d(3, 32, 3, 2, 1) of MobileNetV2 on the
// 224x224 normalised image (SURVEY.md §2.6 "Stem conv 3x3 s2").  The input is
// the output of the GPU augmentation kernel: NHWC with 4 channels (channel 3 is
// an always-zero pad so each pixel is one aligned 8-byte load).
//
// Forward: four threads per group of kPx output pixels, each computing 8 of the
// 32 channels.  The 9 taps are a rolled loop (tap / 3, tap % 3 give the input
// row / column; 32 VGPRs at kPx = 1); per tap the 3 input channels are one 8-B
// load per pixel and each pair of LDS weight reads (8 channels, tap-major
// layout ws[c*9+tap][o]) feeds the kPx pixels (register blocking; kPx = 1, 2 or
// 4).  Each thread stores one 16-B vector per pixel and accumulates the BN0
// partial sums.  The weight gradient is the im2col MFMA kernel in pwconv.hip
// (launch_stem_wgrad).  No input gradient is needed.
#include "../bnfin.h"

namespace {
constexpr int kCo = 32;
}

template <int kPx>
__global__ __launch_bounds__(256) void stem_fwd_kernel(const bf16_t *__restrict__ img,
                                                      const bf16_t *__restrict__ w,  // [32][3][3][3]
                                                      bf16_t *__restrict__ y, float *__restrict__ part,
                                                      int B, int H, int W, int Ho, int Wo, int rep,
                                                      const BnFin *fin) {
  // thread = (group of kPx output pixels, group of 8 output channels): 4 threads per pixel
  // group; each pair of LDS weight reads (8 channels of one input channel x tap) feeds the
  // kPx pixels; each thread stores one 16-B vector per pixel.
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
  const long long step = (long long)gridDim.x * 64 * kPx;
  for (long long pbase = (blockIdx.x * 64ll + (tid >> 2)) * kPx; pbase < npix; pbase += step) {
    int ih0[kPx], iw0[kPx];
    size_t ibase[kPx];
    bool pok[kPx];
#pragma unroll
    for (int q = 0; q < kPx; ++q) {
      const long long pix = pbase + q;
      pok[q] = pix < npix;
      const long long pp = pok[q] ? pix : npix - 1;
      const int b = (int)(pp / (Ho * Wo));
      const int rem = (int)(pp % (Ho * Wo));
      ih0[q] = (rem / Wo) * 2 - 1;
      iw0[q] = (rem % Wo) * 2 - 1;
      ibase[q] = (size_t)b * H * W;
    }
    float acc[kPx][8];
#pragma unroll
    for (int q = 0; q < kPx; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
#pragma unroll 1   // (a 3- or 9-tap unrolled body keeps ~200 VGPRs live)
    for (int tap = 0; tap < 9; ++tap) {
      float x[kPx][3];
#pragma unroll
      for (int q = 0; q < kPx; ++q) {
        const int ih = ih0[q] + tap / 3, iw = iw0[q] + tap % 3;
        const bool in = ih >= 0 && ih < H && iw >= 0 && iw < W;
        uint2 u = make_uint2(0u, 0u);
        if (in) u = *reinterpret_cast<const uint2 *>(img + (ibase[q] + (size_t)ih * W + iw) * 4);
        x[q][0] = __uint_as_float(u.x << 16);
        x[q][1] = __uint_as_float(u.x & 0xffff0000u);
        x[q][2] = __uint_as_float(u.y << 16);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float4 wa = *reinterpret_cast<const float4 *>(&ws[c * 9 + tap][o0]);
        const float4 wb = *reinterpret_cast<const float4 *>(&ws[c * 9 + tap][o0 + 4]);
        const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
        for (int q = 0; q < kPx; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[q][j] = fmaf(x[q][c], wv[j], acc[q][j]);
      }
    }
#pragma unroll
    for (int q = 0; q < kPx; ++q) {
      if (!pok[q]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s0[j] += acc[q][j];
        s1[j] = fmaf(acc[q][j], acc[q][j], s1[j]);
      }
      stg16(y + (pbase + q) * kCo + o0, pack8(acc[q]));
    }
  }
  // block reduction over the 64 pixel-group slots sharing a channel group
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid >> 2][o0 + j] = s == 0 ? s0[j] : s1[j];
    __syncthreads();
    if (tid < kCo) {
      float a = 0.f;
      for (int r = 0; r < 64; ++r) a += red[r][tid];
      bn_part_add(part, blockIdx.x, gridDim.x, rep, kCo, s, tid, a);
    }
    __syncthreads();
  }
  bn_fin_tail(fin);
}

int stem_fwd_num_partials(int B, int H, int W) {
  const long long npix = (long long)B * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  long long g = (npix + 64 * 8 - 1) / (64 * 8);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// px = output pixels per thread (1, 2 or 4; anything else is rejected by the caller and here).
// Measured at bs128 224^2 on MI355X, rolled tap loop: 1 -> 83 us (32 VGPRs), 2 -> 92 us,
// 4 -> 89 us; the fully unrolled 1-pixel loop was 98 us.  The default (1) is chosen in ops.kernels.
bool launch_stem_fwd(const bf16_t *img, const bf16_t *w, bf16_t *y, float *part, int B, int H,
                     int W, int px, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int grid = stem_fwd_num_partials(B, H, W);
  const BnFin *fin = take_bn_fin();
  if (px == 1) hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else if (px == 2) hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else if (px == 4) hipLaunchKernelGGL(stem_fwd_kernel<4>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else return false;
  return true;
}
