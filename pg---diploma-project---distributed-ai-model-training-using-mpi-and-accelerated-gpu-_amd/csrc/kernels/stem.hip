// Stem convolution: 3x3 stride 2 pad 1, 3 -> 32 channels, NHWC bf16.
//
// Reference op: features[0] Conv2d(3, 32, 3, 2, 1) of MobileNetV2 on the
// 224x224 normalised image (SURVEY.md §2.6 "Stem conv 3x3 s2").  The input is
// the output of the GPU augmentation kernel: NHWC with 4 channels (channel 3 is
// an always-zero pad so each pixel is one aligned 8-byte load).
//
// Forward (default, stem_fwd_mfma_kernel below): an implicit GEMM on MFMA.  VALU variant
// (px = 1, 2, 4): four threads per group of kPx output pixels, each computing 8 of the
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

// MFMA variant (px = 0): the stem as an implicit GEMM on v_mfma_f32_16x16x32_bf16.  A wave
// computes 16 output pixels x 32 channels per step: A = im2col rows [16 px][k], k = tap*4 + c
// (the 4th input channel is the zero pad, so one 8-B load per tap and pixel), two 32-k steps
// (taps 0-7, tap 8 + zeros); the weight fragments B[k][32] stay in registers for the whole
// grid-stride sweep.  The 16x32 fp32 result goes through a wave-private LDS tile so every
// lane stores one 16-B row chunk; the BN0 partial sums come from the fp32 accumulators.
__global__ __launch_bounds__(256) void stem_fwd_mfma_kernel(const bf16_t *__restrict__ img,
                                                           const bf16_t *__restrict__ w,  // [32][3][3][3]
                                                           bf16_t *__restrict__ y, float *__restrict__ part,
                                                           int B, int H, int W, int Ho, int Wo, int rep,
                                                           const BnFin *fin) {
  __shared__ __attribute__((aligned(16))) bf16_t ct[4][16][kCo + 8];   // per-wave C tile (padded rows)
  __shared__ float red[4][2][kCo];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kc = lane >> 4;   // A: pixel row / 8-k chunk; B: column / 8-k chunk
  // weight fragments: B[k][n] for k = step*32 + kc*8 + e, n = nt*16 + row
  s16x8_t bw[2][2];
#pragma unroll
  for (int stp = 0; stp < 2; ++stp)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int o = nt * 16 + row;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = stp * 32 + kc * 8 + e, tap = k >> 2, c = k & 3;
        bw[stp][nt][e] = (c < 3 && tap < 9) ? (short)w[o * 27 + c * 9 + tap] : (short)0;
      }
    }
  float s0[2] = {0.f, 0.f}, s1[2] = {0.f, 0.f};
  const long long npix = (long long)B * Ho * Wo;
  const long long ntiles = (npix + 15) / 16;
  const int HoWo = Ho * Wo;
  for (long long t = (long long)blockIdx.x * 4 + wave; t < ntiles; t += (long long)gridDim.x * 4) {
    const long long pix = t * 16 + row;
    const bool pok = pix < npix;
    const long long pp = pok ? pix : npix - 1;
    const int b = (int)(pp / HoWo), rem = (int)(pp % HoWo);
    const int ih0 = (rem / Wo) * 2 - 1, iw0 = (rem % Wo) * 2 - 1;
    const bf16_t *base = img + (size_t)b * H * W * 4;
    auto tap_load = [&](int tap) -> uint2 {
      const int ih = ih0 + tap / 3, iw = iw0 + tap % 3;
      uint2 u = make_uint2(0u, 0u);
      if (pok && tap < 9 && ih >= 0 && ih < H && iw >= 0 && iw < W)
        u = *reinterpret_cast<const uint2 *>(base + ((size_t)ih * W + iw) * 4);
      return u;
    };
    const uint2 u0 = tap_load(2 * kc), u1 = tap_load(2 * kc + 1), u8 = kc == 0 ? tap_load(8) : make_uint2(0u, 0u);
    const s16x8_t a0 = __builtin_bit_cast(s16x8_t, make_uint4(u0.x, u0.y, u1.x, u1.y));
    const s16x8_t a1 = __builtin_bit_cast(s16x8_t, make_uint4(u8.x, u8.y, 0u, 0u));
    f32x4_t acc[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0),
                                                        __builtin_bit_cast(bf16x8_t, bw[0][nt]),
                                                        f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1),
                                                        __builtin_bit_cast(bf16x8_t, bw[1][nt]), acc[nt], 0, 0, 0);
    }
    // acc[nt][j] = C[pixel 4*kc + j][channel nt*16 + row]
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pr = 4 * kc + j;
        const float v = acc[nt][j];
        if (t * 16 + pr < npix) {
          s0[nt] += v;
          s1[nt] = fmaf(v, v, s1[nt]);
        }
        ct[wave][pr][nt * 16 + row] = f2bf(v);
      }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    {
      const int pr = lane >> 2, ch = (lane & 3) * 8;   // 16 pixels x 4 chunks of 8 channels
      const long long op = t * 16 + pr;
      const uint4 v = *reinterpret_cast<const uint4 *>(&ct[wave][pr][ch]);
      if (op < npix) stg16(y + op * kCo + ch, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // lanes with the same column (channel) hold different pixel rows: fold the 4 lane groups
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s0[nt] += __shfl_xor(s0[nt], 16, 64);
    s0[nt] += __shfl_xor(s0[nt], 32, 64);
    s1[nt] += __shfl_xor(s1[nt], 16, 64);
    s1[nt] += __shfl_xor(s1[nt], 32, 64);
  }
  if (lane < 16) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      red[wave][0][nt * 16 + lane] = s0[nt];
      red[wave][1][nt * 16 + lane] = s1[nt];
    }
  }
  __syncthreads();
  if (tid < 2 * kCo) {
    const int st = tid / kCo, c = tid % kCo;
    const float a = ((red[0][st][c] + red[1][st][c]) + red[2][st][c]) + red[3][st][c];
    bn_part_add(part, blockIdx.x, gridDim.x, rep, kCo, st, c, a);
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

// px = output pixels per thread of the VALU kernel (1, 2 or 4), or 0: the MFMA kernel (anything
// else is rejected by the caller and here).
// Measured at bs128 224^2 on MI355X, rolled tap loop: 1 -> 83 us (32 VGPRs), 2 -> 92 us,
// 4 -> 89 us; the fully unrolled 1-pixel loop was 98 us.  The default (1) is chosen in ops.kernels.
bool launch_stem_fwd(const bf16_t *img, const bf16_t *w, bf16_t *y, float *part, int B, int H,
                     int W, int px, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int grid = stem_fwd_num_partials(B, H, W);
  const BnFin *fin = take_bn_fin();
  if (px == 0) hipLaunchKernelGGL(stem_fwd_mfma_kernel, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else if (px == 1) hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else if (px == 2) hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else if (px == 4) hipLaunchKernelGGL(stem_fwd_kernel<4>, dim3(grid), dim3(256), 0, st, img, w, y, part, B, H, W, Ho, Wo, g_bn_rep, fin);
  else return false;
  return true;
}
