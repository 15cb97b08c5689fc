// Depthwise 3x3 convolution (pad 1, stride 1|2), NHWC bf16, for MobileNetV2.
//
// Reference op: the 17 depthwise Conv2d(groups=C) layers of torchvision
// MobileNetV2 run through cuDNN (SURVEY.md §2.6 "Depthwise conv 3x3"); on ROCm
// the library path (MIOpen / CK grouped-conv bwd-weight) takes ~23 ms per call
// at bs=128 (profiles/r1_torch_miopen_baseline_kernel_stats.csv).  Depthwise is
// pure bandwidth (1.8-4.5 FLOP/B), so these kernels are built around bytes:
//
//  * thread = 8 channels (one 16-B vector) x a run of PIX output pixels along W;
//    the 3 x (PIX*S+2) input window is streamed column by column so each input
//    vector is loaded and BN-transformed ONCE per thread (sliding window);
//  * the input operand is the *pre-BN* output of the producer: the producer's
//    BatchNorm-apply + ReLU6 is fused into the load (zero padding is applied in
//    the post-activation space, as in the reference graph);
//  * the forward epilogue emits per-workgroup BN partial sums of the output, the
//    backward epilogue emits the producer-BN backward partials — no standalone
//    BN passes over the activation.
#include "../common.h"

namespace {

constexpr int kMaxThreads = 256;

struct DwGeom {
  int B, H, W, C, Ho, Wo, rows_per_wg;
};

// Load 8 channels at (b, ih, iw) of an NHWC tensor and apply the producer BN (+relu6).
// Out-of-range positions yield 0 (padding in activation space).
template <int ACT>
PG_DEVICE void load_act8(const bf16_t *__restrict__ x, const DwGeom &g, int b, int ih, int iw,
                         int c0, const float (&s)[8], const float (&t)[8], float (&v)[8]) {
  if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.f;
    return;
  }
  const size_t off = (((size_t)b * g.H + ih) * g.W + iw) * g.C + c0;
  unpack8(ldg16(x + off), v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = act_apply<ACT>(v[k], s[k], t[k]);
}

// Block-level reduction of per-thread [NV][8] channel partials into part[blockIdx][NV][C]
// threads are laid out tid = tw * C8 + c8.
template <int NV>
PG_DEVICE void block_channel_partials(float (&acc)[NV][8], float *__restrict__ part, int C, int C8,
                                      int TW, float *lds) {
  const int tid = threadIdx.x;
  const int c8 = tid % C8, tw = tid / C8;
  const bool active = tw < TW;
  for (int v = 0; v < NV; ++v) {
    // lds: [TW][C]
    if (active) {
#pragma unroll
      for (int k = 0; k < 8; ++k) lds[tw * C + c8 * 8 + k] = acc[v][k];
    }
    __syncthreads();
    for (int c = tid; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int w = 0; w < TW; ++w) s += lds[w * C + c];
      part[((size_t)blockIdx.x * NV + v) * C + c] = s;
    }
    __syncthreads();
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// forward: y = dwconv(act(x)), partial (sum y, sum y^2)
// ---------------------------------------------------------------------------
template <int S, int ACT, int PIX>
__global__ __launch_bounds__(kMaxThreads) void dw_fwd_kernel(
    const bf16_t *__restrict__ x, const float *__restrict__ in_s, const float *__restrict__ in_t,
    const bf16_t *__restrict__ w, bf16_t *__restrict__ y, float *__restrict__ part, DwGeom g) {
  __shared__ float lds[2048];
  const int C8 = g.C / 8;
  const int TW = blockDim.x / C8;
  const int tid = threadIdx.x;
  const int c8 = tid % C8, tw = tid / C8;
  const int c0 = c8 * 8;
  constexpr int NCOL = (PIX - 1) * S + 3;

  float wt[8][9], s[8], t[8];
  float stats[2][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int q = 0; q < 9; ++q) wt[k][q] = bf2f(w[(c0 + k) * 9 + q]);
    s[k] = (ACT != ACT_NONE) ? in_s[c0 + k] : 1.f;
    t[k] = (ACT != ACT_NONE) ? in_t[c0 + k] : 0.f;
    stats[0][k] = 0.f;
    stats[1][k] = 0.f;
  }

  const int nch = (g.Wo + PIX - 1) / PIX;
  const int rows_total = g.B * g.Ho;
  const int r0 = blockIdx.x * g.rows_per_wg;
  const int nrows = min(g.rows_per_wg, rows_total - r0);
  const int items = nrows * nch;
  if (tw < TW) {
    for (int it = tw; it < items; it += TW) {
      const int r = r0 + it / nch;
      const int ow0 = (it % nch) * PIX;
      const int b = r / g.Ho, oh = r % g.Ho;
      float acc[PIX][8];
#pragma unroll
      for (int o = 0; o < PIX; ++o)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        const int ih = oh * S - 1 + dh;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int iw = ow0 * S - 1 + j;
          float v[8];
          load_act8<ACT>(x, g, b, ih, iw, c0, s, t, v);
#pragma unroll
          for (int o = 0; o < PIX; ++o) {
            const int dw = j - o * S;
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < 8; ++k) acc[o][k] = fmaf(v[k], wt[k][dh * 3 + dw], acc[o][k]);
            }
          }
        }
      }
#pragma unroll
      for (int o = 0; o < PIX; ++o) {
        if (ow0 + o < g.Wo) {
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow0 + o) * g.C + c0;
          stg16(y + off, pack8(acc[o]));
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            stats[0][k] += acc[o][k];
            stats[1][k] = fmaf(acc[o][k], acc[o][k], stats[1][k]);
          }
        }
      }
    }
  }
  block_channel_partials<2>(stats, part, g.C, C8, TW, lds);
}

// ---------------------------------------------------------------------------
// dgrad: gout = mask_prev * dwconv^T(dy),  dy = a*g + b*y + c (this layer's BN backward)
// partial (sum gout, sum gout*yprev) for the producer BN
// ---------------------------------------------------------------------------
template <int S, int PIX>
__global__ __launch_bounds__(kMaxThreads) void dw_dgrad_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ w, const bf16_t *__restrict__ yprev, const float *__restrict__ ps,
    const float *__restrict__ pt, bf16_t *__restrict__ gout, float *__restrict__ part, DwGeom g) {
  __shared__ float lds[2048];
  const int C8 = g.C / 8;
  const int TW = blockDim.x / C8;
  const int tid = threadIdx.x;
  const int c8 = tid % C8, tw = tid / C8;
  const int c0 = c8 * 8;
  // PIX input pixels per item; needed output columns:
  constexpr int NCOL = (S == 1) ? PIX + 2 : PIX / 2 + 2;

  float wt[8][9], al[8], be[8], ga[8], s[8], t[8];
  float stats[2][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int q = 0; q < 9; ++q) wt[k][q] = bf2f(w[(c0 + k) * 9 + q]);
    al[k] = coef[c0 + k];
    be[k] = coef[g.C + c0 + k];
    ga[k] = coef[2 * g.C + c0 + k];
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
    stats[0][k] = 0.f;
    stats[1][k] = 0.f;
  }
  const int nch = (g.W + PIX - 1) / PIX;
  const int rows_total = g.B * g.H;
  const int r0 = blockIdx.x * g.rows_per_wg;
  const int nrows = min(g.rows_per_wg, rows_total - r0);
  const int items = nrows * nch;
  if (tw < TW) {
    for (int it = tw; it < items; it += TW) {
      const int r = r0 + it / nch;
      const int iw0 = (it % nch) * PIX;
      const int b = r / g.H, ih = r % g.H;
      float acc[PIX][8];
#pragma unroll
      for (int o = 0; o < PIX; ++o)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        int oh;
        if constexpr (S == 1) {
          oh = ih + 1 - dh;
        } else {
          const int num = ih + 1 - dh;
          if (num & 1) continue;
          oh = num >> 1;
        }
        if (oh < 0 || oh >= g.Ho) continue;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int ow = (S == 1) ? iw0 - 1 + j : (iw0 >> 1) - 1 + j;
          if (ow < 0 || ow >= g.Wo) continue;
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow) * g.C + c0;
          float gv[8], yv[8];
          unpack8(ldg16(gin + off), gv);
          unpack8(ldg16(yself + off), yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
#pragma unroll
          for (int i = 0; i < PIX; ++i) {
            const int dw = (S == 1) ? (i - j + 2) : (i + 3 - 2 * j);
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < 8; ++k) acc[i][k] = fmaf(gv[k], wt[k][dh * 3 + dw], acc[i][k]);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < PIX; ++i) {
        if (iw0 + i < g.W) {
          const size_t off = (((size_t)b * g.H + ih) * g.W + iw0 + i) * g.C + c0;
          float yp[8];
          unpack8(ldg16(yprev + off), yp);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float gg = acc[i][k] * relu6_mask(yp[k], s[k], t[k]);
            acc[i][k] = gg;
            stats[0][k] += gg;
            stats[1][k] = fmaf(gg, yp[k], stats[1][k]);
          }
          stg16(gout + off, pack8(acc[i]));
        }
      }
    }
  }
  block_channel_partials<2>(stats, part, g.C, C8, TW, lds);
}

// ---------------------------------------------------------------------------
// wgrad: dW[c][tap] partials per workgroup  [P][9][C]
// ---------------------------------------------------------------------------
template <int S, int PIX>
__global__ __launch_bounds__(kMaxThreads) void dw_wgrad_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ yprev, const float *__restrict__ ps, const float *__restrict__ pt,
    float *__restrict__ part, DwGeom g) {
  __shared__ float lds[2048];
  const int C8 = g.C / 8;
  const int TW = blockDim.x / C8;
  const int tid = threadIdx.x;
  const int c8 = tid % C8, tw = tid / C8;
  const int c0 = c8 * 8;
  constexpr int NCOL = (PIX - 1) * S + 3;

  float al[8], be[8], ga[8], s[8], t[8];
  float accw[9][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    al[k] = coef[c0 + k];
    be[k] = coef[g.C + c0 + k];
    ga[k] = coef[2 * g.C + c0 + k];
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
#pragma unroll
    for (int q = 0; q < 9; ++q) accw[q][k] = 0.f;
  }
  const int nch = (g.Wo + PIX - 1) / PIX;
  const int rows_total = g.B * g.Ho;
  const int r0 = blockIdx.x * g.rows_per_wg;
  const int nrows = min(g.rows_per_wg, rows_total - r0);
  const int items = nrows * nch;
  if (tw < TW) {
    for (int it = tw; it < items; it += TW) {
      const int r = r0 + it / nch;
      const int ow0 = (it % nch) * PIX;
      const int b = r / g.Ho, oh = r % g.Ho;
      float dy[PIX][8];
#pragma unroll
      for (int o = 0; o < PIX; ++o) {
        if (ow0 + o < g.Wo) {
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow0 + o) * g.C + c0;
          float gv[8], yv[8];
          unpack8(ldg16(gin + off), gv);
          unpack8(ldg16(yself + off), yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) dy[o][k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) dy[o][k] = 0.f;
        }
      }
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        const int ih = oh * S - 1 + dh;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int iw = ow0 * S - 1 + j;
          float v[8];
          load_act8<ACT_BN_RELU6>(yprev, DwGeom{g.B, g.H, g.W, g.C, g.Ho, g.Wo, 0}, b, ih, iw, c0, s,
                                  t, v);
#pragma unroll
          for (int o = 0; o < PIX; ++o) {
            const int dw = j - o * S;
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < 8; ++k)
                accw[dh * 3 + dw][k] = fmaf(dy[o][k], v[k], accw[dh * 3 + dw][k]);
            }
          }
        }
      }
    }
  }
  block_channel_partials<9>(accw, part, g.C, C8, TW, lds);
}

// reduce [P][9][C] -> grad [C][9] (torch layout [C,1,3,3]) fp32
__global__ __launch_bounds__(256) void dw_wgrad_reduce_kernel(const float *__restrict__ part, int P,
                                                             int C, float *__restrict__ grad) {
  const int idx = blockIdx.x * 64 + (threadIdx.x & 63);  // over 9*C (tap-major in part)
  const int ty = threadIdx.x >> 6;
  __shared__ float sh[4][64];
  float s = 0.f;
  if (idx < 9 * C)
    for (int p = ty; p < P; p += 4) s += part[(size_t)p * 9 * C + idx];
  sh[ty][threadIdx.x & 63] = s;
  __syncthreads();
  if (ty == 0 && idx < 9 * C) {
    s = sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
    const int tap = idx / C, c = idx % C;
    grad[c * 9 + tap] = s;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int dw_block_threads(int C) {
  const int C8 = C / 8;
  int TW = kMaxThreads / C8;
  if (TW < 1) TW = 1;
  return C8 * TW;
}

static int dw_rows_per_wg(int rows_total, int per_row_items, int TW, int target_items_per_thread) {
  int rpw = (TW * target_items_per_thread + per_row_items - 1) / per_row_items;
  if (rpw < 1) rpw = 1;
  // keep at least ~512 workgroups when possible
  while (rpw > 1 && (rows_total + rpw - 1) / rpw < 512) rpw >>= 1;
  return rpw;
}

int dw_fwd_num_partials(int B, int H, int W, int C, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int TW = dw_block_threads(C) / (C / 8);
  const int rpw = dw_rows_per_wg(B * Ho, (Wo + 6) / 7, TW, 2);
  return (B * Ho + rpw - 1) / rpw;
}

int dw_dgrad_num_partials(int B, int H, int W, int C, int stride) {
  const int TW = dw_block_threads(C) / (C / 8);
  const int pix = stride == 1 ? 7 : 14;
  const int rpw = dw_rows_per_wg(B * H, (W + pix - 1) / pix, TW, 2);
  return (B * H + rpw - 1) / rpw;
}

int dw_wgrad_num_partials(int B, int H, int W, int C, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int TW = dw_block_threads(C) / (C / 8);
  const int rpw = dw_rows_per_wg(B * Ho, (Wo + 6) / 7, TW, 4);
  return (B * Ho + rpw - 1) / rpw;
}

void launch_dw_fwd(const bf16_t *x, const float *in_s, const float *in_t, int act, const bf16_t *w,
                   bf16_t *y, float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int threads = dw_block_threads(C);
  const int TW = threads / (C / 8);
  const int rpw = dw_rows_per_wg(B * Ho, (Wo + 6) / 7, TW, 2);
  const int grid = (B * Ho + rpw - 1) / rpw;
  DwGeom g{B, H, W, C, Ho, Wo, rpw};
  if (stride == 1) {
    if (act == ACT_BN_RELU6)
      hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_BN_RELU6, 7>), dim3(grid), dim3(threads), 0, st, x, in_s, in_t, w, y, part, g);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_NONE, 7>), dim3(grid), dim3(threads), 0, st, x, in_s, in_t, w, y, part, g);
  } else {
    if (act == ACT_BN_RELU6)
      hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_BN_RELU6, 7>), dim3(grid), dim3(threads), 0, st, x, in_s, in_t, w, y, part, g);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_NONE, 7>), dim3(grid), dim3(threads), 0, st, x, in_s, in_t, w, y, part, g);
  }
}

void launch_dw_dgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *w,
                     const bf16_t *yprev, const float *ps, const float *pt, bf16_t *gout,
                     float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int threads = dw_block_threads(C);
  const int TW = threads / (C / 8);
  const int pix = stride == 1 ? 7 : 14;
  const int rpw = dw_rows_per_wg(B * H, (W + pix - 1) / pix, TW, 2);
  const int grid = (B * H + rpw - 1) / rpw;
  DwGeom g{B, H, W, C, Ho, Wo, rpw};
  if (stride == 1)
    hipLaunchKernelGGL((dw_dgrad_kernel<1, 7>), dim3(grid), dim3(threads), 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g);
  else
    hipLaunchKernelGGL((dw_dgrad_kernel<2, 14>), dim3(grid), dim3(threads), 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g);
}

void launch_dw_wgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *yprev,
                     const float *ps, const float *pt, float *part, float *grad, int B, int H, int W,
                     int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int threads = dw_block_threads(C);
  const int TW = threads / (C / 8);
  const int rpw = dw_rows_per_wg(B * Ho, (Wo + 6) / 7, TW, 4);
  const int grid = (B * Ho + rpw - 1) / rpw;
  DwGeom g{B, H, W, C, Ho, Wo, rpw};
  if (stride == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<1, 7>), dim3(grid), dim3(threads), 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  else
    hipLaunchKernelGGL((dw_wgrad_kernel<2, 7>), dim3(grid), dim3(threads), 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((9 * C + 63) / 64), dim3(256), 0, st, part, grid, C, grad);
}
