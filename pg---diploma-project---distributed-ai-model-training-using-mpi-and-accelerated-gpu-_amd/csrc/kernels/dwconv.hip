// Depthwise 3x3 convolution (pad 1, stride 1|2), NHWC bf16, for MobileNetV2.
//
// Reference op: the 17 depthwise Conv2d(groups=C) layers of torchvision
// MobileNetV2 run through cuDNN (SURVEY.md §2.6 "Depthwise conv 3x3"); on ROCm
// the library path (MIOpen / CK grouped-conv bwd-weight) takes ~23 ms per call
// at bs=128 (profiles/r1_torch_miopen_baseline_kernel_stats.csv).  Depthwise is
// pure bandwidth (1.8-4.5 FLOP/B), so these kernels are built around bytes and
// occupancy:
//
//  * thread = 4 channels (one 8-B vector) x a run of PIX output pixels along W;
//    a 64-lane wave still reads >= 256 contiguous bytes per pixel row;
//  * the 3 x (PIX*S+2) input window is streamed one kernel row at a time
//    (rolled loop) so each input vector is loaded and BN-transformed once per
//    row and only one row of the window is live; the 3x3 weights are stored
//    tap-major [9][C] in the flat parameter buffer (three 8-B loads per row) —
//    ~70-100 VGPRs, 4+ waves/SIMD to hide HBM latency;
//  * a workgroup owns a slab of <= 64 channels (blockIdx.y) over many rows, so
//    BN / weight-gradient partial rows stay small and rows stream long;
//  * the input operand is the *pre-BN* output of the producer: the producer's
//    BatchNorm-apply + ReLU6 is fused into the load (zero padding is applied in
//    the post-activation space, as in the reference graph);
//  * the forward epilogue emits per-workgroup BN partial sums of the output, the
//    dgrad epilogue emits the producer-BN backward partials — no standalone BN
//    passes over the activation.
#include "../common.h"

namespace {

constexpr int kMaxThreads = 256;
constexpr int CPT = 4;        // channels per thread

struct DwGeom {
  int B, H, W, C, Ho, Wo, rows_per_wg;
  int CC;  // channels handled by one workgroup (blockIdx.y selects the chunk)
};

PG_DEVICE void unpack4(const uint2 &u, float (&f)[CPT]) {
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
}
PG_DEVICE uint2 pack4(const float (&f)[CPT]) {
  uint2 u;
  u.x = pack2(f[0], f[1]);
  u.y = pack2(f[2], f[3]);
  return u;
}
PG_DEVICE uint2 ldg8(const bf16_t *p) { return *reinterpret_cast<const uint2 *>(p); }
PG_DEVICE void stg8(bf16_t *p, const uint2 &v) { *reinterpret_cast<uint2 *>(p) = v; }

// 4 channels at (b, ih, iw), producer BN (+relu6) applied; out of range -> 0
template <int ACT>
PG_DEVICE void load_act4(const bf16_t *__restrict__ x, const DwGeom &g, int b, int ih, int iw,
                         int c0, const float (&s)[CPT], const float (&t)[CPT], float (&v)[CPT]) {
  if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) v[k] = 0.f;
    return;
  }
  const size_t off = (((size_t)b * g.H + ih) * g.W + iw) * g.C + c0;
  unpack4(ldg8(x + off), v);
#pragma unroll
  for (int k = 0; k < CPT; ++k) v[k] = act_apply<ACT>(v[k], s[k], t[k]);
}

// weights are stored tap-major [9][C] (bf16 shadow of the flat parameter buffer; the
// torch-layout Parameter is a strided view of it), so one kernel row is 3 x 8-B loads
PG_DEVICE void ldw4(const bf16_t *__restrict__ w, int C, int q, int c0, float (&o)[CPT]) {
  unpack4(ldg8(w + (size_t)q * C + c0), o);
}

// Block-level reduction of per-thread [NV][CPT] channel partials of this workgroup's CC
// channels into part[blockIdx.x][NV][C] (columns cbase..cbase+CC); tid = tw * C4 + c4.
// lds must hold TW*CC floats (<= 1024).
template <int NV>
PG_DEVICE void block_channel_partials(float (&acc)[NV][CPT], float *__restrict__ part, int C, int CC,
                                      int cbase, int TW, float *lds) {
  const int tid = threadIdx.x;
  const int C4 = CC / CPT;
  const int c4 = tid % C4, tw = tid / C4;
  const bool active = tw < TW;
  for (int v = 0; v < NV; ++v) {
    if (active) {
      *reinterpret_cast<float4 *>(lds + tw * CC + c4 * CPT) =
          make_float4(acc[v][0], acc[v][1], acc[v][2], acc[v][3]);
    }
    __syncthreads();
    for (int c = tid; c < CC; c += blockDim.x) {
      float s = 0.f;
      for (int w = 0; w < TW; ++w) s += lds[w * CC + c];
      part[((size_t)blockIdx.x * NV + v) * C + cbase + c] = s;
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
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int C4 = g.CC / CPT;
  const int TW = blockDim.x / C4;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, tw = tid / C4;
  const int cbase = blockIdx.y * g.CC;
  const int c0 = cbase + c4 * CPT;
  constexpr int NCOL = (PIX - 1) * S + 3;

  float s[CPT], t[CPT], stats[2][CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    s[k] = (ACT != ACT_NONE) ? in_s[c0 + k] : 1.f;
    t[k] = (ACT != ACT_NONE) ? in_t[c0 + k] : 0.f;
    stats[0][k] = stats[1][k] = 0.f;
  }
  __syncthreads();

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
      float acc[PIX][CPT];
#pragma unroll
      for (int o = 0; o < PIX; ++o)
#pragma unroll
        for (int k = 0; k < CPT; ++k) acc[o][k] = 0.f;
#pragma unroll 1
      for (int dh = 0; dh < 3; ++dh) {
        const int ih = oh * S - 1 + dh;
        float w0[CPT], w1[CPT], w2[CPT];
        ldw4(w, g.C, dh * 3 + 0, c0, w0);
        ldw4(w, g.C, dh * 3 + 1, c0, w1);
        ldw4(w, g.C, dh * 3 + 2, c0, w2);
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int iw = ow0 * S - 1 + j;
          float v[CPT];
          load_act4<ACT>(x, g, b, ih, iw, c0, s, t, v);
#pragma unroll
          for (int o = 0; o < PIX; ++o) {
            const int dw = j - o * S;
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < CPT; ++k)
                acc[o][k] = fmaf(v[k], dw == 0 ? w0[k] : (dw == 1 ? w1[k] : w2[k]), acc[o][k]);
            }
          }
        }
      }
#pragma unroll
      for (int o = 0; o < PIX; ++o) {
        if (ow0 + o < g.Wo) {
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow0 + o) * g.C + c0;
          stg8(y + off, pack4(acc[o]));
#pragma unroll
          for (int k = 0; k < CPT; ++k) {
            stats[0][k] += acc[o][k];
            stats[1][k] = fmaf(acc[o][k], acc[o][k], stats[1][k]);
          }
        }
      }
    }
  }
  __syncthreads();
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, TW, red);
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
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int C4 = g.CC / CPT;
  const int TW = blockDim.x / C4;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, tw = tid / C4;
  const int cbase = blockIdx.y * g.CC;
  const int c0 = cbase + c4 * CPT;
  // PIX input pixels per item; output columns touching them:
  constexpr int NCOL = (S == 1) ? PIX + 2 : PIX / 2 + 2;

  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT], stats[2][CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    al[k] = coef[c0 + k];
    be[k] = coef[g.C + c0 + k];
    ga[k] = coef[2 * g.C + c0 + k];
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
    stats[0][k] = stats[1][k] = 0.f;
  }
  __syncthreads();
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
      float acc[PIX][CPT];
#pragma unroll
      for (int o = 0; o < PIX; ++o)
#pragma unroll
        for (int k = 0; k < CPT; ++k) acc[o][k] = 0.f;
#pragma unroll 1
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
        float w0[CPT], w1[CPT], w2[CPT];
        ldw4(w, g.C, dh * 3 + 0, c0, w0);
        ldw4(w, g.C, dh * 3 + 1, c0, w1);
        ldw4(w, g.C, dh * 3 + 2, c0, w2);
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int ow = (S == 1) ? iw0 - 1 + j : (iw0 >> 1) - 1 + j;
          if (ow < 0 || ow >= g.Wo) continue;
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow) * g.C + c0;
          float gv[CPT], yv[CPT];
          unpack4(ldg8(gin + off), gv);
          unpack4(ldg8(yself + off), yv);
#pragma unroll
          for (int k = 0; k < CPT; ++k) gv[k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
#pragma unroll
          for (int i = 0; i < PIX; ++i) {
            const int dw = (S == 1) ? (i - j + 2) : (i + 3 - 2 * j);
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < CPT; ++k)
                acc[i][k] = fmaf(gv[k], dw == 0 ? w0[k] : (dw == 1 ? w1[k] : w2[k]), acc[i][k]);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < PIX; ++i) {
        if (iw0 + i < g.W) {
          const size_t off = (((size_t)b * g.H + ih) * g.W + iw0 + i) * g.C + c0;
          float yp[CPT];
          unpack4(ldg8(yprev + off), yp);
#pragma unroll
          for (int k = 0; k < CPT; ++k) acc[i][k] *= relu6_mask(yp[k], s[k], t[k]);
          const uint2 packed = pack4(acc[i]);
          float gr[CPT];
          unpack4(packed, gr);  // statistics of the stored (bf16) gradient
#pragma unroll
          for (int k = 0; k < CPT; ++k) {
            stats[0][k] += gr[k];
            stats[1][k] = fmaf(gr[k], yp[k], stats[1][k]);
          }
          stg8(gout + off, packed);
        }
      }
    }
  }
  __syncthreads();
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, TW, red);
}

// ---------------------------------------------------------------------------
// wgrad: dW[c][tap] partials per workgroup  [P][9][C]
// ---------------------------------------------------------------------------
template <int S, int PIX>
__global__ __launch_bounds__(kMaxThreads) void dw_wgrad_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ yprev, const float *__restrict__ ps, const float *__restrict__ pt,
    float *__restrict__ part, DwGeom g) {
  __shared__ __attribute__((aligned(16))) float lds[1024];
  const int C4 = g.CC / CPT;
  const int TW = blockDim.x / C4;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, tw = tid / C4;
  const int cbase = blockIdx.y * g.CC;
  const int c0 = cbase + c4 * CPT;
  constexpr int NCOL = (PIX - 1) * S + 3;

  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT];
  float accw[9][CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
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
      float dy[PIX][CPT];
#pragma unroll
      for (int o = 0; o < PIX; ++o) {
        if (ow0 + o < g.Wo) {
          const size_t off = (((size_t)b * g.Ho + oh) * g.Wo + ow0 + o) * g.C + c0;
          float gv[CPT], yv[CPT];
          unpack4(ldg8(gin + off), gv);
          unpack4(ldg8(yself + off), yv);
#pragma unroll
          for (int k = 0; k < CPT; ++k) dy[o][k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
        } else {
#pragma unroll
          for (int k = 0; k < CPT; ++k) dy[o][k] = 0.f;
        }
      }
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        const int ih = oh * S - 1 + dh;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int iw = ow0 * S - 1 + j;
          float v[CPT];
          load_act4<ACT_BN_RELU6>(yprev, g, b, ih, iw, c0, s, t, v);
#pragma unroll
          for (int o = 0; o < PIX; ++o) {
            const int dw = j - o * S;
            if (dw >= 0 && dw <= 2) {
#pragma unroll
              for (int k = 0; k < CPT; ++k) accw[dh * 3 + dw][k] = fmaf(dy[o][k], v[k], accw[dh * 3 + dw][k]);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep one window row live
      }
    }
  }
  block_channel_partials<9>(accw, part, g.C, g.CC, cbase, TW, lds);
}

// reduce [P][9][C] -> grad [9][C] fp32
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
    grad[idx] = s;  // [9][C] tap-major, the layout of the flat parameter buffer
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
constexpr int kPixF = 4, kPixD1 = 4, kPixD2 = 8, kPixW = 4;

// channels per workgroup: the largest multiple of 4 dividing C that is <= 64, so a
// workgroup covers many pixels of a narrow channel slab (long rows per thread group,
// small BN/weight partial rows) instead of all channels of very few pixels
int dw_cc(int C) {
  for (int cc = 64; cc >= 4; cc -= 4)
    if (C % cc == 0) return cc;
  return 4;
}

int dw_block_threads(int C) {
  const int C4 = dw_cc(C) / CPT;
  int TW = kMaxThreads / C4;
  if (TW < 1) TW = 1;
  return C4 * TW;
}

int dw_rows_per_wg(int rows_total, int per_row_items, int TW, int target_items_per_thread,
                   int min_wgs) {
  int rpw = (TW * target_items_per_thread + per_row_items - 1) / per_row_items;
  if (rpw < 1) rpw = 1;
  while (rpw > 1 && (rows_total + rpw - 1) / rpw < min_wgs) rpw >>= 1;
  return rpw;
}

struct DwLaunch {
  int threads, rpw, grid, chunks;
};

DwLaunch dw_launch(int kind, int B, int H, int W, int C, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int threads = dw_block_threads(C);
  const int TW = threads / (dw_cc(C) / CPT);
  const int chunks = C / dw_cc(C);
  const int min_wgs = (2048 + chunks - 1) / chunks;
  DwLaunch l{threads, 1, 1, chunks};
  if (kind == 0) {  // fwd
    l.rpw = dw_rows_per_wg(B * Ho, (Wo + kPixF - 1) / kPixF, TW, 4, min_wgs);
    l.grid = (B * Ho + l.rpw - 1) / l.rpw;
  } else if (kind == 1) {  // dgrad (over input rows)
    const int pix = stride == 1 ? kPixD1 : kPixD2;
    l.rpw = dw_rows_per_wg(B * H, (W + pix - 1) / pix, TW, 4, min_wgs);
    l.grid = (B * H + l.rpw - 1) / l.rpw;
  } else {  // wgrad
    l.rpw = dw_rows_per_wg(B * Ho, (Wo + kPixW - 1) / kPixW, TW, 8, (1024 + chunks - 1) / chunks);
    l.grid = (B * Ho + l.rpw - 1) / l.rpw;
  }
  return l;
}
}  // namespace

int dw_fwd_num_partials(int B, int H, int W, int C, int stride) { return dw_launch(0, B, H, W, C, stride).grid; }
int dw_dgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_launch(1, B, H, W, C, stride).grid; }
int dw_wgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_launch(2, B, H, W, C, stride).grid; }

void launch_dw_fwd(const bf16_t *x, const float *in_s, const float *in_t, int act, const bf16_t *w,
                   bf16_t *y, float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const DwLaunch l = dw_launch(0, B, H, W, C, stride);
  DwGeom g{B, H, W, C, Ho, Wo, l.rpw, dw_cc(C)};
  if (stride == 1) {
    if (act == ACT_BN_RELU6)
      hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_BN_RELU6, kPixF>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, x, in_s, in_t, w, y, part, g);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_NONE, kPixF>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, x, in_s, in_t, w, y, part, g);
  } else {
    if (act == ACT_BN_RELU6)
      hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_BN_RELU6, kPixF>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, x, in_s, in_t, w, y, part, g);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_NONE, kPixF>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, x, in_s, in_t, w, y, part, g);
  }
}

void launch_dw_dgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *w,
                     const bf16_t *yprev, const float *ps, const float *pt, bf16_t *gout,
                     float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const DwLaunch l = dw_launch(1, B, H, W, C, stride);
  DwGeom g{B, H, W, C, Ho, Wo, l.rpw, dw_cc(C)};
  if (stride == 1)
    hipLaunchKernelGGL((dw_dgrad_kernel<1, kPixD1>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g);
  else
    hipLaunchKernelGGL((dw_dgrad_kernel<2, kPixD2>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g);
}

void launch_colsum(const float *src, int R, long long n, float *dst, int &rows_out, hipStream_t st);

void launch_dw_wgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *yprev,
                     const float *ps, const float *pt, float *part, float *grad, int B, int H, int W,
                     int C, int stride, hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const DwLaunch l = dw_launch(2, B, H, W, C, stride);
  DwGeom g{B, H, W, C, Ho, Wo, l.rpw, dw_cc(C)};
  if (stride == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<1, kPixW>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  else
    hipLaunchKernelGGL((dw_wgrad_kernel<2, kPixW>), dim3(l.grid, l.chunks), dim3(l.threads), 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  // two-level deterministic reduction of the [P][9C] partials (level 1 written after them)
  int rows = l.grid;
  float *tmp = part + (size_t)l.grid * 9 * C;
  launch_colsum(part, l.grid, 9LL * C, tmp, rows, st);
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((9 * C + 63) / 64), dim3(256), 0, st,
                     rows == l.grid ? part : tmp, rows, C, grad);
}
