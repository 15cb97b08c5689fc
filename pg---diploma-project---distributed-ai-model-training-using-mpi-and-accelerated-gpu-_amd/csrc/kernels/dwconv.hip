// Depthwise 3x3 convolution (pad 1, stride 1|2), NHWC bf16, for MobileNetV2.
//
// Reference op: the 17 depthwise Conv2d(groups=C) layers of torchvision
// MobileNetV2 run through cuDNN (SURVEY.md §2.6 "Depthwise conv 3x3"); on ROCm
// the library path (MIOpen / CK grouped-conv bwd-weight) takes ~23 ms per call
// at bs=128 (profiles/r1_torch_miopen_baseline_kernel_stats.csv).  Depthwise is
// pure bandwidth (1.8-4.5 FLOP/B), so these kernels are organised around the
// memory system:
//
//  * vertical strips: a thread owns 4 channels (one 8-B vector) of ONE output
//    column and walks R rows down the image, keeping a rolling 3-row x 3-column
//    window in registers — every input row is loaded once per thread, and the
//    lanes of a wave (channel-fastest, then column) read one contiguous run of
//    pixels per load instruction (the neighbours' halo columns hit the same lines);
//  * a workgroup = a tile of TWc columns x R rows of one image and a slab of
//    CC <= 64 channels (one slab per workgroup): small per-workgroup partial rows, long
//    streams; ~100 VGPRs;
//  * weights are tap-major [9][C] in the flat parameter buffer (one 8-B load per
//    tap and 4 channels);
//  * the producer's BatchNorm-apply + ReLU6 is fused into the input load (zero
//    padding in the post-activation space), the forward epilogue emits this
//    layer's BN partial sums, the dgrad epilogue the producer-BN backward
//    partials; the weight gradient is reduced per workgroup and then by a
//    deterministic two-level column sum.
#include "../common.h"

#include <cstdlib>

namespace {

constexpr int CPT = 4;        // channels per thread
constexpr int kRows = 28;     // rows per strip (swept 4..112 on MI355X: 28 fastest end to end)
#ifndef PGDIST_DGRAD_PF
#define PGDIST_DGRAD_PF 2
#endif
constexpr int kDgradPrefetch = PGDIST_DGRAD_PF;   // rows of loads in flight ahead (stride-1 dgrad)

struct DwGeom {
  int B, H, W, C, Ho, Wo;
  int CC;     // channels per workgroup (tile_of() decodes the slab)
  int TWc;    // columns per workgroup
  int R;      // rows per workgroup
  int tiles_w, tiles_h;
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

PG_DEVICE void zero4(float (&v)[CPT]) {
#pragma unroll
  for (int k = 0; k < CPT; ++k) v[k] = 0.f;
}

// 4 channels at (b, ih, iw) of an [*, H, W, C] tensor, producer BN (+relu6) applied; OOB -> 0
template <int ACT>
PG_DEVICE void load_act4(const bf16_t *__restrict__ x, int H, int W, int C, int b, int ih, int iw,
                         int c0, const float (&s)[CPT], const float (&t)[CPT], float (&v)[CPT]) {
  if (ih < 0 || ih >= H || iw < 0 || iw >= W) {
    zero4(v);
    return;
  }
  unpack4(ldg8(x + (((size_t)b * H + ih) * W + iw) * C + c0), v);
#pragma unroll
  for (int k = 0; k < CPT; ++k) v[k] = act_apply<ACT>(v[k], s[k], t[k]);
}

// dy = a*g + b*y + c at (b, oh, ow) of [*, Ho, Wo, C]; OOB -> 0
PG_DEVICE void load_dy4(const bf16_t *__restrict__ g, const bf16_t *__restrict__ y, int Ho, int Wo, int C,
                        int b, int oh, int ow, int c0, const float (&al)[CPT], const float (&be)[CPT],
                        const float (&ga)[CPT], float (&v)[CPT]) {
  if (oh < 0 || oh >= Ho || ow < 0 || ow >= Wo) {
    zero4(v);
    return;
  }
  const size_t off = (((size_t)b * Ho + oh) * Wo + ow) * C + c0;
  float gv[CPT], yv[CPT];
  unpack4(ldg8(g + off), gv);
  unpack4(ldg8(y + off), yv);
#pragma unroll
  for (int k = 0; k < CPT; ++k) v[k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
}


// Raw (untransformed) 3-column row segment, loaded one strip row ahead so the
// loads are in flight while the current row's FMAs run (software pipelining).
struct Raw3 {
  uint2 v[3];
};
PG_DEVICE void load_raw3(Raw3 &r, const bf16_t *__restrict__ x, int H, int W, int C, int b, int ih,
                         int iw0, int c0) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int iw = iw0 + d;
    r.v[d] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? ldg8(x + (((size_t)b * H + ih) * W + iw) * C + c0)
                                                      : make_uint2(0, 0);
  }
}
// transform a raw row; out-of-range entries must become exactly 0 after the transform
template <int ACT>
PG_DEVICE void act3(const Raw3 &r, int ih, int H, int iw0, int W, const float (&s)[CPT], const float (&t)[CPT],
                    float (&out)[3][CPT]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const bool ok = ih >= 0 && ih < H && iw0 + d >= 0 && iw0 + d < W;
    unpack4(r.v[d], out[d]);
#pragma unroll
    for (int k = 0; k < CPT; ++k) out[d][k] = ok ? act_apply<ACT>(out[d][k], s[k], t[k]) : 0.f;
  }
}

// Workgroup decode.  The 1-D grid enumerates (tile, channel slab) pairs so that the slabs
// of one spatial tile are 8 workgroup ids apart: same XCD (ids are dealt to the 8 XCDs
// round-robin) and dispatched together, so the 128-B lines shared by neighbouring slabs
// (a pixel's C channels are contiguous in NHWC) are fetched from HBM once into that L2.
struct Tile {
  int b, r0, w0;
  int idx;     // tile index (partial row)
  int slab;    // channel slab
};
PG_DEVICE Tile tile_of(const DwGeom &g) {
  const int L = blockIdx.x;
  const int nslab = g.C / g.CC;
  const int ntiles = g.B * g.tiles_h * g.tiles_w;
  const int full = (ntiles / 8) * 8 * nslab;
  int t, sl;
  if (L < full) {
    t = (L / (8 * nslab)) * 8 + L % 8;
    sl = (L / 8) % nslab;
  } else {
    const int rem = ntiles % 8, Lr = L - full;
    t = (ntiles / 8) * 8 + Lr % rem;
    sl = Lr / rem;
  }
  const int tw = t % g.tiles_w;
  const int rest = t / g.tiles_w;
  const int th = rest % g.tiles_h;
  return Tile{rest / g.tiles_h, th * g.R, tw * g.TWc, t, sl};
}

// Block-level reduction of per-thread [NV][CPT] channel partials of this workgroup's CC
// channels into part[prow][NV][C] (columns cbase..cbase+CC); tid = col * C4 + c4.
template <int NV>
PG_DEVICE void block_channel_partials(float (&acc)[NV][CPT], float *__restrict__ part, int C, int CC,
                                      int cbase, int ncol, float *lds, int prow) {
  const int tid = threadIdx.x;
  const int C4 = CC / CPT;
  const int c4 = tid % C4, col = tid / C4;
  for (int v = 0; v < NV; ++v) {
    if (col < ncol)
      *reinterpret_cast<float4 *>(lds + col * CC + c4 * CPT) = make_float4(acc[v][0], acc[v][1], acc[v][2], acc[v][3]);
    __syncthreads();
    for (int c = tid; c < CC; c += blockDim.x) {
      float s = 0.f;
      for (int w = 0; w < ncol; ++w) s += lds[w * CC + c];
      part[((size_t)prow * NV + v) * C + cbase + c] = s;
    }
    __syncthreads();
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// forward: y = dwconv(act(x)), partial (sum y, sum y^2)
// ---------------------------------------------------------------------------
template <int S, int ACT>
__global__ __launch_bounds__(256) void dw_fwd_kernel(
    const bf16_t *__restrict__ x, const float *__restrict__ in_s, const float *__restrict__ in_t,
    const bf16_t *__restrict__ w, bf16_t *__restrict__ y, float *__restrict__ part, DwGeom g) {
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int C4 = g.CC / CPT;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int ow = tl.w0 + col;
  const bool active = col < g.TWc && ow < g.Wo;

  float s[CPT], t[CPT], stats[2][CPT];
  uint2 wt[9];   // packed bf16 taps (unpacked at use: fewer live VGPRs -> more waves)
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    s[k] = (ACT != ACT_NONE) ? in_s[c0 + k] : 1.f;
    t[k] = (ACT != ACT_NONE) ? in_t[c0 + k] : 0.f;
    stats[0][k] = stats[1][k] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) wt[q] = ldg8(w + (size_t)q * g.C + c0);

  if (active) {
    const int oh_end = min(tl.r0 + g.R, g.Ho);
    const int iw0 = ow * S - 1;
    // rolling window win[r][dw][k] = input rows oh*S-1+r; next rows prefetched raw
    float win[3][3][CPT];
    Raw3 n1, n2;
    {
      const int ih0 = tl.r0 * S - 1;
      Raw3 r0, r1, r2;
      load_raw3(r0, x, g.H, g.W, g.C, tl.b, ih0, iw0, c0);
      load_raw3(r1, x, g.H, g.W, g.C, tl.b, ih0 + 1, iw0, c0);
      load_raw3(r2, x, g.H, g.W, g.C, tl.b, ih0 + 2, iw0, c0);
      act3<ACT>(r0, ih0, g.H, iw0, g.W, s, t, win[0]);
      act3<ACT>(r1, ih0 + 1, g.H, iw0, g.W, s, t, win[1]);
      act3<ACT>(r2, ih0 + 2, g.H, iw0, g.W, s, t, win[2]);
    }
    for (int oh = tl.r0; oh < oh_end; ++oh) {
      const int ihb = oh * S - 1;
      if (oh > tl.r0) {
        if constexpr (S == 1) {
#pragma unroll
          for (int dw = 0; dw < 3; ++dw)
#pragma unroll
            for (int k = 0; k < CPT; ++k) {
              win[0][dw][k] = win[1][dw][k];
              win[1][dw][k] = win[2][dw][k];
            }
          act3<ACT>(n1, ihb + 2, g.H, iw0, g.W, s, t, win[2]);
        } else {
#pragma unroll
          for (int dw = 0; dw < 3; ++dw)
#pragma unroll
            for (int k = 0; k < CPT; ++k) win[0][dw][k] = win[2][dw][k];
          act3<ACT>(n1, ihb + 1, g.H, iw0, g.W, s, t, win[1]);
          act3<ACT>(n2, ihb + 2, g.H, iw0, g.W, s, t, win[2]);
        }
      }
      if (oh + 1 < oh_end) {   // prefetch the rows the next output row adds
        const int nb = (oh + 1) * S - 1;
        if constexpr (S == 1) {
          load_raw3(n1, x, g.H, g.W, g.C, tl.b, nb + 2, iw0, c0);
        } else {
          load_raw3(n1, x, g.H, g.W, g.C, tl.b, nb + 1, iw0, c0);
          load_raw3(n2, x, g.H, g.W, g.C, tl.b, nb + 2, iw0, c0);
        }
      }
      float acc[CPT];
      zero4(acc);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          float wv[CPT];
          unpack4(wt[r * 3 + dw], wv);
#pragma unroll
          for (int k = 0; k < CPT; ++k) acc[k] = fmaf(win[r][dw][k], wv[k], acc[k]);
        }
      stg8(y + (((size_t)tl.b * g.Ho + oh) * g.Wo + ow) * g.C + c0, pack4(acc));
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        stats[0][k] += acc[k];
        stats[1][k] = fmaf(acc[k], acc[k], stats[1][k]);
      }
    }
  }
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, g.TWc, red, tl.idx);
}

// ---------------------------------------------------------------------------
// dgrad: gout = mask_prev * dwconv^T(dy),  dy = a*g + b*y + c (this layer's BN backward)
// thread = one INPUT column, strip of input rows; partial (sum gout, sum gout*yprev)
// ---------------------------------------------------------------------------
// WG = true: the weight gradient of the same layer is accumulated on the way (fused dgrad +
// wgrad): every input pixel's z = relu6(BN(yprev)) meets exactly the dy taps the dgrad already
// holds in registers, so dW costs 9 FMAs per pixel and no second read of (g, y, yprev);
// per-workgroup wgrad partials go to wpart[tile][9][C] (reduced like dw_wgrad's).
template <int S, bool WG>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ w, const bf16_t *__restrict__ yprev, const float *__restrict__ ps,
    const float *__restrict__ pt, bf16_t *__restrict__ gout, float *__restrict__ part, DwGeom g,
    float *__restrict__ wpart) {
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int C4 = g.CC / CPT;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  // tiles over the INPUT grid (H x W)
  const int iw = tl.w0 + col;
  const bool active = col < g.TWc && iw < g.W;

  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT], stats[2][CPT];
  uint2 wtp[9];   // packed bf16 taps (unpacked at use: fewer live VGPRs -> more waves)
  float accw[WG ? 9 : 1][CPT];   // fused weight-gradient partials (tap-major)
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    al[k] = coef[c0 + k];
    be[k] = coef[g.C + c0 + k];
    ga[k] = coef[2 * g.C + c0 + k];
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
    stats[0][k] = stats[1][k] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < (WG ? 9 : 1); ++q)
#pragma unroll
    for (int k = 0; k < CPT; ++k) accw[q][k] = 0.f;
#pragma unroll
  for (int q = 0; q < 9; ++q) wtp[q] = ldg8(w + (size_t)q * g.C + c0);

  if (active) {
    const int ih_end = min(tl.r0 + g.R, g.H);
    if constexpr (S == 1) {
      // dx[ih][iw] = sum_{dh,dw} dy[ih+1-dh][iw+1-dw] * w[dh][dw];  window rows ih-1..ih+1 (as dy rows)
      float win[3][3][CPT];   // win[r][c]: dy row ih-1+r, col iw-1+c
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          load_dy4(gin, yself, g.Ho, g.Wo, g.C, tl.b, tl.r0 - 1 + r, iw - 1 + c, c0, al, be, ga, win[r][c]);
      // kPf-deep ring of raw loads (statically indexed: the row loop is unrolled by kPf):
      // dy row (r0 + 1 + i) sits in slot (i - 1) % kPf, yprev row (r0 + i) in slot i % kPf
      constexpr int kPf = kDgradPrefetch;
      Raw3 rg[kPf], ry[kPf];
      uint2 ypr[kPf];
#pragma unroll
      for (int q = 0; q < kPf; ++q) {
        load_raw3(rg[q], gin, g.Ho, g.Wo, g.C, tl.b, tl.r0 + 2 + q, iw - 1, c0);
        load_raw3(ry[q], yself, g.Ho, g.Wo, g.C, tl.b, tl.r0 + 2 + q, iw - 1, c0);
        const int r = tl.r0 + q;
        ypr[q] = r < ih_end ? ldg8(yprev + (((size_t)tl.b * g.H + r) * g.W + iw) * g.C + c0) : make_uint2(0, 0);
      }
      for (int base = 0; tl.r0 + base < ih_end; base += kPf) {
#pragma unroll
        for (int j = 0; j < kPf; ++j) {
          const int i = base + j, ih = tl.r0 + i;
          if (ih >= ih_end) break;
          if (i > 0) {
            const int sl = (j + kPf - 1) % kPf;   // slot of dy row ih + 1 (static after unrolling)
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
              for (int k = 0; k < CPT; ++k) {
                win[0][c][k] = win[1][c][k];
                win[1][c][k] = win[2][c][k];
              }
            const int oh = ih + 1;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const bool ok = oh >= 0 && oh < g.Ho && iw - 1 + c >= 0 && iw - 1 + c < g.Wo;
              float gv[CPT], yv[CPT];
              unpack4(rg[sl].v[c], gv);
              unpack4(ry[sl].v[c], yv);
#pragma unroll
              for (int k = 0; k < CPT; ++k) win[2][c][k] = ok ? fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k])) : 0.f;
            }
            // refill the slot with dy row ih + 1 + kPf
            load_raw3(rg[sl], gin, g.Ho, g.Wo, g.C, tl.b, ih + 1 + kPf, iw - 1, c0);
            load_raw3(ry[sl], yself, g.Ho, g.Wo, g.C, tl.b, ih + 1 + kPf, iw - 1, c0);
          }
          const uint2 ypc = ypr[j];
          {
            const int r = ih + kPf;
            ypr[j] = r < ih_end ? ldg8(yprev + (((size_t)tl.b * g.H + r) * g.W + iw) * g.C + c0) : make_uint2(0, 0);
          }
          float acc[CPT];
          zero4(acc);
          // dy row ih+1-dh = win[2-dh], col iw+1-dw = win[..][2-dw]
#pragma unroll
          for (int dh = 0; dh < 3; ++dh)
#pragma unroll
            for (int dw = 0; dw < 3; ++dw) {
              float wv[CPT];
              unpack4(wtp[dh * 3 + dw], wv);
#pragma unroll
              for (int k = 0; k < CPT; ++k) acc[k] = fmaf(win[2 - dh][2 - dw][k], wv[k], acc[k]);
            }
          const size_t off = (((size_t)tl.b * g.H + ih) * g.W + iw) * g.C + c0;
          float yp[CPT];
          unpack4(ypc, yp);
          if constexpr (WG) {   // dW[dh][dw] += z[ih][iw] * dy[ih+1-dh][iw+1-dw]
            float z[CPT];
#pragma unroll
            for (int k = 0; k < CPT; ++k) z[k] = relu6f(fmaf(yp[k], s[k], t[k]));
#pragma unroll
            for (int dh = 0; dh < 3; ++dh)
#pragma unroll
              for (int dw = 0; dw < 3; ++dw)
#pragma unroll
                for (int k = 0; k < CPT; ++k)
                  accw[WG ? dh * 3 + dw : 0][k] = fmaf(z[k], win[2 - dh][2 - dw][k], accw[WG ? dh * 3 + dw : 0][k]);
          }
#pragma unroll
          for (int k = 0; k < CPT; ++k) acc[k] *= relu6_mask(yp[k], s[k], t[k]);
          const uint2 packed = pack4(acc);
          float gr[CPT];
          unpack4(packed, gr);
#pragma unroll
          for (int k = 0; k < CPT; ++k) {
            stats[0][k] += gr[k];
            stats[1][k] = fmaf(gr[k], yp[k], stats[1][k]);
          }
          stg8(gout + off, packed);
        }
      }
    } else {
      // stride 2.  Column: even iw -> ow = iw/2 (dw=1); odd iw -> ow = (iw+1)/2 (dw=0), (iw-1)/2 (dw=2)
      // Row: even ih = 2o -> dy row o (dh=1); odd ih = 2o+1 -> dy rows o (dh=2), o+1 (dh=0)
      const bool odd_w = iw & 1;
      const int owA = odd_w ? (iw + 1) >> 1 : iw >> 1;   // dw = 0 (odd) or 1 (even)
      const int owB = (iw - 1) >> 1;                      // dw = 2 (odd only)
      // per-thread tap weights (selected with static indices: no runtime-indexed arrays)
      float wA[3][CPT], wB[3][CPT];   // [dh] for column A (dw = 0 if odd else 1) and B (dw = 2)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        float w0[CPT], w1[CPT], w2[CPT];
        unpack4(wtp[r * 3 + 0], w0);
        unpack4(wtp[r * 3 + 1], w1);
        unpack4(wtp[r * 3 + 2], w2);
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          wA[r][k] = odd_w ? w0[k] : w1[k];
          wB[r][k] = odd_w ? w2[k] : 0.f;
        }
      }
      // tiles start at even rows (R even).  Everything one iteration (2 input rows) ahead:
      // raw dy (g, y) of the next dy row and the yprev rows of the next iteration.
      auto ld_raw = [&](uint2 &dst, const bf16_t *src, int H_, int W_, int r, int c) {
        dst = (r >= 0 && r < H_ && c >= 0 && c < W_) ? ldg8(src + (((size_t)tl.b * H_ + r) * W_ + c) * g.C + c0)
                                                     : make_uint2(0, 0);
      };
      auto dy_of = [&](const uint2 &gg, const uint2 &yy, int r, int c, float (&v)[CPT]) {
        const bool ok = r >= 0 && r < g.Ho && c >= 0 && c < g.Wo;
        float gv[CPT], yv[CPT];
        unpack4(gg, gv);
        unpack4(yy, yv);
#pragma unroll
        for (int k = 0; k < CPT; ++k) v[k] = ok ? fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k])) : 0.f;
      };
      float cur[2][CPT], nxt[2][CPT];   // dy row o / o+1 at columns A, B
      float accA[WG ? 3 : 1][CPT], accB[WG ? 3 : 1][CPT];   // fused dW[dh][dwA] / dW[dh][2]
#pragma unroll
      for (int r = 0; r < (WG ? 3 : 1); ++r)
#pragma unroll
        for (int k = 0; k < CPT; ++k) accA[r][k] = accB[r][k] = 0.f;
      uint2 rgA, ryA, rgB, ryB;         // raw dy row o+1 (columns A, B)
      uint2 yp0r, yp1r;                 // raw yprev rows of the current iteration
      int o = tl.r0 >> 1;
      {
        uint2 gA, yA, gB, yB;
        ld_raw(gA, gin, g.Ho, g.Wo, o, owA);
        ld_raw(yA, yself, g.Ho, g.Wo, o, owA);
        ld_raw(gB, gin, g.Ho, g.Wo, o, odd_w ? owB : -1);
        ld_raw(yB, yself, g.Ho, g.Wo, o, odd_w ? owB : -1);
        dy_of(gA, yA, o, owA, cur[0]);
        dy_of(gB, yB, o, odd_w ? owB : -1, cur[1]);
      }
      ld_raw(rgA, gin, g.Ho, g.Wo, o + 1, owA);
      ld_raw(ryA, yself, g.Ho, g.Wo, o + 1, owA);
      ld_raw(rgB, gin, g.Ho, g.Wo, o + 1, odd_w ? owB : -1);
      ld_raw(ryB, yself, g.Ho, g.Wo, o + 1, odd_w ? owB : -1);
      ld_raw(yp0r, yprev, g.H, g.W, tl.r0, iw);
      ld_raw(yp1r, yprev, g.H, g.W, tl.r0 + 1 < ih_end ? tl.r0 + 1 : -1, iw);
      for (int ih = tl.r0; ih < ih_end; ih += 2) {
        o = ih >> 1;
        dy_of(rgA, ryA, o + 1, owA, nxt[0]);
        dy_of(rgB, ryB, o + 1, odd_w ? owB : -1, nxt[1]);
        const uint2 ypc[2] = {yp0r, yp1r};
        if (ih + 2 < ih_end) {   // next iteration's operands, in flight during this one's FMAs
          ld_raw(rgA, gin, g.Ho, g.Wo, o + 2, owA);
          ld_raw(ryA, yself, g.Ho, g.Wo, o + 2, owA);
          ld_raw(rgB, gin, g.Ho, g.Wo, o + 2, odd_w ? owB : -1);
          ld_raw(ryB, yself, g.Ho, g.Wo, o + 2, odd_w ? owB : -1);
          ld_raw(yp0r, yprev, g.H, g.W, ih + 2, iw);
          ld_raw(yp1r, yprev, g.H, g.W, ih + 3 < ih_end ? ih + 3 : -1, iw);
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int r = ih + half;
          if (r >= ih_end) break;
          float acc[CPT];
          zero4(acc);
          if (half == 0) {          // even row: dh = 1, dy row o
#pragma unroll
            for (int k = 0; k < CPT; ++k)
              acc[k] = fmaf(cur[0][k], wA[1][k], fmaf(cur[1][k], wB[1][k], acc[k]));
          } else {                  // odd row: dh = 2 (row o), dh = 0 (row o+1)
#pragma unroll
            for (int k = 0; k < CPT; ++k) {
              acc[k] = fmaf(cur[0][k], wA[2][k], fmaf(cur[1][k], wB[2][k], acc[k]));
              acc[k] = fmaf(nxt[0][k], wA[0][k], fmaf(nxt[1][k], wB[0][k], acc[k]));
            }
          }
          const size_t off = (((size_t)tl.b * g.H + r) * g.W + iw) * g.C + c0;
          float yp[CPT];
          unpack4(ypc[half], yp);
          if constexpr (WG) {
            float z[CPT];
#pragma unroll
            for (int k = 0; k < CPT; ++k) z[k] = relu6f(fmaf(yp[k], s[k], t[k]));
            if (half == 0) {          // dh = 1 with dy row o
#pragma unroll
              for (int k = 0; k < CPT; ++k) {
                accA[WG ? 1 : 0][k] = fmaf(z[k], cur[0][k], accA[WG ? 1 : 0][k]);
                accB[WG ? 1 : 0][k] = fmaf(z[k], cur[1][k], accB[WG ? 1 : 0][k]);
              }
            } else {                  // dh = 2 with row o, dh = 0 with row o+1
#pragma unroll
              for (int k = 0; k < CPT; ++k) {
                accA[WG ? 2 : 0][k] = fmaf(z[k], cur[0][k], accA[WG ? 2 : 0][k]);
                accB[WG ? 2 : 0][k] = fmaf(z[k], cur[1][k], accB[WG ? 2 : 0][k]);
                accA[0][k] = fmaf(z[k], nxt[0][k], accA[0][k]);
                accB[0][k] = fmaf(z[k], nxt[1][k], accB[0][k]);
              }
            }
          }
#pragma unroll
          for (int k = 0; k < CPT; ++k) acc[k] *= relu6_mask(yp[k], s[k], t[k]);
          const uint2 packed = pack4(acc);
          float gr[CPT];
          unpack4(packed, gr);
#pragma unroll
          for (int k = 0; k < CPT; ++k) {
            stats[0][k] += gr[k];
            stats[1][k] = fmaf(gr[k], yp[k], stats[1][k]);
          }
          stg8(gout + off, packed);
        }
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          cur[0][k] = nxt[0][k];
          cur[1][k] = nxt[1][k];
        }
      }
      if constexpr (WG) {   // column A is tap dw = 0 (odd iw) or 1 (even iw); column B is dw = 2
#pragma unroll
        for (int dh = 0; dh < 3; ++dh)
#pragma unroll
          for (int k = 0; k < CPT; ++k) {
            accw[WG ? dh * 3 + 0 : 0][k] = odd_w ? accA[WG ? dh : 0][k] : 0.f;
            accw[WG ? dh * 3 + 1 : 0][k] = odd_w ? 0.f : accA[WG ? dh : 0][k];
            accw[WG ? dh * 3 + 2 : 0][k] = accB[WG ? dh : 0][k];
          }
      }
    }
  }
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, g.TWc, red, tl.idx);
  if constexpr (WG) block_channel_partials<9>(accw, wpart, g.C, g.CC, cbase, g.TWc, red, tl.idx);
}

// ---------------------------------------------------------------------------
// wgrad: dW[tap][c] partials per workgroup  [P][9][C]
// thread = one output column, strip of output rows, rolling z window
// ---------------------------------------------------------------------------
template <int S>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ yprev, const float *__restrict__ ps, const float *__restrict__ pt,
    float *__restrict__ part, DwGeom g) {
  __shared__ __attribute__((aligned(16))) float lds[1024];
  const int C4 = g.CC / CPT;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int ow = tl.w0 + col;
  const bool active = col < g.TWc && ow < g.Wo;

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
  if (active) {
    const int oh_end = min(tl.r0 + g.R, g.Ho);
    const int iw0 = ow * S - 1;
    float win[3][3][CPT];
    Raw3 n1, n2;
    uint2 gnext = make_uint2(0, 0), ynext = make_uint2(0, 0);
    {
      const int ih0 = tl.r0 * S - 1;
      Raw3 r0, r1, r2;
      load_raw3(r0, yprev, g.H, g.W, g.C, tl.b, ih0, iw0, c0);
      load_raw3(r1, yprev, g.H, g.W, g.C, tl.b, ih0 + 1, iw0, c0);
      load_raw3(r2, yprev, g.H, g.W, g.C, tl.b, ih0 + 2, iw0, c0);
      const size_t off = (((size_t)tl.b * g.Ho + tl.r0) * g.Wo + ow) * g.C + c0;
      gnext = ldg8(gin + off);
      ynext = ldg8(yself + off);
      act3<ACT_BN_RELU6>(r0, ih0, g.H, iw0, g.W, s, t, win[0]);
      act3<ACT_BN_RELU6>(r1, ih0 + 1, g.H, iw0, g.W, s, t, win[1]);
      act3<ACT_BN_RELU6>(r2, ih0 + 2, g.H, iw0, g.W, s, t, win[2]);
    }
    for (int oh = tl.r0; oh < oh_end; ++oh) {
      const int ihb = oh * S - 1;
      if (oh > tl.r0) {
        if constexpr (S == 1) {
#pragma unroll
          for (int dw = 0; dw < 3; ++dw)
#pragma unroll
            for (int k = 0; k < CPT; ++k) {
              win[0][dw][k] = win[1][dw][k];
              win[1][dw][k] = win[2][dw][k];
            }
          act3<ACT_BN_RELU6>(n1, ihb + 2, g.H, iw0, g.W, s, t, win[2]);
        } else {
#pragma unroll
          for (int dw = 0; dw < 3; ++dw)
#pragma unroll
            for (int k = 0; k < CPT; ++k) win[0][dw][k] = win[2][dw][k];
          act3<ACT_BN_RELU6>(n1, ihb + 1, g.H, iw0, g.W, s, t, win[1]);
          act3<ACT_BN_RELU6>(n2, ihb + 2, g.H, iw0, g.W, s, t, win[2]);
        }
      }
      float dy[CPT];
      {
        float gv[CPT], yv[CPT];
        unpack4(gnext, gv);
        unpack4(ynext, yv);
#pragma unroll
        for (int k = 0; k < CPT; ++k) dy[k] = fmaf(al[k], gv[k], fmaf(be[k], yv[k], ga[k]));
      }
      if (oh + 1 < oh_end) {   // prefetch next row: z rows and dy
        const int nb = (oh + 1) * S - 1;
        if constexpr (S == 1) {
          load_raw3(n1, yprev, g.H, g.W, g.C, tl.b, nb + 2, iw0, c0);
        } else {
          load_raw3(n1, yprev, g.H, g.W, g.C, tl.b, nb + 1, iw0, c0);
          load_raw3(n2, yprev, g.H, g.W, g.C, tl.b, nb + 2, iw0, c0);
        }
        const size_t off = (((size_t)tl.b * g.Ho + oh + 1) * g.Wo + ow) * g.C + c0;
        gnext = ldg8(gin + off);
        ynext = ldg8(yself + off);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int k = 0; k < CPT; ++k) accw[r * 3 + dw][k] = fmaf(dy[k], win[r][dw][k], accw[r * 3 + dw][k]);
    }
  }
  block_channel_partials<9>(accw, part, g.C, g.CC, cbase, g.TWc, lds, tl.idx);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
// channels per workgroup: the largest multiple of 4 dividing C that is <= 64
int dw_cc(int C) {
  for (int cc = 64; cc >= 4; cc -= 4)
    if (C % cc == 0) return cc;
  return 4;
}

// kind 0 = fwd (tiles over the output grid), 1 = dgrad (input grid), 2 = wgrad (output grid)
DwGeom dw_geom(int kind, int B, int H, int W, int C, int stride) {
  DwGeom g;
  g.B = B;
  g.H = H;
  g.W = W;
  g.C = C;
  g.Ho = (H - 1) / stride + 1;
  g.Wo = (W - 1) / stride + 1;
  g.CC = dw_cc(C);
  const int C4 = g.CC / CPT;
  const int gw = kind == 1 ? W : g.Wo, gh = kind == 1 ? H : g.Ho;
  int twc = 256 / C4;
  if (twc > gw) twc = gw;
  g.TWc = twc;
  static const int env_rows = [] {
    const char *e = getenv("PGDIST_DW_ROWS");
    return e ? atoi(e) : 0;
  }();
  static const int env_wrows = [] {
    const char *e = getenv("PGDIST_DW_WROWS");
    return e ? atoi(e) : 0;
  }();
  int R = env_rows > 0 ? env_rows : kRows;
  if (kind == 2) R = env_wrows > 0 ? env_wrows : kRows;
  // (PGDIST_DW_ROWS / PGDIST_DW_WROWS override the strip length for tuning experiments)
  if (kind == 1 && stride == 2 && (R & 1)) ++R;  // dgrad s2 tiles start on even input rows
  if (R > gh) R = (kind == 1 && stride == 2) ? ((gh + 1) & ~1) : gh;
  g.R = R;
  g.tiles_w = (gw + g.TWc - 1) / g.TWc;
  g.tiles_h = (gh + g.R - 1) / g.R;
  return g;
}

int dw_grid_x(const DwGeom &g) { return g.B * g.tiles_h * g.tiles_w; }
int dw_threads(const DwGeom &g) { return (g.CC / CPT) * g.TWc; }
}  // namespace

int dw_fwd_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(0, B, H, W, C, stride)); }
int dw_dgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(1, B, H, W, C, stride)); }
int dw_wgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(2, B, H, W, C, stride)); }

void launch_dw_fwd(const bf16_t *x, const float *in_s, const float *in_t, int act, const bf16_t *w,
                   bf16_t *y, float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  const DwGeom g = dw_geom(0, B, H, W, C, stride);
  dim3 grid(dw_grid_x(g) * (C / g.CC)), block(dw_threads(g));
  if (stride == 1) {
    if (act == ACT_BN_RELU6) hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_BN_RELU6>), grid, block, 0, st, x, in_s, in_t, w, y, part, g);
    else hipLaunchKernelGGL((dw_fwd_kernel<1, ACT_NONE>), grid, block, 0, st, x, in_s, in_t, w, y, part, g);
  } else {
    if (act == ACT_BN_RELU6) hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_BN_RELU6>), grid, block, 0, st, x, in_s, in_t, w, y, part, g);
    else hipLaunchKernelGGL((dw_fwd_kernel<2, ACT_NONE>), grid, block, 0, st, x, in_s, in_t, w, y, part, g);
  }
}

int colsum_rows(int R);

void launch_dw_dgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *w,
                     const bf16_t *yprev, const float *ps, const float *pt, bf16_t *gout,
                     float *part, int B, int H, int W, int C, int stride, float *wpart, hipStream_t st) {
  const DwGeom g = dw_geom(1, B, H, W, C, stride);
  dim3 grid(dw_grid_x(g) * (C / g.CC)), block(dw_threads(g));
  if (wpart) {
    if (stride == 1)
      hipLaunchKernelGGL((dw_dgrad_kernel<1, true>), grid, block, 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g, wpart);
    else
      hipLaunchKernelGGL((dw_dgrad_kernel<2, true>), grid, block, 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g, wpart);
  } else {
    if (stride == 1)
      hipLaunchKernelGGL((dw_dgrad_kernel<1, false>), grid, block, 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g, wpart);
    else
      hipLaunchKernelGGL((dw_dgrad_kernel<2, false>), grid, block, 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g, wpart);
  }
}

// wpart of the fused dgrad + wgrad: [P][9][C] with P = dgrad tiles, + level-1 rows of the reduction
long long dw_dgrad_wgrad_workspace_floats(int B, int H, int W, int C, int stride) {
  const int P = dw_grid_x(dw_geom(1, B, H, W, C, stride));
  return (long long)(P + colsum_rows(P)) * 9 * C;
}

void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st);

void launch_dw_wgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *yprev,
                     const float *ps, const float *pt, float *part, float *grad, int B, int H, int W,
                     int C, int stride, hipStream_t st) {
  const DwGeom g = dw_geom(2, B, H, W, C, stride);
  const int P = dw_grid_x(g);
  dim3 grid(P * (C / g.CC)), block(dw_threads(g));
  if (stride == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<1>), grid, block, 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  else
    hipLaunchKernelGGL((dw_wgrad_kernel<2>), grid, block, 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  // deterministic two-level reduction of the [P][9C] partials -> grad [9][C] (tap-major)
  launch_wgrad_reduce(part, P, 9LL * C, grad, st);
}
