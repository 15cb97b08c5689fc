// Fused classifier head + loss: BN-apply/ReLU6 of the last 1x1 conv ->
// global average pool -> Dropout(p) -> Linear(C, NC) -> softmax cross-entropy
// (mean over the local batch) -> argmax/correct, AND its backward down to the
// BN-backward partials of features.18 — one workgroup per image.
//
// Reference ops: AdaptiveAvgPool2d(1) + flatten, Dropout(0.2),
// Linear(1280, 10), CrossEntropyLoss, torch.max + .item() metrics
// (cifar10_mpi_mobilenet_224.py:177-185).  Metrics stay on the device (per-image
// loss / correct vectors), so the step needs no host synchronisation.
#include "../common.h"

namespace {
constexpr int kMaxNC = 16;
constexpr int kPix = 8;   // pixel rows loaded per batch in the pooling / gradient loops
}

__global__ __launch_bounds__(256) void head_kernel(
    const bf16_t *__restrict__ y, const float *__restrict__ s, const float *__restrict__ t,
    const float *__restrict__ Wl, const float *__restrict__ bl, const long long *__restrict__ labels,
    int HW, int C, int NC, float drop_p, unsigned long long seed, const float *__restrict__ hyper,
    int train, float loss_scale, float *__restrict__ logits_out, float *__restrict__ loss_out,
    float *__restrict__ correct_out, float *__restrict__ dlogits, float *__restrict__ pd_out,
    bf16_t *__restrict__ g_out, float *__restrict__ part) {
  __shared__ float red[4][kMaxNC];
  __shared__ float dl[kMaxNC];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C8 = C / 8;
  const bool active = tid < C8;
  const int c0 = tid * 8;
  const float inv_hw = 1.f / (float)HW;
  const unsigned long long ctr = hyper ? (unsigned long long)hyper[1] : 0ull;
  float sc[8], sh[8], pd[8], keep[8];
  if (active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = s[c0 + k];
      sh[k] = t[c0 + k];
      pd[k] = 0.f;
    }
    const bf16_t *yb = y + (size_t)b * HW * C + c0;
    for (int h0 = 0; h0 < HW; h0 += kPix) {   // kPix pixel loads in flight (a serial load chain before)
     uint4 raw[kPix];
#pragma unroll
     for (int u = 0; u < kPix; ++u) raw[u] = ldg16(yb + (size_t)min(h0 + u, HW - 1) * C);   // clamped, unconditional
#pragma unroll
     for (int u = 0; u < kPix; ++u) {
      if (h0 + u >= HW) break;
      float v[8];
      unpack8(raw[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) pd[k] += relu6f(fmaf(v[k], sc[k], sh[k]));
     }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pd[k] *= inv_hw;
      keep[k] = 1.f;
      if (train && drop_p > 0.f) {
        const float u = pg_uniform(seed ^ (ctr * 0x9E3779B97F4A7C15ull), (unsigned long long)b * C + c0 + k);
        keep[k] = u >= drop_p ? 1.f / (1.f - drop_p) : 0.f;
      }
      pd[k] *= keep[k];
      if (pd_out) pd_out[(size_t)b * C + c0 + k] = pd[k];
    }
  }
  // logits
  for (int j = 0; j < NC; ++j) {
    float a = 0.f;
    if (active) {
#pragma unroll
      for (int k = 0; k < 8; ++k) a = fmaf(Wl[(size_t)j * C + c0 + k], pd[k], a);
    }
    a = wave_sum(a);
    if (lane == 0) red[wave][j] = a;
  }
  __syncthreads();
  if (tid == 0) {
    float lg[kMaxNC];
    float mx = -INFINITY;
    int arg = 0;
    for (int j = 0; j < NC; ++j) {
      lg[j] = red[0][j] + red[1][j] + red[2][j] + red[3][j] + bl[j];
      if (lg[j] > mx) { mx = lg[j]; arg = j; }
      if (logits_out) logits_out[(size_t)b * NC + j] = lg[j];
    }
    float se = 0.f;
    for (int j = 0; j < NC; ++j) se += __expf(lg[j] - mx);
    const float lse = mx + __logf(se);
    const int lab = labels ? (int)labels[b] : 0;
    if (loss_out) loss_out[b] = lse - lg[lab];
    if (correct_out) correct_out[b] = (arg == lab) ? 1.f : 0.f;
    for (int j = 0; j < NC; ++j) {
      const float pj = __expf(lg[j] - lse);
      const float d = (pj - (j == lab ? 1.f : 0.f)) * loss_scale;
      dl[j] = d;
      if (dlogits) dlogits[(size_t)b * NC + j] = d;
    }
  }
  if (!train) return;
  __syncthreads();
  if (!active) return;
  float dz[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float a = 0.f;
    for (int j = 0; j < NC; ++j) a = fmaf(dl[j], Wl[(size_t)j * C + c0 + k], a);
    dz[k] = a * keep[k] * inv_hw;
  }
  float st0[8], st1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) st0[k] = st1[k] = 0.f;
  for (int h0 = 0; h0 < HW; h0 += kPix) {
   uint4 raw[kPix];
#pragma unroll
   for (int u = 0; u < kPix; ++u) raw[u] = ldg16(y + ((size_t)b * HW + min(h0 + u, HW - 1)) * C + c0);
#pragma unroll
   for (int u = 0; u < kPix; ++u) {
    if (h0 + u >= HW) break;
    const size_t off = ((size_t)b * HW + h0 + u) * C + c0;
    float v[8], g[8];
    unpack8(raw[u], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g[k] = dz[k] * relu6_mask(v[k], sc[k], sh[k]);
    }
    // statistics over the bf16 value actually stored
    const uint4 gp = pack8(g);
    float gr[8];
    unpack8(gp, gr);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      st0[k] += gr[k];
      st1[k] = fmaf(gr[k], v[k], st1[k]);
    }
    stg16(g_out + off, gp);
   }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    part[((size_t)b * 2 + 0) * C + c0 + k] = st0[k];
    part[((size_t)b * 2 + 1) * C + c0 + k] = st1[k];
  }
}

// dW[j][c] = sum_b dlogits[b][j] * pd[b][c];  db[j] = sum_b dlogits[b][j]
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float *__restrict__ dlogits,
                                                        const float *__restrict__ pd, int B, int C,
                                                        int NC, float *__restrict__ dW,
                                                        float *__restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < NC * C) {
    const int j = i / C, c = i % C;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // 16 loads in flight per step
    int b = 0;
    for (; b + 8 <= B; b += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = fmaf(dlogits[(b + u) * NC + j], pd[(size_t)(b + u) * C + c], a[u]);
    }
    for (; b < B; ++b) a[0] = fmaf(dlogits[b * NC + j], pd[(size_t)b * C + c], a[0]);
    dW[i] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  } else if (i < NC * C + NC) {
    const int j = i - NC * C;
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += dlogits[b * NC + j];
    db[j] = a;
  }
}

void launch_head(const bf16_t *y, const float *s, const float *t, const float *Wl, const float *bl,
                 const long long *labels, int B, int HW, int C, int NC, float drop_p,
                 unsigned long long seed, const float *hyper, int train, float loss_scale,
                 float *logits, float *loss, float *correct, float *dlogits, float *pd,
                 bf16_t *g_out, float *part, float *dW, float *db, hipStream_t st) {
  hipLaunchKernelGGL(head_kernel, dim3(B), dim3(256), 0, st, y, s, t, Wl, bl, labels, HW, C, NC,
                     drop_p, seed, hyper, train, loss_scale, logits, loss, correct, dlogits, pd,
                     g_out, part);
  if (train)
    hipLaunchKernelGGL(head_wgrad_kernel, dim3((NC * C + NC + 255) / 256), dim3(256), 0, st, dlogits,
                       pd, B, C, NC, dW, db);
}
