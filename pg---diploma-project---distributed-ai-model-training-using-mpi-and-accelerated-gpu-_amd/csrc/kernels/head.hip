// Fused classifier head + loss: BN-apply/ReLU6 of the last 1x1 conv ->
// global average pool -> Dropout(p) -> Linear(C, NC) -> softmax cross-entropy
// (mean over the local batch) -> argmax/correct, AND its backward down to the
// BN-backward partials of features.18 (pool / CE / backward launches, below).
//
// Reference ops: AdaptiveAvgPool2d(1) + flatten, Dropout(0.2),
// Linear(1280, 10), CrossEntropyLoss, torch.max + .item() metrics
// (cifar10_mpi_mobilenet_224.py:177-185).  Metrics stay on the device (per-image
// loss / correct vectors), so the step needs no host synchronisation.
#include "../bnfin.h"

namespace {
constexpr int kMaxNC = 16;
constexpr int kSlots = 8;        // pixel slots per workgroup (32 channel lanes x 8 slots = 256 threads)
constexpr int kChunk = 32 * 8;   // channels per workgroup (8 per lane)

PG_DEVICE float drop_keep(int train, float drop_p, unsigned long long seed, unsigned long long ctr, size_t i) {
  if (!train || drop_p <= 0.f) return 1.f;
  const float u = pg_uniform(seed ^ (ctr * 0x9E3779B97F4A7C15ull), (unsigned long long)i);
  return u >= drop_p ? 1.f / (1.f - drop_p) : 0.f;
}
}  // namespace

// The head runs as three launches (two when training: the CE is recomputed in the backward) so the 16 MB feature map is streamed by B x C/256
// workgroups (640 at B=128) instead of one workgroup per image (128 workgroups, half the
// CUs idle, a 49-deep per-thread load chain):
//   pool:  z = relu6(BN(y)) averaged over HW, dropout -> pd[B][C]      grid (B, C/256)
//   ce:    logits = pd W^T + b, softmax-CE, argmax, dlogits            grid B
//   bwd:   g = (dlogits W) * keep / HW * relu6'(BN(y)), BN partials    grid (B, C/256)
// Within a workgroup lane l owns channels [8l, 8l+8) of the chunk and slot k the pixels
// k, k+8, ...; the slot sums are combined in LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void head_pool_kernel(
    const bf16_t *__restrict__ y, const float *__restrict__ s, const float *__restrict__ t, int HW, int C,
    float drop_p, unsigned long long seed, const float *__restrict__ hyper, int train, float *__restrict__ pd_out) {
  __shared__ float red[kSlots][kChunk + 4];
  const int b = blockIdx.x, tid = threadIdx.x, cl = tid & 31, slot = tid >> 5;
  const int cbase = blockIdx.y * kChunk;
  const int c0 = cbase + cl * 8;
  const bool active = c0 < C;
  float pd[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) pd[k] = 0.f;
  if (active) {
    float sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = s[c0 + k];
      sh[k] = t[c0 + k];
    }
    const bf16_t *yb = y + (size_t)b * HW * C + c0;
    for (int h0 = slot; h0 < HW; h0 += 4 * kSlots) {   // 4 independent 16-B loads in flight
      uint4 raw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) raw[u] = ldg16(yb + (size_t)min(h0 + u * kSlots, HW - 1) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (h0 + u * kSlots < HW) {
          float v[8];
          unpack8(raw[u], v);
#pragma unroll
          for (int k = 0; k < 8; ++k) pd[k] += relu6f(fmaf(v[k], sc[k], sh[k]));
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[slot][cl * 8 + k] = pd[k];
  __syncthreads();
  const int c = cbase + tid;   // one channel per thread for the slot combine
  if (c < C) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < kSlots; ++k) a += red[k][tid];
    const unsigned long long ctr = hyper ? (unsigned long long)hyper[1] : 0ull;
    pd_out[(size_t)b * C + c] = a * (1.f / (float)HW) * drop_keep(train, drop_p, seed, ctr, (size_t)b * C + c);
  }
}

// Linear + softmax-CE of image b by the whole workgroup (256 threads x 8 channels >= C).  write:
// store logits / loss / correct / dlogits; dl_sh (optional): dlogits[b][:] into LDS for the caller.
PG_DEVICE void ce_row(const float *__restrict__ pd, const float *__restrict__ Wl, const float *__restrict__ bl,
                      const long long *__restrict__ labels, int b, int C, int NC, float loss_scale,
                      float *__restrict__ logits_out, float *__restrict__ loss_out, float *__restrict__ correct_out,
                      float *__restrict__ dlogits, bool write, float (*red)[kMaxNC], float *dl_sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = tid * 8;
  const bool active = c0 < C;
  float p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = active ? pd[(size_t)b * C + c0 + k] : 0.f;
  for (int j = 0; j < NC; ++j) {
    float a = 0.f;
    if (active) {
#pragma unroll
      for (int k = 0; k < 8; ++k) a = fmaf(Wl[(size_t)j * C + c0 + k], p[k], a);
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
      if (write && logits_out) logits_out[(size_t)b * NC + j] = lg[j];
    }
    float se = 0.f;
    for (int j = 0; j < NC; ++j) se += __expf(lg[j] - mx);
    const float lse = mx + __logf(se);
    const int lab = labels ? (int)labels[b] : 0;
    if (write && loss_out) loss_out[b] = lse - lg[lab];
    if (write && correct_out) correct_out[b] = (arg == lab) ? 1.f : 0.f;
    for (int j = 0; j < NC; ++j) {
      const float d = (__expf(lg[j] - lse) - (j == lab ? 1.f : 0.f)) * loss_scale;
      if (dl_sh) dl_sh[j] = d;
      if (write && dlogits) dlogits[(size_t)b * NC + j] = d;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void head_ce_kernel(
    const float *__restrict__ pd, const float *__restrict__ Wl, const float *__restrict__ bl,
    const long long *__restrict__ labels, int C, int NC, float loss_scale, float *__restrict__ logits_out,
    float *__restrict__ loss_out, float *__restrict__ correct_out, float *__restrict__ dlogits) {
  __shared__ float red[4][kMaxNC];
  ce_row(pd, Wl, bl, labels, blockIdx.x, C, NC, loss_scale, logits_out, loss_out, correct_out, dlogits, true, red,
         nullptr);
}

// (training: the CE of image b is recomputed by each of its C/256 workgroups from pd -- 51 KB of
// L2-resident weights -- instead of a separate launch between pool and backward; the chunk-0
// workgroup stores logits / loss / correct / dlogits)
__global__ __launch_bounds__(256) void head_bwd_kernel(
    const bf16_t *__restrict__ y, const float *__restrict__ s, const float *__restrict__ t,
    const float *__restrict__ Wl, const float *__restrict__ pd, const float *__restrict__ bl,
    const long long *__restrict__ labels, float loss_scale, float *__restrict__ logits_out,
    float *__restrict__ loss_out, float *__restrict__ correct_out, float *__restrict__ dlogits, int HW, int C,
    int NC, float drop_p, unsigned long long seed, const float *__restrict__ hyper, bf16_t *__restrict__ g_out,
    float *__restrict__ part, int rep, const BnFin *fin) {
  __shared__ float r0[kSlots][kChunk + 4];
  __shared__ float r1[kSlots][kChunk + 4];
  __shared__ float cred[4][kMaxNC];
  __shared__ float dls[kMaxNC];
  ce_row(pd, Wl, bl, labels, blockIdx.x, C, NC, loss_scale, logits_out, loss_out, correct_out, dlogits,
         blockIdx.y == 0, cred, dls);
  const int b = blockIdx.x, tid = threadIdx.x, cl = tid & 31, slot = tid >> 5;
  const int cbase = blockIdx.y * kChunk;
  const int c0 = cbase + cl * 8;
  const bool active = c0 < C;
  float st0[8], st1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) st0[k] = st1[k] = 0.f;
  if (active) {
    const unsigned long long ctr = hyper ? (unsigned long long)hyper[1] : 0ull;
    const float inv_hw = 1.f / (float)HW;
    float sc[8], sh[8], dz[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = s[c0 + k];
      sh[k] = t[c0 + k];
      dz[k] = 0.f;
    }
    for (int j = 0; j < NC; ++j) {
      const float d = dls[j];
#pragma unroll
      for (int k = 0; k < 8; ++k) dz[k] = fmaf(d, Wl[(size_t)j * C + c0 + k], dz[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) dz[k] *= drop_keep(1, drop_p, seed, ctr, (size_t)b * C + c0 + k) * inv_hw;
    const size_t base = (size_t)b * HW * C + c0;
    for (int h0 = slot; h0 < HW; h0 += 4 * kSlots) {
      uint4 raw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) raw[u] = ldg16(y + base + (size_t)min(h0 + u * kSlots, HW - 1) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (h0 + u * kSlots < HW) {
          float v[8], g[8], gr[8];
          unpack8(raw[u], v);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = dz[k] * relu6_mask(v[k], sc[k], sh[k]);
          const uint4 gp = pack8(g);   // statistics over the bf16 value actually stored
          unpack8(gp, gr);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            st0[k] += gr[k];
            st1[k] = fmaf(gr[k], v[k], st1[k]);
          }
          stg16(g_out + base + (size_t)(h0 + u * kSlots) * C, gp);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r0[slot][cl * 8 + k] = st0[k];
    r1[slot][cl * 8 + k] = st1[k];
  }
  __syncthreads();
  const int c = cbase + tid;
  if (c < C) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
      a0 += r0[k][tid];
      a1 += r1[k][tid];
    }
    bn_part_add(part, b, gridDim.x, rep, C, 0, c, a0);
    bn_part_add(part, b, gridDim.x, rep, C, 1, c, a1);
  }
  bn_fin_tail(fin);
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
  const dim3 grid2(B, (C + kChunk - 1) / kChunk);
  const BnFin *fin = take_bn_fin();   // backward statistics of the final BN (train only)
  hipLaunchKernelGGL(head_pool_kernel, grid2, dim3(256), 0, st, y, s, t, HW, C, drop_p, seed, hyper, train, pd);
  if (!train) {
    hipLaunchKernelGGL(head_ce_kernel, dim3(B), dim3(256), 0, st, pd, Wl, bl, labels, C, NC, loss_scale, logits,
                       loss, correct, nullptr);
    return;
  }
  hipLaunchKernelGGL(head_bwd_kernel, grid2, dim3(256), 0, st, y, s, t, Wl, pd, bl, labels, loss_scale, logits,
                     loss, correct, dlogits, HW, C, NC, drop_p, seed, hyper, g_out, part, g_bn_rep, fin);
  hipLaunchKernelGGL(head_wgrad_kernel, dim3((NC * C + NC + 255) / 256), dim3(256), 0, st, dlogits, pd, B, C,
                     NC, dW, db);
}
