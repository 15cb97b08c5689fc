// Fused inverted-residual block forward for the 14x14 and 7x7 stages of MobileNetV2
// (features 8-13 and 15-17: stride 1, expand ratio 6).  Reference per-batch body:
// cifar10_mpi_mobilenet_224.py:176-180 (the torchvision block expand 1x1 -> BN -> ReLU6 ->
// dw 3x3 -> BN -> ReLU6 -> project 1x1 -> BN, SURVEY.md §2.6, §7.4 "fusing expand -> dw ->
// project ... is the stretch goal").
//
// Unfused, one block is three latency-bound launches of 10-20 us each over ~250 workgroups
// (expand GEMM, depthwise conv, project GEMM: profiles/r4_roofline_mnv2_tilerule.txt, ops
// 30-70), every one a chain of dependent global loads (A tiles, lazy-BN replica rows) at
// 0.7-2.9 TB/s.  Here ONE persistent launch per block does all three: a workgroup owns whole
// output rows of one image (a 7x7 image, or half of a 14x14 one plus a recomputed halo row),
// the hidden tensor never leaves its LDS, and the two training-mode BatchNorms inside the
// block (statistics over the whole batch) are two grid-wide barriers:
//
//   P0  input = BN_p(prev) (+ residual) of the previous block's raw output, staged in LDS and
//       materialised (the previous block's output o) for the owned rows
//   P1  expand GEMM (MFMA 16x16x32 bf16): h1 -> LDS + raw h1 to HBM (the backward reads it) +
//       BN_e statistics (float atomics into the replica rows of the BN's accumulator)
//   --- grid barrier 1 ---
//   P2  BN_e scale / shift from the accumulator (sc1 loads), depthwise 3x3 over relu6(BN_e(h1))
//       from LDS (sliding window per (row, 8-channel group)), raw h2 to HBM + BN_d statistics;
//       h2 overwrites h1 in LDS once every thread has read its taps
//   --- grid barrier 2 ---
//   P3  BN_d scale / shift, relu6(BN_d(h2)) in place, project GEMM -> raw y + BN_p statistics
//
// The block output BN_p(y) (+ x) is materialised by its consumer (the next fused block's P0,
// or the next GEMM's prologue), as on the unfused path; every tensor the backward reads
// (o_prev, h1, h2, y, the accumulators) is written exactly as the unfused kernels write it,
// so the backward is unchanged.  Numerics: the unfused contract (bf16 operands, fp32 MFMA
// accumulation, statistics of the bf16-rounded outputs, fp32 BN + ReLU6 of the depthwise taps).
//
// Grid barrier (MI355X_MICROARCH.md "Persistent kernels"): every wave drains its float atomics
// (vmcnt(0)), one lane per workgroup adds to an arrival counter (agent-scope atomic) and polls
// it with relaxed sc1 loads + s_sleep; the last workgroup to finish re-arms (zeroes) the
// counters, so every launch, replayed or re-run alone, starts from zero.  The statistics are memory-side float atomics
// read back with sc1 loads (the bnfin.h bn_fin_tail hand-off), so no release / acquire fence is
// needed.  Every spin is bounded: a barrier that does not complete within ~0.5 s sets bit 0 of
// the error word and the kernel runs to its end (wrong values, no hang).  All workgroups must be
// co-resident: the host launches only grids of at most (resident workgroups per CU x CUs)
// (ir_fwd_capacity), one workgroup per CU by its LDS footprint.
#include "../bnfin.h"

namespace {
constexpr int kIrThreads = 512;
constexpr unsigned kIrSpinMax = 1u << 20;
typedef __attribute__((address_space(1))) unsigned g_u32;

struct IrArgs {
  const bf16_t *xin;     // [M][CIN] previous block's raw project output (pre-BN)
  const bf16_t *res;     // [M][CIN] residual added to BN_p(xin) (nullptr: none)
  const BnFin *lz_in;    // BN of xin (lazy forward descriptor)
  bf16_t *xout;          // [M][CIN] this block's input (= previous block's output o), owned rows
  const bf16_t *we;      // [CH][CIN]
  const bf16_t *wd;      // [9][CH] (tap-major, engine/flat.py)
  const bf16_t *wp;      // [COUT][CH]
  bf16_t *h1, *h2, *y;   // raw pre-BN outputs [M][CH], [M][CH], [M][COUT]
  const BnFin *de, *dd, *dp;   // BN_e, BN_d, BN_p: accumulators, affine, eps, count
  unsigned *bar;         // barrier 1 / barrier 2 / exit counters, 32 words apart (zero at the first launch)
  unsigned *err;         // sticky error word (bit 0: a grid barrier timed out)
};

// phase trace (diagnostics, scripts/ir_phases.py): when set, thread 0 of every workgroup stamps
// the wall clock (100 MHz) at the phase boundaries into ts[workgroup][16]
__device__ unsigned long long *g_ir_ts = nullptr;
#define IR_MARK(k)                                                                                        \
  do {                                                                                                    \
    if (threadIdx.x == 0) {                                                                               \
      unsigned long long *t_ = g_ir_ts;                                                                   \
      if (t_) t_[(size_t)blockIdx.x * 16 + (k)] = wall_clock64();                                         \
    }                                                                                                     \
  } while (0)

PG_DEVICE void ir_grid_sync(unsigned *ctr, unsigned nwg, unsigned *err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores / float atomics landed
  __syncthreads();
  if (threadIdx.x == 0) {
    g_u32 *c = (g_u32 *)ctr;
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nwg) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > kIrSpinMax) {
        __hip_atomic_fetch_or((g_u32 *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// forward BN parameters of channel c from the replica rows, read with sc1 loads (the rows were
// accumulated by float atomics of other workgroups of THIS launch): bitwise bnfin.h bn_lazy
PG_DEVICE void ir_bn_sc1(const BnFin *d, int c, float &scale, float &shift) {
  const int C = d->C, rows = d->rows;
  float v[2 * kBnRep];
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const int rr = r < rows ? r : 0;
    v[2 * r] = ld_sc1_global(d->acc + (size_t)(2 * rr) * C + c);
    v[2 * r + 1] = ld_sc1_global(d->acc + (size_t)(2 * rr + 1) * C + c);
  }
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const double m = r < rows ? 1.0 : 0.0;
    s0 += m * (double)v[2 * r];
    s1 += m * (double)v[2 * r + 1];
  }
  const double n = (double)d->count;
  const double mean = s0 / n;
  double var = s1 / n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rs = (float)(1.0 / sqrt(var + (double)d->eps));
  const float g = d->gamma ? d->gamma[c] : 1.f, b = d->beta ? d->beta[c] : 0.f;
  scale = g * rs;
  shift = b - (float)mean * g * rs;
}

PG_DEVICE s16x8_t lds_frag(const bf16_t *p) { return *reinterpret_cast<const s16x8_t *>(p); }
PG_DEVICE s16x8_t glb_frag(const bf16_t *p) { return *reinterpret_cast<const s16x8_t *>(p); }
PG_DEVICE f32x4_t mfma16(s16x8_t a, s16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
}  // namespace

// H: map height = width (14 or 7); SPLIT: output-row groups per image (2 for 14x14: 7 rows each
// plus one recomputed halo row; 1 for 7x7: the whole image).
template <int CIN, int CH, int COUT, int H, int SPLIT>
struct IrGeom {
  static constexpr int W = H, ROWS = H / SPLIT, NSPLIT = SPLIT;
  static constexpr int NH = ROWS + (SPLIT > 1 ? 1 : 0);    // staged image rows (owned + halo)
  static constexpr int NPIX = NH * W;                       // staged pixels
  static constexpr int MP = (NPIX + 15) / 16 * 16;          // MFMA rows of the expand GEMM
  static constexpr int NOWN = ROWS * W;                     // owned (output) pixels
  static constexpr int RT3 = (NOWN + 15) / 16;              // MFMA row tiles of the project GEMM
  static constexpr int LDH = CH + 8, LDX = CIN + 8;         // LDS row pitches (bf16)
  static constexpr size_t SLOTS = (size_t)MP * LDH * 2;
  static constexpr size_t XR = (size_t)MP * LDX * 2 > (size_t)4 * CH * 4 ? (size_t)MP * LDX * 2 : (size_t)4 * CH * 4;
  static constexpr size_t LDS = SLOTS + XR + (size_t)2 * CIN * 4;
  static_assert(ROWS * SPLIT == H, "rows split evenly");
  static_assert(CIN % 32 == 0 && CH % 32 == 0 && COUT % 32 == 0, "multiples of 32 channels");
  static_assert(LDS <= 160 * 1024, "one workgroup per CU must fit the LDS");
};

template <int CIN, int CH, int COUT, int H, int SPLIT>
__global__ __launch_bounds__(kIrThreads) void ir_fwd_kernel(IrArgs p) {
  using G = IrGeom<CIN, CH, COUT, H, SPLIT>;
  constexpr int W = G::W, ROWS = G::ROWS, MP = G::MP, LDH = G::LDH, LDX = G::LDX;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t *slots = reinterpret_cast<bf16_t *>(smem);                        // [MP][LDH] h1 / h2
  char *xr = smem + G::SLOTS;
  bf16_t *xs = reinterpret_cast<bf16_t *>(xr);                             // P0/P1: [MP][LDX]
  float *ps = reinterpret_cast<float *>(xr);                               // P2/P3: scale [CH]
  float *pt = ps + CH;                                                     //        shift [CH]
  float *st = pt + CH;                                                     // P2: statistics [2][CH]
  float *pin = reinterpret_cast<float *>(xr + G::XR);                      // input BN [2][CIN]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int b = wg / SPLIT, part = wg % SPLIT;
  const int r0 = part * ROWS, r1 = r0 + ROWS;
  const int hr0 = r0 > 0 ? r0 - 1 : 0, hr1 = r1 < H ? r1 + 1 : H;
  const int npix = (hr1 - hr0) * W;
  const int own0 = (r0 - hr0) * W;                 // slot of the first owned pixel
  const size_t gbase = ((size_t)b * H + hr0) * W;  // global row of slot 0

  IR_MARK(0);
  // ---------------- P0: input BN parameters, staged input tile (+ materialised block input)
  for (int c = tid; c < CIN; c += kIrThreads) {
    float s, t, u;
    bn_lazy(p.lz_in, c, s, t, u);
    pin[c] = s;
    pin[CIN + c] = t;
  }
  __syncthreads();
  {
    constexpr int KC = CIN / 8, NQ = MP * KC, NIT = (NQ + kIrThreads - 1) / kIrThreads;
    const rsrc_t rX = make_rsrc(p.xin, 0x7fffffffu);
    const rsrc_t rR = make_rsrc(p.res ? p.res : p.xin, 0x7fffffffu);
    uint4 xv[NIT], rv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {   // every load in flight first
      const int q = tid + it * kIrThreads, i = q / KC, k = (q % KC) * 8;
      const uint32_t off = (q < NQ && i < npix) ? (uint32_t)(((gbase + i) * CIN + k) * 2) : kOOB;
      xv[it] = bld16(rX, off);
      rv[it] = bld16(rR, p.res ? off : kOOB);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = tid + it * kIrThreads, i = q / KC, k = (q % KC) * 8;
      if (q >= NQ) continue;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (i < npix) {
        float x[8], r[8];
        unpack8(xv[it], x);
        unpack8(rv[it], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], pin[k + j], pin[CIN + k + j]) + r[j];
        v = pack8(x);
        if (i >= own0 && i < own0 + G::NOWN) stg16(p.xout + (gbase + i) * CIN + k, v);
      }
      *reinterpret_cast<uint4 *>(xs + i * LDX + k) = v;
    }
  }
  __syncthreads();
  IR_MARK(1);

  // ---------------- P1: expand GEMM h1[MP][CH] = xs @ We^T, waves over column pairs
  {
    constexpr int KS = CIN / 32, RT = MP / 16, NCP = CH / 32;
    const BnFin *de = p.de;
    float *acc_e = de->acc;
    const int rep = de->rows, rrow = wg % rep;
    auto loadB = [&](int cp, s16x8_t (&bf)[KS][2]) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bf[s][c] = glb_frag(p.we + (size_t)(cp * 32 + c * 16 + (lane & 15)) * CIN + s * 32 + 8 * (lane >> 4));
    };
    auto body = [&](int cp, const s16x8_t (&bcur)[KS][2], s16x8_t (&bnext)[KS][2]) {
      if (cp + 8 < NCP) loadB(cp + 8, bnext);   // next column pair's weights in flight
      f32x4_t acc[RT][2];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt][0] = acc[rt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const s16x8_t af = lds_frag(xs + (rt * 16 + (lane & 15)) * LDX + s * 32 + 8 * (lane >> 4));
          acc[rt][0] = mfma16(af, bcur[s][0], acc[rt][0]);
          acc[rt][1] = mfma16(af, bcur[s][1], acc[rt][1]);
        }
      }
      // epilogue: bf16 h1 -> LDS, statistics of the owned rows' rounded values -> replica row
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = cp * 32 + c * 16 + (lane & 15);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = rt * 16 + 4 * (lane >> 4) + j;
            const bf16_t h = f2bf(acc[rt][c][j]);
            slots[row * LDH + col] = h;
            const float v = bf2f(h);
            const float m = (row >= own0 && row < own0 + G::NOWN) ? 1.f : 0.f;
            s0 = fmaf(m, v, s0);
            s1 = fmaf(m * v, v, s1);
          }
        s0 += __shfl_xor(s0, 16, 64);
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (lane < 16) {
          atomicAdd(acc_e + (size_t)(2 * rrow) * CH + col, s0);
          atomicAdd(acc_e + (size_t)(2 * rrow + 1) * CH + col, s1);
        }
      }
    };
    s16x8_t bfa[KS][2], bfb[KS][2];
    if (wave < NCP) loadB(wave, bfa);
    for (int cp = wave; cp < NCP; cp += 16) {   // ping-pong weight registers (static indexing)
      body(cp, bfa, bfb);
      if (cp + 8 < NCP) body(cp + 8, bfb, bfa);
    }
  }
  __syncthreads();
  IR_MARK(2);
  {   // raw h1 of the owned rows -> HBM (16-B rows pieces)
    constexpr int KC = CH / 8;
    for (int q = tid; q < G::NOWN * KC; q += kIrThreads) {
      const int i = own0 + q / KC, k = (q % KC) * 8;
      stg16(p.h1 + (gbase + i) * CH + k, *reinterpret_cast<const uint4 *>(slots + i * LDH + k));
    }
  }
  IR_MARK(3);
  ir_grid_sync(p.bar, (unsigned)nwg, p.err);
  IR_MARK(4);

  // ---------------- P2: BN_e + ReLU6 in place (bf16 activation, as materialised by the unfused
  // path's consumers), depthwise 3x3 (stride 1, pad 1) from LDS; raw h2 -> HBM only
  for (int c = tid; c < CH; c += kIrThreads) {
    float s, t;
    ir_bn_sc1(p.de, c, s, t);
    ps[c] = s;
    pt[c] = t;
    st[c] = 0.f;
    st[CH + c] = 0.f;
  }
  __syncthreads();
  IR_MARK(5);
  {
    constexpr int KC = CH / 8;
    for (int q = tid; q < npix * KC; q += kIrThreads) {
      const int i = q / KC, k = (q % KC) * 8;
      uint4 *pp = reinterpret_cast<uint4 *>(slots + i * LDH + k);
      float v[8];
      unpack8(*pp, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = relu6f(fmaf(v[j], ps[k + j], pt[k + j]));
      *pp = pack8(v);
    }
  }
  __syncthreads();
  IR_MARK(6);
  {
    constexpr int NG = CH / 8, NITEMS = NG * ROWS;
    for (int item = tid; item < NITEMS; item += kIrThreads) {
      const int g = item % NG, rl = item / NG, c0 = g * 8, r = r0 + rl;
      // rows r-1, r, r+1 (outside the image: weights zeroed, address of row r); columns x-1..x+1
      float wt[9][8];
      int srow[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int rr = r + d - 1;
        const bool ok = rr >= 0 && rr < H;
        srow[d] = (ok ? rr - hr0 : r - hr0) * W;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          unpack8(ldg16(p.wd + (size_t)(d * 3 + e) * CH + c0), wt[d * 3 + e]);
#pragma unroll
          for (int j = 0; j < 8; ++j) wt[d * 3 + e][j] = ok ? wt[d * 3 + e][j] : 0.f;
        }
      }
      float win[3][3][8];
      auto fetch = [&](int d, int x, float (&o)[8]) {
        unpack8(*reinterpret_cast<const uint4 *>(slots + (srow[d] + x) * LDH + c0), o);
      };
#pragma unroll
      for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) win[d][0][j] = 0.f;
        fetch(d, 0, win[d][1]);
      }
      float s0[8], s1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
#pragma unroll
      for (int x = 0; x < W; ++x) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          if (x + 1 < W) fetch(d, x + 1, win[d][2]);
          else
#pragma unroll
            for (int j = 0; j < 8; ++j) win[d][2][j] = 0.f;
        }
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float a = 0.f;
#pragma unroll
          for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) a = fmaf(win[d][e][j], wt[d * 3 + e][j], a);
          o[j] = a;
        }
        const uint4 pk = pack8(o);
        float ov[8];
        unpack8(pk, ov);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0[j] += ov[j];
          s1[j] = fmaf(ov[j], ov[j], s1[j]);
        }
        stg16(p.h2 + (((size_t)b * H + r) * W + x) * CH + c0, pk);
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            win[d][0][j] = win[d][1][j];
            win[d][1][j] = win[d][2][j];
          }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(st + c0 + j, s0[j]);
        atomicAdd(st + CH + c0 + j, s1[j]);
      }
    }
  }
  __syncthreads();
  IR_MARK(7);
  {
    const BnFin *dd = p.dd;
    const int rep = dd->rows, rrow = wg % rep;
    for (int c = tid; c < CH; c += kIrThreads) {
      atomicAdd(dd->acc + (size_t)(2 * rrow) * CH + c, st[c]);
      atomicAdd(dd->acc + (size_t)(2 * rrow + 1) * CH + c, st[CH + c]);
    }
  }
  IR_MARK(8);
  ir_grid_sync(p.bar + 32, (unsigned)nwg, p.err);
  IR_MARK(9);

  // ---------------- P3: h2 of the owned rows back from L2 (this workgroup's own stores) with
  // BN_d + ReLU6 applied -> LDS; project GEMM y[NOWN][COUT] = h2' @ Wp^T
  for (int c = tid; c < CH; c += kIrThreads) {
    float s, t;
    ir_bn_sc1(p.dd, c, s, t);
    ps[c] = s;
    pt[c] = t;
  }
  __syncthreads();
  IR_MARK(10);
  {
    constexpr int KC = CH / 8, NQ = G::NOWN * KC, NB = 8;
    const rsrc_t rH = make_rsrc(p.h2, 0x7fffffffu);
    const size_t obase = ((size_t)b * H + r0) * W;
    for (int q0 = 0; q0 < NQ; q0 += NB * kIrThreads) {
      uint4 v8[NB];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        v8[e] = bld16(rH, q < NQ ? (uint32_t)(((obase + i) * CH + k) * 2) : kOOB);
      }
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        if (q >= NQ) continue;
        float v[8];
        unpack8(v8[e], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = relu6f(fmaf(v[j], ps[k + j], pt[k + j]));
        *reinterpret_cast<uint4 *>(slots + (own0 + i) * LDH + k) = pack8(v);
      }
    }
  }
  __syncthreads();
  IR_MARK(11);
  {
    constexpr int KS = CH / 32, KCH = 6, NCH = KS / KCH, RT3 = G::RT3, NCP = COUT / 32;
    static_assert(KS % KCH == 0, "k chunks");
    // row groups: enough (column pair, row group) blocks for the 8 waves
    constexpr int RG = NCP >= 8 ? 1 : (NCP * 2 >= 8 ? 2 : 4);
    constexpr int RPG = (RT3 + RG - 1) / RG;
    const BnFin *dp = p.dp;
    float *acc_p = dp->acc;
    const int rep = dp->rows, rrow = wg % rep;
    for (int blk = wave; blk < NCP * RG; blk += 8) {
      const int cp = blk % NCP, rg = blk / NCP;
      const int rt0 = rg * RPG;
      f32x4_t acc[RPG][2];
#pragma unroll
      for (int r = 0; r < RPG; ++r) acc[r][0] = acc[r][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      s16x8_t bfr[2][KCH][2];
      auto loadB = [&](int kc, s16x8_t (&bf)[KCH][2]) {
#pragma unroll
        for (int s = 0; s < KCH; ++s)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            bf[s][c] = glb_frag(p.wp + (size_t)(cp * 32 + c * 16 + (lane & 15)) * CH + (kc * KCH + s) * 32 +
                                8 * (lane >> 4));
      };
      loadB(0, bfr[0]);
#pragma unroll
      for (int kc = 0; kc < NCH; ++kc) {
        if (kc + 1 < NCH) loadB(kc + 1, bfr[(kc + 1) & 1]);
#pragma unroll
        for (int s = 0; s < KCH; ++s) {
          const int k0 = (kc * KCH + s) * 32 + 8 * (lane >> 4);
#pragma unroll
          for (int r = 0; r < RPG; ++r) {
            const int t = (rt0 + r) * 16 + (lane & 15);
            const int i = own0 + (t < G::NOWN ? t : 0);   // rows past the owned ones: discarded
            const s16x8_t af = lds_frag(slots + i * LDH + k0);
            acc[r][0] = mfma16(af, bfr[kc & 1][s][0], acc[r][0]);
            acc[r][1] = mfma16(af, bfr[kc & 1][s][1], acc[r][1]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = cp * 32 + c * 16 + (lane & 15);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int t = (rt0 + r) * 16 + 4 * (lane >> 4) + j;
            if (rt0 + r < RT3 && t < G::NOWN) {
              const bf16_t h = f2bf(acc[r][c][j]);
              p.y[(((size_t)b * H + r0) * W + t) * COUT + col] = h;
              const float v = bf2f(h);
              s0 += v;
              s1 = fmaf(v, v, s1);
            }
          }
        s0 += __shfl_xor(s0, 16, 64);
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (lane < 16) {
          atomicAdd(acc_p + (size_t)(2 * rrow) * COUT + col, s0);
          atomicAdd(acc_p + (size_t)(2 * rrow + 1) * COUT + col, s1);
        }
      }
    }
  }
  // re-arm: every workgroup has passed both barriers once it arrives here; the last arrival
  // zeroes the three counters, so a launch needs no memset of them (replays, isolated re-runs)
  __syncthreads();
  IR_MARK(12);
  if (tid == 0) {
    g_u32 *c = (g_u32 *)(p.bar + 64);
    if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nwg - 1) {
      __hip_atomic_store((g_u32 *)p.bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((g_u32 *)(p.bar + 32), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ===========================================================================
// Fused block BACKWARD (same blocks, same geometry): the three main-stream launches of one
// block's backward -- project dgrad (BN_p backward prologue, ReLU6 mask of a2 epilogue), the
// depthwise dgrad (BN_d backward, ReLU6 mask of a1) and the expand dgrad (BN_e backward,
// skip gradient, previous block's BN_p statistics) -- as one launch with grid barriers at the
// two BatchNorm-backward statistics points:
//
//   B0  BN_p backward coefficients (lazy, from the consumer's accumulator rows), dy = a G + b y + c
//       of the owned + halo pixels staged in LDS, raw h2 of those pixels staged in LDS
//   B1  g_d = (dy @ Wp) * relu6'(BN_d(h2)) (MFMA) -> bn_d.g (halo rows too: the neighbour
//       stores identical values) + BN_d backward sums
//   --- grid barrier 1 ---
//   B2  dh2 = a_d g_d + b_d h2 + c_d in LDS (g_d read back from this workgroup's own stores),
//       g_e = dwT(dh2) * relu6'(BN_e(h1)) -> bn_e.g + BN_e backward sums
//   --- grid barrier 2 ---
//   B3  dh1 = a_e g_e + b_e h1 + c_e in LDS, dx = dh1 @ We (+ skip gradient) -> prev.G +
//       the previous block's BN_p backward sums
//
// The weight gradients stay on the side stream (pw_wgrad / dw_wgrad read bn_d.g, bn_e.g, G),
// unchanged.  Numerics: the unfused contract, with dh2 / dh1 rounded to bf16 in LDS.
// ===========================================================================
namespace {
struct IrBwdArgs {
  const bf16_t *G;        // [M][COUT] gradient w.r.t. the block output o
  const bf16_t *y;        // [M][COUT] raw project output (BN_p input)
  const BnFin *lz_p;      // BN_p backward descriptor (accumulated by the previous kernel)
  const bf16_t *wpt;      // [CH][COUT] transposed project weight
  const bf16_t *h2;       // [M][CH] raw depthwise output (BN_d input)
  const float *sd, *td;   // BN_d forward scale / shift
  bf16_t *gd;             // [M][CH] out: dL/d(BN_d output) after the ReLU6 mask (bn_d.g)
  const BnFin *dd;        // BN_d backward descriptor: accumulated HERE
  const bf16_t *wd;       // [9][CH] tap-major depthwise weight
  const bf16_t *h1;       // [M][CH] raw expand output (BN_e input)
  const float *se, *te;   // BN_e forward scale / shift
  bf16_t *ge;             // [M][CH] out: bn_e.g
  const BnFin *de;        // BN_e backward descriptor: accumulated HERE
  const bf16_t *wet;      // [CIN][CH] transposed expand weight
  const bf16_t *R;        // [M][CIN] skip gradient (the block's G when residual) or nullptr
  const bf16_t *yprev;    // [M][CIN] previous block's raw project output
  bf16_t *gout;           // [M][CIN] out: dL/d(block input) (prev.G)
  const BnFin *dprev;     // previous block's BN_p backward descriptor: accumulated HERE
  unsigned *bar, *err;
};

// backward coefficients (dy = a g + b y + c) of channel c from replica rows accumulated by float
// atomics of THIS launch (sc1 loads): bitwise bnfin.h bn_lazy's backward branch
PG_DEVICE void ir_bn_bwd_sc1(const BnFin *d, int c, float &o0, float &o1, float &o2) {
  const int C = d->C, rows = d->rows;
  float v[2 * kBnRep];
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const int rr = r < rows ? r : 0;
    v[2 * r] = ld_sc1_global(d->acc + (size_t)(2 * rr) * C + c);
    v[2 * r + 1] = ld_sc1_global(d->acc + (size_t)(2 * rr + 1) * C + c);
  }
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int r = 0; r < kBnRep; ++r) {
    const double m = r < rows ? 1.0 : 0.0;
    s0 += m * (double)v[2 * r];
    s1 += m * (double)v[2 * r + 1];
  }
  const float g = d->gamma ? d->gamma[c] : 1.f;
  const float mu = d->mean[c], rs = d->rstd[c];
  const double n = (double)d->count;
  const double sgx = (s1 - (double)mu * s0) * rs;
  const double a = (double)g * rs;
  o0 = (float)a;
  o1 = (float)(-a * rs * sgx / n);
  o2 = (float)(-a * s0 / n + a * rs * (double)mu * sgx / n);
}

PG_DEVICE float bf16r(float v) { return bf2f(f2bf(v)); }
}  // namespace

template <int CIN, int CH, int COUT, int H, int SPLIT>
struct IrBwdGeom {
  using F = IrGeom<CIN, CH, COUT, H, SPLIT>;
  static constexpr int LDY = COUT + 8;
  static constexpr size_t YS = (size_t)F::MP * LDY * 2;
  static constexpr size_t TAB = (size_t)7 * CH * 4;           // B2: a, b, c, s_e, t_e, sums [2]
  static constexpr size_t XR = YS > TAB ? YS : TAB;
  static constexpr size_t LDS = F::SLOTS + XR + (size_t)3 * COUT * 4;
  static_assert(LDS <= 160 * 1024, "one workgroup per CU must fit the LDS");
};

template <int CIN, int CH, int COUT, int H, int SPLIT>
__global__ __launch_bounds__(kIrThreads) void ir_bwd_kernel(IrBwdArgs p) {
  using G = IrGeom<CIN, CH, COUT, H, SPLIT>;
  using GB = IrBwdGeom<CIN, CH, COUT, H, SPLIT>;
  constexpr int W = G::W, ROWS = G::ROWS, MP = G::MP, LDH = G::LDH, LDY = GB::LDY;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t *slots = reinterpret_cast<bf16_t *>(smem);                   // [MP][LDH] h2 -> dh2 -> dh1
  char *xr = smem + G::SLOTS;
  bf16_t *ys = reinterpret_cast<bf16_t *>(xr);                        // B0/B1: dy [MP][LDY]
  float *ca = reinterpret_cast<float *>(xr);                          // B2/B3: coefficients [CH] x 3
  float *cb = ca + CH, *cc = cb + CH;
  float *sse = cc + CH, *ste = sse + CH;                              // B2: BN_e forward scale / shift
  float *st = ste + CH;                                               // B2: sums [2][CH]
  float *pc = reinterpret_cast<float *>(xr + GB::XR);                 // BN_p coefficients [3][COUT]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int b = wg / SPLIT, part = wg % SPLIT;
  const int r0 = part * ROWS, r1 = r0 + ROWS;
  const int hr0 = r0 > 0 ? r0 - 1 : 0, hr1 = r1 < H ? r1 + 1 : H;
  const int npix = (hr1 - hr0) * W;
  const int own0 = (r0 - hr0) * W;
  const size_t gbase = ((size_t)b * H + hr0) * W;

  IR_MARK(0);
  // ---------------- B0: BN_p coefficients, h2 and dy of the staged pixels
  for (int c = tid; c < COUT; c += kIrThreads) {
    float a, bb, c2;
    bn_lazy(p.lz_p, c, a, bb, c2);
    pc[c] = a;
    pc[COUT + c] = bb;
    pc[2 * COUT + c] = c2;
  }
  {
    constexpr int KC = CH / 8, NB = 8;
    const rsrc_t rH = make_rsrc(p.h2, 0x7fffffffu);
    for (int q0 = 0; q0 < MP * KC; q0 += NB * kIrThreads) {
      uint4 v8[NB];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        v8[e] = bld16(rH, (q < MP * KC && i < npix) ? (uint32_t)(((gbase + i) * CH + k) * 2) : kOOB);
      }
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        if (q < MP * KC) *reinterpret_cast<uint4 *>(slots + i * LDH + k) = v8[e];
      }
    }
  }
  __syncthreads();   // pc staged
  IR_MARK(1);
  {
    constexpr int KC = COUT / 8, NQ = MP * KC, NIT = (NQ + kIrThreads - 1) / kIrThreads;
    const rsrc_t rG = make_rsrc(p.G, 0x7fffffffu), rY = make_rsrc(p.y, 0x7fffffffu);
    uint4 gv[NIT], yv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = tid + it * kIrThreads, i = q / KC, k = (q % KC) * 8;
      const uint32_t off = (q < NQ && i < npix) ? (uint32_t)(((gbase + i) * COUT + k) * 2) : kOOB;
      gv[it] = bld16(rG, off);
      yv[it] = bld16(rY, off);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = tid + it * kIrThreads, i = q / KC, k = (q % KC) * 8;
      if (q >= NQ) continue;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (i < npix) {
        float g8[8], y8[8];
        unpack8(gv[it], g8);
        unpack8(yv[it], y8);
#pragma unroll
        for (int j = 0; j < 8; ++j) g8[j] = fmaf(pc[k + j], g8[j], fmaf(pc[COUT + k + j], y8[j], pc[2 * COUT + k + j]));
        v = pack8(g8);
      }
      *reinterpret_cast<uint4 *>(ys + i * LDY + k) = v;
    }
  }
  __syncthreads();
  IR_MARK(2);

  // ---------------- B1: g_d = (dy @ Wp) * relu6'(BN_d(h2)) over the staged pixels
  {
    constexpr int KS = COUT / 32, RT = MP / 16, NCP = CH / 32;
    const BnFin *dd = p.dd;
    const int rep = dd->rows, rrow = wg % rep;
    auto loadB = [&](int cp, s16x8_t (&bf)[KS][2]) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bf[s][c] = glb_frag(p.wpt + (size_t)(cp * 32 + c * 16 + (lane & 15)) * COUT + s * 32 + 8 * (lane >> 4));
    };
    auto body = [&](int cp, const s16x8_t (&bcur)[KS][2], s16x8_t (&bnext)[KS][2]) {
      if (cp + 8 < NCP) loadB(cp + 8, bnext);
      f32x4_t acc[RT][2];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt][0] = acc[rt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const s16x8_t af = lds_frag(ys + (rt * 16 + (lane & 15)) * LDY + s * 32 + 8 * (lane >> 4));
          acc[rt][0] = mfma16(af, bcur[s][0], acc[rt][0]);
          acc[rt][1] = mfma16(af, bcur[s][1], acc[rt][1]);
        }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = cp * 32 + c * 16 + (lane & 15);
        const float s_ = p.sd[col], t_ = p.td[col];
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = rt * 16 + 4 * (lane >> 4) + j;
            if (row < npix) {
              const float h = bf2f(slots[row * LDH + col]);
              const float v = bf16r(acc[rt][c][j]) * relu6_mask(h, s_, t_);
              p.gd[(gbase + row) * CH + col] = f2bf(v);
              const float m = (row >= own0 && row < own0 + G::NOWN) ? 1.f : 0.f;
              s0 = fmaf(m, v, s0);
              s1 = fmaf(m * v, h, s1);
            }
          }
        s0 += __shfl_xor(s0, 16, 64);
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (lane < 16) {
          atomicAdd(dd->acc + (size_t)(2 * rrow) * CH + col, s0);
          atomicAdd(dd->acc + (size_t)(2 * rrow + 1) * CH + col, s1);
        }
      }
    };
    s16x8_t bfa[KS][2], bfb[KS][2];
    if (wave < NCP) loadB(wave, bfa);
    for (int cp = wave; cp < NCP; cp += 16) {
      body(cp, bfa, bfb);
      if (cp + 8 < NCP) body(cp + 8, bfb, bfa);
    }
  }
  IR_MARK(3);
  ir_grid_sync(p.bar, (unsigned)nwg, p.err);
  IR_MARK(4);

  // ---------------- B2: dh2 in LDS, depthwise dgrad -> g_e
  for (int c = tid; c < CH; c += kIrThreads) {
    float a, bb, c2;
    ir_bn_bwd_sc1(p.dd, c, a, bb, c2);
    ca[c] = a;
    cb[c] = bb;
    cc[c] = c2;
    sse[c] = p.se[c];
    ste[c] = p.te[c];
    st[c] = 0.f;
    st[CH + c] = 0.f;
  }
  __syncthreads();
  IR_MARK(5);
  {   // dh2 = a g_d + b h2 + c over the staged pixels (g_d: this workgroup's own stores)
    constexpr int KC = CH / 8, NB = 8;
    const rsrc_t rD = make_rsrc(p.gd, 0x7fffffffu);
    for (int q0 = 0; q0 < npix * KC; q0 += NB * kIrThreads) {
      uint4 v8[NB];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        v8[e] = bld16(rD, q < npix * KC ? (uint32_t)(((gbase + i) * CH + k) * 2) : kOOB);
      }
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        if (q >= npix * KC) continue;
        uint4 *pp = reinterpret_cast<uint4 *>(slots + i * LDH + k);
        float g8[8], h8[8];
        unpack8(v8[e], g8);
        unpack8(*pp, h8);
#pragma unroll
        for (int j = 0; j < 8; ++j) g8[j] = fmaf(ca[k + j], g8[j], fmaf(cb[k + j], h8[j], cc[k + j]));
        *pp = pack8(g8);
      }
    }
  }
  __syncthreads();
  IR_MARK(6);
  {
    constexpr int NG = CH / 8, NITEMS = NG * ROWS;
    const rsrc_t rH1 = make_rsrc(p.h1, 0x7fffffffu);
    for (int item = tid; item < NITEMS; item += kIrThreads) {
      const int g = item % NG, rl = item / NG, c0 = g * 8, r = r0 + rl;
      // dx[r][x] = sum over window (d, e) of dh2[r - 1 + d][x - 1 + e] * w[2 - d][2 - e]
      float wt[9][8], s[8], t[8];
      int srow[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int rr = r + d - 1;
        const bool ok = rr >= 0 && rr < H;
        srow[d] = (ok ? rr - hr0 : r - hr0) * W;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          unpack8(ldg16(p.wd + (size_t)((2 - d) * 3 + (2 - e)) * CH + c0), wt[d * 3 + e]);
#pragma unroll
          for (int j = 0; j < 8; ++j) wt[d * 3 + e][j] = ok ? wt[d * 3 + e][j] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] = sse[c0 + j];
        t[j] = ste[c0 + j];
      }
      float win[3][3][8];
      auto fetch = [&](int d, int x, float (&o)[8]) {
        unpack8(*reinterpret_cast<const uint4 *>(slots + (srow[d] + x) * LDH + c0), o);
      };
#pragma unroll
      for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) win[d][0][j] = 0.f;
        fetch(d, 0, win[d][1]);
      }
      float s0[8], s1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
      const size_t orow = ((size_t)b * H + r) * W;
      uint4 hv = bld16(rH1, (uint32_t)((orow * CH + c0) * 2));
#pragma unroll
      for (int x = 0; x < W; ++x) {
        const uint4 hcur = hv;
        if (x + 1 < W) hv = bld16(rH1, (uint32_t)(((orow + x + 1) * CH + c0) * 2));   // next pixel's h1
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          if (x + 1 < W) fetch(d, x + 1, win[d][2]);
          else
#pragma unroll
            for (int j = 0; j < 8; ++j) win[d][2][j] = 0.f;
        }
        float h8[8], o[8];
        unpack8(hcur, h8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float a = 0.f;
#pragma unroll
          for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 3; ++e) a = fmaf(win[d][e][j], wt[d * 3 + e][j], a);
          o[j] = a * relu6_mask(h8[j], s[j], t[j]);
        }
        const uint4 pk = pack8(o);
        float ov[8];
        unpack8(pk, ov);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0[j] += ov[j];
          s1[j] = fmaf(ov[j], h8[j], s1[j]);
        }
        stg16(p.ge + (orow + x) * CH + c0, pk);
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            win[d][0][j] = win[d][1][j];
            win[d][1][j] = win[d][2][j];
          }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(st + c0 + j, s0[j]);
        atomicAdd(st + CH + c0 + j, s1[j]);
      }
    }
  }
  __syncthreads();
  IR_MARK(7);
  {
    const BnFin *de = p.de;
    const int rep = de->rows, rrow = wg % rep;
    for (int c = tid; c < CH; c += kIrThreads) {
      atomicAdd(de->acc + (size_t)(2 * rrow) * CH + c, st[c]);
      atomicAdd(de->acc + (size_t)(2 * rrow + 1) * CH + c, st[CH + c]);
    }
  }
  IR_MARK(8);
  ir_grid_sync(p.bar + 32, (unsigned)nwg, p.err);
  IR_MARK(9);

  // ---------------- B3: dh1 of the owned pixels in LDS, dx = dh1 @ We (+ skip) -> prev.G
  for (int c = tid; c < CH; c += kIrThreads) {
    float a, bb, c2;
    ir_bn_bwd_sc1(p.de, c, a, bb, c2);
    ca[c] = a;
    cb[c] = bb;
    cc[c] = c2;
  }
  __syncthreads();
  IR_MARK(10);
  {
    constexpr int KC = CH / 8, NQ = G::NOWN * KC, NB = 8;
    const rsrc_t rE = make_rsrc(p.ge, 0x7fffffffu), rH1 = make_rsrc(p.h1, 0x7fffffffu);
    const size_t obase = ((size_t)b * H + r0) * W;
    for (int q0 = 0; q0 < NQ; q0 += NB * kIrThreads) {
      uint4 g8v[NB], h8v[NB];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        const uint32_t off = q < NQ ? (uint32_t)(((obase + i) * CH + k) * 2) : kOOB;
        g8v[e] = bld16(rE, off);
        h8v[e] = bld16(rH1, off);
      }
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        const int q = q0 + e * kIrThreads + tid, i = q / KC, k = (q % KC) * 8;
        if (q >= NQ) continue;
        float g8[8], h8[8];
        unpack8(g8v[e], g8);
        unpack8(h8v[e], h8);
#pragma unroll
        for (int j = 0; j < 8; ++j) g8[j] = fmaf(ca[k + j], g8[j], fmaf(cb[k + j], h8[j], cc[k + j]));
        *reinterpret_cast<uint4 *>(slots + (own0 + i) * LDH + k) = pack8(g8);
      }
    }
  }
  __syncthreads();
  IR_MARK(11);
  {
    constexpr int KS = CH / 32, KCH = 6, NCH = KS / KCH, RT3 = G::RT3, NCP = CIN / 32;
    static_assert(KS % KCH == 0, "k chunks");
    constexpr int RG = NCP >= 8 ? 1 : (NCP * 2 >= 8 ? 2 : 4);
    constexpr int RPG = (RT3 + RG - 1) / RG;
    const BnFin *dq = p.dprev;
    const int rep = dq->rows, rrow = wg % rep;
    const size_t obase = ((size_t)b * H + r0) * W;
    for (int blk = wave; blk < NCP * RG; blk += 8) {
      const int cp = blk % NCP, rg = blk / NCP;
      const int rt0 = rg * RPG;
      f32x4_t acc[RPG][2];
#pragma unroll
      for (int r = 0; r < RPG; ++r) acc[r][0] = acc[r][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      s16x8_t bfr[2][KCH][2];
      auto loadB = [&](int kc, s16x8_t (&bf)[KCH][2]) {
#pragma unroll
        for (int s = 0; s < KCH; ++s)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            bf[s][c] = glb_frag(p.wet + (size_t)(cp * 32 + c * 16 + (lane & 15)) * CH + (kc * KCH + s) * 32 +
                                8 * (lane >> 4));
      };
      loadB(0, bfr[0]);
#pragma unroll
      for (int kc = 0; kc < NCH; ++kc) {
        if (kc + 1 < NCH) loadB(kc + 1, bfr[(kc + 1) & 1]);
#pragma unroll
        for (int s = 0; s < KCH; ++s) {
          const int k0 = (kc * KCH + s) * 32 + 8 * (lane >> 4);
#pragma unroll
          for (int r = 0; r < RPG; ++r) {
            const int t = (rt0 + r) * 16 + (lane & 15);
            const int i = own0 + (t < G::NOWN ? t : 0);
            const s16x8_t af = lds_frag(slots + i * LDH + k0);
            acc[r][0] = mfma16(af, bfr[kc & 1][s][0], acc[r][0]);
            acc[r][1] = mfma16(af, bfr[kc & 1][s][1], acc[r][1]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = cp * 32 + c * 16 + (lane & 15);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int t = (rt0 + r) * 16 + 4 * (lane >> 4) + j;
            if (rt0 + r < RT3 && t < G::NOWN) {
              const size_t o = (obase + t) * CIN + col;
              float v = bf16r(acc[r][c][j]);
              if (p.R) v += bf2f(p.R[o]);
              p.gout[o] = f2bf(v);
              s0 += v;
              s1 = fmaf(v, bf2f(p.yprev[o]), s1);
            }
          }
        s0 += __shfl_xor(s0, 16, 64);
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (lane < 16) {
          atomicAdd(dq->acc + (size_t)(2 * rrow) * CIN + col, s0);
          atomicAdd(dq->acc + (size_t)(2 * rrow + 1) * CIN + col, s1);
        }
      }
    }
  }
  __syncthreads();
  IR_MARK(12);
  if (tid == 0) {
    g_u32 *c = (g_u32 *)(p.bar + 64);
    if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nwg - 1) {
      __hip_atomic_store((g_u32 *)p.bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((g_u32 *)(p.bar + 32), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ===========================================================================
// host side
// ===========================================================================
namespace {
template <int CIN, int CH, int COUT, int H, int SPLIT>
struct IrKernel {
  using G = IrGeom<CIN, CH, COUT, H, SPLIT>;
  static const void *fn() { return reinterpret_cast<const void *>(&ir_fwd_kernel<CIN, CH, COUT, H, SPLIT>); }
  static size_t lds() { return G::LDS; }
  static void launch(const IrArgs &a, int B, hipStream_t st) {
    hipLaunchKernelGGL((ir_fwd_kernel<CIN, CH, COUT, H, SPLIT>), dim3(B * SPLIT), dim3(kIrThreads), G::LDS, st, a);
  }
};
template <int CIN, int CH, int COUT, int H, int SPLIT>
struct IrBwdKernel {
  using G = IrGeom<CIN, CH, COUT, H, SPLIT>;
  static const void *fn() { return reinterpret_cast<const void *>(&ir_bwd_kernel<CIN, CH, COUT, H, SPLIT>); }
  static size_t lds() { return IrBwdGeom<CIN, CH, COUT, H, SPLIT>::LDS; }
  static void launch(const IrBwdArgs &a, int B, hipStream_t st) {
    hipLaunchKernelGGL((ir_bwd_kernel<CIN, CH, COUT, H, SPLIT>), dim3(B * SPLIT), dim3(kIrThreads), lds(), st, a);
  }
};

// the backward shapes: as the forward, except 160 -> 960 -> 320 (features.17), whose dy tile
// does not fit the LDS next to the hidden tensor
template <class F>
bool ir_bwd_dispatch(int cin, int ch, int cout, int H, F &&f) {
  if (H == 14 && cin == 64 && ch == 384 && cout == 64) return f(IrBwdKernel<64, 384, 64, 14, 2>{}), true;
  if (H == 14 && cin == 64 && ch == 384 && cout == 96) return f(IrBwdKernel<64, 384, 96, 14, 2>{}), true;
  if (H == 14 && cin == 96 && ch == 576 && cout == 96) return f(IrBwdKernel<96, 576, 96, 14, 2>{}), true;
  if (H == 7 && cin == 160 && ch == 960 && cout == 160) return f(IrBwdKernel<160, 960, 160, 7, 1>{}), true;
  return false;
}

template <class K>
int co_resident_grid(int B) {
  const int nwg = B * K::G::NSPLIT;
  int dev = 0, per_cu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K::fn(), kIrThreads, K::lds()) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (per_cu >= 1 && nwg <= per_cu * prop.multiProcessorCount) ? nwg : 0;
}

// the block shapes of MobileNetV2's 14x14 / 7x7 stride-1 stages (cin, hidden, cout, H)
template <class F>
bool ir_dispatch(int cin, int ch, int cout, int H, F &&f) {
  if (H == 14 && cin == 64 && ch == 384 && cout == 64) return f(IrKernel<64, 384, 64, 14, 2>{}), true;
  if (H == 14 && cin == 64 && ch == 384 && cout == 96) return f(IrKernel<64, 384, 96, 14, 2>{}), true;
  if (H == 14 && cin == 96 && ch == 576 && cout == 96) return f(IrKernel<96, 576, 96, 14, 2>{}), true;
  if (H == 7 && cin == 160 && ch == 960 && cout == 160) return f(IrKernel<160, 960, 160, 7, 1>{}), true;
  if (H == 7 && cin == 160 && ch == 960 && cout == 320) return f(IrKernel<160, 960, 320, 7, 1>{}), true;
  return false;
}
}  // namespace

// workgroups of one launch (B images), or 0 when the shape has no fused kernel or the grid
// would not be co-resident on this device (the grid barriers need every workgroup resident)
void ir_trace_set(void *ts) {   // nullptr: off (the default)
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ir_ts), &ts, sizeof(ts));
}

int ir_fwd_grid(int B, int H, int cin, int ch, int cout) {
  int wgs = 0;
  ir_dispatch(cin, ch, cout, H, [&](auto k) { wgs = co_resident_grid<decltype(k)>(B); });
  return wgs;
}

int ir_bwd_grid(int B, int H, int cin, int ch, int cout) {
  int wgs = 0;
  ir_bwd_dispatch(cin, ch, cout, H, [&](auto k) { wgs = co_resident_grid<decltype(k)>(B); });
  return wgs;
}

void launch_ir_bwd(const bf16_t *G, const bf16_t *y, const void *lz_p, const bf16_t *wpt, const bf16_t *h2,
                   const float *sd, const float *td, bf16_t *gd, const void *dd, const bf16_t *wd, const bf16_t *h1,
                   const float *se, const float *te, bf16_t *ge, const void *de, const bf16_t *wet, const bf16_t *R,
                   const bf16_t *yprev, bf16_t *gout, const void *dprev, unsigned *bar, unsigned *err, int B, int H,
                   int cin, int ch, int cout, hipStream_t st) {
  IrBwdArgs a{G,  y,  static_cast<const BnFin *>(lz_p), wpt, h2, sd, td, gd, static_cast<const BnFin *>(dd), wd, h1,
              se, te, ge, static_cast<const BnFin *>(de), wet, R, yprev, gout, static_cast<const BnFin *>(dprev),
              bar, err};
  ir_bwd_dispatch(cin, ch, cout, H, [&](auto k) { decltype(k)::launch(a, B, st); });
}

void launch_ir_fwd(const bf16_t *xin, const bf16_t *res, const void *lz_in, bf16_t *xout, const bf16_t *we,
                   const bf16_t *wd, const bf16_t *wp, bf16_t *h1, bf16_t *h2, bf16_t *y, const void *de,
                   const void *dd, const void *dp, unsigned *bar, unsigned *err, int B, int H, int cin, int ch,
                   int cout, hipStream_t st) {
  IrArgs a{xin, res, static_cast<const BnFin *>(lz_in), xout, we, wd, wp, h1, h2, y,
           static_cast<const BnFin *>(de), static_cast<const BnFin *>(dd), static_cast<const BnFin *>(dp), bar, err};
  ir_dispatch(cin, ch, cout, H, [&](auto k) { decltype(k)::launch(a, B, st); });
}
