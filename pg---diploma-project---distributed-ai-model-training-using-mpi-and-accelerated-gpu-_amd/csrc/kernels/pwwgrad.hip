// Pointwise (1x1) conv weight gradient on LDS-DMA operand rings, for the MobileNetV2 layers
// whose weight gradient runs on the side stream (14x14 / 7x7 / 28x28 maps, N, K >= 64):
//
//   part[z][n][k] = sum_{m in split z} dy[m][n] x[m][k]
//   dy = a[n]*G + b[n]*Y + c[n]     (this layer's BN backward, G / Y stored bf16 [M][N])
//   x  = act(X)                     (ACT_NONE, or relu6(X*s[k] + t[k]) of the producer BN)
//
// Reference op: the weight gradient of every 1x1 Conv2d in loss.backward()
// (cifar10_mpi_mobilenet_224.py:179; SURVEY.md §2.6 "Pointwise conv 1x1").
//
// Why a second kernel (pwconv.hip pw_wgrad_kernel is the register-staged form): that kernel
// transforms and transposes every operand element through registers into LDS one 64-row step
// ahead, with 2 workgroups of 4 waves per CU; PMC (profiles/r3_pmc_step_mnv2.txt) shows it
// neither VALU- nor bandwidth-bound (VALU issue 16-21 %, 0.7-2 TB/s) but latency-bound: one
// step of global-load latency exposed per 64 rows.  Here the raw G, Y and X rows are streamed
// global -> LDS by buffer_load ... lds (no VGPRs per row in flight) into an NBUF-deep ring, two
// stages ahead, exactly as conv.hip conv_wgrad_dma_kernel streams ResNet-50's materialised
// operands (same 16-B chunk swizzle on the source side, same transposing ds_read_b64_tr_b16
// fragment reads); the BN transforms run on the MFMA fragments in registers instead:
//
//   * a dy fragment (lane: one column n, 8 consecutive m) is read from the G and the Y ring and
//     combined with this lane's a[n], b[n], c[n] (registers, loaded once);
//   * an x fragment (one column k, 8 consecutive m) gets relu6(x*s[k] + t[k]) (or nothing);
//     rows past the split end (only in a partial last stage) are zeroed on the x side.
//
// Each dy element is transformed once per (k tile, wave column) instead of once per element:
// extra VALU on a kernel whose VALU pipe was mostly idle.  The output contract (fp32 split
// partials, reduced by launch_wgrad_reduce) is that of pw_wgrad_kernel.
#include "../common.h"

namespace {
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

struct PwWgDmaArgs {
  const bf16_t *G, *Y;          // [M][N]
  const float *ga, *gb, *gc;    // [N]
  const bf16_t *X;              // [M][K]
  const float *xs, *xt;         // [K] (ACT_BN_RELU6)
  float *part;                  // [S][N][K]
  int M, N, K, rows_per_split;
};

// pair-level swizzle of row r for rows of RB bytes (conv.hip wg_sw): chunk q of row r sits at
// q ^ 2*sw(r); RB = 128 (64 columns) or 256 (128 columns)
template <int RB>
PG_DEVICE int dsw(int r) {
  if constexpr (RB == 256) return (r & 3) | (((r >> 3) & 1) << 2);
  else return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
}

template <int N>
PG_DEVICE void dma_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

PG_DEVICE void s16x8_to_f(const s16x8_t &v, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = __uint_as_float(((uint32_t)(uint16_t)v[j]) << 16);
}

PG_DEVICE s16x8_t f_to_s16x8(const float (&f)[8]) {
  u32x4_t u;
  u.x = pack2(f[0], f[1]);
  u.y = pack2(f[2], f[3]);
  u.z = pack2(f[4], f[5]);
  u.w = pack2(f[6], f[7]);
  return __builtin_bit_cast(s16x8_t, u);
}

// 8 m values of one column (the MFMA operand layout) from a ring stage of rows of RB bytes
template <int RB>
PG_DEVICE s16x8_t tr_frag(const char *base, int row, int blk, int sw, int tc) {
  const char *p = base + row * RB + (((blk + (tc >> 1)) ^ sw) * 16) + (tc & 1) * 8;
  const s16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)p);
  const s16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(p + 4 * RB));
  return __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
}
}  // namespace

template <int XPRO, int TN, int TK, int NBUF>
__global__ __launch_bounds__(256) void pw_wgrad_dma_kernel(PwWgDmaArgs p, int gx, int gy, int total) {
  constexpr int MK = 64;                                  // m rows per stage
  static_assert(NBUF >= 2 && NBUF <= 4, "2 to 4 stages");
  static_assert((TN == 64 || TN == 128) && (TK == 64 || TK == 128), "64/128-wide tiles");
  constexpr int RBN = TN * 2, RBK = TK * 2;               // staged row bytes
  constexpr int CPN = RBN / 16, CPK = RBK / 16;           // 16-B chunks per row
  constexpr int PN = MK * RBN / 1024, PK = MK * RBK / 1024;   // 1-KiB pieces per operand and stage
  constexpr int PNW = PN / 4, PKW = PK / 4;
  constexpr int PW = 2 * PNW + PKW;                       // DMA instructions per wave and stage
  constexpr int DBYTES = MK * RBN, SBYTES = MK * (2 * RBN + RBK);
  constexpr int QN = TN / 2, QK = TK / 2, RN = QN / 16, RK = QK / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  // XCD-aware order: the (n, k) tiles of one m split are contiguous logical ids on one XCD
  int L = blockIdx.x;
  if (total % 8 == 0) L = (L % 8) * (total / 8) + L / 8;
  const int bx = L % gx, by = (L / gx) % gy, bz = L / (gx * gy);
  const int n0 = bx * TN, k0 = by * TK;
  const int mbeg = bz * p.rows_per_split;
  const int mend = min(p.M, mbeg + p.rows_per_split);
  const int nsteps = (mend - mbeg + MK - 1) / MK;
  const rsrc_t rg = make_rsrc(p.G, (uint32_t)((size_t)p.M * p.N * 2));
  const rsrc_t ry = make_rsrc(p.Y, (uint32_t)((size_t)p.M * p.N * 2));
  const rsrc_t rx = make_rsrc(p.X, (uint32_t)((size_t)p.M * p.K * 2));
  const int drow0 = lane / CPN, dq = lane % CPN;
  const int xrow0 = lane / CPK, xq = lane % CPK;

  auto issue = [&](int step, int buf) {
    const int m0 = mbeg + step * MK;
    char *gbase = smem + buf * SBYTES;
    char *ybase = gbase + DBYTES;
    char *xbase = ybase + DBYTES;
#pragma unroll
    for (int i = 0; i < PNW; ++i) {
      const int piece = wave * PNW + i;
      const int row = piece * (1024 / RBN) + drow0;
      const int c = dq ^ (2 * dsw<RBN>(row));
      const int m = m0 + row, n = n0 + c * 8;
      const uint32_t off = (m < mend && n < p.N) ? (uint32_t)(((size_t)m * p.N + n) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (__attribute__((address_space(3))) void *)(gbase + piece * 1024), 16,
                                               off, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (__attribute__((address_space(3))) void *)(ybase + piece * 1024), 16,
                                               off, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PKW; ++i) {
      const int piece = wave * PKW + i;
      const int row = piece * (1024 / RBK) + xrow0;
      const int c = xq ^ (2 * dsw<RBK>(row));
      const int m = m0 + row, k = k0 + c * 8;
      const uint32_t off = (m < mend && k < p.K) ? (uint32_t)(((size_t)m * p.K + k) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void *)(xbase + piece * 1024), 16,
                                               off, 0, 0, 0);
    }
  };

  // this lane's per-column parameters (columns past N / K: 0, so padded columns contribute 0)
  float pa[RN], pb[RN], pc[RN], ps[RK], pt[RK];
#pragma unroll
  for (int a = 0; a < RN; ++a) {
    const int n = n0 + wn * QN + a * 16 + (lane & 15);
    const bool ok = n < p.N;
    pa[a] = ok ? p.ga[n] : 0.f;
    pb[a] = ok ? p.gb[n] : 0.f;
    pc[a] = ok ? p.gc[n] : 0.f;
  }
#pragma unroll
  for (int b = 0; b < RK; ++b) {
    const int k = k0 + wk * QK + b * 16 + (lane & 15);
    const bool ok = XPRO == ACT_BN_RELU6 && k < p.K;
    ps[b] = ok ? p.xs[k] : 0.f;
    pt[b] = ok ? p.xt[k] : 0.f;
  }

  f32x4_t acc[RN][RK];
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // transposed-read addressing (conv.hip conv_wgrad_dma_kernel): lane reads rows trow, trow + 4
  // of each 32-row sub-step; 8-B column piece tc of a 16-column block
  const int trow = 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int tc = lane & 3;
  const int swn = 2 * dsw<RBN>(trow), swk = 2 * dsw<RBK>(trow);
  const int mlane = 8 * (lane >> 4);                      // first of this lane's 8 m values per sub-step

  auto mma = [&](int buf, int m0) {
    const char *Gb = smem + buf * SBYTES;
    const char *Yb = Gb + DBYTES;
    const char *Xb = Yb + DBYTES;
    const bool partial = m0 + MK > mend;                  // workgroup-uniform
#pragma unroll
    for (int sub = 0; sub < MK / 32; ++sub) {
      s16x8_t af[RN], bfr[RK];
#pragma unroll
      for (int a = 0; a < RN; ++a) {
        const int blk = (wn * QN + a * 16) / 8;
        const s16x8_t g = tr_frag<RBN>(Gb, sub * 32 + trow, blk, swn, tc);
        const s16x8_t y = tr_frag<RBN>(Yb, sub * 32 + trow, blk, swn, tc);
        float gf[8], yf[8], d[8];
        s16x8_to_f(g, gf);
        s16x8_to_f(y, yf);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = fmaf(pa[a], gf[j], fmaf(pb[a], yf[j], pc[a]));
        af[a] = f_to_s16x8(d);
      }
#pragma unroll
      for (int b = 0; b < RK; ++b) {
        const int blk = (wk * QK + b * 16) / 8;
        const s16x8_t x = tr_frag<RBK>(Xb, sub * 32 + trow, blk, swk, tc);
        if constexpr (XPRO == ACT_BN_RELU6) {
          float xf[8];
          s16x8_to_f(x, xf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xf[j] = relu6f(fmaf(xf[j], ps[b], pt[b]));
            if (partial && m0 + sub * 32 + mlane + j >= mend) xf[j] = 0.f;   // rows past the split
          }
          bfr[b] = f_to_s16x8(xf);
        } else {
          bfr[b] = x;   // stored activations; rows past the split were read as 0
        }
      }
#pragma unroll
      for (int a = 0; a < RN; ++a)
#pragma unroll
        for (int b = 0; b < RK; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[a]),
                                                             __builtin_bit_cast(bf16x8_t, bfr[b]), acc[a][b], 0, 0, 0);
    }
  };

  if constexpr (NBUF == 2) {
    if (nsteps > 0) issue(0, 0);
    for (int s = 0; s < nsteps; ++s) {
      const int buf = s & 1;
      if (s + 1 < nsteps) {
        issue(s + 1, buf ^ 1);
        dma_wait_barrier<PW>();
      } else {
        dma_wait_barrier<0>();
      }
      mma(buf, mbeg + s * MK);
      dma_wait_barrier<PW>();
    }
  } else {
    // ring: NBUF - 1 stages in flight, one barrier per stage (stage s landed everywhere AND every
    // wave is done with stage s - 1, whose buffer the next issue refills)
#pragma unroll
    for (int q = 0; q < NBUF - 1; ++q)
      if (q < nsteps) issue(q, q);
    int buf = 0, nbuf = NBUF - 1;
    for (int s = 0; s < nsteps; ++s) {
      if (s + NBUF - 2 < nsteps) dma_wait_barrier<(NBUF - 2) * PW>();
      else if (NBUF == 4 && s + 1 < nsteps) dma_wait_barrier<PW>();
      else dma_wait_barrier<0>();
      if (s + NBUF - 1 < nsteps) issue(s + NBUF - 1, nbuf);
      mma(buf, mbeg + s * MK);
      buf = buf == NBUF - 1 ? 0 : buf + 1;
      nbuf = nbuf == NBUF - 1 ? 0 : nbuf + 1;
    }
  }
  // acc[a][b][j] = dW[n0 + wn*QN + a*16 + 4*(lane>>4) + j][k0 + wk*QK + b*16 + (lane&15)]
  float *dst = p.part + (size_t)bz * p.N * p.K;
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * QN + a * 16 + 4 * (lane >> 4) + j;
        const int k = k0 + wk * QK + b * 16 + (lane & 15);
        if (n < p.N && k < p.K) dst[(size_t)n * p.K + k] = acc[a][b][j];
      }
}

// ===========================================================================
// host
// ===========================================================================
// tiles: 128 wide for dimensions above 64 (fewer re-reads and re-transforms), else 64;
// ring depth 3 (two stages in flight, one barrier per stage).  Returns false (caller keeps the
// register-staged kernel) for shapes outside the DMA contract.
// Opt-in (PGDIST_PWWG_DMA=1): measured SLOWER than the register-staged kernel on every MobileNetV2
// shape (profiles/r4_roofline_pwwg_dma.txt: 22 launches 677 us at 128-wide tiles, 627 us at 64-wide,
// vs 548 us; bench 4.71 vs 4.64-4.65 ms/step): with 4-8 stages per split the ring never reaches
// steady state, and the per-fragment BN transforms (done once per (k tile, wave column) here instead
// of once per element) cost more VALU than the staging they replace.
bool pw_wgrad_dma_supported(int N, int K) {
  static const int on = [] { const char *e = getenv("PGDIST_PWWG_DMA"); return e ? atoi(e) : 0; }();
  return on && N >= 64 && K >= 64 && N % 8 == 0 && K % 8 == 0;
}

void pw_wgrad_dma_tiles(int N, int K, int &TN, int &TK) {
  static const int wide = [] { const char *e = getenv("PGDIST_PWWG_DMA_WIDE"); return e ? atoi(e) : 1; }();
  // the split geometry (pwconv.hip wgrad_geom) counts tiles with the same rule
  TN = (wide && N > 64) ? 128 : 64;
  TK = (wide && K > 64) ? 128 : 64;
}

template <int XPRO, int TN, int TK>
static void launch_pwwd_t(const PwWgDmaArgs &a, int S, hipStream_t st) {
  constexpr int NBUF = 3;
  const int gx = (a.N + TN - 1) / TN, gy = (a.K + TK - 1) / TK, total = gx * gy * S;
  const size_t lds = (size_t)NBUF * 64 * (2 * TN * 2 + TK * 2);
  hipLaunchKernelGGL((pw_wgrad_dma_kernel<XPRO, TN, TK, NBUF>), dim3(total), dim3(256), lds, st, a, gx, gy, total);
}

void launch_pw_wgrad_dma(const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb, const float *gc,
                         const bf16_t *X, const float *xs, const float *xt, int xact, float *part, int M, int N,
                         int K, int rps, int S, hipStream_t st) {
  PwWgDmaArgs a{G, Y, ga, gb, gc, X, xs, xt, part, M, N, K, rps};
  int TN, TK;
  pw_wgrad_dma_tiles(N, K, TN, TK);
#define PWWD_CASE(XP, A_, B_) \
  if (xact == XP && TN == A_ && TK == B_) { launch_pwwd_t<XP, A_, B_>(a, S, st); return; }
  PWWD_CASE(ACT_NONE, 64, 64) PWWD_CASE(ACT_NONE, 64, 128) PWWD_CASE(ACT_NONE, 128, 64) PWWD_CASE(ACT_NONE, 128, 128)
  PWWD_CASE(ACT_BN_RELU6, 64, 64) PWWD_CASE(ACT_BN_RELU6, 64, 128) PWWD_CASE(ACT_BN_RELU6, 128, 64)
  PWWD_CASE(ACT_BN_RELU6, 128, 128)
#undef PWWD_CASE
}
