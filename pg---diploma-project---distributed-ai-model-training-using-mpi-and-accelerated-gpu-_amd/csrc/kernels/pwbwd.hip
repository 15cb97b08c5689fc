// Fused pointwise-conv backward for the large-M layers (112x112 .. 28x28):
// dgrad AND wgrad from ONE read of this layer's (G, Y).
//
// Reference ops: the backward of the 1x1 convs of torchvision MobileNetV2
// (SURVEY.md §2.6), i.e. what cuDNN runs as two separate kernels (data grad,
// filter grad) each re-reading the output gradient.  In the fused NHWC pipeline
// the output gradient of a 1x1 conv is  dy = a[n]*G + b[n]*Y + c[n]  (the
// layer's own BN backward), so a separate wgrad would re-read two [M][N_l]
// bf16 tensors — for the 112x112 expand conv that is 616 MB per step.
//
// Per 64-row tile (4 waves, grid-stride over M, ALL loads of a tile — G, Y and the
// epilogue operands — prefetched one tile ahead; one N tile spans the whole Ng
// of the project convs so G, Y are read exactly once):
//   * dy is computed once from (G, Y) and written to LDS once, row-major dyN[m][kg]: the
//     dgrad MFMA reads it by rows (A operand), the wgrad MFMA (reduction over m) reads the
//     same image column-wise with the gfx950 transposing read ds_read_b64_tr_b16;
//   * the wgrad's second operand x (this conv's input) is staged row-major xN[m][ng], also
//     read transposed (the former transposed copies dyT / xT cost 8 ds_write_b64 per item at
//     8-10 bank-conflict cycles per LDS instruction, SQ_LDS_BANK_CONFLICT):
//       EPI_BWD_RELU6 (project conv): x = relu6(Yt*s + t) — Yt is the tensor the
//         dgrad epilogue reads anyway for the ReLU6 mask, so x costs no HBM bytes;
//       EPI_BWD_LIN   (expand conv):  x = X, the materialised block input;
//   * dgrad:  out[m][ng] = sum_kg dy[m][kg] W^T[ng][kg]  (W^T resident in LDS),
//     epilogue identical to pw_gemm_kernel (mask / residual, BN partials);
//   * wgrad:  dW[kg][ng] += sum_m dyT[kg][m] xT[ng][m], accumulated in registers
//     across the workgroup's tiles and written once as a split-M partial
//     [gridDim.x][Kg][Ng] (deterministic fixed-order reduction afterwards).
//   * RECOMP (expand convs, EPI_BWD_LIN with Ng <= 32): the BN input Y = X We^T of this conv is
//     NOT read from HBM but re-formed from the X tile already staged for the wgrad: one
//     16x16x32 MFMA per 16 x 16 piece of Y (K = Cin = 16..32, zero-padded), written as bf16
//     into the dy image and transformed there in place.  Y is the block's hidden tensor h1
//     (6x the input's channels): 308 of the 770 MB the 112x112 expand backward read.
#include "../bnfin.h"

#include <cstdlib>

enum { EPI_BWD_RELU6_ = 1, EPI_BWD_LIN_ = 2 };   // same values as pwconv.hip
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// Phase trace (diagnostics builds only, PGDIST_DEFINES=PGDIST_PWT_TRACE): thread 0 of every
// workgroup sums the wall clock (100 MHz ticks) spent per phase over its tiles and writes the
// sums to g_pwb_ts[wg][8]: 0 prologue, 1 staging (incl. the wait for the prefetched tile),
// 2 MFMAs, 3 C tile, 4 epilogue stores, 5 tail, 6 tiles
#ifdef PGDIST_PWT_TRACE
__device__ unsigned long long *g_pwb_ts = nullptr;
#define PWB_T0() unsigned long long pwb_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pwb_last_ = wall_clock64()
#define PWB_MARK(k)                                       \
  do {                                                    \
    const unsigned long long n_ = wall_clock64();         \
    pwb_acc_[k] += n_ - pwb_last_;                        \
    pwb_last_ = n_;                                       \
  } while (0)
#define PWB_DONE()                                                                  \
  do {                                                                              \
    unsigned long long *t_ = g_pwb_ts;                                              \
    if (t_ && threadIdx.x == 0)                                                     \
      for (int k_ = 0; k_ < 8; ++k_) t_[(size_t)blockIdx.x * 8 + k_] = pwb_acc_[k_]; \
  } while (0)
#else
#define PWB_T0() ((void)0)
#define PWB_MARK(k) ((void)0)
#define PWB_DONE() ((void)0)
#endif

namespace {
struct PwBwdArgs {
  const bf16_t *G, *Y;          // [M][Kg]
  const float *ca, *cb, *cc;    // [Kg] BN backward coefficients of this layer
  const bf16_t *WT;             // [Ng][Kg] transposed conv weight
  bf16_t *out;                  // [M][Ng]
  const bf16_t *Yt;             // [M][Ng] producer BN input
  const float *es, *et;         // [Ng] producer BN scale / shift (RELU6 mode)
  const bf16_t *R;              // [M][Ng] residual gradient (LIN mode, optional)
  const bf16_t *X;              // [M][Ng] conv input (LIN mode)
  const bf16_t *We;             // [Kg][Ng] forward conv weight (RECOMP: Y = X We^T, Y unused)
  float *part;                  // [gx][2][Ng]
  float *wpart;                 // [gx][Kg][Ng]
  int M, Kg, Ng;
  int bn_rep;                   // BN-statistics replica rows (g_bn_rep)
  const BnFin *fin;             // fused BN finalize in the tail (nullptr: none)
  const BnFin *lz;              // lazy finalize of ca / cb / cc (nullptr: materialised)
};
// RAWX (project convs with one wide N tile): xN holds the RAW producer activation Yt, the
// ReLU6(BN) of the wgrad operand is applied after the transposed read and the epilogue takes
// its mask operand from xN, so no register copy of the tile's Yt is kept (those registers
// spilled at Ng = 144 / 192); the C tile then gets its own LDS region
template <int KP, int BN, int BM, bool RAWX = false, bool RECOMP = false>
struct BwdLds {
  static constexpr int LDA = KP + 8, LDX = BN + 8, LDC = BN + 8, LDW = BN + 8;
  static constexpr int WT = 0;                              // [BN][LDA] W^T tile (resident)
  static constexpr int WE = WT + BN * LDA * 2;              // [KP][LDW] W tile (RECOMP, resident)
  static constexpr int STG = WE + (RECOMP ? KP * LDW * 2 : 0);   // per-tile staging:
  static constexpr int DYN = STG;                           //   dyN [BM][LDA]
  static constexpr int XN = DYN + BM * LDA * 2;             //   xN  [BM][LDX]
  static constexpr int STG_END = XN + BM * LDX * 2;
  static constexpr int CS = RAWX ? STG_END : STG;           // C tile [BM][LDC] (aliases the staging)
  static constexpr int RED = STG;                           // [BM/4][BN] floats at the very end
  static constexpr int CS_END = CS + BM * LDC * 2;
  static constexpr int RED_END = RED + (BM / 4) * BN * 4;
  static constexpr int M1 = STG_END > CS_END ? STG_END : CS_END;
  static constexpr int PS = M1 > RED_END ? M1 : RED_END;     // a | b | c [KP], s | t [BN]
  static constexpr int BYTES = PS + (3 * KP + 2 * BN) * 4;
};
}  // namespace

// BM = 64 rows per tile (4 waves x 16 rows for the dgrad MFMA) or 32 (2 row groups x
// 2 column halves; used when KP is large so the prefetched tile fits in registers)
template <int EPI, int KP, int BN, int BM, bool RECOMP = false>
// 2 waves per SIMD for the register allocation (3 would spill 12-328 B per variant)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void pw_bwd_fused_kernel(PwBwdArgs p) {
  constexpr bool RAWX = EPI != EPI_BWD_LIN_ && BN >= 96;
  static_assert(!RECOMP || (EPI == EPI_BWD_LIN_ && BN == 32), "Y recompute: expand convs with Cin <= 32");
  using L = BwdLds<KP, BN, BM, RAWX, RECOMP>;
  constexpr int LDA = L::LDA, LDX = L::LDX, LDC = L::LDC;
  constexpr int CT = BN / 16;
  constexpr int RGS = BM / 16;                   // dgrad row groups of 16
  constexpr int RPW = RGS >= 4 ? RGS / 4 : 1;    // row groups per wave
  constexpr int CSPLIT = RGS >= 4 ? 1 : 4 / RGS; // waves sharing a row group (column split)
  constexpr int CTW = CT / CSPLIT;               // dgrad column tiles per wave
  static_assert(CTW * CSPLIT == CT, "column tiles must split evenly over the waves");
  constexpr int DYC = KP / 8;                    // 16-B chunks per dy row
  constexpr int NDY = (BM / 4) * DYC;            // dy items (4 rows x 8 cols)
  constexpr int IDY = (NDY + 255) / 256;
  constexpr int XC = BN / 8;
  constexpr int NX = (BM / 4) * XC;              // x / epilogue items (4 rows x 8 cols)
  constexpr int IX = (NX + 255) / 256;
  constexpr int WTILES = (KP / 16) * (BN / 16);
  constexpr int WPW = (WTILES + 3) / 4;          // wgrad output tiles per wave
  constexpr bool LIN = EPI == EPI_BWD_LIN_;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t *WTs = reinterpret_cast<bf16_t *>(smem + L::WT);
  bf16_t *WEs = reinterpret_cast<bf16_t *>(smem + L::WE);
  bf16_t *dyN = reinterpret_cast<bf16_t *>(smem + L::DYN);
  bf16_t *xN = reinterpret_cast<bf16_t *>(smem + L::XN);
  bf16_t *Cs = reinterpret_cast<bf16_t *>(smem + L::CS);
  float *Red = reinterpret_cast<float *>(smem + L::RED);
  float *Ps = reinterpret_cast<float *>(smem + L::PS);

  PWB_T0();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rw = RGS >= 4 ? wave : wave % RGS, cw = RGS >= 4 ? 0 : wave / RGS;   // rows rw + 4*r
  const int n0 = blockIdx.y * BN;
  const int nmt = (p.M + BM - 1) / BM;

  // ---- resident operands: W^T tile, BN-backward coefficients, producer BN scale/shift
  for (int i = tid; i < BN * DYC; i += 256) {
    const int r = i / DYC, c8 = (i % DYC) * 8, n = n0 + r;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < p.Ng && c8 < p.Kg) v = ldg16(p.WT + (size_t)n * p.Kg + c8);
    *reinterpret_cast<uint4 *>(WTs + r * LDA + c8) = v;
  }
  if constexpr (RECOMP) {   // W [kg][ng] (B operand of the Y recompute), zero past Kg / Ng
    for (int i = tid; i < KP * (BN / 8); i += 256) {
      const int r = i / (BN / 8), c8 = (i % (BN / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < p.Kg && c8 < p.Ng) v = ldg16(p.We + (size_t)r * p.Ng + c8);
      *reinterpret_cast<uint4 *>(WEs + r * L::LDW + c8) = v;
    }
  }
  for (int i = tid; i < KP; i += 256) {
    const bool ok = i < p.Kg;
    if (p.lz) {
      float a = 0.f, b = 0.f, c = 0.f;
      if (ok) bn_lazy(p.lz, i, a, b, c);
      Ps[i] = a;
      Ps[KP + i] = b;
      Ps[2 * KP + i] = c;
    } else {
      Ps[i] = ok ? p.ca[i] : 0.f;
      Ps[KP + i] = ok ? p.cb[i] : 0.f;
      Ps[2 * KP + i] = ok ? p.cc[i] : 0.f;
    }
  }
  for (int i = tid; i < BN; i += 256) {
    const bool ok = !LIN && n0 + i < p.Ng;
    Ps[3 * KP + i] = ok ? p.es[n0 + i] : 0.f;
    Ps[3 * KP + BN + i] = ok ? p.et[n0 + i] : 0.f;
  }
  __syncthreads();

  float st0[IX][8], st1[IX][8];
#pragma unroll
  for (int i = 0; i < IX; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) st0[i][j] = st1[i][j] = 0.f;
  f32x4_t accW[WPW];
#pragma unroll
  for (int u = 0; u < WPW; ++u) accW[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- staging registers (one tile ahead): G, Y; Yt (both modes); X and R (LIN)
  uint4 gq[IDY][4], yq[IDY][4], tq[IX][4], xq[LIN ? IX : 1][4], rq[LIN ? IX : 1][4];
  // bounds-checked buffer loads issued unconditionally (masked lanes and the prefetch past the
  // last tile read 0 through an out-of-range offset): no branch, so hipcc keeps the next
  // tile's loads in flight instead of draining vmcnt(0) at a join
  const uint32_t gbytes = (uint32_t)((size_t)p.M * p.Kg * 2), tbytes = (uint32_t)((size_t)p.M * p.Ng * 2);
  const rsrc_t rG = make_rsrc(p.G, gbytes), rY = make_rsrc(p.Y, gbytes), rT = make_rsrc(p.Yt, tbytes);
  const rsrc_t rX = make_rsrc(LIN ? p.X : p.Yt, tbytes), rR = make_rsrc(p.R, p.R ? tbytes : 0u);
  auto load_tile = [&](int m0, bool valid) {
#pragma unroll
    for (int i = 0; i < IDY; ++i) {
      const int it = tid + i * 256;
      const int c8 = (it % DYC) * 8, m4 = it / DYC;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + m4 * 4 + q;
        const uint32_t off = boff(valid && it < NDY && row < p.M && c8 < p.Kg, (size_t)row * p.Kg + c8);
        gq[i][q] = bld16(rG, off);
        if constexpr (!RECOMP) yq[i][q] = bld16(rY, off);
      }
    }
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int it = tid + i * 256;
      const int c8 = (it % XC) * 8, m4 = it / XC;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + m4 * 4 + q;
        const uint32_t off = boff(valid && it < NX && row < p.M && n0 + c8 < p.Ng, (size_t)row * p.Ng + n0 + c8);
        tq[i][q] = bld16(rT, off);
        if constexpr (LIN) {
          xq[i][q] = bld16(rX, off);
          rq[i][q] = bld16(rR, off);
        }
      }
    }
  };

  load_tile(blockIdx.x * BM, blockIdx.x < nmt);
  PWB_MARK(0);
  for (int mt = blockIdx.x; mt < nmt; mt += gridDim.x) {
    const int m0 = mt * BM;
    __syncthreads();                 // previous tile's epilogue is done with Cs (aliases the staging)
    // ---- stage dy and x (row-major) for this tile (RECOMP: x first, Y re-formed from it, then dy)
    auto stage_dy = [&]() {
#pragma unroll
    for (int i = 0; i < IDY; ++i) {
      const int it = tid + i * 256;
      if (it < NDY) {
        const int c8 = (it % DYC) * 8, m4 = it / DYC;
        float a[8], b[8], c[8], v[4][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = Ps[c8 + j];
          b[j] = Ps[KP + c8 + j];
          c[j] = Ps[2 * KP + c8 + j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float g[8], y[8];
          unpack8(gq[i][q], g);
          if constexpr (RECOMP) unpack8(*reinterpret_cast<const uint4 *>(dyN + (m4 * 4 + q) * LDA + c8), y);
          else unpack8(yq[i][q], y);
          const bool valid = m0 + m4 * 4 + q < p.M;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] = valid ? bf2f(f2bf(fmaf(a[j], g[j], fmaf(b[j], y[j], c[j])))) : 0.f;
          *reinterpret_cast<uint4 *>(dyN + (m4 * 4 + q) * LDA + c8) = pack8(v[q]);
        }
      }
    }
    };
    if constexpr (!RECOMP) stage_dy();
    uint4 ct[RAWX ? 1 : IX][4], cr[LIN ? IX : 1][4];   // this tile's epilogue operands (raw Yt, R)
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int it = tid + i * 256;
      const int c8 = (it % XC) * 8, m4 = it / XC;
      float v[4][8];
      if constexpr (RAWX) {   // raw Yt row-major into xN (ReLU6(BN) applied at the wgrad read)
        if (it < NX) {
#pragma unroll
          for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4 *>(xN + (m4 * 4 + q) * LDX + c8) = tq[i][q];
        }
        continue;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ct[RAWX ? 0 : i][q] = tq[i][q];
        if constexpr (LIN) {
          cr[i][q] = rq[i][q];
          unpack8(xq[i][q], v[q]);
        } else {
          const bool valid = m0 + m4 * 4 + q < p.M;
          unpack8(tq[i][q], v[q]);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[q][j] = valid ? relu6f(fmaf(v[q][j], Ps[3 * KP + c8 + j], Ps[3 * KP + BN + c8 + j])) : 0.f;
        }
      }
      if (it < NX) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4 *>(xN + (m4 * 4 + q) * LDX + c8) = pack8(v[q]);
      }
    }
    if constexpr (RECOMP) {
      __syncthreads();   // x staged
      // Y[m][kg] = sum_ng X[m][ng] W[kg][ng]: one MFMA per 16 x 16 piece (K = 32 >= Cin), bf16
      // (the value the expand forward stored) into the dy image
      constexpr int YT = (BM / 16) * (KP / 16);
#pragma unroll
      for (int u = 0; u < (YT + 3) / 4; ++u) {
        const int t = wave + 4 * u;
        if (t < YT) {
          const int rg = t / (KP / 16), kt = t % (KP / 16);
          const s16x8_t xa = *reinterpret_cast<const s16x8_t *>(xN + (rg * 16 + (lane & 15)) * LDX + 8 * (lane >> 4));
          const s16x8_t wb =
              *reinterpret_cast<const s16x8_t *>(WEs + (kt * 16 + (lane & 15)) * L::LDW + 8 * (lane >> 4));
          const f32x4_t yv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, xa), __builtin_bit_cast(bf16x8_t, wb), f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) dyN[(rg * 16 + 4 * (lane >> 4) + j) * LDA + kt * 16 + (lane & 15)] = f2bf(yv[j]);
        }
      }
      __syncthreads();   // Y image complete
      stage_dy();        // in place: each item reads and rewrites its own 4 x 8 piece
    }
    __syncthreads();
    PWB_MARK(1);
    load_tile((mt + gridDim.x) * BM, mt + gridDim.x < nmt);   // next tile in flight from here on
    // ---- dgrad MFMA: wave -> rows rw*16 .. +16, column tiles cw*CTW .. +CTW
    f32x4_t acc[RPW][CTW];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < CTW; ++c) acc[r][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KP / 32; ++ks) {
      s16x8_t af[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r)
        af[r] = *reinterpret_cast<const s16x8_t *>(dyN + ((rw + 4 * r) * 16 + (lane & 15)) * LDA + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int c = 0; c < CTW; ++c) {
        const s16x8_t bf = *reinterpret_cast<const s16x8_t *>(WTs + ((cw * CTW + c) * 16 + (lane & 15)) * LDA + ks * 32 + 8 * (lane >> 4));
#pragma unroll
        for (int r = 0; r < RPW; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[r]),
                                                              __builtin_bit_cast(bf16x8_t, bf), acc[r][c], 0, 0, 0);
      }
    }
    // ---- wgrad MFMA: dW[kg][ng] over this tile's rows.  Both operands are transposed reads of
    // the row-major images: lane 4q+p of each 16-lane group addresses row m0+q, columns 4p..4p+3
    // of a 4 x 16 block and receives one column (4 rows); rows 8g..8g+3 and 8g+4..8g+7 of the
    // 32-row step give lane (i, g) the 8 k-values of column i (EXEC is full: t is wave-uniform)
    const int trow = 8 * (lane >> 4) + ((lane & 15) >> 2), tcol = 4 * (lane & 3);
#pragma unroll
    for (int u = 0; u < WPW; ++u) {
      const int t = wave + 4 * u;
      if (t < WTILES) {
        const int ti = t / (BN / 16), tj = t % (BN / 16);
#pragma unroll
        for (int ms = 0; ms < BM / 32; ++ms) {
          const bf16_t *pa = dyN + (ms * 32 + trow) * LDA + ti * 16 + tcol;
          const bf16_t *pb = xN + (ms * 32 + trow) * LDX + tj * 16 + tcol;
          const s16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)pa);
          const s16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(pa + 4 * LDA));
          const s16x4_t b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)pb);
          const s16x4_t b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(pb + 4 * LDX));
          const s16x8_t af = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
          s16x8_t bf = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
          if constexpr (RAWX) {   // lane holds 8 rows of ONE column tj*16 + (lane & 15): x = relu6(Yt*s + t)
            const int col = tj * 16 + (lane & 15);
            const float s_ = Ps[3 * KP + col], t_ = Ps[3 * KP + BN + col];
            float xv[8];
            unpack8(__builtin_bit_cast(uint4, bf), xv);
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = relu6f(fmaf(xv[j], s_, t_));
            bf = __builtin_bit_cast(s16x8_t, pack8(xv));
          }
          accW[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af),
                                                            __builtin_bit_cast(bf16x8_t, bf), accW[u], 0, 0, 0);
        }
      }
    }
    __syncthreads();                 // staging reads done: Cs may overwrite it
    PWB_MARK(2);
    // acc[r][c][j] = C[(rw + 4r)*16 + 4*(lane>>4) + j][(cw*CTW + c)*16 + (lane&15)]
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          Cs[((rw + 4 * r) * 16 + 4 * (lane >> 4) + j) * LDC + (cw * CTW + c) * 16 + (lane & 15)] = f2bf(acc[r][c][j]);
    __syncthreads();
    PWB_MARK(3);
    // ---- epilogue, item mapping (4 rows x 8 cols, operands already in registers)
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int it = tid + i * 256;
      if (it < NX) {
        const int c8 = (it % XC) * 8, m4 = it / XC;
        float es[8], et[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          es[j] = Ps[3 * KP + c8 + j];
          et[j] = Ps[3 * KP + BN + c8 + j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = m0 + m4 * 4 + q;
          if (row < p.M && n0 + c8 < p.Ng) {
            float v[8], yt[8];
            unpack8(*reinterpret_cast<const uint4 *>(Cs + (m4 * 4 + q) * LDC + c8), v);
            if constexpr (RAWX) unpack8(*reinterpret_cast<const uint4 *>(xN + (m4 * 4 + q) * LDX + c8), yt);
            else unpack8(ct[i][q], yt);
            if constexpr (!LIN) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] *= relu6_mask(yt[j], es[j], et[j]);
            } else {
              float rv[8];
              unpack8(cr[i][q], rv);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += rv[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              st0[i][j] += v[j];
              st1[i][j] = fmaf(v[j], yt[j], st1[i][j]);
            }
            stg16(p.out + (size_t)row * p.Ng + n0 + c8, pack8(v));
          }
        }
      }
    }
    PWB_MARK(4);
#ifdef PGDIST_PWT_TRACE
    pwb_acc_[6] += 1;
#endif
  }
  __syncthreads();
  // ---- wgrad partial of this workgroup: accW[u][j] = dW[ti*16 + 4*(lane>>4) + j][n0 + tj*16 + (lane&15)]
  float *wdst = p.wpart + (size_t)blockIdx.x * p.Kg * p.Ng;
#pragma unroll
  for (int u = 0; u < WPW; ++u) {
    const int t = wave + 4 * u;
    if (t < WTILES) {
      const int ti = t / (BN / 16), tj = t % (BN / 16);
      const int ng = n0 + tj * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kg = ti * 16 + 4 * (lane >> 4) + j;
        if (kg < p.Kg && ng < p.Ng) wdst[(size_t)kg * p.Ng + ng] = accW[u][j];
      }
    }
  }
  // ---- BN partials of the produced gradient (sum g, sum g*yt): Red[m4][col], 16 row groups
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int it = tid + i * 256;
      if (it < NX) {
        const int c8 = (it % XC) * 8, m4 = it / XC;
#pragma unroll
        for (int j = 0; j < 8; ++j) Red[m4 * BN + c8 + j] = s == 0 ? st0[i][j] : st1[i][j];
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      float a = 0.f;
#pragma unroll
      for (int g = 0; g < BM / 4; ++g) a += Red[g * BN + c];
      if (n0 + c < p.Ng) bn_part_add(p.part, blockIdx.x, gridDim.x, p.bn_rep, p.Ng, s, n0 + c, a);
    }
    __syncthreads();
  }
  bn_fin_tail(p.fin);
  PWB_MARK(5);
  PWB_DONE();
}

void pwb_trace_set(void *ts) {   // nullptr: off; no-op unless built with PGDIST_PWT_TRACE
#ifdef PGDIST_PWT_TRACE
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pwb_ts), &ts, sizeof(ts));
#else
  (void)ts;
#endif
}

// ===========================================================================
// host side
// ===========================================================================
void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st, bool stem36 = false);
int colsum_rows(int R);

int g_pwb_min_m = 65536;   // smallest M the fused dgrad + wgrad takes (pw_bwd_set_min_m)
namespace {
struct BwdGeom {
  int KP, BN, BM, nt, gx;
  bool ok;
};
BwdGeom bwd_geom(int M, int Kg, int Ng, bool recomp = false) {
  BwdGeom g{};
  g.KP = (Kg + 31) / 32 * 32;
  // one N tile covering all of Ng where it is small enough (no re-read of G, Y per tile)
  if (Ng <= 32) g.BN = 32;
  else if (Ng % 64 == 0 || Ng % 48 != 0 || g.KP >= 160) g.BN = 64;
  else g.BN = 48;
  // project convs (small Kg, wide Ng = 96 / 144 / 192): ONE N tile spanning the whole row.
  // With 48- / 64-column tiles each workgroup read and wrote 96- / 128-byte pieces of the
  // 192..384-byte NHWC rows (partial 128-B lines, G and Y re-read per N tile): 1.6-2.0 TB/s
  // (profiles/r3_roofline_base.txt; 909 -> 783 us with the wide tiles)
  if (g.KP <= 32 && (Ng == 96 || Ng == 144 || Ng == 192)) g.BN = Ng;
  // rows per tile: enough 4x8 staging items for all 256 threads, while the prefetched
  // (G, Y) tile stays within 2 waves/SIMD of registers
  const int chunks = (g.KP > g.BN ? g.KP : g.BN) / 8;
  g.BM = g.KP >= 160 ? 32 : (chunks <= 4 ? 256 : (chunks <= 8 ? 128 : 64));
  // the Y-recompute form loads no Y tile: twice the rows per tile keep the bytes in flight per
  // workgroup (the loop is bound by one tile's load latency, not by its bytes)
  if (recomp && g.BN == 32 && g.BM <= 64) g.BM *= 2;
  // M >= 64k (the 112x112 .. 28x28 layers), or the narrow-K small maps (the 14x14 project convs
  // at batch 128, Kg = 64 / 96): their weight gradient leaves the side stream, 4.198-4.213 vs
  // 4.222-4.234 ms/step; the 7x7 project convs too (Kg = 160, M = 6272): 4.264-4.276, slower
  // (docs/PERF_NOTES.md round 6)
  g.ok = (M >= g_pwb_min_m || (M >= 16384 && g.KP <= 96)) && g.KP <= 192 && Kg % 8 == 0 && Ng % 8 == 0 &&
         Kg > 0 && Ng > 0;
  g.nt = (Ng + g.BN - 1) / g.BN;
  const int nmt = (M + g.BM - 1) / g.BM;
  int gx = 512 / g.nt;   // grid target 512 (768 / 1024: slower, docs/PERF_NOTES.md round 2)
  if (gx > nmt) gx = nmt;
  gx = (gx + 7) & ~7;
  if (gx < 8) gx = 8;
  g.gx = gx;
  return g;
}

template <int EPI, int KP, int BN, int BM>
void launch_bwd_t(const PwBwdArgs &a, const BwdGeom &g, hipStream_t st) {
  if constexpr (EPI == EPI_BWD_LIN_ && BN == 32) {
    if (a.We) {   // Y re-formed from the staged X tile
      hipLaunchKernelGGL((pw_bwd_fused_kernel<EPI, KP, BN, BM, true>), dim3(g.gx, g.nt), dim3(256),
                         (BwdLds<KP, BN, BM, false, true>::BYTES), st, a);
      return;
    }
  }
  hipLaunchKernelGGL((pw_bwd_fused_kernel<EPI, KP, BN, BM>), dim3(g.gx, g.nt), dim3(256),
                     (BwdLds<KP, BN, BM, EPI != EPI_BWD_LIN_ && BN >= 96>::BYTES), st, a);
}

template <int EPI>
void launch_bwd_epi(const PwBwdArgs &a, const BwdGeom &g, hipStream_t st) {
#define BWD_CASE(KQ, BQ, MQ) \
  if (g.KP == KQ && g.BN == BQ && g.BM == MQ) { launch_bwd_t<EPI, KQ, BQ, MQ>(a, g, st); return; }
  BWD_CASE(32, 32, 256) BWD_CASE(64, 32, 128) BWD_CASE(96, 32, 64) BWD_CASE(128, 32, 64)
  BWD_CASE(32, 48, 128) BWD_CASE(64, 48, 128) BWD_CASE(96, 48, 64) BWD_CASE(128, 48, 64)
  BWD_CASE(32, 64, 128) BWD_CASE(64, 64, 128) BWD_CASE(96, 64, 64) BWD_CASE(128, 64, 64)
  BWD_CASE(160, 32, 32) BWD_CASE(192, 32, 32) BWD_CASE(160, 64, 32) BWD_CASE(192, 64, 32)
  if constexpr (EPI == EPI_BWD_LIN_) {   // Y-recompute geometries (twice the rows)
    BWD_CASE(96, 32, 128) BWD_CASE(160, 32, 64) BWD_CASE(192, 32, 64)
  }
  if constexpr (EPI != EPI_BWD_LIN_) {   // wide project tiles (RAWX): the project convs only
    BWD_CASE(32, 96, 64) BWD_CASE(32, 144, 64) BWD_CASE(32, 192, 64)
  }
#undef BWD_CASE
}
}  // namespace

bool pw_bwd_supported(int M, int Kg, int Ng) { return bwd_geom(M, Kg, Ng).ok; }
void pw_bwd_set_min_m(int m) { g_pwb_min_m = m; }
// the expand-conv form that re-forms Y from X (pw_bwd with We): one 32-wide N tile
bool pw_bwd_recompute_supported(int M, int Kg, int Ng) {
  const BwdGeom g = bwd_geom(M, Kg, Ng);
  return g.ok && g.BN == 32 && g.nt == 1;
}
int pw_bwd_num_partials(int M, int Kg, int Ng) { return bwd_geom(M, Kg, Ng).gx; }
long long pw_bwd_wgrad_workspace_floats(int M, int Kg, int Ng) {
  const int S = bwd_geom(M, Kg, Ng).gx;
  return (long long)(S + colsum_rows(S)) * Kg * Ng;
}

// epi: 1 = EPI_BWD_RELU6 (project conv; wgrad x = relu6(Yt*es+et)), 2 = EPI_BWD_LIN (x = X)
void launch_pw_bwd(int epi, const bf16_t *G, const bf16_t *Y, const float *ca, const float *cb,
                   const float *cc, const bf16_t *WT, bf16_t *out, const bf16_t *Yt, const float *es,
                   const float *et, const bf16_t *R, const bf16_t *X, const bf16_t *We, float *part,
                   float *wpart, float *grad, int M, int Kg, int Ng, hipStream_t st) {
  const BwdGeom g = bwd_geom(M, Kg, Ng, We != nullptr);
  const BnFin *fin = take_bn_fin();
  const BnFin *lz = take_bn_lz();
  if (!g.ok) return;
  if (We && !(epi == EPI_BWD_LIN_ && pw_bwd_recompute_supported(M, Kg, Ng))) return;   // (checked by the caller)
  PwBwdArgs a{G, Y, ca, cb, cc, WT, out, Yt, es, et, R, X, We, part, wpart, M, Kg, Ng, g_bn_rep, fin, lz};
  if (epi == EPI_BWD_RELU6_) launch_bwd_epi<EPI_BWD_RELU6_>(a, g, st);
  else launch_bwd_epi<EPI_BWD_LIN_>(a, g, st);
  // grad == nullptr: the caller reduces wpart itself (e.g. on its weight-gradient stream)
  if (grad) launch_wgrad_reduce(wpart, g.gx, (long long)Kg * Ng, grad, st);
}
