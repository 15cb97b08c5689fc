// Dense convolutions for ResNet-50 (BASELINE.json config 4) on gfx950 MFMA.
//
// The reference trains through cuDNN ("cuDNN conv fwd/bwd"); here every
// dense convolution of a bottleneck network (7x7 s2 stem, 1x1, 3x3 s1/s2, 1x1 s2
// projection shortcut) is an NHWC implicit GEMM on v_mfma_f32_16x16x32_bf16:
//
//   forward   y[m][n]  = sum_k A[m][k] W[n][k]        m = (b, oh, ow), k = (r, s, ci)
//             A gathered from x at (oh*st - pad + r, ow*st - pad + s), zero outside;
//             optional BN+ReLU of the producer applied while the tile is staged
//             (padding stays zero); epilogue: bf16 y + per-tile BN partial sums.
//   dgrad     dx = conv^T(dy): the output pixels are split into st x st parity classes;
//             class (ph, pw) only meets the taps with (ph + pad - r) % st == 0, so a
//             stride-2 3x3 layer does 9 taps of work over its 4 classes instead of 36
//             (no MFMA time on the structural zeros of the transposed convolution).
//             A = BN-backward(dy) (a*G + b*Y + c, this layer's BN) applied while staging;
//             B = W^T [ci][r][s][co] (transposed once per step); epilogue: ReLU mask of
//             the producer's BN (+ BN partials), or (acc + shortcut grad) * (x > 0) with
//             partials against up to two pre-BN tensors (bn3 and the projection BN of
//             the previous block share that gradient).
//   wgrad     dW[n][k] = sum_m dy[m][n] x[m][k]: split over m (deterministic partial
//             slabs + one reduction launch), both operands transposed into m-contiguous
//             LDS rows while staged, BN-backward on dy and BN+ReLU on x in the staging pass.
//
// Tiles: 4 waves (2 x 2), BM x BN in {128, 64}^2, k-steps of 32 or 64 bf16 with both
// operand tiles double-buffered in LDS and the next step's global loads in flight during
// the current step's MFMAs.  When Ci % KSTEP == 0 a k-step lies inside one filter tap, so
// the tap decomposition is one scalar division per step.  Workgroup ids put the N tiles
// of one M tile 8 ids apart (same XCD L2; T1 of the CDNA guide).
#include "../bnfin.h"
#include "../common.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {
enum { CM_FWD = 0, CM_DGRAD = 1 };
enum { CP_NONE = 0, CP_BN_RELU = 1, CP_BNBWD = 3 };
// backward epilogues: ReLU mask of the producer BN, or (+R) (*1[X>0]) with statistics against
// Yt (and Yt2); the operand set is a template choice so every epilogue load is unconditional
// CE_BWD_RXYM / CE_BWD_RXYYM: the ReLU mask 1[X > 0] comes from a bit mask Xm [M][N/8] (bit j of
// byte (m*N + n)/8 = channel n % 8 ... of pixel m) written by res_out instead of the bf16 X itself
enum { CE_FWD = 0, CE_BWD_RELU = 1, CE_BWD_PLAIN = 2, CE_BWD_R = 3, CE_BWD_RXY = 4, CE_BWD_RXYY = 5,
       CE_BWD_RXYM = 6, CE_BWD_RXYYM = 7 };

struct ConvArgs {
  const bf16_t *A;      // gathered image [Nb][Hi][Wi][Ci]  (fwd: x, dgrad: G of this layer's BN)
  const bf16_t *A2;     // dgrad: pre-BN output Y of this layer (same layout as A)
  const float *pa, *pb, *pc;   // per-Ci prologue parameters
  const bf16_t *W;      // fwd: [N][R][S][Ci] ; dgrad: [N=Cin][R][S][Ci=Cout]
  bf16_t *out;          // [Nb][Ho][Wo][N]
  const bf16_t *Yt;     // epilogue statistics partner [Nb][Ho][Wo][N]
  const bf16_t *Yt2;    // second partner (CE_BWD_RES)
  const bf16_t *X;      // CE_BWD_RES: mask tensor (x > 0), may be null
  const uint8_t *Xm;    // CE_BWD_RXYM / RXYYM: the same mask as bits (res_out mask output)
  const bf16_t *Rg;     // CE_BWD_RES: added gradient, may be null
  const float *es, *et; // CE_BWD_RELU: producer BN scale / shift (mask y*s+t > 0)
  float *part, *part2;  // [P][2][N]
  int Hi, Wi, Ci;
  int Ho, Wo, N;
  int R, S, stride, pad;
  int Kw;               // weight row pitch (elements)
  int K;                // GEMM K of class 0 (fwd) ; dgrad: per class ntap * Ci
  int Mc;               // GEMM rows per class
  int Hc, Wc;           // dgrad: class image (Ho / st, Wo / st); fwd: Ho, Wo
  int nmt;              // M tiles per class
  int Nb;               // images (operand extents for the buffer descriptors)
  int bn_rep;           // BN-statistics replica rows (g_bn_rep): P = ncls * nmt partial rows are
                        // added atomically into min(P, bn_rep) rows of a zeroed accumulator;
                        // bn_rep >= P (deterministic mode): one plainly stored row per tile
  const float *fbias;   // FOLD: per-output-channel bias added to the accumulators (conv_glds)
  int ntap[4];
  signed char tr[4][9], ts[4][9], tdh[4][9], tdw[4][9];
  int tapx[4][9];       // the same taps packed per dword (dh | dw << 8 | (tr * S + ts) << 16):
                        // a wave-uniform index then reads them with scalar loads
};

// 16x16x32 bf16 MFMA on raw 8 x bf16 fragments
PG_DEVICE f32x4_t mfma16(const s16x8_t &a, const s16x8_t &b, const f32x4_t &c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

PG_DEVICE float reluf(float x) { return fmaxf(x, 0.f); }

// load 8 floats (two float4) of a per-channel vector
PG_DEVICE void ld8f(const float *p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// Lazy BN finalize (bnfin.h bn_lazy) of channels [0, C) into LDS, sm[q*C + c] = parameter q
// (forward: scale, shift; backward: a, b, c).  Every workgroup reduces the <= 8 replica rows
// of the producer itself instead of waiting for a finalize launch between the two kernels;
// the caller synchronises the workgroup before reading sm.
// (bnfin.h bn_stage_params: loads batched 4 chunks of 256 channels at a time)
PG_DEVICE void lz_stage(const BnFin *d, float *sm, int C, int npar) {
  if (npar == 3) bn_stage_params<3, 4>(d, nullptr, nullptr, nullptr, C, C, sm);
  else bn_stage_params<2, 4>(d, nullptr, nullptr, nullptr, C, C, sm);
}
}  // namespace

// ===========================================================================
// forward / dgrad implicit GEMM
// ===========================================================================
// Epilogue shared by the register-staged and the LDS-DMA implicit-GEMM kernels: the bf16 C
// tile goes through LDS (smem, free after the K loop), then 16-B row chunks with the fused
// backward operands and the BN partial sums of the tile's columns.
template <int MODE, int EPI, int BM, int BN>
PG_DEVICE void conv_epilogue(const ConvArgs &p, f32x4_t (&acc)[BM / 32][BN / 32], char *smem, int m0, int n0,
                             int mt, int cls, int ph, int pw) {
  constexpr int RT = BM / 32, CTW = BN / 32;
  constexpr int LDC = BN + 8;
  constexpr int CH = BN / 8, RSTEP = 256 / CH, NP = BM / RSTEP;
  bf16_t *Cs = reinterpret_cast<bf16_t *>(smem);     // [BM][LDC]
  float *Red = reinterpret_cast<float *>(smem);      // [RSTEP][BN] (end)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nmt = p.nmt;
  const int HWc = p.Hc * p.Wc;
  // bf16 C tile in LDS, then 16-B row chunks.  The epilogue operands of the
  // first EB rows are loaded before the C tile is staged; rows past the end are clamped to
  // a valid row (loads are unconditional, results discarded) so hipcc keeps them in flight.
  constexpr bool E_XM = EPI == CE_BWD_RXYM || EPI == CE_BWD_RXYYM;
  constexpr bool E_R = EPI == CE_BWD_R || EPI == CE_BWD_RXY || EPI == CE_BWD_RXYY || E_XM;
  constexpr bool E_X = EPI == CE_BWD_RXY || EPI == CE_BWD_RXYY;
  constexpr bool E_YT = EPI == CE_BWD_RELU || EPI == CE_BWD_RXY || EPI == CE_BWD_RXYY || E_XM;
  constexpr bool E_YT2 = EPI == CE_BWD_RXYY || EPI == CE_BWD_RXYYM;
  constexpr bool STATS = EPI == CE_FWD || E_YT;
  constexpr int EB = NP < 4 ? NP : 4;
  const int my_chunk = tid % CH;
  const bool colok = n0 + my_chunk * 8 < p.N;
  const int ncol0 = colok ? n0 + my_chunk * 8 : 0;
  float s0[8], s1[8], s2[8], es[8], et[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = s2[j] = 0.f;
  if constexpr (EPI == CE_BWD_RELU) {
    ld8f(p.es + ncol0, es);
    ld8f(p.et + ncol0, et);
  }
  uint4 oy[EB], orr[EB], ox[EB], oy2[EB];
  uint32_t oxm[EB];
  size_t offs[EB];
  bool okr[EB];
  auto issue = [&](int i0) {
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int rr = tid / CH + (i0 + e) * RSTEP;
      int m = m0 + rr;
      okr[e] = m < p.Mc && colok;
      if (m >= p.Mc) m = p.Mc - 1;
      size_t pix;
      if constexpr (MODE == CM_FWD) {
        pix = m;
      } else {
        const int b = m / HWc, rem = m % HWc, hh = rem / p.Wc, ww = rem % p.Wc;
        pix = ((size_t)b * p.Ho + hh * p.stride + ph) * p.Wo + ww * p.stride + pw;
      }
      offs[e] = pix * p.N + ncol0;
      if constexpr (E_YT) oy[e] = ldg16(p.Yt + offs[e]);
      if constexpr (E_R) orr[e] = ldg16(p.Rg + offs[e]);
      if constexpr (E_X) ox[e] = ldg16(p.X + offs[e]);
      if constexpr (E_XM) oxm[e] = p.Xm[offs[e] >> 3];   // ncol0 % 8 == 0: one byte per 8 channels
      if constexpr (E_YT2) oy2[e] = ldg16(p.Yt2 + offs[e]);
    }
  };
  issue(0);
  // C tile to LDS as 4-byte column pairs (common.h frag_store_bf16)
#pragma unroll
  for (int c = 0; c < CTW; ++c)
#pragma unroll
    for (int r = 0; r < RT; ++r)
      frag_store_bf16(Cs, LDC, wm * (BM / 2) + r * 16, wn * (BN / 2) + c * 16, acc[r][c][0], acc[r][c][1],
                      acc[r][c][2], acc[r][c][3]);
  __syncthreads();
#pragma unroll
  for (int i0 = 0; i0 < NP; i0 += EB) {
    if (i0 > 0) issue(i0);
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int rr = tid / CH + (i0 + e) * RSTEP;
      float v[8];
      unpack8(*reinterpret_cast<const uint4 *>(Cs + rr * LDC + my_chunk * 8), v);
      if constexpr (EPI == CE_FWD) {
        if (okr[e]) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { s0[j] += v[j]; s1[j] = fmaf(v[j], v[j], s1[j]); }
        }
      } else {
        float yt[8];
        if constexpr (E_YT) unpack8(oy[e], yt);
        if constexpr (EPI == CE_BWD_RELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaf(yt[j], es[j], et[j]) > 0.f ? v[j] : 0.f;
        }
        if constexpr (E_R) {
          float rv[8];
          unpack8(orr[e], rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += rv[j];
        }
        if constexpr (E_X) {
          float xv[8];
          unpack8(ox[e], xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = xv[j] > 0.f ? v[j] : 0.f;
        }
        if constexpr (E_XM) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (oxm[e] >> j) & 1u ? v[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j]));
        if (okr[e]) {
          if constexpr (E_YT) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { s0[j] += v[j]; s1[j] = fmaf(v[j], yt[j], s1[j]); }
          }
          if constexpr (E_YT2) {
            float y2[8];
            unpack8(oy2[e], y2);
#pragma unroll
            for (int j = 0; j < 8; ++j) s2[j] = fmaf(v[j], y2[j], s2[j]);
          }
        }
      }
      if (okr[e]) stg16(p.out + offs[e], pack8(v));
    }
  }
  if constexpr (!STATS) return;
  const bool has_yt2 = E_YT2;
  __syncthreads();
  // ---- BN partials of this tile's columns -> row cls*nmt + mt of part[P][2][N] (and part2):
  // stored, or added into replica row (cls*nmt + mt) % bn_rep (bn_part_add) when bn_rep < P
  const int prow = cls * nmt + mt;
  const int P = (int)gridDim.y * nmt;
  const bool rows_own = p.bn_rep >= P;
  const int nstat = has_yt2 ? 3 : 2;
  auto put = [&](float *dst, int s, int col, float a) {
    if (rows_own) dst[((size_t)prow * 2 + s) * p.N + col] = a;
    else bn_part_add(dst, prow, P, p.bn_rep, p.N, s, col, a);
  };
  for (int s = 0; s < nstat; ++s) {
    const int rgrp = tid / CH;
#pragma unroll
    for (int j = 0; j < 8; ++j) Red[rgrp * BN + my_chunk * 8 + j] = s == 0 ? s0[j] : (s == 1 ? s1[j] : s2[j]);
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      float a = 0.f;
      for (int g = 0; g < RSTEP; ++g) a += Red[g * BN + c];
      if (n0 + c < p.N) {
        if (s < 2) put(p.part, s, n0 + c, a);
        if (s == 0 && has_yt2) put(p.part2, 0, n0 + c, a);
        if (s == 2) put(p.part2, 1, n0 + c, a);
      }
    }
    __syncthreads();
  }
}

// CV: channels per gathered chunk (8 = one 16-B load; 4 = the 4-channel padded stem input,
// one 8-B load per chunk).  UT: Ci % KSTEP == 0 (uniform tap per k-step).
template <int MODE, int PRO, int EPI, int BM, int BN, int KSTEP, int CV, bool UT>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs p) {
  static_assert(CV == 8 || (CV == 4 && PRO == CP_NONE && MODE == CM_FWD), "4-channel chunks: stem forward only");
  constexpr int kLDK = KSTEP + 8;                    // staged row pitch (bf16): 16-B pad
  constexpr int KCH = KSTEP / CV;                    // chunks per staged row
  constexpr int RT = BM / 32, CTW = BN / 32;         // per-wave 16x16 tiles
  constexpr int ACH = BM * KCH / 256, BCH = BN * KCH / 256;
  constexpr bool HAS_A2 = PRO == CP_BNBWD;
  static_assert(ACH >= 1 && BCH >= 1 && BM >= 256 / (BN / 8), "tile too small for 256 threads");
  typedef typename std::conditional<CV == 8, uint4, uint2>::type chunk_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t *As = reinterpret_cast<bf16_t *>(smem);     // [2][BM][kLDK]
  bf16_t *Bs = As + 2 * BM * kLDK;                   // [2][BN][kLDK]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int NT = (p.N + BN - 1) / BN;
  const int nmt = p.nmt;
  // workgroup -> (class, mt, nt): N tiles of one M tile 8 ids apart
  const int cls = MODE == CM_DGRAD ? blockIdx.y : 0;
  int mt, nt;
  {
    const int L = blockIdx.x, full = (nmt / 8) * 8 * NT;
    if (L < full) {
      mt = (L / (8 * NT)) * 8 + L % 8;
      nt = (L / 8) % NT;
    } else {
      const int rem = nmt % 8, Lr = L - full;
      mt = (nmt / 8) * 8 + Lr % rem;
      nt = Lr / rem;
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int ph = MODE == CM_DGRAD ? cls / p.stride : 0, pw = MODE == CM_DGRAD ? cls % p.stride : 0;
  const int Kc = MODE == CM_DGRAD ? p.ntap[cls] * p.Ci : p.K;
  const int nk = (Kc + KSTEP - 1) / KSTEP;
  const int HWc = p.Hc * p.Wc;

  // ---- per-chunk row state (rows are fixed across k-steps)
  int rb[ACH], rh[ACH], rw[ACH];     // image index, base h, base w; rb < 0: row out of range
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int c = tid + i * 256, row = c / KCH;
    const int m = m0 + row;
    if (m < p.Mc) {
      const int b = m / HWc, rem = m % HWc, hh = rem / p.Wc, ww = rem % p.Wc;
      rb[i] = b;
      if constexpr (MODE == CM_FWD) {
        rh[i] = hh * p.stride - p.pad;
        rw[i] = ww * p.stride - p.pad;
      } else {
        rh[i] = hh;
        rw[i] = ww;
      }
    } else {
      rb[i] = -1; rh[i] = 0; rw[i] = 0;
    }
  }

  struct Stage {
    chunk_t ra[ACH], ry[HAS_A2 ? ACH : 1], rbw[BCH];
    bool va[ACH];
  };
  Stage S0;
  float pa8[8], pb8[8], pc8[8];
  // tap of a k offset: (dh, dw, weight tap index)
  auto tap_of = [&](int j, int &dh, int &dw, int &wt) {
    if constexpr (MODE == CM_FWD) {
      const int r = j / p.S, s = j - r * p.S;
      dh = r; dw = s; wt = j;
    } else {
      dh = p.tdh[cls][j]; dw = p.tdw[cls][j];
      wt = p.tr[cls][j] * p.S + p.ts[cls][j];
    }
  };
  auto load = [&](Stage &st, int k0) {
    int u_dh = 0, u_dw = 0, u_wt = 0, u_c0 = 0;
    if constexpr (UT) {
      const int j = k0 / p.Ci;
      u_c0 = k0 - j * p.Ci;
      tap_of(j, u_dh, u_dw, u_wt);
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, kk = (c % KCH) * CV;
      int dh, dw, ci;
      bool ok = rb[i] >= 0 && k0 + kk < Kc;
      if constexpr (UT) {
        dh = u_dh; dw = u_dw; ci = u_c0 + kk;
      } else {
        const int k = k0 + kk, j = k / p.Ci;
        int wt;
        ci = k - j * p.Ci;
        if (MODE == CM_FWD && j >= p.R * p.S) ok = false;
        tap_of(ok ? j : 0, dh, dw, wt);
      }
      const int ih = rh[i] + dh, iw = rw[i] + dw;
      ok = ok && ih >= 0 && ih < p.Hi && iw >= 0 && iw < p.Wi;
      st.va[i] = ok;
      const size_t off = (((size_t)rb[i] * p.Hi + ih) * p.Wi + iw) * p.Ci + ci;
      if constexpr (CV == 8) {
        st.ra[i] = ok ? ldg16(p.A + off) : make_uint4(0, 0, 0, 0);
        if constexpr (HAS_A2) st.ry[i] = ok ? ldg16(p.A2 + off) : make_uint4(0, 0, 0, 0);
      } else {
        st.ra[i] = ok ? *reinterpret_cast<const uint2 *>(p.A + off) : make_uint2(0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, n = c / KCH, kk = (c % KCH) * CV;
      const int gn = n0 + n, k = k0 + kk;
      bool ok = gn < p.N && k < Kc;
      size_t off;
      if constexpr (MODE == CM_FWD) {
        off = (size_t)gn * p.Kw + k;
        if constexpr (CV == 4) ok = ok && k < p.Kw;
      } else {
        int dh, dw, wt, ci;
        if constexpr (UT) { dh = u_dh; dw = u_dw; wt = u_wt; ci = u_c0 + kk; }
        else { const int j = k / p.Ci; ci = k - j * p.Ci; tap_of(ok ? j : 0, dh, dw, wt); }
        off = (size_t)gn * p.Kw + (size_t)wt * p.Ci + ci;
      }
      if constexpr (CV == 8) st.rbw[i] = ok ? ldg16(p.W + off) : make_uint4(0, 0, 0, 0);
      else st.rbw[i] = ok ? *reinterpret_cast<const uint2 *>(p.W + off) : make_uint2(0, 0);
    }
  };
  // per-channel prologue parameters of the k-step written next (every chunk of this thread
  // sits at the same kk, ACH rows apart -> one parameter set)
  auto load_par = [&](int k0) {
    if constexpr (PRO != CP_NONE) {
      const int kk = (tid % KCH) * CV;
      int ci;
      if constexpr (UT) ci = k0 % p.Ci + kk;
      else ci = (k0 + kk) % p.Ci;
      ld8f(p.pa + ci, pa8);
      ld8f(p.pb + ci, pb8);
      if constexpr (PRO == CP_BNBWD) ld8f(p.pc + ci, pc8);
    }
  };
  auto write = [&](Stage &st, int buf) {
    bf16_t *Ab = As + buf * BM * kLDK;
    bf16_t *Bb = Bs + buf * BN * kLDK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, row = c / KCH, kk = (c % KCH) * CV;
      if constexpr (CV == 8) {
        uint4 v = st.ra[i];
        if constexpr (PRO != CP_NONE) {
          float x[8];
          unpack8(st.ra[i], x);
          if constexpr (PRO == CP_BNBWD) {
            float y[8];
            unpack8(st.ry[i], y);
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = fmaf(pa8[j], x[j], fmaf(pb8[j], y[j], pc8[j]));
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = reluf(fmaf(x[j], pa8[j], pb8[j]));
          }
          if (!st.va[i]) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
          }
          v = pack8(x);
        }
        *reinterpret_cast<uint4 *>(Ab + row * kLDK + kk) = v;
      } else {
        *reinterpret_cast<uint2 *>(Ab + row * kLDK + kk) = st.ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, n = c / KCH, kk = (c % KCH) * CV;
      if constexpr (CV == 8) *reinterpret_cast<uint4 *>(Bb + n * kLDK + kk) = st.rbw[i];
      else *reinterpret_cast<uint2 *>(Bb + n * kLDK + kk) = st.rbw[i];
    }
  };

  f32x4_t acc[RT][CTW];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CTW; ++c) acc[r][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int buf) {
    const bf16_t *Ab = As + buf * BM * kLDK;
    const bf16_t *Bb = Bs + buf * BN * kLDK;
#pragma unroll
    for (int sub = 0; sub < KSTEP / 32; ++sub) {
      s16x8_t af[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r)
        af[r] = *reinterpret_cast<const s16x8_t *>(Ab + (wm * (BM / 2) + r * 16 + (lane & 15)) * kLDK + sub * 32 +
                                                   8 * (lane >> 4));
#pragma unroll
      for (int c = 0; c < CTW; ++c) {
        const s16x8_t bf = *reinterpret_cast<const s16x8_t *>(Bb + (wn * (BN / 2) + c * 16 + (lane & 15)) * kLDK +
                                                              sub * 32 + 8 * (lane >> 4));
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r][c] = mfma16(af[r], bf, acc[r][c]);
      }
    }
  };

  // one register stage: the loads of step k+1 are in flight during the MFMAs of step k (a
  // two-stage variant -- loads two steps ahead -- measured slower on MI355X: it needs ~400
  // registers for the 128 x 128 tile, i.e. one wave per SIMD)
  if (nk > 0) {
    load(S0, 0);
    load_par(0);
    write(S0, 0);
  }
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) {
      load_par((ks + 1) * KSTEP);
      load(S0, (ks + 1) * KSTEP);
    }
    mma(buf);
    if (ks + 1 < nk) write(S0, buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<MODE, EPI, BM, BN>(p, acc, smem, m0, n0, mt, cls, ph, pw);
}

// ===========================================================================
// LDS-DMA implicit GEMM (operands already materialised: no prologue).  Both operand tiles are
// streamed global -> LDS by buffer_load_dwordx4 ... lds, so the staging costs no VGPRs, no
// ds_write and no per-element VALU (the register-staged kernel above spends ~40 VALU per 16-B
// chunk on its BN prologue and address math, and is issue-bound on MI355X).  Requires
// Ci % 64 == 0: a 64-wide k-step lies inside one filter tap.
//   * one wave-instruction fills a 1-KiB piece = 8 staged rows x 128 B, lane-linear in LDS;
//     lane l loads k-chunk (l & 7) ^ (l >> 3) of row l >> 3 (XOR swizzle on the SOURCE
//     address), so the ds_read_b128 fragment reads are bank-conflict free;
//   * zero padding and rows past M / N come from the descriptor range check (offset kOOB);
//   * NBUF = 2: two barriers per k-step (wait for this step's DMAs, then for every wave's reads
//     before the buffer is refilled); NBUF = 3: one barrier per k-step, the DMA two steps ahead
//     stays in flight across it (counted vmcnt + raw s_barrier, never __syncthreads()).
// ===========================================================================
template <int N>
PG_DEVICE void glds_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// KS = 32 (64-B staged rows, 16 rows per piece): half the LDS per stage, so twice the
// workgroups per CU at the same ring depth -- the 64-wide loop is latency-bound at two
// workgroups per CU (PMC: 34 % of wave cycles parked at s_waitcnt / s_barrier).  Chunk kc of
// row r sits at kc ^ f(r), f(r) = (4 - ((r >> 2) & 3)) & 3: the four rows of a 16-lane
// ds_read_b128 group that share a bank window get distinct chunk slots.
template <int KS>
PG_DEVICE int glds_sw(int r) {
  if constexpr (KS == 64) return r & 7;
  else return (4 - ((r >> 2) & 3)) & 3;
}

// MT (multi-tap k-steps, Ci < KS, e.g. the space-to-depth stem with Ci = 16): the 8 chunks of a
// staged 128-B row belong to different filter taps, so each lane decodes its own chunk's tap
// (an integer division per k-step) and the bounds check is per chunk.  Without MT the tap is
// uniform per k-step (Ci % KS == 0).
// FOLD (1x1 data gradient with this layer's BN backward folded into the GEMM, see
// launch_conv_dgrad_fold): tap 0 streams G and tap 1 streams Y as the A operand (K = 2 Cout,
// B = [a.W | b.W]), and the epilogue adds the per-channel term fbias.
template <int MODE, int EPI, int BM, int BN, int NBUF, int KS = 64, bool MT = false, bool FOLD = false>
__global__ __launch_bounds__(256) void conv_glds_kernel(ConvArgs p) {
  constexpr int ROWB = KS * 2;                        // staged row bytes
  constexpr int RPP = 1024 / ROWB, CPR = ROWB / 16;   // rows per 1-KiB piece, 16-B chunks per row
  constexpr int APW = BM / RPP / 4, BPW = BN / RPP / 4;   // pieces per wave per k-step
  constexpr int PW = APW + BPW;
  constexpr int RT = BM / 32, CTW = BN / 32;
  constexpr int ABYTES = BM * ROWB, BUFB = (BM + BN) * ROWB;
  static_assert(NBUF >= 2 && NBUF <= 4, "2 to 4 LDS buffers");
  static_assert(KS == 32 || KS == 64, "k-step 32 or 64");
  static_assert(APW >= 1 && BPW >= 1, "whole pieces per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int NT = (p.N + BN - 1) / BN;
  const int nmt = p.nmt;
  const int cls = MODE == CM_DGRAD ? blockIdx.y : 0;
  int mt, nt;
  {
    const int L = blockIdx.x, full = (nmt / 8) * 8 * NT;
    if (L < full) {
      mt = (L / (8 * NT)) * 8 + L % 8;
      nt = (L / 8) % NT;
    } else {
      const int rem = nmt % 8, Lr = L - full;
      mt = (nmt / 8) * 8 + Lr % rem;
      nt = Lr / rem;
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int ph = MODE == CM_DGRAD ? cls / p.stride : 0, pw = MODE == CM_DGRAD ? cls % p.stride : 0;
  const int Kc = MODE == CM_DGRAD ? p.ntap[cls] * p.Ci : p.K;
  const int nk = Kc / KS;
  const int HWc = p.Hc * p.Wc;
  const int lrow = lane / CPR;                          // row of this lane inside a 1-KiB piece
  const int lch = (lane % CPR) ^ glds_sw<KS>(lrow);     // k-chunk this lane fetches (source swizzle)
  // raw descriptors for the inline-asm DMA (common.h lds_dma16)
  const u32x4_t ra = make_srd(p.A, (uint32_t)p.Nb * p.Hi * p.Wi * p.Ci * 2);
  const u32x4_t ra2 = make_srd(FOLD ? p.A2 : p.A, (uint32_t)p.Nb * p.Hi * p.Wi * p.Ci * 2);
  const u32x4_t rw = make_srd(p.W, (uint32_t)p.N * p.Kw * 2);

  // A rows of this wave's pieces (fixed across k-steps): image, base h / w; rb < 0: past M
  int rb[APW], rh[APW], rwc[APW];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int m = m0 + (wave * APW + i) * RPP + lrow;
    if (m < p.Mc) {
      const int b = m / HWc, rem = m % HWc, hh = rem / p.Wc, ww = rem % p.Wc;
      rb[i] = b;
      rh[i] = MODE == CM_FWD ? hh * p.stride - p.pad : hh;
      rwc[i] = MODE == CM_FWD ? ww * p.stride - p.pad : ww;
    } else {
      rb[i] = -1; rh[i] = 0; rwc[i] = 0;
    }
  }
  uint32_t wrow[BPW];   // weight row byte offsets (kOOB past N)
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int n = n0 + (wave * BPW + i) * RPP + lrow;
    wrow[i] = n < p.N ? (uint32_t)n * p.Kw * 2 : kOOB;
  }

  auto issue = [&](int ks, int buf) {
    const int k0 = ks * KS;
    int j, ci;
    if constexpr (MT) {
      const int kk = k0 + lch * 8;
      j = kk / p.Ci;
      ci = kk - j * p.Ci;
    } else {
      j = k0 / p.Ci;
      ci = k0 - j * p.Ci + lch * 8;
    }
    int dh, dw, wt;
    if constexpr (MODE == CM_FWD) {
      dh = j / p.S; dw = j - dh * p.S; wt = j;
    } else if constexpr (!MT) {
      // j is wave-uniform here: as a scalar the tap tables are read by scalar loads from the
      // kernel arguments (lgkmcnt), not by per-lane global loads whose vmcnt wait each k-step
      // also waited for the DMAs in flight (and put the table latency on every step's path)
      const int v = p.tapx[cls][__builtin_amdgcn_readfirstlane(j)];
      dh = (int)(signed char)(v & 0xff);
      dw = (int)(signed char)((v >> 8) & 0xff);
      wt = v >> 16;
    } else {
      dh = p.tdh[cls][j]; dw = p.tdw[cls][j];
      wt = p.tr[cls][j] * p.S + p.ts[cls][j];
    }
    char *abase = smem + buf * BUFB;
    char *bbase = abase + ABYTES;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int ih = rh[i] + dh, iw = rwc[i] + dw;
      const bool ok = rb[i] >= 0 && ih >= 0 && ih < p.Hi && iw >= 0 && iw < p.Wi;
      const uint32_t off = ok ? (uint32_t)((((rb[i] * p.Hi + ih) * p.Wi + iw) * p.Ci + ci) * 2) : kOOB;
      if (FOLD && wt) lds_dma16(ra2, abase + (wave * APW + i) * 1024, off);   // (wt: wave-uniform)
      else lds_dma16(ra, abase + (wave * APW + i) * 1024, off);
    }
    const uint32_t kb = (uint32_t)(wt * p.Ci + ci) * 2;
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      const uint32_t off = wrow[i] == kOOB ? kOOB : wrow[i] + kb;
      lds_dma16(rw, bbase + (wave * BPW + i) * 1024, off);
    }
  };

  f32x4_t acc[RT][CTW];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CTW; ++c) acc[r][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // fragment reads: row (lane & 15) of a 16-row block, k-chunk kc = 4*sub + (lane >> 4) stored at
  // position kc ^ glds_sw(row) (16-row blocks start at multiples of every swizzle period)
  const int fsw = glds_sw<KS>(lane & 15);
  auto mma = [&](int buf) {
    const char *Ab = smem + buf * BUFB;
    const char *Bb = Ab + ABYTES;
#pragma unroll
    for (int sub = 0; sub < KS / 32; ++sub) {
      const int pos = ((4 * sub + (lane >> 4)) ^ fsw) * 16;
      s16x8_t af[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r)
        af[r] = *reinterpret_cast<const s16x8_t *>(Ab + (wm * (BM / 2) + r * 16 + (lane & 15)) * ROWB + pos);
#pragma unroll
      for (int c = 0; c < CTW; ++c) {
        const s16x8_t bf =
            *reinterpret_cast<const s16x8_t *>(Bb + (wn * (BN / 2) + c * 16 + (lane & 15)) * ROWB + pos);
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r][c] = mfma16(af[r], bf, acc[r][c]);
      }
    }
  };

  if constexpr (NBUF == 2) {
    if (nk > 0) issue(0, 0);
    for (int ks = 0; ks < nk; ++ks) {
      const int buf = ks & 1;
      if (ks + 1 < nk) {
        issue(ks + 1, buf ^ 1);
        glds_wait_barrier<PW>();        // this step's pieces landed (every wave)
      } else {
        glds_wait_barrier<0>();
      }
      mma(buf);
      glds_wait_barrier<PW>();          // every wave done reading buf before it is refilled
    }
  } else {
    // ring: NBUF - 1 stages in flight; one barrier per k-step (stage ks landed everywhere AND
    // every wave is done with stage ks - 1, whose buffer the next issue refills)
#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
      if (s < nk) issue(s, s);
    int buf = 0, nbuf = NBUF - 1;
    for (int ks = 0; ks < nk; ++ks) {
      if (ks + NBUF - 2 < nk) glds_wait_barrier<(NBUF - 2) * PW>();
      else if (NBUF == 4 && ks + 1 < nk) glds_wait_barrier<PW>();
      else glds_wait_barrier<0>();
      if (ks + NBUF - 1 < nk) issue(ks + NBUF - 1, nbuf);
      mma(buf);
      buf = buf == NBUF - 1 ? 0 : buf + 1;
      nbuf = nbuf == NBUF - 1 ? 0 : nbuf + 1;
    }
    glds_wait_barrier<0>();             // every wave done reading before the C tile reuses LDS
  }
  if constexpr (FOLD) {   // acc[r][c][j] = C[m][n], n = n0 + wn*BN/2 + 16c + (lane & 15)
#pragma unroll
    for (int c = 0; c < CTW; ++c) {
      const int n = n0 + wn * (BN / 2) + c * 16 + (lane & 15);
      const float bv = n < p.N ? p.fbias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][c][j] += bv;
    }
  }
  conv_epilogue<MODE, EPI, BM, BN>(p, acc, smem, m0, n0, mt, cls, ph, pw);
}

// ===========================================================================
// BN materialisation for the LDS-DMA convs (operands without a prologue), [M][C] bf16:
//   MODE 0: act = relu(Y*a + b)        (forward: the producer BN + ReLU, consumer input)
//   MODE 1: dy  = a*G + b*Y + c        (backward: this layer's BN backward, dgrad + wgrad input)
// Thread t owns channel chunk t % C8 (coefficients in registers), rows t / C8 + i*(256/C8);
// UR rows in flight per thread.  C8 = C/8 must divide 256 (checked by the launcher).
// ===========================================================================
// LZ: the coefficients come from the producer's replica rows (lz, lz_stage), not from a, b, c
template <int MODE, bool LZ>
__global__ __launch_bounds__(256) void bn_mat_kernel(const bf16_t *__restrict__ G, const bf16_t *__restrict__ Y,
                                                    const float *__restrict__ a, const float *__restrict__ b,
                                                    const float *__restrict__ c, bf16_t *__restrict__ out, int M,
                                                    int C, const BnFin *lz) {
  extern __shared__ __attribute__((aligned(16))) float lzs[];
  constexpr int UR = 4;
  const int C8 = C >> 3, rpi = 256 / C8;
  const int cc = threadIdx.x % C8, r0 = threadIdx.x / C8;
  float a8[8], b8[8], c8[8];
  if constexpr (LZ) {
    lz_stage(lz, lzs, C, MODE == 1 ? 3 : 2);
    __syncthreads();
    a = lzs; b = lzs + C; c = lzs + 2 * C;
  }
  ld8f(a + cc * 8, a8);
  ld8f(b + cc * 8, b8);
  if constexpr (MODE == 1) ld8f(c + cc * 8, c8);
  const rsrc_t ry = make_rsrc(Y, (uint32_t)M * C * 2), ro = make_rsrc(out, (uint32_t)M * C * 2);
  const rsrc_t rg = make_rsrc(MODE == 1 ? G : Y, (uint32_t)M * C * 2);
  const int stride = gridDim.x * rpi * UR;
  for (int m = blockIdx.x * rpi * UR + r0; m < M; m += stride) {
    uint4 yv[UR], gv[UR];
    uint32_t off[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int row = m + u * rpi;
      off[u] = row < M ? (uint32_t)(row * C + cc * 8) * 2 : kOOB;
      yv[u] = bld16(ry, off[u]);
      if constexpr (MODE == 1) gv[u] = bld16(rg, off[u]);
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      float y[8], v[8];
      unpack8(yv[u], y);
      if constexpr (MODE == 1) {
        float g[8];
        unpack8(gv[u], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(a8[j], g[j], fmaf(b8[j], y[j], c8[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = reluf(fmaf(y[j], a8[j], b8[j]));
      }
      bst16(ro, off[u], pack8(v));
    }
  }
}

// ===========================================================================
// weight gradient (split over m):  part[z][n][k] = sum_{m in split z} dy[m][n] * x[m][k]
//   dy = a[n]*G + b[n]*Y + c[n]      (this layer's BN backward)
//   x  = gather(X) at the forward taps, with ReLU(BN of the producer) (XPRO) or as stored
// ===========================================================================
namespace {
struct WgArgs {
  const bf16_t *G, *Y;
  const float *ga, *gb, *gc;
  const bf16_t *X;
  const float *xs, *xt;
  float *out;           // [nsplit][N][Kw]  (or the gradient itself when nsplit == 1)
  int N;                // output channels (dy channels)
  int Hi, Wi, Ci;       // x image
  int Ho, Wo;           // dy image
  int R, S, stride, pad;
  int Kw;               // R*S*Ci
  int M;                // Nb*Ho*Wo
  int rows_per_split;
};
constexpr int kWgMK = 64;             // m rows per step
constexpr int kWgLD = kWgMK + 8;      // transposed row pitch (bf16)
}  // namespace

template <int XPRO, int TN, int TK, int CV, bool DM>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgArgs p) {
  constexpr int QN = TN / 2, QK = TK / 2, RN = QN / 16, RK = QK / 16;
  constexpr int M4 = kWgMK / 4;
  constexpr int IDY = M4 * (TN / 8), IX = M4 * (TK / 8);   // items: 4 rows x 8 columns
  constexpr int PD = (IDY + 255) / 256, PX = (IX + 255) / 256;
  static_assert(IDY % 64 == 0 && IX % 64 == 0, "items are handed out in whole waves");
  __shared__ __attribute__((aligned(16))) bf16_t Tdy[2][TN * kWgLD];
  __shared__ __attribute__((aligned(16))) bf16_t Tx[2][TK * kWgLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * TN, k0 = blockIdx.y * TK;
  const int mbeg = blockIdx.z * p.rows_per_split;
  const int mend = min(p.M, mbeg + p.rows_per_split);
  const int HWo = p.Ho * p.Wo;
  // dy items on threads [0, IDY), x items start at thread IDY % 256 (whole waves either way)
  const int xtid = (tid + 256 - (IDY % 256)) % 256;

  // ---- dy items: fixed (m4, 8 output channels)
  int d_col[PD], d_m4[PD];
  bool d_on[PD];
  float ga8[PD][8], gb8[PD][8], gc8[PD][8];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int it = tid + i * 256;
    d_on[i] = it < IDY;
    d_m4[i] = it % M4;
    d_col[i] = n0 + (it / M4) * 8;
    const bool ok = d_on[i] && d_col[i] < p.N;
#pragma unroll
    for (int j = 0; j < 8; ++j) ga8[i][j] = gb8[i][j] = gc8[i][j] = 0.f;
    if (ok && !DM) {
      ld8f(p.ga + d_col[i], ga8[i]);
      ld8f(p.gb + d_col[i], gb8[i]);
      ld8f(p.gc + d_col[i], gc8[i]);
    }
  }
  // ---- x items: fixed (m4, 8 columns of k = (r, s, ci)); CV == 4: two taps of 4 channels
  constexpr int NH = CV == 8 ? 1 : 2;
  int x_col[PX], x_m4[PX], x_dh[PX][NH], x_dw[PX][NH], x_ci[PX][NH];
  bool x_on[PX], x_kok[PX][NH];
  float xs8[PX][8], xt8[PX][8];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int xi = xtid + i * 256;
    x_on[i] = xi < IX;
    x_m4[i] = xi % M4;
    const int k = k0 + (xi / M4) * 8;
    x_col[i] = k;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int kh = k + 4 * h;
      const int j = kh / p.Ci;
      x_kok[i][h] = x_on[i] && kh < p.Kw;
      x_ci[i][h] = kh - j * p.Ci;
      const int r = j / p.S;
      x_dh[i][h] = r - p.pad;
      x_dw[i][h] = j - r * p.S - p.pad;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xs8[i][j] = xt8[i][j] = 0.f;
    if constexpr (XPRO == CP_BN_RELU) {
      if (x_kok[i][0]) {
        ld8f(p.xs + x_ci[i][0], xs8[i]);
        ld8f(p.xt + x_ci[i][0], xt8[i]);
      }
    }
  }

  f32x4_t acc[RN][RK];
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 dg[PD][4], dyv[PD][4], xv[PX][4];
  uint32_t dvm[PD], xvm[PX];   // validity bits of the staged rows
  auto load_step = [&](int m0) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int mr = m0 + d_m4[i] * 4;
      const bool cok = d_on[i] && d_col[i] < p.N;
      dvm[i] = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = cok && mr + q < mend;
        dvm[i] |= ok ? 1u << q : 0u;
        const size_t off = (size_t)(mr + q) * p.N + d_col[i];
        dg[i][q] = ok ? ldg16(p.G + off) : make_uint4(0, 0, 0, 0);
        if constexpr (!DM) dyv[i][q] = ok ? ldg16(p.Y + off) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      int m = m0 + x_m4[i] * 4;
      int b = m / HWo, rem = m - b * HWo, oh = rem / p.Wo, ow = rem - oh * p.Wo;
      xvm[i] = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool mok = x_on[i] && m < mend;
        const int bh = oh * p.stride, bw = ow * p.stride;
        if constexpr (CV == 8) {
          const int ih = bh + x_dh[i][0], iw = bw + x_dw[i][0];
          const bool ok = mok && x_kok[i][0] && ih >= 0 && ih < p.Hi && iw >= 0 && iw < p.Wi;
          xvm[i] |= ok ? 1u << q : 0u;
          xv[i][q] = ok ? ldg16(p.X + (((size_t)b * p.Hi + ih) * p.Wi + iw) * p.Ci + x_ci[i][0])
                        : make_uint4(0, 0, 0, 0);
        } else {
          uint2 h2[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int ih = bh + x_dh[i][h], iw = bw + x_dw[i][h];
            const bool ok = mok && x_kok[i][h] && ih >= 0 && ih < p.Hi && iw >= 0 && iw < p.Wi;
            h2[h] = ok ? *reinterpret_cast<const uint2 *>(p.X + (((size_t)b * p.Hi + ih) * p.Wi + iw) * p.Ci +
                                                          x_ci[i][h])
                       : make_uint2(0, 0);
          }
          xv[i][q] = make_uint4(h2[0].x, h2[0].y, h2[1].x, h2[1].y);
        }
        ++m; ++ow;
        if (ow == p.Wo) { ow = 0; ++oh; if (oh == p.Ho) { oh = 0; ++b; } }
      }
    }
  };
  // 4 rows x 8 columns -> T[col][m] (8 x ds_write_b64)
  auto put = [&](bf16_t *T, int tcol, int tm, const float (&v)[4][8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint2 w;
      w.x = pack2(v[0][j], v[1][j]);
      w.y = pack2(v[2][j], v[3][j]);
      *reinterpret_cast<uint2 *>(T + (tcol + j) * kWgLD + tm) = w;
    }
  };
  auto write_step = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      if (!d_on[i]) continue;
      float v[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float g[8], y[8];
        unpack8(dg[i][q], g);
        if constexpr (DM) {   // materialised dy (invalid rows were loaded as zeros)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] = g[j];
        } else {
          unpack8(dyv[i][q], y);
          const bool ok = (dvm[i] >> q) & 1u;   // a*0 + b*0 + c != 0: invalid rows must be zeroed
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] = ok ? fmaf(ga8[i][j], g[j], fmaf(gb8[i][j], y[j], gc8[i][j])) : 0.f;
        }
      }
      put(Tdy[buf], d_col[i] - n0, d_m4[i] * 4, v);
    }
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      if (!x_on[i]) continue;
      float v[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        unpack8(xv[i][q], v[q]);
        if constexpr (XPRO == CP_BN_RELU) {
          const bool ok = (xvm[i] >> q) & 1u;   // padding stays zero (not relu(shift))
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] = ok ? reluf(fmaf(v[q][j], xs8[i][j], xt8[i][j])) : 0.f;
        }
      }
      put(Tx[buf], x_col[i] - k0, x_m4[i] * 4, v);
    }
  };

  int buf = 0;
  if (mbeg < mend) {
    load_step(mbeg);
    write_step(0);
  }
  __syncthreads();
  for (int m0 = mbeg; m0 < mend; m0 += kWgMK) {
    const bool has_next = m0 + kWgMK < mend;
    if (has_next) load_step(m0 + kWgMK);
    const bf16_t *Td = Tdy[buf], *Tq = Tx[buf];
#pragma unroll
    for (int sub = 0; sub < kWgMK / 32; ++sub) {
      s16x8_t af[RN], bfr[RK];
#pragma unroll
      for (int a = 0; a < RN; ++a)
        af[a] = *reinterpret_cast<const s16x8_t *>(Td + (wn * QN + a * 16 + (lane & 15)) * kWgLD + sub * 32 +
                                                   8 * (lane >> 4));
#pragma unroll
      for (int b = 0; b < RK; ++b)
        bfr[b] = *reinterpret_cast<const s16x8_t *>(Tq + (wk * QK + b * 16 + (lane & 15)) * kWgLD + sub * 32 +
                                                    8 * (lane >> 4));
#pragma unroll
      for (int a = 0; a < RN; ++a)
#pragma unroll
        for (int b = 0; b < RK; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
    if (has_next) write_step(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float *dst = p.out + (size_t)blockIdx.z * p.N * p.Kw;
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * QN + a * 16 + 4 * (lane >> 4) + j;
        const int k = k0 + wk * QK + b * 16 + (lane & 15);
        if (n < p.N && k < p.Kw) dst[(size_t)n * p.Kw + k] = acc[a][b][j];
      }
}

// ===========================================================================
// weight gradient on LDS-DMA operands (materialised dy, x without a prologue):
//   part[z][n][k] = sum_{m in split z} dy[m][n] x[m][k]
// Both operand tiles are streamed global -> LDS by buffer_load ... lds in their stored
// (m-major) layout: a stage is 64 rows of dy [TN cols] and 64 gathered rows of x [TK cols of
// one filter tap], 16-B chunks placed at chunk ^ 2*sw(row) (the swizzle is applied on the
// source side: lane q of a row fetches chunk q ^ 2*sw(row)).  The MFMA operands are the
// transposes (dy^T: n x m, x^T: k x m), read with the gfx950 transposing ds_read_b64_tr_b16:
// a 16-lane group addresses 4 rows x 16 columns and every lane receives one column; rows
// 8g .. 8g+3 of the two lane halves land in 8 distinct 32-B bank windows under the swizzle
// (conflict-free).  No register staging, no ds_write: the former transposing stores of
// conv_wgrad_kernel cost more LDS cycles than its MFMAs.  NBUF-deep stage ring as in
// conv_glds_kernel; 1-D grid remapped so the workgroups of one m split share an XCD (its L2
// holds the split's rows once for all (n, k) tiles).
// ===========================================================================
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

namespace {
// pair-level swizzle of row r for rows of RB bytes (see above)
template <int RB>
PG_DEVICE int wg_sw(int r) {
  if constexpr (RB == 256) return (r & 3) | (((r >> 3) & 1) << 2);
  else return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
}
// q = n / d for 0 <= n < 2^24 (float reciprocal + one correction step each way)
PG_DEVICE int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  if (q * d > n) --q;
  else if ((q + 1) * d <= n) ++q;
  return q;
}
}  // namespace

// MK: m rows per stage (64, or 32 for a deeper ring in the same LDS: with 4 stages of 32 rows
// three stages are in flight instead of one, for the latency-bound splits with few MFMAs per
// stage); NBUF: ring depth (2..4, one barrier per stage from 3 on)
template <int TN, int TK, int NBUF, int MK = 64>
__global__ __launch_bounds__(256) void conv_wgrad_dma_kernel(WgArgs p, int gx, int gy, int total) {
  static_assert(MK == 32 || MK == 64, "32- or 64-row stages");
  static_assert(NBUF >= 2 && NBUF <= 4, "2 to 4 stages");
  constexpr int RBN = TN * 2, RBK = TK * 2;              // staged row bytes
  constexpr int CPN = RBN / 16, CPK = RBK / 16;          // 16-B chunks per row
  constexpr int PN = MK * RBN / 1024, PK = MK * RBK / 1024;   // 1-KiB pieces per stage
  constexpr int PNW = PN / 4, PKW = PK / 4, PW = PNW + PKW;   // per wave
  constexpr int DBYTES = MK * RBN, SBYTES = MK * (RBN + RBK);
  constexpr int QN = TN / 2, QK = TK / 2, RN = QN / 16, RK = QK / 16;
  static_assert(PN % 4 == 0 && PK % 4 == 0, "whole pieces per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  // XCD-aware tile order: hardware ids go round-robin over the 8 XCDs; logical ids of one XCD
  // are contiguous, and a split's (n, k) tiles are contiguous logical ids
  int L = blockIdx.x;
  if (total % 8 == 0) L = (L % 8) * (total / 8) + L / 8;
  const int bx = L % gx, by = (L / gx) % gy, bz = L / (gx * gy);
  const int n0 = bx * TN, k0 = by * TK;
  const int mbeg = bz * p.rows_per_split;
  const int mend = min(p.M, mbeg + p.rows_per_split);
  const int nsteps = (mend - mbeg + MK - 1) / MK;
  const int HWo = p.Ho * p.Wo;
  const float inv_hw = 1.f / (float)HWo, inv_w = 1.f / (float)p.Wo;
  // this k tile lies inside one filter tap (Ci % TK == 0)
  const int tap = k0 / p.Ci, ci0 = k0 - tap * p.Ci;
  const int tr = tap / p.S, ts = tap - tr * p.S;
  // raw descriptors for the inline-asm DMA (common.h lds_dma16)
  const u32x4_t rg = make_srd(p.G, (uint32_t)((size_t)p.M * p.N * 2));
  const u32x4_t rx = make_srd(p.X, (uint32_t)((size_t)(p.M / HWo) * p.Hi * p.Wi * p.Ci * 2));
  // this lane's rows / source chunks in its pieces
  const int drow0 = lane / CPN, dq = lane % CPN;
  const int xrow0 = lane / CPK, xq = lane % CPK;

  auto issue = [&](int step, int buf) {
    const int m0 = mbeg + step * MK;
    char *dbase = smem + buf * SBYTES;
    char *xbase = dbase + DBYTES;
#pragma unroll
    for (int i = 0; i < PNW; ++i) {
      const int piece = wave * PNW + i;
      const int row = piece * (1024 / RBN) + drow0;
      const int c = dq ^ (2 * wg_sw<RBN>(row));
      const int m = m0 + row;
      const uint32_t off = m < mend ? (uint32_t)(((size_t)m * p.N + n0 + c * 8) * 2) : kOOB;
      lds_dma16(rg, dbase + piece * 1024, off);
    }
#pragma unroll
    for (int i = 0; i < PKW; ++i) {
      const int piece = wave * PKW + i;
      const int row = piece * (1024 / RBK) + xrow0;
      const int c = xq ^ (2 * wg_sw<RBK>(row));
      const int m = m0 + row;
      uint32_t off = kOOB;
      if (m < mend) {
        const int b = fdiv(m, HWo, inv_hw), rem = m - b * HWo;
        const int oh = fdiv(rem, p.Wo, inv_w), ow = rem - oh * p.Wo;
        const int ih = oh * p.stride - p.pad + tr, iw = ow * p.stride - p.pad + ts;
        if (ih >= 0 && ih < p.Hi && iw >= 0 && iw < p.Wi)
          off = (uint32_t)(((((size_t)b * p.Hi + ih) * p.Wi + iw) * p.Ci + ci0 + c * 8) * 2);
      }
      lds_dma16(rx, xbase + piece * 1024, off);
    }
  };

  f32x4_t acc[RN][RK];
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // transposed-read addressing: lane (i = lane & 15, g = lane >> 4) reads rows trow, trow + 4
  // (+32 per sub-step), 8-B column piece tcol of a 16-column block; the swizzle term is the
  // same for all of this lane's rows (sw ignores bit 2 and bits >= 4)
  const int trow = 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int tc = lane & 3;                          // 8-B piece: chunk 2*blk + (tc >> 1), half tc & 1
  const int swn = 2 * wg_sw<RBN>(trow), swk = 2 * wg_sw<RBK>(trow);
  auto mma = [&](int buf) {
    const char *Db = smem + buf * SBYTES;
    const char *Xb = Db + DBYTES;
#pragma unroll
    for (int sub = 0; sub < MK / 32; ++sub) {
      s16x8_t af[RN], bfr[RK];
#pragma unroll
      for (int a = 0; a < RN; ++a) {
        const int blk = (wn * QN + a * 16) / 8;     // first chunk of the 16-column block
        const char *pa = Db + (sub * 32 + trow) * RBN + (((blk + (tc >> 1)) ^ swn) * 16) + (tc & 1) * 8;
        const s16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)pa);
        const s16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(pa + 4 * RBN));
        af[a] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int b = 0; b < RK; ++b) {
        const int blk = (wk * QK + b * 16) / 8;
        const char *pb = Xb + (sub * 32 + trow) * RBK + (((blk + (tc >> 1)) ^ swk) * 16) + (tc & 1) * 8;
        const s16x4_t b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)pb);
        const s16x4_t b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(pb + 4 * RBK));
        bfr[b] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int a = 0; a < RN; ++a)
#pragma unroll
        for (int b = 0; b < RK; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  if constexpr (NBUF == 2) {
    if (nsteps > 0) issue(0, 0);
    for (int s = 0; s < nsteps; ++s) {
      const int buf = s & 1;
      if (s + 1 < nsteps) {
        issue(s + 1, buf ^ 1);
        glds_wait_barrier<PW>();
      } else {
        glds_wait_barrier<0>();
      }
      mma(buf);
      glds_wait_barrier<PW>();
    }
  } else {
    // ring: NBUF - 1 stages in flight, one barrier per stage (stage s landed everywhere AND every
    // wave is done with stage s - 1, whose buffer the next issue refills)
#pragma unroll
    for (int q = 0; q < NBUF - 1; ++q)
      if (q < nsteps) issue(q, q);
    int buf = 0, nbuf = NBUF - 1;
    for (int s = 0; s < nsteps; ++s) {
      if (s + NBUF - 2 < nsteps) glds_wait_barrier<(NBUF - 2) * PW>();
      else if (NBUF == 4 && s + 1 < nsteps) glds_wait_barrier<PW>();
      else glds_wait_barrier<0>();
      if (s + NBUF - 1 < nsteps) issue(s + NBUF - 1, nbuf);
      mma(buf);
      buf = buf == NBUF - 1 ? 0 : buf + 1;
      nbuf = nbuf == NBUF - 1 ? 0 : nbuf + 1;
    }
  }
  float *dst = p.out + (size_t)bz * p.N * p.Kw;
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * QN + a * 16 + 4 * (lane >> 4) + j;
        const int k = k0 + wk * QK + b * 16 + (lane & 15);
        if (n < p.N) dst[(size_t)n * p.Kw + k] = acc[a][b][j];
      }
}

// ===========================================================================
// weight transposes for dgrad: dst[ci][t][co] = src[co][t][ci]  (bf16, batched by table)
// tab int32 [n][5] = (src offset, dst offset, Cout, taps, Cin)
// ===========================================================================
__global__ __launch_bounds__(256) void conv_wt_kernel(const bf16_t *__restrict__ src, bf16_t *__restrict__ dst,
                                                      const int *__restrict__ tab) {
  __shared__ bf16_t T[32][33];
  const int *e = tab + blockIdx.y * 5;
  const long long so = e[0], dof = e[1];
  const int Co = e[2], RS = e[3], Ci = e[4];
  const int tco = (Co + 31) / 32, tci = (Ci + 31) / 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int t = blockIdx.x; t < tco * tci * RS; t += gridDim.x) {
    const int tap = t / (tco * tci), rem = t % (tco * tci);
    const int co0 = (rem / tci) * 32, ci0 = (rem % tci) * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + ty + 8 * i, ci = ci0 + tx;
      T[ty + 8 * i][tx] = (co < Co && ci < Ci) ? src[so + ((long long)co * RS + tap) * Ci + ci] : bf16_t(0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ci = ci0 + ty + 8 * i, co = co0 + tx;
      if (co < Co && ci < Ci) dst[dof + ((long long)ci * RS + tap) * Co + co] = T[tx][ty + 8 * i];
    }
    __syncthreads();
  }
}

// ===========================================================================
// bottleneck output:  o = relu(y3*s3 + t3 + (yd*sd + td  |  x))       [M][C]
// ===========================================================================
// mask (optional, [M][C/8] bytes): bit j of byte i = out element 8i + j > 0 (the ReLU mask the
// next block's conv1 dgrad applies, CE_BWD_RXYM: 1/16 of the bytes of re-reading out)
template <bool PROJ, bool LZ>
__global__ __launch_bounds__(256) void res_out_kernel(const bf16_t *__restrict__ y, const float *__restrict__ s,
                                                      const float *__restrict__ t, const bf16_t *__restrict__ r,
                                                      const float *__restrict__ rs, const float *__restrict__ rt,
                                                      bf16_t *__restrict__ out, long long n8, int C8,
                                                      const BnFin *lz, const BnFin *lz2, uint8_t *__restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float lzs[];
  if constexpr (LZ) {   // BN3 (and the projection BN) finalized from the replica rows
    const int C = C8 * 8;
    lz_stage(lz, lzs, C, 2);
    if constexpr (PROJ) lz_stage(lz2, lzs + 2 * C, C, 2);
    __syncthreads();
    s = lzs; t = lzs + C;
    if constexpr (PROJ) { rs = lzs + 2 * C; rt = lzs + 3 * C; }
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % C8) * 8;
    float v[8], rv[8], a[8], b[8];
    unpack8(ldg16(y + i * 8), v);
    unpack8(ldg16(r + i * 8), rv);
    ld8f(s + c0, a);
    ld8f(t + c0, b);
    if constexpr (PROJ) {
      float ra[8], rb[8];
      ld8f(rs + c0, ra);
      ld8f(rt + c0, rb);
#pragma unroll
      for (int k = 0; k < 8; ++k) rv[k] = fmaf(rv[k], ra[k], rb[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = reluf(fmaf(v[k], a[k], b[k]) + rv[k]);
    const uint4 o = pack8(v);
    stg16(out + i * 8, o);
    if (mask) {   // from the stored bf16 values (relu >= 0: nonzero bits <=> > 0)
      const uint32_t w[4] = {o.x, o.y, o.z, o.w};
      uint32_t m = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= ((w[k] & 0xffffu) ? 1u : 0u) << (2 * k) | ((w[k] >> 16) ? 1u : 0u) << (2 * k + 1);
      mask[i] = (uint8_t)m;
    }
  }
}

// ===========================================================================
// 3x3 s2 p1 max-pool of relu(bn(y)) (stem output), forward with the arg-max tap (uint8)
// and backward (gather over the <= 4 windows that contain an input pixel) fused with the
// stem BN's ReLU mask and its backward partial sums.  8 channels per thread.
// ===========================================================================
template <bool LZ>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t *__restrict__ y, const float *__restrict__ s,
                                                          const float *__restrict__ t, bf16_t *__restrict__ out,
                                                          uint8_t *__restrict__ idx, int Nb, int H, int W, int C,
                                                          int Ho, int Wo, const BnFin *lz) {
  extern __shared__ __attribute__((aligned(16))) float lzs[];
  if constexpr (LZ) {
    lz_stage(lz, lzs, C, 2);
    __syncthreads();
    s = lzs; t = lzs + C;
  }
  const int C8 = C / 8;
  const long long total = (long long)Nb * Ho * Wo * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % C8) * 8;
    const long long pix = i / C8;
    const int ow = (int)(pix % Wo), oh = (int)((pix / Wo) % Ho), b = (int)(pix / ((long long)Wo * Ho));
    float a[8], sh[8], best[8];
    int bi[8];
    ld8f(s + c0, a);
    ld8f(t + c0, sh);
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -1.f; bi[k] = 0; }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ih = oh * 2 - 1 + r, iw = ow * 2 - 1 + q;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        float v[8];
        unpack8(ldg16(y + (((size_t)b * H + ih) * W + iw) * C + c0), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = reluf(fmaf(v[k], a[k], sh[k]));
          if (z > best[k]) { best[k] = z; bi[k] = r * 3 + q; }
        }
      }
    stg16(out + pix * C + c0, pack8(best));
    uint2 u;
    u.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    u.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2 *>(idx + pix * C + c0) = u;
  }
}

// one workgroup per (image, strip of rows): 256 threads = 32 pixels x 8 channel chunks (C = 64)
// part[blockIdx][2][C]: sum g, sum g*y
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t *__restrict__ gp, const uint8_t *__restrict__ idx,
                                                          const bf16_t *__restrict__ y, const float *__restrict__ s,
                                                          const float *__restrict__ t, bf16_t *__restrict__ g,
                                                          float *__restrict__ part, int Nb, int H, int W, int C,
                                                          int Ho, int Wo, int pix_per_wg, int rep) {
  __shared__ float red[2][32][64];
  const int C8 = C / 8;   // == 8
  const int cc = threadIdx.x % C8, pl = threadIdx.x / C8, PPI = 256 / C8;
  const int c0 = cc * 8;
  float a[8], sh[8], s0[8], s1[8];
  ld8f(s + c0, a);
  ld8f(t + c0, sh);
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0.f;
  const long long total = (long long)Nb * H * W;
  const long long p0 = (long long)blockIdx.x * pix_per_wg;
  for (long long pix = p0 + pl; pix < min(total, p0 + pix_per_wg); pix += PPI) {
    const int w = (int)(pix % W), h = (int)((pix / W) % H), b = (int)(pix / ((long long)W * H));
    // the (at most 2 x 2) windows (oh, ow) with oh*2-1 <= h <= oh*2+1: oh0 = h / 2, and oh0 + 1
    // for odd h (same for w).  All four candidates are loaded unconditionally (an invalid one
    // re-reads window (oh0, ow0) and is masked), so the loads of a pixel are in flight together
    // instead of sitting behind data-dependent loop branches (vmcnt(0) at every join)
    const int oh0 = h >> 1, ow0 = w >> 1;
    const bool oh1ok = (h & 1) && oh0 + 1 < Ho, ow1ok = (w & 1) && ow0 + 1 < Wo;
    uint2 u[4];
    uint4 gq[4];
    int tp[4];
    bool ok[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dy = q >> 1, dx = q & 1;
      ok[q] = (dy == 0 || oh1ok) && (dx == 0 || ow1ok);
      const int oh = ok[q] ? oh0 + dy : oh0, ow = ok[q] ? ow0 + dx : ow0;
      tp[q] = (h - (oh * 2 - 1)) * 3 + (w - (ow * 2 - 1));
      const size_t o = (((size_t)b * Ho + oh) * Wo + ow) * C + c0;
      u[q] = *reinterpret_cast<const uint2 *>(idx + o);
      gq[q] = ldg16(gp + o);
    }
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float gv[8];
      unpack8(gq[q], gv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t word = k < 4 ? u[q].x : u[q].y;
        const int ti = (word >> (8 * (k & 3))) & 0xff;
        acc[k] += (ok[q] && ti == tp[q]) ? gv[k] : 0.f;
      }
    }
    float yv[8];
    const size_t io = pix * C + c0;
    unpack8(ldg16(y + io), yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gk = fmaf(yv[k], a[k], sh[k]) > 0.f ? acc[k] : 0.f;
      gk = bf2f(f2bf(gk));
      acc[k] = gk;
      s0[k] += gk;
      s1[k] = fmaf(gk, yv[k], s1[k]);
    }
    stg16(g + io, pack8(acc));
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[0][pl][c0 + k] = s0[k]; red[1][pl][c0 + k] = s1[k]; }
  __syncthreads();
  if (threadIdx.x < 2 * C) {
    const int st = threadIdx.x / C, c = threadIdx.x % C;
    float v = 0.f;
    for (int q = 0; q < PPI; ++q) v += red[st][q][c];
    if (rep >= (int)gridDim.x) part[((size_t)blockIdx.x * 2 + st) * C + c] = v;
    else bn_part_add(part, blockIdx.x, gridDim.x, rep, C, st, c, v);
  }
}

// ===========================================================================
// head: global average pool (fp32 [B][C]) and the pooled-gradient broadcast back
// through the last ReLU, fused with the last BN's backward partial sums
// ===========================================================================
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16_t *__restrict__ x, float *__restrict__ out, int HW,
                                                      int C) {
  const int b = blockIdx.x;
  for (int c8 = threadIdx.x; c8 < C / 8; c8 += blockDim.x) {
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int i = 0; i < HW; ++i) {
      float v[8];
      unpack8(ldg16(x + ((size_t)b * HW + i) * C + c8 * 8), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    float *o = out + (size_t)b * C + c8 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = acc[k] / (float)HW;
  }
}

// G[b][i][c] = dpool[b][c] / HW * (x > 0);  part[b][2][C] = (sum G, sum G*y) over the image
__global__ __launch_bounds__(256) void head_bwd_kernel(const float *__restrict__ dpool, const bf16_t *__restrict__ x,
                                                       const bf16_t *__restrict__ y, bf16_t *__restrict__ G,
                                                       float *__restrict__ part, int HW, int C, int rep) {
  const int b = blockIdx.x;
  const bool own = rep >= (int)gridDim.x;
  for (int c8 = threadIdx.x; c8 < C / 8; c8 += blockDim.x) {
    float d[8], s0[8], s1[8];
    ld8f(dpool + (size_t)b * C + c8 * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) { d[k] /= (float)HW; s0[k] = s1[k] = 0.f; }
    for (int i = 0; i < HW; ++i) {
      const size_t o = ((size_t)b * HW + i) * C + c8 * 8;
      float xv[8], yv[8], g[8];
      unpack8(ldg16(x + o), xv);
      unpack8(ldg16(y + o), yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[k] = bf2f(f2bf(xv[k] > 0.f ? d[k] : 0.f));
        s0[k] += g[k];
        s1[k] = fmaf(g[k], yv[k], s1[k]);
      }
      stg16(G + o, pack8(g));
    }
    if (own) {
      float *p0 = part + (size_t)b * 2 * C + c8 * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) { p0[k] = s0[k]; p0[C + k] = s1[k]; }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bn_part_add(part, b, gridDim.x, rep, C, 0, c8 * 8 + k, s0[k]);
        bn_part_add(part, b, gridDim.x, rep, C, 1, c8 * 8 + k, s1[k]);
      }
    }
  }
}

// softmax cross-entropy over NC classes, one wave per image: loss[b], correct[b],
// dlogits[b][:] = (softmax - onehot) * scale
__global__ __launch_bounds__(64) void softmax_ce_kernel(const float *__restrict__ logits, const long long *__restrict__ labels,
                                                        int NC, float scale, float *__restrict__ loss,
                                                        float *__restrict__ correct, float *__restrict__ dlogits) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float *z = logits + (size_t)b * NC;
  float mx = -INFINITY;
  int am = 0;
  for (int i = lane; i < NC; i += 64) if (z[i] > mx) { mx = z[i]; am = i; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float se = 0.f;
  for (int i = lane; i < NC; i += 64) se += __expf(z[i] - mx);
  se = wave_sum(se);
  const int lab = (int)labels[b];
  const float lse = mx + __logf(se);
  if (lane == 0) {
    loss[b] = lse - z[lab];
    correct[b] = am == lab ? 1.f : 0.f;
  }
  if (dlogits) {
    for (int i = lane; i < NC; i += 64) dlogits[(size_t)b * NC + i] = (__expf(z[i] - lse) - (i == lab ? 1.f : 0.f)) * scale;
  }
}

// ===========================================================================
// synthetic ImageNet-shaped input: uint8 [n][H][W][3] pool -> random horizontal flip,
// ImageNet normalisation, NHWC bf16 with a zero 4th channel
// ===========================================================================
__global__ __launch_bounds__(256) void image_prep_kernel(const uint8_t *__restrict__ src, const long long *__restrict__ idx,
                                                         const long long *__restrict__ lab_src, int HW, int W,
                                                         unsigned long long seed, const float *__restrict__ hyper,
                                                         bf16_t *__restrict__ out, long long *__restrict__ lab_out,
                                                         int s2d) {
  const int b = blockIdx.y;
  const long long si = idx[b];
  const uint64_t step = hyper ? (uint64_t)hyper[1] : 0;
  const bool flip = hyper != nullptr && pg_uniform(seed ^ (step * 0x9E3779B97F4A7C15ull), (uint64_t)b) < 0.5f;   // no hyper: test transform
  const float mean[3] = {0.485f, 0.456f, 0.406f}, inv[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const int h = p / W, w = p % W;
    const int sw = flip ? W - 1 - w : w;
    const uint8_t *s = src + ((size_t)si * HW + (size_t)h * W + sw) * 3;
    float v[4];
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = ((float)s[c] * (1.f / 255.f) - mean[c]) * inv[c];
    v[3] = 0.f;
    uint2 u;
    u.x = pack2(v[0], v[1]);
    u.y = pack2(v[2], v[3]);
    // s2d: space-to-depth by 2, [B][H/2][W/2][16] with channel (dh*2 + dw)*4 + c (the ResNet stem)
    const size_t o = s2d ? ((((size_t)b * (HW / W / 2) + (h >> 1)) * (W >> 1) + (w >> 1)) * 16 + ((h & 1) * 2 + (w & 1)) * 4)
                         : ((size_t)b * HW + p) * 4;
    *reinterpret_cast<uint2 *>(out + o) = u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) lab_out[b] = lab_src[si];
}

// ===========================================================================
// host side
// ===========================================================================
namespace {
struct Geom {
  int BM, BN, KS, nmt, nt, ncls;
  size_t lds;
};

Geom igemm_geom(int M, int N, int Kmax, int Ci, int ncls) {
  Geom g{};
  // largest tile that still gives min_wgs workgroups (128 x 128 tiles run at 1.3-1.8x the
  // MFMA rate of the smaller ones on MI355X, so the bar is about one workgroup per CU)
  constexpr int min_wgs = 256;   // (512 / 1024: smaller tiles, slower; docs/PERF_NOTES.md round 3)
  static constexpr int cand[4][2] = {{128, 128}, {64, 128}, {128, 64}, {64, 64}};
  int pick = 3;
  for (int i = 0; i < 4; ++i) {
    if (cand[i][1] == 128 && N <= 64) continue;   // no half-empty N tiles
    const long long wgs = (long long)((M + cand[i][0] - 1) / cand[i][0]) * ((N + cand[i][1] - 1) / cand[i][1]) * ncls;
    if (wgs >= min_wgs) { pick = i; break; }
  }
  g.BM = cand[pick][0];
  g.BN = cand[pick][1];
  g.nmt = (M + g.BM - 1) / g.BM;
  g.nt = (N + g.BN - 1) / g.BN;
  g.ncls = ncls;
  g.KS = (Kmax >= 256 && Ci % 64 == 0) ? 64 : 32;
  const size_t ops = (size_t)2 * (g.BM + g.BN) * (g.KS + 8) * 2;
  const size_t ctile = (size_t)g.BM * (g.BN + 8) * 2;
  const size_t red = (size_t)(256 / (g.BN / 8)) * g.BN * 4;
  g.lds = ops > ctile ? ops : ctile;
  if (red > g.lds) g.lds = red;
  return g;
}

template <int MODE, int PRO, int EPI, int BM, int BN, int KS, int CV>
void launch_t(const ConvArgs &a, const Geom &g, bool ut, hipStream_t st) {
  const dim3 grid(g.nmt * g.nt, g.ncls);
  if (ut) hipLaunchKernelGGL((conv_igemm_kernel<MODE, PRO, EPI, BM, BN, KS, CV, true>), grid, dim3(256), g.lds, st, a);
  else hipLaunchKernelGGL((conv_igemm_kernel<MODE, PRO, EPI, BM, BN, KS, CV, false>), grid, dim3(256), g.lds, st, a);
}

template <int MODE, int PRO, int EPI, int CV>
void launch_geom(const ConvArgs &a, const Geom &g, hipStream_t st) {
  const bool ut = a.Ci % g.KS == 0;
  if constexpr (CV == 4) {   // stem: K = 196 -> 32-wide k-steps
    if (g.BM == 128 && g.BN == 64) { launch_t<MODE, PRO, EPI, 128, 64, 32, CV>(a, g, false, st); return; }
    launch_t<MODE, PRO, EPI, 64, 64, 32, CV>(a, g, false, st);
    return;
  } else {
#define LG_TILE(BM_, BN_)                                                                              \
  if (g.BM == BM_ && g.BN == BN_) {                                                                    \
    if (g.KS == 64) launch_t<MODE, PRO, EPI, BM_, BN_, 64, CV>(a, g, ut, st);                          \
    else launch_t<MODE, PRO, EPI, BM_, BN_, 32, CV>(a, g, ut, st);                                     \
    return;                                                                                            \
  }
    LG_TILE(128, 128)
    LG_TILE(128, 64)
    LG_TILE(64, 128)
    LG_TILE(64, 64)
#undef LG_TILE
  }
}

// LDS-DMA kernel (conv_glds_kernel) for operands without a prologue: g_conv_glds = 2 LDS
// buffers (default), 0 off (the register-staged kernel; conv_set_glds: tests).  (A 3-stage ring
// at 128x128 -- 96 KB of LDS, one workgroup per CU -- and 32-wide k steps with 2-4 stages
// measured slower: fwd 3657 / ~2990 vs 2843 us network total, docs/PERF_NOTES.md round 3.)
int g_conv_glds = 2;
bool glds_ok(int Ci) { return g_conv_glds != 0 && Ci % 64 == 0; }

template <int MODE, int EPI, int BM, int BN, int NBUF, int KS, bool MT = false, bool FOLD = false>
void launch_glds_t(const ConvArgs &a, const Geom &g, hipStream_t st) {
  // one k-step (K <= KS: the 1x1 convs on 64 channels, memory-bound): the kernel only ever fills
  // buffer 0, so one stage of LDS (the C tile sets the size) lets twice the workgroups per CU
  // share the memory latency
  int kmax = a.K;
  if (MODE == CM_DGRAD)
    for (int c = 0; c < g.ncls; ++c) kmax = a.ntap[c] * a.Ci > kmax ? a.ntap[c] * a.Ci : kmax;
  const int stages = kmax <= KS ? 1 : NBUF;
  size_t lds = (size_t)stages * (BM + BN) * KS * 2;
  const size_t ctile = (size_t)BM * (BN + 8) * 2, red = (size_t)(256 / (BN / 8)) * BN * 4;
  if (ctile > lds) lds = ctile;
  if (red > lds) lds = red;
  hipLaunchKernelGGL((conv_glds_kernel<MODE, EPI, BM, BN, NBUF, KS, MT, FOLD>), dim3(g.nmt * g.nt, g.ncls), dim3(256),
                     lds, st, a);
}


// (256 x 128 tiles, one workgroup of 4 waves per CU at 2 or 3 LDS stages, measured slower on
// every ResNet-50 layer: forward network total 2826 -> 3150 us, dgrad 3875 -> 4533 us; the
// loop is latency-bound at one wave per SIMD, not operand-bandwidth-bound -- docs/PERF_NOTES.md)
template <int MODE, int EPI>
void launch_glds(const ConvArgs &a, const Geom &g, hipStream_t st) {
#define LG_GLDS(BM_, BN_)                                  \
  if (g.BM == BM_ && g.BN == BN_) {                        \
    launch_glds_t<MODE, EPI, BM_, BN_, 2, 64>(a, g, st);   \
    return;                                                \
  }
  LG_GLDS(128, 128)
  LG_GLDS(128, 64)
  LG_GLDS(64, 128)
  LG_GLDS(64, 64)
#undef LG_GLDS
}

// dgrad parity classes of a (R, S, stride, pad) convolution
void dgrad_classes(ConvArgs &a, int R, int S, int st, int pad) {
  for (int cls = 0; cls < st * st; ++cls) {
    const int ph = cls / st, pw = cls % st;
    int n = 0;
    for (int r = 0; r < R; ++r) {
      if (((ph + pad - r) % st + st) % st) continue;
      for (int s = 0; s < S; ++s) {
        if (((pw + pad - s) % st + st) % st) continue;
        a.tr[cls][n] = (signed char)r;
        a.ts[cls][n] = (signed char)s;
        a.tdh[cls][n] = (signed char)((ph + pad - r) / st);   // exact division (multiple of st)
        a.tdw[cls][n] = (signed char)((pw + pad - s) / st);
        a.tapx[cls][n] = (int)(uint8_t)a.tdh[cls][n] | ((int)(uint8_t)a.tdw[cls][n] << 8) | ((r * S + s) << 16);
        ++n;
      }
    }
    a.ntap[cls] = n;
  }
}
}  // namespace

void conv_set_glds(int mode) { g_conv_glds = mode == 0 ? 0 : 2; }
int conv_get_glds() { return g_conv_glds; }

// BN partial rows a forward conv writes (per M tile)
int conv_fwd_num_partials(int Nb, int Ho, int Wo, int N, int K, int Ci) {
  const int M = Nb * Ho * Wo;
  return igemm_geom(M, N, K, Ci, 1).nmt;
}
// ... and a dgrad (all parity classes)
int conv_dgrad_num_partials(int Nb, int H, int W, int N, int Cout, int R, int S, int st) {
  const int M = Nb * (H / st) * (W / st);
  return igemm_geom(M, N, R * S * Cout, Cout, st * st).nmt * st * st;
}

// forward conv.  x [Nb][H][W][Ci] (Ci % 8 == 0, or Ci == 4 for the stem), w [N][R][S][Ci]
// pro: 0 none, 1 relu(x*pa+pb) of the producer BN
void launch_conv_fwd(int pro, const bf16_t *x, const float *pa, const float *pb, const bf16_t *w, bf16_t *y,
                     float *part, int Nb, int H, int W, int Ci, int N, int R, int S, int st, int pad,
                     hipStream_t stream) {
  ConvArgs a{};
  a.A = x; a.pa = pa; a.pb = pb; a.W = w; a.out = y; a.part = part;
  a.Hi = H; a.Wi = W; a.Ci = Ci;
  a.Ho = (H + 2 * pad - R) / st + 1;
  a.Wo = (W + 2 * pad - S) / st + 1;
  a.N = N; a.R = R; a.S = S; a.stride = st; a.pad = pad;
  a.Kw = R * S * Ci;
  a.K = Ci == 4 ? (a.Kw + 31) / 32 * 32 : a.Kw;
  a.Mc = Nb * a.Ho * a.Wo;
  a.Hc = a.Ho; a.Wc = a.Wo;
  a.Nb = Nb;
  const Geom g = igemm_geom(a.Mc, N, a.Kw, Ci, 1);
  a.nmt = g.nmt;
  a.bn_rep = g_bn_rep;
  if (Ci == 4) { launch_geom<CM_FWD, CP_NONE, CE_FWD, 4>(a, g, stream); return; }
  if (pro == CP_NONE && glds_ok(Ci)) { launch_glds<CM_FWD, CE_FWD>(a, g, stream); return; }
  if (pro == CP_BN_RELU) launch_geom<CM_FWD, CP_BN_RELU, CE_FWD, 8>(a, g, stream);
  else launch_geom<CM_FWD, CP_NONE, CE_FWD, 8>(a, g, stream);
}

// dgrad.  G, Y [Nb][Ho][Wo][Cout] (this layer's BN-backward: dy = ga*G + gb*Y + gc),
// wt [Cin][R][S][Cout]; out dx [Nb][H][W][Cin]   (H % st == 0, W % st == 0)
// epi 1: dx * (Yt*es + et > 0) + partials (sum, sum*Yt)
// epi 2: (dx + Rg) * (X > 0) + partials against Yt (part) and Yt2 (part2); operand sets:
//        {} | {Rg} | {Rg, X, Yt} | {Rg, X, Yt, Yt2}
void launch_conv_dgrad(int epi, const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb, const float *gc,
                       const bf16_t *wt, bf16_t *dx, const bf16_t *Yt, const float *es, const float *et,
                       const bf16_t *Rg, const bf16_t *X, const bf16_t *Yt2, float *part, float *part2, int Nb, int H,
                       int W, int Cin, int Cout, int R, int S, int st, int pad, const uint8_t *Xm,
                       hipStream_t stream) {
  ConvArgs a{};
  a.A = G; a.A2 = Y; a.pa = ga; a.pb = gb; a.pc = gc; a.W = wt; a.out = dx;
  a.Yt = Yt; a.Yt2 = Yt2; a.X = X; a.Xm = Xm; a.Rg = Rg; a.es = es; a.et = et; a.part = part; a.part2 = part2;
  a.Hi = (H + 2 * pad - R) / st + 1;
  a.Wi = (W + 2 * pad - S) / st + 1;
  a.Ci = Cout;
  a.Ho = H; a.Wo = W; a.N = Cin;
  a.R = R; a.S = S; a.stride = st; a.pad = pad;
  a.Kw = R * S * Cout;
  a.Hc = H / st; a.Wc = W / st;
  a.Mc = Nb * a.Hc * a.Wc;
  dgrad_classes(a, R, S, st, pad);
  int kmax = 0;
  for (int c = 0; c < st * st; ++c) kmax = a.ntap[c] * Cout > kmax ? a.ntap[c] * Cout : kmax;
  a.K = kmax;
  const Geom g = igemm_geom(a.Mc, Cin, kmax, Cout, st * st);
  a.nmt = g.nmt;
  a.Nb = Nb;
  a.bn_rep = g_bn_rep;
  if (Y == nullptr) {   // G is the materialised dy (launch_bn_mat): LDS-DMA kernel, no prologue
    if (epi == CE_BWD_RELU) { launch_glds<CM_DGRAD, CE_BWD_RELU>(a, g, stream); return; }
    if (!Rg && !X && !Xm && !Yt && !Yt2) launch_glds<CM_DGRAD, CE_BWD_PLAIN>(a, g, stream);
    else if (Rg && !X && !Xm && !Yt && !Yt2) launch_glds<CM_DGRAD, CE_BWD_R>(a, g, stream);
    else if (Rg && Xm && Yt && !Yt2) launch_glds<CM_DGRAD, CE_BWD_RXYM>(a, g, stream);
    else if (Rg && Xm && Yt && Yt2) launch_glds<CM_DGRAD, CE_BWD_RXYYM>(a, g, stream);
    else if (Rg && X && Yt && !Yt2) launch_glds<CM_DGRAD, CE_BWD_RXY>(a, g, stream);
    else if (Rg && X && Yt && Yt2) launch_glds<CM_DGRAD, CE_BWD_RXYY>(a, g, stream);
    return;
  }
  if (epi == CE_BWD_RELU) { launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_RELU, 8>(a, g, stream); return; }
  // (dx + Rg) * 1[X > 0] with statistics against Yt (, Yt2): supported operand sets
  if (!Rg && !X && !Xm && !Yt && !Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_PLAIN, 8>(a, g, stream);
  else if (Rg && !X && !Xm && !Yt && !Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_R, 8>(a, g, stream);
  else if (Rg && Xm && Yt && !Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_RXYM, 8>(a, g, stream);
  else if (Rg && Xm && Yt && Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_RXYYM, 8>(a, g, stream);
  else if (Rg && X && Yt && !Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_RXY, 8>(a, g, stream);
  else if (Rg && X && Yt && Yt2) launch_geom<CM_DGRAD, CP_BNBWD, CE_BWD_RXYY, 8>(a, g, stream);
}

// ---- 1x1 data gradient with the BN backward folded into the GEMM
// dy = a*G + b*Y + c (per output channel k of the conv)  =>  dx[m][n] = sum_k G[m][k] (a_k W[n][k])
// + sum_k Y[m][k] (b_k W[n][k]) + sum_k c_k W[n][k]: one GEMM with K = 2 Cout over [G | Y] and the
// per-step weights W2[n] = [a.W[n] | b.W[n]] (bf16), instead of materialising dy (a read of G and Y
// and a write of dy) and reading it back.  The bias also carries the rounding of b.W against the
// channel means: fbias[n] = sum_k c_k W[n][k] + sum_k mu_k (b_k W[n][k] - bf16(b_k W[n][k])), so the
// bf16 rounding of b.W multiplies the centred Y - mu only (no error from the cancelling means).
__global__ __launch_bounds__(256) void conv_fold_w_kernel(const bf16_t *__restrict__ wt, const float *__restrict__ a,
                                                          const float *__restrict__ b, const float *__restrict__ c,
                                                          const float *__restrict__ mu, bf16_t *__restrict__ w2,
                                                          float *__restrict__ fbias, int K) {
  __shared__ float red[256];
  const int n = blockIdx.x, tid = threadIdx.x;
  const bf16_t *wr = wt + (size_t)n * K;
  bf16_t *o = w2 + (size_t)n * 2 * K;
  float acc = 0.f;
  for (int k = tid; k < K; k += 256) {
    const float w = bf2f(wr[k]);
    const float bw = b[k] * w;
    const bf16_t q = f2bf(bw);
    o[k] = f2bf(a[k] * w);
    o[K + k] = q;
    acc = fmaf(c[k], w, fmaf(mu[k], bw - bf2f(q), acc));
  }
  red[tid] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  if (tid == 0) fbias[n] = red[0];
}

void launch_conv_fold_w(const bf16_t *wt, const float *a, const float *b, const float *c, const float *mu, bf16_t *w2,
                        float *fbias, int Cin, int Cout, hipStream_t st) {
  hipLaunchKernelGGL(conv_fold_w_kernel, dim3(Cin), dim3(256), 0, st, wt, a, b, c, mu, w2, fbias, Cout);
}

// dx = conv1x1^T(dy) with dy folded as above (w2 / fbias from launch_conv_fold_w), epilogue
// CE_BWD_RELU: dx * 1[Yt*es + et > 0], BN partials (sum dx, sum dx*Yt).  Stride 1, Cout % 64 == 0.
void launch_conv_dgrad_fold(const bf16_t *G, const bf16_t *Y, const bf16_t *w2, const float *fbias, bf16_t *dx,
                            const bf16_t *Yt, const float *es, const float *et, float *part, int Nb, int H, int W,
                            int Cin, int Cout, hipStream_t stream) {
  ConvArgs a{};
  a.A = G; a.A2 = Y; a.W = w2; a.out = dx; a.fbias = fbias;
  a.Yt = Yt; a.es = es; a.et = et; a.part = part;
  a.Hi = H; a.Wi = W; a.Ci = Cout;
  a.Ho = H; a.Wo = W; a.N = Cin;
  a.R = 1; a.S = 1; a.stride = 1; a.pad = 0;
  a.Kw = 2 * Cout;
  a.Hc = H; a.Wc = W;
  a.Mc = Nb * H * W;
  a.ntap[0] = 2;   // tap 0: G with a.W, tap 1: Y with b.W (same pixel)
  a.tapx[0][0] = 0;
  a.tapx[0][1] = 1 << 16;
  a.tr[0][0] = a.tr[0][1] = 0;
  a.ts[0][0] = 0; a.ts[0][1] = 1;
  a.K = 2 * Cout;
  // the BN partial rows must match conv_dgrad_num_partials of the unfolded 1x1 dgrad: same M
  // tiles (igemm_geom picks the tile from M and N only, K decides the k-step alone)
  const Geom g = igemm_geom(a.Mc, Cin, 2 * Cout, Cout, 1);
  a.nmt = g.nmt;
  a.Nb = Nb;
  a.bn_rep = g_bn_rep;
#define LG_FOLD(BM_, BN_)                                                                \
  if (g.BM == BM_ && g.BN == BN_) {                                                      \
    launch_glds_t<CM_DGRAD, CE_BWD_RELU, BM_, BN_, 2, 64, false, true>(a, g, stream);    \
    return;                                                                              \
  }
  LG_FOLD(128, 128)
  LG_FOLD(128, 64)
  LG_FOLD(64, 128)
  LG_FOLD(64, 64)
#undef LG_FOLD
}

// ---- weight gradient
namespace {
struct WgGeom {
  int TN, TK, nsplit, rows;
};
// LDS-DMA weight gradient (conv_wgrad_dma_kernel): materialised dy, x without a prologue,
// Ci and N multiples of 64 (4584 -> 4029 us of ResNet-50 weight gradients, round 3).
bool wg_dma_ok(bool dm, int xpro, int Ci, int N) {
  return dm && xpro == CP_NONE && Ci % 64 == 0 && N % 64 == 0;
}
// Per-shape configuration of the LDS-DMA weight gradient: split-M grid-size target, m rows per
// stage and ring depth.  Measured per ResNet-50 layer at bs128 on MI355X (scripts/conv_bench.py
// wgradma, profiles/r3b_wgrad_dma_cfg.txt): the 3x3 layers are latency-bound (few MFMAs per
// stage): the 64x64-tile ones (32 KB of LDS per workgroup, up to 5 per CU) and the 14x14 maps
// want a 1024-workgroup grid (l1.c2 150 -> 98 us, l3.c2 84 -> 76), the 7x7 maps (3-4 splits) a
// 3-deep ring of 32-row stages (l4.c2 103 -> 82); the 1x1 layers and the 28x28 3x3 ones keep
// 512 workgroups and 2 x 64-row stages (network total 4024 -> ~3750 us).
struct WgDmaCfg {
  int target, mk, nbuf;
};
WgDmaCfg wg_dma_cfg(int N, int Ci, int M, int taps) {
  const int TN = N % 128 == 0 ? 128 : 64, TK = Ci % 128 == 0 ? 128 : 64;
  WgDmaCfg c{512, 64, 2};   // (1x1 grid target 256 / 128: slower, profiles/r3c_resnet50_side_ab.txt)
  if (taps > 1) {
    if (M <= 8192) { c.mk = 32; c.nbuf = 3; }
    else if (M <= 32768 || (TN == 64 && TK == 64)) c.target = 1024;
  }
  return c;
}

WgGeom wg_geom(int N, int Kw, int M, bool dma = false, int Ci = 0) {
  WgGeom g{};
  if (dma) {
    g.TN = N % 128 == 0 ? 128 : 64;
    g.TK = Ci % 128 == 0 ? 128 : 64;
  } else {
    g.TN = N >= 128 ? 128 : 64;
    g.TK = Kw >= 128 ? 128 : 64;
  }
  const long long tiles = (long long)((N + g.TN - 1) / g.TN) * ((Kw + g.TK - 1) / g.TK);
  constexpr int target = 1024;   // split-M grid target (512 / 2048 / 4096: slower, round 1)
  long long ns = ((dma ? wg_dma_cfg(N, Ci, M, Kw / Ci).target : target) + tiles - 1) / tiles;
  const long long max_ns = (M + 4 * kWgMK - 1) / (4 * kWgMK);   // >= 4 steps per split
  if (ns > max_ns) ns = max_ns;
  if (ns < 1) ns = 1;
  g.rows = (int)(((M + ns - 1) / ns + kWgMK - 1) / kWgMK * kWgMK);
  g.nsplit = (M + g.rows - 1) / g.rows;
  return g;
}
}  // namespace

int colsum_rows(int R);
void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st, bool stem36 = false);

long long conv_wgrad_workspace_floats(int Nb, int H, int W, int Ci, int N, int R, int S, int st, int pad) {
  const int Ho = (H + 2 * pad - R) / st + 1, Wo = (W + 2 * pad - S) / st + 1;
  long long need = 0;
  for (int dma = 0; dma < 2; ++dma) {   // either kernel may run (dy materialised or not)
    if (dma && !wg_dma_ok(true, CP_NONE, Ci, N)) continue;
    const WgGeom g = wg_geom(N, R * S * Ci, Nb * Ho * Wo, dma != 0, Ci);
    if (g.nsplit == 1) continue;
    const long long n = (long long)(g.nsplit + colsum_rows(g.nsplit)) * N * R * S * Ci;
    need = n > need ? n : need;
  }
  return need;
}

// dW [N][R][S][Ci] (fp32, overwritten) of y = conv(x);  G, Y [Nb][Ho][Wo][N];  x [Nb][H][W][Ci]
// xpro 1: x = relu(x*xs + xt) (producer BN), 0: as stored
void launch_conv_wgrad(const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb, const float *gc,
                       const bf16_t *x, const float *xs, const float *xt, int xpro, float *ws, float *grad, int Nb,
                       int H, int W, int Ci, int N, int R, int S, int st, int pad, hipStream_t stream) {
  WgArgs a{};
  a.G = G; a.Y = Y; a.ga = ga; a.gb = gb; a.gc = gc; a.X = x; a.xs = xs; a.xt = xt;
  a.N = N; a.Hi = H; a.Wi = W; a.Ci = Ci;
  a.Ho = (H + 2 * pad - R) / st + 1;
  a.Wo = (W + 2 * pad - S) / st + 1;
  a.R = R; a.S = S; a.stride = st; a.pad = pad;
  a.Kw = R * S * Ci;
  a.M = Nb * a.Ho * a.Wo;
  const bool dm = Y == nullptr;   // G is the materialised dy (launch_bn_mat)
  if (wg_dma_ok(dm, xpro, Ci, N)) {
    const WgGeom g = wg_geom(N, a.Kw, a.M, true, Ci);
    a.rows_per_split = g.rows;
    a.out = g.nsplit == 1 ? grad : ws;
    const int gx = N / g.TN, gy = a.Kw / g.TK, total = gx * gy * g.nsplit;
    const WgDmaCfg cfg = wg_dma_cfg(N, Ci, a.M, R * S);
    const int nb = cfg.nbuf, mk = cfg.mk;
    const size_t lds = (size_t)nb * mk * (g.TN + g.TK) * 2;
#define WGD_K(TN_, TK_, NB_, MK_) \
  hipLaunchKernelGGL((conv_wgrad_dma_kernel<TN_, TK_, NB_, MK_>), dim3(total), dim3(256), lds, stream, a, gx, gy, total)
#define WGD_L(TN_, TK_)                                       \
  do {                                                        \
    if (mk == 32) WGD_K(TN_, TK_, 3, 32);   /* 7x7 3x3 maps */ \
    else WGD_K(TN_, TK_, 2, 64);                              \
  } while (0)
    if (g.TN == 128 && g.TK == 128) WGD_L(128, 128);
    else if (g.TN == 128) WGD_L(128, 64);
    else if (g.TK == 128) WGD_L(64, 128);
    else WGD_L(64, 64);
#undef WGD_L
#undef WGD_K
    if (g.nsplit > 1) launch_wgrad_reduce(ws, g.nsplit, (long long)N * a.Kw, grad, stream);
    return;
  }
  const WgGeom g = wg_geom(N, a.Kw, a.M);
  a.rows_per_split = g.rows;
  a.out = g.nsplit == 1 ? grad : ws;
  const dim3 grid((N + g.TN - 1) / g.TN, (a.Kw + g.TK - 1) / g.TK, g.nsplit);
#define WG_L(XP, TN_, TK_, CV_)                                                                                  \
  do {                                                                                                          \
    if (dm) hipLaunchKernelGGL((conv_wgrad_kernel<XP, TN_, TK_, CV_, true>), grid, dim3(256), 0, stream, a);     \
    else hipLaunchKernelGGL((conv_wgrad_kernel<XP, TN_, TK_, CV_, false>), grid, dim3(256), 0, stream, a);       \
  } while (0)
  if (Ci == 4) {
    if (g.TN == 128) WG_L(CP_NONE, 128, 128, 4); else WG_L(CP_NONE, 64, 128, 4);
  } else if (xpro == CP_BN_RELU) {
    if (g.TN == 128 && g.TK == 128) WG_L(CP_BN_RELU, 128, 128, 8);
    else if (g.TN == 128) WG_L(CP_BN_RELU, 128, 64, 8);
    else if (g.TK == 128) WG_L(CP_BN_RELU, 64, 128, 8);
    else WG_L(CP_BN_RELU, 64, 64, 8);
  } else {
    if (g.TN == 128 && g.TK == 128) WG_L(CP_NONE, 128, 128, 8);
    else if (g.TN == 128) WG_L(CP_NONE, 128, 64, 8);
    else if (g.TK == 128) WG_L(CP_NONE, 64, 128, 8);
    else WG_L(CP_NONE, 64, 64, 8);
  }
#undef WG_L
  if (g.nsplit > 1) launch_wgrad_reduce(ws, g.nsplit, (long long)N * a.Kw, grad, stream);
}

void launch_conv_wt(const bf16_t *src, bf16_t *dst, const int *tab, int n, hipStream_t st) {
  hipLaunchKernelGGL(conv_wt_kernel, dim3(256, n), dim3(256), 0, st, src, dst, tab);
}

// lz / lz2 (device BnFin descriptors, both or neither; lz2 only with the projection): lazy finalize
void launch_res_out(const bf16_t *y, const float *s, const float *t, const bf16_t *r, const float *rs,
                    const float *rt, bf16_t *out, long long M, int C, const void *lz, const void *lz2,
                    uint8_t *mask, hipStream_t st) {
  const long long n8 = M * (C / 8);
  int grid = (int)((n8 + 255) / 256);
  const int cap = lz ? (C > 256 ? 512 : 2048) : 16384;
  if (grid > cap) grid = cap;
  const BnFin *d = static_cast<const BnFin *>(lz), *d2 = static_cast<const BnFin *>(lz2);
  const size_t lds = lz ? (size_t)(rs ? 4 : 2) * C * sizeof(float) : 0;
#define RO(PJ, LZ_) \
  hipLaunchKernelGGL((res_out_kernel<PJ, LZ_>), dim3(grid), dim3(256), lds, st, y, s, t, r, rs, rt, out, n8, C / 8, d, d2, \
                     mask)
  if (rs) { if (lz) RO(true, true); else RO(true, false); }
  else { if (lz) RO(false, true); else RO(false, false); }
#undef RO
}

void launch_maxpool_fwd(const bf16_t *y, const float *s, const float *t, bf16_t *out, uint8_t *idx, int Nb, int H,
                        int W, int C, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long total = (long long)Nb * Ho * Wo * (C / 8);
  int grid = (int)((total + 255) / 256);
  const BnFin *lz = take_bn_lz();
  const int cap = lz ? 2048 : 16384;
  if (grid > cap) grid = cap;
  if (lz)
    hipLaunchKernelGGL((maxpool_fwd_kernel<true>), dim3(grid), dim3(256), (size_t)2 * C * sizeof(float), st, y, s, t,
                       out, idx, Nb, H, W, C, Ho, Wo, lz);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<false>), dim3(grid), dim3(256), 0, st, y, s, t, out, idx, Nb, H, W, C, Ho,
                       Wo, lz);
}

constexpr int kMpPix = 512;   // input pixels per backward workgroup
int maxpool_bwd_num_partials(int Nb, int H, int W) {
  return (int)(((long long)Nb * H * W + kMpPix - 1) / kMpPix);
}

void launch_maxpool_bwd(const bf16_t *gp, const uint8_t *idx, const bf16_t *y, const float *s, const float *t,
                        bf16_t *g, float *part, int Nb, int H, int W, int C, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(maxpool_bwd_num_partials(Nb, H, W)), dim3(256), 0, st, gp, idx, y, s, t,
                     g, part, Nb, H, W, C, Ho, Wo, kMpPix, g_bn_rep);
}

void launch_avgpool(const bf16_t *x, float *out, int Nb, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_kernel, dim3(Nb), dim3(256), 0, st, x, out, HW, C);
}

void launch_head_bwd(const float *dpool, const bf16_t *x, const bf16_t *y, bf16_t *G, float *part, int Nb, int HW,
                     int C, hipStream_t st) {
  hipLaunchKernelGGL(head_bwd_kernel, dim3(Nb), dim3(256), 0, st, dpool, x, y, G, part, HW, C, g_bn_rep);
}

void launch_softmax_ce(const float *logits, const long long *labels, int B, int NC, float scale, float *loss,
                       float *correct, float *dlogits, hipStream_t st) {
  hipLaunchKernelGGL(softmax_ce_kernel, dim3(B), dim3(64), 0, st, logits, labels, NC, scale, loss, correct, dlogits);
}

void launch_image_prep(const uint8_t *src, const long long *idx, const long long *lab_src, int B, int H, int W,
                       unsigned long long seed, const float *hyper, bf16_t *out, long long *lab_out, int s2d,
                       hipStream_t st) {
  const int HW = H * W;
  hipLaunchKernelGGL(image_prep_kernel, dim3((HW + 255) / 256 < 64 ? (HW + 255) / 256 : 64, B), dim3(256), 0, st, src,
                     idx, lab_src, HW, W, seed, hyper, out, lab_out, s2d);
}

// ===========================================================================
// Space-to-depth ResNet stem.  The 7x7 s2 p3 conv over the 4-channel image equals a 4x4 s1 conv
// over its space-to-depth-by-2 image x2 [B][H/2][W/2][16] (channel (dh*2 + dw)*4 + c) with the
// window rows oh-2 .. oh+1 (top / left padding 2, H/2 outputs):
//   w2[n][r][s][(dh*2 + dw)*4 + c] = w[n][2r + dh - 1][2s + dw - 1][c]   (0 outside the 7x7)
// so the GEMM K is 4*4*16 = 256 (four 64-wide k-steps of 4 taps x 16 channels, 128 contiguous
// bytes of one x2 row per staged row) instead of 49 taps of 4 channels (8-B gathers).
// ===========================================================================
__global__ __launch_bounds__(256) void stem_w_s2d_kernel(const bf16_t *__restrict__ w, bf16_t *__restrict__ w2,
                                                         int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // [N][4][4][16] element
  if (i >= N * 256) return;
  const int n = i >> 8, k = i & 255;
  const int r = k >> 6, s = (k >> 4) & 3, q = k & 15, dh = q >> 3, dw = (q >> 2) & 1, c = q & 3;
  const int kh = 2 * r + dh - 1, kw = 2 * s + dw - 1;
  w2[i] = (kh >= 0 && kh < 7 && kw >= 0 && kw < 7) ? w[((n * 7 + kh) * 7 + kw) * 4 + c] : bf16_t(0);
}

// grad [N][7][7][4] of the 7x7 stem from the space-to-depth weight gradient g2 [N][4][4][16]
__global__ __launch_bounds__(256) void stem_wgrad_s2d_kernel(const float *__restrict__ g2, float *__restrict__ grad,
                                                             int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // [N][7][7][4] element
  if (i >= N * 196) return;
  const int n = i / 196, rem = i - n * 196, kh = rem / 28, kw = (rem / 4) % 7, c = rem & 3;
  const int r = (kh + 1) >> 1, dh = (kh + 1) & 1, s = (kw + 1) >> 1, dw = (kw + 1) & 1;
  grad[i] = g2[(size_t)n * 256 + ((r * 4 + s) * 16 + (dh * 2 + dw) * 4 + c)];
}

// NHWC 4-channel image [B][H][W][4] -> space-to-depth x2 [B][H/2][W/2][16] (one 8-B pixel per thread)
__global__ __launch_bounds__(256) void s2d_image_kernel(const bf16_t *__restrict__ img, bf16_t *__restrict__ x2,
                                                        long long npix, int H, int W) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const int w = (int)(i % W), h = (int)((i / W) % H);
  const long long b = i / ((long long)W * H);
  const uint2 v = *reinterpret_cast<const uint2 *>(img + i * 4);
  *reinterpret_cast<uint2 *>(x2 + (((b * (H / 2) + (h >> 1)) * (W / 2) + (w >> 1)) * 16 + ((h & 1) * 2 + (w & 1)) * 4)) = v;
}

void launch_s2d_image(const bf16_t *img, bf16_t *x2, int B, int H, int W, hipStream_t st) {
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(s2d_image_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, img, x2, n, H, W);
}

void launch_stem_w_s2d(const bf16_t *w, bf16_t *w2, int N, hipStream_t st) {
  hipLaunchKernelGGL(stem_w_s2d_kernel, dim3((N * 256 + 255) / 256), dim3(256), 0, st, w, w2, N);
}

namespace {
ConvArgs stem_s2d_args(int Nb, int H2, int N) {
  ConvArgs a{};
  a.Hi = a.Wi = H2; a.Ci = 16;
  a.Ho = a.Wo = H2;          // rows oh-2 .. oh+1: H2 outputs (not the H2 + 1 of a symmetric pad 2)
  a.N = N; a.R = a.S = 4; a.stride = 1; a.pad = 2;
  a.Kw = a.K = 256;
  a.Mc = Nb * H2 * H2;
  a.Hc = a.Wc = H2;
  a.Nb = Nb;
  a.bn_rep = g_bn_rep;
  return a;
}
}  // namespace

// y = stem(x2, w2) [Nb][H2][H2][N] + BN partials (P = conv_fwd_num_partials(Nb, H2, H2, N, 256, 16))
void launch_conv_fwd_s2d(const bf16_t *x2, const bf16_t *w2, bf16_t *y, float *part, int Nb, int H2, int N,
                         hipStream_t stream) {
  ConvArgs a = stem_s2d_args(Nb, H2, N);
  a.A = x2; a.W = w2; a.out = y; a.part = part;
  const Geom g = igemm_geom(a.Mc, N, 256, 16, 1);
  a.nmt = g.nmt;
  if (g.BM == 128 && g.BN == 128) launch_glds_t<CM_FWD, CE_FWD, 128, 128, 2, 64, true>(a, g, stream);
  else if (g.BM == 128 && g.BN == 64) launch_glds_t<CM_FWD, CE_FWD, 128, 64, 2, 64, true>(a, g, stream);
  else if (g.BM == 64 && g.BN == 128) launch_glds_t<CM_FWD, CE_FWD, 64, 128, 2, 64, true>(a, g, stream);
  else launch_glds_t<CM_FWD, CE_FWD, 64, 64, 2, 64, true>(a, g, stream);
}

long long conv_wgrad_s2d_workspace_floats(int Nb, int H2, int N) {
  const WgGeom g = wg_geom(N, 256, Nb * H2 * H2);
  return (long long)(g.nsplit + colsum_rows(g.nsplit)) * N * 256 + (long long)N * 256;
}

void wgrad_reduce_defer(bool on);
bool wgrad_reduce_deferring();

// stem weight gradient grad [N][7][7][4] (fp32, overwritten) from dy = ga*G + gb*Y + gc
// ([Nb][H2][H2][N]) and the space-to-depth image x2 (register-staged split-M kernel, 16-B
// gathers), reduced into a [N][256] scratch and permuted back to the 7x7 layout
void launch_conv_wgrad_s2d(const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb, const float *gc,
                           const bf16_t *x2, float *ws, float *grad, int Nb, int H2, int N, hipStream_t stream) {
  const ConvArgs c = stem_s2d_args(Nb, H2, N);
  WgArgs a{};
  a.G = G; a.Y = Y; a.ga = ga; a.gb = gb; a.gc = gc; a.X = x2;
  a.N = N; a.Hi = c.Hi; a.Wi = c.Wi; a.Ci = c.Ci; a.Ho = c.Ho; a.Wo = c.Wo;
  a.R = c.R; a.S = c.S; a.stride = 1; a.pad = c.pad; a.Kw = 256; a.M = c.Mc;
  const WgGeom g = wg_geom(N, 256, a.M);
  a.rows_per_split = g.rows;
  float *g2 = ws + (size_t)(g.nsplit + colsum_rows(g.nsplit)) * N * 256;
  a.out = g.nsplit == 1 ? g2 : ws;
  const dim3 grid((N + g.TN - 1) / g.TN, (256 + g.TK - 1) / g.TK, g.nsplit);
  const bool dm = Y == nullptr;
#define WGS_L(TN_, TK_)                                                                                        \
  do {                                                                                                        \
    if (dm) hipLaunchKernelGGL((conv_wgrad_kernel<CP_NONE, TN_, TK_, 8, true>), grid, dim3(256), 0, stream, a);  \
    else hipLaunchKernelGGL((conv_wgrad_kernel<CP_NONE, TN_, TK_, 8, false>), grid, dim3(256), 0, stream, a);    \
  } while (0)
  if (g.TN == 128) WGS_L(128, 128); else WGS_L(64, 128);
#undef WGS_L
  if (g.nsplit > 1) {
    const bool deferring = wgrad_reduce_deferring();   // the permute below reads g2 right away
    wgrad_reduce_defer(false);
    launch_wgrad_reduce(ws, g.nsplit, (long long)N * 256, g2, stream);
    wgrad_reduce_defer(deferring);
  }
  hipLaunchKernelGGL(stem_wgrad_s2d_kernel, dim3((N * 196 + 255) / 256), dim3(256), 0, stream, g2, grad, N);
}

// BN materialisation (bn_mat_kernel): mode 0 act = relu(Y*a + b); mode 1 dy = a*G + b*Y + c
void launch_bn_mat(int mode, const bf16_t *G, const bf16_t *Y, const float *a, const float *b, const float *c,
                   bf16_t *out, int M, int C, hipStream_t stream) {
  const BnFin *lz = take_bn_lz();
  const int C8 = C / 8, rpi = 256 / C8;
  long long blocks = ((long long)M + rpi * 4 - 1) / (rpi * 4);
  // lazy: every workgroup finalizes all C channels (16 replica-row loads each), so fewer
  // (grid-stride) workgroups on the wide layers
  const long long cap = lz && C > 256 ? 512 : 2048;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  const size_t lds = lz ? (size_t)(mode == 1 ? 3 : 2) * C * sizeof(float) : 0;
#define BNM(MODE_)                                                                                             \
  if (lz) hipLaunchKernelGGL((bn_mat_kernel<MODE_, true>), dim3((unsigned)blocks), dim3(256), lds, stream, G, Y, a, \
                             b, c, out, M, C, lz);                                                             \
  else hipLaunchKernelGGL((bn_mat_kernel<MODE_, false>), dim3((unsigned)blocks), dim3(256), 0, stream, G, Y, a, b, \
                          c, out, M, C, lz);
  if (mode == 1) { BNM(1) } else { BNM(0) }
#undef BNM
}
