// Pointwise (1x1) conv GEMM for the small-M layers (14x14 and 7x7 feature maps,
// M = 25,088 / 6,272 at batch 128) — forward and dgrad, same fused BN prologue /
// epilogue contract as pw_gemm_kernel (pwconv.hip).
//
// At these shapes K and N (64 .. 1280) are no longer tiny next to M, so the
// operands are re-read by many workgroups and a classic two-operand LDS tiling
// wins over the row-stream kernel: BM x BN output tile per workgroup (4 waves in
// a 2 x 2 arrangement, each (BM/2) x (BN/2) of v_mfma_f32_16x16x32_bf16 tiles),
// k-steps of 32 or 64 with both operand tiles double-buffered in LDS and the next
// step's global loads in flight during the current step's MFMAs.  The BN
// prologue (ReLU6(BN) of the producer, or this layer's BN backward
// a*G + b*Y + c) is applied once per element while staging A.  Workgroup ids
// put the N tiles of an M tile 8 ids apart (same XCD, dispatched together) so
// the A tile is fetched from HBM once into that XCD's L2.
//
// (Split-K over workgroups for the long-K 7x7 / 14x14 layers was built and measured slower --
// 5.30 vs 4.70 ms/step, the fp32 slab round trip outweighs the shorter k chains -- and removed;
// docs/PERF_NOTES.md round 4.)
#include "../bnfin.h"


enum { PRO_BNBWD_T = 3, PRO_BNRES_T = 5 };
enum { EPI_FWD_T = 0, EPI_BWD_RELU6_T = 1, EPI_BWD_LIN_T = 2 };

// Phase trace (diagnostics builds only, PGDIST_DEFINES=PGDIST_PWT_TRACE): thread 0 of every
// workgroup stamps the wall clock (100 MHz) at the phase boundaries into g_pwt_ts[wg][8]
#ifdef PGDIST_PWT_TRACE
__device__ unsigned long long *g_pwt_ts = nullptr;
#define PWT_MARK(k)                                                                              \
  do {                                                                                           \
    if (threadIdx.x == 0) {                                                                      \
      unsigned long long *t_ = g_pwt_ts;                                                         \
      if (t_) t_[(size_t)blockIdx.x * 8 + (k)] = wall_clock64();                                 \
    }                                                                                            \
  } while (0)
#else
#define PWT_MARK(k) ((void)0)
#endif

namespace {
struct PwTArgs {
  const bf16_t *A;      // [M][K]
  const bf16_t *A2;     // [M][K] (Y for the BN backward prologue)
  const float *pa, *pb, *pc;
  const bf16_t *W;      // [N][K]
  bf16_t *out;          // [M][N]
  const bf16_t *Yt;     // [M][N]
  const float *es, *et;
  const bf16_t *R;      // [M][N]
  float *part;          // [nmt][2][N]
  int M, N, K;
  bf16_t *Aout;         // optional [M][K]: transformed A (block output), written by N-tile 0
  const uint8_t *W8;    // F8: e4m3 weights [N][ldw8] (k zero-padded), dequant scale wsc[n]
  const float *wsc;
  float asc;            // F8: the prologue output is scaled by asc before its e4m3 conversion
  int ldw8;
  int bn_rep;           // BN-statistics replica rows (g_bn_rep)
  const BnFin *fin;     // fused BN finalize in the tail (nullptr: none)
  const BnFin *lz;      // lazy finalize of the prologue parameters (nullptr: materialised pa/pb/pc)
};
}  // namespace

// KSTEP: k per pipeline step (32, or 64 for long K: half the steps / barriers, twice the
// bytes in flight per step)
// F8: forward in e4m3 (v_mfma_f32_16x16x32_fp8_fp8): A is converted to e4m3 after the
// prologue while it is staged, B is staged from the e4m3 weight copy; both LDS tiles are
// half the bytes of the bf16 ones.  F8 with KSTEP = 128: one block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16 fragment and k step (e4m3 x e4m3, unit E8M0
// scales: the per-channel scales stay in the epilogue), the gfx950 double-rate fp8 form; lane l
// holds A[row l & 15][k 32 (l >> 4) .. +31] and B[k 32 (l >> 4) .. +31][col l & 15], 32
// contiguous bytes of a staged row each.
template <int PRO, int EPI, int BM, int BN, int KSTEP, bool F8 = false>
__global__ __launch_bounds__(256) void pw_tile_kernel(PwTArgs p) {
  static_assert(!F8 || (EPI == EPI_FWD_T && PRO != PRO_BNBWD_T && PRO != PRO_BNRES_T), "fp8: forward only");
  constexpr int kLDK = KSTEP + 8;                      // staged operand row pitch (bf16)
  constexpr int kLDK8 = KSTEP + 16;                    // F8 staged row pitch (bytes)
  constexpr int B8CH = BN * KSTEP / 16, B8PT = (B8CH + 255) / 256;   // F8 16-B weight chunks
  constexpr int KCH = KSTEP / 8;                       // 16-B chunks per staged row
  constexpr int NPAR = PRO == ACT_NONE ? 0 : (PRO == PRO_BNBWD_T ? 3 : 2);
  constexpr int RT = BM / 32, CTW = BN / 32;          // per-wave 16x16 tiles (rows, cols)
  constexpr int ACH = BM * KCH / 256, BCH = BN * KCH / 256;
  constexpr int LDC = BN + 8;
  constexpr int CH = BN / 8, RSTEP = 256 / CH, NP = BM / RSTEP;
  constexpr int EB = NP < 4 ? NP : 4;
  static_assert(ACH >= 1 && BCH >= 1 && NP >= 1, "tile too small for 256 threads");
  PWT_MARK(0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t *As = reinterpret_cast<bf16_t *>(smem);                         // [2][BM][kLDK]
  bf16_t *Bs = As + 2 * BM * kLDK;                                       // [2][BN][kLDK]
  uint8_t *As8 = reinterpret_cast<uint8_t *>(smem);                      // F8: [2][BM][kLDK8]
  uint8_t *Bs8 = As8 + 2 * BM * kLDK8;                                   // F8: [2][BN][kLDK8]
  float *Ps = F8 ? reinterpret_cast<float *>(Bs8 + 2 * BN * kLDK8)
                 : reinterpret_cast<float *>(Bs + 2 * BN * kLDK);        // [NPAR][Kp]
  bf16_t *Cs = reinterpret_cast<bf16_t *>(smem);                         // [BM][LDC] (after the K loop)
  float *Red = reinterpret_cast<float *>(smem);                          // [RSTEP][BN] (at the end)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int NT = (p.N + BN - 1) / BN;
  const int nmt = (p.M + BM - 1) / BM;
  // workgroup -> (mt, nt): the NT workgroups of one M tile are 8 ids apart (same XCD)
  int mt, nt;
  {
    const int NTS = NT;
    const int L = blockIdx.x, full = (nmt / 8) * 8 * NTS;
    int j;
    if (L < full) {
      mt = (L / (8 * NTS)) * 8 + L % 8;
      j = (L / 8) % NTS;
    } else {
      const int rem = nmt % 8, Lr = L - full;
      mt = (nmt / 8) * 8 + Lr % rem;
      j = Lr / rem;
    }
    nt = j;
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int Kp = (p.K + KSTEP - 1) / KSTEP * KSTEP;
  const int kb = 0, ke = Kp / KSTEP;                    // k steps [kb, ke)

  constexpr bool HAS_A2 = PRO == PRO_BNBWD_T || PRO == PRO_BNRES_T;
  constexpr bool AOUT = EPI == EPI_FWD_T && (PRO == PRO_BNRES_T || PRO == ACT_BN);
  // PF2 (64-row tiles with 64-wide k steps: the long-K project / dgrad GEMMs, K >= 256): two
  // register sets, the loads of step ks + 2 issued while step ks + 1's land in the other set
  // (two k steps of global-load latency hidden instead of one).  Elsewhere one set: the
  // 128-row tiles would double their VGPRs, and K < 256 is at most 8 steps.
  constexpr bool PF2 = BM == 64 && KSTEP == 64 && !F8;
  uint4 ra0[ACH], ry0[HAS_A2 ? ACH : 1], rb0[F8 ? B8PT : BCH];
  uint4 ra1[PF2 ? ACH : 1], ry1[PF2 && HAS_A2 ? ACH : 1], rb1[PF2 ? BCH : 1];
  // bounds-checked buffer loads issued unconditionally (masked: out-of-range offset, reads 0),
  // so the one-step-ahead prefetch is not drained by a vmcnt(0) at a branch join
  const rsrc_t rA = make_rsrc(p.A, (uint32_t)((size_t)p.M * p.K * 2));
  const rsrc_t rA2 = make_rsrc(HAS_A2 ? p.A2 : p.A, (uint32_t)((size_t)p.M * p.K * 2));
  const rsrc_t rW = F8 ? make_rsrc(p.W8, (uint32_t)((size_t)p.N * p.ldw8)) : make_rsrc(p.W, (uint32_t)((size_t)p.N * p.K * 2));
  auto load = [&](auto &ra, auto &ry, auto &rb, int k0, bool valid) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, row = c / KCH, kk = (c % KCH) * 8;
      const int gr = m0 + row, k = k0 + kk;
      const uint32_t off = boff(valid && gr < p.M && k < p.K, (size_t)gr * p.K + k);
      ra[i] = bld16(rA, off);
      if constexpr (HAS_A2) ry[i] = bld16(rA2, off);
    }
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < B8PT; ++i) {
        const int c = tid + i * 256, n = c / (KSTEP / 16), kk = (c % (KSTEP / 16)) * 16;
        const int gn = n0 + n;
        const bool ok = valid && c < B8CH && gn < p.N && k0 + kk < p.ldw8;
        rb[i] = bld16(rW, ok ? (uint32_t)((size_t)gn * p.ldw8 + k0 + kk) : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int c = tid + i * 256, n = c / KCH, kk = (c % KCH) * 8;
        const int gn = n0 + n, k = k0 + kk;
        rb[i] = bld16(rW, boff(valid && gn < p.N && k < p.K, (size_t)gn * p.K + k));
      }
    }
  };
  auto write = [&](const auto &ra, const auto &ry, const auto &rb, int buf, int k0) {
    bf16_t *Ab = As + buf * BM * kLDK;
    bf16_t *Bb = Bs + buf * BN * kLDK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, row = c / KCH, kk = (c % KCH) * 8;
      uint4 v = ra[i];
      if constexpr (PRO != ACT_NONE) {
        const int k = k0 + kk;
        float x[8];
        unpack8(ra[i], x);
        if constexpr (PRO == PRO_BNBWD_T) {
          float y[8];
          unpack8(ry[i], y);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = fmaf(Ps[k + j], x[j], fmaf(Ps[Kp + k + j], y[j], Ps[2 * Kp + k + j]));
        } else if constexpr (PRO == PRO_BNRES_T) {
          float r[8];
          unpack8(ry[i], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], Ps[k + j], Ps[Kp + k + j]) + r[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = act_apply<PRO>(x[j], Ps[k + j], Ps[Kp + k + j]);
        }
        if constexpr (F8) {
          const long q = pack_fp8x8(x, p.asc);
          *reinterpret_cast<long *>(As8 + (buf * BM + row) * kLDK8 + kk) = q;
          continue;
        }
        v = pack8(x);
        // materialise the block output once (N-tile 0); compiled only into the consumer forms
        // that take one (a possibly-issued store in the k loop shares the vmcnt queue with the
        // prefetch loads, and the waitcnt pass then drains the queue at the loop header)
        if (AOUT && p.Aout && nt == 0) {
          const int gr = m0 + row;
          if (gr < p.M && k < p.K) stg16(p.Aout + (size_t)gr * p.K + k, v);
        }
      }
      if constexpr (F8) {   // ACT_NONE: convert the raw bf16 A
        float x[8];
        unpack8(v, x);
        *reinterpret_cast<long *>(As8 + (buf * BM + row) * kLDK8 + kk) = pack_fp8x8(x, p.asc);
      } else {
        *reinterpret_cast<uint4 *>(Ab + row * kLDK + kk) = v;
      }
    }
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < B8PT; ++i) {
        const int c = tid + i * 256, n = c / (KSTEP / 16), kk = (c % (KSTEP / 16)) * 16;
        if (c < B8CH) *reinterpret_cast<uint4 *>(Bs8 + (buf * BN + n) * kLDK8 + kk) = rb[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int c = tid + i * 256, n = c / KCH, kk = (c % KCH) * 8;
        *reinterpret_cast<uint4 *>(Bb + n * kLDK + kk) = rb[i];
      }
    }
  };

  f32x4_t acc[RT][CTW];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CTW; ++c) acc[r][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // first operand loads (PF2: first two steps) in flight during the prologue-parameter staging
  load(ra0, ry0, rb0, kb * KSTEP, kb < ke);
  if constexpr (PF2) load(ra1, ry1, rb1, min(kb + 1, ke - 1) * KSTEP, true);
  // parameter chunks staged with one memory latency: K < 256 (32-wide k steps) needs one; the
  // long-K 64 x 64 tiles take K up to 1280, the 64 x 128 ones (N = 96) up to 576; more would
  // cost the wider tiles occupancy
  constexpr int PMAX = KSTEP == 32 ? 1 : (BM == 64 ? (BN == 64 ? 5 : 3) : 2);
  if constexpr (NPAR > 0) bn_stage_params<NPAR, PMAX>(p.lz, p.pa, p.pb, p.pc, p.K, Kp, Ps);
  __syncthreads();   // Ps staged
  PWT_MARK(1);
  write(ra0, ry0, rb0, 0, kb * KSTEP);
  __syncthreads();
  PWT_MARK(2);
  auto step = [&](int buf) {   // MFMAs of the k step staged in LDS buffer buf
    const bf16_t *Ab = As + buf * BM * kLDK;
    const bf16_t *Bb = Bs + buf * BN * kLDK;
    if constexpr (F8 && KSTEP == 128) {
      const uint8_t *A8 = As8 + buf * BM * kLDK8, *B8 = Bs8 + buf * BN * kLDK8;
      i32x8_t af[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const uint4 *q = reinterpret_cast<const uint4 *>(A8 + (wm * (BM / 2) + r * 16 + (lane & 15)) * kLDK8 +
                                                         32 * (lane >> 4));
        const uint4 lo = q[0], hi = q[1];
        af[r] = i32x8_t{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int c = 0; c < CTW; ++c) {
        const uint4 *q = reinterpret_cast<const uint4 *>(B8 + (wn * (BN / 2) + c * 16 + (lane & 15)) * kLDK8 +
                                                         32 * (lane >> 4));
        const uint4 lo = q[0], hi = q[1];
        const i32x8_t bf = i32x8_t{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w,
                                   (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
#pragma unroll
        for (int r = 0; r < RT; ++r)   // formats 0 / 0: e4m3 x e4m3; scales 0x7f = 2^0 in every byte
          acc[r][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[r], bf, acc[r][c], 0, 0, 0, 0x7f7f7f7f,
                                                                       0, 0x7f7f7f7f);
      }
    } else
#pragma unroll
    for (int sub = 0; sub < KSTEP / 32; ++sub) {
      if constexpr (F8) {
        const uint8_t *A8 = As8 + buf * BM * kLDK8, *B8 = Bs8 + buf * BN * kLDK8;
        long af8[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r)
          af8[r] = *reinterpret_cast<const long *>(A8 + (wm * (BM / 2) + r * 16 + (lane & 15)) * kLDK8 + sub * 32 +
                                                   8 * (lane >> 4));
#pragma unroll
        for (int c = 0; c < CTW; ++c) {
          const long bf8 = *reinterpret_cast<const long *>(B8 + (wn * (BN / 2) + c * 16 + (lane & 15)) * kLDK8 +
                                                           sub * 32 + 8 * (lane >> 4));
#pragma unroll
          for (int r = 0; r < RT; ++r)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af8[r], bf8, acc[r][c], 0, 0, 0);
        }
        continue;
      }
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
        for (int r = 0; r < RT; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[r]),
                                                              __builtin_bit_cast(bf16x8_t, bf), acc[r][c], 0, 0, 0);
      }
    }
  };
  if constexpr (PF2) {
    // two k steps per iteration so each register set has a static index.  Every load is
    // issued unconditionally (past the end: the last step again, never used) -- a load under a
    // wave-uniform branch makes the loop header join paths with different loads in flight,
    // where the waitcnt pass then drains the queue (vmcnt(0)) and the second stage is lost
    for (int ks = kb; ks < ke; ks += 2) {
      load(ra0, ry0, rb0, min(ks + 2, ke - 1) * KSTEP, true);
      step(0);
      if (ks + 1 < ke) write(ra1, ry1, rb1, 1, (ks + 1) * KSTEP);
      __syncthreads();
      if (ks + 1 >= ke) break;
      load(ra1, ry1, rb1, min(ks + 3, ke - 1) * KSTEP, true);
      step(1);
      if (ks + 2 < ke) write(ra0, ry0, rb0, 0, (ks + 2) * KSTEP);
      __syncthreads();
    }
  } else {
    for (int ks = kb; ks < ke; ++ks) {   // one step ahead
      const int buf = (ks - kb) & 1;
      load(ra0, ry0, rb0, (ks + 1) * KSTEP, ks + 1 < ke);
      step(buf);
      if (ks + 1 < ke) write(ra0, ry0, rb0, buf ^ 1, (ks + 1) * KSTEP);
      __syncthreads();
    }
  }

  PWT_MARK(3);
  {
  // ---- epilogue: bf16 C tile in LDS, then 16-B row chunks (same contract as pw_gemm_kernel)
#pragma unroll
  for (int c = 0; c < CTW; ++c) {
    const int col = wn * (BN / 2) + c * 16 + (lane & 15);
    const float csc = (F8 && n0 + col < p.N) ? p.wsc[n0 + col] / p.asc : 1.f;
#pragma unroll
    for (int r = 0; r < RT; ++r)
      frag_store_bf16(Cs, LDC, wm * (BM / 2) + r * 16, wn * (BN / 2) + c * 16, acc[r][c][0] * csc,
                      acc[r][c][1] * csc, acc[r][c][2] * csc, acc[r][c][3] * csc);
  }
  __syncthreads();
  const int my_chunk = tid % CH, ncol0 = n0 + my_chunk * 8;
  float st0[8], st1[8], es[8], et[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st0[j] = st1[j] = 0.f;
    es[j] = (EPI == EPI_BWD_RELU6_T && ncol0 + j < p.N) ? p.es[ncol0 + j] : 0.f;
    et[j] = (EPI == EPI_BWD_RELU6_T && ncol0 + j < p.N) ? p.et[ncol0 + j] : 0.f;
  }
#pragma unroll
  for (int i0 = 0; i0 < NP; i0 += EB) {
    uint4 ytr[EB], rsr[EB];
    if constexpr (EPI != EPI_FWD_T) {
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        const int rr = tid / CH + (i0 + e) * RSTEP, row = m0 + rr;
        const bool ok = row < p.M && ncol0 < p.N;
        const size_t off = (size_t)row * p.N + ncol0;
        ytr[e] = ok ? ldg16(p.Yt + off) : make_uint4(0, 0, 0, 0);
        if constexpr (EPI == EPI_BWD_LIN_T) rsr[e] = (ok && p.R) ? ldg16(p.R + off) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int rr = tid / CH + (i0 + e) * RSTEP, row = m0 + rr;
      if (row < p.M && ncol0 < p.N) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4 *>(Cs + rr * LDC + my_chunk * 8), v);
        if constexpr (EPI == EPI_FWD_T) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            st0[j] += v[j];
            st1[j] = fmaf(v[j], v[j], st1[j]);
          }
        } else {
          float yt[8];
          unpack8(ytr[e], yt);
          if constexpr (EPI == EPI_BWD_RELU6_T) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] *= relu6_mask(yt[j], es[j], et[j]);
          } else {
            float rv[8];
            unpack8(rsr[e], rv);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += rv[j];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            st0[j] += v[j];
            st1[j] = fmaf(v[j], yt[j], st1[j]);
          }
        }
        stg16(p.out + (size_t)row * p.N + ncol0, pack8(v));
      }
    }
  }
  __syncthreads();
  PWT_MARK(4);
  // ---- BN partials of this tile's columns -> part[mt][2][N]
  for (int s = 0; s < 2; ++s) {
    const int rgrp = tid / CH;
#pragma unroll
    for (int j = 0; j < 8; ++j) Red[rgrp * BN + my_chunk * 8 + j] = s == 0 ? st0[j] : st1[j];
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      float a = 0.f;
      for (int g = 0; g < RSTEP; ++g) a += Red[g * BN + c];
      if (n0 + c < p.N) bn_part_add(p.part, mt, nmt, p.bn_rep, p.N, s, n0 + c, a);
    }
    __syncthreads();
  }
  }
  PWT_MARK(5);
  bn_fin_tail(p.fin);
  PWT_MARK(6);
}

// ===========================================================================
// host side
// ===========================================================================
namespace {
struct TileGeom {
  int BM, BN, KS, nmt, nt;
  size_t lds;
};

// Tile shape by a shape rule, from the per-op tile sweep of the 14x14 / 7x7 MobileNetV2 GEMMs
// (profiles/r4_pw_tile_sweep.txt; the earlier "largest tile with >= 384 workgroups" heuristic,
// 32-row tiles and 128-wide k steps measured slower, docs/PERF_NOTES.md round 4):
//   N > K (expand-shaped): 128 x 64, or 128 x 128 when N*K >= 300k (1280x320, 960x320);
//   N <= K (project / long-K): 64 rows, 128 columns when one tile covers an N of 65..127
//   (N = 96), else 64 (N = 64, 160, 320: 64-wide column tiles waste less than 128-wide ones);
// 64-wide k steps from K >= 256.
TileGeom tile_geom(int M, int N, int K, int pro) {
  TileGeom g{};
  if (N > K) {
    g.BM = 128;
    g.BN = (long long)N * K >= 300000 ? 128 : 64;
  } else {
    g.BM = 64;
    g.BN = (N > 64 && N < 128) ? 128 : 64;
  }
  g.nmt = (M + g.BM - 1) / g.BM;
  g.nt = (N + g.BN - 1) / g.BN;
  g.KS = K >= 256 ? 64 : 32;
  const int npar = pro == ACT_NONE ? 0 : (pro == PRO_BNBWD_T ? 3 : 2);
  const size_t kp = (size_t)((K + g.KS - 1) / g.KS * g.KS);
  const size_t ops = (size_t)2 * (g.BM + g.BN) * (g.KS + 8) * 2;
  const size_t ctile = (size_t)g.BM * (g.BN + 8) * 2;
  const size_t red = (size_t)(256 / (g.BN / 8)) * g.BN * 4;
  size_t body = ops > ctile ? ops : ctile;
  if (red > body) body = red;
  g.lds = body + npar * kp * 4;
  return g;
}

template <int PRO, int EPI, int BM, int BN, bool F8>
void launch_tile_t(PwTArgs a, const TileGeom &g, hipStream_t st) {
  const dim3 grid(g.nmt * g.nt);
  if constexpr (F8) {
    if (g.KS == 128) {
      hipLaunchKernelGGL((pw_tile_kernel<PRO, EPI, BM, BN, 128, F8>), grid, dim3(256), g.lds, st, a);
      return;
    }
  }
  if (g.KS == 64) hipLaunchKernelGGL((pw_tile_kernel<PRO, EPI, BM, BN, 64, F8>), grid, dim3(256), g.lds, st, a);
  else hipLaunchKernelGGL((pw_tile_kernel<PRO, EPI, BM, BN, 32, F8>), grid, dim3(256), g.lds, st, a);
}

template <int PRO, int EPI, bool F8 = false>
void launch_tile_pe(const PwTArgs &a, const TileGeom &g, hipStream_t st) {
  if (g.BM == 128 && g.BN == 128) launch_tile_t<PRO, EPI, 128, 128, F8>(a, g, st);
  else if (g.BM == 64 && g.BN == 128) launch_tile_t<PRO, EPI, 64, 128, F8>(a, g, st);
  else if (g.BM == 128 && g.BN == 64) launch_tile_t<PRO, EPI, 128, 64, F8>(a, g, st);
  else launch_tile_t<PRO, EPI, 64, 64, F8>(a, g, st);
}
}  // namespace

void pwt_trace_set(void *ts) {   // nullptr: off; no-op unless built with PGDIST_PWT_TRACE
#ifdef PGDIST_PWT_TRACE
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pwt_ts), &ts, sizeof(ts));
#else
  (void)ts;
#endif
}

// BN partial rows: one per M tile of the smallest tile height any launch picks (64 rows)
int pw_tile_num_partials(int M, int N, int K) { return (M + 63) / 64; }

void launch_pw_tile(int pro, int epi, const bf16_t *A, const bf16_t *A2, const float *pa, const float *pb,
                    const float *pc, const bf16_t *W, bf16_t *out, const bf16_t *Yt, const float *es,
                    const float *et, const bf16_t *R, float *part, int M, int N, int K, bf16_t *Aout,
                    hipStream_t st) {
  PwTArgs a{A, A2, pa, pb, pc, W, out, Yt, es, et, R, part, M, N, K, Aout};
  a.bn_rep = g_bn_rep;
  a.fin = take_bn_fin();
  a.lz = take_bn_lz();
  const TileGeom g = tile_geom(M, N, K, pro);
#define PT_CASE(P, E) \
  if (pro == P && epi == E) { launch_tile_pe<P, E>(a, g, st); return; }
  PT_CASE(ACT_NONE, EPI_FWD_T)
  PT_CASE(ACT_BN_RELU6, EPI_FWD_T)
  PT_CASE(ACT_BN, EPI_FWD_T)
  PT_CASE(PRO_BNRES_T, EPI_FWD_T)
  PT_CASE(PRO_BNBWD_T, EPI_BWD_RELU6_T)
  PT_CASE(PRO_BNBWD_T, EPI_BWD_LIN_T)
#undef PT_CASE
}

// the double-rate block-scaled fp8 MFMA in the tile path (128-wide k steps): 2 (default) on the
// <= 64-row tiles, 1 on every tile, 0: the 16x16x32 fp8 MFMA (pw_f8_set_mx: tests).  bs512, one
// box: 14.889-14.900 (2) vs 14.923-14.967 (1) vs 14.896-14.940 (0) vs bf16 14.906-14.919 ms/step
// (profiles/r4_fp8_mx_bs512_ab.txt)
static int g_f8_mx = 2;
void pw_f8_set_mx(int on) { g_f8_mx = on; }
int pw_f8_mx() { return g_f8_mx; }

void launch_pw_tile_f8(int pro, const bf16_t *A, const float *pa, const float *pb, const uint8_t *W8, int ldw8,
                       const float *wsc, float asc, bf16_t *out, float *part, int M, int N, int K,
                       hipStream_t st) {
  PwTArgs a{A, nullptr, pa, pb, nullptr, nullptr, out, nullptr, nullptr, nullptr, nullptr, part, M, N, K,
            nullptr, W8, wsc, asc, ldw8, g_bn_rep, take_bn_fin(), take_bn_lz()};
  TileGeom g = tile_geom(M, N, K, pro);   // the bf16 LDS size bounds the e4m3 one at KS <= 64
  // mode 2: only the <= 64-row tiles (the 128-row ones need 157-202 VGPRs at KSTEP 128)
  if (g_f8_mx && (g_f8_mx == 1 || g.BM <= 64)) {
    g.KS = 128;
    const int npar = pro == ACT_NONE ? 0 : 2;
    const size_t kp = (size_t)((K + 127) / 128 * 128);
    const size_t ops = (size_t)2 * (g.BM + g.BN) * (128 + 16);
    const size_t ctile = (size_t)g.BM * (g.BN + 8) * 2;
    const size_t red = (size_t)(256 / (g.BN / 8)) * g.BN * 4;
    size_t body = ops > ctile ? ops : ctile;
    if (red > body) body = red;
    g.lds = body + npar * kp * 4;
  }
  if (pro == ACT_NONE) launch_tile_pe<ACT_NONE, EPI_FWD_T, true>(a, g, st);
  else if (pro == ACT_BN_RELU6) launch_tile_pe<ACT_BN_RELU6, EPI_FWD_T, true>(a, g, st);
  else if (pro == ACT_BN) launch_tile_pe<ACT_BN, EPI_FWD_T, true>(a, g, st);
}
