// Pointwise (1x1) convolution as an MFMA bf16 GEMM with fused BatchNorm
// prologue/epilogue, NHWC:  C[M][N] = act(A)[M][K] . W[N][K]^T,  M = B*H*W.
//
// Reference ops: the 16 expand + 17 project + final 1x1 convs of MobileNetV2
// (shapes M in {6,272 .. 1,605,632}, K,N in {16 .. 1280}).
// These shapes are memory-bound on MI355X (K and N are tiny next to M), so the
// kernel is organised as a row stream:
//
//  * 256-thread workgroup = 4 waves x 32 rows; each wave owns 2 x (BN/16)
//    v_mfma_f32_16x16x32_bf16 tiles, N tile BN in {32,64};
//  * the A fragment (lane: row l&15, k = 8*(l>>4)..+7) is one 16-B global load
//    per lane, issued one 64-k step AHEAD (also across M tiles of the
//    grid-stride sweep) and transformed in registers by the fused prologue
//    (per-k parameters staged in LDS):
//      ACT_NONE      A as stored (materialised block output)
//      ACT_BN_RELU6  relu6(A*s[k]+t[k])      -- producer BN + ReLU6 (forward)
//      PRO_BNBWD     a[k]*G + b[k]*Y + c[k]   -- this layer's BN backward (dgrad,
//                    with the transposed weight produced by wt_transpose_kernel)
//  * large M / small K (K <= 192): the whole weight tile [BN][K] is resident in
//    LDS (padded rows -> conflict-free ds_read_b128) for the grid-stride sweep
//    over M tiles (gridDim.x a multiple of 8, so the N tiles of one M tile share
//    an XCD L2);
//  * small M (14x14 / 7x7 layers) or large K: weight fragments are prefetched
//    straight from L2 like A, and K is split over the 4 waves (KS = 2 or 4,
//    M tile 64 or 32 rows) so the grid keeps >= ~1.5k workgroups; the KS fp32
//    partial tiles are summed in a fixed order in LDS (deterministic);
//  * the epilogue goes through an LDS tile so every global load/store is a
//    coalesced 16-B row chunk:
//      EPI_FWD       store y, partial (sum y, sum y^2) for this layer's BN
//      EPI_BWD_RELU6 g = c * 1[0 < yt*s+t < 6], partial (sum g, sum g*yt)
//      EPI_BWD_LIN   g = c (+ R residual grad),  partial (sum g, sum g*yt)
//
// The weight gradient dW[N][K] = sum_m dy[m][n] x[m][k] reduces over M; it is
// a split-M MFMA kernel whose operands are staged TRANSPOSED in LDS (4 rows of
// m packed per ds_write_b64) so both fragments are plain ds_read_b128.
#include "../bnfin.h"

#include <cstdlib>

enum { PRO_BNBWD = 3, IM2COL_STEM = 4, PRO_BNRES = 5 };
// PRO_BNRES: A = A*s + t + A2 (the linear BN of a block output plus its residual): the block
// output is materialised by its consumer GEMM (Aout) instead of a separate BN-apply pass
enum { EPI_FWD = 0, EPI_BWD_RELU6 = 1, EPI_BWD_LIN = 2 };

namespace {
constexpr int kBPad = 8;       // bf16 pad per staged weight row (16 B)
constexpr int kCPad = 8;       // bf16 pad per staged C row

struct PwArgs {
  const bf16_t *A;      // [M][K]
  const bf16_t *A2;     // [M][K] (Y for PRO_BNBWD)
  const float *pa;      // prologue per-k params: s | a
  const float *pb;      // t | b
  const float *pc;      // - | c
  const bf16_t *W;      // [N][K]
  bf16_t *out;          // [M][N]
  const bf16_t *Yt;     // [M][N] epilogue BN input (bwd modes)
  const float *es;      // epilogue per-n scale (relu6 mask)
  const float *et;      // epilogue per-n shift
  const bf16_t *R;      // [M][N] residual gradient (EPI_BWD_LIN, optional)
  float *part;          // [gridDim.x][2][N]
  int M, N, K;
  bf16_t *Aout;         // optional [M][K]: the transformed A (block output), written by N-tile 0
  // fp8 forward (F8 instantiations): e4m3 weights [N][ldw8] (zero-padded k), per-n dequant
  // scale wsc[n]; the prologue output is multiplied by asc before its e4m3 conversion
  const uint8_t *W8;
  const float *wsc;
  float asc;
  int ldw8;
  int bn_rep;           // BN-statistics replica rows (g_bn_rep)
  const BnFin *fin;     // fused BN finalize in the tail (nullptr: none)
  const BnFin *lz;      // lazy finalize of the prologue parameters pa/pb(/pc) (nullptr: materialised)
};
}  // namespace

// transform one raw 16-B A fragment (8 consecutive k of one row) by the fused prologue;
// per-k parameters come from LDS (zero for k >= K, so padded k stay exactly 0)
template <int PRO>
PG_DEVICE void a_transform_f(const uint4 &raw, const uint4 &raw2, const float *Ps, int Kp, int kl, float (&v)[8]) {
  unpack8(raw, v);
  if constexpr (PRO != ACT_NONE) {
    const float4 a0 = *reinterpret_cast<const float4 *>(Ps + kl), a1 = *reinterpret_cast<const float4 *>(Ps + kl + 4);
    const float4 b0 = *reinterpret_cast<const float4 *>(Ps + Kp + kl), b1 = *reinterpret_cast<const float4 *>(Ps + Kp + kl + 4);
    const float aa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    if constexpr (PRO == PRO_BNBWD) {
      float y[8];
      unpack8(raw2, y);
      const float4 c0 = *reinterpret_cast<const float4 *>(Ps + 2 * Kp + kl), c1 = *reinterpret_cast<const float4 *>(Ps + 2 * Kp + kl + 4);
      const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(aa[j], v[j], fmaf(bb[j], y[j], cc[j]));
    } else if constexpr (PRO == PRO_BNRES) {
      float r[8];
      unpack8(raw2, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], aa[j], bb[j]) + r[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_apply<PRO>(v[j], aa[j], bb[j]);
    }
  }
}
template <int PRO>
PG_DEVICE s16x8_t a_transform(const uint4 &raw, const uint4 &raw2, const float *Ps, int Kp, int kl) {
  if constexpr (PRO == ACT_NONE) {
    return __builtin_bit_cast(s16x8_t, raw);
  } else {
    float v[8];
    a_transform_f<PRO>(raw, raw2, Ps, Kp, kl, v);
    return __builtin_bit_cast(s16x8_t, pack8(v));
  }
}

// Registers of one pipeline step (64 k) of a wave: A fragments for 2 sub-steps x 2
// row fragments (+ the Y operand of the BN backward), and with BDIRECT the weight
// fragments 2 sub-steps x CT column tiles.
template <int PRO, int SUBS, int CTB>
struct PwRaw {
  uint4 a[SUBS][2];
  uint4 y[(PRO == PRO_BNBWD || PRO == PRO_BNRES) ? SUBS : 1][2];
  uint4 b[SUBS][CTB > 0 ? CTB : 1];
  // keep the registers allocated up to here: the epilogue then cannot reuse them, so hipcc has
  // no write-after-write on registers a load may still target (it would wait vmcnt for the
  // next tile's prefetch, which is meant to land behind the epilogue)
  PG_DEVICE void hold() const {
#pragma unroll
    for (int i = 0; i < SUBS; ++i)
#pragma unroll
      for (int f = 0; f < 2; ++f) asm volatile("" ::"v"(a[i][f].x), "v"(a[i][f].y), "v"(a[i][f].z), "v"(a[i][f].w));
  }
};

// F8: e4m3 forward (v_mfma_f32_16x16x32_fp8_fp8): the weight tile is staged as e4m3
// bytes and each transformed A fragment is converted to e4m3 in registers; the fp32
// accumulators are dequantised by wsc[n] / asc before the bf16 C tile.
template <int PRO, int EPI, int BN, int KS, bool BDIRECT, bool F8 = false>
__global__ __launch_bounds__(256) void pw_gemm_kernel(PwArgs p) {
  static_assert(!F8 || (!BDIRECT && EPI == EPI_FWD && PRO != PRO_BNBWD && PRO != PRO_BNRES), "fp8: forward only");
  constexpr int CT = BN / 16;               // col tiles per wave
  constexpr int RG = 4 / KS;                // wave row groups (each 32 rows)
  constexpr int BM = 32 * RG;               // rows per M tile
  constexpr int CH = BN / 8;                // 16-B chunks per C row
  constexpr int RSTEP = 256 / CH;           // rows covered per epilogue pass
  // BN = 96 / 144 (one N tile over the whole expand width): 256 % CH != 0, the last
  // 256 - RSTEP * CH threads sit out the epilogue passes and the partial-sum reduction
  constexpr bool EP_ALL = RSTEP * CH == 256;
  constexpr int NP = (BM + RSTEP - 1) / RSTEP;
  constexpr int NPAR = PRO == ACT_NONE ? 0 : (PRO == PRO_BNBWD ? 3 : 2);
  constexpr bool HAS_A2 = PRO == PRO_BNBWD || PRO == PRO_BNRES;
  constexpr bool AOUT = PRO == PRO_BNRES || PRO == ACT_BN;   // consumers of a pending block output
  constexpr int SUBS = BDIRECT ? 1 : 2;     // 32-k MFMA sub-steps per pipeline step
  constexpr int KSTEP = 32 * SUBS;
  constexpr int EB = NP < 4 ? NP : 4;       // epilogue rows whose operands are loaded together
  constexpr int LDC = BN + kCPad;           // bf16 C tile pitch (KS == 1)
  constexpr int LDF = BN + 4;               // fp32 C partial pitch (KS > 1)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rg = wave % RG, kp = wave / RG;
  const int n0 = blockIdx.y * BN;
  const int Kp = (p.K + KSTEP - 1) / KSTEP * KSTEP;
  const int nsteps = Kp / KSTEP;
  const int LDB = Kp + kBPad;
  const int LDB8 = Kp + 16;                 // e4m3 weight row pitch (bytes)
  const int bs_bytes = BDIRECT ? 0 : (F8 ? BN * LDB8 : BN * LDB * 2);
  const int nmt = (p.M + BM - 1) / BM;
  bf16_t *Bs = reinterpret_cast<bf16_t *>(smem);                                      // [BN][LDB]
  uint8_t *Bs8 = reinterpret_cast<uint8_t *>(smem);                                   // [BN][LDB8] (F8)
  float *Ps = reinterpret_cast<float *>(smem + bs_bytes);                             // [NPAR][Kp]
  char *cbase = smem + bs_bytes + NPAR * Kp * 4;
  bf16_t *Cs = reinterpret_cast<bf16_t *>(cbase);                                      // [BM][LDC]
  float *Cf = reinterpret_cast<float *>(cbase);                                        // [KS][BM][LDF]
  float *Red = reinterpret_cast<float *>(cbase);                                       // [RSTEP][BN] (end)

  using Raw = PwRaw<PRO, SUBS, BDIRECT ? CT : 0>;
  // Bounds-checked buffer loads, issued unconditionally (masked lanes / the prefetch past the
  // last tile use an out-of-range offset and read 0): a load behind a branch makes hipcc wait
  // vmcnt(0) at the join, which drained this one-step-ahead prefetch right after issuing it.
  const rsrc_t rA = make_rsrc(p.A, (uint32_t)((size_t)p.M * p.K * 2));
  const rsrc_t rA2 = make_rsrc(HAS_A2 ? p.A2 : p.A, (uint32_t)((size_t)p.M * p.K * 2));
  const rsrc_t rW = make_rsrc(p.W, (uint32_t)((size_t)p.N * p.K * 2));
  auto load = [&](Raw &r, int m0, int s, bool valid) {
#pragma unroll
    for (int ss = 0; ss < SUBS; ++ss) {
      const int k = s * KSTEP + ss * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int row = m0 + rg * 32 + f * 16 + (lane & 15);
        const bool ok = valid && row < p.M && k < p.K;
        const uint32_t off = ok ? (uint32_t)(((size_t)row * p.K + k) * 2) : kOOB;
        r.a[ss][f] = bld16(rA, off);
        if constexpr (HAS_A2) r.y[ss][f] = bld16(rA2, off);
      }
      if constexpr (BDIRECT) {
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int n = n0 + c * 16 + (lane & 15);
          r.b[ss][c] = bld16(rW, (valid && n < p.N && k < p.K) ? (uint32_t)(((size_t)n * p.K + k) * 2) : kOOB);
        }
      }
    }
  };

  // the first A fragments are in flight during the weight / prologue-parameter staging below
  Raw cur, nxt;
  load(cur, blockIdx.x * BM, kp, blockIdx.x < nmt);

  // ---- stage the weight tile (once per workgroup) and the per-k prologue parameters
  if constexpr (F8) {
    const int per_row = Kp / 16;            // W8 rows are zero-padded to ldw8 >= Kp
    for (int i = tid; i < BN * per_row; i += 256) {
      const int r = i / per_row, c16 = (i % per_row) * 16;
      const int n = n0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < p.N) v = ldg16(p.W8 + (size_t)n * p.ldw8 + c16);
      *reinterpret_cast<uint4 *>(Bs8 + r * LDB8 + c16) = v;
    }
  } else if constexpr (!BDIRECT) {
    const int per_row = Kp / 8;
    for (int i = tid; i < BN * per_row; i += 256) {
      const int r = i / per_row, c8 = (i % per_row) * 8;
      const int n = n0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < p.N && c8 < p.K) v = ldg16(p.W + (size_t)n * p.K + c8);
      *reinterpret_cast<uint4 *>(Bs + r * LDB + c8) = v;
    }
  }
  if constexpr (NPAR > 0) {
    for (int i = tid; i < Kp; i += 256) {
      const bool ok = i < p.K;
      if (p.lz) {
        float a = 0.f, b = 0.f, c = 0.f;
        if (ok) bn_lazy(p.lz, i, a, b, c);
        Ps[i] = a;
        Ps[Kp + i] = b;
        if constexpr (NPAR == 3) Ps[2 * Kp + i] = c;
      } else {
        Ps[i] = ok ? p.pa[i] : 0.f;
        Ps[Kp + i] = ok ? p.pb[i] : 0.f;
        if constexpr (NPAR == 3) Ps[2 * Kp + i] = ok ? p.pc[i] : 0.f;
      }
    }
  }
  __syncthreads();

  const int my_chunk = tid % CH;            // fixed epilogue column chunk
  const int ncol0 = n0 + my_chunk * 8;
  const bool ep_on = EP_ALL || tid < RSTEP * CH;
  float st0[8], st1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) st0[j] = st1[j] = 0.f;
  float es[8], et[8];
  if constexpr (EPI == EPI_BWD_RELU6) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      es[j] = ncol0 + j < p.N ? p.es[ncol0 + j] : 0.f;
      et[j] = ncol0 + j < p.N ? p.et[ncol0 + j] : 0.f;
    }
  }

  f32x4_t acc[2][CT];
  int cur_m0 = 0;
  float csc[CT];                            // F8: per-column dequant scale of this lane's C columns
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int n = n0 + c * 16 + (lane & 15);
    csc[c] = (F8 && n < p.N) ? p.wsc[n] / p.asc : 1.f;
  }
  auto compute = [&](const Raw &r, int s) {
#pragma unroll
    for (int ss = 0; ss < SUBS; ++ss) {
      const int kl = s * KSTEP + ss * 32 + 8 * (lane >> 4);
      if constexpr (F8) {
        long a8[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          float v[8];
          a_transform_f<PRO>(r.a[ss][f], r.y[0][f], Ps, Kp, kl, v);
          a8[f] = pack_fp8x8(v, p.asc);
        }
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const long b8 = *reinterpret_cast<const long *>(Bs8 + (c * 16 + (lane & 15)) * LDB8 + kl);
#pragma unroll
          for (int f = 0; f < 2; ++f)
            acc[f][c] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a8[f], b8, acc[f][c], 0, 0, 0);
        }
        continue;
      }
      s16x8_t af[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) af[f] = a_transform<PRO>(r.a[ss][f], r.y[HAS_A2 ? ss : 0][f], Ps, Kp, kl);
      // (only the block-output consumers pass Aout: a possible store here would make hipcc wait
      // for the next tile's prefetch before it reuses these registers in the epilogue)
      if (AOUT && p.Aout && blockIdx.y == 0) {   // materialise the transformed A (block output) once
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int row = cur_m0 + rg * 32 + f * 16 + (lane & 15);
          if (row < p.M && kl < p.K) stg16(p.Aout + (size_t)row * p.K + kl, __builtin_bit_cast(uint4, af[f]));
        }
      }
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        s16x8_t bf;
        if constexpr (BDIRECT) bf = __builtin_bit_cast(s16x8_t, r.b[ss][BDIRECT ? c : 0]);
        else bf = *reinterpret_cast<const s16x8_t *>(Bs + (c * 16 + (lane & 15)) * LDB + kl);
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[f][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, af[f]), __builtin_bit_cast(bf16x8_t, bf), acc[f][c], 0, 0, 0);
      }
    }
  };

  // ---- flattened (M tile, k step) stream, prefetching one step ahead (across tiles too)
  for (int mt = blockIdx.x; mt < nmt; mt += gridDim.x) {
    const int m0 = mt * BM;
    cur_m0 = m0;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int c = 0; c < CT; ++c) acc[f][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = kp; s < nsteps; s += KS) {
      int ns = s + KS, nm = mt;
      if (ns >= nsteps) { ns = kp; nm = mt + gridDim.x; }
      load(nxt, nm * BM, ns, nm < nmt);
      compute(cur, s);
      // the next tile's first fragments are taken over after the epilogue below, so their
      // load latency hides behind it (a copy here waits vmcnt(0) for them right after issue)
      if (s + KS < nsteps) cur = nxt;
    }
    // ---- C tile to LDS: acc[f][c][j] = C[rg*32 + f*16 + 4*(lane>>4) + j][c*16 + (lane&15)]
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        if constexpr (KS == 1) {   // bf16 column pairs (common.h frag_store_bf16)
          const float sc = F8 ? csc[c] : 1.f;
          frag_store_bf16(Cs, LDC, rg * 32 + f * 16, c * 16, acc[f][c][0] * sc, acc[f][c][1] * sc,
                          acc[f][c][2] * sc, acc[f][c][3] * sc);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            Cf[(kp * BM + rg * 32 + f * 16 + 4 * (lane >> 4) + j) * LDF + c * 16 + (lane & 15)] = acc[f][c][j];
        }
      }
    __syncthreads();
    // take over the next tile's first fragments before this tile's stores are issued (vmcnt
    // counts loads and stores in one queue: a wait placed after the stores would drain them too)
    cur.hold();
    cur = nxt;
#pragma unroll
    for (int i0 = 0; i0 < NP; i0 += EB) {
      // bwd epilogue operands of EB rows are loaded together (one latency per batch)
      uint4 ytr[EB], rsr[EB];
      if constexpr (EPI != EPI_FWD) {
#pragma unroll
        for (int e = 0; e < EB; ++e) {
          const int rr = tid / CH + (i0 + e) * RSTEP, row = m0 + rr;
          const bool ok = i0 + e < NP && rr < BM && row < p.M && ncol0 < p.N;
          const size_t off = (size_t)row * p.N + ncol0;
          ytr[e] = ok ? ldg16(p.Yt + off) : make_uint4(0, 0, 0, 0);
          if constexpr (EPI == EPI_BWD_LIN) rsr[e] = (ok && p.R) ? ldg16(p.R + off) : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int e = 0; e < EB; ++e) {
      const int i = i0 + e;
      const int rr = tid / CH + i * RSTEP, row = m0 + rr;
      if (ep_on && i < NP && rr < BM && row < p.M && ncol0 < p.N) {
        float v[8];
        if constexpr (KS == 1) {
          unpack8(*reinterpret_cast<const uint4 *>(Cs + rr * LDC + my_chunk * 8), v);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = 0.f;
#pragma unroll
          for (int q = 0; q < KS; ++q) {
            const float4 u0 = *reinterpret_cast<const float4 *>(Cf + (q * BM + rr) * LDF + my_chunk * 8);
            const float4 u1 = *reinterpret_cast<const float4 *>(Cf + (q * BM + rr) * LDF + my_chunk * 8 + 4);
            v[0] += u0.x; v[1] += u0.y; v[2] += u0.z; v[3] += u0.w;
            v[4] += u1.x; v[5] += u1.y; v[6] += u1.z; v[7] += u1.w;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j]));
        }
        const size_t off = (size_t)row * p.N + ncol0;
        if constexpr (EPI == EPI_FWD) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            st0[j] += v[j];
            st1[j] = fmaf(v[j], v[j], st1[j]);
          }
        } else {
          float yt[8];
          unpack8(ytr[e], yt);
          if constexpr (EPI == EPI_BWD_RELU6) {
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
        stg16(p.out + off, pack8(v));
      }
      }
    }
    __syncthreads();
  }
  // ---- per-workgroup BN partials: reduce the RSTEP threads sharing a column chunk
  for (int s = 0; s < 2; ++s) {
    const int rgrp = tid / CH;
    if (ep_on) {
#pragma unroll
      for (int j = 0; j < 8; ++j) Red[rgrp * BN + my_chunk * 8 + j] = s == 0 ? st0[j] : st1[j];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      float a = 0.f;
      for (int g = 0; g < RSTEP; ++g) a += Red[g * BN + c];
      if (n0 + c < p.N) bn_part_add(p.part, blockIdx.x, gridDim.x, p.bn_rep, p.N, s, n0 + c, a);
    }
    __syncthreads();
  }
  bn_fin_tail(p.fin);
}

// dgrad weights: W^T of every 1x1 conv, batched (one table entry per layer):
// dst[off + c*R + r] = src[off + r*C + c]   (R = Cout, C = Cin), 32x32 tiles via LDS
__global__ __launch_bounds__(256) void wt_transpose_kernel(const bf16_t *__restrict__ src,
                                                           bf16_t *__restrict__ dst,
                                                           const int *__restrict__ tab) {
  __shared__ bf16_t T[32][33];
  const int *e = tab + blockIdx.y * 3;
  const long long off = e[0];
  const int R = e[1], C = e[2];
  const int tr = (R + 31) / 32, tc = (C + 31) / 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int t = blockIdx.x; t < tr * tc; t += gridDim.x) {
    const int r0 = (t / tc) * 32, c0 = (t % tc) * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + ty + 8 * i, c = c0 + tx;
      T[ty + 8 * i][tx] = (r < R && c < C) ? src[off + (long long)r * C + c] : bf16_t(0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + ty + 8 * i, r = r0 + tx;
      if (r < R && c < C) dst[off + (long long)c * R + r] = T[tx][ty + 8 * i];
    }
    __syncthreads();
  }
}

// ===========================================================================
// weight gradient: dW[N][K] += sum_m dy[m][n] * x[m][k]
//   dy = a[n]*G + b[n]*Y + c[n]   (this layer's BN backward; PRO_BNBWD)
//   x  = act(X)                   (ACT_NONE or ACT_BN_RELU6 of the producer BN)
// split-M: blockIdx.z = split; part[split][N][K]
// ===========================================================================
namespace {
struct PwWgArgs {
  const bf16_t *G, *Y;          // [M][N]
  const float *ga, *gb, *gc;    // [N]
  const bf16_t *X;              // [M][K]
  const float *xs, *xt;         // [K]
  float *part;                  // [S][N][K]
  int M, N, K, rows_per_split;
  int ih, iw, oh, ow;           // IM2COL_STEM geometry (image H/W, output H/W)
};
constexpr int kWMK = 64;              // m rows per pipeline step
constexpr int kWLD = kWMK + 8;        // transposed tile row pitch (elements): 144 B, conflict-free b128 reads
}  // namespace

// One staging item = 4 consecutive rows (m) x 8 consecutive columns of a [M][ld]
// bf16 operand; it is loaded raw into registers one step ahead (prefetch) and
// written transposed into LDS as T[col][m] (4 rows of m packed per 8-B store)
// after the current step's MFMAs, with the BN transform applied on the way.
// Loads are bounds-checked buffer loads issued unconditionally (rows past M / columns past
// ncols read 0 through the out-of-range offset): no branch around a memory instruction, so
// hipcc does not drain the one-step-ahead prefetch with a vmcnt(0) at a join.
struct WgItem {
  uint4 a[4];   // rows of G (dy items) or X (x items)
  uint4 b[4];   // rows of Y (dy items only)
};

template <bool DY>
PG_DEVICE void wg_load(WgItem &it, rsrc_t r1, rsrc_t r2, int ld, int ncols, int c, int m0, int M) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + q;
    const uint32_t off = (m < M && c < ncols) ? (uint32_t)(((size_t)m * ld + c) * 2) : kOOB;
    it.a[q] = bld16(r1, off);
    if constexpr (DY) it.b[q] = bld16(r2, off);
  }
}

// rows beyond M must contribute exactly 0 after the transform (columns beyond ncols read 0 and
// have zero parameters).  P: this item's 8 per-column parameters (a | b | c, stride ldp) in LDS,
// staged once per workgroup (loop-invariant: the former per-step global loads of pa / pb / pc
// were 16-24 dword loads per item per step behind branches).
template <int PRO>
PG_DEVICE void wg_write(const WgItem &it, const float *P, int ldp, int m0, int M, bf16_t *T, int tcol, int tm) {
  float v[4][8];
  float aa[8], bb[8], cc[8];
  if constexpr (PRO != ACT_NONE) {
    const float4 a0 = *reinterpret_cast<const float4 *>(P), a1 = *reinterpret_cast<const float4 *>(P + 4);
    const float4 b0 = *reinterpret_cast<const float4 *>(P + ldp), b1 = *reinterpret_cast<const float4 *>(P + ldp + 4);
    aa[0] = a0.x; aa[1] = a0.y; aa[2] = a0.z; aa[3] = a0.w; aa[4] = a1.x; aa[5] = a1.y; aa[6] = a1.z; aa[7] = a1.w;
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
  }
  if constexpr (PRO == PRO_BNBWD) {
    const float4 c0 = *reinterpret_cast<const float4 *>(P + 2 * ldp), c1 = *reinterpret_cast<const float4 *>(P + 2 * ldp + 4);
    cc[0] = c0.x; cc[1] = c0.y; cc[2] = c0.z; cc[3] = c0.w; cc[4] = c1.x; cc[5] = c1.y; cc[6] = c1.z; cc[7] = c1.w;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unpack8(it.a[q], v[q]);
    const bool valid = m0 + q < M;
    if constexpr (PRO == PRO_BNBWD) {
      float y[8];
      unpack8(it.b[q], y);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[q][j] = valid ? fmaf(aa[j], v[q][j], fmaf(bb[j], y[j], cc[j])) : 0.f;
    } else if constexpr (PRO == ACT_BN_RELU6) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[q][j] = valid ? relu6f(fmaf(v[q][j], aa[j], bb[j])) : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint2 w;
    w.x = pack2(v[0][j], v[1][j]);
    w.y = pack2(v[2][j], v[3][j]);
    *reinterpret_cast<uint2 *>(T + (tcol + j) * kWLD + tm) = w;
  }
}

// im2col of the stem input (NHWC, 4 channels incl. one zero pad channel, 3x3 s2 p1):
// X[m][k], m -> (b, oh, ow), k = tap*4 + c, tap = kh*3 + kw;  K = 36.  Item = 4 rows x 2 taps.
PG_DEVICE void wg_load_im2col(WgItem &it, const PwWgArgs &p, rsrc_t rx, int chunk, int m0, int M) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + q;
    const int b = m / (p.oh * p.ow), rem = m % (p.oh * p.ow);
    const int oh = rem / p.ow, ow = rem % p.ow;
    uint2 u[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // bounds-checked buffer loads: no branch around the load
      const int tap = chunk * 2 + h;
      const int ih = oh * 2 - 1 + tap / 3, iw = ow * 2 - 1 + tap % 3;
      const bool ok = m < M && tap < 9 && ih >= 0 && ih < p.ih && iw >= 0 && iw < p.iw;
      u[h] = bld8(rx, ok ? (uint32_t)((((size_t)b * p.ih + ih) * p.iw + iw) * 8) : kOOB);
    }
    it.a[q] = make_uint4(u[0].x, u[0].y, u[1].x, u[1].y);
  }
}

// Phase trace (diagnostics builds only, PGDIST_DEFINES=PGDIST_PWT_TRACE): thread 0 of every
// pw_wgrad workgroup stamps the wall clock (100 MHz) into g_pwg_ts[wg][8]: start (0), prologue
// parameters staged (1), first tile in LDS (2), k loop done (3), partial tile stored (4)
#ifdef PGDIST_PWT_TRACE
__device__ unsigned long long *g_pwg_ts = nullptr;
#define PWG_MARK(k)                                                                                \
  do {                                                                                             \
    if (threadIdx.x == 0) {                                                                        \
      unsigned long long *t_ = g_pwg_ts;                                                           \
      const size_t wg_ = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z); \
      if (t_) t_[wg_ * 8 + (k)] = wall_clock64();                                                  \
    }                                                                                              \
  } while (0)
#else
#define PWG_MARK(k) ((void)0)
#endif

template <int XPRO, int TN, int TK>
__global__ __launch_bounds__(256) void pw_wgrad_kernel(PwWgArgs p) {
  PWG_MARK(0);
  // output tile TN x TK split over 4 waves as 2 x 2 quadrants
  constexpr int QN = TN / 2, QK = TK / 2;
  constexpr int RN = QN / 16, RK = QK / 16;
  constexpr int M4 = kWMK / 4;                       // 4-row groups per step
  constexpr int ITEMS_DY = M4 * (TN / 8), ITEMS_X = M4 * (TK / 8);
  constexpr int ITEMS = ITEMS_DY + ITEMS_X;
  constexpr int IPT = (ITEMS + 255) / 256;           // items per thread
  __shared__ __attribute__((aligned(16))) bf16_t Tdy[2][TN * kWLD];
  __shared__ __attribute__((aligned(16))) bf16_t Tx[2][TK * kWLD];
  __shared__ __attribute__((aligned(16))) float Pdy[3 * TN];   // a | b | c of this tile's columns n
  __shared__ __attribute__((aligned(16))) float Px[2 * TK];    // s | t of this tile's columns k
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * TN, k0 = blockIdx.y * TK;
  const int mbeg = blockIdx.z * p.rows_per_split;
  const int mend = min(p.M, mbeg + p.rows_per_split);
  for (int i = tid; i < TN; i += 256) {
    const bool ok = n0 + i < p.N;
    Pdy[i] = ok ? p.ga[n0 + i] : 0.f;
    Pdy[TN + i] = ok ? p.gb[n0 + i] : 0.f;
    Pdy[2 * TN + i] = ok ? p.gc[n0 + i] : 0.f;
  }
  if constexpr (XPRO == ACT_BN_RELU6) {
    for (int i = tid; i < TK; i += 256) {
      const bool ok = k0 + i < p.K;
      Px[i] = ok ? p.xs[k0 + i] : 0.f;
      Px[TK + i] = ok ? p.xt[k0 + i] : 0.f;
    }
  }
  const rsrc_t rG = make_rsrc(p.G, (uint32_t)((size_t)p.M * p.N * 2));
  const rsrc_t rY = make_rsrc(p.Y, (uint32_t)((size_t)p.M * p.N * 2));
  const rsrc_t rX = make_rsrc(p.X, XPRO == IM2COL_STEM ? (uint32_t)((size_t)(p.M / (p.oh * p.ow)) * p.ih * p.iw * 8)
                                                     : (uint32_t)((size_t)p.M * p.K * 2));
  __syncthreads();
  PWG_MARK(1);

  f32x4_t acc[RN][RK];
#pragma unroll
  for (int a = 0; a < RN; ++a)
#pragma unroll
    for (int b = 0; b < RK; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  WgItem items[IPT];
  auto load_step = [&](int m0) {
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int it = tid + i * 256;
      if (it < ITEMS_DY) {
        const int m4 = it % M4, chunk = it / M4;
        wg_load<true>(items[i], rG, rY, p.N, p.N, n0 + chunk * 8, m0 + m4 * 4, mend);
      } else if (it < ITEMS) {
        const int xi = it - ITEMS_DY;
        const int m4 = xi % M4, chunk = xi / M4;
        if constexpr (XPRO == IM2COL_STEM) wg_load_im2col(items[i], p, rX, chunk, m0 + m4 * 4, mend);
        else wg_load<false>(items[i], rX, rX, p.K, p.K, k0 + chunk * 8, m0 + m4 * 4, mend);
      }
    }
  };
  auto write_step = [&](int m0, int buf) {
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int it = tid + i * 256;
      if (it < ITEMS_DY) {
        const int m4 = it % M4, chunk = it / M4;
        wg_write<PRO_BNBWD>(items[i], Pdy + chunk * 8, TN, m0 + m4 * 4, mend, Tdy[buf], chunk * 8, m4 * 4);
      } else if (it < ITEMS) {
        const int xi = it - ITEMS_DY;
        const int m4 = xi % M4, chunk = xi / M4;
        if constexpr (XPRO == IM2COL_STEM)
          wg_write<ACT_NONE>(items[i], nullptr, 0, m0 + m4 * 4, mend, Tx[buf], chunk * 8, m4 * 4);
        else
          wg_write<XPRO>(items[i], Px + chunk * 8, TK, m0 + m4 * 4, mend, Tx[buf], chunk * 8, m4 * 4);
      }
    }
  };

  int buf = 0;
  if (mbeg < mend) {
    load_step(mbeg);
    write_step(mbeg, 0);
  }
  __syncthreads();
  PWG_MARK(2);
  for (int m0 = mbeg; m0 < mend; m0 += kWMK) {
    const bool has_next = m0 + kWMK < mend;
    if (has_next) load_step(m0 + kWMK);           // global loads in flight during the MFMAs
    const bf16_t *Td = Tdy[buf], *Tq = Tx[buf];
#pragma unroll
    for (int ks = 0; ks < kWMK; ks += 32) {
      s16x8_t af[RN], bfr[RK];
#pragma unroll
      for (int a = 0; a < RN; ++a)
        af[a] = *reinterpret_cast<const s16x8_t *>(Td + (wn * QN + a * 16 + (lane & 15)) * kWLD + ks + 8 * (lane >> 4));
#pragma unroll
      for (int b = 0; b < RK; ++b)
        bfr[b] = *reinterpret_cast<const s16x8_t *>(Tq + (wk * QK + b * 16 + (lane & 15)) * kWLD + ks + 8 * (lane >> 4));
#pragma unroll
      for (int a = 0; a < RN; ++a)
#pragma unroll
        for (int b = 0; b < RK; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[a]),
                                                             __builtin_bit_cast(bf16x8_t, bfr[b]), acc[a][b], 0, 0, 0);
    }
    if (has_next) write_step(m0 + kWMK, buf ^ 1);  // other buffer: last read before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  PWG_MARK(3);
  // acc[a][b][j] = dW[n0 + wn*QN + a*16 + 4*(lane>>4) + j][k0 + wk*QK + b*16 + (lane&15)]
  float *dst = p.part + (size_t)blockIdx.z * p.N * p.K;
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
  PWG_MARK(4);
}

void pwg_trace_set(void *ts) {   // nullptr: off; no-op unless built with PGDIST_PWT_TRACE
#ifdef PGDIST_PWT_TRACE
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pwg_ts), &ts, sizeof(ts));
#else
  (void)ts;
#endif
}

// ===========================================================================
// host launchers
// ===========================================================================
// geometry of one pointwise GEMM launch (also sizes the BN partial workspace: P = gx)
//  * large M, K <= 192: weight tile resident in LDS for the whole grid-stride sweep;
//  * small M or large K: weight fragments read straight from L2 alongside A, and the
//    K dimension split over the 4 waves (KS) so the grid still has >= ~1.5k workgroups.
struct PwGeom {
  int BN, KS, bdirect, nt, nmt, gx;
  size_t lds;
};
// allow_wide: BN = N for N = 96 / 144 (bf16 forward only; the fp8 launcher passes false).  The
// partial-row count P = gx of a wide launch is >= that of the narrow one, so sizing the BN
// accumulators with pw_gemm_num_partials (which assumes wide) covers every launch.
static PwGeom pw_geom(int M, int N, int K, int pro, bool allow_wide = true) {
  PwGeom g;
  const int Kp64 = (K + 63) / 64 * 64;
  g.bdirect = (Kp64 > 192) || (M < 65536);
  const int kstep = g.bdirect ? 32 : 64;
  const int Kp = (K + kstep - 1) / kstep * kstep;
  const int nsteps = Kp / kstep;
  if (!g.bdirect) {
    g.BN = N <= 32 ? 32 : 64;     // BN = 128 costs occupancy (1-2 waves/SIMD) for no bandwidth gain
    // N = 96 / 144 (the expand convs at 112x112 / 56x56): one N tile over the whole row (full
    // 192 / 288-B output rows instead of 64 + 32 or 64 + 64 + 16 column slices, no MFMA / LDS
    // work on padding columns, A read once)
    if (allow_wide && pro != PRO_BNBWD && (N == 96 || N == 144)) g.BN = N;
    g.KS = 1;
  } else {
    g.BN = (N % 64 == 0) ? 64 : 32;
    g.KS = 1;
    const int nt = (N + g.BN - 1) / g.BN;
    while (g.KS < 4 && g.KS * 2 <= nsteps && (long long)nt * ((M + 128 / g.KS - 1) / (128 / g.KS)) < 1536) g.KS *= 2;
  }
  g.nt = (N + g.BN - 1) / g.BN;
  const int BM = 128 / g.KS;
  g.nmt = (M + BM - 1) / BM;
  // grid-size targets (docs/PERF_NOTES.md round 2 sweeps): LDS-resident path 2048 (1024:
  // +0.2-0.5 % step time), B-direct path 1024
  int gx = (g.bdirect ? 1024 : 2048) / g.nt;
  if (gx > g.nmt) gx = g.nmt;
  gx = (gx + 7) & ~7;                  // multiple of 8: the N tiles of one M tile share an XCD L2
  if (gx < 8) gx = 8;
  g.gx = gx;
  const int npar = pro == ACT_NONE ? 0 : (pro == PRO_BNBWD ? 3 : 2);   // PRO_BNRES: s, t (+ A2)
  const size_t cbuf = g.KS == 1 ? (size_t)BM * (g.BN + kCPad) * 2 : (size_t)g.KS * BM * (g.BN + 4) * 4;
  const size_t red = (size_t)(256 / (g.BN / 8)) * g.BN * 4;
  g.lds = (g.bdirect ? 0 : (size_t)g.BN * (Kp + kBPad) * 2) + (size_t)npar * Kp * 4 + (cbuf > red ? cbuf : red);
  return g;
}

int pw_tile_num_partials(int M, int N, int K);
void launch_pw_tile(int pro, int epi, const bf16_t *A, const bf16_t *A2, const float *pa, const float *pb,
                    const float *pc, const bf16_t *W, bf16_t *out, const bf16_t *Yt, const float *es,
                    const float *et, const bf16_t *R, float *part, int M, int N, int K, bf16_t *Aout,
                    hipStream_t st);

// small M or large K -> the two-operand LDS-tiled kernel (pwtile.hip)
int pw_gemm_num_partials(int M, int N, int K) {
  const PwGeom g = pw_geom(M, N, K, ACT_NONE);
  return g.bdirect ? pw_tile_num_partials(M, N, K) : g.gx;
}

template <int PRO, int EPI, int BN, int KS, bool BD>
static void launch_pw_t(const PwArgs &a, const PwGeom &g, hipStream_t st) {
  hipLaunchKernelGGL((pw_gemm_kernel<PRO, EPI, BN, KS, BD>), dim3(g.gx, g.nt), dim3(256), g.lds, st, a);
}

template <int PRO, int EPI>
static void launch_pw_geom(const PwArgs &a, const PwGeom &g, hipStream_t st) {
  if (!g.bdirect) {
    if constexpr (EPI == EPI_FWD) {
      if (g.BN == 96) { launch_pw_t<PRO, EPI, 96, 1, false>(a, g, st); return; }
      if (g.BN == 144) { launch_pw_t<PRO, EPI, 144, 1, false>(a, g, st); return; }
      if (g.BN == 192) { launch_pw_t<PRO, EPI, 192, 1, false>(a, g, st); return; }
    }
    if (g.BN == 32) launch_pw_t<PRO, EPI, 32, 1, false>(a, g, st);
    else launch_pw_t<PRO, EPI, 64, 1, false>(a, g, st);
    return;
  }
}

// pro: 0 none, 1 bn+relu6, 3 bnbwd ; epi: 0 fwd, 1 bwd relu6, 2 bwd lin.
// W is [N][K] in GEMM terms for every mode (dgrad passes the transposed conv weight).
void launch_pw_gemm(int pro, int epi, const bf16_t *A, const bf16_t *A2, const float *pa,
                    const float *pb, const float *pc, const bf16_t *W, bf16_t *out,
                    const bf16_t *Yt, const float *es, const float *et, const bf16_t *R, float *part,
                    int M, int N, int K, bf16_t *Aout, hipStream_t st) {
  PwArgs a{A, A2, pa, pb, pc, W, out, Yt, es, et, R, part, M, N, K, Aout};
  a.bn_rep = g_bn_rep;
  a.fin = nullptr;
  const PwGeom g = pw_geom(M, N, K, pro);
  if (g.bdirect) {
    launch_pw_tile(pro, epi, A, A2, pa, pb, pc, W, out, Yt, es, et, R, part, M, N, K, Aout, st);
    return;
  }
  a.fin = take_bn_fin();
  a.lz = take_bn_lz();
#define PW_CASE(P, E) \
  if (pro == P && epi == E) { launch_pw_geom<P, E>(a, g, st); return; }
  PW_CASE(ACT_NONE, EPI_FWD)
  PW_CASE(ACT_BN_RELU6, EPI_FWD)
  PW_CASE(ACT_BN, EPI_FWD)
  PW_CASE(PRO_BNRES, EPI_FWD)
  PW_CASE(PRO_BNBWD, EPI_BWD_RELU6)
  PW_CASE(PRO_BNBWD, EPI_BWD_LIN)
#undef PW_CASE
}

void launch_pw_tile_f8(int pro, const bf16_t *A, const float *pa, const float *pb, const uint8_t *W8, int ldw8,
                       const float *wsc, float asc, bf16_t *out, float *part, int M, int N, int K,
                       hipStream_t st);

// fp8 forward GEMM (fwd epilogue only): out = dequant(e4m3(asc * prologue(A)) . W8^T)
void launch_pw_gemm_f8(int pro, const bf16_t *A, const float *pa, const float *pb, const uint8_t *W8, int ldw8,
                       const float *wsc, float asc, bf16_t *out, float *part, int M, int N, int K,
                       hipStream_t st) {
  PwGeom g = pw_geom(M, N, K, pro, false);
  if (g.bdirect) {
    launch_pw_tile_f8(pro, A, pa, pb, W8, ldw8, wsc, asc, out, part, M, N, K, st);
    return;
  }
  PwArgs a{A, nullptr, pa, pb, nullptr, nullptr, out, nullptr, nullptr, nullptr, nullptr, part, M, N, K, nullptr,
           W8, wsc, asc, ldw8, g_bn_rep, take_bn_fin(), take_bn_lz()};
  const int Kp = (K + 63) / 64 * 64;
  g.lds -= (size_t)g.BN * (Kp + kBPad) * 2;
  g.lds += (size_t)g.BN * (Kp + 16);
#define PW8_CASE(P)                                                                                          \
  if (pro == P) {                                                                                            \
    if (g.BN == 32) hipLaunchKernelGGL((pw_gemm_kernel<P, EPI_FWD, 32, 1, false, true>), dim3(g.gx, g.nt),   \
                                       dim3(256), g.lds, st, a);                                             \
    else hipLaunchKernelGGL((pw_gemm_kernel<P, EPI_FWD, 64, 1, false, true>), dim3(g.gx, g.nt), dim3(256),   \
                            g.lds, st, a);                                                                   \
    return;                                                                                                  \
  }
  PW8_CASE(ACT_NONE)
  PW8_CASE(ACT_BN_RELU6)
  PW8_CASE(ACT_BN)
#undef PW8_CASE
}

// Per-output-channel e4m3 quantisation of the 1x1 conv weights (fp32 master), one wave
// per weight row; tab int32 [n][5] = (src element offset, rows N, cols K, dst byte offset,
// scale offset); each layer's e4m3 rows have pitch ldw8 = K rounded up to 64 (zero padded).
// w8[n][k] = e4m3(w[n][k] / s_n), s_n = max_k |w[n][k]| / 448 (1 for an all-zero row).
__global__ __launch_bounds__(256) void w8_quant_kernel(const float *__restrict__ src, uint8_t *__restrict__ dst,
                                                       float *__restrict__ wsc, const int *__restrict__ tab) {
  const int *e = tab + blockIdx.y * 5;
  const int N = e[1], K = e[2], ldw8 = (K + 63) / 64 * 64;
  const int lane = threadIdx.x & 63;
  for (int n = blockIdx.x * 4 + (threadIdx.x >> 6); n < N; n += gridDim.x * 4) {
    const float *w = src + e[0] + (size_t)n * K;
    float amax = 0.f;
    for (int k = lane; k < K; k += 64) amax = fmaxf(amax, fabsf(w[k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    const float s = amax > 0.f ? amax / kFp8Max : 1.f, inv = 1.f / s;
    uint8_t *d = dst + e[3] + (size_t)n * ldw8;
    for (int k = lane; k < ldw8; k += 64) {
      const float q = k < K ? fminf(fmaxf(w[k] * inv, -kFp8Max), kFp8Max) : 0.f;
      d[k] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, 0.f, 0, false) & 0xff);
    }
    if (lane == 0) wsc[e[4] + n] = s;
  }
}

void launch_w8_quant(const float *src, uint8_t *dst, float *wsc, const int *tab, int n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(w8_quant_kernel, dim3(64, n), dim3(256), 0, st, src, dst, wsc, tab);
}

// tab: int32 [n][3] = (element offset, rows R = Cout, cols C = Cin) into src/dst
void launch_wt_transpose(const bf16_t *src, bf16_t *dst, const int *tab, int n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(wt_transpose_kernel, dim3(64, n), dim3(256), 0, st, src, dst, tab);
}

int colsum_rows(int R);
void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st, bool stem36 = false);
void wgrad_reduce_defer(bool on);
bool wgrad_reduce_deferring();

// split-M geometry: tiles of TN x TK outputs, S splits of >= min_rows rows each.  The floor is
// 512 rows for large weights and 256 when N*K <= 200k: the 14x14 / 7x7 MobileNetV2 weight
// gradients (M = 25088 / 6272) then run 2x the splits (e.g. 147 -> 294 workgroups for
// 64x384), 718 -> 604 us over the 22 pw_wgrad launches; the 1280x320 / 320x960 weights got
// slower at 256 (twice the fp32 partials to write and reduce): profiles/r3b_pwwg_sweep.txt.
static constexpr int kMinRowsPerSplit = 512, kMinRowsSmallW = 256;
static constexpr long long kSmallW = 200000;
static void wgrad_geom(int M, int N, int K, int &TN, int &TK, int &S, int &rps) {
  const int min_rows = (long long)N * K <= kSmallW ? kMinRowsSmallW : kMinRowsPerSplit;
  TN = N <= 32 ? 32 : (N <= 64 ? 64 : 128);
  TK = K <= 32 ? 32 : (K <= 64 ? 64 : 128);
  const int tiles = ((N + TN - 1) / TN) * ((K + TK - 1) / TK);
  constexpr int target = 1024;   // split-M grid-size target (512 / 2048: neutral, round 2-3 sweeps)
  S = (target + tiles - 1) / tiles;
  const int max_s = (M + min_rows - 1) / min_rows;
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  rps = ((M + S - 1) / S + kWMK - 1) / kWMK * kWMK;
  S = (M + rps - 1) / rps;
}

long long pw_wgrad_workspace_floats(int M, int N, int K) {
  int TN, TK, S, rps;
  wgrad_geom(M, N, K, TN, TK, S, rps);
  return (long long)(S + colsum_rows(S)) * N * K;
}

template <int XPRO, int TN, int TK>
static void launch_wg_t(const PwWgArgs &a, int S, hipStream_t st) {
  dim3 grid((a.N + TN - 1) / TN, (a.K + TK - 1) / TK, S);
  hipLaunchKernelGGL((pw_wgrad_kernel<XPRO, TN, TK>), grid, dim3(256), 0, st, a);
}

template <int XPRO>
static void launch_wg_x(const PwWgArgs &a, int TN, int TK, int S, hipStream_t st) {
#define WG_CASE(A_, B_) \
  if (TN == A_ && TK == B_) { launch_wg_t<XPRO, A_, B_>(a, S, st); return; }
  WG_CASE(32, 32) WG_CASE(32, 64) WG_CASE(32, 128)
  WG_CASE(64, 32) WG_CASE(64, 64) WG_CASE(64, 128)
  WG_CASE(128, 32) WG_CASE(128, 64) WG_CASE(128, 128)
#undef WG_CASE
}

long long stem_wgrad_workspace_floats(int M, int O) {
  int TN, TK, S, rps;
  wgrad_geom(M, O, 36, TN, TK, S, rps);
  return (long long)(S + colsum_rows(S)) * O * 36;
}

void launch_stem_wgrad(const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb,
                       const float *gc, const bf16_t *img, float *part, float *grad, int B, int H,
                       int W, int O, hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int M = B * Ho * Wo;
  int TN, TK, S, rps;
  wgrad_geom(M, O, 36, TN, TK, S, rps);
  PwWgArgs a{G, Y, ga, gb, gc, img, nullptr, nullptr, part, M, O, 36, rps, H, W, Ho, Wo};
  launch_wg_x<IM2COL_STEM>(a, TN, TK, S, st);
  // the split reduction stores straight into the torch [O][3][3][3] layout (no permute launch)
  launch_wgrad_reduce(part, S, (long long)O * 36, grad, st, /*stem36=*/true);
}

void launch_pw_wgrad(const bf16_t *G, const bf16_t *Y, const float *ga, const float *gb,
                     const float *gc, const bf16_t *X, const float *xs, const float *xt, int xact,
                     float *part, float *grad, int M, int N, int K, hipStream_t st) {
  int TN, TK, S, rps;
  wgrad_geom(M, N, K, TN, TK, S, rps);
  PwWgArgs a{G, Y, ga, gb, gc, X, xs, xt, part, M, N, K, rps, 0, 0, 0, 0};
  if (xact == ACT_BN_RELU6) launch_wg_x<ACT_BN_RELU6>(a, TN, TK, S, st);
  else launch_wg_x<ACT_NONE>(a, TN, TK, S, st);
  launch_wgrad_reduce(part, S, (long long)N * K, grad, st);
}

