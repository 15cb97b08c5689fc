// Depthwise 3x3 convolution (pad 1, stride 1|2), NHWC bf16, for MobileNetV2.
//
// Reference op: the 17 depthwise Conv2d(groups=C) layers of torchvision
// MobileNetV2 run through cuDNN (SURVEY.md §2.6 "Depthwise conv 3x3"); on ROCm
// the library path (MIOpen / CK grouped-conv bwd-weight) takes ~23 ms per call
// at bs=128 (profiles/r1_torch_miopen_baseline_kernel_stats.csv).  Depthwise is
// pure bandwidth (1.8-4.5 FLOP/B), so these kernels are organised around the
// memory system:
//
//  * a workgroup = a tile of TWc columns x R rows of one image and a slab of
//    CC <= 64 channels (a multiple of 8: 16-B chunks; up to 128 on narrow 7x7 / 14x14 maps,
//    see dw_geom); a thread owns 4 channels of ONE
//    column (output column for fwd / wgrad, input column for dgrad) and walks the R rows,
//    keeping a rolling 3-row x 3-column window in registers;
//  * every row the tile needs is streamed once into an LDS ring by LDS-DMA
//    (buffer_load_dwordx4 ... lds, see the "LDS-DMA row-streaming" section below) and the
//    three tap columns are read from LDS;
//  * weights are tap-major [9][C] in the flat parameter buffer;
//  * the producer's BatchNorm-apply + ReLU6 is fused into the input read (zero
//    padding in the post-activation space), the forward epilogue emits this
//    layer's BN partial sums, the dgrad epilogue the producer-BN backward
//    partials; the weight gradient is reduced per workgroup and then by a
//    deterministic two-level column sum.
#include "../bnfin.h"

#include <cstdlib>

namespace {

constexpr int CPT = 4;        // channels per thread
// rows per strip of the forward / dgrad tiles and of the weight-gradient tiles: round 1 swept
// 4..112 (28 fastest then); with the LDS-DMA kernels, the lazy BN prologue and depth-3 dgrad
// rings 56 is fastest for forward / dgrad (MobileNetV2 bs128: 4.84 -> 4.80 ms/step; 112 equal,
// 40 and 14 slower), the side-stream weight gradients keep 28
constexpr int kRows = 56;
constexpr int kWRows = 28;

struct DwGeom {
  int B, H, W, C, Ho, Wo;
  int CC;     // channels per workgroup (tile_of() decodes the slab)
  int TWc;    // columns per workgroup
  int R;      // rows per workgroup
  int tiles_w, tiles_h;
  int Hi;     // image height (stride 1: rows of the 3x3 window masked at image edges); a "tall"
              // geometry stacks the batch as one B*Hi-row image (B = 1, H = Ho = B*Hi)
  int bn_rep;         // BN-statistics replica rows (g_bn_rep)
  const BnFin *fin;   // fused BN finalize in the tail (nullptr: none)
  const BnFin *lz;    // lazy finalize (fwd: the input BN's scale / shift; dgrad: this layer's coef)
};

// Lazy BN finalize of this workgroup's channel slab [cbase, cbase + CC) into LDS (one
// channel per thread, CC <= 128), then a barrier: every thread reads its CPT channels from
// LDS instead of each computing them (the slab is shared by C4 = CC/4 threads per column).
// npar = 2: forward scale / shift; 3: backward coefficients.
__shared__ float lzp[3][128];
PG_DEVICE void lazy_stage(const DwGeom &g, int cbase, int npar) {
  if ((int)threadIdx.x < g.CC) {
    float a, b, c;
    bn_lazy(g.lz, cbase + threadIdx.x, a, b, c);
    lzp[0][threadIdx.x] = a;
    lzp[1][threadIdx.x] = b;
    if (npar == 3) lzp[2][threadIdx.x] = c;
  }
  __syncthreads();
}

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




// Workgroup decode.  The 1-D grid enumerates (tile, channel slab) pairs so that the slabs
// of one spatial tile are 8 workgroup ids apart: same XCD (ids are dealt to the 8 XCDs
// round-robin) and dispatched together, so the 128-B lines shared by neighbouring slabs
// (a pixel's C channels are contiguous in NHWC) are fetched from HBM once into that L2.
struct Tile {
  int b, r0, w0;
  int idx;     // tile index (partial row)
  int slab;    // channel slab
};
PG_DEVICE int dw_tiles(const DwGeom &g) { return g.B * g.tiles_h * g.tiles_w; }   // partial rows
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
// nrows > 0 (BN statistics, NV == 2): accumulated atomically into replica row prow % rep
// (bn_part_add); nrows == 0: plain store of row prow (weight-gradient split partials).
template <int NV>
PG_DEVICE void block_channel_partials(float (&acc)[NV][CPT], float *__restrict__ part, int C, int CC,
                                      int cbase, int ncol, float *lds, int prow, int nrows = 0,
                                      int rep = 0) {
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
      if (NV == 2 && nrows > 0) bn_part_add(part, prow, nrows, rep, C, v, cbase + c, s);
      else part[((size_t)prow * NV + v) * C + cbase + c] = s;
    }
    __syncthreads();
  }
}

}  // namespace

// ===========================================================================
// LDS-DMA row-streaming variants (default).  Measured on MI355X (rocprofv3 --pmc,
// scripts/gpu_pmc_dw.sh; per-layer times: scripts/dw_bench.py): the register-window kernels
// above load each input row THREE times per thread (the 3 tap columns, 8 B per lane), so the
// texture-data return path (TD_TD_BUSY) runs 80-85 % busy at 2-3 TB/s, and their loads sit
// behind branches (image borders, strip ends), so hipcc drains vmcnt(0) at every join and the
// one-row register prefetch never overlaps; staging rows through registers two or four rows
// ahead only trades occupancy for depth (same bytes in flight per CU).
// Here every row a tile needs is streamed ONCE, 16 B per lane, straight into an LDS ring by
// buffer_load_dwordx4 ... lds (no VGPRs per row in flight), kDepth rows ahead of the row being
// computed.  Every global access is a bounds-checked buffer op whose masked lanes use an
// out-of-range offset (common.h), so the loop body has no per-lane branch around a memory
// instruction and every wave issues the same VMEM instructions per step: the wait for a ring
// slot is a counted `s_waitcnt vmcnt(N)` + s_barrier (one per row), never a drain.
// The 3 tap columns are read from LDS (ds_read_b64); the rolling 3x3 register window, the
// fused BN/ReLU6 prologue, the BN partial epilogues and the fused weight gradient are those
// of the kernels above.
// ===========================================================================
namespace {

constexpr int kDepth = 4;   // rows in flight per stream (forward; the dgrad rings use 3)
constexpr int kRing = kDepth + 1;         // ring slots: the row being read + kDepth in flight
// per-slot LDS bytes (whole 1 KiB wave pieces): halo row segments (TWc + 2) x CC8 <= 144
// chunks, own-column segments TWc x CC8 <= 128, stride-2 input segments (2 TWc + 1) x CC8 <= 256
constexpr int kSlotHalo = 3072, kSlotOwn = 2048, kSlotS2 = 4096;

// One streamed tensor: a row segment of ncol columns starting at col0 x CC channels = nchunk
// 16-B chunks (t = col * CC8 + part), lane-linear in LDS (wave w fills chunks [64w, 64w+64)).
// Waves with no chunk of the segment still issue, into a dummy LDS piece with out-of-range
// offsets, so that every wave issues the same number of VMEM instructions per step.
struct Stream {
  rsrc_t rs;
  u32x4_t srd;         // the same descriptor as raw words (inline-asm DMA)
  int H, W, C, b, col0;
  int lane_col;        // segment column of this lane's chunk (-1: none)
  int lane_coff;       // channel byte offset of this lane's chunk
  bool wave_used;      // wave-uniform
  PG_DEVICE void set(const void *base, uint32_t bytes) {
    rs = make_rsrc(base, bytes);
    srd = make_srd(base, bytes);
  }
  PG_DEVICE void init(const void *base, uint32_t bytes, int H_, int W_, int C_, int b_, int col0_, int nchunk,
                      int CC8, int cbase) {
    set(base, bytes);
    H = H_;
    W = W_;
    C = C_;
    b = b_;
    col0 = col0_;
    const int t = threadIdx.x;
    lane_col = t < nchunk ? t / CC8 : -1;
    lane_coff = (cbase + (t < nchunk ? t % CC8 : 0) * 8) * 2;
    wave_used = (t & ~63) < nchunk;
  }
  // DMA row ih into `slot` of a ring of `stride`-byte slots at `ring` (inline asm, common.h
  // lds_dma16: a builtin DMA made hipcc wait for the rows issued kDepth ahead before every
  // ring read; the ring's own counted ring_sync waits are the ordering)
  PG_DEVICE void issue(char *ring, int stride, int slot, int ih, char *dummy) const {
    const int iw = col0 + lane_col;
    const bool ok = wave_used && lane_col >= 0 && ih >= 0 && ih < H && iw >= 0 && iw < W;
    const uint32_t off = ok ? (uint32_t)(((b * H + ih) * W + iw) * C) * 2u + (uint32_t)lane_coff : kOOB;
    char *dst = wave_used ? ring + slot * stride + (threadIdx.x & ~63) * 16 : dummy;
    lds_dma16(srd, dst, off);
  }
};

// wait until at most N of this wave's VMEM instructions are outstanding, then a workgroup
// barrier (every wave's share of the slot is in LDS; every read of the slot about to be
// refilled is done).  N counts only the DMAs issued after the awaited row: stores may retire
// out of order with loads (an out-of-range store immediately — a budget that counted the
// stores let the wait pass before the DMA had landed; measured), loads retire in order.
// Inline asm: hipcc must neither drain vmcnt(0) at the barrier nor move LDS reads across it.
template <int N>
PG_DEVICE void ring_sync() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
PG_DEVICE void mem_fence_compiler() { asm volatile("" ::: "memory"); }
// vmcnt(0) as the s_waitcnt builtin (vmcnt 0, expcnt 7, lgkmcnt 15): unlike an asm wait, hipcc's
// waitcnt pass sees it, so it knows the parameter loads issued before the row loop have landed
// and does not wait for them again (vmcnt(N) / vmcnt(0) before their first use inside the
// loop, which then also waits for the ring's in-flight rows)
PG_DEVICE void params_landed() {
  mem_fence_compiler();   // no load sinks below the wait
  __builtin_amdgcn_s_waitcnt(0x0F70);
  mem_fence_compiler();
}

PG_DEVICE uint2 lds8(const char *slot, int col, int CC, int c) {
  return *reinterpret_cast<const uint2 *>(slot + (col * CC + c) * 2);
}

PG_DEVICE uint32_t nhwc_off(int b, int H, int W, int C, int h, int w, int c) {
  return (uint32_t)((((b * H + h) * W + w) * C + c) * 2);
}

}  // namespace

// forward: y = dwconv(act(x)), partial (sum y, sum y^2); tiles over the output grid.
// Per step (one input row): 1 DMA + 1 store (out of range when no output row completes).
// The row loop is unrolled over the window period (3 rows for stride 1, 4 for stride 2) so
// the window rows rotate by register renaming instead of copies; weights stay unpacked.
template <int S, int ACT, int D = kDepth>
__global__ __launch_bounds__(256) void dw_fwd_lds_kernel(
    const bf16_t *__restrict__ x, const float *__restrict__ in_s, const float *__restrict__ in_t,
    const bf16_t *__restrict__ w, bf16_t *__restrict__ y, float *__restrict__ part, DwGeom g) {
  constexpr int kDepth = D, kRing = D + 1;
  constexpr int kSlot = S == 1 ? kSlotHalo : kSlotS2;
  constexpr int U = S == 1 ? 3 : 4;                 // window period in input rows
  __shared__ __attribute__((aligned(16))) char ring[kRing * kSlot + 1024];
  __shared__ __attribute__((aligned(16))) float red[1024];
  char *dummy = ring + kRing * kSlot;
  const int C4 = g.CC / CPT, CC8 = g.CC / 8;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int ow = tl.w0 + col;
  const bool active = col < g.TWc && ow < g.Wo;
  const int lcol = active ? col * S : 0;            // segment column of tap 0 (clamped when inactive)
  const rsrc_t ry = make_rsrc(y, (uint32_t)g.B * g.Ho * g.Wo * g.C * 2);


  const int oh_end = min(tl.r0 + g.R, g.Ho);
  const int j0 = tl.r0 * S - 1;                     // input rows j0 .. j0 + nrows - 1
  const int nrows = (oh_end - 1) * S + 1 - j0 + 1;
  const int iw0 = ow * S - 1;
  // column validity of the 3 taps (rows are checked per step)
  bool cok[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) cok[d] = active && iw0 + d >= 0 && iw0 + d < g.W;
  Stream sx;
  sx.init(x, (uint32_t)g.B * g.H * g.W * g.C * 2, g.H, g.W, g.C, tl.b, tl.w0 * S - 1,
          ((g.TWc - 1) * S + 3) * CC8, CC8, cbase);
#pragma unroll
  for (int q = 0; q < kDepth; ++q) sx.issue(ring, kSlot, q, j0 + q, dummy);
  // BN / weight parameters staged while the first kDepth rows are in flight
  float s[CPT], t[CPT], stats[2][CPT], wt[9][CPT];
  const bool lazy = ACT != ACT_NONE && g.lz != nullptr;
  uint2 wraw[9];   // weight loads in flight across the lazy-finalize round trips
#pragma unroll
  for (int q = 0; q < 9; ++q) wraw[q] = ldg8(w + (size_t)q * g.C + c0);
  if (lazy) lazy_stage(g, cbase, 2);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    if (lazy) {
      s[k] = lzp[0][c4 * CPT + k];
      t[k] = lzp[1][c4 * CPT + k];
    } else {
      s[k] = (ACT != ACT_NONE) ? in_s[c0 + k] : 1.f;
      t[k] = (ACT != ACT_NONE) ? in_t[c0 + k] : 0.f;
    }
    stats[0][k] = stats[1][k] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) unpack4(wraw[q], wt[q]);
  params_landed();   // parameters in registers (and the first rows in LDS)
  float win[3][3][CPT];   // three input rows x three tap columns (roles rotate with the unroll)
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int d = 0; d < 3; ++d) zero4(win[r][d]);
  int slot = 0;
  // image-local row of input row j0 + k (stride 1): the taps above an image's first output row
  // and below its last are zero padding even where the strip continues into the next image
  int ihl = j0 % g.Hi;
  if (ihl < 0) ihl += g.Hi;
  // one input row: wait for its slot, refill the ring, load it into window row `into`;
  // emit an output row from window rows (ra, rb, rc) when `emit`
  auto step = [&](int k, int into, bool emit, int ra, int rb, int rc) {
    ring_sync<(kDepth - 1) * 1>();
    sx.issue(ring, kSlot, slot + kDepth < kRing ? slot + kDepth : slot + kDepth - kRing, j0 + k + kDepth, dummy);
    mem_fence_compiler();
    const char *sl = ring + slot * kSlot;
    slot = slot + 1 == kRing ? 0 : slot + 1;
    const int ih = j0 + k;
    const bool rok = ih >= 0 && ih < g.H;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float v[CPT];
      unpack4(lds8(sl, lcol + d, g.CC, c4 * CPT), v);
      const float m = (rok && cok[d]) ? 1.f : 0.f;
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) {
        const float a = m * act_apply<ACT>(v[kk], s[kk], t[kk]);
        if (into == 0) win[0][d][kk] = a;
        if (into == 1) win[1][d][kk] = a;
        if (into == 2) win[2][d][kk] = a;
      }
    }
    const int oh = S == 1 ? ih - 1 : (ih - 1) >> 1;
    float m0 = 1.f, m2 = 1.f;   // tap rows 0 / 2 inside this output row's image
    if constexpr (S == 1) {
      const int ohl = ihl == 0 ? g.Hi - 1 : ihl - 1;
      m0 = ohl != 0 ? 1.f : 0.f;
      m2 = ohl != g.Hi - 1 ? 1.f : 0.f;
      ihl = ihl + 1 == g.Hi ? 0 : ihl + 1;
    }
    float ar[3][CPT];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int wr = r == 0 ? ra : r == 1 ? rb : rc;
      zero4(ar[r]);
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int kk = 0; kk < CPT; ++kk) ar[r][kk] = fmaf(win[wr][dw][kk], wt[r * 3 + dw][kk], ar[r][kk]);
    }
    float acc[CPT];
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) acc[kk] = fmaf(m2, ar[2][kk], fmaf(m0, ar[0][kk], ar[1][kk]));
    bst8(ry, (emit && active) ? nhwc_off(tl.b, g.Ho, g.Wo, g.C, oh, ow, c0) : kOOB, pack4(acc));
    const float e = emit ? 1.f : 0.f;
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) {
      stats[0][kk] = fmaf(e, acc[kk], stats[0][kk]);
      stats[1][kk] = fmaf(e * acc[kk], acc[kk], stats[1][kk]);
    }
  };
  for (int k = 0; k < nrows; k += U) {
    if constexpr (S == 1) {   // row k -> slot k % 3; output rows use (k-2, k-1, k) % 3
      step(k, 0, k >= 2, 1, 2, 0);
      if (k + 1 < nrows) step(k + 1, 1, k + 1 >= 2, 2, 0, 1);
      if (k + 2 < nrows) step(k + 2, 2, true, 0, 1, 2);
    } else {                  // k%4: 0 -> A (emit C,B,A if k > 0), 1 -> B, 2 -> C (emit A,B,C), 3 -> B
      step(k, 0, k > 0, 2, 1, 0);
      if (k + 1 < nrows) step(k + 1, 1, false, 0, 1, 2);
      if (k + 2 < nrows) step(k + 2, 2, true, 0, 1, 2);
      if (k + 3 < nrows) step(k + 3, 1, false, 0, 1, 2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may still target the ring
  __syncthreads();
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, g.TWc, red, tl.idx, dw_tiles(g), g.bn_rep);
  bn_fin_tail(g.fin);
}

// dgrad (stride 1): thread = one INPUT column, strip of input rows.  Streams per step k: the dy
// rows (g, y of this layer's BN backward, halo columns) of dy row r0-1+k and yprev (the
// producer's pre-BN activation, own columns: ReLU6 mask + fused weight gradient) of input row
// r0+k-2; step k >= 2 emits input row r0+k-2.  Per step: 3 DMA + 1 store.
// (The fused weight-gradient variant needs 175 VGPRs: 2 waves per SIMD; forcing 3 with
// amdgpu_waves_per_eu spilled in the row loop and measured 30-80 % slower: 56x56x144 209.6 ->
// 277.4 us, 112x112x32 152.9 -> 271.1 us; profiles/r3b_pwwg_sweep.txt.)
template <bool WG, int D = kDepth>
__global__ __launch_bounds__(256) void dw_dgrad_s1_lds_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ w, const bf16_t *__restrict__ yprev, const float *__restrict__ ps,
    const float *__restrict__ pt, bf16_t *__restrict__ gout, float *__restrict__ part, DwGeom g,
    float *__restrict__ wpart) {
  // D rows in flight: 3 gives 39 KB of LDS per workgroup (4 per CU) instead of 48 KB (3 per CU)
  constexpr int kDepth = D, kRing = D + 1;
  constexpr int kStep = 2 * kSlotHalo + kSlotOwn;   // g, y, yprev pieces of one ring slot
  __shared__ __attribute__((aligned(16))) char ring[kRing * kStep + 1024];
  __shared__ __attribute__((aligned(16))) float red[1024];
  char *dummy = ring + kRing * kStep;
  const int C4 = g.CC / CPT, CC8 = g.CC / 8;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int iw = tl.w0 + col;
  const bool active = col < g.TWc && iw < g.W;
  const int lcol = active ? col : 0;
  const uint32_t nbytes = (uint32_t)g.B * g.H * g.W * g.C * 2;   // stride 1: dy grid == input grid
  const rsrc_t ro = make_rsrc(gout, nbytes);


  const int ih_end = min(tl.r0 + g.R, g.H);
  const int j0 = tl.r0 - 1;                         // dy rows j0 .. ih_end (window ih-1..ih+1)
  const int nrows = ih_end - j0 + 1;
  bool cok[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) cok[c] = active && iw - 1 + c >= 0 && iw - 1 + c < g.W;
  Stream sg, sy, sp;
  sg.init(gin, nbytes, g.H, g.W, g.C, tl.b, tl.w0 - 1, (g.TWc + 2) * CC8, CC8, cbase);
  sy = sg;
  sy.set(yself, nbytes);
  sp.init(yprev, nbytes, g.H, g.W, g.C, tl.b, tl.w0, g.TWc * CC8, CC8, cbase);
  auto issue = [&](int slot, int k) {
    char *base = ring + slot * kStep;
    sg.issue(base, 0, 0, j0 + k, dummy);
    sy.issue(base + kSlotHalo, 0, 0, j0 + k, dummy);
    sp.issue(base + 2 * kSlotHalo, 0, 0, tl.r0 + k - 2, dummy);
  };
#pragma unroll
  for (int q = 0; q < kDepth; ++q) issue(q, q);
  // BN / weight parameters staged while the first kDepth rows are in flight
  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT], stats[2][CPT], wt[9][CPT];
  float accw[WG ? 9 : 1][CPT];
  // weight and producer-BN loads in flight across the lazy-finalize round trips
  uint2 wraw[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) wraw[q] = ldg8(w + (size_t)q * g.C + c0);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
  }
  if (g.lz) lazy_stage(g, cbase, 3);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    if (g.lz) {
      al[k] = lzp[0][c4 * CPT + k];
      be[k] = lzp[1][c4 * CPT + k];
      ga[k] = lzp[2][c4 * CPT + k];
    } else {
      al[k] = coef[c0 + k];
      be[k] = coef[g.C + c0 + k];
      ga[k] = coef[2 * g.C + c0 + k];
    }
    stats[0][k] = stats[1][k] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < (WG ? 9 : 1); ++q) zero4(accw[q]);
#pragma unroll
  for (int q = 0; q < 9; ++q) unpack4(wraw[q], wt[q]);
  params_landed();   // parameters in registers (and the first rows in LDS)
  float win[3][3][CPT];   // three dy rows x three columns iw-1..iw+1 (roles rotate with the unroll)
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int d = 0; d < 3; ++d) zero4(win[r][d]);
  int slot = 0;
  // image-local row of input row ih = j0 + k - 1: its dy taps ih-1 / ih+1 are zero padding
  // across an image edge even where a tall strip continues into the next image
  int ihl = (j0 - 1) % g.Hi;
  if (ihl < 0) ihl += g.Hi;
  // dy row j0+k -> window row `into`; rows (ra, rb, rc) = dy rows ih-1, ih, ih+1 of input row
  // ih = j0+k-1, emitted when `emit`
  auto step = [&](int k, int into, bool emit, int ra, int rb, int rc) {
    ring_sync<(kDepth - 1) * 3>();
    issue(slot + kDepth < kRing ? slot + kDepth : slot + kDepth - kRing, k + kDepth);
    mem_fence_compiler();
    const char *sl = ring + slot * kStep;
    slot = slot + 1 == kRing ? 0 : slot + 1;
    const int oh = j0 + k;
    const bool rok = oh >= 0 && oh < g.H;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float m = (rok && cok[c]) ? 1.f : 0.f;
      float gv[CPT], yv[CPT];
      unpack4(lds8(sl, lcol + c, g.CC, c4 * CPT), gv);
      unpack4(lds8(sl + kSlotHalo, lcol + c, g.CC, c4 * CPT), yv);
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) {
        const float v = m * fmaf(al[kk], gv[kk], fmaf(be[kk], yv[kk], ga[kk]));
        if (into == 0) win[0][c][kk] = v;
        if (into == 1) win[1][c][kk] = v;
        if (into == 2) win[2][c][kk] = v;
      }
    }
    const int ih = oh - 1;
    float yp[CPT];
    unpack4(lds8(sl + 2 * kSlotHalo, lcol, g.CC, c4 * CPT), yp);
    const float mk[3] = {ihl != g.Hi - 1 ? 1.f : 0.f, 1.f, ihl != 0 ? 1.f : 0.f};   // dy rows ih+1, ih, ih-1
    ihl = ihl + 1 == g.Hi ? 0 : ihl + 1;
    float ar[3][CPT];
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {   // dx[ih][iw] += dy[ih+1-dh][iw+1-dw] * w[dh][dw]
      const int wr = dh == 0 ? rc : dh == 1 ? rb : ra;
      zero4(ar[dh]);
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int kk = 0; kk < CPT; ++kk) ar[dh][kk] = fmaf(win[wr][2 - dw][kk], wt[dh * 3 + dw][kk], ar[dh][kk]);
    }
    float acc[CPT];
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) acc[kk] = fmaf(mk[2], ar[2][kk], fmaf(mk[0], ar[0][kk], ar[1][kk]));
    const float e = emit ? 1.f : 0.f;
    if constexpr (WG) {
      float z[CPT];
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) z[kk] = e * relu6f(fmaf(yp[kk], s[kk], t[kk]));
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        const int wr = dh == 0 ? rc : dh == 1 ? rb : ra;
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int kk = 0; kk < CPT; ++kk)
            accw[WG ? dh * 3 + dw : 0][kk] = fmaf(mk[dh] * z[kk], win[wr][2 - dw][kk], accw[WG ? dh * 3 + dw : 0][kk]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) acc[kk] *= relu6_mask(yp[kk], s[kk], t[kk]);
    const uint2 packed = pack4(acc);
    float gr[CPT];
    unpack4(packed, gr);
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) {
      stats[0][kk] = fmaf(e, gr[kk], stats[0][kk]);
      stats[1][kk] = fmaf(e * gr[kk], yp[kk], stats[1][kk]);
    }
    bst8(ro, (emit && active) ? nhwc_off(tl.b, g.H, g.W, g.C, ih, iw, c0) : kOOB, packed);
  };
  for (int k = 0; k < nrows; k += 3) {   // dy row k -> window row k % 3
    step(k, 0, k >= 2, 1, 2, 0);
    if (k + 1 < nrows) step(k + 1, 1, k + 1 >= 2, 2, 0, 1);
    if (k + 2 < nrows) step(k + 2, 2, true, 0, 1, 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, g.TWc, red, tl.idx, dw_tiles(g), g.bn_rep);
  if constexpr (WG) block_channel_partials<9>(accw, wpart, g.C, g.CC, cbase, g.TWc, red, tl.idx);
  bn_fin_tail(g.fin);
}

// dgrad (stride 2): thread = one INPUT column iw; it needs dy columns owA (tap dw = 0 for odd
// iw, 1 for even iw) and owB = (iw-1)/2 (tap dw = 2, odd iw only).  Streams per step k: dy
// row o = o0 + k (g, y over the dy columns the tile touches) and yprev input rows 2(o-1),
// 2(o-1)+1 (own columns); step k >= 1 emits those two input rows (tap dh = 1 with dy row o-1;
// dh = 2 with row o-1 and dh = 0 with row o).  Per step: 4 DMA + 2 stores.
template <bool WG, int D = kDepth>
__global__ __launch_bounds__(256) void dw_dgrad_s2_lds_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ w, const bf16_t *__restrict__ yprev, const float *__restrict__ ps,
    const float *__restrict__ pt, bf16_t *__restrict__ gout, float *__restrict__ part, DwGeom g,
    float *__restrict__ wpart) {
  constexpr int kDepth = D, kRing = D + 1;
  constexpr int kStep = 4 * kSlotOwn;   // g, y (<= TWc/2 + 2 dy columns), yprev x 2
  __shared__ __attribute__((aligned(16))) char ring[kRing * kStep + 1024];
  __shared__ __attribute__((aligned(16))) float red[1024];
  char *dummy = ring + kRing * kStep;
  const int C4 = g.CC / CPT, CC8 = g.CC / 8;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int iw = tl.w0 + col;
  const bool active = col < g.TWc && iw < g.W;
  const int lcol = active ? col : 0;
  const int dcol0 = (tl.w0 - 1) >> 1;               // first dy column of the segment (may be -1)
  const int dcol1 = (tl.w0 + g.TWc) >> 1;           // last dy column (inclusive)
  const bool odd_w = iw & 1;
  const int owA = odd_w ? (iw + 1) >> 1 : iw >> 1;
  const int owB = odd_w ? (iw - 1) >> 1 : -1;       // -1: no tap (masked)
  const bool okA = active && owA < g.Wo, okB = active && owB >= 0;
  const int lA = okA ? owA - dcol0 : 0, lB = okB ? owB - dcol0 : 0;
  const uint32_t nin = (uint32_t)g.B * g.H * g.W * g.C * 2, nout = (uint32_t)g.B * g.Ho * g.Wo * g.C * 2;
  const rsrc_t ro = make_rsrc(gout, nin);

  float accA[WG ? 3 : 1][CPT], accB[WG ? 3 : 1][CPT];
#pragma unroll
  for (int r = 0; r < (WG ? 3 : 1); ++r) {
    zero4(accA[r]);
    zero4(accB[r]);
  }

  const int ih_end = min(tl.r0 + g.R, g.H);
  const int o0 = tl.r0 >> 1;                            // r0 even
  const int nrows = ((ih_end - 1) >> 1) + 1 - o0 + 1;   // dy rows o0 .. (ih_end-1)/2 + 1
  Stream sg, sy, sp;
  sg.init(gin, nout, g.Ho, g.Wo, g.C, tl.b, dcol0, (dcol1 - dcol0 + 1) * CC8, CC8, cbase);
  sy = sg;
  sy.set(yself, nout);
  sp.init(yprev, nin, g.H, g.W, g.C, tl.b, tl.w0, g.TWc * CC8, CC8, cbase);
  auto issue = [&](int slot, int k) {
    char *base = ring + slot * kStep;
    const int o = o0 + k;
    sg.issue(base, 0, 0, o, dummy);
    sy.issue(base + kSlotOwn, 0, 0, o, dummy);
    sp.issue(base + 2 * kSlotOwn, 0, 0, 2 * (o - 1), dummy);
    sp.issue(base + 3 * kSlotOwn, 0, 0, 2 * (o - 1) + 1, dummy);
  };
#pragma unroll
  for (int q = 0; q < kDepth; ++q) issue(q, q);
  // BN / weight parameters staged while the first kDepth rows are in flight
  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT], stats[2][CPT];
  // weight and producer-BN loads in flight across the lazy-finalize round trips
  uint2 wraw[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) wraw[q] = ldg8(w + (size_t)q * g.C + c0);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
  }
  if (g.lz) lazy_stage(g, cbase, 3);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    if (g.lz) {
      al[k] = lzp[0][c4 * CPT + k];
      be[k] = lzp[1][c4 * CPT + k];
      ga[k] = lzp[2][c4 * CPT + k];
    } else {
      al[k] = coef[c0 + k];
      be[k] = coef[g.C + c0 + k];
      ga[k] = coef[2 * g.C + c0 + k];
    }
    stats[0][k] = stats[1][k] = 0.f;
  }
  float wA[3][CPT], wB[3][CPT];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    float w0[CPT], w1[CPT], w2[CPT];
    unpack4(wraw[r * 3 + 0], w0);
    unpack4(wraw[r * 3 + 1], w1);
    unpack4(wraw[r * 3 + 2], w2);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      wA[r][k] = odd_w ? w0[k] : w1[k];
      wB[r][k] = odd_w ? w2[k] : 0.f;
    }
  }
  params_landed();   // parameters in registers (and the first rows in LDS)
  float dyb[2][2][CPT];   // two dy rows (roles alternate with the unroll) x columns A, B
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    zero4(dyb[r][0]);
    zero4(dyb[r][1]);
  }
  int slot = 0;
  // dy row o = o0+k -> dyb[into]; dyb[from] holds row o-1; emits input rows 2(o-1), 2(o-1)+1
  auto step = [&](int k, int into, int from) {
    ring_sync<(kDepth - 1) * 4>();
    issue(slot + kDepth < kRing ? slot + kDepth : slot + kDepth - kRing, k + kDepth);
    mem_fence_compiler();
    const char *sl = ring + slot * kStep;
    slot = slot + 1 == kRing ? 0 : slot + 1;
    const int o = o0 + k;
    const float mA = (okA && o < g.Ho) ? 1.f : 0.f, mB = (okB && o < g.Ho) ? 1.f : 0.f;
    {
      float gv[CPT], yv[CPT], hv[CPT], zv[CPT];
      unpack4(lds8(sl, lA, g.CC, c4 * CPT), gv);
      unpack4(lds8(sl + kSlotOwn, lA, g.CC, c4 * CPT), yv);
      unpack4(lds8(sl, lB, g.CC, c4 * CPT), hv);
      unpack4(lds8(sl + kSlotOwn, lB, g.CC, c4 * CPT), zv);
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) {
        const float va = mA * fmaf(al[kk], gv[kk], fmaf(be[kk], yv[kk], ga[kk]));
        const float vb = mB * fmaf(al[kk], hv[kk], fmaf(be[kk], zv[kk], ga[kk]));
        if (into == 0) {
          dyb[0][0][kk] = va;
          dyb[0][1][kk] = vb;
        } else {
          dyb[1][0][kk] = va;
          dyb[1][1][kk] = vb;
        }
      }
    }
    float(&cur)[2][CPT] = dyb[from];
    float(&nxt)[2][CPT] = dyb[into];
    float ypa[CPT], ypb[CPT];
    unpack4(lds8(sl + 2 * kSlotOwn, lcol, g.CC, c4 * CPT), ypa);
    unpack4(lds8(sl + 3 * kSlotOwn, lcol, g.CC, c4 * CPT), ypb);
    const int r = 2 * (o - 1);
    const float ea = k > 0 ? 1.f : 0.f;                      // row r exists (r < ih_end always)
    const float eb = (k > 0 && r + 1 < ih_end) ? 1.f : 0.f;
    float acc0[CPT], acc1[CPT];
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) {
      acc0[kk] = fmaf(cur[0][kk], wA[1][kk], cur[1][kk] * wB[1][kk]);
      acc1[kk] = fmaf(cur[0][kk], wA[2][kk], cur[1][kk] * wB[2][kk]);
      acc1[kk] = fmaf(nxt[0][kk], wA[0][kk], fmaf(nxt[1][kk], wB[0][kk], acc1[kk]));
    }
    if constexpr (WG) {
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) {
        const float za = ea * relu6f(fmaf(ypa[kk], s[kk], t[kk]));
        const float zb = eb * relu6f(fmaf(ypb[kk], s[kk], t[kk]));
        accA[WG ? 1 : 0][kk] = fmaf(za, cur[0][kk], accA[WG ? 1 : 0][kk]);
        accB[WG ? 1 : 0][kk] = fmaf(za, cur[1][kk], accB[WG ? 1 : 0][kk]);
        accA[WG ? 2 : 0][kk] = fmaf(zb, cur[0][kk], accA[WG ? 2 : 0][kk]);
        accB[WG ? 2 : 0][kk] = fmaf(zb, cur[1][kk], accB[WG ? 2 : 0][kk]);
        accA[0][kk] = fmaf(zb, nxt[0][kk], accA[0][kk]);
        accB[0][kk] = fmaf(zb, nxt[1][kk], accB[0][kk]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) {
      acc0[kk] *= relu6_mask(ypa[kk], s[kk], t[kk]);
      acc1[kk] *= relu6_mask(ypb[kk], s[kk], t[kk]);
    }
    const uint2 p0 = pack4(acc0), p1 = pack4(acc1);
    float g0[CPT], g1[CPT];
    unpack4(p0, g0);
    unpack4(p1, g1);
#pragma unroll
    for (int kk = 0; kk < CPT; ++kk) {
      stats[0][kk] = fmaf(ea, g0[kk], fmaf(eb, g1[kk], stats[0][kk]));
      stats[1][kk] = fmaf(ea * g0[kk], ypa[kk], fmaf(eb * g1[kk], ypb[kk], stats[1][kk]));
    }
    bst8(ro, (k > 0 && active) ? nhwc_off(tl.b, g.H, g.W, g.C, r, iw, c0) : kOOB, p0);
    bst8(ro, (eb != 0.f && active) ? nhwc_off(tl.b, g.H, g.W, g.C, r + 1, iw, c0) : kOOB, p1);
  };
  for (int k = 0; k < nrows; k += 2) {
    step(k, 0, 1);
    if (k + 1 < nrows) step(k + 1, 1, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float accw[WG ? 9 : 1][CPT];
  if constexpr (WG) {
#pragma unroll
    for (int dh = 0; dh < 3; ++dh)
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        accw[WG ? dh * 3 + 0 : 0][k] = odd_w ? accA[WG ? dh : 0][k] : 0.f;
        accw[WG ? dh * 3 + 1 : 0][k] = odd_w ? 0.f : accA[WG ? dh : 0][k];
        accw[WG ? dh * 3 + 2 : 0][k] = accB[WG ? dh : 0][k];
      }
  }
  __syncthreads();
  block_channel_partials<2>(stats, part, g.C, g.CC, cbase, g.TWc, red, tl.idx, dw_tiles(g), g.bn_rep);
  if constexpr (WG) block_channel_partials<9>(accw, wpart, g.C, g.CC, cbase, g.TWc, red, tl.idx);
  bn_fin_tail(g.fin);
}

// wgrad: dW[tap][c] partials per workgroup [P][9][C]; thread = one output column.  Streams per
// step k: input row j0+k (z = relu6(BN(yprev)), halo columns) and the dy rows (g, y; own
// columns) of the output row the step may complete.  Per step: 3 DMA.  T: tall strips (masks
// for the taps across an image edge; a separate instantiation, the masks cost the plain kernel
// its 4th wave per SIMD: 126 -> 130 VGPRs).
template <int S, bool T = false>
__global__ __launch_bounds__(256) void dw_wgrad_lds_kernel(
    const bf16_t *__restrict__ gin, const bf16_t *__restrict__ yself, const float *__restrict__ coef,
    const bf16_t *__restrict__ yprev, const float *__restrict__ ps, const float *__restrict__ pt,
    float *__restrict__ part, DwGeom g) {
  constexpr int kSlotX = S == 1 ? kSlotHalo : kSlotS2;
  constexpr int kStep = kSlotX + 2 * kSlotOwn;
  __shared__ __attribute__((aligned(16))) char ring[kRing * kStep + 1024];
  __shared__ __attribute__((aligned(16))) float lds[1024];
  char *dummy = ring + kRing * kStep;
  const int C4 = g.CC / CPT, CC8 = g.CC / 8;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, col = tid / C4;
  const Tile tl = tile_of(g);
  const int cbase = tl.slab * g.CC;
  const int c0 = cbase + c4 * CPT;
  const int ow = tl.w0 + col;
  const bool active = col < g.TWc && ow < g.Wo;
  const int lcol = active ? col * S : 0, lown = active ? col : 0;
  const uint32_t nin = (uint32_t)g.B * g.H * g.W * g.C * 2, nout = (uint32_t)g.B * g.Ho * g.Wo * g.C * 2;

  const int oh_end = min(tl.r0 + g.R, g.Ho);
  const int j0 = tl.r0 * S - 1;
  const int nrows = (oh_end - 1) * S + 1 - j0 + 1;
  const int iw0 = ow * S - 1;
  bool cok[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) cok[d] = active && iw0 + d >= 0 && iw0 + d < g.W;
  Stream sx, sg, sy;
  sx.init(yprev, nin, g.H, g.W, g.C, tl.b, tl.w0 * S - 1, ((g.TWc - 1) * S + 3) * CC8, CC8, cbase);
  sg.init(gin, nout, g.Ho, g.Wo, g.C, tl.b, tl.w0, g.TWc * CC8, CC8, cbase);
  sy = sg;
  sy.set(yself, nout);
  // output row completed at step k: S = 1: r0 + k - 2; S = 2 (even k): r0 + (k - 2) / 2
  auto out_row = [&](int k) { return S == 1 ? tl.r0 + k - 2 : tl.r0 + ((k - 2) >> 1); };
  auto issue = [&](int slot, int k) {
    char *base = ring + slot * kStep;
    sx.issue(base, 0, 0, j0 + k, dummy);
    const int oh = out_row(k);
    const int ohc = oh < oh_end ? oh : -1;   // rows of the next tile are never needed
    sg.issue(base + kSlotX, 0, 0, ohc, dummy);
    sy.issue(base + kSlotX + kSlotOwn, 0, 0, ohc, dummy);
  };
#pragma unroll
  for (int q = 0; q < kDepth; ++q) issue(q, q);
  // BN / weight parameters staged while the first kDepth rows are in flight
  float al[CPT], be[CPT], ga[CPT], s[CPT], t[CPT];
  float accw[9][CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    al[k] = coef[c0 + k];
    be[k] = coef[g.C + c0 + k];
    ga[k] = coef[2 * g.C + c0 + k];
    s[k] = ps[c0 + k];
    t[k] = pt[c0 + k];
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) zero4(accw[q]);
  // a use of every parameter here: hipcc waits for their loads at this point (the restrict
  // loads may otherwise sink below the wait and be waited for inside the row loop, where the
  // wait also covers the ring's in-flight rows)
#pragma unroll
  for (int k = 0; k < CPT; ++k) asm volatile("" ::"v"(al[k]), "v"(be[k]), "v"(ga[k]), "v"(s[k]), "v"(t[k]));
  params_landed();   // parameters in registers (and the first rows in LDS)
  float win[3][3][CPT];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int d = 0; d < 3; ++d) zero4(win[r][d]);
  int slot = 0;
  // image-local row of input row j0 + k (stride 1, tall strips: see the forward)
  int ihl = j0 % g.Hi;
  if (ihl < 0) ihl += g.Hi;
  auto step = [&](int k, int into, bool emit, int ra, int rb, int rc) {
    ring_sync<(kDepth - 1) * 3>();
    issue(slot + kDepth < kRing ? slot + kDepth : slot + kDepth - kRing, k + kDepth);
    mem_fence_compiler();
    const char *sl = ring + slot * kStep;
    slot = slot + 1 == kRing ? 0 : slot + 1;
    const int ih = j0 + k;
    const bool rok = ih >= 0 && ih < g.H;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float v[CPT];
      unpack4(lds8(sl, lcol + d, g.CC, c4 * CPT), v);
      const float m = (rok && cok[d]) ? 1.f : 0.f;
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) {
        const float a = m * relu6f(fmaf(v[kk], s[kk], t[kk]));
        if (into == 0) win[0][d][kk] = a;
        if (into == 1) win[1][d][kk] = a;
        if (into == 2) win[2][d][kk] = a;
      }
    }
    float mr[3] = {1.f, 1.f, 1.f};   // tap rows 0 / 2 inside the output row's image (stride 1)
    if constexpr (T) {
      const int ohl = ihl == 0 ? g.Hi - 1 : ihl - 1;
      mr[0] = ohl != 0 ? 1.f : 0.f;
      mr[2] = ohl != g.Hi - 1 ? 1.f : 0.f;
      ihl = ihl + 1 == g.Hi ? 0 : ihl + 1;
    }
    if (emit) {
      float dy[CPT], gv[CPT], yv[CPT];
      unpack4(lds8(sl + kSlotX, lown, g.CC, c4 * CPT), gv);
      unpack4(lds8(sl + kSlotX + kSlotOwn, lown, g.CC, c4 * CPT), yv);
      const float m = active ? 1.f : 0.f;
#pragma unroll
      for (int kk = 0; kk < CPT; ++kk) dy[kk] = m * fmaf(al[kk], gv[kk], fmaf(be[kk], yv[kk], ga[kk]));
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int wr = r == 0 ? ra : r == 1 ? rb : rc;
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int kk = 0; kk < CPT; ++kk)
            accw[r * 3 + dw][kk] = fmaf(T ? mr[r] * dy[kk] : dy[kk], win[wr][dw][kk], accw[r * 3 + dw][kk]);
      }
    }
  };
  for (int k = 0; k < nrows; k += (S == 1 ? 3 : 4)) {
    if constexpr (S == 1) {
      step(k, 0, k >= 2, 1, 2, 0);
      if (k + 1 < nrows) step(k + 1, 1, k + 1 >= 2, 2, 0, 1);
      if (k + 2 < nrows) step(k + 2, 2, true, 0, 1, 2);
    } else {
      step(k, 0, k > 0, 2, 1, 0);
      if (k + 1 < nrows) step(k + 1, 1, false, 0, 1, 2);
      if (k + 2 < nrows) step(k + 2, 2, true, 0, 1, 2);
      if (k + 3 < nrows) step(k + 3, 1, false, 0, 1, 2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  block_channel_partials<9>(accw, part, g.C, g.CC, cbase, g.TWc, lds, tl.idx);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
// channels per workgroup: the largest multiple of 8 dividing C that is <= 64 (C % 8 == 0 is
// checked by the caller): 16-B channel chunks for the LDS-staged row segments
int dw_cc(int C) {
  for (int cc = 64; cc >= 8; cc -= 8)
    if (C % cc == 0) return cc;
  return 8;
}

// Widest tile (columns) a CC-channel slab supports: 256 threads of CPT channels, and the
// LDS-DMA row segments of every kernel kind within their ring slots (whole 64-chunk wave
// pieces: halo rows kSlotHalo = 192 chunks, own-column rows kSlotOwn = 128, stride-2 input
// rows kSlotS2 = 256; the dgrad s2 dy segment spans ~TWc/2 + 2 columns in an own slot).
static int dw_twc_max(int cc, int kind, int stride) {
  const int c4 = cc / CPT, cc8 = cc / 8;
  auto fits = [&](int t) {
    if (t * cc8 > 128) return false;
    if (stride == 1) return (t + 2) * cc8 <= 192;
    if (kind != 1) return (2 * t + 1) * cc8 <= 256;
    return (t / 2 + 2) * cc8 <= 128;
  };
  int t = 256 / c4;
  while (t > 0 && !fits(t)) --t;
  return t;
}

// Channel slab of a narrow map: with the default CC (<= 64) a 7-column map leaves half of
// the 256 threads without a column (C4 = 16 threads x 7 columns); a wider slab (a multiple
// of 8 dividing C, <= 128) gives every column more channel lanes: 7x7x960 -> CC = 120,
// 210 active threads instead of 112 (MobileNetV2 bs128: 5.17 -> 5.05 ms/step, round 2).
static int dw_cc_narrow(int C, int gw, int kind, int stride, int cc0) {
  if (dw_twc_max(cc0, kind, stride) <= gw) return cc0;
  int best = cc0, best_act = (cc0 / CPT) * gw;
  for (int cc = 8; cc <= 128; cc += 8) {
    if (C % cc) continue;
    const int t = dw_twc_max(cc, kind, stride);
    if (t < 1) continue;
    const int act = (cc / CPT) * (t < gw ? t : gw);
    if (act > best_act) best = cc, best_act = act;
  }
  return best;
}

// Occupancy-aware geometry (bit per kind in g_dw_geom_mask: 1 fwd, 2 dgrad, 4 wgrad).  A
// workgroup walks its R-row strip step by step (one DMA-ring row per step), so a launch lasts
// about ceil(workgroups / resident slots) rounds x (steps per strip + ring fill); the default
// geometry (CC <= 64, R = 56) can land just past a round: 56x56x144 dgrad = 1152 workgroups
// on 512 slots (the fused-wgrad dgrad holds 175 VGPRs: 2 per CU) = 3 rounds, where 72-channel
// slabs of 14 columns (56 = 4 x 14) make 1024 = 2 rounds.  The model picks (CC, R) over the
// multiples of 8 dividing C (<= 128) and 1..8 strips per map, and replaces the default only
// when it predicts >= 10 % fewer step-rounds.  Slots = 256 CUs x resident workgroups per CU of
// each kernel family at its default ring depth (VGPR / LDS bound, from the gfx950 ISA):
// forward 4, weight gradient 3, dgrad stride 2: 3, stride 1: 2 on the >= 56-row maps (the
// executor fuses the weight gradient there; the partial count must not depend on whether a
// launch fuses it) and 3 below.
// Measured (profiles/r3c_dw_geom_ab.txt): 56x56x144 dgrad 209 -> 157 us and forward 57 -> 48 us
// (both 72-channel slabs of 14 columns), but the model's stride-2 picks (forward 112x112x96:
// 91 -> 116 us, dgrad 56x56x144: 89 -> 117 us) and the 28x28 dgrad (38 -> 45 us) were slower --
// rounds are not the whole cost where the kernel is bandwidth-bound or the strip gets short.
// So by default (mask 3) it applies to the stride-1 forward / dgrad on >= 56-row maps only;
// bit 8 lifts that restriction (experiments: dw_set_geom_mode).
int g_dw_geom_mask = 3;
// Tall geometry for the stride-1 forward / dgrad on small maps (<= 14 rows): the batch is
// stacked into one B*H-row image and a workgroup walks a strip of g_dw_tall rows across image
// boundaries (the window taps that would cross an image edge are masked per row), so the DMA
// ring fill, the parameter staging and the statistics epilogue are paid per strip instead of
// per 7- or 14-row image.  g_dw_tall = strip rows, 0: off (dw_set_tall_rows).  Measured (scripts/dw_bench.py,
// profiles/r4_dw_tall_sweep.txt): 14-row strips (two 7x7 images) take 7x7x960 forward 18.8 -> 17.7
// and dgrad 35.4 -> 30.2 us (bench 4.525 / 4.530 vs 4.535 / 4.551 ms/step); longer strips are
// slower (21 / 28 / 42 / 56 rows: fewer workgroups, and a strip row costs ~0.2 us of DMA latency
// per workgroup), 14 leaves the 14x14 tiling unchanged.
int g_dw_tall = 14;
// Small-map stride-1 dgrad (tall geometry on): slab width and strip length chosen together so
// the launch fits one round of resident workgroups (3 per CU) where it can -- e.g. 14x14x384:
// 64-channel slabs of all 14 columns (768 workgroups) instead of 96-channel slabs of 10 columns
// (1024, two rounds).  Cost = rounds x (strip rows + g_dw_fix), ties to more active lanes.
// dw_set_small_dgrad(0): off; kDwFix: the fixed per-strip cost in rows.  Measured
// (profiles/r4_dw_small_dgrad.txt): 14x14x576 59.7 -> 52.6-54.8 us (21-row strips of 72-channel
// slabs, 688 workgroups); 14x14x384 unchanged at 37.1 us although it now fits one round;
// bench 4.506-4.516 vs 4.507-4.526 ms/step.
int g_dw_small_dgrad = 1;
// (tall strips for the side-stream weight gradient measured neutral at 28 rows and slower at 14,
// profiles/r4_dw_tall_wgrad.txt: the weight gradient keeps per-image strips)
static constexpr int kDwFix = 12;
static int dw_occ(int kind, int stride, int gh) {
  return kind == 0 ? 4 : kind == 2 ? 3 : (stride == 1 && gh >= 56 ? 2 : 3);
}
static int dw_fix_rows(int kind, int stride, int R, int gh) {
  if (kind == 1 && stride == 2 && (R & 1)) ++R;  // dgrad s2 tiles start on even input rows
  if (R > gh) R = (kind == 1 && stride == 2) ? ((gh + 1) & ~1) : gh;
  return R;
}
static long long dw_cost(int kind, int stride, int B, int gh, int gw, int C, int cc, int twc, int R) {
  const long long nwg = (long long)B * ((gh + R - 1) / R) * ((gw + twc - 1) / twc) * (C / cc);
  const long long slots = 256LL * dw_occ(kind, stride, gh);
  const int steps = (kind == 1 && stride == 2) ? R / 2 : R;
  return ((nwg + slots - 1) / slots) * (steps + 4);
}

// kind 0 = fwd (tiles over the output grid), 1 = dgrad (input grid), 2 = wgrad (output grid)
DwGeom dw_geom(int kind, int B, int H, int W, int C, int stride) {
  DwGeom g;
  g.bn_rep = g_bn_rep;
  g.fin = nullptr;
  g.lz = nullptr;
  g.B = B;
  g.H = H;
  g.W = W;
  g.C = C;
  g.Ho = (H - 1) / stride + 1;
  g.Wo = (W - 1) / stride + 1;
  g.Hi = H;
  const bool tall = kind <= 1 && g_dw_tall > 0 && stride == 1 && H <= 14 && B > 1;
  if (tall) {
    g.B = 1;
    g.H = g.Ho = B * H;
  }
  const int gw = kind == 1 ? W : g.Wo, gh = kind == 1 ? g.H : g.Ho;
  g.CC = dw_cc_narrow(C, gw, kind, stride, dw_cc(C));
  int twc = dw_twc_max(g.CC, kind, stride);
  if (twc > gw) twc = gw;
  g.TWc = twc;
  int R = tall ? g_dw_tall : (kind == 2 ? kWRows : kRows);
  R = dw_fix_rows(kind, stride, R, gh);
  if (tall && kind == 1 && g_dw_small_dgrad) {
    long long best = -1;
    int best_act = 0;
    const int rcand[3] = {g_dw_tall, 21, 28};
    for (int i = 0; i < 3; ++i) {
      const int r = rcand[i] < gh ? rcand[i] : gh;
      for (int cc = 8; cc <= 128; cc += 8) {
        if (C % cc) continue;
        int t = dw_twc_max(cc, kind, stride);
        if (t < 1) continue;
        if (t > gw) t = gw;
        const long long nwg = (long long)((gh + r - 1) / r) * ((gw + t - 1) / t) * (C / cc);
        const long long cost = ((nwg + 767) / 768) * (r + kDwFix);
        const int act = (cc / CPT) * gw / ((gw + t - 1) / t);   // active lanes per workgroup, on average
        if (best < 0 || cost < best || (cost == best && act > best_act))
          best = cost, best_act = act, g.CC = cc, g.TWc = t, R = r;
      }
    }
  }
  if (!tall && (g_dw_geom_mask & (1 << kind)) && ((g_dw_geom_mask & 8) || (kind <= 1 && stride == 1 && gh >= 56))) {
    const long long cur = dw_cost(kind, stride, B, gh, gw, C, g.CC, g.TWc, R);
    long long best = cur;
    int bcc = g.CC, btw = g.TWc, bR = R;
    for (int ns = 1; ns <= 8; ++ns) {
      const int r = dw_fix_rows(kind, stride, (gh + ns - 1) / ns, gh);
      if (ns > 1 && r < 7) break;
      for (int cc = 8; cc <= 128; cc += 8) {
        if (C % cc) continue;
        int t = dw_twc_max(cc, kind, stride);
        if (t < 1) continue;
        if (t > gw) t = gw;
        const long long c = dw_cost(kind, stride, B, gh, gw, C, cc, t, r);
        if (c < best) best = c, bcc = cc, btw = t, bR = r;
      }
    }
    if (best * 10 <= cur * 9) g.CC = bcc, g.TWc = btw, R = bR;
  }
  g.R = R;
  g.tiles_w = (gw + g.TWc - 1) / g.TWc;
  g.tiles_h = (gh + g.R - 1) / g.R;
  return g;
}

int dw_grid_x(const DwGeom &g) { return g.B * g.tiles_h * g.tiles_w; }
}  // namespace

// geometry mode (tests / tuning): must not change while workspaces sized by the *_num_partials /
// *_workspace_floats of another mode are in use
void dw_set_geom_mode(int mask) { g_dw_geom_mask = mask; }
int dw_geom_mode() { return g_dw_geom_mask; }
void dw_set_tall_rows(int rows) { g_dw_tall = rows; }
void dw_set_small_dgrad(int on) { g_dw_small_dgrad = on; }
int dw_small_dgrad() { return g_dw_small_dgrad; }
int dw_tall_rows() { return g_dw_tall; }

int dw_fwd_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(0, B, H, W, C, stride)); }
int dw_dgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(1, B, H, W, C, stride)); }
int dw_wgrad_num_partials(int B, int H, int W, int C, int stride) { return dw_grid_x(dw_geom(2, B, H, W, C, stride)); }

void launch_dw_fwd(const bf16_t *x, const float *in_s, const float *in_t, int act, const bf16_t *w,
                   bf16_t *y, float *part, int B, int H, int W, int C, int stride, hipStream_t st) {
  DwGeom g = dw_geom(0, B, H, W, C, stride);
  g.fin = take_bn_fin();
  g.lz = take_bn_lz();
  const dim3 grid(dw_grid_x(g) * (C / g.CC)), block(256);
  // ring depth 4 rows in flight (3: neutral; 6 / 8 on the small maps: neutral, round 2 / 4 sweeps)
#define DWF(S_, A_) \
  hipLaunchKernelGGL((dw_fwd_lds_kernel<S_, A_, 4>), grid, block, 0, st, x, in_s, in_t, w, y, part, g);
  if (stride == 1) {
    if (act == ACT_BN_RELU6) { DWF(1, ACT_BN_RELU6) }
    else { DWF(1, ACT_NONE) }
  } else {
    if (act == ACT_BN_RELU6) { DWF(2, ACT_BN_RELU6) }
    else { DWF(2, ACT_NONE) }
  }
#undef DWF
}

int colsum_rows(int R);

void launch_dw_dgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *w,
                     const bf16_t *yprev, const float *ps, const float *pt, bf16_t *gout,
                     float *part, int B, int H, int W, int C, int stride, float *wpart, hipStream_t st) {
  DwGeom g = dw_geom(1, B, H, W, C, stride);
  g.fin = take_bn_fin();
  g.lz = take_bn_lz();
  const dim3 grid(dw_grid_x(g) * (C / g.CC)), block(256);
  // ring depth (rows in flight) 3: 39 KB of LDS per workgroup, 4 workgroups per CU instead of 3
  // at depth 4 (MobileNetV2 bs128: 5.02 -> 4.94 ms/step); 2 / 4 / 5 (also for the VGPR-bound fused
  // dgrad + wgrad variants) measured neutral or slower (profiles/r3c_dw_ddepth_ab.txt)
#define DWD(KER, WGF) \
  hipLaunchKernelGGL((KER<WGF, 3>), grid, block, 0, st, gin, yself, coef, w, yprev, ps, pt, gout, part, g, wpart);
  if (wpart) {
    if (stride == 1) { DWD(dw_dgrad_s1_lds_kernel, true) }
    else { DWD(dw_dgrad_s2_lds_kernel, true) }
  } else {
    if (stride == 1) { DWD(dw_dgrad_s1_lds_kernel, false) }
    else { DWD(dw_dgrad_s2_lds_kernel, false) }
  }
#undef DWD
}

// wpart of the fused dgrad + wgrad: [P][9][C] with P = dgrad tiles, + level-1 rows of the reduction
long long dw_dgrad_wgrad_workspace_floats(int B, int H, int W, int C, int stride) {
  const int P = dw_grid_x(dw_geom(1, B, H, W, C, stride));
  return (long long)(P + colsum_rows(P)) * 9 * C;
}

void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st, bool stem36 = false);

void launch_dw_wgrad(const bf16_t *gin, const bf16_t *yself, const float *coef, const bf16_t *yprev,
                     const float *ps, const float *pt, float *part, float *grad, int B, int H, int W,
                     int C, int stride, hipStream_t st) {
  const DwGeom g = dw_geom(2, B, H, W, C, stride);
  const int P = dw_grid_x(g);
  const dim3 grid(P * (C / g.CC)), block(256);
  if (stride == 1)
    hipLaunchKernelGGL((dw_wgrad_lds_kernel<1>), grid, block, 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  else
    hipLaunchKernelGGL((dw_wgrad_lds_kernel<2>), grid, block, 0, st, gin, yself, coef, yprev, ps, pt, part, g);
  // deterministic two-level reduction of the [P][9C] partials -> grad [9][C] (tap-major)
  launch_wgrad_reduce(part, P, 9LL * C, grad, st);
}
