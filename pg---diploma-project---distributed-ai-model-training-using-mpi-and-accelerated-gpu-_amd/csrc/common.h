// Shared device helpers for the pgdist gfx950 (MI355X / CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16, viewed as row-major [M = N*H*W][C]
//   * bf16 values travel as raw 16-bit patterns (uint16) in memory and are
//     converted with the gfx950 v_cvt_pk_bf16_f32 instruction (RNE, NaN-safe)
//   * all global traffic of streaming kernels is 16 B per lane (8 x bf16)
//   * wave = 64 lanes; workgroups are multiples of 64 threads
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short bf16_t;  // raw bf16 bits
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef int i32x8_t __attribute__((ext_vector_type(8)));

#define PG_DEVICE __device__ __forceinline__

PG_DEVICE float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
PG_DEVICE bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// 8 x bf16 packed in a uint4 (16 bytes)
struct alignas(16) bf16x8_pack { uint4 v; };

PG_DEVICE void unpack8(const uint4 &u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// two floats -> two round-to-nearest-even bf16 in one v_cvt_pk_bf16_f32 (converting them one
// at a time costs two conversions and an OR; the ext_vector __builtin_convertvector form of the
// same instruction kept some arrays of conv_wgrad_kernel out of registers -> scratch)
PG_DEVICE uint32_t pack2(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Store one 16x16 f32 MFMA accumulator fragment (lane: rows row0 + 4*(lane>>4) + j, j = 0..3, of
// column col0 + (lane & 15)) as bf16 into a row-major LDS tile T (pitch ld elements): one
// ds_write_b16 per element.  (Completing 4-byte column pairs across lanes with a DPP move was
// measured slower on MI355X -- MobileNetV2 4.69-4.70 vs 4.66 ms/step, ResNet-50 11.90-11.94 vs
// 11.68-11.69 -- the epilogue is not bound by its LDS write count; docs/PERF_NOTES.md round 3.)
PG_DEVICE void frag_store_bf16(bf16_t *T, int ld, int row0, int col0, float v0, float v1, float v2, float v3) {
  const int lane = threadIdx.x & 63;
  const float v[4] = {v0, v1, v2, v3};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    T[(row0 + 4 * (lane >> 4) + j) * ld + col0 + (lane & 15)] = __builtin_bit_cast(bf16_t, (__bf16)v[j]);
}

PG_DEVICE uint4 pack8(const float (&f)[8]) {
  uint4 u;
  u.x = pack2(f[0], f[1]);
  u.y = pack2(f[2], f[3]);
  u.z = pack2(f[4], f[5]);
  u.w = pack2(f[6], f[7]);
  return u;
}

PG_DEVICE uint4 ldg16(const void *p) { return *reinterpret_cast<const uint4 *>(p); }
PG_DEVICE void stg16(void *p, const uint4 &v) { *reinterpret_cast<uint4 *>(p) = v; }

PG_DEVICE float relu6f(float x) { return fminf(fmaxf(x, 0.f), 6.f); }

// Wave-level reductions (64 lanes)
PG_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Counter-based RNG (splitmix64 finaliser) — deterministic per (seed, counter).
PG_DEVICE uint64_t pg_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
PG_DEVICE float pg_uniform(uint64_t seed, uint64_t ctr) {  // [0,1)
  return (float)(pg_mix64(seed ^ pg_mix64(ctr)) >> 40) * (1.0f / 16777216.0f);
}

// Prologue transform applied to an activation operand when it is read.
enum ActMode : int {
  ACT_NONE = 0,      // x as stored (materialised tensor)
  ACT_BN_RELU6 = 1,  // relu6(x * scale[c] + shift[c])  (BN-apply of the producer, fused)
  ACT_BN = 2,        // x * scale[c] + shift[c]
};

template <int MODE>
PG_DEVICE float act_apply(float x, float s, float t) {
  if constexpr (MODE == ACT_BN_RELU6) return relu6f(fmaf(x, s, t));
  else if constexpr (MODE == ACT_BN) return fmaf(x, s, t);
  else return x;
}

// relu6 pass-through mask on the pre-clamp value a = y*s+t
PG_DEVICE float relu6_mask(float y, float s, float t) {
  float a = fmaf(y, s, t);
  return (a > 0.f && a < 6.f) ? 1.f : 0.f;
}

// OCP fp8 e4m3fn (gfx950 native format): largest finite magnitude
constexpr float kFp8Max = 448.f;

// 8 floats -> 8 e4m3 bytes (element j in byte j), scaled by sc and saturated to +-448:
// the A/B fragment of v_mfma_f32_16x16x32_fp8_fp8 (k = 8*(lane>>4) .. +7 of one row)
PG_DEVICE long pack_fp8x8(const float (&v)[8], float sc) {
  float q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = fminf(fmaxf(v[j] * sc, -kFp8Max), kFp8Max);
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
  return (long)(unsigned)lo | ((long)(unsigned)hi << 32);
}

// ---------------------------------------------------------------------------
// Raw buffer loads / stores with hardware bounds checking (gfx950 SRD, stride 0).  A masked
// lane passes the offset kOOB: its load returns 0 and its store is dropped, so a kernel needs
// no branch around a memory instruction — hipcc then counts vmcnt exactly instead of waiting
// vmcnt(0) at every join (conditional loads defeat software prefetching).  The descriptor is
// built from kernel arguments only (wave-uniform: no waterfall loops).  Tensors < 2 GiB.
// ---------------------------------------------------------------------------
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;

PG_DEVICE rsrc_t make_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
// the same descriptor as raw SGPR words, for inline-asm buffer instructions
PG_DEVICE u32x4_t make_srd(const void *base, uint32_t bytes) {
  const size_t a = (size_t)base;
  return u32x4_t{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}
// LDS DMA by inline asm: one buffer_load_dwordx4 ... lds, 16 B per lane into the wave's
// 1-KiB piece at `dst` (wave-uniform).  hipcc tracks the builtin form as a pending write to
// the LDS object and waits for it (vmcnt) before any later read of that object it cannot prove
// disjoint, i.e. also for stages issued ahead of the one being read: software pipelines over
// a ring then serialise.  Users order their ring reads with their own counted waits.  Sets M0
// (no other code in the users' translation units uses it).
PG_DEVICE void lds_dma16(const u32x4_t &srd, const void *dst, uint32_t voff) {
  const uint32_t m0v =
      __builtin_amdgcn_readfirstlane((uint32_t)(size_t)((const __attribute__((address_space(3))) char *)dst));
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0v), "v"(voff), "s"(srd)
               : "memory", "m0");
}
PG_DEVICE uint4 bld16(rsrc_t r, uint32_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
PG_DEVICE uint2 bld8(rsrc_t r, uint32_t off) {
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  return make_uint2(v.x, v.y);
}
PG_DEVICE void bst8(rsrc_t r, uint32_t off, const uint2 &v) {
  u32x2_t d;
  d.x = v.x;
  d.y = v.y;
  __builtin_amdgcn_raw_buffer_store_b64(d, r, (int)off, 0, 0);
}

PG_DEVICE void bst16(rsrc_t r, uint32_t off, const uint4 &v) {
  u32x4_t d;
  d.x = v.x;
  d.y = v.y;
  d.z = v.z;
  d.w = v.w;
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)off, 0, 0);
}
// byte offset of element i of a bf16 tensor, or kOOB
PG_DEVICE uint32_t boff(bool ok, size_t i) { return ok ? (uint32_t)(i * 2) : kOOB; }

// ---------------------------------------------------------------------------
// BatchNorm statistics of the MobileNetV2 producers: every workgroup adds its per-channel
// partial sums (sum, sum of squares | sum g, sum g*y) with float atomics into one of
// kBnRep replica rows of a zeroed accumulator [rows][2][C] (rows = min(kBnRep, workgroup
// partial rows)); the finalize then reduces rows <= kBnRep instead of one row per workgroup
// (up to ~2k), and the accumulator of every BN of a step is zeroed by one memset.
// Replicas (row % rep) spread the same-address atomics over separate lines.
// The replica count is a launch argument taken from g_bn_rep (host): kBnRep by default, or
// "unbounded" in deterministic mode (bn_set_rep), where every workgroup owns its row, adds to
// zero exactly once, and the finalize sums the rows in a fixed order (bitwise reproducible).
// ---------------------------------------------------------------------------
constexpr int kBnRep = 8;
extern int g_bn_rep;   // host: replica rows the launchers pass to the producers
PG_DEVICE void bn_part_add(float *part, int row, int nrows, int rep, int C, int s, int c, float v) {
  rep = nrows < rep ? nrows : rep;
  atomicAdd(part + ((size_t)(row % rep) * 2 + s) * C + c, v);
}

#define PG_CHECK_LAUNCH() ((void)hipGetLastError())
