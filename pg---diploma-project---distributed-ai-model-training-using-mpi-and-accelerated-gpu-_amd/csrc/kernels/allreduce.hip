// Peer-to-peer collectives over xGMI for the data-parallel gradient buckets.
//
// Reference: the DDP Reducer's bucketed NCCL all-reduce AVG overlapped with backward
// (cifar10_mpi_mobilenet_224.py:142-145,179) and the BN-buffer broadcast
// from rank 0 (N5).  On an MI355X node every GPU has 7 point-to-point xGMI links, so a
// ring moves each byte over ONE link per step, while a direct scheme reads all 7 peers at
// once; the MobileNetV2 gradient (8.95 MB per step, ~1.5 MiB buckets) is latency-bound,
// which is where these kernels are meant to beat RCCL's rings:
//
//   one-shot  (AR_ONESHOT): every rank writes its bucket into its own staging region, one
//             barrier, then every rank reads the N staged buffers (N-1 of them over xGMI, all
//             links at once) and sums them in rank order 0..N-1 (fp32) — bitwise identical on
//             every rank, one barrier of latency.
//   two-shot  (AR_TWOSHOT): copy-in, barrier, rank r reduces segment r (1/N of the bucket)
//             from every rank's staging and publishes it, barrier, every rank gathers the
//             other N-1 reduced segments: 2(N-1)/N of the bucket over the links instead of
//             (N-1), two barriers.
//   broadcast (AR_BROADCAST): root copy-in, barrier, every other rank copies root's region.
//
// Optional bf16 wire format (all-reduce): the staged copy is bf16, sums are fp32; the result
// is rounded to bf16 identically on every rank, so replicas stay bitwise equal.
//
// Memory model (p2p.h): staging is UNCACHED device memory; payload stores and loads use
// system-coherent buffer instructions (sc0 sc1), every storing wave drains its stores
// (vmcnt(0)) before the block barrier, then a system-scope release fence and ONE lane per
// peer stores {call signature, epoch} into the peer's 8-byte signal slot with a system-scope
// atomic; ONE wave polls this rank's slots with relaxed system-scope loads (+ s_sleep) and
// issues a system-scope acquire fence once every peer is there.  The poll is bounded by the
// realtime clock: a rank that never arrives, or one that is out of step (skipped, added or
// reordered collectives), makes the kernel set its error word and exit instead of hanging the
// GPU or reducing mismatched buffers.  A set error word poisons the communicator: every later
// collective of that rank exits at once without signalling, so its peers time out as well and
// every rank's host check (Comm::error -> NativeComm.check_all) fails the job.
//
// Single-process emulation: the grid holds nlocal * G blocks, block -> (local rank, block),
// each local rank with its own descriptor, buffer and staging (tests / microbenchmarks of N
// ranks on one GPU; all N*G blocks are co-resident: N*G <= 8 * 64 one-wave-per-SIMD blocks).
#include "../common.h"
#include "../p2p.h"

namespace {

constexpr int kSysCoherent = 1 | 16;   // buffer cache policy sc0 | sc1: system scope, no stale copies

PG_DEVICE uint4 ld_sys(rsrc_t r, uint32_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kSysCoherent);
  return make_uint4(v.x, v.y, v.z, v.w);
}

PG_DEVICE void st_sys(rsrc_t r, uint32_t off, const uint4 &v) {
  u32x4_t d;
  d.x = v.x;
  d.y = v.y;
  d.z = v.z;
  d.w = v.w;
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)off, 0, kSysCoherent);
}

PG_DEVICE void add8(float (&acc)[8], const uint4 &lo, const uint4 &hi) {
  acc[0] += __uint_as_float(lo.x);
  acc[1] += __uint_as_float(lo.y);
  acc[2] += __uint_as_float(lo.z);
  acc[3] += __uint_as_float(lo.w);
  acc[4] += __uint_as_float(hi.x);
  acc[5] += __uint_as_float(hi.y);
  acc[6] += __uint_as_float(hi.z);
  acc[7] += __uint_as_float(hi.w);
}

PG_DEVICE void add8_bf(float (&acc)[8], const uint4 &u) {
  float f[8];
  unpack8(u, f);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += f[j];
}

PG_DEVICE uint4 f4u(const float a, const float b, const float c, const float d) {
  return make_uint4(__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d));
}

// Block-wide barrier with the same block of every rank (see the file comment).  Returns false
// (and sets this rank's error word) if a peer did not arrive within the timeout (bit 0), a peer
// is out of step with this rank (bit 1: its epoch for this block is more than one barrier ahead,
// or it entered the same barrier for a collective with a different signature — a rank that
// skipped or reordered collectives), or another block of this rank already failed.
//
// Ordering: every storing wave drains its payload stores (vmcnt(0)), the block barrier, then the
// signalling wave issues a SYSTEM-scope release fence (L2 write-back; the explicit vmcnt(0) after
// it guards against the compiler dropping the fence's own wait) and stores the signal with a
// system-scope atomic; the polling wave reads the peers' slots with relaxed system-scope loads
// and, once every peer is there, issues a system-scope acquire fence + vmcnt(0) before the block
// barrier that releases the payload loads (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ bool ar_barrier(const ArDesc &d, int b, unsigned e, unsigned tag, int *s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's payload stores are done
  __syncthreads();
  if (threadIdx.x < 64) {
    const int p = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");       // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long sig = ((unsigned long long)tag << 32) | e;
    if (p < d.world) {
      unsigned long long *slot = reinterpret_cast<unsigned long long *>(d.stage[p]) + b * 32 + d.rank;
      __hip_atomic_store(slot, sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const unsigned long long *mine = reinterpret_cast<const unsigned long long *>(d.stage[d.rank]) + b * 32;
    const unsigned long long t0 = wall_clock64();
    unsigned fail = 0;
    for (;;) {
      int here = 1, bad = 0;
      if (p < d.world) {
        const unsigned long long v = __hip_atomic_load(mine + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const int dlt = (int)((unsigned)v - e);
        here = dlt >= 0;
        bad = dlt > 1 || (dlt == 0 && (unsigned)(v >> 32) != tag);
      }
      if (__any(bad)) {
        fail = kArErrDesync;
        break;
      }
      if (__all(here)) break;
      if (wall_clock64() - t0 > (unsigned long long)d.timeout_ticks) {
        fail = kArErrTimeout;
        break;
      }
      if (__hip_atomic_load(d.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {   // poisoned meanwhile
        fail = kArErrPoisoned;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!fail) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");     // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (p == 0) {
      if (fail) atomicOr(d.err, fail);
      *s_ok = fail ? 0 : 1;
    }
  }
  __syncthreads();
  return *s_ok != 0;
}

template <bool BF>
__global__ __launch_bounds__(kArThreads) void p2p_collective_kernel(const ArCall call) {
  __shared__ int s_ok;
  const int G = call.blocks;
  const int lr = blockIdx.x / G;
  const int b = blockIdx.x - lr * G;
  const ArDesc &d = call.desc[lr];
  float *buf = call.buf[lr];
  const int N = d.world, r = d.rank;
  const long long n = call.n;
  const int tid = threadIdx.x;
  const long long stride = (long long)G * kArThreads;
  // a communicator whose error word is set is poisoned: every later collective exits at once,
  // sends no signal and leaves the buffer untouched (peers then time out too), so no rank can
  // continue on desynchronised epochs; the host reports the word (Comm::check) and aborts
  if (tid == 0) s_ok = __hip_atomic_load(d.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
  __syncthreads();
  if (!s_ok) return;
  const unsigned tag = call.tag;
  unsigned e = __hip_atomic_load(d.ctr + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned calls = __hip_atomic_load(d.ctr + kArMaxBlocks + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long offA = kArSigBytes + (long long)(calls & 1) * d.region_bytes;
  const long long offR = kArSigBytes + 2 * d.region_bytes;
  const uint32_t stage_bytes = (uint32_t)ar_stage_bytes(d.region_bytes);
  const rsrc_t rb = make_rsrc(buf, (uint32_t)(n * 4));
  rsrc_t rs[kArMaxRanks];
#pragma unroll
  for (int p = 0; p < kArMaxRanks; ++p) rs[p] = make_rsrc(d.stage[p < N ? p : r], stage_bytes);
  bool ok = true;

  if (call.algo == AR_BROADCAST) {
    const long long nv = n / 4;   // 16-B units
    if (r == call.root)
      for (long long i = (long long)b * kArThreads + tid; i < nv; i += stride)
        st_sys(rs[r], (uint32_t)(offA + i * 16), bld16(rb, (uint32_t)(i * 16)));
    ok = ar_barrier(d, b, ++e, tag, &s_ok);
    if (ok && r != call.root)
      for (long long i = (long long)b * kArThreads + tid; i < nv; i += stride)
        bst16(rb, (uint32_t)(i * 16), ld_sys(rs[call.root], (uint32_t)(offA + i * 16)));
  } else {
    constexpr int VB = BF ? 16 : 32;   // staged bytes per 8-float vector
    const long long nv = n / 8;
    const bool two = call.algo == AR_TWOSHOT;
    const long long segv = two ? (nv + N - 1) / N : nv;
    const int nseg = two ? N : 1;
    // ---- copy-in: vector i = s * segv + j is staged by block (j / threads) % G of every rank
    for (long long j = (long long)b * kArThreads + tid; j < segv; j += stride) {
      for (int s = 0; s < nseg; ++s) {
        const long long i = s * segv + j;
        if (i >= nv) break;
        const uint4 lo = bld16(rb, (uint32_t)(i * 32)), hi = bld16(rb, (uint32_t)(i * 32 + 16));
        if constexpr (BF) {
          const float f[8] = {__uint_as_float(lo.x), __uint_as_float(lo.y), __uint_as_float(lo.z),
                              __uint_as_float(lo.w), __uint_as_float(hi.x), __uint_as_float(hi.y),
                              __uint_as_float(hi.z), __uint_as_float(hi.w)};
          st_sys(rs[r], (uint32_t)(offA + i * VB), pack8(f));
        } else {
          st_sys(rs[r], (uint32_t)(offA + i * VB), lo);
          st_sys(rs[r], (uint32_t)(offA + i * VB + 16), hi);
        }
      }
    }
    ok = ar_barrier(d, b, ++e, tag, &s_ok);
    // ---- reduce: one-shot the whole bucket, two-shot this rank's segment; rank order 0..N-1
    const long long rbase = two ? (long long)r * segv : 0;
    if (ok) {
      for (long long j = (long long)b * kArThreads + tid; j < segv; j += stride) {
        const long long i = rbase + j;
        if (i >= nv) break;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        uint4 v0[kArMaxRanks], v1[kArMaxRanks];
#pragma unroll
        for (int p = 0; p < kArMaxRanks; ++p) {   // all loads in flight; ranks >= N read 0 (OOB)
          const uint32_t off = p < N ? (uint32_t)(offA + i * VB) : kOOB;
          v0[p] = ld_sys(rs[p], off);
          if constexpr (!BF) v1[p] = ld_sys(rs[p], p < N ? off + 16 : kOOB);
        }
#pragma unroll
        for (int p = 0; p < kArMaxRanks; ++p) {
          if constexpr (BF) add8_bf(acc, v0[p]);
          else add8(acc, v0[p], v1[p]);
        }
        uint4 lo, hi;
        if constexpr (BF) {
          const uint4 q = pack8(acc);   // every rank keeps the same bf16-rounded sum
          if (two) st_sys(rs[r], (uint32_t)(offR + j * VB), q);
          float f[8];
          unpack8(q, f);
          lo = f4u(f[0], f[1], f[2], f[3]);
          hi = f4u(f[4], f[5], f[6], f[7]);
        } else {
          lo = f4u(acc[0], acc[1], acc[2], acc[3]);
          hi = f4u(acc[4], acc[5], acc[6], acc[7]);
          if (two) {
            st_sys(rs[r], (uint32_t)(offR + j * VB), lo);
            st_sys(rs[r], (uint32_t)(offR + j * VB + 16), hi);
          }
        }
        bst16(rb, (uint32_t)(i * 32), lo);
        bst16(rb, (uint32_t)(i * 32 + 16), hi);
      }
    }
    // ---- two-shot: gather the other ranks' reduced segments
    if (ok && two) {
      ok = ar_barrier(d, b, ++e, tag, &s_ok);
      if (ok) {
        for (long long j = (long long)b * kArThreads + tid; j < segv; j += stride) {
          for (int s = 0; s < N; ++s) {
            if (s == r) continue;
            const long long i = s * segv + j;
            if (i >= nv) continue;
            const uint4 q = ld_sys(rs[s], (uint32_t)(offR + j * VB));
            if constexpr (BF) {
              float f[8];
              unpack8(q, f);
              bst16(rb, (uint32_t)(i * 32), f4u(f[0], f[1], f[2], f[3]));
              bst16(rb, (uint32_t)(i * 32 + 16), f4u(f[4], f[5], f[6], f[7]));
            } else {
              bst16(rb, (uint32_t)(i * 32), q);
              bst16(rb, (uint32_t)(i * 32 + 16), ld_sys(rs[s], (uint32_t)(offR + j * VB + 16)));
            }
          }
        }
      }
    }
  }
  // advance this block's epoch / call counters (read by the next collective's block b)
  if (ok && tid == 0) {
    __hip_atomic_store(d.ctr + b, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.ctr + kArMaxBlocks + b, calls + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

void launch_p2p_collective(const ArCall &call, int nlocal, hipStream_t st) {
  const dim3 grid(nlocal * call.blocks);
  if (call.bf16_wire && call.algo != AR_BROADCAST)
    p2p_collective_kernel<true><<<grid, kArThreads, 0, st>>>(call);
  else
    p2p_collective_kernel<false><<<grid, kArThreads, 0, st>>>(call);
  PG_CHECK_LAUNCH();
}

// Fault injection for the communicator watchdog tests (comm_inject_stall): one lane spins on
// the realtime clock for `ticks` (100 MHz) on the comm stream, between a collective's start
// marker and the collective itself -- a peer that never arrives, as the watchdog sees it.
// Bounded by construction (the host caps it at 30 s).
__global__ void comm_stall_kernel(long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while ((long long)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(127);
}

void launch_comm_stall(double seconds, hipStream_t st) {
  const double s = seconds < 30.0 ? seconds : 30.0;
  hipLaunchKernelGGL(comm_stall_kernel, dim3(1), dim3(64), 0, st, (long long)(s * 1e8));
}
