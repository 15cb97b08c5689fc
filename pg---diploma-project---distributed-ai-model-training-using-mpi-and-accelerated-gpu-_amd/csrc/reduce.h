// Deterministic single-launch two-level column reductions.
//
// Producers (conv epilogues) leave per-workgroup partial rows [R][ncols] (BN
// statistics, split-M weight-gradient slabs).  A reduction launch with grid
// (column blocks, nch row chunks) sums each chunk (level 1), and the LAST
// workgroup of every column block to arrive sums the nch level-1 rows in a
// fixed order and runs the consumer's epilogue (BN finalize, gradient store) —
// one launch instead of a fold kernel plus a finalize kernel, and independent of
// which workgroup happens to arrive last (bitwise deterministic).
//
// Cross-workgroup hand-off (gfx950, MI355X_MICROARCH.md "inter-workgroup
// visibility", first row of the measured hand-off table): level-1 values are
// written with agent-scope (sc1) stores, every storing wave waits vmcnt(0),
// a workgroup barrier, then ONE lane adds to the column block's counter
// (agent-scope atomic); the workgroup whose add returned nch-1 reads the
// level-1 rows with agent-scope (sc1) loads after a barrier, and resets the
// counter for the next launch on the stream.
#pragma once
#include "common.h"

// zero-initialised arrival counters (>= n entries) private to (current device, stream); host side
int *reduce_counters(int n, hipStream_t st);

PG_DEVICE void st_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
PG_DEVICE void st_sc1(float *p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned int *>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
PG_DEVICE double ld_sc1(const double *p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
PG_DEVICE float ld_sc1(const float *p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned int *>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// arrive_last with an explicit counter (the caller picked its column block's entry)
PG_DEVICE bool arrive_last_at(int *c, int nch, int *lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nch - 1;
    if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// Call with every thread of the workgroup after the level-1 values were stored with
// st_sc1 (by any subset of threads).  Returns true (uniformly) in the last-arriving
// workgroup of column block blockIdx.x; that workgroup also re-arms the counter.
PG_DEVICE bool arrive_last(int *ctr, int nch, int *lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ctr + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nch - 1;
    if (last) __hip_atomic_store(ctr + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// row-chunk geometry shared by the host launchers and the workspace queries
inline int red_rch(int R, int min_rows) {
  int r = (R + 31) / 32;
  return r < min_rows ? min_rows : r;
}
inline int red_nch(int R, int min_rows) {
  const int r = red_rch(R, min_rows);
  return (R + r - 1) / r;
}
