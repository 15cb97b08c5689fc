// Peer-to-peer (xGMI) collective descriptors shared by the host communicator
// (runtime/comm.cpp) and the device kernels (kernels/allreduce.hip).
//
// Every rank owns ONE staging allocation (hipExtMallocWithFlags(..., hipDeviceMallocUncached):
// no L2 copy of it exists on any GPU, so a peer's load over xGMI always sees memory) that
// every other rank maps through hipIpcOpenMemHandle:
//
//   [0, kArSigBytes)                  signal slots: uint64 sig[block * 32 + src_rank] =
//                                     {call signature << 32 | epoch}
//   A0 = kArSigBytes                  copy-in region, even calls   (region_bytes)
//   A1 = A0 + region_bytes            copy-in region, odd calls    (region_bytes)
//   R  = A1 + region_bytes            two-shot reduced segment     (region_bytes)
//
// A signal slot is written ONLY by its source rank (system-scope atomic store of a
// monotonically increasing epoch tagged with the collective's signature) and polled only by the slot's owner, so no slot is ever
// reset.  A block's epoch / call counters live in the owner's ordinary device memory and are
// advanced by the kernel itself (never a host argument: a recorded launch replays with frozen
// arguments).  Every rank issues the same collectives in the same order with the same block
// count, so block b of every rank sees the same epoch sequence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kArMaxRanks = 8;
constexpr int kArMaxBlocks = 64;                    // blocks per rank of one collective
constexpr int kArThreads = 256;                     // 4 waves
constexpr long long kArSigBytes = 64 * 1024;        // kArMaxBlocks blocks x 32 source slots x 8 B, padded
static_assert(kArMaxBlocks * 32 * sizeof(uint64_t) <= kArSigBytes, "signal slots exceed their region");
static_assert(kArMaxRanks <= 32, "32 source slots per block");
constexpr int kArCtrWords = 2 * kArMaxBlocks;       // [epoch][calls] per block

enum ArAlgo : int {
  AR_ONESHOT = 1,    // copy-in, 1 barrier, every rank sums all ranks' buffers
  AR_TWOSHOT = 2,    // copy-in, barrier, reduce own 1/N segment, barrier, gather the others
  AR_BROADCAST = 3,  // root copy-in, barrier, the others copy root's buffer
};

struct ArDesc {
  unsigned char *stage[kArMaxRanks];   // every rank's staging base, mapped in this process
  unsigned int *ctr;                   // this rank's counters [kArCtrWords]
  unsigned int *err;                   // this rank's error word (bit 0: barrier timeout)
  long long region_bytes;              // bytes of each of A0 / A1 / R
  long long timeout_ticks;             // barrier give-up, in 100 MHz realtime ticks
  int rank, world;
  int pad[2];
};

// one collective over `n` fp32 elements at grad[local rank] (n % 8 == 0 for all-reduce,
// n % 4 == 0 for broadcast); up to kArMaxRanks local ranks (single-process emulation)
struct ArCall {
  ArDesc desc[kArMaxRanks];
  float *buf[kArMaxRanks];
  long long n;
  int blocks;      // G: blocks per rank; grid = nlocal * G
  int algo;
  int bf16_wire;   // all-reduce: stage bf16 (sum in fp32)
  int root;        // broadcast
  unsigned tag;    // call signature (algo, n, wire, root): peers in one barrier must agree
  int pad;
};

// bits of the error word
constexpr unsigned kArErrTimeout = 1u;   // a peer did not arrive within the timeout
constexpr unsigned kArErrDesync = 2u;    // a peer is out of step (epoch or call signature)
constexpr unsigned kArErrPoisoned = 4u;  // another block of this rank had already failed

__host__ __device__ inline long long ar_stage_bytes(long long region_bytes) { return kArSigBytes + 3 * region_bytes; }
