// Native data-parallel communicator: RCCL + peer-to-peer xGMI collectives on a dedicated
// HIP stream, with every launch recordable into a launch plan (plan.h).
//
// Reference: the gradient all-reduce of DistributedDataParallel over NCCL and the fp64
// metric all-reduce (cifar10_mpi_mobilenet_224.py:34-35,142-145,187-196; SURVEY.md §2.4,
// §2.7, §5.8).  pgdist drives RCCL directly instead of through c10d's Python work objects:
//
//  * the RCCL library is the one PyTorch already loaded (dlopen RTLD_NOLOAD "librccl.so"),
//    so one RCCL instance serves both c10d and this communicator;
//  * the unique id travels through the c10d TCPStore (Python side: parallel/comm.py);
//  * collectives run on the communicator's own high-priority stream; each launch first makes
//    that stream wait (events) for the streams that produced its input, and `join` makes a
//    consumer stream wait for the collectives issued so far — all as plan ops, so a replayed
//    training step contains no Python;
//  * the P2P path (kernels/allreduce.hip) maps every peer's uncached staging buffer through
//    hipIpc handles and runs one-shot / two-shot all-reduces and a broadcast over xGMI;
//  * `nlocal > 1` builds a single-process emulation of `world` ranks on one GPU (own staging,
//    counters and buffers per rank; one launch drives all of them) for tests and
//    microbenchmarks of the P2P kernels.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

namespace pgdist_rt {

enum CommAlgo : int { COMM_RCCL = 0, COMM_ONESHOT = 1, COMM_TWOSHOT = 2 };

bool rccl_available();
std::string rccl_version();
std::string comm_unique_id();   // ncclGetUniqueId, 128 bytes

// rank/world: this process's rank (nlocal == 1) or the emulated group (nlocal == world, rank 0);
// uid: RCCL unique id ("" = no RCCL communicator); region_bytes: P2P staging region (0 = no P2P)
int comm_create(int rank, int world, int device, const std::string &uid, long long region_bytes, int blocks,
                int nlocal, double timeout_s);
std::string comm_p2p_handle(int id);                               // IPC handle of this rank's staging
void comm_p2p_open(int id, const std::vector<std::string> &handles);  // every rank's handle, in rank order
bool comm_p2p_ready(int id);
uintptr_t comm_stream(int id);
int comm_blocks(int id);
void comm_set_timeout(int id, double seconds);   // P2P barrier give-up for collectives issued afterwards
long long comm_region_bytes(int id);

// in-place sum over ranks of n fp32 elements at bufs[local rank]; the comm stream first waits
// for every stream in `wait` (recordable)
void comm_allreduce(int id, const std::vector<uintptr_t> &bufs, long long n, int algo, bool bf16_wire,
                    const std::vector<uintptr_t> &wait);
// broadcast n fp32 elements from `root` (RCCL or P2P), after `wait`
void comm_broadcast(int id, const std::vector<uintptr_t> &bufs, long long n, int root, int algo,
                    const std::vector<uintptr_t> &wait);
// RCCL all-reduce of n doubles (op 0 sum, 2 max), after `wait`
void comm_allreduce_f64(int id, uintptr_t buf, long long n, int op, const std::vector<uintptr_t> &wait);
// `waiter` waits for every collective issued so far (recordable)
void comm_join(int id, uintptr_t waiter);
// microbenchmark: `iters` back-to-back all-reduces on the comm stream, us per call (host-synchronous)
double comm_time_allreduce(int id, const std::vector<uintptr_t> &bufs, long long n, int algo, bool bf16_wire,
                           int iters);
// error state (sticky: a nonzero result poisons the communicator, later collectives throw):
// P2P error-word bits (p2p.h kArErr*) | RCCL async error << 8 | kCommErrRccl for a synchronous
// RCCL failure at launch; synchronises the comm stream
constexpr int kCommErrRccl = 1 << 16;
constexpr int kCommErrPeer = 1 << 17;   // poisoned because ANOTHER rank failed (comm_poison)
constexpr int kCommErrStall = 1 << 18;  // the watchdog saw a started collective miss its deadline
int comm_error(int id);
// poison this rank's communicator because a peer failed (host flag + device error word)
void comm_poison(int id, const std::string &why);
// un-poison after a failure every rank has agreed on and reacted to (the P2P path is then
// abandoned: its epochs may be out of step) — used only by the start-up P2P validation
void comm_clear_error(int id);
std::string comm_error_string(int id);   // what poisoned the communicator ("" if healthy)
int comm_rccl_ranks(int id);             // ncclCommCount of the RCCL communicator (0: none)
// watchdog: a collective that started on the comm stream but has not completed `seconds` later
// (P2P: twice that; their kernels time out by themselves) poisons the communicator, aborts the
// RCCL communicator and, with exit_status != 0, ends the process with that status (0 s: off)
void comm_set_watchdog(int id, double seconds, int exit_status);
double comm_watchdog(int id);
// fault injection (tests): the next collective's kernel is preceded on the comm stream, after its
// start marker, by a kernel that spins `seconds` (<= 30)
void comm_inject_stall(int id, double seconds);
// device address of this rank's error word (nonzero once a P2P collective failed or the
// communicator was poisoned): the fused Adam skips its update while it is set
uintptr_t comm_error_word(int id);
// copy the error word to pinned host memory on the comm stream, after the collectives issued so
// far (no synchronisation: the caller reads it one step later)
void comm_error_async(int id, uintptr_t host_dst);
void comm_destroy(int id);

}  // namespace pgdist_rt
