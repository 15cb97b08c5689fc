// Launch plans: the host side of one training step, recorded once and replayed from C++.
//
// The eager step is ~330 kernel launches on two HIP streams plus the cross-stream event
// waits between them; issued from Python through the validated wrappers (ops/kernels.py)
// that costs ~13 us of host time per launch, enough for the host to fall behind the GPU in
// the backward of the small late layers.  A hipGraph removes the host cost but on ROCm its
// replay serialises the side-stream branches (measured slower than eager, bench.py --graph).
// A plan keeps the eager multi-stream structure: while a step runs eagerly under
// plan_record_begin/end, every native launch, stream wait, memset and Python callback that
// goes through run_op is also appended to the plan; plan_replay re-issues the same
// sequence on the same streams with no Python in between (Python callbacks — e.g. the DDP
// bucket hand-off — are the only exception, and run with the GIL the caller holds).
//
// Valid while every recorded argument stays valid: the MobileNetV2 step is written to be
// capture-safe (fixed device buffers, per-step scalars live in device memory), the same
// contract a hipGraph capture needs.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <functional>
#include <utility>
#include <vector>

namespace pgdist_rt {

using PlanOp = std::function<void()>;

void plan_record_begin();        // throws if a recording is already open
int plan_record_end();           // closes the recording, returns the plan id
void plan_record_abort();        // drops an open recording
bool plan_recording();
void plan_append(PlanOp op);     // no-op unless recording
void plan_replay(int id);
void plan_free(int id);
std::size_t plan_size(int id);
std::size_t plan_recording_size();   // ops recorded so far in the open recording (0: none)
// diagnostics: for each [first, last) op range, run it `iters` times in isolation (device
// synchronised before and after) and return the mean wall time per repetition in us
std::vector<double> plan_time_ops(int id, const std::vector<std::pair<int, int>> &ranges, int iters);

// run now; also record when a plan is being recorded
template <class F>
void run_op(F &&f) {
  f();
  if (plan_recording()) plan_append(PlanOp(std::forward<F>(f)));
}

// `waiter` waits for the work enqueued so far on `signaler` (event record + stream wait);
// a recorded wait owns its event, eager waits reuse a small event ring
void stream_wait(hipStream_t waiter, hipStream_t signaler);
// flags of device-side join events (no timing, no system-scope fence unless PGDIST_EVENT_FLAGS
// says otherwise): the events of stream_wait, and the communicator's bucket joins / watchdog markers
unsigned join_event_flags();
// hipMemsetAsync(ptr, value, bytes, stream) as a plan op
void memset_async(void *ptr, int value, std::size_t bytes, hipStream_t st);

}  // namespace pgdist_rt
