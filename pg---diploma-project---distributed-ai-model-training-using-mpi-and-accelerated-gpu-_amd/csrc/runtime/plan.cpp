// Launch plans (plan.h).
#include "plan.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

int bn_rep();               // kernels/bn.hip: BN-statistics replica rows the producers use
void bn_disarm();
void wgrad_reduce_reset();  // kernels/reduce.hip

namespace pgdist_rt {
namespace {

struct Plan {
  std::vector<PlanOp> ops;
  int bn_rep = 0;   // the replica rows the recorded launches' BN accumulators were sized for
};

// heap-allocated and never destroyed: a plan may hold Python callbacks, which must not be
// released after the interpreter has finalised
std::map<int, Plan> &plans() {
  static auto *m = new std::map<int, Plan>();
  return *m;
}
Plan *g_rec = nullptr;
int g_next_id = 1;

void check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// flags of the cross-stream join events (PGDIST_EVENT_FLAGS overrides).  Both streams are on
// this device and every kernel ends with its own device-scope release, so a join needs no
// system-scope fence of its own: without it the record costs the main stream less
// (4.320 vs 4.342 ms/step, docs/PERF_NOTES.md).  Host-visible waits use other events.
unsigned event_flags() {
  static const unsigned f = [] {
    const char *s = std::getenv("PGDIST_EVENT_FLAGS");
    return s ? static_cast<unsigned>(std::strtoul(s, nullptr, 0))
             : static_cast<unsigned>(hipEventDisableTiming | hipEventDisableSystemFence);
  }();
  return f;
}

struct Event {
  hipEvent_t e = nullptr;
  Event() { check(hipEventCreateWithFlags(&e, event_flags()), "hipEventCreateWithFlags"); }
  ~Event() {
    if (e) (void)hipEventDestroy(e);
  }
  Event(const Event &) = delete;
  Event &operator=(const Event &) = delete;
};

// eager (unrecorded) waits: a ring of events; reusing one is safe because its record and the
// wait on it are both enqueued before the next reuse (the wait binds the record at call time)
hipEvent_t ring_event() {
  static auto *ring = new std::vector<std::unique_ptr<Event>>();
  static std::size_t next = 0;
  if (ring->size() < 64) {
    ring->push_back(std::make_unique<Event>());
    return ring->back()->e;
  }
  hipEvent_t e = (*ring)[next]->e;
  next = (next + 1) % ring->size();
  return e;
}

}  // namespace

void plan_record_begin() {
  if (g_rec) throw std::runtime_error("plan_record_begin: a recording is already open");
  g_rec = new Plan();
  g_rec->bn_rep = bn_rep();
}

int plan_record_end() {
  if (!g_rec) throw std::runtime_error("plan_record_end: no open recording");
  const int id = g_next_id++;
  plans()[id] = std::move(*g_rec);
  delete g_rec;
  g_rec = nullptr;
  return id;
}

void plan_record_abort() {
  delete g_rec;
  g_rec = nullptr;
}

bool plan_recording() { return g_rec != nullptr; }

void plan_append(PlanOp op) {
  if (g_rec) g_rec->ops.push_back(std::move(op));
}

void plan_replay(int id) {
  auto it = plans().find(id);
  if (it == plans().end()) throw std::out_of_range("plan_replay: unknown plan " + std::to_string(id));
  if (g_rec) throw std::runtime_error("plan_replay: not allowed while recording");
  // the recorded producers read the host's replica-row count at launch: replaying after a BN
  // mode switch would write rows past the accumulators sized at record time
  if (it->second.bn_rep != bn_rep())
    throw std::runtime_error("plan_replay: the BN statistics mode changed since this plan was recorded "
                             "(set_deterministic before building the step); re-record it");
  (void)hipGetLastError();
  try {
    for (auto &op : it->second.ops) op();
  } catch (...) {
    // a failed op (e.g. a Python callback raising) must not leave host launch state behind:
    // deferred weight-gradient reductions or an armed BN descriptor would leak into later launches
    wgrad_reduce_reset();
    bn_disarm();
    throw;
  }
  const hipError_t e = hipGetLastError();
  // no device at all: a host-only plan (Python callbacks) on a machine without a GPU
  if (e != hipSuccess && e != hipErrorNoDevice) throw std::runtime_error(std::string("plan_replay: launch failed: ") + hipGetErrorString(e));
}

void plan_free(int id) { plans().erase(id); }

std::size_t plan_recording_size() { return g_rec ? g_rec->ops.size() : 0; }

std::vector<double> plan_time_ops(int id, const std::vector<std::pair<int, int>> &ranges, int iters) {
  auto it = plans().find(id);
  if (it == plans().end()) throw std::out_of_range("plan_time_ops: unknown plan " + std::to_string(id));
  if (g_rec) throw std::runtime_error("plan_time_ops: not allowed while recording");
  auto &ops = it->second.ops;
  std::vector<double> out;
  for (const auto &r : ranges) {
    if (r.first < 0 || r.second > (int)ops.size() || r.first > r.second)
      throw std::out_of_range("plan_time_ops: bad op range");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
      for (int k = r.first; k < r.second; ++k) ops[k]();
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const auto t1 = std::chrono::steady_clock::now();
    out.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / (iters > 0 ? iters : 1));
  }
  return out;
}

std::size_t plan_size(int id) {
  auto it = plans().find(id);
  return it == plans().end() ? 0 : it->second.ops.size();
}

unsigned join_event_flags() { return event_flags(); }

void stream_wait(hipStream_t waiter, hipStream_t signaler) {
  if (waiter == signaler) return;
  if (!plan_recording()) {
    hipEvent_t e = ring_event();
    check(hipEventRecord(e, signaler), "hipEventRecord");
    check(hipStreamWaitEvent(waiter, e, 0), "hipStreamWaitEvent");
    return;
  }
  auto ev = std::make_shared<Event>();
  run_op([ev, waiter, signaler] {
    (void)hipEventRecord(ev->e, signaler);
    (void)hipStreamWaitEvent(waiter, ev->e, 0);
  });
}

void memset_async(void *ptr, int value, std::size_t bytes, hipStream_t st) {
  run_op([=] { (void)hipMemsetAsync(ptr, value, bytes, st); });
}

}  // namespace pgdist_rt
