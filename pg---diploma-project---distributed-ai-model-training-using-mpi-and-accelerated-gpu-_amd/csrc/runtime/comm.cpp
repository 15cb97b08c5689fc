// Native data-parallel communicator (comm.h).
#include "comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../p2p.h"
#include "plan.h"

void launch_p2p_collective(const ArCall &call, int nlocal, hipStream_t st);
void launch_comm_stall(double seconds, hipStream_t st);

namespace pgdist_rt {
namespace {

void hcheck(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------- RCCL (dlopen'd)
struct Rccl {
  void *h = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
  decltype(&ncclCommCount) commCount = nullptr;
};

template <class F>
void sym(void *h, F &f, const char *name) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
}

Rccl &rccl() {
  static Rccl *r = [] {
    auto *x = new Rccl();
    // the instance PyTorch loaded (libtorch_hip NEEDS "librccl.so"); else the ROCm one
    for (const char *name : {"librccl.so", "librccl.so.1"}) {
      x->h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (x->h) break;
    }
    if (!x->h) x->h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!x->h) return x;
    sym(x->h, x->getUniqueId, "ncclGetUniqueId");
    sym(x->h, x->commInitRank, "ncclCommInitRank");
    sym(x->h, x->commDestroy, "ncclCommDestroy");
    sym(x->h, x->commAbort, "ncclCommAbort");
    sym(x->h, x->getAsyncError, "ncclCommGetAsyncError");
    sym(x->h, x->allReduce, "ncclAllReduce");
    sym(x->h, x->broadcast, "ncclBroadcast");
    sym(x->h, x->errorString, "ncclGetErrorString");
    sym(x->h, x->getVersion, "ncclGetVersion");
    sym(x->h, x->commCount, "ncclCommCount");
    return x;
  }();
  return *r;
}

Rccl &rccl_or_throw() {
  Rccl &r = rccl();
  if (!r.h) throw std::runtime_error("RCCL (librccl.so) is not loadable in this process");
  return r;
}

void ncheck(ncclResult_t e, const char *what) {
  if (e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + rccl().errorString(e));
}

// Device-side join / marker events.  The communicator's events are recorded on the main and
// side streams before every bucket (the collective's wait) and around every tracked collective
// (the watchdog polls them from the host with hipEventQuery, which needs no fence): created
// like the plan's join events, without a system-scope fence.  A kernel's own
// device-scope release already makes its gradient writes visible to the comm stream's kernels
// and to RCCL / P2P peers (which read staging written by this device's comm kernels).
struct Event {
  hipEvent_t e = nullptr;
  Event() { hcheck(hipEventCreateWithFlags(&e, join_event_flags()), "hipEventCreateWithFlags"); }
  ~Event() {
    if (e) (void)hipEventDestroy(e);
  }
  Event(const Event &) = delete;
  Event &operator=(const Event &) = delete;
};

// ---------------------------------------------------------------- watchdog
// A collective that has STARTED on the comm stream (its start marker completed: every
// producer it waited for is done) but not finished within the deadline means a peer is dead
// or out of step.  The P2P kernels time out by themselves (error word); an RCCL kernel waits
// forever.  The watchdog thread polls the oldest outstanding collective's two events
// (hipEventQuery, no synchronisation) and, past the deadline, prints the stalled collective,
// poisons the communicator, calls ncclCommAbort and -- by default -- ends the process with a
// nonzero status, so a data-parallel job fails on every rank instead of hanging (the peers'
// own watchdogs fire the same way).
struct Tracked {
  std::shared_ptr<Event> start, done;
  std::string label;
  double seen = -1.0;   // host time the start marker was first seen complete
  double limit = 0.0;
};

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- communicator
struct Comm {
  int rank = 0, world = 1, device = 0, nlocal = 1, blocks = 32;
  hipStream_t stream = nullptr;
  ncclComm_t nccl = nullptr;
  long long region = 0;
  long long timeout_ticks = 0;
  std::vector<void *> own;        // staging allocations owned by this process (nlocal of them)
  std::vector<void *> opened;     // IPC-mapped peer staging
  unsigned char *stage[kArMaxRanks] = {};
  unsigned int *ctr = nullptr;    // nlocal * (kArCtrWords + 8) words: counters, error word
  bool p2p = false;
  // sticky host-side failure state: a synchronous RCCL error at launch (record or replay time),
  // or an error word / RCCL async error seen by comm_error.  Once set the communicator is
  // poisoned: every later collective (recorded ops included) throws instead of launching.
  std::atomic<int> host_err{0};
  mutable std::mutex what_mu;   // `what` is written by the op / replay / watchdog threads
  std::string what;

  // watchdog state (mu guards q / pool; the thread runs while wd_s > 0)
  std::mutex mu;
  std::deque<Tracked> q;
  std::vector<std::pair<std::shared_ptr<Event>, std::shared_ptr<Event>>> pool;
  double wd_s = 0.0;        // deadline after a collective started (0: watchdog off)
  int wd_exit = 0;          // process exit status on a stall (0: poison + abort only)
  std::thread wd;
  std::atomic<bool> wd_stop{false};
  std::atomic<long long> stall_ms{0};   // fault injection: stall the next collective this long
  // the RCCL handle is shared with the watchdog: on a stall the watchdog takes it (nccl_mu),
  // nulls it and hands it to the aborter thread, so no later comm_error / comm_rccl_ranks / comm_destroy
  // touches an aborted (freed) communicator; comm_destroy joins the aborter first
  std::mutex nccl_mu;
  std::thread aborter;
  std::atomic<bool> abort_done{false};
  ncclComm_t rccl_handle() {
    std::lock_guard<std::mutex> g(nccl_mu);
    return nccl;
  }

  void fail(int code, const std::string &msg) {
    std::lock_guard<std::mutex> g(what_mu);
    if (host_err.fetch_or(code) == 0) what = msg;
  }
  std::string what_str() const {
    std::lock_guard<std::mutex> g(what_mu);
    return what;
  }
  void ensure_usable() const {
    if (host_err.load())
      throw std::runtime_error("native communicator is poisoned after an earlier failure (" + what_str() + ")");
  }

  // called by a collective op on the comm stream (op / replay thread): start marker, the
  // injected stall if one is armed, then the collective, then end_track's done marker
  Tracked begin_track(hipStream_t st, const std::string &label, double limit_mult = 1.0) {
    Tracked t;
    const long long ms = stall_ms.exchange(0);
    if (wd_s <= 0.0 && ms == 0) return t;
    {
      std::lock_guard<std::mutex> g(mu);
      if (!pool.empty()) {
        t.start = pool.back().first;
        t.done = pool.back().second;
        pool.pop_back();
      }
    }
    if (!t.start) {
      t.start = std::make_shared<Event>();
      t.done = std::make_shared<Event>();
    }
    t.label = label;
    t.limit = wd_s * limit_mult;
    (void)hipEventRecord(t.start->e, st);
    if (ms > 0) launch_comm_stall(ms * 1e-3, st);
    return t;
  }
  void end_track(Tracked &&t, hipStream_t st) {
    if (!t.start) return;
    (void)hipEventRecord(t.done->e, st);
    if (wd_s <= 0.0) {
      std::lock_guard<std::mutex> g(mu);
      pool.emplace_back(t.start, t.done);
      return;
    }
    std::lock_guard<std::mutex> g(mu);
    q.push_back(std::move(t));
  }
  void watchdog_loop();
  void stop_watchdog() {
    wd_stop.store(true);
    if (wd.joinable()) wd.join();
  }

  unsigned int *ctr_of(int l) const { return ctr + (size_t)l * (kArCtrWords + 8); }
  unsigned int *err_of(int l) const { return ctr_of(l) + kArCtrWords; }

  ArCall make_call(const std::vector<uintptr_t> &bufs, long long n, int algo, bool bf16, int root) const {
    ArCall c;
    std::memset(&c, 0, sizeof(c));
    for (int l = 0; l < nlocal; ++l) {
      ArDesc &d = c.desc[l];
      for (int p = 0; p < world; ++p) d.stage[p] = stage[p];
      d.ctr = ctr_of(l);
      d.err = err_of(l);
      d.region_bytes = region;
      d.timeout_ticks = timeout_ticks;
      d.rank = nlocal > 1 ? l : rank;
      d.world = world;
      c.buf[l] = reinterpret_cast<float *>(bufs[l]);
    }
    c.n = n;
    c.blocks = blocks;
    c.algo = algo;
    c.bf16_wire = bf16 ? 1 : 0;
    c.root = root;
    // call signature: every rank entering one barrier must be in the same collective
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)algo;
    for (uint64_t v : {(uint64_t)n, (uint64_t)(bf16 ? 1 : 0), (uint64_t)(root + 1)}) {
      h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
      h *= 0xff51afd7ed558ccdull;
    }
    c.tag = (unsigned)(h ^ (h >> 32)) | 1u;
    return c;
  }
};

std::map<int, std::unique_ptr<Comm>> &comms() {
  static auto *m = new std::map<int, std::unique_ptr<Comm>>();
  return *m;
}
int g_next_comm = 1;

Comm &get(int id) {
  auto it = comms().find(id);
  if (it == comms().end()) throw std::out_of_range("unknown communicator " + std::to_string(id));
  return *it->second;
}

// an op that makes `st` wait for the work enqueued so far on every stream of `wait`
std::vector<std::shared_ptr<Event>> make_events(size_t k) {
  std::vector<std::shared_ptr<Event>> v;
  for (size_t i = 0; i < k; ++i) v.push_back(std::make_shared<Event>());
  return v;
}

void wait_all(hipStream_t st, const std::vector<uintptr_t> &wait, const std::vector<std::shared_ptr<Event>> &ev) {
  for (size_t i = 0; i < wait.size(); ++i) {
    hipStream_t w = reinterpret_cast<hipStream_t>(wait[i]);
    if (w == st) continue;
    (void)hipEventRecord(ev[i]->e, w);
    (void)hipStreamWaitEvent(st, ev[i]->e, 0);
  }
}

void check_p2p_call(const Comm &c, const std::vector<uintptr_t> &bufs, long long n, long long bytes_needed) {
  if (!c.p2p) throw std::runtime_error("communicator has no peer-to-peer path (staging not opened)");
  if ((int)bufs.size() != c.nlocal) throw std::invalid_argument("one buffer per local rank expected");
  for (uintptr_t b : bufs)
    if (!b || b % 16) throw std::invalid_argument("P2P buffers must be non-null and 16-byte aligned");
  if (n <= 0 || n * 4 >= (1ll << 31)) throw std::invalid_argument("P2P collective: 0 < n*4 < 2 GiB");
  if (bytes_needed > c.region)
    throw std::invalid_argument("P2P collective of " + std::to_string(bytes_needed) + " bytes exceeds the " +
                                std::to_string(c.region) + "-byte staging region");
}

// a synchronous RCCL failure (bad argument, communicator in error, ...) poisons the
// communicator and throws; plan_replay propagates the exception to the caller
void rccl_result(Comm *c, ncclResult_t r, const char *what) {
  if (r == ncclSuccess || r == ncclInProgress) return;
  const std::string msg = std::string(what) + ": " + rccl().errorString(r);
  c->fail(kCommErrRccl, msg);
  throw std::runtime_error(msg);
}

void Comm::watchdog_loop() {
  (void)hipSetDevice(device);
  while (!wd_stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    std::string stalled;
    double waited = 0.0;
    {
      std::lock_guard<std::mutex> g(mu);
      while (!q.empty()) {
        Tracked &f = q.front();
        if (hipEventQuery(f.done->e) == hipSuccess) {
          pool.emplace_back(f.start, f.done);
          q.pop_front();
          continue;
        }
        if (hipEventQuery(f.start->e) == hipSuccess) {
          const double t = now_s();
          if (f.seen < 0.0) f.seen = t;
          else if (t - f.seen > f.limit) {
            stalled = f.label;
            waited = t - f.seen;
          }
        }
        break;   // collectives complete in order on the comm stream
      }
      (void)hipGetLastError();
    }
    if (stalled.empty()) continue;
    char msg[512];
    std::snprintf(msg, sizeof(msg),
                  "[pgdist] comm watchdog: rank %d of %d: %s started %.1f s ago and has not completed "
                  "(limit %.1f s): a peer is dead or out of step; aborting the communicator",
                  rank, world, stalled.c_str(), waited, wd_s);
    std::fprintf(stderr, "%s\n", msg);
    std::fflush(stderr);
    fail(kCommErrStall, msg);
    // (the device error word is not written here: any HIP copy from this thread can queue
    // behind the stalled work -- streams share the hardware queues -- and delay the exit.  With
    // the default exit status the process ends before the stalled step's optimizer runs; in
    // poison-only mode the step in flight may apply what the aborted collective left, and the
    // next host poll / collective fails)
    // ncclCommAbort makes RCCL's own kernels give up, but it can block behind work queued on
    // the stream (measured: until an injected stall kernel ended): run it beside, and with an
    // exit status end the process after a bounded grace period whether or not it returned.
    // The handle leaves the communicator before the abort starts (nothing else uses it again).
    ncclComm_t nc = nullptr;
    {
      std::lock_guard<std::mutex> g(nccl_mu);
      nc = nccl;
      nccl = nullptr;
    }
    if (nc && rccl().commAbort) {
      aborter = std::thread([nc, this] {
        (void)rccl().commAbort(nc);
        abort_done.store(true);
      });
    } else {
      abort_done.store(true);
    }
    if (wd_exit) {
      for (int i = 0; i < 100 && !abort_done.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(20));
      std::fflush(stdout);
      std::fflush(stderr);
      std::_Exit(wd_exit);
    }
    return;   // poisoned: every later collective throws
  }
}

}  // namespace

bool rccl_available() { return rccl().h != nullptr; }

std::string rccl_version() {
  Rccl &r = rccl();
  if (!r.h) return "";
  int v = 0;
  if (r.getVersion(&v) != ncclSuccess) return "";
  return std::to_string(v);
}

std::string comm_unique_id() {
  Rccl &r = rccl_or_throw();
  ncclUniqueId id;
  ncheck(r.getUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

int comm_create(int rank, int world, int device, const std::string &uid, long long region_bytes, int blocks,
                int nlocal, double timeout_s) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("comm_create: bad rank/world");
  if (nlocal != 1 && nlocal != world) throw std::invalid_argument("comm_create: nlocal must be 1 or world");
  if (nlocal > 1 && !uid.empty()) throw std::invalid_argument("comm_create: the emulated group has no RCCL");
  if (region_bytes > 0 && world > kArMaxRanks)
    throw std::invalid_argument("comm_create: the P2P path supports up to 8 ranks");
  if (blocks < 1 || blocks > kArMaxBlocks) throw std::invalid_argument("comm_create: 1 <= blocks <= 64");
  if (region_bytes < 0 || region_bytes % 256 || ar_stage_bytes(region_bytes) >= (1ll << 31))
    throw std::invalid_argument("comm_create: region_bytes must be a multiple of 256 and the staging < 2 GiB");
  hcheck(hipSetDevice(device), "hipSetDevice");
  auto c = std::make_unique<Comm>();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->nlocal = nlocal;
  c->blocks = blocks;
  c->region = region_bytes;
  c->timeout_ticks = (long long)(timeout_s * 1e8);   // s_memrealtime: 100 MHz
  int lo = 0, hi = 0;
  hcheck(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  hcheck(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
  if (!uid.empty()) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("comm_create: unique id must be 128 bytes");
    Rccl &r = rccl_or_throw();
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), sizeof(id.internal));
    ncheck(r.commInitRank(&c->nccl, world, id, rank), "ncclCommInitRank");
  }
  {   // counters + error word (also without P2P: the optimizer skips its update while it is set)
    const size_t words = (size_t)nlocal * (kArCtrWords + 8);
    hcheck(hipMalloc(reinterpret_cast<void **>(&c->ctr), words * 4), "hipMalloc(counters)");
    hcheck(hipMemset(c->ctr, 0, words * 4), "hipMemset(counters)");
  }
  if (region_bytes > 0) {
    for (int l = 0; l < nlocal; ++l) {
      void *p = nullptr;
      hcheck(hipExtMallocWithFlags(&p, (size_t)ar_stage_bytes(region_bytes), hipDeviceMallocUncached),
             "hipExtMallocWithFlags(uncached staging)");
      hcheck(hipMemset(p, 0, (size_t)kArSigBytes), "hipMemset(signal slots)");
      c->own.push_back(p);
    }
    hcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (nlocal > 1) {   // emulation: every rank's staging is ours
      for (int p = 0; p < world; ++p) c->stage[p] = static_cast<unsigned char *>(c->own[p]);
      c->p2p = true;
    } else if (world == 1) {
      c->stage[0] = static_cast<unsigned char *>(c->own[0]);
      c->p2p = true;
    }
  }
  const int id = g_next_comm++;
  comms()[id] = std::move(c);
  return id;
}

std::string comm_p2p_handle(int id) {
  Comm &c = get(id);
  if (c.own.empty() || c.nlocal != 1) throw std::runtime_error("comm_p2p_handle: no single-rank staging");
  hipIpcMemHandle_t h;
  hcheck(hipIpcGetMemHandle(&h, c.own[0]), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char *>(&h), sizeof(h));
}

void comm_p2p_open(int id, const std::vector<std::string> &handles) {
  Comm &c = get(id);
  if (c.own.empty() || c.nlocal != 1) throw std::runtime_error("comm_p2p_open: no single-rank staging");
  if ((int)handles.size() != c.world) throw std::invalid_argument("comm_p2p_open: one handle per rank");
  hcheck(hipSetDevice(c.device), "hipSetDevice");
  for (int p = 0; p < c.world; ++p) {
    if (p == c.rank) {
      c.stage[p] = static_cast<unsigned char *>(c.own[0]);
      continue;
    }
    if (handles[p].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("comm_p2p_open: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[p].data(), sizeof(h));
    void *ptr = nullptr;
    hcheck(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    c.opened.push_back(ptr);
    c.stage[p] = static_cast<unsigned char *>(ptr);
  }
  c.p2p = true;
}

bool comm_p2p_ready(int id) { return get(id).p2p; }
uintptr_t comm_stream(int id) { return reinterpret_cast<uintptr_t>(get(id).stream); }
int comm_blocks(int id) { return get(id).blocks; }
void comm_set_timeout(int id, double seconds) {
  if (!(seconds > 0)) throw std::invalid_argument("comm_set_timeout: seconds > 0");
  get(id).timeout_ticks = (long long)(seconds * 1e8);
}
long long comm_region_bytes(int id) { return get(id).region; }

void comm_allreduce(int id, const std::vector<uintptr_t> &bufs, long long n, int algo, bool bf16_wire,
                    const std::vector<uintptr_t> &wait) {
  Comm &c = get(id);
  auto ev = make_events(wait.size());
  hipStream_t st = c.stream;
  if (algo == COMM_RCCL) {
    if (!c.rccl_handle()) throw std::runtime_error("communicator has no RCCL path");
    if (bufs.size() != 1 || !bufs[0]) throw std::invalid_argument("RCCL all-reduce: one buffer");
    if (bf16_wire) throw std::invalid_argument("RCCL all-reduce: fp32 only (bf16 wire is a P2P option)");
    void *b = reinterpret_cast<void *>(bufs[0]);
    ncclComm_t nc = c.rccl_handle();
    Rccl *r = &rccl();
    Comm *cp = &c;
    const std::string label = "RCCL all-reduce of " + std::to_string(n) + " floats";
    run_op([=] {
      cp->ensure_usable();
      wait_all(st, wait, ev);
      Tracked t = cp->begin_track(st, label);
      rccl_result(cp, r->allReduce(b, b, (size_t)n, ncclFloat32, ncclSum, nc, st), "ncclAllReduce");
      cp->end_track(std::move(t), st);
    });
    return;
  }
  if (algo != COMM_ONESHOT && algo != COMM_TWOSHOT) throw std::invalid_argument("comm_allreduce: unknown algo");
  if (n % 8) throw std::invalid_argument("P2P all-reduce: n must be a multiple of 8");
  check_p2p_call(c, bufs, n, n * (bf16_wire ? 2 : 4));
  const ArCall call = c.make_call(bufs, n, algo == COMM_ONESHOT ? AR_ONESHOT : AR_TWOSHOT, bf16_wire, 0);
  const int nl = c.nlocal;
  auto cp = std::make_shared<ArCall>(call);
  Comm *comm = &c;
  const std::string label = std::string(algo == COMM_ONESHOT ? "one-shot" : "two-shot") + " P2P all-reduce of " +
                            std::to_string(n) + " floats";
  run_op([=] {
    comm->ensure_usable();
    wait_all(st, wait, ev);
    // the P2P kernels time out by themselves (error word); the watchdog is the backstop
    Tracked t = comm->begin_track(st, label, 2.0);
    launch_p2p_collective(*cp, nl, st);
    comm->end_track(std::move(t), st);
  });
}

void comm_broadcast(int id, const std::vector<uintptr_t> &bufs, long long n, int root, int algo,
                    const std::vector<uintptr_t> &wait) {
  Comm &c = get(id);
  if (root < 0 || root >= c.world) throw std::invalid_argument("comm_broadcast: bad root");
  auto ev = make_events(wait.size());
  hipStream_t st = c.stream;
  if (algo == COMM_RCCL) {
    if (!c.rccl_handle()) throw std::runtime_error("communicator has no RCCL path");
    if (bufs.size() != 1 || !bufs[0]) throw std::invalid_argument("RCCL broadcast: one buffer");
    void *b = reinterpret_cast<void *>(bufs[0]);
    ncclComm_t nc = c.rccl_handle();
    Rccl *r = &rccl();
    Comm *cp = &c;
    const std::string label = "RCCL broadcast of " + std::to_string(n) + " floats";
    run_op([=] {
      cp->ensure_usable();
      wait_all(st, wait, ev);
      Tracked t = cp->begin_track(st, label);
      rccl_result(cp, r->broadcast(b, b, (size_t)n, ncclFloat32, root, nc, st), "ncclBroadcast");
      cp->end_track(std::move(t), st);
    });
    return;
  }
  if (n % 4) throw std::invalid_argument("P2P broadcast: n must be a multiple of 4");
  check_p2p_call(c, bufs, n, n * 4);
  auto cp = std::make_shared<ArCall>(c.make_call(bufs, n, AR_BROADCAST, false, root));
  const int nl = c.nlocal;
  Comm *comm = &c;
  const std::string label = "P2P broadcast of " + std::to_string(n) + " floats";
  run_op([=] {
    comm->ensure_usable();
    wait_all(st, wait, ev);
    Tracked t = comm->begin_track(st, label, 2.0);
    launch_p2p_collective(*cp, nl, st);
    comm->end_track(std::move(t), st);
  });
}

void comm_allreduce_f64(int id, uintptr_t buf, long long n, int op, const std::vector<uintptr_t> &wait) {
  Comm &c = get(id);
  if (!c.rccl_handle()) throw std::runtime_error("communicator has no RCCL path");
  if (op != 0 && op != 2) throw std::invalid_argument("comm_allreduce_f64: op 0 (sum) or 2 (max)");
  auto ev = make_events(wait.size());
  hipStream_t st = c.stream;
  ncclComm_t nc = c.rccl_handle();
  Rccl *r = &rccl();
  void *b = reinterpret_cast<void *>(buf);
  Comm *cp = &c;
  const std::string label = "RCCL fp64 all-reduce of " + std::to_string(n) + " doubles";
  run_op([=] {
    cp->ensure_usable();
    wait_all(st, wait, ev);
    Tracked t = cp->begin_track(st, label);
    rccl_result(cp, r->allReduce(b, b, (size_t)n, ncclFloat64, op == 0 ? ncclSum : ncclMax, nc, st),
                "ncclAllReduce(f64)");
    cp->end_track(std::move(t), st);
  });
}

void comm_join(int id, uintptr_t waiter) {
  Comm &c = get(id);
  hipStream_t st = c.stream, w = reinterpret_cast<hipStream_t>(waiter);
  if (w == st) return;
  auto ev = std::make_shared<Event>();
  run_op([=] {
    (void)hipEventRecord(ev->e, st);
    (void)hipStreamWaitEvent(w, ev->e, 0);
  });
}

double comm_time_allreduce(int id, const std::vector<uintptr_t> &bufs, long long n, int algo, bool bf16_wire,
                           int iters) {
  Comm &c = get(id);
  if (plan_recording()) throw std::runtime_error("comm_time_allreduce: not while recording a plan");
  hipEvent_t t0, t1;
  hcheck(hipEventCreate(&t0), "hipEventCreate");
  hcheck(hipEventCreate(&t1), "hipEventCreate");
  comm_allreduce(id, bufs, n, algo, bf16_wire, {});   // warm-up (and argument validation)
  hcheck(hipEventRecord(t0, c.stream), "hipEventRecord");
  for (int i = 0; i < iters; ++i) comm_allreduce(id, bufs, n, algo, bf16_wire, {});
  hcheck(hipEventRecord(t1, c.stream), "hipEventRecord");
  hcheck(hipEventSynchronize(t1), "hipEventSynchronize");
  float ms = 0.f;
  hcheck(hipEventElapsedTime(&ms, t0, t1), "hipEventElapsedTime");
  (void)hipEventDestroy(t0);
  (void)hipEventDestroy(t1);
  return ms * 1e3 / (iters > 0 ? iters : 1);
}

int comm_error(int id) {
  Comm &c = get(id);
  // (after a watchdog abort the comm stream may hold a collective that never completes)
  if (!(c.host_err.load() & kCommErrStall)) hcheck(hipStreamSynchronize(c.stream), "hipStreamSynchronize(comm)");
  int err = 0;
  if (c.ctr) {
    std::vector<unsigned int> w((size_t)c.nlocal * (kArCtrWords + 8));
    hcheck(hipMemcpy(w.data(), c.ctr, w.size() * 4, hipMemcpyDeviceToHost), "hipMemcpy(error words)");
    for (int l = 0; l < c.nlocal; ++l) err |= (int)(w[(size_t)l * (kArCtrWords + 8) + kArCtrWords] & 0xff);
    if (err)
      c.fail(err, std::string("P2P barrier failure:") + ((err & kArErrTimeout) ? " peer timeout" : "") +
                      ((err & kArErrDesync) ? " peer out of step" : "") +
                      ((err & kArErrPoisoned) ? " poisoned" : ""));
  }
  if (ncclComm_t nc = c.rccl_handle()) {   // (null once the watchdog aborted it)
    ncclResult_t ae = ncclSuccess;
    if (rccl().getAsyncError(nc, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      err |= ((int)ae & 0xff) << 8;
      c.fail(((int)ae & 0xff) << 8, std::string("RCCL async error: ") + rccl().errorString(ae));
    }
  }
  return err | (c.host_err.load() & (kCommErrRccl | kCommErrPeer | kCommErrStall));
}

void comm_poison(int id, const std::string &why) {
  Comm &c = get(id);
  c.fail(kCommErrPeer, why);
  const unsigned w = kArErrPoisoned;
  for (int l = 0; c.ctr && l < c.nlocal; ++l)
    hcheck(hipMemcpyAsync(c.err_of(l), &w, 4, hipMemcpyHostToDevice, c.stream), "hipMemcpyAsync(error word)");
  hcheck(hipStreamSynchronize(c.stream), "hipStreamSynchronize(comm)");
}

void comm_clear_error(int id) {
  Comm &c = get(id);
  hcheck(hipStreamSynchronize(c.stream), "hipStreamSynchronize(comm)");
  for (int l = 0; c.ctr && l < c.nlocal; ++l)
    hcheck(hipMemset(c.err_of(l), 0, 4), "hipMemset(error word)");
  hcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  c.host_err.store(0);
  std::lock_guard<std::mutex> g(c.what_mu);
  c.what.clear();
}

std::string comm_error_string(int id) {
  Comm &c = get(id);
  return c.host_err.load() ? c.what_str() : std::string();
}

namespace {
void stop_all_watchdogs() {   // before static destruction / HIP teardown at process exit
  for (auto &kv : comms()) kv.second->stop_watchdog();
}
}  // namespace

void comm_set_watchdog(int id, double seconds, int exit_status) {
  static const bool registered = (std::atexit(stop_all_watchdogs), true);
  (void)registered;
  Comm &c = get(id);
  if (seconds < 0) throw std::invalid_argument("comm_set_watchdog: seconds >= 0");
  c.stop_watchdog();
  c.wd_stop.store(false);
  c.wd_s = seconds;
  c.wd_exit = exit_status;
  if (seconds > 0) c.wd = std::thread([cp = &c] { cp->watchdog_loop(); });
}

double comm_watchdog(int id) { return get(id).wd_s; }

void comm_inject_stall(int id, double seconds) {
  if (!(seconds > 0) || seconds > 30) throw std::invalid_argument("comm_inject_stall: 0 < seconds <= 30");
  get(id).stall_ms.store((long long)(seconds * 1e3));
}

uintptr_t comm_error_word(int id) { return reinterpret_cast<uintptr_t>(get(id).err_of(0)); }

void comm_error_async(int id, uintptr_t host_dst) {
  Comm &c = get(id);
  hcheck(hipMemcpyAsync(reinterpret_cast<void *>(host_dst), c.err_of(0), 4, hipMemcpyDeviceToHost, c.stream),
         "hipMemcpyAsync(error word)");
}

int comm_rccl_ranks(int id) {
  Comm &c = get(id);
  ncclComm_t nc = c.rccl_handle();
  if (!nc) return 0;
  int n = 0;
  ncheck(rccl().commCount(nc, &n), "ncclCommCount");
  return n;
}

void comm_destroy(int id) {
  auto it = comms().find(id);
  if (it == comms().end()) return;
  Comm &c = *it->second;
  c.stop_watchdog();
  (void)hipSetDevice(c.device);
  const bool aborted = c.aborter.joinable();
  if (aborted) c.aborter.join();   // the watchdog's ncclCommAbort has returned
  // a stalled (aborted) comm stream is not waited for: its collective may never complete
  if (c.stream && !aborted) (void)hipStreamSynchronize(c.stream);
  if (ncclComm_t nc = c.rccl_handle()) (void)rccl().commDestroy(nc);
  for (void *p : c.opened) (void)hipIpcCloseMemHandle(p);
  for (void *p : c.own) (void)hipFree(p);
  if (c.ctr) (void)hipFree(c.ctr);
  if (c.stream && !aborted) (void)hipStreamDestroy(c.stream);   // (an aborted one is leaked)
  comms().erase(it);
}

}  // namespace pgdist_rt
