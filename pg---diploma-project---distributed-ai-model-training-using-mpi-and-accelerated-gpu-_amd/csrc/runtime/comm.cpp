// Native data-parallel communicator (comm.h).
#include "comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../p2p.h"
#include "plan.h"

void launch_p2p_collective(const ArCall &call, int nlocal, hipStream_t st);

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

struct Event {
  hipEvent_t e = nullptr;
  Event() { hcheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags"); }
  ~Event() {
    if (e) (void)hipEventDestroy(e);
  }
  Event(const Event &) = delete;
  Event &operator=(const Event &) = delete;
};

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
  std::string what;

  void fail(int code, const std::string &msg) {
    if (host_err.fetch_or(code) == 0) what = msg;
  }
  void ensure_usable() const {
    if (host_err.load())
      throw std::runtime_error("native communicator is poisoned after an earlier failure (" + what + ")");
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
  if (region_bytes > 0) {
    const size_t words = (size_t)nlocal * (kArCtrWords + 8);
    hcheck(hipMalloc(reinterpret_cast<void **>(&c->ctr), words * 4), "hipMalloc(counters)");
    hcheck(hipMemset(c->ctr, 0, words * 4), "hipMemset(counters)");
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
    if (!c.nccl) throw std::runtime_error("communicator has no RCCL path");
    if (bufs.size() != 1 || !bufs[0]) throw std::invalid_argument("RCCL all-reduce: one buffer");
    if (bf16_wire) throw std::invalid_argument("RCCL all-reduce: fp32 only (bf16 wire is a P2P option)");
    void *b = reinterpret_cast<void *>(bufs[0]);
    ncclComm_t nc = c.nccl;
    Rccl *r = &rccl();
    Comm *cp = &c;
    run_op([=] {
      cp->ensure_usable();
      wait_all(st, wait, ev);
      rccl_result(cp, r->allReduce(b, b, (size_t)n, ncclFloat32, ncclSum, nc, st), "ncclAllReduce");
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
  run_op([=] {
    comm->ensure_usable();
    wait_all(st, wait, ev);
    launch_p2p_collective(*cp, nl, st);
  });
}

void comm_broadcast(int id, const std::vector<uintptr_t> &bufs, long long n, int root, int algo,
                    const std::vector<uintptr_t> &wait) {
  Comm &c = get(id);
  if (root < 0 || root >= c.world) throw std::invalid_argument("comm_broadcast: bad root");
  auto ev = make_events(wait.size());
  hipStream_t st = c.stream;
  if (algo == COMM_RCCL) {
    if (!c.nccl) throw std::runtime_error("communicator has no RCCL path");
    if (bufs.size() != 1 || !bufs[0]) throw std::invalid_argument("RCCL broadcast: one buffer");
    void *b = reinterpret_cast<void *>(bufs[0]);
    ncclComm_t nc = c.nccl;
    Rccl *r = &rccl();
    Comm *cp = &c;
    run_op([=] {
      cp->ensure_usable();
      wait_all(st, wait, ev);
      rccl_result(cp, r->broadcast(b, b, (size_t)n, ncclFloat32, root, nc, st), "ncclBroadcast");
    });
    return;
  }
  if (n % 4) throw std::invalid_argument("P2P broadcast: n must be a multiple of 4");
  check_p2p_call(c, bufs, n, n * 4);
  auto cp = std::make_shared<ArCall>(c.make_call(bufs, n, AR_BROADCAST, false, root));
  const int nl = c.nlocal;
  Comm *comm = &c;
  run_op([=] {
    comm->ensure_usable();
    wait_all(st, wait, ev);
    launch_p2p_collective(*cp, nl, st);
  });
}

void comm_allreduce_f64(int id, uintptr_t buf, long long n, int op, const std::vector<uintptr_t> &wait) {
  Comm &c = get(id);
  if (!c.nccl) throw std::runtime_error("communicator has no RCCL path");
  if (op != 0 && op != 2) throw std::invalid_argument("comm_allreduce_f64: op 0 (sum) or 2 (max)");
  auto ev = make_events(wait.size());
  hipStream_t st = c.stream;
  ncclComm_t nc = c.nccl;
  Rccl *r = &rccl();
  void *b = reinterpret_cast<void *>(buf);
  Comm *cp = &c;
  run_op([=] {
    cp->ensure_usable();
    wait_all(st, wait, ev);
    rccl_result(cp, r->allReduce(b, b, (size_t)n, ncclFloat64, op == 0 ? ncclSum : ncclMax, nc, st),
                "ncclAllReduce(f64)");
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
  hcheck(hipStreamSynchronize(c.stream), "hipStreamSynchronize(comm)");
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
  if (c.nccl) {
    ncclResult_t ae = ncclSuccess;
    if (rccl().getAsyncError(c.nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      err |= ((int)ae & 0xff) << 8;
      c.fail(((int)ae & 0xff) << 8, std::string("RCCL async error: ") + rccl().errorString(ae));
    }
  }
  return err | (c.host_err.load() & kCommErrRccl);
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
  c.what.clear();
}

std::string comm_error_string(int id) {
  Comm &c = get(id);
  return c.host_err.load() ? c.what : std::string();
}

int comm_rccl_ranks(int id) {
  Comm &c = get(id);
  if (!c.nccl) return 0;
  int n = 0;
  ncheck(rccl().commCount(c.nccl, &n), "ncclCommCount");
  return n;
}

void comm_destroy(int id) {
  auto it = comms().find(id);
  if (it == comms().end()) return;
  Comm &c = *it->second;
  (void)hipSetDevice(c.device);
  if (c.stream) (void)hipStreamSynchronize(c.stream);
  if (c.nccl) (void)rccl().commDestroy(c.nccl);
  for (void *p : c.opened) (void)hipIpcCloseMemHandle(p);
  for (void *p : c.own) (void)hipFree(p);
  if (c.ctr) (void)hipFree(c.ctr);
  if (c.stream) (void)hipStreamDestroy(c.stream);
  comms().erase(it);
}

}  // namespace pgdist_rt
