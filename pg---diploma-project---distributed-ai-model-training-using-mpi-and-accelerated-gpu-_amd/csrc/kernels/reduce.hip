// Single-launch deterministic column reductions (see reduce.h): the weight-gradient
// split-M reduction  out[n] = sum_r part[r][n]  used by every wgrad kernel, and the
// per-device arrival counters of the last-workgroup hand-off.
#include "../reduce.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace {
// Arrival counters per device in two lanes: lane 1 for streams registered as side
// streams (the executor's weight-gradient stream), lane 0 for every other stream, so
// reductions running concurrently on the two streams never share a counter.  Keyed by
// lane rather than by stream handle because hipGraph capture swaps the main stream.
constexpr int kMaxDev = 64, kLaneCtrs = 65536;
int *g_ctr[kMaxDev] = {};
std::vector<hipStream_t> g_side;
std::mutex g_mu;
}  // namespace

void register_side_stream(hipStream_t st) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_side.push_back(st);
}

int *reduce_counters(int n, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  if (n > kLaneCtrs) return nullptr;   // callers size their grids far below this
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_ctr[dev]) {
    // first use happens in an eager step (before any hipGraph capture)
    hipMalloc(&g_ctr[dev], (size_t)2 * kLaneCtrs * sizeof(int));
    hipMemset(g_ctr[dev], 0, (size_t)2 * kLaneCtrs * sizeof(int));
    hipDeviceSynchronize();
  }
  bool side = false;
  for (auto s : g_side) side |= s == st;
  return g_ctr[dev] + (side ? kLaneCtrs : 0);
}

// Geometry: a workgroup covers 16 column groups of V floats x 16 row stripes (each row
// read as 16 x 16-B pieces = 256 contiguous bytes); the rows are split into nch chunks so
// the grid has ~2k workgroups, and the last-arriving workgroup of a column block sums the
// nch level-1 rows (<= kWredMaxChunks) the same way.
constexpr int kWredMaxChunks = 128;
constexpr int kWredTargetWgs = 512;
// main-stream grid target kWredTargetWgs: 512 vs the former 2048, same box
// (scripts/gpu_r4_wred3.sh): MobileNetV2 4.498-4.509 vs 4.510-4.522 ms/step, ResNet-50
// 11.688 / 11.708 vs 11.712 / 11.733 (small: these reductions are short, but a 2k-workgroup
// grid delays the side stream's dispatches behind it)
static int wred_main_wgs() { return kWredTargetWgs; }
constexpr int kWredSideWgs = 384;

bool is_side_stream(hipStream_t st) {
  std::lock_guard<std::mutex> lock(g_mu);
  for (auto s : g_side)
    if (s == st) return true;
  return false;
}

// level-1 rows the wgrad reduction of R partial rows may need after the partials
int colsum_rows(int R) {
  const int c = (R + 15) / 16;
  return c < 1 ? 1 : (c > kWredMaxChunks ? kWredMaxChunks : c);
}

// Output index of reduced column oc.  stem36: the stem weight gradient, reduced as
// [O][tap*4 + c] (3 channels padded to 4) and stored as torch [O][c][kh][kw]; -1: padding.
PG_DEVICE long long red_out_index(long long oc, bool stem36) {
  if (!stem36) return oc;
  const int o = (int)(oc / 36), r = (int)(oc % 36), tap = r >> 2, c = r & 3;
  return c == 3 ? -1 : (long long)o * 27 + c * 9 + tap;
}

// One workgroup's share of a column reduction: column block bx, row chunk by (ctr: the
// arrival counter of column block bx).
template <int V>
PG_DEVICE void col_reduce_body(const float *__restrict__ part, int R, long long n, int rch, int nch,
                               float *__restrict__ lvl1, int *__restrict__ ctr, float *__restrict__ out, int bx,
                               int by, bool stem36 = false) {
  __shared__ float sh[16][16 * V + 1];
  __shared__ int flag;
  const int cg = threadIdx.x & 15, stripe = threadIdx.x >> 4;
  const long long c0 = ((long long)bx * 16 + cg) * V;
  const bool cok = c0 < n;
  float acc[V], acc2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = acc2[j] = 0.f;
  auto ld = [&](const float *p, float (&v)[V]) {
    if constexpr (V == 4) {
      const float4 q = *reinterpret_cast<const float4 *>(p);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      v[0] = *p;
    }
  };
  const int r0 = by * rch, r1 = min(R, r0 + rch);
  if (cok) {
    int r = r0 + stripe;
    // (four rows in flight per thread measured slower: ResNet-50 11.81-11.83 -> 11.93-12.00
    // ms/step, the side-stream reduction then takes HBM bandwidth from the main stream's
    // convolutions; profiles/r3c_reduce_ab.txt)
    for (; r + 16 < r1; r += 32) {   // two rows in flight per thread, fixed order
      float a[V], b[V];
      ld(part + (size_t)r * n + c0, a);
      ld(part + (size_t)(r + 16) * n + c0, b);
#pragma unroll
      for (int j = 0; j < V; ++j) { acc[j] += a[j]; acc2[j] += b[j]; }
    }
    if (r < r1) {
      float a[V];
      ld(part + (size_t)r * n + c0, a);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += a[j];
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) sh[stripe][cg * V + j] = acc[j] + acc2[j];
  __syncthreads();
  const int col = threadIdx.x;   // < 16 * V: one output column per thread
  const long long oc = (long long)bx * 16 * V + col;
  float s1 = 0.f;
  if (col < 16 * V) {
#pragma unroll
    for (int k = 0; k < 16; ++k) s1 += sh[k][col];
  }
  const long long od = red_out_index(oc, stem36);
  if (nch == 1) {
    if (col < 16 * V && oc < n && od >= 0) out[od] = s1;
    return;
  }
  if (col < 16 * V && oc < n) st_sc1(lvl1 + (size_t)by * n + oc, s1);
  if (!arrive_last_at(ctr, nch, &flag)) return;
  float b[V];
#pragma unroll
  for (int j = 0; j < V; ++j) b[j] = 0.f;
  if (cok) {
    for (int k = stripe; k < nch; k += 16) {
#pragma unroll
      for (int j = 0; j < V; ++j) b[j] += ld_sc1(lvl1 + (size_t)k * n + c0 + j);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < V; ++j) sh[stripe][cg * V + j] = b[j];
  __syncthreads();
  if (col < 16 * V && oc < n && od >= 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += sh[k][col];
    out[od] = s;
  }
}

template <int V>
__global__ __launch_bounds__(256) void col_reduce_kernel(const float *__restrict__ part, int R, long long n, int rch,
                                                         int nch, float *__restrict__ lvl1, int *__restrict__ ctr,
                                                         float *__restrict__ out, int stem36) {
  col_reduce_body<V>(part, R, n, rch, nch, lvl1, ctr ? ctr + blockIdx.x : nullptr, out, blockIdx.x, blockIdx.y,
                     stem36 != 0);
}

// Several independent reductions in ONE launch (the weight gradients of a group of layers
// flushed together to the side stream): workgroups [wg0, wg0 + nb * nch) belong to segment k.
namespace {
constexpr int kRedMaxSeg = 8;
struct RedSeg {
  const float *part;
  float *grad;
  long long n;
  int S, rch, nch, nb, wg0, ctr0;
};
struct RedSegs {
  RedSeg s[kRedMaxSeg];
  int nseg;
  int *ctr;
};
}  // namespace

template <int V>
__global__ __launch_bounds__(256) void col_reduce_multi_kernel(RedSegs a) {
  const int id = blockIdx.x;
  int k = 0;
  while (k + 1 < a.nseg && id >= a.s[k + 1].wg0) ++k;
  const RedSeg &g = a.s[k];
  const int local = id - g.wg0, bx = local % g.nb, by = local / g.nb;
  col_reduce_body<V>(g.part, g.S, g.n, g.rch, g.nch, const_cast<float *>(g.part) + (size_t)g.S * g.n,
                     g.nch > 1 ? a.ctr + g.ctr0 + bx : nullptr, g.grad, bx, by);
}

// Deferred mode (wgrad_reduce_defer): launch_wgrad_reduce records the reduction instead of
// launching it; wgrad_reduce_flush launches every recorded one in col_reduce_multi launches.
namespace {
struct PendingRed {
  float *part;
  int S;
  long long n;
  float *grad;
};
bool g_red_defer = false;
std::vector<PendingRed> g_red_pending;
}  // namespace

void wgrad_reduce_defer(bool on) { g_red_defer = on; }
bool wgrad_reduce_deferring() { return g_red_defer; }
// error recovery (plan.cpp): stop deferring and drop reductions recorded but not launched
void wgrad_reduce_reset() {
  g_red_defer = false;
  g_red_pending.clear();
}

static void red_geom(int S, long long n, int target, int V, int &nb, int &rch, int &nch) {
  const long long nbl = (n + 16 * V - 1) / (16 * V);
  long long want = target / (nbl > 0 ? nbl : 1);
  nch = (int)(want < 1 ? 1 : want);
  const int cap = colsum_rows(S);
  if (nch > cap) nch = cap;
  rch = (S + nch - 1) / nch;
  nch = (S + rch - 1) / rch;
  nb = (int)nbl;
}

void wgrad_reduce_flush(hipStream_t st) {
  std::vector<PendingRed> segs;
  segs.swap(g_red_pending);
  bool vec = true;
  for (const auto &r : segs)
    vec &= (r.n % 4 == 0) && ((uintptr_t)r.part % 16 == 0) && ((uintptr_t)r.grad % 16 == 0);
  const int V = vec ? 4 : 1;
  for (size_t b = 0; b < segs.size(); b += kRedMaxSeg) {
    RedSegs a{};
    a.nseg = (int)std::min<size_t>(kRedMaxSeg, segs.size() - b);
    const int target = std::max(64, (is_side_stream(st) ? kWredSideWgs : wred_main_wgs()) / a.nseg);
    int wg = 0, ctrs = 0;
    for (int k = 0; k < a.nseg; ++k) {
      const PendingRed &r = segs[b + k];
      RedSeg &g = a.s[k];
      g.part = r.part;
      g.grad = r.grad;
      g.n = r.n;
      g.S = r.S;
      red_geom(r.S, r.n, target, V, g.nb, g.rch, g.nch);
      g.wg0 = wg;
      g.ctr0 = ctrs;
      wg += g.nb * g.nch;
      ctrs += g.nb;
    }
    a.ctr = reduce_counters(ctrs, st);
    if (vec) hipLaunchKernelGGL(col_reduce_multi_kernel<4>, dim3(wg), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(col_reduce_multi_kernel<1>, dim3(wg), dim3(256), 0, st, a);
  }
}

// grad[n] = sum over S split rows of part[S][n] (fixed order); part needs S + colsum_rows(S) rows.
// stem36: grad is the stem weight gradient in torch layout (red_out_index); never deferred.
void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st, bool stem36) {
  if (g_red_defer && !stem36) {
    g_red_pending.push_back(PendingRed{part, S, n, grad});
    return;
  }
  const bool vec = (n % 4 == 0) && ((uintptr_t)part % 16 == 0) && ((uintptr_t)grad % 16 == 0);
  const int V = vec ? 4 : 1;
  const long long nb = (n + 16 * V - 1) / (16 * V);
  const int perm = stem36 ? 1 : 0;
  // on a weight-gradient side stream a smaller grid: the reduction is off the critical path,
  // and a 2k-workgroup launch there holds up the dispatch of the main stream's next kernel
  // (MobileNetV2 bs128 on MI355X: 5.07 ms/step at 2048, 5.00 at 512, 4.98-5.00 at 256)
  const int target = is_side_stream(st) ? kWredSideWgs : wred_main_wgs();
  long long want = target / (nb > 0 ? nb : 1);
  int nch = (int)(want < 1 ? 1 : want);
  const int cap = colsum_rows(S);
  if (nch > cap) nch = cap;
  const int rch = (S + nch - 1) / nch;
  nch = (S + rch - 1) / rch;
  int *ctr = nch > 1 ? reduce_counters((int)nb, st) : nullptr;
  if (vec)
    hipLaunchKernelGGL(col_reduce_kernel<4>, dim3((unsigned)nb, nch), dim3(256), 0, st, part, S, n, rch, nch,
                       part + (size_t)S * n, ctr, grad, perm);
  else
    hipLaunchKernelGGL(col_reduce_kernel<1>, dim3((unsigned)nb, nch), dim3(256), 0, st, part, S, n, rch, nch,
                       part + (size_t)S * n, ctr, grad, perm);
}
