// Single-launch deterministic column reductions (see reduce.h): the weight-gradient
// split-M reduction  out[n] = sum_r part[r][n]  used by every wgrad kernel, and the
// per-device arrival counters of the last-workgroup hand-off.
#include "../reduce.h"

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
constexpr int kWredMinRows = 8;
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

// level-1 rows the wgrad reduction of R partial rows needs after the partials
int colsum_rows(int R) { return red_nch(R, kWredMinRows); }

__global__ __launch_bounds__(256) void col_reduce_kernel(const float *__restrict__ part, int R, long long n,
                                                         int rch, int nch, float *__restrict__ lvl1,
                                                         int *__restrict__ ctr, float *__restrict__ out) {
  __shared__ int flag;
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  const int r0 = blockIdx.y * rch, r1 = min(R, r0 + rch);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < n) {
    int r = r0;
    for (; r + 3 < r1; r += 4) {
      a0 += part[(size_t)r * n + i];
      a1 += part[(size_t)(r + 1) * n + i];
      a2 += part[(size_t)(r + 2) * n + i];
      a3 += part[(size_t)(r + 3) * n + i];
    }
    for (; r < r1; ++r) a0 += part[(size_t)r * n + i];
  }
  const float s1 = (a0 + a1) + (a2 + a3);
  if (nch == 1) {
    if (i < n) out[i] = s1;
    return;
  }
  if (i < n) st_sc1(lvl1 + (size_t)blockIdx.y * n + i, s1);
  if (!arrive_last(ctr, nch, &flag)) return;
  if (i < n) {
    float s = 0.f;
    for (int k = 0; k < nch; ++k) s += ld_sc1(lvl1 + (size_t)k * n + i);
    out[i] = s;
  }
}

// grad[n] = sum over S split rows of part[S][n] (fixed order); part needs S + colsum_rows(S) rows
void launch_wgrad_reduce(float *part, int S, long long n, float *grad, hipStream_t st) {
  const int rch = red_rch(S, kWredMinRows), nch = red_nch(S, kWredMinRows);
  const unsigned nb = (unsigned)((n + 255) / 256);
  int *ctr = nch > 1 ? reduce_counters((int)nb, st) : nullptr;
  hipLaunchKernelGGL(col_reduce_kernel, dim3(nb, nch), dim3(256), 0, st, part, S, n, rch, nch,
                     part + (size_t)S * n, ctr, grad);
}
