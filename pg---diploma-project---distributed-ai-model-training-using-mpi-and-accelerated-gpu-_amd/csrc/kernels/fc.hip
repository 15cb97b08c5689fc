// fp32 GEMMs of the ResNet-50 classifier head: logits = pooled . W^T + b, dW = dlogits^T . pooled,
// dpool = dlogits . W, db = column sums of dlogits (batch 128 x 2048 features x 1000 classes).
//
// Reference: the final nn.Linear of the torchvision model, run by cuBLAS in fp32 under the
// reference's plain fp32 training (SURVEY.md §2.5 "cuBLAS GEMM (Linear)").  These replace the
// torch.addmm / mm / sum (hipBLASLt) calls the ResNet executor used, so a training step is
// native launches only (recordable into a launch plan).
//
// One strided kernel serves all three products:  C[m][n] = sum_k A(m,k) B(k,n) (+ bias[n]),
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn].  Tiles of 64 x 64 outputs, 4 x 4 per
// thread (two 16-B LDS reads per 16 FMAs; the former 32 x 32 tiles with 2 x 2 per thread
// spent one LDS read per FMA and ran at 0.2-0.4 TB/s, 24-45 us per GEMM, round 4 roofline),
// operands staged through LDS k-major with the unit-stride dimension mapped to consecutive
// threads (coalesced whichever operand is transposed).  The shapes are small (0.5 GFLOP each),
// so parallelism comes from splitting K: every split writes its partial tile to a workspace
// and a second kernel sums the splits in a FIXED order (+ bias) -- deterministic, unlike
// atomic split-K.  The bias gradient is a fixed-order column sum.
#include "../common.h"

namespace {
constexpr int kTM = 64, kTN = 64, kTK = 16;

__global__ __launch_bounds__(256) void fc_gemm_kernel(const float *__restrict__ A, long long sam, long long sak,
                                                      const float *__restrict__ B, long long sbk, long long sbn,
                                                      float *__restrict__ out, int M, int N, int K, int kchunk) {
  __shared__ __attribute__((aligned(16))) float As[kTK][kTM + 4];
  __shared__ __attribute__((aligned(16))) float Bs[kTK][kTN + 4];
  const int tid = threadIdx.x;
  const int tx = tid % 16, ty = tid / 16;   // 4 x 4 outputs: rows ty*4.., cols tx*4..
  const int n0 = blockIdx.x * kTN, m0 = blockIdx.y * kTM;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  float acc[4][4] = {};
  for (int k0 = kb; k0 < ke; k0 += kTK) {
#pragma unroll
    for (int i = 0; i < (kTM * kTK) / 256; ++i) {
      const int e = tid + i * 256;
      int mm, kk;
      if (sak == 1) { kk = e % kTK; mm = e / kTK; }   // k contiguous in memory
      else { mm = e % kTM; kk = e / kTM; }
      const int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < M && k < ke) ? A[(long long)m * sam + (long long)k * sak] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < (kTN * kTK) / 256; ++i) {
      const int e = tid + i * 256;
      int nn, kk;
      if (sbn == 1) { nn = e % kTN; kk = e / kTN; }   // n contiguous in memory
      else { kk = e % kTK; nn = e / kTK; }
      const int n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < N && k < ke) ? B[(long long)k * sbk + (long long)n * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kTK; ++kk) {
      const float4 a = *reinterpret_cast<const float4 *>(&As[kk][ty * 4]);
      const float4 b = *reinterpret_cast<const float4 *>(&Bs[kk][tx * 4]);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float *dst = out + (size_t)blockIdx.z * M * N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < N) dst[(size_t)m * N + n] = acc[i][j];
    }
  }
}

// C[m][n] = (bias[n]) + sum_s P[s][m][n], splits summed in order s = 0..S-1
__global__ __launch_bounds__(256) void fc_splits_kernel(const float *__restrict__ P, int S, const float *__restrict__ bias,
                                                        float *__restrict__ C, int M, int N) {
  const long long MN = (long long)M * N;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < MN; i += (long long)gridDim.x * 256) {
    float v = bias ? bias[i % N] : 0.f;
    for (int s = 0; s < S; ++s) v += P[s * MN + i];
    C[i] = v;
  }
}

// out[n] = sum_m X[m][n], m in order
__global__ __launch_bounds__(256) void col_sum_kernel(const float *__restrict__ X, int M, int N, float *__restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  // 16 rows in flight per thread (the loads are independent; the sum stays in row order)
  float v = 0.f;
  int m = 0;
  for (; m + 16 <= M; m += 16) {
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = X[(size_t)(m + i) * N + n];
#pragma unroll
    for (int i = 0; i < 16; ++i) v += x[i];
  }
  for (; m < M; ++m) v += X[(size_t)m * N + n];
  out[n] = v;
}
}  // namespace

// split count and workspace floats of one fc GEMM (0 workspace: no split)
int fc_gemm_splits(int M, int N, int K) {
  const long long tiles = (long long)((M + kTM - 1) / kTM) * ((N + kTN - 1) / kTN);
  int S = 1;
  while (S < 16 && tiles * S < 512 && K / (S * 2) >= 4 * kTK) S *= 2;
  return S;
}
long long fc_gemm_workspace_floats(int M, int N, int K) {
  const int S = fc_gemm_splits(M, N, K);
  return S > 1 ? (long long)S * M * N : 0;
}

void launch_fc_gemm(const float *A, long long sam, long long sak, const float *B, long long sbk, long long sbn,
                    const float *bias, float *C, int M, int N, int K, float *ws, hipStream_t st) {
  const int S = fc_gemm_splits(M, N, K);
  const int kchunk = ((K + S - 1) / S + kTK - 1) / kTK * kTK;
  const dim3 grid((N + kTN - 1) / kTN, (M + kTM - 1) / kTM, S);
  if (S == 1 && !bias) {
    hipLaunchKernelGGL(fc_gemm_kernel, grid, dim3(256), 0, st, A, sam, sak, B, sbk, sbn, C, M, N, K, kchunk);
    return;
  }
  float *P = S > 1 ? ws : C;
  hipLaunchKernelGGL(fc_gemm_kernel, grid, dim3(256), 0, st, A, sam, sak, B, sbk, sbn, P, M, N, K, kchunk);
  const long long MN = (long long)M * N;
  const int nb = (int)std::min<long long>((MN + 255) / 256, 1024);
  if (S > 1) {
    hipLaunchKernelGGL(fc_splits_kernel, dim3(nb), dim3(256), 0, st, (const float *)P, S, bias, C, M, N);
  } else {   // S == 1 with a bias: add it in place (P == C)
    hipLaunchKernelGGL(fc_splits_kernel, dim3(nb), dim3(256), 0, st, (const float *)C, 1, bias, C, M, N);
  }
}

void launch_col_sum(const float *X, int M, int N, float *out, hipStream_t st) {
  hipLaunchKernelGGL(col_sum_kernel, dim3((N + 255) / 256), dim3(256), 0, st, X, M, N, out);
}
