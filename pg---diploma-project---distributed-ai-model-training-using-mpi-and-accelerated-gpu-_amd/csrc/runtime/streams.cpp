// CU-masked HIP streams.
//
// The MobileNetV2 backward runs its weight gradients on a second stream beside the critical
// dgrad chain (engine/executor.py).  A side-stream launch of a few thousand workgroups takes
// every free CU slot, and the main stream's next dependent kernel then waits for slots to
// drain (kernel traces: 30-60 us main-stream gaps right after the side-stream flushes).
// Confining the side stream to a subset of the CUs (hipExtStreamCreateWithCUMask: the stream
// gets a HW queue whose dispatches may only use the masked CUs) keeps most of the chip
// available to the critical path while the side work still overlaps it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace pgdist_rt {

// a stream on `device` whose kernels may use CU i iff (i % den) < num (num / den of the CUs,
// spread evenly over the logical CU ids)
uintptr_t cu_masked_stream(int device, int num, int den) {
  if (den < 1 || num < 1 || num > den) throw std::invalid_argument("cu_masked_stream: 1 <= num <= den");
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) throw std::runtime_error(std::string("hipSetDevice: ") + hipGetErrorString(e));
  int ncu = 0;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || ncu <= 0) throw std::runtime_error("cu_masked_stream: CU count unavailable");
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i)
    if (i % den < num) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
  return reinterpret_cast<uintptr_t>(s);
}

}  // namespace pgdist_rt
