// Host-side native runtime pieces of pgdist (C++17, no torch dependency).
//
// core.h holds the plain C++ implementations (also built standalone, with
// AddressSanitizer / ThreadSanitizer, by tests/test_native_sanitizers.py);
// this header adds the Python (pybind11) entry points.
#pragma once
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <string>
#include <vector>

#include "core.h"

namespace pgdist_rt {
namespace py = pybind11;

// Parallel reader for the CIFAR-10 *binary* distribution (data_batch_{1..5}.bin,
// test_batch.bin): records of 1 label byte + 3072 planar (R,G,B 32x32) bytes.
// Returns (uint8 [N,32,32,3] NHWC, int64 [N]) — the layout the device-resident
// dataset and the GPU augmentation kernel consume.
py::tuple read_cifar10_bin(const std::vector<std::string> &paths, int num_threads);

// DistributedSampler index math (torch.utils.data.distributed.DistributedSampler):
// pad `perm` by wrapping around to a multiple of num_replicas (or truncate when
// drop_last) and take every num_replicas-th element starting at rank.
py::array_t<long long> shard_indices(py::array_t<long long, py::array::c_style> perm,
                                     int num_replicas, int rank, bool drop_last);
}  // namespace pgdist_rt
