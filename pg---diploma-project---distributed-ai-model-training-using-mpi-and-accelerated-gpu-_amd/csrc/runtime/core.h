// Plain C++17 core of the native host runtime (no Python, no HIP): CIFAR-10 binary
// decoding with a thread pool and DistributedSampler index math.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace pgdist_rt {

constexpr size_t kCifarRecord = 1 + 3072;   // label byte + planar 3x32x32

// Number of records in each CIFAR-10 .bin file; throws std::runtime_error on a bad size.
std::vector<size_t> cifar_bin_counts(const std::vector<std::string> &paths);

// Decode the files (record order preserved) into imgs [N][32][32][3] (NHWC) and labels [N];
// files are distributed over num_threads threads, each writing disjoint output ranges.
// Throws std::runtime_error on I/O errors.
void cifar_bin_decode(const std::vector<std::string> &paths, const std::vector<size_t> &counts,
                      int num_threads, unsigned char *imgs, long long *labels);

// torch.utils.data.DistributedSampler: number of indices of one rank, and the indices.
long long shard_count(long long n, int num_replicas, bool drop_last);
void shard_fill(const long long *perm, long long n, int num_replicas, int rank, bool drop_last,
                long long *out);

}  // namespace pgdist_rt
