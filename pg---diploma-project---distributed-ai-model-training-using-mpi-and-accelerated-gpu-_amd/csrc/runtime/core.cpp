// Plain C++17 core of the native host runtime (see core.h).  Built into the
// Python extension and, standalone with sanitizers, by tests/test_native_sanitizers.py.
#include "core.h"

#include <cstdio>
#include <stdexcept>
#include <thread>

namespace pgdist_rt {

std::vector<size_t> cifar_bin_counts(const std::vector<std::string> &paths) {
  std::vector<size_t> counts(paths.size());
  for (size_t f = 0; f < paths.size(); ++f) {
    FILE *fp = std::fopen(paths[f].c_str(), "rb");
    if (!fp) throw std::runtime_error("cannot open " + paths[f]);
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fclose(fp);
    if (sz < 0 || (size_t)sz % kCifarRecord != 0)
      throw std::runtime_error(paths[f] + ": size is not a multiple of 3073 (not a CIFAR-10 .bin)");
    counts[f] = (size_t)sz / kCifarRecord;
  }
  return counts;
}

void cifar_bin_decode(const std::vector<std::string> &paths, const std::vector<size_t> &counts,
                      int num_threads, unsigned char *imgs, long long *labels) {
  std::vector<size_t> first(paths.size());
  for (size_t f = 0, acc = 0; f < paths.size(); ++f) {
    first[f] = acc;
    acc += counts[f];
  }
  if (num_threads < 1) num_threads = 1;
  std::vector<std::string> errs(paths.size());   // one slot per file: no shared writes
  std::vector<std::thread> pool;
  for (int t = 0; t < num_threads; ++t) {
    pool.emplace_back([&, t]() {
      std::vector<unsigned char> buf;
      for (size_t f = t; f < paths.size(); f += num_threads) {
        FILE *fp = std::fopen(paths[f].c_str(), "rb");
        if (!fp) { errs[f] = "cannot open " + paths[f]; continue; }
        buf.resize(counts[f] * kCifarRecord);
        const size_t got = std::fread(buf.data(), 1, buf.size(), fp);
        std::fclose(fp);
        if (got != buf.size()) { errs[f] = "short read " + paths[f]; continue; }
        for (size_t r = 0; r < counts[f]; ++r) {
          const unsigned char *rec = buf.data() + r * kCifarRecord;
          const size_t n = first[f] + r;
          labels[n] = rec[0];
          unsigned char *dst = imgs + n * 3072;
          const unsigned char *R = rec + 1, *G = rec + 1 + 1024, *B = rec + 1 + 2048;
          for (int p = 0; p < 1024; ++p) {  // planar CHW -> interleaved HWC
            dst[p * 3 + 0] = R[p];
            dst[p * 3 + 1] = G[p];
            dst[p * 3 + 2] = B[p];
          }
        }
      }
    });
  }
  for (auto &th : pool) th.join();
  for (auto &e : errs)
    if (!e.empty()) throw std::runtime_error(e);
}

long long shard_count(long long n, int num_replicas, bool drop_last) {
  // torch: drop_last and n % r != 0 -> ceil((n - r) / r) == n / r ; else ceil(n / r)
  return (drop_last && n % num_replicas != 0) ? n / num_replicas : (n + num_replicas - 1) / num_replicas;
}

void shard_fill(const long long *perm, long long n, int num_replicas, int rank, bool drop_last,
                long long *out) {
  const long long m = shard_count(n, num_replicas, drop_last);
  for (long long i = 0; i < m; ++i) {
    const long long gi = rank + i * num_replicas;  // index into the padded list
    out[i] = gi < n ? perm[gi] : perm[(gi - n) % n];   // padding repeats the head (wrapping)
  }
}

}  // namespace pgdist_rt
