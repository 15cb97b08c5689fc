// Standalone self-test of the native runtime core, built with -fsanitize=address,undefined
// and with -fsanitize=thread by tests/test_native_sanitizers.py (race / memory-error
// detection for the threaded CIFAR-10 decoder).
//   selftest <tmpdir>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../runtime/core.h"

using namespace pgdist_rt;

static unsigned char pix(size_t n, int c, int p) { return (unsigned char)((n * 131 + c * 17 + p * 7) & 255); }

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string dir = argv[1];
  const size_t per_file[] = {37, 5, 64, 1, 19, 40};
  std::vector<std::string> paths;
  size_t n0 = 0;
  for (size_t f = 0; f < 6; ++f) {
    const std::string p = dir + "/batch_" + std::to_string(f) + ".bin";
    FILE *fp = std::fopen(p.c_str(), "wb");
    if (!fp) return 3;
    for (size_t r = 0; r < per_file[f]; ++r) {
      const size_t n = n0 + r;
      unsigned char rec[kCifarRecord];
      rec[0] = (unsigned char)(n % 10);
      for (int c = 0; c < 3; ++c)
        for (int q = 0; q < 1024; ++q) rec[1 + c * 1024 + q] = pix(n, c, q);
      std::fwrite(rec, 1, sizeof(rec), fp);
    }
    std::fclose(fp);
    n0 += per_file[f];
    paths.push_back(p);
  }
  for (int threads : {1, 3, 8}) {
    const std::vector<size_t> counts = cifar_bin_counts(paths);
    size_t total = 0;
    for (size_t c : counts) total += c;
    if (total != n0) return 4;
    std::vector<unsigned char> imgs(total * 3072);
    std::vector<long long> labels(total);
    cifar_bin_decode(paths, counts, threads, imgs.data(), labels.data());
    for (size_t n = 0; n < total; ++n) {
      if (labels[n] != (long long)(n % 10)) return 5;
      for (int q = 0; q < 1024; ++q)
        for (int c = 0; c < 3; ++c)
          if (imgs[n * 3072 + q * 3 + c] != pix(n, c, q)) return 6;
    }
  }
  // sampler: every index appears, shards are disjoint up to the padding, sizes match torch
  for (long long n : {1LL, 7LL, 100LL, 50000LL})
    for (int R : {1, 2, 3, 8})
      for (bool drop : {false, true}) {
        std::vector<long long> perm(n);
        for (long long i = 0; i < n; ++i) perm[i] = (i * 7919) % n;
        std::vector<int> seen(n, 0);
        for (int r = 0; r < R; ++r) {
          const long long m = shard_count(n, R, drop);
          std::vector<long long> out(m > 0 ? m : 1);
          shard_fill(perm.data(), n, R, r, drop, out.data());
          for (long long i = 0; i < m; ++i) {
            if (out[i] < 0 || out[i] >= n) return 7;
            seen[out[i]]++;
          }
        }
        if (!drop)
          for (long long i = 0; i < n; ++i)
            if (!seen[i]) return 8;
      }
  std::printf("selftest ok\n");
  return 0;
}
