// Native host runtime: CIFAR-10 binary reader (threaded) and sampler index math.
//
// Reference data path: torchvision.datasets.CIFAR10(root="./data") unpickles the
// python batches and hands PIL images to 2 DataLoader worker processes per rank
// (cifar10_mpi_mobilenet_224.py:104-133).  pgdist instead reads the whole split
// once, natively, into one NHWC uint8 array that is uploaded to HBM and stays
// resident (150 MB for the train split); augmentation then runs on the GPU.
#include "runtime.h"

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace pgdist_rt {

static constexpr size_t kRec = 1 + 3072;

py::tuple read_cifar10_bin(const std::vector<std::string> &paths, int num_threads) {
  std::vector<size_t> counts(paths.size());
  size_t total = 0;
  for (size_t f = 0; f < paths.size(); ++f) {
    FILE *fp = std::fopen(paths[f].c_str(), "rb");
    if (!fp) throw std::runtime_error("cannot open " + paths[f]);
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fclose(fp);
    if (sz < 0 || (size_t)sz % kRec != 0)
      throw std::runtime_error(paths[f] + ": size is not a multiple of 3073 (not a CIFAR-10 .bin)");
    counts[f] = (size_t)sz / kRec;
    total += counts[f];
  }
  py::array_t<unsigned char> imgs({(py::ssize_t)total, (py::ssize_t)32, (py::ssize_t)32, (py::ssize_t)3});
  py::array_t<long long> labels({(py::ssize_t)total});
  unsigned char *ip = imgs.mutable_data();
  long long *lp = labels.mutable_data();
  std::vector<size_t> first(paths.size());
  for (size_t f = 0, acc = 0; f < paths.size(); ++f) { first[f] = acc; acc += counts[f]; }

  std::string err;
  {
    py::gil_scoped_release nogil;
    if (num_threads < 1) num_threads = 1;
    std::vector<std::thread> pool;
    std::vector<std::string> errs(paths.size());
    for (int t = 0; t < num_threads; ++t) {
      pool.emplace_back([&, t]() {
        std::vector<unsigned char> buf;
        for (size_t f = t; f < paths.size(); f += num_threads) {
          FILE *fp = std::fopen(paths[f].c_str(), "rb");
          if (!fp) { errs[f] = "cannot open " + paths[f]; continue; }
          buf.resize(counts[f] * kRec);
          const size_t got = std::fread(buf.data(), 1, buf.size(), fp);
          std::fclose(fp);
          if (got != buf.size()) { errs[f] = "short read " + paths[f]; continue; }
          for (size_t r = 0; r < counts[f]; ++r) {
            const unsigned char *rec = buf.data() + r * kRec;
            const size_t n = first[f] + r;
            lp[n] = rec[0];
            unsigned char *dst = ip + n * 3072;
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
    for (auto &e : errs) if (!e.empty()) { err = e; break; }
  }
  if (!err.empty()) throw std::runtime_error(err);
  return py::make_tuple(imgs, labels);
}

py::array_t<long long> shard_indices(py::array_t<long long, py::array::c_style> perm,
                                     int num_replicas, int rank, bool drop_last) {
  if (num_replicas < 1 || rank < 0 || rank >= num_replicas)
    throw std::invalid_argument("invalid num_replicas/rank");
  const long long n = perm.size();
  const long long *p = perm.data();
  // torch: drop_last and n % r != 0 -> ceil((n - r) / r) == n / r ; else ceil(n / r)
  const long long num_samples = (drop_last && n % num_replicas != 0)
                                    ? n / num_replicas
                                    : (n + num_replicas - 1) / num_replicas;
  py::array_t<long long> out({(py::ssize_t)num_samples});
  long long *o = out.mutable_data();
  for (long long i = 0; i < num_samples; ++i) {
    const long long gi = rank + i * num_replicas;  // index into padded list
    long long src;
    if (gi < n) src = p[gi];
    else src = p[(gi - n) % n];  // padding repeats the head (wraps as often as needed)
    o[i] = src;
  }
  return out;
}

}  // namespace pgdist_rt
