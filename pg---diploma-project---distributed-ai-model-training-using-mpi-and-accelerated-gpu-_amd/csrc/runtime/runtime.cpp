// Native host runtime: CIFAR-10 binary reader (threaded) and sampler index math.
//
// Reference data path: torchvision.datasets.CIFAR10(root="./data") unpickles the
// python batches and hands PIL images to 2 DataLoader worker processes per rank
// (cifar10_mpi_mobilenet_224.py:104-133).  pgdist instead reads the whole split
// once, natively, into one NHWC uint8 array that is uploaded to HBM and stays
// resident (150 MB for the train split); augmentation then runs on the GPU.
#include "runtime.h"

#include <stdexcept>

namespace pgdist_rt {

// ------------------------------------------------------------------ Python entry points
py::tuple read_cifar10_bin(const std::vector<std::string> &paths, int num_threads) {
  const std::vector<size_t> counts = cifar_bin_counts(paths);
  size_t total = 0;
  for (size_t c : counts) total += c;
  py::array_t<unsigned char> imgs({(py::ssize_t)total, (py::ssize_t)32, (py::ssize_t)32, (py::ssize_t)3});
  py::array_t<long long> labels({(py::ssize_t)total});
  unsigned char *ip = imgs.mutable_data();
  long long *lp = labels.mutable_data();
  {
    py::gil_scoped_release nogil;
    cifar_bin_decode(paths, counts, num_threads, ip, lp);
  }
  return py::make_tuple(imgs, labels);
}

py::array_t<long long> shard_indices(py::array_t<long long, py::array::c_style> perm,
                                     int num_replicas, int rank, bool drop_last) {
  if (num_replicas < 1 || rank < 0 || rank >= num_replicas)
    throw std::invalid_argument("invalid num_replicas/rank");
  const long long n = perm.size();
  py::array_t<long long> out({(py::ssize_t)shard_count(n, num_replicas, drop_last)});
  shard_fill(perm.data(), n, num_replicas, rank, drop_last, out.mutable_data());
  return out;
}

}  // namespace pgdist_rt
