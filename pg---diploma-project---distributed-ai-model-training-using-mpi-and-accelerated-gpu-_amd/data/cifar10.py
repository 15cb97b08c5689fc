"""CIFAR-10 dataset readers (no network access: the files must already exist).

Reference: ``torchvision.datasets.CIFAR10(root="./data", train, download)``
(``cifar10_mpi_mobilenet_224.py:93-109``; rank 0 downloads, barrier, then every
rank opens it).  Supported on-disk forms under ``root``:

* ``cifar-10-batches-bin/{data_batch_1..5,test_batch}.bin`` — the binary
  distribution, read by the native threaded reader (``_pgdist_C.read_cifar10_bin``)
* ``cifar-10-batches-py/{data_batch_1..5,test_batch}`` — the python
  distribution (what torchvision downloads), read with a *restricted*
  unpickler that only reconstructs plain containers and numpy arrays
  (no arbitrary code execution from the file)
* ``cifar10_{train,test}.npz`` — cache written by this module (``allow_pickle=False``)

All return :class:`CIFAR10Arrays` with uint8 NHWC ``[N,32,32,3]`` images and int64 labels.
"""
import io
import os
import pickle
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .. import CIFAR10_CLASSES


@dataclass
class CIFAR10Arrays:
    images: np.ndarray        # uint8 [N,32,32,3]
    labels: np.ndarray        # int64 [N]
    classes: tuple = CIFAR10_CLASSES

    def __len__(self):
        return len(self.labels)


TRAIN_FILES = [f"data_batch_{i}" for i in range(1, 6)]
TEST_FILES = ["test_batch"]


class _SafeUnpickler(pickle.Unpickler):
    """Allow only what a CIFAR python batch needs (dicts/lists/bytes + numpy arrays)."""
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("_codecs", "encode"), ("builtins", "bytes"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            import importlib
            return getattr(importlib.import_module(module), name)
        raise pickle.UnpicklingError(f"blocked global {module}.{name} in CIFAR batch")


def _read_py_batch(path: str):
    with open(path, "rb") as fh:
        d = _SafeUnpickler(io.BytesIO(fh.read()), encoding="latin1").load()
    data = np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    labels = np.asarray(d.get("labels", d.get("fine_labels")), dtype=np.int64)
    return np.ascontiguousarray(data), labels


def load_cifar10(root: str = "./data", train: bool = True, native_threads: int = 4) -> CIFAR10Arrays:
    files = TRAIN_FILES if train else TEST_FILES
    npz = os.path.join(root, f"cifar10_{'train' if train else 'test'}.npz")
    bin_dir = os.path.join(root, "cifar-10-batches-bin")
    py_dir = os.path.join(root, "cifar-10-batches-py")
    if os.path.isdir(bin_dir) and all(os.path.exists(os.path.join(bin_dir, f + ".bin")) for f in files):
        from ..ops._lib import lib
        imgs, labels = lib().read_cifar10_bin([os.path.join(bin_dir, f + ".bin") for f in files],
                                              native_threads)
        return CIFAR10Arrays(np.asarray(imgs), np.asarray(labels))
    if os.path.isdir(py_dir) and all(os.path.exists(os.path.join(py_dir, f)) for f in files):
        parts = [_read_py_batch(os.path.join(py_dir, f)) for f in files]
        return CIFAR10Arrays(np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    if os.path.exists(npz):
        z = np.load(npz, allow_pickle=False)
        return CIFAR10Arrays(z["images"], z["labels"].astype(np.int64))
    raise FileNotFoundError(
        f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-bin/, cifar-10-batches-py/ or "
        f"cifar10_{{train,test}}.npz). There is no network access to download it; use --data synthetic.")


def write_cifar10_bin(path: str, images: np.ndarray, labels: np.ndarray):
    """Write arrays in the CIFAR-10 binary record format (used by tests / converters)."""
    n = len(labels)
    rec = np.empty((n, 3073), dtype=np.uint8)
    rec[:, 0] = labels.astype(np.uint8)
    rec[:, 1:] = images.transpose(0, 3, 1, 2).reshape(n, 3072)
    rec.tofile(path)


def load_dataset(name: str, root: str, train: bool, synthetic_size: Optional[int] = None, seed: int = 0,
                 signal: Optional[float] = None):
    if name == "cifar10":
        return load_cifar10(root, train)
    if name == "synthetic":
        from .synthetic import synthetic_cifar
        n = synthetic_size or (50000 if train else 10000)
        imgs, labels = synthetic_cifar(n, seed=seed + (0 if train else 1))
        return CIFAR10Arrays(imgs, labels)
    if name == "synthetic-hard":   # weak, spatially spread class signal + 10 % label noise
        from .synthetic import synthetic_cifar_hard
        n = synthetic_size or (50000 if train else 10000)
        kw = {} if signal is None else {"signal": float(signal)}
        imgs, labels = synthetic_cifar_hard(n, seed=seed, split="train" if train else "test", **kw)
        return CIFAR10Arrays(imgs, labels)
    raise ValueError(f"unknown dataset {name!r}")
