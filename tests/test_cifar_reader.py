"""CIFAR-10 readers: native binary reader and restricted python-pickle reader."""
import os
import pickle

import numpy as np
import pytest

from pgdist.data.cifar10 import load_cifar10, write_cifar10_bin, TRAIN_FILES


def _fake(n, seed):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8), g.integers(0, 10, n).astype(np.int64)


def test_binary_reader_roundtrip(tmp_path):
    pytest.importorskip("pgdist._pgdist_C")
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    imgs, labs = [], []
    for i, f in enumerate(TRAIN_FILES + ["test_batch"]):
        im, lb = _fake(13 + i, i)
        write_cifar10_bin(str(d / (f + ".bin")), im, lb)
        if f != "test_batch":
            imgs.append(im)
            labs.append(lb)
    tr = load_cifar10(str(tmp_path), train=True)
    assert np.array_equal(tr.images, np.concatenate(imgs))
    assert np.array_equal(tr.labels, np.concatenate(labs))
    te = load_cifar10(str(tmp_path), train=False)
    assert len(te) == 18


def test_python_batches_safe_unpickle(tmp_path):
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()
    im, lb = _fake(7, 3)
    batch = {"data": im.transpose(0, 3, 1, 2).reshape(7, 3072), "labels": lb.tolist()}
    with open(d / "test_batch", "wb") as fh:
        pickle.dump(batch, fh)
    te = load_cifar10(str(tmp_path), train=False)
    assert np.array_equal(te.images, im) and np.array_equal(te.labels, lb)


def test_python_batches_reject_code(tmp_path):
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    with open(d / "test_batch", "wb") as fh:
        pickle.dump({"data": Evil(), "labels": []}, fh)
    with pytest.raises(pickle.UnpicklingError):
        load_cifar10(str(tmp_path), train=False)


def test_missing_dataset_message(tmp_path):
    with pytest.raises(FileNotFoundError, match="synthetic"):
        load_cifar10(str(tmp_path), train=True)
