"""Loader for the in-tree native library ``_pgdist_C``.

On a GPU box the HIP path is mandatory: if the library is missing or was built
for the wrong target, ``lib()`` raises instead of silently falling back to
PyTorch ops (the CPU-only ``torch`` backend exists for tests and as the
semantic oracle, and is selected explicitly).
"""
import importlib
import os

_LIB = None
_ERR = None


def lib():
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (loads the HIP runtime the extension links against)
    try:
        _LIB = importlib.import_module("pgdist._pgdist_C")
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        if os.environ.get("PGDIST_AUTOBUILD", "1") == "1":
            from .. import _build
            _build.build()
            _LIB = importlib.import_module("pgdist._pgdist_C")
        else:
            _ERR = e
            raise RuntimeError(
                "pgdist native library _pgdist_C is not built; run `python -m pgdist._build` "
                "(or __graft_entry__.build())") from e
    if os.environ.get("PGDIST_DETERMINISTIC", "0") == "1":
        _LIB.bn_set_rep(1 << 30)   # ops.kernels.set_deterministic(True)
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def lib_path() -> str:
    return lib().__file__
