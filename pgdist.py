"""Import shim: exposes the framework package under the importable name ``pgdist``.

The package directory is named
``pg---diploma-project---distributed-ai-model-training-using-mpi-and-accelerated-gpu-_amd``
(the project's required layout), which is not a valid Python identifier.  This
module loads that directory as the package ``pgdist`` and replaces itself in
``sys.modules`` so ``import pgdist`` / ``from pgdist.models import ...`` work.
"""
import importlib.util
import os
import sys

PKG_DIRNAME = "pg---diploma-project---distributed-ai-model-training-using-mpi-and-accelerated-gpu-_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), PKG_DIRNAME)


def _load():
    spec = importlib.util.spec_from_file_location(
        "pgdist", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["pgdist"] = mod
    spec.loader.exec_module(mod)
    return mod


_load()
