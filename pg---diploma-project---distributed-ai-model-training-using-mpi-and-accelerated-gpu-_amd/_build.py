"""In-tree build of the native library ``_pgdist_C`` (HIP kernels for gfx950 +
C++ host runtime + pybind11 bindings).

Every ``csrc/kernels/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950``
(no hipify, no CUDA, no Triton), host C++ with hipcc as plain C++17, and the
objects are linked into ``pgdist/_pgdist_C<EXT_SUFFIX>`` next to this file, so
the built library travels with the repository snapshot to the GPU box.
Incremental: an object is rebuilt when its source, a shared header or the
flags change.

CLI:  python -m pgdist._build [-v] [-j N] [--force]
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
BUILD_DIR = os.path.join(REPO, "build", "pgdist")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB_NAME = "_pgdist_C"
OUT = os.path.join(PKG_DIR, LIB_NAME + EXT_SUFFIX)
ARCH = os.environ.get("PGDIST_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build pgdist native code)")


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _flags():
    common = ["-O3", "-std=c++17", "-fPIC", "-I" + CSRC, "-Wno-unused-result"]
    # extra preprocessor defines for same-box A/B builds of a variant copy (e.g.
    # PGDIST_DEFINES="NAME=VALUE ..."); empty for the in-tree build
    common += ["-D" + d for d in os.environ.get("PGDIST_DEFINES", "").split()]
    hip = common + [f"--offload-arch={ARCH}", "-x", "hip", "-munsafe-fp-atomics"]
    # host translation units (bindings, runtime) contain no kernels; target gfx950 only as well
    host = common + [f"--offload-arch={ARCH}", "-fvisibility=hidden"] + ["-I" + p for p in _pybind_includes()]
    return hip, host


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _needs(src, obj, flags, headers):
    stamp = obj + ".flags"
    h = hashlib.sha1(" ".join(flags).encode()).hexdigest()
    if not os.path.exists(obj) or not os.path.exists(stamp):
        return True, h
    if open(stamp).read().strip() != h:
        return True, h
    mt = os.path.getmtime(obj)
    if os.path.getmtime(src) > mt or any(os.path.getmtime(x) > mt for x in headers):
        return True, h
    return False, h


def _compile(src, obj, flags, verbose):
    cmd = [_hipcc()] + flags + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return src


def build(verbose: bool = False, jobs: int = 8, force: bool = False) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    hip_flags, host_flags = _flags()
    headers = _headers()
    jobs_list = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        jobs_list.append((src, hip_flags))
    for src in [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
        jobs_list.append((src, host_flags))
    objs, todo = [], []
    for src, fl in jobs_list:
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(BUILD_DIR, rel + ".o")
        objs.append(obj)
        need, h = _needs(src, obj, fl, headers)
        if need or force:
            todo.append((src, obj, fl, h))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = {ex.submit(_compile, s, o, f, verbose): (o, h) for s, o, f, h in todo}
            for fut in cf.as_completed(futs):
                fut.result()
                o, h = futs[fut]
                with open(o + ".flags", "w") as fh:
                    fh.write(h)
    relink = bool(todo) or force or not os.path.exists(OUT) or any(
        os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs)
    if relink:
        import torch  # link against the HIP runtime torch ships (same soname, one runtime per process)
        torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
        tmp = OUT + ".tmp"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            "-L" + torch_lib, "-Wl,-rpath," + torch_lib, "-lamdhip64"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    out = build(a.verbose, a.jobs, a.force)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
