#!/bin/bash
# Build the A/B baseline on the CPU host: the package, bench.py and the entry point of git
# revision $1 (default HEAD) extracted under ab/base/ and built there (its own .so, its own
# Python), so scripts/gpu_ab_so.sh can run it beside the working tree on one GPU box.
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
PKG=pg---diploma-project---distributed-ai-model-training-using-mpi-and-accelerated-gpu-_amd
rm -rf ab/base && mkdir -p ab/base
git archive "$REV" bench.py pgdist.py __graft_entry__.py $PKG | tar -x -C ab/base
(cd ab/base && python -c "import __graft_entry__ as g; g.build()" 2>&1 | tail -1)
rm -rf ab/base/build ab/base/$PKG/build ab/base/$PKG/csrc/*.o
