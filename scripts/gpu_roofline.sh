#!/bin/bash
# Per-op roofline table of the MobileNetV2 step ($1: tag, $2...: extra roofline.py args)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-cur}; shift
timeout -k 10 300 python -u scripts/roofline.py --out gpurun_out/roofline_$TAG.txt "$@" > gpurun_out/roofline_$TAG.log 2>&1
rc=$?; tail -30 gpurun_out/roofline_$TAG.log; exit $rc
