#!/bin/bash
# dw_bench A/B over env settings: $1 kinds, then "TAG:ENV=V,ENV2=V2" specs
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/dw_ab && export TMPDIR=/tmp
KINDS=$1; shift
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 300 python -u scripts/dw_bench.py --kinds $KINDS --reps 11 > gpurun_out/dw_ab/$tag.txt 2>&1 \
    || { echo "$tag failed"; tail -20 gpurun_out/dw_ab/$tag.txt; exit 1; }
  echo "== $tag ($envs)"; grep -v amdgpu.ids gpurun_out/dw_ab/$tag.txt
done
