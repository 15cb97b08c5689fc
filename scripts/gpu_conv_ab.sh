#!/bin/bash
# conv_bench A/B over env settings: $1 kinds, then "TAG:ENV=V,ENV2=V2" specs
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/conv_ab && export TMPDIR=/tmp
KINDS=$1; shift
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 300 python -u scripts/conv_bench.py --kinds $KINDS --reps 9 > gpurun_out/conv_ab/$tag.txt 2>&1 \
    || { echo "$tag failed"; tail -20 gpurun_out/conv_ab/$tag.txt; exit 1; }
  echo "== $tag ($envs)"; grep -v amdgpu.ids gpurun_out/conv_ab/$tag.txt
done
