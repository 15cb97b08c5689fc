#!/bin/bash
# ResNet-50 bench A/B over env settings: each arg is "TAG:ENV=V,ENV2=V2"
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rn_ab && export TMPDIR=/tmp
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  envs=${envs//,/ }
  env $envs timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn_ab/$tag.json 2> gpurun_out/rn_ab/$tag.err \
    || { echo "$tag failed"; tail -20 gpurun_out/rn_ab/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/rn_ab/$tag.json')); print('$tag', '$envs', d['ms_per_step'], d['value'])"
done
