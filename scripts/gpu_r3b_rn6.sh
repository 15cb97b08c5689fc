#!/bin/bash
# ResNet-50 materialisation policy re-check after the wgrad / epilogue changes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
for cfg in "-" "PGDIST_RN_ACT=all" "PGDIST_RN_ACT=none" "-" "PGDIST_RN_ACT=all" "PGDIST_RN_ACT=none"; do
  [ "$cfg" = "-" ] && c="" || c="$cfg"
  env $c timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn6_b.json 2> $O/rn6_b.err || { tail -20 $O/rn6_b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rn6_b.json')); print('$cfg', d['ms_per_step'], d['value'])"
done
