#!/bin/bash
# A/B benchmark over environment settings: AB_VAR=NAME AB_VALS="a b c" [AB_ARGS="bench args"]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for v in $AB_VALS; do
  env "$AB_VAR=$v" timeout -k 10 300 python bench.py --steps 40 --warmup 10 $AB_ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 4; }
  echo "$AB_VAR=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['ms_per_step'], d['value'])")"
done
done
