#!/bin/bash
# HIP runtime knob A/B on the default bench (host-side launch throttling)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { env "$@" timeout -k 10 120 python bench.py --steps 50 --warmup 10 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; return 0; }
  echo "$* -> $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'])")"; }
for rep in 1 2; do
run X=0
run ROC_SIGNAL_POOL_SIZE=1024
run ROC_AQL_QUEUE_SIZE=16384
run ROC_SIGNAL_POOL_SIZE=1024 ROC_AQL_QUEUE_SIZE=16384
run DEBUG_CLR_MAX_BATCH_SIZE=1024
run ROC_SKIP_KERNEL_ARG_COPY=1
run HIP_FORCE_DEV_KERNARG=0
run HIP_FORCE_DEV_KERNARG=1
run AMD_DIRECT_DISPATCH=0
done
