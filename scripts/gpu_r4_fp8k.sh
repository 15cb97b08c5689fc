#!/bin/bash
# Round 4: fp8 layer policy threshold re-swept with the 16x16x128 MFMA tile GEMMs (bs512)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fp8k && export TMPDIR=/tmp
O=gpurun_out/fp8k
for i in 1 2; do
  for v in bf16 64 160 384; do
    a="--batch-size 512 --steps 20 --warmup 5"; k=64
    [ $v != bf16 ] && { a="$a --fp8 1"; k=$v; }
    PGDIST_FP8_MIN_K=$k timeout -k 10 300 python -u bench.py $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('bs512 $v', d['ms_per_step'], d['value'])"
  done
done
