#!/bin/bash
# Round 4: 16x16x128 fp8 MFMA on every tile (PGDIST_F8_MX=1), on the <= 64-row tiles only (2),
# off (0), bf16 reference; bs512, interleaved
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mx2 && export TMPDIR=/tmp
O=gpurun_out/mx2
timeout -k 10 300 env PGDIST_F8_MX=2 python -u -m pytest tests/test_kernels_gpu.py -k "fp8" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in bf16 1 2 0; do
    a="--batch-size 512 --steps 20 --warmup 5"; e=1
    [ $v != bf16 ] && { a="$a --fp8 1"; e=$v; }
    PGDIST_F8_MX=$e timeout -k 10 300 python -u bench.py $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('bs512 mx=$v', d['ms_per_step'], d['value'])"
  done
done
