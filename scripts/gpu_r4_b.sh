#!/bin/bash
# Round 4 B: per-op isolated roofline with the LDS-DMA pw wgrad on / off, bench A/B, executor tests
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
for v in dma nodma narrow; do
  case $v in dma) E="X=1";; nodma) E="PGDIST_PWWG_DMA=0";; narrow) E="PGDIST_PWWG_DMA_WIDE=0";; esac
  env $E timeout -k 10 300 python -u scripts/roofline.py --out $O/roofline_$v.txt > $O/roofline_$v.log 2>&1 || { tail -20 $O/roofline_$v.log; exit 1; }
  echo "== $v"; grep -E "pw_wgrad|wgrad_reduce|total" $O/roofline_$v.txt | tail -8
done
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'], d['value'])"
}
for i in 1 2; do ab dma X=1; ab nodma PGDIST_PWWG_DMA=0; ab narrow PGDIST_PWWG_DMA_WIDE=0; done
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exe.log 2>&1
rc=$?; tail -3 $O/pytest_exe.log; [ $rc -eq 0 ] || exit $rc
