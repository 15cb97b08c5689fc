#!/bin/bash
# Round 4: depthwise small-map knobs re-swept after the block-output fusion and the prologue
# load reordering (same box, 2 reps each, bench ms/step)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4k2 && export TMPDIR=/tmp
O=gpurun_out/r4k2
ab() {
  t=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 60 --warmup 10 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$t', d['ms_per_step'])"
}
for i in 1 2; do
  ab default X=1
  ab fdepth_small6 PGDIST_DW_FDEPTH_SMALL=6
  ab fdepth_small8 PGDIST_DW_FDEPTH_SMALL=8
  ab dw_wide0 PGDIST_DW_WIDE=0
  ab dw_geom0 PGDIST_DW_GEOM=0
  ab dw_wrows14 PGDIST_DW_WROWS=14
  ab fuse_hw784 PGDIST_FUSE_BLOCK_OUT_HW=784
  ab dw_rows28 PGDIST_DW_ROWS=28
done
