#!/bin/bash
# Session re-entry sanity: MobileNetV2 + ResNet-50 bench on the rebuilt tree, per-layer conv table.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/s_mnv2.json 2> $O/s_mnv2.err || { tail -20 $O/s_mnv2.err; exit 1; }
cat $O/s_mnv2.json
timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $O/s_rn.json 2> $O/s_rn.err || { tail -20 $O/s_rn.err; exit 1; }
cat $O/s_rn.json
timeout -k 10 300 python -u scripts/conv_bench.py --kinds fwd,fwdbn,dgradm,wgradma > $O/s_conv.txt 2>&1 || { tail -20 $O/s_conv.txt; exit 1; }
cat $O/s_conv.txt
