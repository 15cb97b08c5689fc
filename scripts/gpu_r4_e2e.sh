#!/bin/bash
# Round-4 end-to-end evidence on the HARDER synthetic set (synthetic-hard: weak spread class
# signal + 10 % label noise): two 20-epoch gpu128 runs (stability), a planted gradient bug,
# bf16 vs fp8 bs512, 2-rank mpi preset on one GPU (gloo + native P2P, per-step BN broadcast)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2e4 && export TMPDIR=/tmp
O=gpurun_out/e2e4
EP=${EP:-20}
step() { echo "== $1"; }
for s in 1 2; do
  step gpu128_hard_run$s
  timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs $EP --seed $s \
    --save-path $O/best_hard_$s.pth > $O/gpu128_hard_${EP}ep_run$s.log 2>&1 || { tail -10 $O/gpu128_hard_${EP}ep_run$s.log; exit 1; }
  grep -E "^Epoch|Best" $O/gpu128_hard_${EP}ep_run$s.log | tail -4
done
for bug in features.18.0.weight features.1.conv.0.0.weight; do
  step planted_bug_$bug
  PGDIST_FAULT_ZERO_GRAD=$bug timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs $EP \
    --seed 1 --save-path $O/best_bug.pth > $O/gpu128_hard_${EP}ep_bug_$bug.log 2>&1 || { tail -10 $O/gpu128_hard_${EP}ep_bug_$bug.log; exit 1; }
  grep -E "^Epoch|Best" $O/gpu128_hard_${EP}ep_bug_$bug.log | tail -3
done
for p in bf16 fp8; do
  step curve_$p
  timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic-hard --epochs ${EP8:-8} --batch-size 512 --precision $p --seed 1 \
    --save-path $O/best_$p.pth > $O/hard_bs512_${p}.log 2>&1 || { tail -10 $O/hard_bs512_${p}.log; exit 1; }
  grep -E "^Epoch|Best" $O/hard_bs512_${p}.log | tail -3
done
step mpi_2rank
PGDIST_COMM=p2p timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 train.py --preset mpi --data synthetic-hard --epochs ${EPM:-10} --dist-backend gloo \
  --bn-sync broadcast --save-path $O/best_mpi.pth > $O/mpi_2rank_hard.log 2>&1 || { tail -20 $O/mpi_2rank_hard.log; exit 1; }
tail -8 $O/mpi_2rank_hard.log
