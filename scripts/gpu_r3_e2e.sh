#!/bin/bash
# Round-3 end-to-end evidence: same-box bf16 vs fp8 bs512 bench, 20-epoch gpu128 run,
# 3-epoch bf16 vs fp8 bs512 loss curves, 2-rank mpi preset (one GPU, gloo + native P2P) with
# the per-step BN broadcast and the replica check
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/e2e && export TMPDIR=/tmp
O=gpurun_out/e2e
step() { echo "== $1"; }
step bench_bf16_bs512
timeout -k 10 300 python -u bench.py --batch-size 512 --steps 10 --warmup 3 > $O/bench_bf16_bs512.json 2> $O/bench_bf16_bs512.err || { tail -5 $O/bench_bf16_bs512.err; exit 1; }
cat $O/bench_bf16_bs512.json
step bench_fp8_bs512
timeout -k 10 300 python -u bench.py --batch-size 512 --fp8 1 --steps 10 --warmup 3 > $O/bench_fp8_bs512.json 2> $O/bench_fp8_bs512.err || { tail -5 $O/bench_fp8_bs512.err; exit 1; }
cat $O/bench_fp8_bs512.json
step gpu128_20ep
timeout -k 10 600 python -u train.py --preset gpu128 --data synthetic --epochs 20 --save-path $O/best_gpu128.pth > $O/gpu128_synthetic_20ep.log 2>&1 || { tail -10 $O/gpu128_synthetic_20ep.log; exit 1; }
tail -4 $O/gpu128_synthetic_20ep.log
for p in bf16 fp8; do
  step curve_$p
  timeout -k 10 300 python -u train.py --preset gpu128 --data synthetic --epochs 3 --batch-size 512 --precision $p \
    --save-path $O/best_$p.pth > $O/curve_bs512_${p}_3ep.log 2>&1 || { tail -10 $O/curve_bs512_${p}_3ep.log; exit 1; }
  grep -i "epoch" $O/curve_bs512_${p}_3ep.log | tail -3
done
step mpi_2rank
PGDIST_COMM=p2p timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 train.py --preset mpi --data synthetic --epochs 2 --dist-backend gloo --max-steps-per-epoch 80 \
  --bn-sync broadcast --save-path $O/best_mpi.pth > $O/mpi_2rank_gloo_p2p_broadcast.log 2>&1 || { tail -20 $O/mpi_2rank_gloo_p2p_broadcast.log; exit 1; }
tail -8 $O/mpi_2rank_gloo_p2p_broadcast.log
