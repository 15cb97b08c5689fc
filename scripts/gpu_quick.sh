cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/ckpt_ddp gpurun_out/best_mpi.pth
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/t_q.log 2>&1; rc=$?; tail -5 gpurun_out/t_q.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/t_q.log | head -80; exit $rc; }
