cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head" > gpurun_out/t_q.log 2>&1; rc=$?; tail -3 gpurun_out/t_q.log; [ $rc -eq 0 ] || { grep -B5 -A25 "Error\|assert" gpurun_out/t_q.log | head -60; exit $rc; }
