#!/bin/bash
# gpu tests + kernel micro-bench (one GPU call)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/kbench.py --iters 10 "$@" > gpurun_out/kbench.log 2>&1 || { cat gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
