#!/bin/bash
# gpu parity tests (not slow) + kernel micro-bench, one GPU call
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread ${PYT:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/kbench.py --iters 10 ${KB:-c2_plain c2_sm c3_sm} > gpurun_out/kbench.log 2>&1 || { cat gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
