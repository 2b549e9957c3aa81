#!/bin/bash
# gpu tests, then the C5 bench line with the parity check
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u bench.py --config c5 --check > gpurun_out/bench_c5.log 2>&1 || { tail -30 gpurun_out/bench_c5.log; exit 1; }
grep '^{' gpurun_out/bench_c5.log | cut -c1-1500
