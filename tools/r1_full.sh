#!/bin/bash
# gpu tests, smoke, the default bench line and a rocprofv3 kernel-stats pass of it
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
