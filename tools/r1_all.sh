#!/bin/bash
# bench lines (with CPU baseline) and rocprofv3 kernel stats for c2, c3, c4 (one GPU call)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --check > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  grep '^{' gpurun_out/bench_$c.log | cut -c1-300
  rm -rf gpurun_out/prof_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
done
