#!/bin/bash
# bench line + rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per config
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof && export TMPDIR=/tmp
for CFG in ${CFGS:-c2}; do
  timeout -k 10 300 python3 -u bench.py --config $CFG > gpurun_out/prof/bench_$CFG.log 2>&1 || { tail -20 gpurun_out/prof/bench_$CFG.log; exit 1; }
  grep '^{' gpurun_out/prof/bench_$CFG.log > gpurun_out/prof/bench_$CFG.json
  rm -rf gpurun_out/prof/ks_$CFG gpurun_out/prof/fetch_$CFG gpurun_out/prof/write_$CFG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/ks_$CFG -o run -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof/ks_$CFG.log 2>&1 || { tail -20 gpurun_out/prof/ks_$CFG.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_$CFG -o fetch -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch_$CFG.log 2>&1 || { tail -20 gpurun_out/prof/fetch_$CFG.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_$CFG -o write -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write_$CFG.log 2>&1 || { tail -20 gpurun_out/prof/write_$CFG.log; exit 1; }
  echo "== $CFG"; cut -c1-400 gpurun_out/prof/bench_$CFG.json
done
