#!/bin/bash
# one GPU call: per workload, the rocprofv3 kernel-trace summary and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, as MI355X_MICROARCH.md prescribes) of the same
# bench command, collected under gpurun_out/prof/ as <round>_<cfg>_{kernel_stats,pmc_fetch,pmc_write}.csv
# usage: R=r03 CFGS="c2 c3 c4 c5 c5d" bash tools/round_profiles.sh
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${R:-r03}
for c in ${CFGS:-c2 c3 c4 c5 c5d}; do
  run="python3 bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2"
  rm -rf gpurun_out/prof/$c && mkdir -p gpurun_out/prof/$c
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$c/ks -o ks -- $run \
    > gpurun_out/prof/$c.ks.log 2>&1 || { tail -20 gpurun_out/prof/$c.ks.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/$c/f -o f -- $run \
    > gpurun_out/prof/$c.f.log 2>&1 || { tail -20 gpurun_out/prof/$c.f.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/$c/w -o w -- $run \
    > gpurun_out/prof/$c.w.log 2>&1 || { tail -20 gpurun_out/prof/$c.w.log; exit 1; }
  cp "$(find gpurun_out/prof/$c/ks -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/${R}_${c}_kernel_stats.csv
  cp "$(find gpurun_out/prof/$c/f -name '*counter_collection.csv' | head -1)" gpurun_out/prof/${R}_${c}_pmc_fetch.csv
  cp "$(find gpurun_out/prof/$c/w -name '*counter_collection.csv' | head -1)" gpurun_out/prof/${R}_${c}_pmc_write.csv
  rm -rf gpurun_out/prof/$c
  echo "$c done"
done
