#!/bin/bash
# one GPU call: the current bench.py against another bench script (OLD, same library), alternated
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then s=$OLD; else s=bench.py; fi
    timeout -k 10 200 python3 $s --config ${CFG:-c2} --no-cpu-baseline > gpurun_out/bab_$v.json 2> gpurun_out/bab_$v.err || { tail -20 gpurun_out/bab_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bab_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['kernel_ms'],4), round(d['roofline']['path_frac'],3), round(d['roofline']['kernel_avg_ms'],4))"
  done
done
