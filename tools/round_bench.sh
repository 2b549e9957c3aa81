#!/bin/bash
# one GPU call: the bench line of every workload (CPU leg included) -> gpurun_out/prof/<round>_bench_<cfg>.json
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof
R=${R:-r03}
for c in ${CFGS:-c2 c3 c4 c5 c5d wire}; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/prof/${R}_bench_$c.json 2> gpurun_out/prof/${R}_bench_$c.err \
    || { tail -20 gpurun_out/prof/${R}_bench_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/prof/${R}_bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('path_frac'), d.get('cpu_check_equal'))"
done
