#!/bin/bash
# one GPU call: -m "gpu and not slow" parity, then bench c2 without the CPU leg (A/B of a step change)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread ${PYT:-} > gpurun_out/r4_tests.log 2>&1 || { tail -30 gpurun_out/r4_tests.log; exit 1; }
tail -3 gpurun_out/r4_tests.log
for c in ${CFGS:-c2}; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r4_bench_$c.json 2> gpurun_out/r4_bench_$c.err || { tail -20 gpurun_out/r4_bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4_bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['roofline'].get('path_frac'), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
