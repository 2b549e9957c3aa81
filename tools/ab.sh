#!/bin/bash
# one GPU call: A/B of the bench step, base build (agnes_amd/_exp/lib_base.so) vs the in-tree build,
# alternated (REPS times) on the same box; optional parity first (PAR=1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "${PAR:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread ${PYT:-} > gpurun_out/r4_tests.log 2>&1 || { tail -30 gpurun_out/r4_tests.log; exit 1; }
  tail -2 gpurun_out/r4_tests.log
fi
summ() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), round(d['roofline'].get('path_frac') or 0,3), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"; }
for r in $(seq ${REPS:-2}); do
  for c in ${CFGS:-c2}; do
    timeout -k 10 200 python3 tools/withlib.py agnes_amd/_exp/lib_base.so bench.py --config $c --no-cpu-baseline > gpurun_out/ab_base_$c.json 2> gpurun_out/ab_base_$c.err || { tail -20 gpurun_out/ab_base_$c.err; exit 1; }
    summ gpurun_out/ab_base_$c.json "base $c"
    timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/ab_new_$c.json 2> gpurun_out/ab_new_$c.err || { tail -20 gpurun_out/ab_new_$c.err; exit 1; }
    summ gpurun_out/ab_new_$c.json "new  $c"
  done
done
