#!/bin/bash
# one GPU call: the bench step of several library builds, alternated on one box.
# LIBS="name=path ..." (path "-" = the in-tree library), CFGS, REPS; optional parity first (PAR="pytest -k expr")
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "${PAR:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread -k "$PAR" > gpurun_out/abn_tests.log 2>&1 || { tail -30 gpurun_out/abn_tests.log; exit 1; }
  tail -2 gpurun_out/abn_tests.log
fi
summ() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), round(d['roofline'].get('path_frac') or 0,3), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()}, {k:round(v.get('avg_ms', v.get('ms_per_call', 0)),4) for k,v in d.get('event_stream',{}).items() if isinstance(v,dict)})"; }
for r in $(seq ${REPS:-2}); do
  for c in ${CFGS:-c2}; do
    for spec in ${LIBS:-new=-}; do
      name=${spec%%=*}; path=${spec#*=}
      if [ "$path" = "-" ]; then run="python3 bench.py"; else run="python3 tools/withlib.py $path bench.py"; fi
      timeout -k 10 200 $run --config $c --no-cpu-baseline ${BARGS:-} > gpurun_out/abn_${name}_$c.json 2> gpurun_out/abn_${name}_$c.err || { tail -20 gpurun_out/abn_${name}_$c.err; exit 1; }
      summ gpurun_out/abn_${name}_$c.json "$name $c"
    done
  done
done
