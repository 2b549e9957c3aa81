#!/bin/bash
# one GPU call: the C2 edge summary (count, scan, emit) for several library builds
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for spec in ${LIBS:-cur=-}; do
  name=${spec%%=*}; path=${spec#*=}
  if [ "$path" = "-" ]; then run="python3 bench.py"; else run="python3 tools/withlib.py $path bench.py"; fi
  timeout -k 10 200 $run --config ${CFG:-c2} --no-cpu-baseline --steps 5 > gpurun_out/ed_$name.json 2> gpurun_out/ed_$name.err || { tail -20 gpurun_out/ed_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ed_$name.json').read().strip().splitlines()[-1]); e=d['edge_summary']; print('$name', {k:(round(v['avg_ms'],4), v.get('traffic')) for k,v in e.items() if isinstance(v,dict)})"
done
