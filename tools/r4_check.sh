#!/bin/bash
# one GPU call: the edge stream kernel's parity (fast tests, then the full-size records),
# the u64 flow's parity, then the bench lines of c2w / c2 / c3 / c4 with their edge timings
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > gpurun_out/ck_edges.log 2>&1 || { tail -30 gpurun_out/ck_edges.log; exit 1; }
tail -1 gpurun_out/ck_edges.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ck_par.log 2>&1 || { tail -30 gpurun_out/ck_par.log; exit 1; }
tail -1 gpurun_out/ck_par.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_records.py tests/test_gpu_full.py -m gpu -x -q -k "c2w or records or edges" --timeout 500 --timeout-method thread > gpurun_out/ck_full.log 2>&1 || { tail -30 gpurun_out/ck_full.log; exit 1; }
tail -1 gpurun_out/ck_full.log
for c in ${CFGS:-c2w c2 c3 c4}; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --steps 10 > gpurun_out/ck_$c.json 2> gpurun_out/ck_$c.err || { tail -20 gpurun_out/ck_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ck_$c.json').read().strip().splitlines()[-1]); e=d.get('edge_summary',{}); print('$c', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()}, {k:round(v['avg_ms'],4) for k,v in e.items() if isinstance(v,dict)})"
done
