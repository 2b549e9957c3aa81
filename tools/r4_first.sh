#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_partials.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -2 gpurun_out/r4a_tests.log
for c in c4 c3shard c2w c3; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 > gpurun_out/r4a_bench_$c.json 2> gpurun_out/r4a_bench_$c.err || { tail -20 gpurun_out/r4a_bench_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4a_bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('path_frac'), d.get('cpu_check_equal'), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
