#!/bin/bash
# one GPU call: the u64-sum route (tally_fast<W64>) — generated parity, the full-size c2w
# parity, then the c2w and c2 bench lines
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/w64_tests.log 2>&1 || { tail -30 gpurun_out/w64_tests.log; exit 1; }
tail -2 gpurun_out/w64_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q -k c2w --timeout 500 --timeout-method thread > gpurun_out/w64_full.log 2>&1 || { tail -30 gpurun_out/w64_full.log; exit 1; }
tail -2 gpurun_out/w64_full.log
for c in c2w c2; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/w64_$c.json 2> gpurun_out/w64_$c.err || { tail -20 gpurun_out/w64_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/w64_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], round(d['ms_per_step'],4), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
