#!/bin/bash
# round-5 GPU call A: the C4 ceiling micro-bench, the new W64 / multi parity tests, c2w / c3w lines
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
timeout -k 10 300 python3 tools/kbench.py c4_full c4_dedup_sm c4_skip_sm c4_ref_z c4_ref_u c4_ref_u_noh c3shard --iters 10 > gpurun_out/r5/ceil.jsonl 2> gpurun_out/r5/ceil.err || { tail -20 gpurun_out/r5/ceil.err; exit 1; }
cat gpurun_out/r5/ceil.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "multi or w64 or c3w or c2w or routes" > gpurun_out/r5/tests_a.log 2>&1 || { tail -30 gpurun_out/r5/tests_a.log; exit 1; }
tail -2 gpurun_out/r5/tests_a.log
for c in c2w c3w; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r5/b_$c.json 2> gpurun_out/r5/b_$c.err || { tail -20 gpurun_out/r5/b_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5/b_$c.json').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('path_frac'), {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
timeout -k 10 300 python3 tools/flowdiag.py agnes_amd/_exp/lib_diag.so c3shard c3 c2 > gpurun_out/r5/flowdiag.jsonl 2> gpurun_out/r5/flowdiag.err || { tail -20 gpurun_out/r5/flowdiag.err; exit 1; }
cut -c1-600 gpurun_out/r5/flowdiag.jsonl
