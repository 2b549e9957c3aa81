#!/bin/bash
# one GPU call: GPU parity (not slow) with the stream kernel on the AUTO route (experiment
# build agnes_amd/_exp/lib_dflow.so), then A/B: c4 (dflow vs ALIAS vs in-tree route),
# c3shard (batch-size heuristics), and the c2w line (i64 stakes)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
[ -n "${NOPAR:-}" ] || timeout -k 10 700 python -u tools/withlib.py agnes_amd/_exp/lib_dflow.so tools/pytest_main.py tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread ${PYT:-} > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
[ -n "${NOPAR:-}" ] || tail -3 gpurun_out/r4b_tests.log
LIBS="dflow=agnes_amd/_exp/lib_dflow.so alias=agnes_amd/_exp/lib_alias.so cur=-" CFGS=c4 REPS=2 bash tools/abn.sh || exit 1
LIBS="cur=- bpw4=agnes_amd/_exp/lib_bpw4.so bpw8=agnes_amd/_exp/lib_bpw8.so" CFGS=c3shard REPS=1 bash tools/abn.sh || exit 1
timeout -k 10 200 python3 bench.py --config c2w --no-cpu-baseline --steps 5 > gpurun_out/r4b_c2w.json 2> gpurun_out/r4b_c2w.err || { tail -20 gpurun_out/r4b_c2w.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4b_c2w.json').read().strip().splitlines()[-1]); print('c2w', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
