#!/bin/bash
# round-5 GPU call C: the non-slow GPU suite (records, edges, W64 rounds, RCCL check, queue tail), the c2
# line with the records / edges, then the A/B of call B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" --timeout 200 --timeout-method thread > gpurun_out/r5/tests_c.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r5/tests_c.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/r5/b_c2.json 2> gpurun_out/r5/b_c2.err || { tail -20 gpurun_out/r5/b_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r5/b_c2.json').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'], d['roofline'].get('frac'), json.dumps(d['event_stream']['tally_events'])[:300]); print(json.dumps(d['event_stream']['tally_records'])[:600]); print(json.dumps(d['edge_summary'])[:900])"
bash tools/r5_b.sh
