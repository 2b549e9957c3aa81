#!/bin/bash
# round-5 GPU call E: edges v2 / records / flow parity, then A/B of the look-ahead, tail and XWPE variants
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" --timeout 200 --timeout-method thread -k "edges or tally_events or routes or generated or full_records" > gpurun_out/r5/tests_e.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r5/tests_e.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/flowdiag.py agnes_amd/_exp/lib_diag.so c3shard c3 > gpurun_out/r5/flowdiag_a1.jsonl 2> gpurun_out/r5/flowdiag_a1.err || { tail -20 gpurun_out/r5/flowdiag_a1.err; exit 1; }
cut -c1-300 gpurun_out/r5/flowdiag_a1.jsonl
LIBS="new=- ahead2=agnes_amd/_exp/lib_ahead2.so a1t1024=agnes_amd/_exp/lib_a1t1024.so xwpe2=agnes_amd/_exp/lib_xwpe2.so" CFGS="c3shard c3 c2" REPS=2 bash tools/abn.sh
python3 -c "import json; d=json.loads(open('gpurun_out/abn_new_c2.json').read().strip().splitlines()[-1]); print(json.dumps(d['edge_summary'].get('tally_edges'))[:500])"
python3 -c "import json; d=json.loads(open('gpurun_out/abn_xwpe2_c2.json').read().strip().splitlines()[-1]); print(json.dumps(d['edge_summary'].get('tally_edges'))[:500]); print(json.dumps(d['event_stream'].get('tally_records'))[:300])"
