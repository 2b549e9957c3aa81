#!/bin/bash
# one GPU call: the records / edges GPU parity tests, then per workload (CFGS) the step, the
# fused records and edges calls and the round-4 edge walks (ms per call)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" --timeout 200 --timeout-method thread -k "edges or tally_events" > gpurun_out/r5/tests_f.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r5/tests_f.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for c in ${CFGS:-c2 c3}; do
timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r5/f_$c.json 2> gpurun_out/r5/f_$c.err || { tail -20 gpurun_out/r5/f_$c.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r5/f_$c.json').read().strip().splitlines()[-1])
e=d['event_stream']; g=d['edge_summary']
print('$c', round(d['ms_per_step'],4), 'events', round(e['tally_events']['ms_per_call'],4), 'records', round(e['tally_records']['ms_per_call'],4), round(e['tally_records']['records_ms'],4), e['tally_records']['compacted_equal_to_two_call_stream'], 'edges', round(g['tally_edges']['ms_per_call'],4), round(g['tally_edges']['edges_ms'],4), g['tally_edges']['compacted_equal_to_two_call_summary'], 'old edges', round(g['edge_count']['avg_ms']+g['edge_scan']['avg_ms']+g['edge_emit']['avg_ms'],4))
"
done
