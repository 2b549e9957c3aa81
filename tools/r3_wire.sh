#!/bin/bash
# wire config: bench line + rocprofv3 kernel trace (one GPU call)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof && export TMPDIR=/tmp
O=gpurun_out/prof
timeout -k 10 300 python3 bench.py --config wire > $O/bench_wire.json 2> $O/bench_wire.err || { tail -20 $O/bench_wire.err; exit 1; }
cat $O/bench_wire.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_wire -o kt -- python3 bench.py --config wire --no-cpu-baseline > $O/kt_wire.log 2>&1 || { tail -20 $O/kt_wire.log; exit 1; }
echo profiled
