#!/bin/bash
# bench + rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes for one workload
# (CFG, default c2); one GPU call.  Outputs under gpurun_out/prof/.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof && export TMPDIR=/tmp
C=${CFG:-c2}
O=gpurun_out/prof
timeout -k 10 300 python3 bench.py --config $C > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
cat $O/bench_$C.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$C -o kt -- python3 bench.py --config $C --no-cpu-baseline > $O/kt_$C.log 2>&1 || { tail -20 $O/kt_$C.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$C -o f -- python3 bench.py --config $C --no-cpu-baseline --steps 5 --warmup 2 > $O/f_$C.log 2>&1 || { tail -20 $O/f_$C.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$C -o w -- python3 bench.py --config $C --no-cpu-baseline --steps 5 --warmup 2 > $O/w_$C.log 2>&1 || { tail -20 $O/w_$C.log; exit 1; }
echo profiled $C
