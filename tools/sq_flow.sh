#!/bin/bash
# one GPU call: SQ counters of the flow variants of one workload (CFG, default c2): the step, the
# record counts, the records and the edges (KS: ";"-separated kernel-name substrings)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
CNT=${CNT:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU"}
rm -rf gpurun_out/r5/sq_${CFG:-c2}
timeout -s KILL 150 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/r5/sq_${CFG:-c2} -o sq -- python3 bench.py --config ${CFG:-c2} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5/sq_${CFG:-c2}.log 2>&1 || { tail -20 gpurun_out/r5/sq_${CFG:-c2}.log; exit 1; }
IFS=";" read -ra KS <<< "${KS:-false, false, false, false>;true, false, false, false>;true, false, true, false>;true, false, false, true>}"
for k in "${KS[@]}"; do
  echo "== $k"; python3 tools/pmc_sum.py gpurun_out/r5/sq_${CFG:-c2} "$k" | head -9
done
