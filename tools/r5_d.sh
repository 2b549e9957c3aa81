#!/bin/bash
# round-5 GPU call D: SQ counters of the flow variants on C2 (plain step, record counts, records, edges),
# then the queue-tail A/B and the flow timeline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sq5 && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf gpurun_out/sq5/c2_$i
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq5/c2_$i -o p -- python3 bench.py --config c2 --no-cpu-baseline --steps 3 --warmup 1 \
    > gpurun_out/sq5/c2_$i.log 2>&1 || { tail -20 gpurun_out/sq5/c2_$i.log; exit 1; }
done
python3 tools/pmc_by_kernel.py gpurun_out/sq5/c2_1 gpurun_out/sq5/c2_2 --sub=flow
bash tools/r5_b.sh
