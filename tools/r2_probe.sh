#!/bin/bash
# round 2 baseline probe: kbench timing (normal / memory-only) + SQ counter passes on c2_plain
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/kbench.py --iters 10 --dbg 0,1 c2_plain c2_sm > gpurun_out/kb.log 2>&1 || { tail -30 gpurun_out/kb.log; exit 1; }
cat gpurun_out/kb.log
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python3 tools/kbench.py --iters 2 c2_plain > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
echo done
