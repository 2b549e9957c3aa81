#!/bin/bash
# SQ counter passes + kernel stats over tools/kbench.py variants (one rocprofv3 run per pass)
O=${OUT:-gpurun_out/pmc}
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o p$i --output-format csv -- python3 tools/kbench.py --iters 2 ${KB:-c2_sm} > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/kbench.py --iters 5 ${KB:-c2_sm} > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
