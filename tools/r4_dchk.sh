#!/bin/bash
# one GPU call: the bounds-checked stream kernel (lib_dchk.so) over the generated DEDUP /
# RoundSkip configs (codes vs the checker), then the parity + A/B script
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for c in c4_small c4_ref_skip phased_dedup many_rounds sorted_tiny_sets; do
  timeout -k 10 150 python -u tools/withlib.py agnes_amd/_exp/lib_dchk.so tools/diag_c4.py $c > gpurun_out/dchk_$c.log 2>&1 || { echo "FAIL $c"; tail -30 gpurun_out/dchk_$c.log; exit 1; }
  grep "violations\|mismatches" gpurun_out/dchk_$c.log
done
bash tools/r4_dflow.sh
