#!/bin/bash
# r2_profile.sh over every bench config, one GPU call (outputs under gpurun_out/prof/)
cd "$GRAFT_REPO_ROOT" || exit 1
for c in ${CFGS:-c2 c3 c4 c5 c5d}; do
  CFG=$c bash tools/r2_profile.sh > gpurun_out/prof_$c.log 2>&1 || { echo "profile $c failed"; tail -20 gpurun_out/prof_$c.log; exit 1; }
  echo "profiled $c"
done
