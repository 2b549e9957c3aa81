#!/bin/bash
# kbench with development knobs (no tests)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/dbg.log
for d in ${DBGS:-0 1}; do
  echo "== AGNES_DEBUG_SKIP=$d ${EXTRA:-}" >> gpurun_out/dbg.log
  AGNES_DEBUG_SKIP=$d timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-c2_plain} >> gpurun_out/dbg.log 2>&1 || { cat gpurun_out/dbg.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/dbg.log
