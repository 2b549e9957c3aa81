#!/bin/bash
# kbench per experiment library (AGNES_LIB) and stream setting; no tests
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/libs.log
for L in ${LIBS:-default}; do
  for st in ${STREAMS:-1}; do
    if [ "$L" = default ]; then unset AGNES_LIB; else export AGNES_LIB=$L; fi
    echo "== lib $L stream $st" >> gpurun_out/libs.log
    AGNES_STREAM=$st timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-c2_sm} >> gpurun_out/libs.log 2>&1 || { cat gpurun_out/libs.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/libs.log | sed 's/"instances.*"kernel_ms"/"kernel_ms"/; s/, "votes_per_s.*//'
