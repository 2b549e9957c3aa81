#!/bin/bash
# gpu tests, then kbench per fast-kernel variant and stream setting (separate
# processes: the launcher caches its choice)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
fi
: > gpurun_out/sweep.log
for st in ${STREAMS:-1}; do
  export AGNES_STREAM=$st
  for v in ${VARIANTS:-auto}; do
    if [ "$v" = auto ]; then unset AGNES_FAST_VARIANT; else export AGNES_FAST_VARIANT=$v; fi
    echo "== stream $st variant $v bpc ${AGNES_BLOCKS_PER_CU:-}" >> gpurun_out/sweep.log
    timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-} >> gpurun_out/sweep.log 2>&1 || { cat gpurun_out/sweep.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/sweep.log
