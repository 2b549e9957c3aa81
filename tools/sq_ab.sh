#!/bin/bash
# one GPU call: SQ counters of the bench step's kernels for several library builds (LIBS="name=path", "-" = in-tree)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CNT=${CNT:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"}
for spec in ${LIBS:-new=-}; do
  name=${spec%%=*}; path=${spec#*=}
  if [ "$path" = "-" ]; then run="python3 bench.py"; else run="python3 tools/withlib.py $path bench.py"; fi
  rm -rf gpurun_out/sq_$name
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/sq_$name -o sq -- $run --config ${CFG:-c4} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_$name.log 2>&1 || { tail -20 gpurun_out/sq_$name.log; exit 1; }
  echo "== $name"; python3 tools/pmc_sum.py gpurun_out/sq_$name "${KSUB:-}" | head -12
done
