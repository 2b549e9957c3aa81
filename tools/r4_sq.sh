#!/bin/bash
# one GPU call: SQ instruction / cycle counters of the C4 step, for the stream kernel
# (experiment build) and the in-tree route; summaries printed per kernel
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sq && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"
for spec in ${LIBS:-cur=-}; do
  name=${spec%%=*}; path=${spec#*=}
  if [ "$path" = "-" ]; then run="python3 bench.py"; else run="python3 tools/withlib.py $path bench.py"; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1)); rm -rf gpurun_out/sq/${name}_${CFG:-c4}_$i
    timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq/${name}_${CFG:-c4}_$i -o p -- $run --config ${CFG:-c4} --no-cpu-baseline --steps 3 --warmup 1 \
      > gpurun_out/sq/${name}_${CFG:-c4}_$i.log 2>&1 || { tail -20 gpurun_out/sq/${name}_${CFG:-c4}_$i.log; exit 1; }
  done
  echo "== $name"; python3 tools/pmc_sum.py gpurun_out/sq/${name}_${CFG:-c4}_1 "${KSUB:-}" ; python3 tools/pmc_sum.py gpurun_out/sq/${name}_${CFG:-c4}_2 "${KSUB:-}"
done
