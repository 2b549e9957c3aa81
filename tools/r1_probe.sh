#!/bin/bash
# round-1 probe: gpu tests, kernel bench, SQ counters of the c2 tally kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u tools/kbench.py --iters 10 > gpurun_out/kbench.log 2>&1 || { cat gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_sq1 -o sq1 --output-format csv -- python3 tools/kbench.py c2_sm --iters 2 > gpurun_out/pmc_sq1.log 2>&1 || { tail -20 gpurun_out/pmc_sq1.log; exit 1; }
echo PMC1 done
