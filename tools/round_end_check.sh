#!/bin/bash
# one GPU call, the driver's round-end order: every -m gpu test, smoke(), the default bench line
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fc_tests.log 2>&1 || { tail -30 gpurun_out/fc_tests.log; exit 1; }
tail -2 gpurun_out/fc_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { tail -20 gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/fc_bench.json 2> gpurun_out/fc_bench.err || { tail -20 gpurun_out/fc_bench.err; exit 1; }
tail -c 400 gpurun_out/fc_bench.json
