#!/bin/bash
# one GPU call: GPU parity of the in-tree build (PAR: pytest -k expression, or "all"), then the A/B bench
# (LIBS / CFGS / REPS as tools/abn.sh)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
K=(); if [ "${PAR:-all}" != "all" ]; then K=(-k "$PAR"); fi
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread "${K[@]}" > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
bash tools/abn.sh
