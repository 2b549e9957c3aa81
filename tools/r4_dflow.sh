#!/bin/bash
# one GPU call: GPU parity (not slow) with the stream kernel on the AUTO route (experiment
# build agnes_amd/_exp/lib_dflow.so), then the c4 step A/B: dflow vs its ALIAS variant vs
# the in-tree route (tally_fast + apply_codes)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u tools/withlib.py agnes_amd/_exp/lib_dflow.so tools/pytest_main.py tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread ${PYT:-} > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
LIBS=${LIBS:-"dflow=agnes_amd/_exp/lib_dflow.so alias=agnes_amd/_exp/lib_alias.so cur=-"} CFGS=${CFGS:-c4} REPS=${REPS:-2} bash tools/abn.sh
