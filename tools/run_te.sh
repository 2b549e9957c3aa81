cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tally_events.py tests/test_gpu_events.py -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > gpurun_out/te_tests.log 2>&1 || { tail -40 gpurun_out/te_tests.log; exit 1; }
tail -3 gpurun_out/te_tests.log
LIBS="new=-" REPS=2 bash tools/abn.sh
