#!/bin/bash
# flow-kernel change check (one GPU call): GPU parity (all -m gpu tests, or TESTS), then
# kbench of the in-tree library against the saved base build.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_tests.log 2>&1 || { tail -30 gpurun_out/r3_tests.log; exit 1; }
tail -3 gpurun_out/r3_tests.log
for v in ${VARS:-base}; do
  echo "== $v"
  AGNES_LIB=agnes_amd/_exp/lib_$v.so timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-c2_sm c3_sm} 2>/dev/null | python3 -c "import sys,json; [print('  %-10s %.4f ms' % (d['variant'], d['kernel_ms'])) for d in map(json.loads, sys.stdin)]" || exit 1
done
echo "== new"
timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-c2_sm c3_sm} 2>/dev/null | python3 -c "import sys,json; [print('  %-10s %.4f ms' % (d['variant'], d['kernel_ms'])) for d in map(json.loads, sys.stdin)]"
