#!/bin/bash
# kbench over the ablation builds of tools/ablate.py (one GPU call)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in ${VARS:-base nomulti nophase2 nosm noroles novalid nostore}; do
  echo "== $v"
  AGNES_LIB=agnes_amd/_exp/lib_$v.so timeout -k 10 120 python -u tools/kbench.py --iters 10 ${KB:-c2_plain c2_sm} 2>/dev/null | python3 -c "import sys,json; [print('  %-10s %.4f ms' % (d['variant'], d['kernel_ms'])) for d in map(json.loads, sys.stdin)]" || exit 1
done
