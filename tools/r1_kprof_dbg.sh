#!/bin/bash
# apply-pass cost split: per-kernel times of kbench under AGNES_DEBUG_SKIP values
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for d in ${DBGS:-0 16 32 48}; do
  echo "== AGNES_DEBUG_SKIP=$d"
  rm -rf gpurun_out/kprof
  AGNES_DEBUG_SKIP=$d timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o run -- python3 tools/kbench.py --iters 5 ${KB:-c2_sm} > gpurun_out/kprof.log 2>&1 || { tail -30 gpurun_out/kprof.log; exit 1; }
  f=$(find gpurun_out/kprof -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    if "gen_kernel" in r["Name"]: continue
    print(f'{int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:10.1f} us  {r["Name"][:90]}')
PY
done
