#!/bin/bash
# SQ instruction counters of one kernel (KN substring) per kbench variant, two --pmc passes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sq && export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVES"
P2="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for k in ${KB:-c4_full}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq/$k.$i -o sq -- python3 tools/kbench.py --iters 1 $k > gpurun_out/sq/$k.$i.log 2>&1 || { tail -5 gpurun_out/sq/$k.$i.log; exit 1; }
  done
done
KN="${KN:-tally_fast}" python3 - <<'PY'
import csv, glob, collections, os
kn = os.environ["KN"].split(",")
for f in sorted(glob.glob("gpurun_out/sq/*/**/sq_counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if not any(k in r["Kernel_Name"] for k in kn): continue
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:50]
    for d_id in list(acc)[-2:]:
        print(f.split("/")[2], names[d_id], {k: int(v) for k, v in sorted(acc[d_id].items())})
PY
