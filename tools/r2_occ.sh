#!/bin/bash
# kernel trace (grid size, VGPR, LDS, scratch) of the flow kernel per ablation build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/occ && export TMPDIR=/tmp
for v in ${VARS:-base w4}; do
  AGNES_LIB=agnes_amd/_exp/lib_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/occ/$v -o kt -- python3 tools/kbench.py --iters 2 ${KB:-c2_sm} > gpurun_out/occ/$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/occ/*/**/kt_kernel_trace.csv", recursive=True)):
    seen = set()
    for r in csv.DictReader(open(f)):
        if "flow::flow" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"][:40], r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Arch_VGPR_Count"), r.get("LDS_Block_Size", r.get("Lds_Size")), r.get("Scratch_Size"))
        if key in seen:
            continue
        seen.add(key)
        print(f.split("/")[2], {k: r[k] for k in r if any(x in k for x in ("Grid", "VGPR", "SGPR", "LDS", "Lds", "Scratch", "Workgroup"))})
PY
