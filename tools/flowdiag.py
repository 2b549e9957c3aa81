#!/usr/bin/env python3
"""Per-wave timeline of the flow kernel (development diagnostics, round 5):

    python tools/buildvar.py diag -DAGNES_FLOW_DIAG      # agnes_amd/_exp/lib_diag.so
    python tools/flowdiag.py agnes_amd/_exp/lib_diag.so c3shard c3 [--out DIR]

Loads the diagnostics build (every flow wave writes s_memrealtime at its start, at
each batch start and at its end, plus each batch's instances / chunks / votes), runs
one tally of each workload and prints, per workload, one JSON line: the kernel's
span, how the waves' end times spread (the tail), the per-wave busy fraction, batch
and chunk counts, and the chunk fill (votes / (512 x chunks)).  The raw records go to
DIR/<workload>_flowdiag.npz."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agnes_amd import abi, lib  # noqa: E402

WORKLOADS = {
    "c3shard": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
    "c3": (dict(n_instances=1_000_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
           (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
    "c2": (dict(n_instances=1_000_000, n_vals=100, nil_permille=200),
           (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1),
}
MAXW = 256 * 64  # waves the buffer covers (256 CUs x 16 blocks x 4 waves at most)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("workloads", nargs="+")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r5"))
    args = ap.parse_args()
    lib.LIB_PATH = os.path.join(ROOT, args.lib)
    from agnes_amd.engine import Engine, states_to_device  # noqa: E402
    eng = Engine(0)
    arm = C.CDLL(lib.LIB_PATH).agnes_flow_diag_arm
    arm.argtypes, arm.restype = [C.c_void_p], C.c_int
    buf = torch.zeros(MAXW * 64, dtype=torch.int64, device=eng.device)
    assert arm(buf.data_ptr()) == 0
    os.makedirs(args.out, exist_ok=True)
    for name in args.workloads:
        gp, (kind, lo, hi, n_sets), mode, flags, R = WORKLOADS[name]
        p = abi.gen_params(seed=0xA6E5, **gp)
        eng.upload_power(eng.gen_power(0xA6E5, n_sets, p.n_vals, kind, lo, hi))
        b = eng.gen_batch(p)
        cfg = abi.config(mode, flags, R)
        st0 = states_to_device(abi.new_states(p.n_instances, 1, abi.STEP_PREVOTE), eng.device)
        st = torch.empty_like(st0)
        codes = torch.empty(b.n_votes, dtype=torch.uint8, device=eng.device)
        for _ in range(3):
            st.copy_(st0)
            buf.zero_()
            eng.tally(cfg, b, codes, st)
        torch.cuda.synchronize()
        d = buf.view(MAXW, 64).cpu().numpy().astype(np.uint64)
        live = d[:, 0] != 0
        w = d[live]
        t0 = w[:, 0].min()
        start = (w[:, 0] - t0) / 100.0  # us (100 MHz)
        end = (w[:, 1] - t0) / 100.0
        span = float(end.max())
        nb = w[:, 2].astype(np.int64)
        nc = w[:, 3].astype(np.int64)
        recs = []
        for i in range(len(w)):
            for k in range(min(int(nb[i]), 30)):
                x = int(w[i, 5 + 2 * k])
                recs.append((i, (int(w[i, 4 + 2 * k]) - int(t0)) / 100.0, x & 0xFFFF, (x >> 16) & 0xFFFF, x >> 32))
        recs = np.array(recs, dtype=np.float64) if recs else np.zeros((0, 5))
        votes = float(recs[:, 4].sum()) if len(recs) else 0.0
        chunks = float(nc.sum())
        busy = (end - start) / span
        q = np.percentile(end, [0, 10, 50, 90, 99, 100])
        out = dict(workload=name, waves=int(live.sum()), span_us=span,
                   start_us_max=float(start.max()),
                   end_us_pct={"min": q[0], "p10": q[1], "p50": q[2], "p90": q[3], "p99": q[4], "max": q[5]},
                   mean_busy_frac=float(busy.mean()), idle_tail_frac=float(1.0 - busy.mean()),
                   batches=int(nb.sum()), batches_per_wave={"min": int(nb.min()), "mean": float(nb.mean()),
                                                            "max": int(nb.max())},
                   chunks=int(chunks), chunks_per_wave={"min": int(nc.min()), "mean": float(nc.mean()),
                                                        "max": int(nc.max())},
                   votes=votes, chunk_fill=votes / (512.0 * chunks) if chunks else None,
                   us_per_chunk_wave=float(np.mean((end - start) / np.maximum(nc, 1))),
                   batch_instances_mean=float(recs[:, 2].mean()) if len(recs) else None)
        hist, edges = np.histogram(end, bins=20, range=(0.0, span))
        out["end_hist_us"] = {"edges": [round(float(e), 1) for e in edges], "counts": hist.tolist()}
        print(json.dumps(out), flush=True)
        np.savez_compressed(os.path.join(args.out, f"{name}_flowdiag.npz"), waves=w, batches=recs)
        del b, codes, st, st0
        torch.cuda.empty_cache()
    arm(None)


if __name__ == "__main__":
    main()
