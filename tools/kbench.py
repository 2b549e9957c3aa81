#!/usr/bin/env python3
"""Kernel micro-bench: times agnes_tally on several workload/flag variants in one
process (HIP events on the launch stream) and prints one JSON line per variant.
Development tool; the headline number is bench.py's."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agnes_amd import abi  # noqa: E402
from agnes_amd.engine import Engine, states_to_device  # noqa: E402

VARIANTS = {
    "c2_plain": (dict(n_instances=1_000_000, n_vals=100, nil_permille=200),
                 (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE, 0, 1),
    "c2_sm": (dict(n_instances=1_000_000, n_vals=100, nil_permille=200),
              (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1),
    "c2_sm_commit": (dict(n_instances=1_000_000, n_vals=100, nil_permille=200),
                     (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE,
                     abi.FLAG_STATE_MACHINE, 1),
    "c2_sm_phased": (dict(n_instances=1_000_000, n_vals=100, nil_permille=200,
                          order=abi.ORDER_PHASED),
                     (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE,
                     abi.FLAG_STATE_MACHINE, 1),
    "c3_sm": (dict(n_instances=250_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
              (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
    "c3_1set": (dict(n_instances=250_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                (abi.POWER_UNIFORM, 1, 1000, 1), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
    "c3_r1": (dict(n_instances=625_000, n_vals=150, rounds_min=1, rounds_max=1, nil_permille=300),
              (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
    "c3_r1only": (dict(n_instances=625_000, n_vals=150, rounds_min=1, rounds_max=1, nil_permille=300),
                  (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1),
    "c4_full": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                     nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50),
                (abi.POWER_ZIPF, 1, 1_000_000, 1024), abi.MODE_DEDUP,
                abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 5),
    "c4_dedup_only": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                           nil_permille=300, dup_permille=100, equiv_permille=100),
                      (abi.POWER_ZIPF, 1, 1_000_000, 1024), abi.MODE_DEDUP, 0, 5),
    # round-5 C4 ceiling: the C4 stream (dup/equiv/next-round votes) tallied in REFERENCE mode
    # without RoundSkip, powers inside flow's domain (maxpow < 4096)
    "c4_ref_u": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                      nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50),
                 (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5),
    "c4_ref_u_noh": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                          nil_permille=300, dup_permille=100, equiv_permille=100),
                     (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5),
    "c4_ref_z": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                      nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50),
                 (abi.POWER_ZIPF, 1, 1_000_000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5),
    "c4_dedup_sm": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                         nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50),
                    (abi.POWER_ZIPF, 1, 1_000_000, 1024), abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE, 5),
    "c4_skip_sm": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                        nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50),
                   (abi.POWER_ZIPF, 1, 1_000_000, 1024), abi.MODE_REFERENCE,
                   abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 5),
    "c3shard": (dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                (abi.POWER_UNIFORM, 1, 1000, 1024), abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4),
}


def run(eng, name, iters):
    gp, (kind, lo, hi, n_sets), mode, flags, R = VARIANTS[name]
    p = abi.gen_params(seed=0xA6E5, **gp)
    eng.upload_power(eng.gen_power(0xA6E5, n_sets, p.n_vals, kind, lo, hi))
    b = eng.gen_batch(p)
    cfg = abi.config(mode, flags, R)
    step0 = abi.STEP_COMMIT if name.endswith("_commit") else abi.STEP_PREVOTE
    st0 = states_to_device(abi.new_states(p.n_instances, 1, step0), eng.device)
    st = torch.empty_like(st0)
    codes = torch.empty(b.n_votes, dtype=torch.uint8, device=eng.device)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        st.copy_(st0)
        eng.tally(cfg, b, codes, st, stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        st.copy_(st0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.tally(cfg, b, codes, st, stream)
        e1.record(stream)
        ts.append((e0, e1))
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(c) for a, c in ts]))
    gbs = 15 * b.n_votes / (ms * 1e-3) / 1e9
    out = dict(variant=name, votes=b.n_votes, instances=p.n_instances, kernel_ms=ms,
               votes_per_s=b.n_votes / (ms * 1e-3), algo_GBps=gbs, frac=gbs / 8000.0,
               lds_per_wave=eng.lds_bytes_per_wave(cfg))
    print(json.dumps(out), flush=True)
    del b, codes, st, st0
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=list(VARIANTS))
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    eng = Engine(0)
    for v in args.variants:
        run(eng, v, args.iters)


if __name__ == "__main__":
    main()
