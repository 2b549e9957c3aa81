"""In-tree build of the HIP engine (hipcc, gfx950) — no JIT cache, the .so
travels with the repository snapshot to the GPU box."""
from __future__ import annotations

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
SOURCES = ["agnes_kernels.hip", "agnes_fast.hip", "agnes_sweep.hip", "agnes_flow.hip", "agnes_apply.hip", "agnes_edges.hip", "agnes_events.hip", "agnes_fold.hip", "agnes_onesm.hip", "agnes_dedup.hip", "agnes_multi.hip", "agnes_valset.hip", "agnes_wire.hip", "agnes_api.cpp"]
HEADERS = ["agnes_device.h", "agnes_ed25519.h", "agnes_fast.h", "agnes_gen.h", "agnes_gen_host.h", "agnes_internal.h", "../../include/agnes.h"]
OUT = os.path.join(PKG_DIR, "libagnes_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("AGNES_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + HEADERS + ["../build.py"]
    return any(os.path.getmtime(os.path.join(CSRC, d)) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if force or _stale():
        cmd = [HIPCC] + FLAGS + ["-o", OUT] + [os.path.join(CSRC, s) for s in SOURCES]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=CSRC)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
