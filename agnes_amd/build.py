"""In-tree build of the HIP engine (hipcc, gfx950) — no JIT cache, the .so
travels with the repository snapshot to the GPU box.

Each source compiles to its own object under agnes_amd/_obj/ (in parallel, only
the stale ones), then one link."""
from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
OBJ = os.path.join(PKG_DIR, "_obj")
SOURCES = ["agnes_kernels.hip", "agnes_fast.hip", "agnes_sweep.hip", "agnes_flow.hip", "agnes_apply.hip",
           "agnes_edges.hip", "agnes_events.hip", "agnes_partials.hip", "agnes_fold.hip", "agnes_onesm.hip", "agnes_dedup.hip",
           "agnes_multi.hip", "agnes_valset.hip", "agnes_wire.hip", "agnes_api.cpp"]
HEADERS = ["agnes_device.h", "agnes_ed25519.h", "agnes_fast.h", "agnes_gen.h", "agnes_gen_host.h",
           "agnes_internal.h", "agnes_flow_chunks.inc", "../../include/agnes.h"]
OUT = os.path.join(PKG_DIR, "libagnes_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("AGNES_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}"]
LDFLAGS = ["-shared", "-fPIC", f"--offload-arch={ARCH}", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def _mtime(p: str) -> float:
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _obj(src: str) -> str:
    return os.path.join(OBJ, os.path.splitext(src)[0] + ".o")


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS + ["../build.py"])
    stale = [s for s in SOURCES
             if force or _mtime(_obj(s)) < max(hdr_t, _mtime(os.path.join(CSRC, s)))]

    def cc(src: str):
        cmd = [HIPCC] + CFLAGS + ["-c", "-o", _obj(src), os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        return r.stderr

    if stale:
        with ThreadPoolExecutor(max_workers=min(len(stale), max(1, (os.cpu_count() or 4)))) as ex:
            for msg in ex.map(cc, stale):
                if verbose and msg.strip():
                    print(msg)
    if stale or _mtime(OUT) < max(_mtime(_obj(s)) for s in SOURCES):
        cmd = [HIPCC] + LDFLAGS + ["-o", OUT] + [_obj(s) for s in SOURCES]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)
    return OUT


if __name__ == "__main__":
    import sys
    print(build(force="--force" in sys.argv, verbose=True))
