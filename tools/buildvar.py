#!/usr/bin/env python3
"""Build an experiment variant of the engine library (development A/B only):

    python tools/buildvar.py NAME -DFOO [-DBAR=1 ...]   -> agnes_amd/_exp/lib_NAME.so

Same sources and flags as agnes_amd/build.py plus the given defines; objects under
agnes_amd/_exp/NAME/.  Load it with tools/withlib.py."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agnes_amd import build as b  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
od = os.path.join(ROOT, "agnes_amd", "_exp", name)
os.makedirs(od, exist_ok=True)


def cc(src):
    o = os.path.join(od, os.path.splitext(src)[0] + ".o")
    subprocess.run([b.HIPCC] + b.CFLAGS + defs + ["-c", "-o", o, os.path.join(b.CSRC, src)], check=True, cwd=b.CSRC)
    return o


with ThreadPoolExecutor(max_workers=8) as ex:
    objs = list(ex.map(cc, b.SOURCES))
out = os.path.join(ROOT, "agnes_amd", "_exp", f"lib_{name}.so")
subprocess.run([b.HIPCC] + b.LDFLAGS + ["-o", out] + objs, check=True, cwd=b.CSRC)
print(out)
