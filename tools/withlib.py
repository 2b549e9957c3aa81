#!/usr/bin/env python3
"""Run a script against another build of the engine library (development A/B only).

    python tools/withlib.py agnes_amd/_exp/lib_base.so bench.py --config c2 ...

The product loader (agnes_amd/lib.py) always loads agnes_amd/libagnes_amd.so; this
tool points it at an experiment build before the script imports the package."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) < 3:
    raise SystemExit(__doc__)
from agnes_amd import lib  # noqa: E402

lib.LIB_PATH = os.path.join(ROOT, sys.argv[1])
script = sys.argv[2]
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
