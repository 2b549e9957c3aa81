#!/usr/bin/env python3
"""Run a script against another build of the engine library (development A/B only).

    python tools/withlib.py agnes_amd/_exp/lib_base.so bench.py --config c2 ...

The product loader (agnes_amd/lib.py) always loads agnes_amd/libagnes_amd.so and
checks the ABI version; this tool points it at an experiment build (an older
commit's library may lack newer entry points: those are skipped, and its ABI
version is accepted) before the script imports the package."""
import ctypes as C
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) < 3:
    raise SystemExit(__doc__)
from agnes_amd import abi, lib  # noqa: E402

lib.LIB_PATH = os.path.join(ROOT, sys.argv[1])
_orig_cdll = C.CDLL


class _Tolerant:
    """the experiment library: missing symbols become AttributeError on use only"""

    def __init__(self, path):
        self._L = _orig_cdll(path)
        abi.ABI_VERSION = self._L.agnes_abi_version()  # accept the build's own ABI version

    def __getattr__(self, name):
        try:
            return getattr(self._L, name)
        except AttributeError:
            class _Missing:
                argtypes = restype = None

                def __call__(self, *a):
                    raise AttributeError(f"{name} not in {lib.LIB_PATH}")
            return _Missing()


lib.C = type("C", (), {k: getattr(C, k) for k in dir(C) if not k.startswith("__")})
lib.C.CDLL = _Tolerant  # (loaded by lib.load(): after the script imported torch and its HIP runtime)
script = sys.argv[2]
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
