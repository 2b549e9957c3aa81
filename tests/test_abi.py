"""CPU checks of the drop-in boundary: the engine library builds for gfx950,
loads, exports every function include/agnes.h declares, and its struct layout
matches the Python/ctypes mirror.  No compute calls (no GPU here)."""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi, build, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def so():
    build.build()
    return C.CDLL(lib.LIB_PATH)


def test_exports_every_declared_function(so):
    names = lib.header_functions()
    assert len(names) >= 18
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_loader_and_abi_version():
    L = lib.load()
    assert L.agnes_abi_version() == abi.ABI_VERSION


def test_struct_layout_matches_header():
    src = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "agnes.h"
    int main(void) {
      printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(agnes_vote), sizeof(agnes_event),
             sizeof(agnes_message), sizeof(agnes_state), sizeof(agnes_config),
             sizeof(agnes_vote_batch), sizeof(agnes_gen_params));
      printf("%zu %zu %zu %zu\n", offsetof(agnes_state, step), offsetof(agnes_state, decided),
             offsetof(agnes_vote_batch, n_votes), offsetof(agnes_message, kind));
      return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    sizes = list(map(int, out[:7]))
    assert sizes == [C.sizeof(abi.Vote), C.sizeof(abi.Event), C.sizeof(abi.Message),
                     C.sizeof(abi.StateRec), C.sizeof(abi.Config), C.sizeof(abi.VoteBatch),
                     C.sizeof(abi.GenParams)]
    offs = list(map(int, out[7:]))
    assert offs == [abi.StateRec.step.offset, abi.StateRec.decided.offset,
                    abi.VoteBatch.n_votes.offset, abi.Message.kind.offset]
    assert abi.STATE_DTYPE.fields["step"][1] == abi.StateRec.step.offset


@pytest.mark.skipif(torch.cuda.is_available(), reason="only meaningful without a GPU")
def test_no_gpu_means_no_engine():
    """No CPU fallback: without a device the engine refuses to run."""
    L = lib.load()
    h = C.c_void_p()
    assert L.agnes_ctx_create(0, C.byref(h)) == abi.E_NODEVICE
    assert L.agnes_ve_new(1, 4) is None


def test_host_generator_matches_checker_generator():
    """agnes_gen_offsets / agnes_gen_power (host helpers of the engine library)
    and the checker's copies compile the same header — same numbers."""
    L = lib.load()
    p = abi.gen_params(seed=77, n_instances=64, n_vals=33, rounds_min=1, rounds_max=4,
                       dup_permille=100, equiv_permille=50, higher_permille=50)
    off = np.zeros(65, np.uint64)
    assert L.agnes_gen_offsets(C.byref(p), off.ctypes.data) == 0
    assert (off == ol.gen_offsets(p)).all()
    pw = np.zeros((5, 33), np.int64)
    assert L.agnes_gen_power(5, 5, 33, abi.POWER_ZIPF, 1, 100000, pw.ctypes.data) == 0
    assert (pw == ol.gen_power(5, 5, 33, abi.POWER_ZIPF, 1, 100000)).all()


def test_lds_budget_query():
    L = lib.load()
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP, 5)
    b = L.agnes_lds_bytes_per_wave(C.byref(cfg), 150)
    assert 0 < b <= 36 * 1024
    big = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP, 256)
    assert L.agnes_lds_bytes_per_wave(C.byref(big), 1_000_000) == abi.E_UNSUPPORTED
