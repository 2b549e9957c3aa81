"""The reference's unit tests restated in C++ over include/agnes.hpp.

CPU: the mirror header compiles (g++, C++17) and links against the engine
library.  GPU: the binary runs the tests on the device."""
import os
import subprocess

import pytest

from agnes_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "reference_tests.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "reference_tests")


def _compile():
    lib = build.build()
    libdir = os.path.dirname(lib)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", EXE, "-L", libdir, "-lagnes_amd", f"-Wl,-rpath,{libdir}"], check=True)
    return EXE


def test_cpp_mirror_compiles_and_links():
    assert os.path.exists(_compile())


@pytest.mark.gpu
def test_reference_tests_on_gpu():
    exe = _compile()
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "reference tests: ok" in out.stdout
