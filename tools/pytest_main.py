#!/usr/bin/env python3
"""pytest as a script (development A/B only): `python tools/withlib.py <lib.so>
tools/pytest_main.py tests/... -k ...` runs the GPU tests against an experiment build."""
import sys

import pytest

sys.exit(pytest.main(sys.argv[1:]))
