#!/usr/bin/env python3
"""pytest as a script (for tools/withlib.py: the GPU tests against an experiment build)."""
import sys

import pytest

sys.exit(pytest.main(sys.argv[1:]))
