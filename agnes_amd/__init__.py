"""agnes_amd — MI355X-native batch engine for Agnes's vote-tally hot path.

Importing the package loads no native code; the HIP engine library
(agnes_amd/libagnes_amd.so) is loaded on first use and its absence is an error:
there is no CPU fallback.
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
