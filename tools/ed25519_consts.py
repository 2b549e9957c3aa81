#!/usr/bin/env python3
"""Limb constants of agnes_amd/csrc/agnes_ed25519.h (radix 2^25.5, ten limbs)."""
P = 2**255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)
OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
W = [26 if i % 2 == 0 else 25 for i in range(10)]


def limbs(x):
    return [(x >> OFF[i]) & ((1 << W[i]) - 1) for i in range(10)]


for name, x in (("d", D), ("2d", 2 * D % P), ("sqrtm1", SQRT_M1)):
    print(name, ", ".join(str(v) for v in limbs(x)))

# the base point B (y = 4/5, x even), extended coordinates with Z = 1
import sys
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
from oracle import ed25519_ref as E  # noqa: E402
bx, by = E.B[0] % P, E.B[1] % P
for name, x in (("bx", bx), ("by", by), ("bt", bx * by % P)):
    print(name, ", ".join(str(v) for v in limbs(x)))
