"""CPU checker for the wire-format ingest — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker; the product path (agnes_amd/csrc/agnes_wire.hip) never
imports or calls it.

The reference has no wire format and no signature check: its README
(/root/reference/README.md:8-14, 36-41) leaves "signature validation" and "the
structure of data sent on the wire" to the consumer, and `Validator` holds the
public key the votes would be checked against (src/validators.rs:4-8, 15-17:
address() = public_key).  So this module restates a published algorithm, not
reference code:

* Ed25519 verification, RFC 8032 §5.1.7, in the cofactorless form OpenSSL 3.0
  implements (crypto/ec/curve25519.c ED25519_verify): reject S >= L, decode A
  (RFC 8032 §5.1.3; reject a point that does not decode), k = SHA-512(R || A ||
  M) mod L, accept iff encode([S]B - [k]A) == R byte for byte.
* Ed25519 signing, RFC 8032 §5.1.6 (deterministic), to cross-check the fixtures.

Parity pin: tests/golden/wire_ed25519.json holds keys, messages and signatures
made by the OpenSSL 3.0.2 command line (tests/golden/make_wire_golden.py), plus
tampered copies; this module must accept exactly the untampered ones and
reproduce OpenSSL's signatures bit for bit (RFC 8032 signatures are
deterministic).

The 104-byte wire record (include/agnes.h agnes_wire_vote), little-endian:
  0 magic u32 "AGV1" | 4 instance u32 | 8 height i64 | 16 round i64 |
  24 validator u32 | 28 value u32 (0xFFFFFFFF = nil) | 32 type u8 | 33 pad[7] = 0 |
  40 signature R || S (64 B) over bytes 0..39.
"""
from __future__ import annotations

import hashlib
import struct

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

MAGIC = 0x31564741  # "AGV1"
WIRE_BYTES = 104
SIGNED_BYTES = 40
NIL = 0xFFFFFFFF

# verdicts (include/agnes.h AGNES_WIRE_*)
OK, BAD_FORMAT, BAD_VALIDATOR, BAD_SIGNATURE, BAD_HEIGHT = 0, 1, 2, 3, 4


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


# points in extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, x*y = T/Z
def _add(p, q):
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * t1 * t2 * D % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _mul(s: int, p):
    q = (0, 1, 1, 0)
    while s > 0:
        if s & 1:
            q = _add(q, p)
        p = _add(p, p)
        s >>= 1
    return q


def _encode(p) -> bytes:
    x, y, z, _ = p
    zi = _inv(z)
    x, y = x * zi % P, y * zi % P
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


def _recover_x(y: int, sign: int):
    """RFC 8032 §5.1.3 steps 2-4; None when no x exists."""
    if y >= P:
        return None
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    if (v * x * x - u) % P == 0:
        pass
    elif (v * x * x + u) % P == 0:
        x = x * SQRT_M1 % P
    else:
        return None
    if x == 0 and sign:
        return None
    if (x & 1) != sign:
        x = P - x
    return x


def decode(s: bytes):
    y = int.from_bytes(s, "little")
    sign = y >> 255
    y &= (1 << 255) - 1
    x = _recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, x * y % P)


_BY = 4 * _inv(5) % P
B = (_recover_x(_BY, 0), _BY, 1, _recover_x(_BY, 0) * _BY % P)


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    if len(pub) != 32 or len(sig) != 64:
        return False
    r, s = sig[:32], int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    a = decode(pub)
    if a is None:
        return False
    k = int.from_bytes(hashlib.sha512(r + pub + msg).digest(), "little") % L
    neg_a = ((P - a[0]) % P, a[1], a[2], (P - a[3]) % P)
    return _encode(_add(_mul(s, B), _mul(k, neg_a))) == r


def public_key(seed: bytes) -> bytes:
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return _encode(_mul(a, B))


def sign(seed: bytes, msg: bytes) -> bytes:
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    pub = _encode(_mul(a, B))
    r = int.from_bytes(hashlib.sha512(h[32:] + msg).digest(), "little") % L
    rb = _encode(_mul(r, B))
    k = int.from_bytes(hashlib.sha512(rb + pub + msg).digest(), "little") % L
    return rb + int.to_bytes((r + k * a) % L, 32, "little")


# ---- the wire record ----

def signed_bytes(instance: int, height: int, round_: int, validator: int, value: int, typ: int) -> bytes:
    return struct.pack("<IIqqIIB7x", MAGIC, instance, height, round_, validator, value, typ)


def record(seed: bytes, instance: int, height: int, round_: int, validator: int, value: int, typ: int) -> bytes:
    m = signed_bytes(instance, height, round_, validator, value, typ)
    return m + sign(seed, m)


def ingest(records: bytes, pubkeys: bytes, n_sets: int, n_vals: int, height: int,
           instance_set=None, max_rounds: int = 256):
    """The checker's decode + verify of n 104-byte records.  Returns (verdict u8[n],
    instance u32[n], round u8[n], type u8[n], value u32[n], validator u32[n]); a
    record that fails gets type 0xFF (the tally then codes it INVALID) and round 0.
    pubkeys: n_sets * n_vals * 32 bytes, set-major (the validator addresses,
    validators.rs:15-17).  instance_set None: set = instance % n_sets."""
    n = len(records) // WIRE_BYTES
    out = {k: [] for k in ("verdict", "instance", "round", "type", "value", "validator")}
    for i in range(n):
        rec = records[i * WIRE_BYTES:(i + 1) * WIRE_BYTES]
        magic, inst, h, rnd, val, value, typ = struct.unpack_from("<IIqqIIB", rec, 0)
        pad = rec[33:40]
        verdict = OK
        if magic != MAGIC or typ > 1 or any(pad) or rnd < 0 or rnd >= max_rounds:
            verdict = BAD_FORMAT
        elif h != height:
            verdict = BAD_HEIGHT
        else:
            s = (instance_set[inst] if instance_set is not None and inst < len(instance_set)
                 else (inst % n_sets if n_sets else 0))
            if instance_set is not None and inst >= len(instance_set):
                verdict = BAD_VALIDATOR
            elif s >= n_sets or val >= n_vals:
                verdict = BAD_VALIDATOR
            else:
                pk = pubkeys[(s * n_vals + val) * 32:(s * n_vals + val + 1) * 32]
                if not verify(pk, rec[:SIGNED_BYTES], rec[SIGNED_BYTES:]):
                    verdict = BAD_SIGNATURE
        out["verdict"].append(verdict)
        out["instance"].append(inst)
        out["round"].append(rnd & 0xFF if verdict == OK else 0)
        out["type"].append(typ if verdict == OK else 0xFF)
        out["value"].append(value)
        out["validator"].append(val)
    return out
