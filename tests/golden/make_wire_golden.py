#!/usr/bin/env python3
"""Make tests/golden/wire_ed25519.json: signed wire records and OpenSSL's verdicts.

Everything signature-related here is produced by the OpenSSL 3.0 command line
(`openssl pkeyutl -sign/-verify -rawin`, Ed25519), an implementation independent
of both the engine and oracle/ed25519_ref.py, so the fixture pins both:
  * RFC 8032 §7.1 TEST 2 (seed, public key, one-byte message, signature);
  * 8 validators with deterministic seeds, 48 wire records (include/agnes.h
    agnes_wire_vote) signed by OpenSSL;
  * tampered copies (a message bit, an R bit, an S bit, S + L, the wrong
    validator's key, a changed value) with OpenSSL's own verify verdict.
Run once in the build container (the GPU box does not run it):
    python tests/golden/make_wire_golden.py
"""
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import ed25519_ref as E  # noqa: E402  (only to build the record bytes)

PKCS8_PREFIX = bytes.fromhex("302e020100300506032b657004220420")
SPKI_PREFIX = bytes.fromhex("302a300506032b6570032100")


def _run(args, inp=None):
    return subprocess.run(args, input=inp, capture_output=True, check=False)


def ossl_pub(seed, d):
    k = os.path.join(d, "k.der")
    open(k, "wb").write(PKCS8_PREFIX + seed)
    r = _run(["openssl", "pkey", "-inform", "DER", "-in", k, "-pubout", "-outform", "DER"])
    assert r.returncode == 0, r.stderr
    return r.stdout[-32:]


def ossl_sign(seed, msg, d):
    k, m, s = (os.path.join(d, x) for x in ("k.der", "m.bin", "s.bin"))
    open(k, "wb").write(PKCS8_PREFIX + seed)
    open(m, "wb").write(msg)
    r = _run(["openssl", "pkeyutl", "-sign", "-keyform", "DER", "-inkey", k, "-rawin", "-in", m, "-out", s])
    assert r.returncode == 0, r.stderr
    return open(s, "rb").read()


def ossl_verify(pub, msg, sig, d):
    k, m, s = (os.path.join(d, x) for x in ("p.der", "m.bin", "s.bin"))
    open(k, "wb").write(SPKI_PREFIX + pub)
    open(m, "wb").write(msg)
    open(s, "wb").write(sig)
    r = _run(["openssl", "pkeyutl", "-verify", "-pubin", "-keyform", "DER", "-inkey", k, "-rawin",
              "-in", m, "-sigfile", s])
    return r.returncode == 0


def main():
    out = {"generator": "OpenSSL " + _run(["openssl", "version"]).stdout.decode().strip()}
    with tempfile.TemporaryDirectory() as d:
        # RFC 8032 §7.1 TEST 2 (TEST 1's message is empty, which this openssl CLI cannot sign)
        seed = bytes.fromhex("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb")
        pub = ossl_pub(seed, d)
        sig = ossl_sign(seed, b"\x72", d)
        out["rfc8032_test2"] = {"seed": seed.hex(), "pub": pub.hex(), "msg": "72", "sig": sig.hex()}

        n_vals, height = 8, 7
        seeds = [hashlib.sha512(b"agnes-wire-%d" % i).digest()[:32] for i in range(n_vals)]
        pubs = [ossl_pub(s, d) for s in seeds]
        out["n_vals"], out["height"] = n_vals, height
        out["seeds"] = [s.hex() for s in seeds]
        out["pubkeys"] = [p.hex() for p in pubs]
        recs, verdicts, kinds = [], [], []
        # 3 instances x 8 validators x prevote + precommit, values / nil mixed
        for inst in range(3):
            for typ in (0, 1):
                for v in range(n_vals):
                    value = E.NIL if (inst + v + typ) % 5 == 0 else 100 + inst
                    m = E.signed_bytes(inst, height, inst % 2, v, value, typ)
                    s = ossl_sign(seeds[v], m, d)
                    recs.append(m + s)
                    verdicts.append(ossl_verify(pubs[v], m, s, d))
                    kinds.append("signed")
        # tampered copies of the first 8 records, OpenSSL's verdict on each
        L = E.L
        for i in range(8):
            base = recs[i]
            m, s = base[:40], base[40:]
            v = struct.unpack_from("<I", m, 24)[0]
            cases = {
                "msg_bit": (bytes([m[0]]) + bytes([m[1] ^ 0x10]) + m[2:], s),
                "r_bit": (m, bytes([s[0] ^ 0x01]) + s[1:]),
                "s_bit": (m, s[:40] + bytes([s[40] ^ 0x04]) + s[41:]),
                "s_plus_l": (m, s[:32] + int.to_bytes(int.from_bytes(s[32:], "little") + L, 32, "little")),
                "value_changed": (m[:28] + struct.pack("<I", 999) + m[32:], s),
            }
            for name, (mm, ss) in cases.items():
                recs.append(mm + ss)
                verdicts.append(ossl_verify(pubs[v], mm, ss, d))
                kinds.append(name)
        # the right record checked against another validator's key: sign with seed[(v+1) % n]
        for i in range(4):
            m = E.signed_bytes(0, height, 0, i, 100, 0)
            s = ossl_sign(seeds[(i + 1) % n_vals], m, d)
            recs.append(m + s)
            verdicts.append(ossl_verify(pubs[i], m, s, d))
            kinds.append("wrong_key")
        out["records"] = [r.hex() for r in recs]
        out["openssl_verifies"] = verdicts
        out["kinds"] = kinds
    json.dump(out, open(os.path.join(HERE, "wire_ed25519.json"), "w"), indent=1)
    print("records", len(out["records"]), "accepted", sum(out["openssl_verifies"]))


if __name__ == "__main__":
    main()
