"""Wire format + Ed25519 ingest (include/agnes.h agnes_wire_ingest).

The reference has no wire format or signature check (README.md:8-14, 36-41), so
parity is anchored on an independent implementation of the published algorithm:
tests/golden/wire_ed25519.json holds keys, signed records and OpenSSL 3.0's own
verify verdicts (tests/golden/make_wire_golden.py).  The checker
oracle/ed25519_ref.py (RFC 8032 restated with Python integers) is pinned to those
verdicts and signatures and to RFC 8032 §7.1 TESTs 1 and 2; the GPU kernel is then
compared with the checker on the fixtures, on edge cases of the record format,
at 92k records, and end to end through agnes_tally.
"""
import json
import os
import struct

import numpy as np
import pytest

from oracle import ed25519_ref as E

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "wire_ed25519.json")))
PUBS = [bytes.fromhex(p) for p in G["pubkeys"]]
RECS = [bytes.fromhex(r) for r in G["records"]]
HEIGHT = G["height"]


def _validator(r):
    return struct.unpack_from("<I", r, 24)[0]


# ---------------- the checker, pinned (CPU) ----------------

def test_rfc8032_vectors():
    t = G["rfc8032_test2"]  # made by OpenSSL
    seed = bytes.fromhex(t["seed"])
    assert E.public_key(seed).hex() == t["pub"]
    assert E.sign(seed, bytes.fromhex(t["msg"])).hex() == t["sig"]
    assert E.verify(bytes.fromhex(t["pub"]), bytes.fromhex(t["msg"]), bytes.fromhex(t["sig"]))
    # RFC 8032 §7.1 TEST 1 (empty message), from the RFC text
    s1 = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    assert E.public_key(s1).hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    assert E.sign(s1, b"").hex() == (
        "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd"
        "25bf5f0595bbe24655141438e7a100b")


def test_checker_matches_openssl_verdicts():
    assert len(RECS) == len(G["openssl_verifies"]) == 92
    for r, ok, kind in zip(RECS, G["openssl_verifies"], G["kinds"]):
        assert E.verify(PUBS[_validator(r)], r[:40], r[40:]) == ok, kind
    assert sum(G["openssl_verifies"]) == 48  # every untampered record, no tampered one


def test_checker_reproduces_openssl_signatures():
    """RFC 8032 signatures are deterministic: same seed and message, same bytes."""
    for r, kind in zip(RECS, G["kinds"]):
        if kind == "signed":
            assert E.sign(bytes.fromhex(G["seeds"][_validator(r)]), r[:40]) == r[40:]


def test_checker_ingest_format_rules():
    r = RECS[0]
    keys = b"".join(PUBS)
    cases = {
        "ok": (r, E.OK),
        "magic": (b"\0" + r[1:], E.BAD_FORMAT),
        "type2": (r[:32] + b"\x02" + r[33:], E.BAD_FORMAT),
        "pad": (r[:39] + b"\x01" + r[40:], E.BAD_FORMAT),
        "round_high": (r[:16] + struct.pack("<q", 4) + r[24:], E.BAD_FORMAT),
        "round_neg": (r[:16] + struct.pack("<q", -1) + r[24:], E.BAD_FORMAT),
        "height": (r[:8] + struct.pack("<q", HEIGHT + 1) + r[16:], E.BAD_HEIGHT),
        "validator": (r[:24] + struct.pack("<I", 8) + r[28:], E.BAD_VALIDATOR),
        "sig": (r[:40] + bytes(64), E.BAD_SIGNATURE),
    }
    for name, (rec, want) in cases.items():
        out = E.ingest(rec, keys, 1, 8, HEIGHT, max_rounds=4)
        assert out["verdict"] == [want], name
        assert out["type"][0] == (r[32] if want == E.OK else 0xFF), name


# ---------------- the engine on the GPU ----------------

def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from agnes_amd.engine import Engine
    return torch, Engine(0)


def _run(eng, torch, recs, pubs, n_sets, n_vals, height, max_rounds, instance_set=None, offsets=None):
    dev = eng.device
    rt = torch.from_numpy(np.frombuffer(b"".join(recs), dtype=np.uint8).reshape(-1, 104).copy()).to(dev)
    kt = torch.from_numpy(np.frombuffer(b"".join(pubs), dtype=np.uint8).copy()).to(dev)
    if offsets is None:
        offsets = torch.tensor([0, len(recs)], dtype=torch.int64, device=dev)
    iset = None if instance_set is None else torch.tensor(instance_set, dtype=torch.int32, device=dev)
    b, verdict = eng.wire_ingest(rt, kt, n_sets, n_vals, height, max_rounds, offsets, iset)
    torch.cuda.synchronize()
    h = b.to_host()
    return b, verdict.cpu().numpy(), {k: np.asarray(h[k][: len(recs)]) for k in
                                      ("instance", "round", "type", "value", "validator")}


def _expect(recs, pubs, n_sets, n_vals, height, max_rounds, instance_set=None):
    return E.ingest(b"".join(recs), b"".join(pubs), n_sets, n_vals, height, instance_set, max_rounds)


def _compare(got_v, cols, want):
    assert np.array_equal(got_v, np.array(want["verdict"], dtype=np.uint8))
    for k in ("instance", "round", "type", "value", "validator"):
        assert np.array_equal(cols[k].astype(np.uint64), np.array(want[k], dtype=np.uint64)), k


@pytest.mark.gpu
def test_gpu_fixture_verdicts_equal_openssl():
    torch, eng = _engine()
    _, v, cols = _run(eng, torch, RECS, PUBS, 1, 8, HEIGHT, 4)
    ok = v == E.OK
    sig_ok = np.array(G["openssl_verifies"])
    # the record format rejects some tampered records first (a changed magic byte)
    assert np.array_equal(ok, sig_ok)
    _compare(v, cols, _expect(RECS, PUBS, 1, 8, HEIGHT, 4))
    eng.close()


@pytest.mark.gpu
def test_gpu_format_edges_and_sets():
    torch, eng = _engine()
    r = RECS[0]
    recs = [r, b"\0" + r[1:], r[:32] + b"\x02" + r[33:], r[:39] + b"\x01" + r[40:],
            r[:16] + struct.pack("<q", 4) + r[24:], r[:16] + struct.pack("<q", -1) + r[24:],
            r[:8] + struct.pack("<q", HEIGHT + 1) + r[16:], r[:24] + struct.pack("<I", 8) + r[28:],
            r[:40] + bytes(64), r[:72] + bytes([r[72] ^ 0x80]) + r[73:],
            r[:40] + r[40:72] + bytes([0xFF] * 32)]
    _, v, cols = _run(eng, torch, recs, PUBS, 1, 8, HEIGHT, 4)
    _compare(v, cols, _expect(recs, PUBS, 1, 8, HEIGHT, 4))
    # two sets: set 1 holds the keys in reverse, instance_set maps the fixture's
    # instances 0..2 to sets 0, 1, 0 -> instance 1's records check against the wrong keys
    pubs2 = PUBS + PUBS[::-1]
    _, v, cols = _run(eng, torch, RECS[:48], pubs2, 2, 8, HEIGHT, 4, instance_set=[0, 1, 0])
    want = _expect(RECS[:48], pubs2, 2, 8, HEIGHT, 4, instance_set=[0, 1, 0])
    _compare(v, cols, want)
    assert want["verdict"][16:32].count(E.BAD_SIGNATURE) == 16 and want["verdict"][:16].count(E.OK) == 16
    # an instance outside instance_set, and no set at all
    _, v, cols = _run(eng, torch, RECS[:48], pubs2, 2, 8, HEIGHT, 4, instance_set=[0])
    _compare(v, cols, _expect(RECS[:48], pubs2, 2, 8, HEIGHT, 4, instance_set=[0]))
    _, v, _ = _run(eng, torch, RECS[:4], PUBS, 0, 8, HEIGHT, 4)
    assert (v == E.BAD_VALIDATOR).all()
    eng.close()


@pytest.mark.gpu
def test_gpu_many_records():
    """92k records (the fixture x 1000): every lane and block of a large grid."""
    torch, eng = _engine()
    rep = 1000
    _, v, cols = _run(eng, torch, RECS * rep, PUBS, 1, 8, HEIGHT, 4)
    want = _expect(RECS, PUBS, 1, 8, HEIGHT, 4)
    assert np.array_equal(v, np.tile(np.array(want["verdict"], dtype=np.uint8), rep))
    assert np.array_equal(cols["type"], np.tile(np.array(want["type"], dtype=np.uint8), rep))
    eng.close()


@pytest.mark.gpu
def test_gpu_ingest_then_tally():
    """wire records -> agnes_wire_ingest -> agnes_tally: codes equal the checker's
    tally of the decoded columns; a record whose signature fails is coded INVALID."""
    torch, eng = _engine()
    import oracle_lib as ol
    from agnes_amd import abi
    from agnes_amd.engine import states_to_device, states_to_host
    recs = list(RECS[:48])
    # tamper one signature in each instance
    for i in (3, 20, 40):
        recs[i] = recs[i][:100] + bytes([recs[i][100] ^ 1]) + recs[i][101:]
    offsets = torch.tensor([0, 16, 32, 48], dtype=torch.int64, device=eng.device)
    b, v, cols = _run(eng, torch, recs, PUBS, 1, 8, HEIGHT, 4, offsets=offsets)
    assert (v[[3, 20, 40]] == E.BAD_SIGNATURE).all() and (np.delete(v, [3, 20, 40]) == E.OK).all()
    power = np.ones((1, 8), dtype=np.int64)
    eng.upload_power(power)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)
    st0 = abi.new_states(3, HEIGHT, abi.STEP_PREVOTE)
    codes = torch.zeros(48, dtype=torch.uint8, device=eng.device)
    dst = states_to_device(st0, eng.device)
    eng.tally(cfg, b, codes, dst)
    torch.cuda.synchronize()

    hb = ol.batch_from_lists(cols["instance"], cols["round"], cols["type"], cols["value"], cols["validator"],
                             [0, 16, 32, 48])
    o_codes, o_states, _ = ol.tally(cfg, hb, power, None, st0)
    g = codes.cpu().numpy()
    assert np.array_equal(g, o_codes)
    assert (g[[3, 20, 40]] == abi.CODE_INVALID).all()
    assert states_to_host(dst).tobytes() == o_states.tobytes()
    eng.close()
