"""The C CPU port (oracle/c/blsport.c, the bench's cpu_baseline) against the golden fixtures.
Test infrastructure checking test infrastructure: keeps the CPU baseline honest."""
import ctypes
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "fixtures.json")))


@pytest.fixture(scope="module")
def lib():
    from oracle import cpu_baseline
    return cpu_baseline.load()


def _aff(lib, pk48):
    out = ctypes.create_string_buffer(96)
    assert lib.port_g1_decompress(pk48, out) == 0
    return out.raw


def test_port_same_message_fixtures(lib):
    pks = [bytes.fromhex(p) for p in FIX["keys"]["pks"]]
    cases = FIX["same_message"]
    off, pk_aff, sigs, msgs, exp = [0], b"", b"", b"", []
    for c in cases:
        for i, s in zip(c["indices"], c["sigs"]):
            pk_aff += _aff(lib, pks[i])
            sigs += bytes.fromhex(s)
        off.append(off[-1] + len(c["indices"]))
        msgs += bytes.fromhex(c["msg"])
        exp.extend(c["expected"])
    n = off[-1]
    valid = (ctypes.c_uint8 * n)()
    o = np.array(off, dtype=np.uint32)
    lib.port_verify_same_message_batch(3, len(cases), o.ctypes.data, pk_aff, sigs, msgs, valid, 7)
    assert [bool(x) for x in valid] == exp


def test_port_verify_single(lib):
    for c in FIX["verify_sets"]:
        if c["name"] in ("single_valid", "single_invalid"):
            s = c["sets"][0]
            pk = bytes.fromhex(FIX["keys"]["pks"][s["indices"][0]])
            assert bool(lib.port_verify(pk, bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]))) == c["expected"]


def test_port_hash_to_g2(lib):
    for c in FIX["hash_to_g2"]:
        out = ctypes.create_string_buffer(192)
        lib.port_hash_to_g2(bytes.fromhex(c["msg"]), out)
        assert out.raw.hex() == c["expected"]


def test_port_verify_sets_c4_block(lib):
    """The port's verifySignatureSets (cpu_baseline of C1/C3/C4) on the oracle's C4 block fixture:
    the clean block true, every corruption false (one call each, pool shape, 4 workers)."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import c4_block as C
    from oracle import block_oracle as BO
    from oracle import cpu_baseline
    fix = C.load()
    rows = cpu_baseline.affine_rows(lib, [bytes.fromhex(p) for p in fix["pubkeys"]])
    extra = []

    def to_call(sets):
        call = []
        for kind, key, root, sig in sets:
            if kind == "raw":
                extra.append(key)
                call.append(([C.N_KEYS + len(extra) - 1], root, sig))
            elif kind == "single":
                call.append(([key % C.N_KEYS], root, sig))
            else:
                call.append(([v % C.N_KEYS for v in key], root, sig))
        return call
    calls = [to_call(BO.block_signature_sets(fix))]
    for kind in C.CORRUPTIONS:
        b2, com2, _ = C.corrupt(fix, kind)
        calls.append(to_call(BO.block_signature_sets(fix, b2, com2)))
    rows += cpu_baseline.affine_rows(lib, extra)
    res, _ = cpu_baseline.run_verify_sets(lib, calls, rows, threads=4)
    assert res == [True] + [False] * len(C.CORRUPTIONS)
    # empty call false, as verifySignatureSetsMaybeBatch([])
    assert cpu_baseline.run_verify_sets(lib, [[]], rows)[0] == [False]
