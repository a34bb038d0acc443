"""MembershipRecordTest (cluster/src/test/java/io/scalecube/cluster/membership/MembershipRecordTest.java:15-109),
the reference's only bit-exact golden, against the oracle (CPU) and the gfx950 kernel (GPU)."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_py

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "membership_record_kat.json")))["rows"]


def test_kat_has_all_33_assertions():
    # 3 x 10 truth-table rows + 3 equal-record rows; the 34th assertion (different member ids
    # throw, :35-44) cannot be expressed: a packed cell is always about its own (observer, subject).
    assert len(KAT) == 33


@pytest.mark.parametrize("row", KAT, ids=[f"{r['test']}-{r['r0_name']}" for r in KAT])
def test_oracle_is_overrides(row):
    assert oracle_py.is_overrides(row["r1"], row["r0"]) == row["expected"]


def test_python_record_decode_roundtrip():
    from swimhip import MembershipRecord, native

    assert MembershipRecord.decode(3, native.pack(5, native.SUSPECT)) == MembershipRecord(3, "SUSPECT", 5)
    assert MembershipRecord.decode(3, 0) is None


@pytest.mark.gpu
def test_device_is_overrides_matches_kat():
    from swimhip import native

    lib = native.load_swimhip()
    r1 = np.array([r["r1"] for r in KAT], dtype=np.uint32)
    r0 = np.array([r["r0"] for r in KAT], dtype=np.uint32)
    out = np.zeros(len(KAT), dtype=np.uint8)
    P = ctypes.POINTER(ctypes.c_uint32)
    rc = lib.swim_kat_is_overrides(r1.ctypes.data_as(P), r0.ctypes.data_as(P),
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(KAT))
    assert rc == 0
    assert out.astype(bool).tolist() == [r["expected"] for r in KAT]


@pytest.mark.gpu
def test_device_is_overrides_exhaustive_small_lattice():
    """Every (r1, r0) over incarnations 0..63 x {ALIVE, SUSPECT} U {absent, DEAD}: device == oracle."""
    from swimhip import native

    lib = native.load_swimhip()
    cells = [0, 0xFFFFFFFF] + [(i << 2) | c for i in range(64) for c in (1, 2)]
    a = np.array([x for x in cells for _ in cells], dtype=np.uint32)
    b = np.array([y for _ in cells for y in cells], dtype=np.uint32)
    out = np.zeros(len(a), dtype=np.uint8)
    P = ctypes.POINTER(ctypes.c_uint32)
    assert lib.swim_kat_is_overrides(a.ctypes.data_as(P), b.ctypes.data_as(P),
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(a)) == 0
    ref = np.array([oracle_py.is_overrides(int(x), int(y)) for x, y in zip(a, b)], dtype=np.uint8)
    assert np.array_equal(out, ref)
