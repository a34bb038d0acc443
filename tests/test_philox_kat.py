"""Philox4x32-10 pinned to its published algorithm: the Random123 known-answer vectors
(Salmon et al., SC'11; Random123 kat_vectors, philox4x32_10) for the oracle (CPU) and the
device (gfx950, `swim_kat_philox4`). Every random choice on the path (ping targets, proxies,
gossip peers, SYNC peers, loss draws) is drawn from this generator, keyed as
key = {seed_lo ^ kind * 0x9E3779B9, seed_hi}, counter = {a, b, c, tick} (swim_rng.h); with
kind = 0 the key is the seed itself, so the vectors apply unchanged."""
import ctypes

import numpy as np
import pytest

import oracle_py

# (counter, key {k0, k1}) -> output; Random123 philox4x32_10 known answers
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
]


def seed_of(key):
    return key[0] | (key[1] << 32)


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_oracle_philox_random123_kat(ctr, key, want):
    assert oracle_py.philox4(seed_of(key), 0, *ctr) == list(want)
    assert oracle_py.philox(seed_of(key), 0, *ctr) == want[0]


@pytest.mark.gpu
def test_device_philox_random123_kat():
    from swimhip import native

    lib = native.load_swimhip()
    abct = np.array([k[0] for k in KAT], dtype=np.uint32)
    P = ctypes.POINTER(ctypes.c_uint32)
    for i, (ctr, key, want) in enumerate(KAT):
        out = np.zeros(4, dtype=np.uint32)
        assert lib.swim_kat_philox4(seed_of(key), 0, abct[i:i + 1].ctypes.data_as(P), out.ctypes.data_as(P), 1) == 0
        assert out.tolist() == list(want)
