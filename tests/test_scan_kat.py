"""The wave and block scans every compaction, commit offset and list build rests on
(`wave_excl_scan`: DPP row shifts + GFX9 row broadcasts; `block_excl_scan1024`), checked on the
device against numpy prefix sums (`swim_kat_scan`). No reference counterpart: these are the
build's own primitives; the parity suites cover them only indirectly."""
import ctypes

import numpy as np
import pytest


def _host_scans(x):
    w = x.reshape(-1, 64).astype(np.uint64)
    b = x.reshape(-1, 1024).astype(np.uint64)
    wex = (np.cumsum(w, axis=1) - w).astype(np.uint32).ravel()
    bex = (np.cumsum(b, axis=1) - b).astype(np.uint32).ravel()
    return wex, w.sum(axis=1).astype(np.uint32), bex, b.sum(axis=1).astype(np.uint32)


def test_host_reference_scans_are_prefix_sums():
    x = np.arange(2048, dtype=np.uint32)
    wex, wt, bex, bt = _host_scans(x)
    assert wex[64] == 0 and wex[65] == 64 and wt[0] == sum(range(64))
    assert bex[1025] == 1024 and bt[1] == sum(range(1024, 2048))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bits", "small", "wide", "sparse"])
def test_device_wave_and_block_scans(kind):
    from swimhip import _native as nat

    lib = nat.load_swimhip()
    rng = np.random.default_rng(7)
    n = 1024 * 37
    x = {"bits": rng.integers(0, 2, n), "small": rng.integers(0, 33, n),
         "wide": rng.integers(0, 1 << 20, n), "sparse": (rng.random(n) < 0.01) * rng.integers(1, 5000, n)}[kind]
    x = np.ascontiguousarray(x.astype(np.uint32))
    wex = np.zeros(n, np.uint32)
    wt = np.zeros(n // 64, np.uint32)
    bex = np.zeros(n, np.uint32)
    bt = np.zeros(n // 1024, np.uint32)
    P = ctypes.POINTER(ctypes.c_uint32)
    rc = lib.swim_kat_scan(x.ctypes.data_as(P), n, wex.ctypes.data_as(P), wt.ctypes.data_as(P),
                           bex.ctypes.data_as(P), bt.ctypes.data_as(P))
    assert rc == 0
    hw, hwt, hb, hbt = _host_scans(x)
    assert np.array_equal(wex, hw)
    assert np.array_equal(wt, hwt)
    assert np.array_equal(bex, hb)
    assert np.array_equal(bt, hbt)


def test_scan_kat_rejects_ragged_sizes():
    import torch

    if torch.cuda.is_available():
        pytest.skip("the size check is exercised without a device")
    from swimhip import _native as nat

    lib = nat.load_swimhip()
    x = np.zeros(1000, np.uint32)
    P = ctypes.POINTER(ctypes.c_uint32)
    assert lib.swim_kat_scan(x.ctypes.data_as(P), 1000, x.ctypes.data_as(P), x.ctypes.data_as(P),
                             x.ctypes.data_as(P), x.ctypes.data_as(P)) == nat.SWIM_EINVAL
