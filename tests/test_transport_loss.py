"""TransportTest.testNetworkSettings (transport-parent/transport-netty/src/test/java/io/scalecube/
transport/netty/TransportTest.java:111-133) restated on the simulator's loss model.

The reference sends 1,000 messages client -> server through a NetworkEmulator set to 50 % outbound
loss (NetworkEmulator.evaluateLoss, cluster-testlib/.../NetworkEmulator.java:348-351: lost iff
nextInt(100) < lossPercent) and asserts that fewer than 550 arrive (50 % + 5 % slack). The
simulator draws one Philox value per directed message: a message is lost iff
draw < loss_bp * 2^32 / 10^4. The same 1,000 messages are drawn here — message k of the pair
(client, server) keyed by (kind, client, server, k, tick) — on the oracle (CPU) and on the device
(`swim_kat_philox`, bit-exact with the oracle), and checked against the reference's bound for
every seed, plus a binomial check of the loss rate over all seeds pooled.
"""
import ctypes
import math

import numpy as np
import pytest

import oracle_py

K_GOSSIP = 7  # swim_rng.h: the kind of a GossipRequest (any kind gives the same statistics)
CLIENT, SERVER = 0, 1
TOTAL = 1000
LOSS_PCT = 50
SEEDS = range(32)


def _thr(loss_pct):
    return ((loss_pct * 100) << 32) // 10000  # loss in basis points, as swim_set_loss


def _counters(tick=3):
    return np.array([[CLIENT, SERVER, k, tick] for k in range(TOTAL)], dtype=np.uint32)


def _delivered(draws):
    return int(np.count_nonzero(np.asarray(draws, dtype=np.uint64) >= _thr(LOSS_PCT)))


def _expected_max():
    return TOTAL // 100 * LOSS_PCT + TOTAL // 100 * 5  # TransportTest.java:128-129


def test_oracle_loss_within_reference_bound():
    ctr = _counters()
    pooled = 0
    for seed in SEEDS:
        d = [oracle_py.philox(seed, K_GOSSIP, *map(int, c)) for c in ctr]
        got = _delivered(d)
        assert got < _expected_max(), (seed, got)  # TransportTest.java:130-131
        pooled += got
    # pooled over seeds: a binomial(n, 1/2) count within 4 standard deviations of n/2
    n = TOTAL * len(SEEDS)
    assert abs(pooled - n / 2) < 4 * math.sqrt(n / 4), pooled


@pytest.mark.gpu
def test_device_loss_draws_match_oracle_and_bound():
    from swimhip import native

    lib = native.load_swimhip()
    ctr = _counters()
    P = ctypes.POINTER(ctypes.c_uint32)
    for seed in SEEDS[:8]:
        out = np.zeros(TOTAL, dtype=np.uint32)
        assert lib.swim_kat_philox(seed, K_GOSSIP, ctr.ctypes.data_as(P), out.ctypes.data_as(P), TOTAL) == 0
        ref = [oracle_py.philox(seed, K_GOSSIP, *map(int, c)) for c in ctr]
        assert out.tolist() == ref
        assert _delivered(out) < _expected_max()
