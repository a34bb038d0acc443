"""ClusterMath (cluster/src/main/java/io/scalecube/cluster/ClusterMath.java:8-136): exact integer
formulas at the BASELINE configs, host mirror == oracle, plus the BASELINE.md derived-constant table."""
import pytest

import oracle_py
from swimhip import cluster_math as cm

NS = [2, 3, 5, 10, 32, 50, 4096, 65536, 262144, 1048576]


@pytest.mark.parametrize("n", NS)
def test_ceil_log2_is_bit_length(n):
    assert cm.ceilLog2(n) == n.bit_length() == oracle_py.cluster_math(0, 0, n)


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("rm", [2, 3])
def test_spread_sweep(n, rm):
    assert cm.gossipPeriodsToSpread(rm, n) == oracle_py.cluster_math(1, rm, n) == rm * n.bit_length()
    assert cm.gossipPeriodsToSweep(rm, n) == oracle_py.cluster_math(2, rm, n) == 2 * (rm * n.bit_length() + 1)


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("mult", [3, 5, 6])
def test_suspicion(n, mult):
    assert cm.suspicionTimeout(mult, n, 1000) == 1000 * oracle_py.cluster_math(3, mult, n)


def test_baseline_table():
    # BASELINE.md "Derived protocol constants": (N, rm, mult) -> (bitlen, spread, sweep, suspicion)
    table = {
        (32, 2, 3): (6, 12, 26, 18),
        (4096, 3, 5): (13, 39, 80, 65),
        (65536, 3, 5): (17, 51, 104, 85),
        (262144, 3, 5): (19, 57, 116, 95),
        (1048576, 3, 5): (21, 63, 128, 105),
    }
    for (n, rm, mult), (b, sp, sw, su) in table.items():
        assert cm.ceilLog2(n) == b
        assert cm.gossipPeriodsToSpread(rm, n) == sp
        assert cm.gossipPeriodsToSweep(rm, n) == sw
        assert cm.suspicionTimeout(mult, n, 1) == su


def test_max_messages_and_timeouts():
    assert cm.maxMessagesPerGossipPerNode(3, 3, 50) == 3 * 3 * 6 == oracle_py.cluster_math(4, 3, 50, 3)
    assert cm.maxMessagesPerGossipTotal(3, 3, 50) == 50 * 54
    # GossipProtocolTest.java:119-120 timeout used by the reference's gossip experiments
    assert cm.gossipTimeoutToSweep(3, 50, 200) == 2 * (3 * 6 + 1) * 200
    assert cm.gossipDisseminationTime(3, 10, 200) == 3 * 4 * 200


def test_convergence_probability_monotone():
    p0 = cm.gossipConvergencePercent(3, 3, 50, 0)
    p50 = cm.gossipConvergencePercent(3, 3, 50, 50)
    assert 99.9 < p0 <= 100 and p50 < p0
