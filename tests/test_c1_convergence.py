"""C1 (BASELINE configs[0]): periods-to-DEAD distribution of a 32-member local cluster after one
crash. CPU: the oracle's per-seed values against the committed fixture and ClusterMath's bounds.
GPU: libswimhip.so must give the same periods-to-DEAD as the oracle for every seed.

Regenerate the fixture (oracle only): `python tests/test_c1_convergence.py --regen`.
"""
import collections
import json
import os
import sys

import pytest

import convergence as cv
from oracle_py import OracleCluster

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1_periods_to_dead.json")
SEEDS = range(300)
GPU_SEEDS = range(64)


def _oracle(cfg, n, seed):
    return OracleCluster(cfg, n, seed, event_capacity=1 << 16)


def _gpu(cfg, n, seed):
    from swimhip import SwimCluster

    return SwimCluster(cfg, n, seed, event_capacity=1 << 16)


def _fixture():
    with open(FIXTURE) as f:
        return json.load(f)


def test_oracle_matches_c1_fixture():
    fx = _fixture()
    got = [cv.periods_to_dead(_oracle, s)[0] for s in SEEDS]
    assert got == fx["periods_to_dead"]


def test_c1_distribution_within_clustermath_bounds():
    """Every survivor needs the 18-period suspicion timer (ClusterMath.java:123-125) plus at least
    the detecting probe's period; with 10 gossip rounds per period and fanout 3, SUSPECT reaches
    all 31 survivors within a period or two, so the tail is short."""
    d = _fixture()["periods_to_dead"]
    susp = cv.suspicion_periods()
    assert susp == 18
    assert min(d) >= susp + 1
    assert max(d) <= susp + 8
    hist = collections.Counter(d)
    # the direct probe of a crashed member by one of 31 round-robin observers lands in the first
    # period for most seeds: the mode is the earliest possible value
    assert hist.most_common(1)[0][0] == susp + 1


@pytest.mark.gpu
def test_gpu_c1_periods_to_dead_match_oracle():
    fx = _fixture()["periods_to_dead"]
    got = [cv.periods_to_dead(_gpu, s)[0] for s in GPU_SEEDS]
    assert got == fx[: len(got)]


if __name__ == "__main__" and "--regen" in sys.argv:
    d = [cv.periods_to_dead(_oracle, s)[0] for s in SEEDS]
    with open(FIXTURE, "w") as f:
        json.dump({"config": "C1: 32 members, defaultLocalConfig, crash at t0=10 of "
                             "np.random.default_rng(seed).integers(32)", "seeds": [SEEDS.start, SEEDS.stop],
                   "periods_to_dead": d, "histogram": dict(sorted(collections.Counter(d).items()))}, f)
        f.write("\n")
