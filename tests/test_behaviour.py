"""Reference test assertions (FailureDetectorTest, MembershipProtocolTest, GossipProtocolTest)
restated on the discrete replay (tests/behaviour.py), run on the CPU oracle and on the GPU."""
import pytest

import behaviour
from oracle_py import OracleCluster


def _oracle(cfg, n, seed, **kw):
    return OracleCluster(cfg, n, seed, event_capacity=1 << 16, **kw)


def _gpu(cfg, n, seed, **kw):
    from swimhip import SwimCluster

    return SwimCluster(cfg, n, seed, event_capacity=1 << 16, **kw)


@pytest.mark.parametrize("case", behaviour.ALL, ids=[f.__name__ for f in behaviour.ALL])
def test_oracle_behaviour(case):
    case(_oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("case", behaviour.ALL, ids=[f.__name__ for f in behaviour.ALL])
def test_gpu_behaviour(case):
    case(_gpu)
