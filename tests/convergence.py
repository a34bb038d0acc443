"""BASELINE config 1: 32 members, `ClusterConfig.defaultLocalConfig()`,
converged start, one member killed at t0 = 10 without a leave gossip, run until every survivor
has emitted REMOVED for it. The measured quantity is periods-to-DEAD per seed.

Reference shape: `MembershipProtocolTest.java:935-983` (cluster of local configs over the
NetworkEmulator) and the suspicion timer `MembershipProtocolImpl.java:620-647` with
`ClusterMath.suspicionTimeout` (`core/ClusterMath.java:123-125`): 3 · bit_length(32) = 18 periods
at pingInterval 1 s. The periods-to-DEAD distribution of the unmodified reactive reference needs
a JVM (absent here), so the per-seed values are pinned GPU vs oracle and the
oracle's distribution is checked against ClusterMath's analytic bounds.
"""
from __future__ import annotations

import numpy as np

from swimhip import ClusterConfig, cluster_math

N = 32
T0 = 10
MAX_PERIODS = 80


def victim(seed: int) -> int:
    return int(np.random.default_rng(seed).integers(N))


def suspicion_periods() -> int:
    cfg = ClusterConfig.defaultLocalConfig()
    mult = cfg.membershipConfig().suspicionMult()
    return cluster_math.suspicionTimeout(mult, N, 1000) // 1000


def periods_to_dead(make, seed: int):
    """Run C1 for one seed; return (periods from the crash until the last survivor's REMOVED,
    first REMOVED period offset). `make(cfg, n, seed)` builds a SwimCluster or OracleCluster."""
    c = make(ClusterConfig.defaultLocalConfig(), N, seed)
    c.step(T0)
    list(c.events())
    v = victim(seed)
    c.crash([v])
    removed = set()
    first = None
    for t in range(1, MAX_PERIODS + 1):
        c.step(1)
        for e in c.events():
            if e.isRemoved() and e.member == v:
                removed.add(e.observer)
                first = t if first is None else first
        if len(removed) == N - 1:
            return t, first
    raise AssertionError(f"seed {seed}: only {len(removed)} of {N - 1} survivors removed member {v}")
