"""Quiet periods: the library skips the gossip rounds of a period in which no member
holds a gossip (k_quiet_check after the FD commit; one k_quiet_rounds launch instead of ~15 per round).
A/B against handles created with SWIMHIP_QUIET=0, which always run their rounds: every parity counter,
event, digest, membership and deadline table equal, period by period, and the protocol-level work counters
that are exact run to run, through quiet stretches, storms, joins and restarts, and the return to quiet.
The oracle parity file runs with the skip on as well (it is the default)."""
import os

import numpy as np
import pytest

import scenarios
from swimhip import ClusterConfig, SwimCluster

pytestmark = pytest.mark.gpu


def _make(flag):
    def make(cfg, n, seed, **kw):
        old = os.environ.get("SWIMHIP_QUIET")
        os.environ["SWIMHIP_QUIET"] = flag  # read once, by swim_create
        try:
            return SwimCluster(cfg, n, seed, **kw)
        finally:
            if old is None:
                del os.environ["SWIMHIP_QUIET"]
            else:
                os.environ["SWIMHIP_QUIET"] = old
    return make


# protocol-level counters beyond the parity keys: exact run to run. (The kernels' own work counters are
# not: gossips with equal commit sort keys take ring slots in the order their stage entries were claimed
# by atomics, slot order being unobservable, and run tops, record ranges, list words,
# pull probes and merge-mark skips follow the slots; two runs of the same always-running handle differ in
# them.)
EXACT = list(scenarios.PARITY_KEYS) + ["sweep_cells", "merge_cells", "ack_cells"]


@pytest.mark.parametrize("name", ["c1_local32_crash", "lan256_loss5_crash3", "local128_partition_heal",
                                  "local40_restart_join", "local64_update_metadata", "local64_user_gossips_loss10",
                                  "local32_leave2"])
def test_quiet_skip_matches_full_rounds(name):
    """Every parity counter, event, digest and table equal period by period (run_pair), and the exact
    protocol-level counters at the end; the skip taken (fault-free periods before the faults)."""
    a, b = scenarios.run_pair(name, _make("1"), _make("0"))
    sa, sb = a.stats(), b.stats()
    assert {k: sa[k] for k in EXACT} == {k: sb[k] for k in EXACT}
    assert sb["quiet_periods"] == 0
    print(name, "quiet periods:", sa["quiet_periods"], "of", sa["period"])


@pytest.mark.parametrize("tracked", [0, 256])
def test_quiet_stretches_around_a_storm(tracked):
    """LAN, 4,096 members (dense, or N x K with 256 columns): 20 fault-free periods (all quiet from
    the first test on), a 1 % crash, its storm and suspicion timeouts (busy), then quiet again once the
    last gossip is swept; equal to the always-running handle at every period."""
    cfg = ClusterConfig.defaultLanConfig()
    kw = {"tracked_subjects": tracked} if tracked else {}
    n = 4096
    a = _make("1")(cfg, n, 5, event_capacity=1 << 20, **kw)
    b = _make("0")(cfg, n, 5, event_capacity=1 << 20, **kw)
    busy_seen = quiet_after = 0
    for t in range(140):
        if t == 20:
            ids = scenarios.crash_ids(n, 41, 5)
            a.crash(ids)
            b.crash(ids)
        q0 = a.stats()["quiet_periods"]
        a.step(1)
        b.step(1)
        sa, sb = a.stats(), b.stats()
        quiet = sa["quiet_periods"] > q0
        if t < 20:
            assert quiet, f"fault-free period {t} ran its rounds"
        elif not quiet:
            busy_seen += 1
        elif busy_seen:
            quiet_after += 1
        assert {k: sa[k] for k in EXACT} == {k: sb[k] for k in EXACT}, f"period {t}"
        assert a.digest() == b.digest(), f"period {t}"
        assert [e.key() for e in a.events()] == [e.key() for e in b.events()], f"period {t}"
    assert busy_seen > 10 and quiet_after > 0 and sb["quiet_periods"] == 0
    for i in range(0, n, 97):
        assert np.array_equal(a.view(i), b.view(i))
        assert np.array_equal(a.deadlines(i), b.deadlines(i))
