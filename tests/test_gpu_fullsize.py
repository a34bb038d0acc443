"""C3 at full size on the GPU (BASELINE configs[2]: 65,536 members, dense N x N views, LAN
defaults, 10 % simultaneous crash + the bench's 2-way partition for 40 periods, healed via SYNC).

The oracle cannot run this size (the gossip storm holds ~1e6 gossips for 65,536 members), so the
run is checked through properties the reference's semantics guarantee:
  * no alive member is ever removed by an alive observer (presence of alive subjects stays at
    alive - 1 and nobody ever recorded removing one);
  * the crashed members are SUSPECT or absent in every alive row checked, and absent
    everywhere once converged (suspicion timeout 85 periods + the storm);
  * every bounded buffer held (swim_step raises SWIM_EOVERFLOW otherwise; the stats' mask is 0);
  * the run is deterministic: a second handle with the same seed reaches the same digests.
It exercises the 150 GiB layout, the 2^20-slot gossip ring, the apply kernel's LDS-hash spill path
and the infectedFrom bookkeeping at the sizes the bench uses."""
import numpy as np
import pytest

import bench
from swimhip import SwimCluster

pytestmark = pytest.mark.gpu

N = 65536


def _run(periods_a, periods_b):
    w = bench.WORKLOADS["c3"]
    c = bench.make_cluster("c3", 0, seed=1)
    c.step(3)
    crashed = bench.inject_faults(c, "c3", 3, 1)
    c.step(periods_a)
    d_a = c.digest()
    st_a = c.stats()
    # rows outside the 16-member partitioned group (ids k * N / 16), which is cut off until t0 + 40
    views_a = {i: c.view(i) for i in range(1, N, 4099)}
    c.step(periods_b)
    out = (d_a, st_a, views_a, c.digest(), c.stats(), c.presence(), crashed)
    c.close()
    return out


def test_c3_fullsize_properties_and_determinism():
    d_a, st_a, views_a, d_b, st_b, (pres, last), crashed = _run(30, 120)
    alive = np.ones(N, dtype=bool)
    alive[crashed] = False
    n_alive = int(alive.sum())
    assert st_a["overflow"] == 0 and st_b["overflow"] == 0
    assert st_a["gossips_created"] > 100_000  # the SYNC re-spread storm really happened
    # after 30 periods: crashed members are SUSPECT or absent in every sampled alive row of the
    # large side
    for i, row in views_a.items():
        if not alive[i]:
            continue
        cr = row[crashed]
        assert np.all((cr == 0) | ((cr & 3) == 2)), f"row {i} still trusts a crashed member"
        al = row[alive]
        assert np.all(al != 0), f"row {i} lost an alive member"
    # at the end (150 periods after the crash): no alive member was ever removed ...
    assert np.all(pres[alive] == n_alive - 1)
    assert np.all(last[alive] == 0)
    # ... and every crashed member is gone from every alive view
    assert st_b["not_converged"] == 0
    assert np.all(pres[crashed] == 0)
    assert st_b["events_removed"] == len(crashed) * n_alive
    # determinism: a second handle, same seed, same schedule
    d_a2, st_a2, _, d_b2, st_b2, _, _ = _run(30, 120)
    assert (d_a, d_b) == (d_a2, d_b2)
    assert {k: st_b[k] for k in ("gossips_created", "gossip_first_receipts", "gossip_sends", "events_removed")} == \
           {k: st_b2[k] for k in ("gossips_created", "gossip_first_receipts", "gossip_sends", "events_removed")}
