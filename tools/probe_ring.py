"""Gossip ids issued and the peak of live ring slots per scenario, to size a non-power-of-two ring
that wraps several times in a parity test (ids mod GC on rings that are not powers of two)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "scalecube-cluster_amd"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)
import bench  # noqa: E402
import scenarios  # noqa: E402
from swimhip import SwimCluster  # noqa: E402


def probe(name, batching):
    cfg, n, seed, script, kw = scenarios.scenario(name)
    c = SwimCluster(cfg, n, seed, gossip_capacity=1 << 17, gossip_batching=batching, **kw)
    peak = 0
    for _ in script(c):
        peak = max(peak, c.stats()["live_gossip_slots"])
    s = c.stats()
    print(f"{name} batching={batching}: created {s['gossips_created']} peak live slots {peak}", flush=True)


def probe_c3(batching, wl="c3"):
    n = 1024
    c = SwimCluster(bench.preset_config("lan"), n, seed=1, gossip_capacity=1 << 17, gossip_batching=batching)
    c.step(3)
    bench.inject_faults(c, wl, 3, 1, n=n)
    peak = 0
    for _ in range(40):
        c.step(1)
        peak = max(peak, c.stats()["live_gossip_slots"])
    s = c.stats()
    print(f"{wl}@1024 batching={batching}: created {s['gossips_created']} peak live slots {peak}", flush=True)


for nm in ("lan256_loss5_crash3", "lan1024_loss5_crash10", "local100_loss20"):
    probe(nm, True)
probe_c3(True)
probe_c3(False)
