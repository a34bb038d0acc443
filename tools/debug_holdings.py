"""Debug: drive a scenario on GPU + oracle, compare per-member gossip holdings each step."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "scalecube-cluster_amd")]

import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402
from swimhip import SwimCluster  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "local48_links"
cfg, n, seed, script, kw = scenarios.scenario(name)
a = SwimCluster(cfg, n, seed, event_capacity=1 << 20, **kw)
b = OracleCluster(cfg, n, seed, event_capacity=1 << 20, **kw)
ga, gb = script(a), script(b)
step = 0
for _ in ga:
    next(gb)
    step += 1
    sa, sb = a.stats(), b.stats()
    diffs = {k: (sa[k], sb[k]) for k in scenarios.PARITY_KEYS if sa[k] != sb[k]}
    hd = []
    for m in range(n):
        ha, hb = a.debug_holdings(m), b.debug_holdings(m)
        if ha != hb:
            sa_, sb_ = set(ha), set(hb)
            hd.append((m, sorted(sa_ - sb_)[:6], sorted(sb_ - sa_)[:6], len(ha), len(hb)))
    print(f"step {step} period {sa['period']} stats_diff={diffs} holding_diffs={len(hd)}")
    for x in hd[:8]:
        print("   member", x[0], "gpu-only", x[1], "oracle-only", x[2], "sizes", x[3], x[4])
    if diffs or hd:
        if step > 3 and (diffs or hd):
            pass
    a.events(), b.events()
