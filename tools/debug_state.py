"""Debug: per-step comparison of member cursors, holdings and views between GPU and oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "scalecube-cluster_amd")]

import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402
from swimhip import SwimCluster  # noqa: E402

name = sys.argv[1]
cfg, n, seed, script, kw = scenarios.scenario(name)
a = SwimCluster(cfg, n, seed, event_capacity=1 << 20, **kw)
b = OracleCluster(cfg, n, seed, event_capacity=1 << 20, **kw)
ga, gb = script(a), script(b)
step = 0
for _ in ga:
    next(gb)
    step += 1
    ma, mb = a.debug_member_state(), b.debug_member_state()
    bad = {k: np.nonzero(ma[k] != mb[k])[0][:8].tolist() for k in ma if not np.array_equal(ma[k], mb[k])}
    vd = [i for i in range(n) if not np.array_equal(a.view(i), b.view(i))]
    hd = [m for m in range(n) if a.debug_holdings(m) != b.debug_holdings(m)]
    print(f"step {step}: state_diff={bad} view_rows_diff={vd[:8]} holdings_diff={hd[:8]}")
    for k, idx in bad.items():
        for i in idx[:4]:
            print(f"    {k}[{i}] gpu={ma[k][i]} oracle={mb[k][i]}  (gpu g_ep/cur {ma['g_epoch'][i]}/{ma['g_cursor'][i]}"
                  f" oracle {mb['g_epoch'][i]}/{mb['g_cursor'][i]})")
    if bad or vd:
        break
