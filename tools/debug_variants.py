"""Debug: run variants of a churn scenario GPU vs oracle and report the first divergence of each."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "scalecube-cluster_amd")]

import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402
from swimhip import ClusterConfig, SwimCluster  # noqa: E402

LAN = ClusterConfig.defaultLanConfig().membership(lambda o: o.seedMembers([0, 1, 2, 3]))
CR = [5, 40, 41, 100, 200, 255]
VARIANTS = {
    "full": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [256, 257, 258, 259], [260, 261, 262], 5.0)),
    "noloss": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [256, 257, 258, 259], [260, 261, 262], 0.0)),
    "restart_only": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [256, 257, 258, 259], [], 5.0)),
    "join_only": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [], [260, 261, 262], 5.0)),
    "crash_only": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [], [], 5.0)),
    "restart1": (LAN, 288, 12, lambda c: scenarios._churn(c, CR, [256], [], 5.0)),
}

for name, (cfg, n, seed, script) in VARIANTS.items():
    if len(sys.argv) > 1 and name not in sys.argv[1:]:
        continue
    a = SwimCluster(cfg, n, seed, event_capacity=1 << 20, n_initial=256)
    b = OracleCluster(cfg, n, seed, event_capacity=1 << 20, n_initial=256)
    ga, gb = script(a), script(b)
    step, verdict = 0, "ok"
    for _ in ga:
        next(gb)
        step += 1
        sa, sb = a.stats(), b.stats()
        bad = {k: (sa[k], sb[k]) for k in scenarios.PARITY_KEYS if sa[k] != sb[k]}
        ea = [e.key() for e in a.events()]
        eb = [e.key() for e in b.events()]
        if bad or ea != eb or a.digest() != b.digest():
            ma, mb = a.debug_member_state(), b.debug_member_state()
            sd = {k: np.nonzero(ma[k] != mb[k])[0][:8].tolist() for k in ma if not np.array_equal(ma[k], mb[k])}
            hd = [m for m in range(n) if a.debug_holdings(m) != b.debug_holdings(m)]
            verdict = f"step {step}: stats {bad} events_equal={ea == eb} state_diff={sd} holdings_diff={hd[:10]}"
            (ra, sa_), (rb, sb_) = a.debug_sends(), b.debug_sends()
            for i in np.nonzero((ra != rb) | (sa_ != sb_))[0][:20]:
                verdict += f"\n    sender {i}: raw gpu {ra[i]} oracle {rb[i]}  supp gpu {sa_[i]} oracle {sb_[i]}"
            break
    print(f"{name}: {verdict}", flush=True)
