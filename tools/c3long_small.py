"""The c3long schedule (10 % crash + a 16-member group cut for 120 periods past the suspicion
timeout, seeds 0..15) at N = 1,024 on the GPU and the oracle: parity every 25 periods and the
not-converged count, to tell reference semantics from a device bug in the slow convergence."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "scalecube-cluster_amd")]

import bench  # noqa: E402
import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402
from swimhip import SwimCluster  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
periods = int(sys.argv[2]) if len(sys.argv) > 2 else 400
cfg = bench.preset_config("lan").membership(lambda o: o.seedMembers(list(range(16))))
a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 18)
b = OracleCluster(cfg, n, seed=1)
for c in (a, b):
    c.step(3)
    crashed = bench.inject_faults(c, "c3long", 3, 1, n=n)
t = time.time()
for k in range(periods // 25):
    for c in (a, b):
        c.step(25)
    sa, sb = a.stats(), b.stats()
    same = a.digest() == b.digest() and all(sa[x] == sb[x] for x in scenarios.PARITY_KEYS)
    pres, _ = a.presence()
    held = {int(s): int(pres[s]) for s in crashed if pres[s]}
    print(f"t0+{25 * (k + 1)}: parity={same} not_converged gpu={sa['not_converged']} oracle={sb['not_converged']} "
          f"crashed subjects still held: {len(held)} (max holders {max(held.values()) if held else 0}) "
          f"[{time.time() - t:.0f} s]", flush=True)
    if not same:
        bad = {x: (sa[x], sb[x]) for x in scenarios.PARITY_KEYS if sa[x] != sb[x]}
        print("  differs:", bad, flush=True)
        break
if held:
    s0 = sorted(held)[0]
    obs = [i for i in range(n) if i not in set(crashed) and a.view(i)[s0]]
    print(f"subject {s0}: held by {len(obs)} alive observers, e.g. {obs[:10]}; records {[int(a.view(i)[s0]) for i in obs[:10]]}")
    g = bench.partition_groups(n, 16)
    print(f"  observers in the cut group: {sum(int(g[i]) for i in obs)}")
