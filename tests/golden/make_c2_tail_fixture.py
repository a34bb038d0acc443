"""Golden fixture for tests/test_gpu_fullsize.py::test_c2_convergence_tail_is_fd_driven: the
oracle on the bench's C2 schedule (bench.py workload c2, seed 1: 4,096 dense, LAN, 5 % loss, 41
crashes at t0 = 3) up to t0 + 75 periods — past the 65-period suspicion timeout — with the view
and deadline digests, the parity counters, and the (observer, crashed subject) pairs not yet
converged. The oracle needs ~15 minutes for this (the SYNC re-spread storm at 4,096 members), so
the GPU test compares against this file instead of running it.

  python tests/golden/make_c2_tail_fixture.py > tests/golden/c2_tail_oracle.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "scalecube-cluster_amd"),
                os.path.dirname(HERE)]

import bench  # noqa: E402
import oracle_py  # noqa: E402
import scenarios  # noqa: E402

w = bench.WORKLOADS["c2"]
n = w["n"]
b = oracle_py.OracleCluster(bench.preset_config("lan"), n, seed=1)
b.set_loss(w["loss"])
b.step(3)
crashed = bench.inject_faults(b, "c2", 3, 1, n=n)
checkpoints = []
for k in range(5):
    b.step(15)
    st = b.stats()
    checkpoints.append({"period": 3 + 15 * (k + 1), "digest": [int(x) for x in b.digest()],
                        "stats": {key: int(st[key]) for key in scenarios.PARITY_KEYS}})
    print(f"t0+{15 * (k + 1)}: not_converged={st['not_converged']}", file=sys.stderr, flush=True)
pres, _ = b.presence()
subj = [int(s) for s in crashed if pres[s]]
pairs = []
cs = set(crashed)
for i in range(n):
    if i in cs:
        continue
    row = b.view(i)
    pairs += [[i, s, int(row[s])] for s in subj if row[s]]
json.dump({"workload": "c2", "seed": 1, "t0": 3, "crashed": [int(x) for x in crashed], "checkpoints": checkpoints,
           "stragglers": pairs}, sys.stdout, indent=1)
