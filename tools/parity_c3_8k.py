"""C3's schedule (LAN, 10 % simultaneous crash + the 16-member partition, bench.py's c3) at 8,192 members,
the GPU handle against the CPU oracle: digests, every parity counter and the MembershipEvent stream every 4
periods through 24 periods from the crash, every view and deadline row at the end. The oracle needs ~2
minutes and ~23 GB in the build container (43 s on the GPU box's host): tests/test_gpu_fullsize.py runs it;
`python tools/parity_c3_8k.py 16384` is the one-off at 16,384 members (~90 GB of oracle state).
Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "scalecube-cluster_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402
from swimhip import SwimCluster  # noqa: E402


def main(n=8192, periods=24, every=4):
    cfg = bench.preset_config("lan")
    t0 = time.time()
    a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 17, sync_capacity=8192, event_capacity=1 << 24)
    b = OracleCluster(cfg, n, seed=1, event_capacity=1 << 24)
    for c in (a, b):
        c.step(3)
        bench.inject_faults(c, "c3", 3, 1, n=n)
    checks = 0
    for t in range(periods // every):
        for c in (a, b):
            c.step(every)
        ea = [e.key() for e in a.events()]
        eb = [e.key() for e in b.events()]
        assert ea == eb, f"events differ by period {3 + every * (t + 1)}"
        sa, sb = a.stats(), b.stats()
        bad = {k: (sa[k], sb[k]) for k in scenarios.PARITY_KEYS if sa[k] != sb[k]}
        assert not bad, bad
        assert a.digest() == b.digest()
        checks += 1
        print(f"period {3 + every * (t + 1)}: equal; gossips {sb['gossips_created']}, {time.time() - t0:.0f} s", flush=True)
    for i in range(n):
        assert np.array_equal(a.view(i), b.view(i)), f"view row {i}"
        assert np.array_equal(a.deadlines(i), b.deadlines(i)), f"deadline row {i}"
    s = a.stats()
    print(json.dumps({"members": n, "periods_after_crash": periods, "checks": checks, "rows_compared": n,
                      "gossips_created": s["gossips_created"], "first_receipts": s["gossip_first_receipts"],
                      "equal": True, "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
