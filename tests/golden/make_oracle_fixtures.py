"""Writes oracle_scenarios.json: self-consistency fixtures of the CPU oracle.

For every scenario of tests/scenarios.py (restatements of FailureDetectorTest,
MembershipProtocolTest, GossipProtocolTest and the BASELINE config shapes) it records, after each
step, the view/deadline digests, the protocol counters and a SHA-256 of the ordered
MembershipEvent stream. These pin the oracle itself across rounds (the reference cannot run in
this image): tests/test_oracle_fixtures.py re-runs the oracle and compares.

    python tests/golden/make_oracle_fixtures.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(REPO, "scalecube-cluster_amd"), os.path.join(REPO, "oracle"), os.path.dirname(HERE)):
    sys.path.insert(0, p)

import scenarios  # noqa: E402
from oracle_py import OracleCluster  # noqa: E402

OUT = os.path.join(HERE, "oracle_scenarios.json")


def trace(name):
    cfg, n, seed, script, kw = scenarios.scenario(name)
    c = OracleCluster(cfg, n, seed, event_capacity=1 << 20, **kw)
    steps = []
    ev_hash = hashlib.sha256()
    for _ in script(c):
        evs = [e.key() for e in c.events()]
        for k in evs:
            ev_hash.update(repr(k).encode())
        st = c.stats()
        vd, dd = c.digest()
        steps.append({"period": st["period"], "view_digest": f"{vd:016x}", "deadline_digest": f"{dd:016x}",
                      "events": len(evs), "events_sha256": ev_hash.hexdigest()[:16],
                      "stats": {k: st[k] for k in scenarios.PARITY_KEYS}})
    c.close()
    return {"n": n, "seed": seed, "steps": steps}


def main():
    out = {"generator": "tests/golden/make_oracle_fixtures.py", "scenarios": {}}
    for name in scenarios.SCENARIOS:
        out["scenarios"][name] = trace(name)
        print(name, len(out["scenarios"][name]["steps"]), "steps")
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
