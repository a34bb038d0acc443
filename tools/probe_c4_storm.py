"""Probe: the gossip storm of C4's schedule (LAN defaults, 1 % uniform loss, 0.1 % simultaneous crash)
at a given cluster size, on one GPU (dense views). Under probabilistic loss every gossip takes its own
ring slot, so the live-slot count is the per-(member, slot) state the run needs.

python tools/probe_c4_storm.py N [log2 ring slots] [periods] [warmup] [tracked subjects K: N x K views]

Prints one line per period and, at the end, one JSON line: peak live gossips, created per period
(steady part), the ring size used and whether it overflowed (SWIM_EOVERFLOW ends the probe)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
import bench  # noqa: E402
from swimhip import SwimCluster  # noqa: E402
from swimhip.cluster import SwimError  # noqa: E402

n = int(sys.argv[1])
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 20
periods = int(sys.argv[3]) if len(sys.argv) > 3 else 40
warmup = int(sys.argv[4]) if len(sys.argv) > 4 else 5
k = int(sys.argv[5]) if len(sys.argv) > 5 else 0
kw = {"tracked_subjects": k} if k else {}
c = SwimCluster(bench.preset_config("lan"), n, seed=1, gossip_capacity=1 << lg, **kw)
c.set_loss(1.0)
crashed = bench.crash_set(n, 0.001, 1)
rows, err, t = [], None, time.time()
prev = 0
for p in range(warmup + periods):
    if p == warmup and crashed:
        c.crash(crashed)
    t1 = time.time()
    try:
        c.step(1)
    except SwimError as e:
        err = str(e)
        print("period", p, "ERROR", e, flush=True)
        break
    s = c.stats()
    row = {"period": p, "created": s["gossips_created"] - prev, "live": s["live_gossip_records"],
           "received": s["gossip_first_receipts"], "sends": s["gossip_sends"],
           "slots": s["live_gossip_slots"], "escapes": s["escape_entries"], "fd_suspect": s["fd_suspect_events"], "removed": s["events_removed"],
           "dt": round(time.time() - t1, 3)}
    prev = s["gossips_created"]
    rows.append(row)
    print(json.dumps(row), flush=True)
c.close()
steady = [r["created"] for r in rows[2:warmup]] + [r["created"] for r in rows[warmup + 2:]]
print(json.dumps({"n": n, "ring_log2": lg, "tracked_subjects": k or None, "periods_run": len(rows), "overflow": err,
                  "peak_live": max((r["live"] for r in rows), default=0),
                  "created_per_period": sum(steady) / max(1, len(steady)),
                  "crashed": len(crashed), "wall_s": round(time.time() - t, 1)}), flush=True)
