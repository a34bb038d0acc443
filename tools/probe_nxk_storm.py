"""Probe: gossip-storm size of N x K tracked-subject runs on the GPU (live gossip slots per period).
python tools/probe_nxk_storm.py N K crashes log2_ring_slots periods"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
import bench
from swimhip import SwimCluster
from swimhip.cluster import SwimError

n, k, nc, lg, periods = (int(x) for x in sys.argv[1:6])
c = SwimCluster(bench.preset_config("lan"), n, seed=1, gossip_capacity=1 << lg, tracked_subjects=k)
c.step(3)
c.crash(bench.crash_set(n, nc / n, 1))
peak = 0
for p in range(periods):
    t1 = time.time()
    try:
        c.step(1)
    except SwimError as e:
        print("period", p, "ERROR", e, flush=True)
        break
    s = c.stats()
    peak = max(peak, s["live_gossip_slots"])
    print(f"N {n} period {p} created {s['gossips_created']} live {s['live_gossip_slots']} syncs {s['syncs_delivered']} "
          f"receipts {s['gossip_first_receipts']} removed {s['events_removed']} dt {time.time() - t1:.3f}s", flush=True)
print(f"N {n} peak live {peak}", flush=True)
c.close()
