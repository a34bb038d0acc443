"""Probe: gossip-storm size of a bench workload on the GPU (live gossip slots per period).
python tools/probe_storm.py [workload] [log2 ring slots] [periods] [log2 record capacity] [members]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
import bench
from swimhip import SwimCluster
from swimhip.cluster import SwimError

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 20
periods = int(sys.argv[3]) if len(sys.argv) > 3 else 60
if len(sys.argv) > 4:
    kw_r = {"record_capacity": 1 << int(sys.argv[4])}
else:
    kw_r = {}
w = dict(bench.WORKLOADS[wl])
if len(sys.argv) > 5:
    w["n"] = int(sys.argv[5])
kw = {"tracked_subjects": w["tracked"]} if w.get("tracked") else {}
kw.update(kw_r)
c = SwimCluster(bench.preset_config(w["preset"]), w["n"], seed=1, gossip_capacity=1 << lg, sync_capacity=w.get("scap", 0), **kw)
if w["loss"]:
    c.set_loss(w["loss"])
c.step(3)
if "crash_n" in w:  # the same number of crashes at any size
    c.crash(bench.crash_set(w["n"], w["crash_n"] / w["n"], 1))
else:
    bench.inject_faults(c, wl, 3, 1, n=w["n"])
t = time.time()
for p in range(periods):
    t1 = time.time()
    try:
        c.step(1)
    except SwimError as e:
        print("period", p, "ERROR", e, flush=True)
        break
    s = c.stats()
    print(f"period {p} created {s['gossips_created']} live {s['live_gossip_slots']} records {s['live_gossip_records']} "
          f"syncs {s['syncs_delivered']} "
          f"removed {s['events_removed']} dt {time.time() - t1:.3f}s", flush=True)
c.close()
