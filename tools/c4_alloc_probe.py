"""Memory plan check on one MI355X: build rank 0's shard of a bench workload row-sharded over
`world` GPUs (default C4: the 262,144-member dense cluster, 32,768 observer rows per GPU; `c5`: 2^20
members in N x K mode, 131,072 rows) plus its exchange buffers, and report the HBM it holds.
No period is stepped (that needs the other ranks); allocation and initialisation are the test.
python tools/c4_alloc_probe.py [world] [workload]"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scalecube-cluster_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from swimhip import SwimCluster  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
wl = sys.argv[2] if len(sys.argv) > 2 else "c4"  # any bench workload (c5: the N x K node config)
w = bench.WORKLOADS[wl]
kw = {"tracked_subjects": w["tracked"]} if w.get("tracked") else {}
if w.get("rcap"):
    kw["record_capacity"] = w["rcap"]
if w.get("dsub"):
    kw["dict_subjects"] = w["dsub"]
free0, total = torch.cuda.mem_get_info(0)
c = SwimCluster(bench.preset_config(w["preset"]), w["n"], seed=1, gossip_capacity=w["gcap"], device=0,
                sync_capacity=w.get("scap", 0), _shard=(0, world), **kw)
free1, _ = torch.cuda.mem_get_info(0)
sw, rw = ctypes.c_uint64(), ctypes.c_uint64()
c._call("shard_buffer_words", c._h, ctypes.byref(sw), ctypes.byref(rw))
send = torch.empty(sw.value, dtype=torch.int32, device="cuda:0")
recv = torch.empty(rw.value, dtype=torch.int32, device="cuda:0")
free2, _ = torch.cuda.mem_get_info(0)
G = 1 << 30
print(json.dumps({"workload": wl, "members": w["n"], "world": world, "rows_per_gpu": w["n"] // world,
                  "gossip_ring_slots": w["gcap"], "sync_capacity": w.get("scap", 0), "tracked_subjects": w.get("tracked"),
                  "infection_round_bits": 4 if c.stats()["escape_capacity"] else 8,
                  "hbm_total_gib": round(total / G, 1), "shard_state_gib": round((free0 - free1) / G, 1),
                  "exchange_buffers_gib": round((free1 - free2) / G, 1),
                  "hbm_used_gib": round((free0 - free2) / G, 1), "hbm_left_gib": round(free2 / G, 1)}))
