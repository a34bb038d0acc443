"""bench.py's own multi-rank launch on the GPU box (VERDICT r05 "next" #1).

`python bench.py --gpus 4` (no torch.distributed.run around it) must start 4 ranks itself, report
`n_gpus: 4`, and do the same protocol work as `--gpus 1`: the cluster is one cluster whatever its
observer rows are split into, and sharding is bit-exact. The 4 ranks share cuda:0 and
exchange over gloo here (one GPU per box); the node run uses the library's RCCL communicator.
The exchanged messages are GossipRequests (GossipProtocolImpl.java:225-239) and SYNC / SYNC_ACK
(MembershipProtocolImpl.java:457-473).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args, "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_gpus4_spawns_ranks_with_equal_work():
    common = ["--workload", "c2", "--steps", "5", "--warmup", "3", "--converge", "0"]
    one = _bench("--gpus", "1", *common)
    four = _bench("--gpus", "4", "--backend", "gloo", *common)
    assert one["n_gpus"] == 1 and four["n_gpus"] == 4
    assert four["config"]["members_per_gpu"] == one["config"]["members"] // 4
    # the protocol's work is the same cluster's; the kernels' internal walk counters (words scanned,
    # probes, apply runs) depend on how the rows are split and are not compared
    proto = ("fd_probes", "gossips_created", "gossip_first_receipts", "syncs_delivered", "merge_cells",
             "events_removed", "gossip_sends", "infected_suppressed", "infected_pruned_pairs", "infected_records")
    assert {k: four["work"][k] for k in proto} == {k: one["work"][k] for k in proto}
    assert one["work"]["gossips_created"] > 0 and one["work"]["gossip_sends"] > 0
    assert four["gossip_slots"] == one["gossip_slots"]
