"""bench.py's workload and byte-model helpers and its rank launching (CPU only)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c3_workload_matches_baseline_config():
    w = bench.WORKLOADS["c3"]
    assert w["n"] == 65536 and w["crash"] == 0.10 and w["part"] == 40 and w["preset"] == "lan"
    assert w["part"] < 85  # heals before the 85-period suspicion timeout (ClusterMath at N = 65,536)


def test_partition_groups_spread_evenly():
    g = bench.partition_groups(65536, 16)
    ids = np.nonzero(g)[0]
    assert len(ids) == 16 and ids.tolist() == [k * 4096 for k in range(16)]
    assert bench.partition_groups(8192, 16).sum() == 16


def test_crash_set_is_seeded_and_sized():
    a, b = bench.crash_set(65536, 0.10, 1), bench.crash_set(65536, 0.10, 1)
    assert a == b and len(a) == 6554 and len(set(a)) == 6554 and a == sorted(a)
    assert bench.crash_set(100, 0.0, 1) == []


def test_kernel_bytes_covers_every_timed_class():
    from swimhip import SwimCluster

    d = {k: 1 for k in ("merge_cells", "ack_cells", "gossip_scanned", "gossip_hd_words", "gossip_window_words",
                        "gossip_pull_words", "gossip_probes", "gossip_first_receipts", "sweep_cells", "fd_probes",
                        "infected_pruned_pairs", "infected_records", "apply_words", "apply_runs", "apply_subjects",
                        "suspicion_timeouts")}
    for name in SwimCluster.KERNEL_CLASSES:
        if name != "bookkeeping":
            assert bench.kernel_bytes(name, d) > 0, name


def test_pmc_traffic_reads_committed_summary():
    t = bench.pmc_traffic("k_gossip_select")
    assert t is None or t > 0
    assert bench.pmc_traffic("no_such_kernel") is None


def test_pmc_traffic_is_per_workload_and_single_gpu():
    # the committed summary is of the default C3 run on one GPU: no other workload, no shard
    if bench.pmc_traffic("k_gossip_select") is not None:
        assert bench.pmc_traffic("k_gossip_select", "c3", 2) is None
    assert bench.pmc_traffic("k_gossip_select", "no_such_workload") is None


def test_rank_launch_single_gpu_runs_in_process():
    assert bench.rank_launch(1, ["--steps", "2"], env={}) is None


def test_rank_launch_spawns_n_ranks_without_launcher():
    cmd = bench.rank_launch(4, ["--gpus", "4", "--workload", "c2"], env={})
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--workload", "c2"] and cmd[-5].endswith("bench.py")


def test_rank_launch_under_launcher_checks_world_size():
    assert bench.rank_launch(8, ["--gpus", "8"], env={"WORLD_SIZE": "8"}) is None
    with pytest.raises(ValueError, match="WORLD_SIZE=2"):
        bench.rank_launch(8, ["--gpus", "8"], env={"WORLD_SIZE": "2"})
    with pytest.raises(ValueError, match="WORLD_SIZE=4"):
        bench.rank_launch(1, [], env={"WORLD_SIZE": "4"})
    with pytest.raises(ValueError):
        bench.rank_launch(0, [], env={})


def test_bench_cli_refuses_world_size_mismatch():
    # the refusal happens at argument handling, before the library or any GPU is touched
    env = dict(os.environ, WORLD_SIZE="2")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""
