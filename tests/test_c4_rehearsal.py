"""C4's and C5's node runs rehearsed on one GPU: the schedules of
BASELINE configs[3] and [4], row-sharded over 8 ranks (8 processes sharing cuda:0, gloo, the
library-driven exchanges), against the unsharded handle on rank 0: view and deadline digests, every
parity counter and the presence vectors equal every few periods, and no buffer overflows.

* C4 (LAN, 1 % loss, 0.1 % simultaneous crash after a 5-period warmup), dense views: at 32,768 members
  for 24 periods, and at 65,536 members (the largest dense N for which 8 shards plus the unsharded
  handle fit one MI355X's 288 GB) through 44 storm periods. The 1 % loss starts a storm (false
  suspicions re-spread by SYNC, MembershipProtocolImpl.java:649-656; one GossipRequest per gossip,
  each lost independently, GossipProtocolImpl.java:225-239 / NetworkEmulator.java:166-180).
* C5 (LAN, N x K views with K = 256, 256 simultaneous crashes = concurrent churn): at 262,144 members
  through 110 periods, past the suspicion timeouts (5 x bit_length(262,143) = 90 periods of suspicion,
  MembershipProtocolImpl.java:620-647, then the removals; GossipProtocolImpl.java:171-183).
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SEED = 41


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, kw, loss, n_crash, warmup, periods, every, min_timeouts):
    import scenarios
    from swimhip import ClusterConfig, SwimCluster
    from swimhip.sharded import ShardedSwimCluster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # nine processes on one GPU: one hardware queue each (HIP's default is 4 per process), so the card's
    # queues are not oversubscribed (set before this process's first HIP call)
    os.environ["GPU_MAX_HW_QUEUES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        cfg = ClusterConfig.defaultLanConfig()
        a = ShardedSwimCluster(cfg, n, SEED, **kw)
        b = SwimCluster(cfg, n, SEED, **kw) if rank == 0 else None
        crashed = scenarios.crash_ids(n, n_crash, SEED)
        t0 = time.perf_counter()
        for c in (a, b):
            if c is not None:
                if loss:
                    c.set_loss(loss)
                c.step(warmup)
                c.crash(crashed)
        for t in range(periods // every):
            a.step(every)
            if b is not None:
                b.step(every)
            da, sa, pa = a.digest(), a.stats(), a.presence()  # (collective)
            if rank == 0:
                db, sb, pb = b.digest(), b.stats(), b.presence()
                p = warmup + every * (t + 1)
                bad = {k: (sa[k], sb[k]) for k in scenarios.PARITY_KEYS if sa[k] != sb[k]}
                assert not bad, f"period {p}: counters differ {bad}"
                assert da == db, f"period {p}: digests differ"
                assert np.array_equal(pa[0], pb[0]) and np.array_equal(pa[1], pb[1])
                assert sa["overflow"] == 0 and sb["overflow"] == 0
                print(f"period {p}: equal; gossips {sb['gossips_created']}, live slots {sb['live_gossip_slots']}, "
                      f"timeouts {sb['suspicion_timeouts']}, removed {sb['events_removed']}, "
                      f"{time.perf_counter() - t0:.1f} s", flush=True)
        if rank == 0:
            s = b.stats()
            assert s["gossips_created"] > 0 and s["suspicion_timeouts"] >= min_timeouts
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_c4_schedule_32768_world8_matches_unsharded():
    mp.spawn(_worker, args=(8, _free_port(), 32768, dict(gossip_capacity=1 << 18, sync_capacity=2048), 1.0, 32, 5,
                            24, 4, 0), nprocs=8, join=True)


@pytest.mark.gpu
def test_c4_schedule_65536_world8_matches_unsharded():
    """C4's schedule at 65,536 members: 8 shards of 8,192 rows plus the unsharded handle (a 2^19-slot
    ring each, 2x the ~2.6e5 live one-gossip slots of the storm's peak at this N),
    compared every 4 periods through 44 storm periods."""
    mp.spawn(_worker, args=(8, _free_port(), 65536, dict(gossip_capacity=1 << 19, sync_capacity=4096), 1.0, 66, 5,
                            44, 4, 0), nprocs=8, join=True)


@pytest.mark.gpu
def test_c5_schedule_262144_world8_matches_unsharded():
    """C5's schedule at 262,144 members - a quarter of BASELINE configs[4]'s 2^20 - (N x K, K = 256, 256
    simultaneous crashes) over 8 shards, compared every 10 periods through 110 periods: the crashed
    members' suspicion timeouts fire (every alive observer removes all 256: 67,043,328 removals) within
    the window. The ring has 80 x 1,024 slots (not a power of two), 1.85x this storm's ~44,300 live batch
    slots: two copies of the cluster with 2^18 slots do not fit one GPU. ~25 s."""
    mp.spawn(_worker, args=(8, _free_port(), 1 << 18, dict(gossip_capacity=80 * 1024, tracked_subjects=256), 0.0,
                            256, 3, 110, 10, 1), nprocs=8, join=True)
