"""C4's node run rehearsed on one GPU: BASELINE configs[3]'s schedule (LAN, 1 %
loss, 0.1 % simultaneous crash after a 5-period warmup) at 32,768 members, dense views row-sharded
over 8 ranks (8 processes sharing cuda:0, gloo, the library-driven exchanges), against the unsharded
handle on rank 0: view and deadline digests, every parity counter and the presence vectors equal
every 4 periods through the storm the 1 % loss starts (false suspicions re-spread by SYNC,
MembershipProtocolImpl.java:649-656; one GossipRequest per gossip, each lost independently,
GossipProtocolImpl.java:225-239 / NetworkEmulator.java:166-180), and no buffer overflows."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N = 32768
WORLD = 8
SEED = 41
WARMUP, PERIODS, EVERY = 5, 24, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port):
    import scenarios
    from swimhip import ClusterConfig, SwimCluster
    from swimhip.sharded import ShardedSwimCluster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        cfg = ClusterConfig.defaultLanConfig()
        kw = dict(gossip_capacity=1 << 18, sync_capacity=2048)
        a = ShardedSwimCluster(cfg, N, SEED, **kw)
        b = SwimCluster(cfg, N, SEED, **kw) if rank == 0 else None
        crashed = scenarios.crash_ids(N, N // 1000, SEED)
        for c in (a, b):
            if c is not None:
                c.set_loss(1.0)
                c.step(WARMUP)
                c.crash(crashed)
        for t in range(PERIODS // EVERY):
            a.step(EVERY)
            if b is not None:
                b.step(EVERY)
            da, sa, pa = a.digest(), a.stats(), a.presence()  # (collective)
            if rank == 0:
                db, sb, pb = b.digest(), b.stats(), b.presence()
                bad = {k: (sa[k], sb[k]) for k in scenarios.PARITY_KEYS if sa[k] != sb[k]}
                assert not bad, f"period {WARMUP + EVERY * (t + 1)}: counters differ {bad}"
                assert da == db, f"period {WARMUP + EVERY * (t + 1)}: digests differ"
                assert np.array_equal(pa[0], pb[0]) and np.array_equal(pa[1], pb[1])
                assert sa["overflow"] == 0 and sb["overflow"] == 0
                print(f"period {WARMUP + EVERY * (t + 1)}: equal; gossips {sb['gossips_created']}, live slots "
                      f"{sb['live_gossip_slots']}, removed {sb['events_removed']}", flush=True)
        if rank == 0:
            s = b.stats()
            assert s["gossips_created"] > 0 and s["suspicion_timeouts"] >= 0
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_c4_schedule_32768_world8_matches_unsharded():
    mp.spawn(_worker, args=(WORLD, _free_port()), nprocs=WORLD, join=True)
