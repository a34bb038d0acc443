"""Observer-row sharding: the host exchange protocol on CPU (gloo, 2 ranks), and
the sharded HIP path against the unsharded one, bit for bit, on one GPU (2 ranks, gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from swimhip import _native as nat
from swimhip.cluster import SwimError
from swimhip.sharded import ShardedSwimCluster


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "gloo" and world > 1:  # ranks sharing one GPU: one hardware queue each (HIP's default: 4)
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)


def _exchange_worker(rank, world, port, backend="gloo"):
    """Drive ShardedSwimCluster._exchange and check every op's semantics: host buffers over gloo,
    or (backend "nccl") HBM buffers over RCCL, the path bench.py --gpus N takes."""
    _init(rank, world, port, backend)
    try:
        c = object.__new__(ShardedSwimCluster)
        c._dist, c._torch, c._group = dist, torch, None
        c.rank, c.world, c._gloo = rank, world, backend == "gloo"
        dev = "cpu" if backend == "gloo" else "cuda:0"
        c._send = torch.zeros(64, dtype=torch.int32, device=dev)
        c._recv = torch.zeros(256, dtype=torch.int32, device=dev)
        x = c._x = nat.SwimXchg()
        # all-gather of unequal contributions, padded to the max
        n = 2 + 3 * rank
        c._send[:n] = torch.arange(n, dtype=torch.int32, device=dev) + 100 * rank
        x.op, x.send_words = nat.X_ALLGATHER, n
        c._exchange(c._status(None))
        m = int(x.recv_stride)
        assert m == 2 + 3 * (world - 1)
        for q in range(world):
            cnt = int(x.recv_counts[q])
            assert cnt == 2 + 3 * q
            assert c._recv[q * m:q * m + cnt].tolist() == [100 * q + i for i in range(cnt)]
        # all-to-all-v: rank r sends (q + 1) words of value 10 r + q to rank q
        x.op = nat.X_ALLTOALLV
        off = 0
        for q in range(world):
            x.send_counts[q] = q + 1
            c._send[off:off + q + 1] = 10 * rank + q
            off += q + 1
        c._exchange(c._status(None))
        got, off = [], 0
        for q in range(world):
            cnt = int(x.recv_counts[q])
            assert cnt == rank + 1
            got.append(c._recv[off:off + cnt].tolist())
            off += cnt
        assert got == [[10 * q + rank] * (rank + 1) for q in range(world)]
        # a failure on one rank is raised on every rank at the next status all-gather
        x.op = nat.X_DONE
        err = SwimError(-75, "shard_step: simulator buffer overflow") if rank == world - 1 else None
        with pytest.raises(SwimError) as ei:
            c._status(err)
        assert ei.value.code == -75
        # ranks out of step (different exchange ops) are an error too, never a mismatched collective
        if world > 1:
            x.op = nat.X_ALLGATHER if rank == 0 else nat.X_DONE
            x.send_words = 0
            with pytest.raises(SwimError):
                c._status(None)
    finally:
        dist.destroy_process_group()


def test_exchange_protocol_gloo_cpu():
    mp.spawn(_exchange_worker, args=(2, _free_port()), nprocs=2, join=True)


@pytest.mark.gpu
def test_exchange_protocol_rccl_one_rank():
    """The RCCL ("nccl" backend) calls of the sharded path — status all-gather, all_gather_into_tensor
    and all_to_all_single on int32 HBM buffers with split sizes — on a one-rank group: RCCL refuses
    two ranks on one GPU, so this is how far the collectives can be exercised before the driver's
    multi-GPU run."""
    mp.spawn(_exchange_worker, args=(1, _free_port(), "nccl"), nprocs=1, join=True)


def _parity_worker(rank, world, port, names, shard_kw=None):
    import scenarios
    from swimhip import SwimCluster

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        for name in names:
            scenarios.run_pair(name, lambda *a, **k: ShardedSwimCluster(*a, **k, **(shard_kw or {})), SwimCluster)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,names", [(2, ["c1_local32_crash", "local48_links"]),
                                         (2, ["lan256_loss5_crash3", "local128_partition_heal"]),
                                         (2, ["test64_long_partition_rejoin"]),
                                         (4, ["local128_partition_heal", "lan1024_loss5_crash10"])])
def test_shards_match_unsharded(world, names):
    """`world` ranks sharing cuda:0, gloo exchanges: views, deadlines, events, counters, digests
    and presence equal the unsharded handle's after every period."""
    mp.spawn(_parity_worker, args=(world, _free_port(), names), nprocs=world, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,names", [(2, ["local32_leave2", "lan256_leave3_loss5"]),
                                         (4, ["local64_delay100_loss10", "lan256_delay200_crash3"]),
                                         (2, ["test48_delay30_partition", "local64_update_metadata"]),
                                         (4, ["local64_user_gossips_loss10", "local32_leave2"])])
def test_shard_lifecycle_and_delays_match_unsharded(world, names):
    """The calls sharded handles now take: graceful leaves (the leaver's shard
    announces its stop in the next commit exchange; liveness is replicated), message delays (a
    receiver shard asks for every window word, since every message draws its delay), metadata
    updates and user gossips. Bit-exact with the unsharded handle, period by period."""
    mp.spawn(_parity_worker, args=(world, _free_port(), names), nprocs=world, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,names", [(2, ["local40_restart_join"]),
                                         (4, ["local40_restart_join", "lan288_restart_join_loss5"])])
def test_shard_joins_and_restarts_match_unsharded(world, names):
    """Joins and restarts on sharded handles (round 6): spare slots on every shard, the
    joiner's row on its own shard, liveness and addresses replicated; an initial SYNC to a seed on
    another shard travels in the SYNC exchange as [JOIN_REQ | joiner, seed, table] and the seed it
    takes the SYNC_ACK of answers in the same record (MembershipProtocolImpl.start0, :222-257); a
    restarted member takes an address whose old id's pings answer DEST_GONE (FailureDetectorImpl.java:
    231-235). Crashes, restarts on the same addresses and joins through the seeds, with 5 % loss on the
    LAN one, bit-exact with the unsharded handle every period."""
    mp.spawn(_parity_worker, args=(world, _free_port(), names), nprocs=world, join=True)


@pytest.mark.gpu
def test_non_power_of_two_ring_shards_match_unsharded():
    """A 3,072-slot ring (not a power of two: ids mod GC) wrapping ~4 times, over 2 shards: every commit
    exchange assigns the same ids on both, bit-exact with the unsharded handle every period."""
    mp.spawn(_parity_worker, args=(2, _free_port(), ["local100_loss20_ring3k"]), nprocs=2, join=True)


@pytest.mark.gpu
def test_host_driven_exchanges_match_unsharded():
    """The host-driven protocol (swim_shard_step: the host performs each exchange the library
    describes, as a Java host with its own collectives would) against the unsharded handle; every
    other sharded test runs the library-driven exchanges (swim_step with a transport)."""
    mp.spawn(_parity_worker, args=(2, _free_port(), ["lan256_loss5_crash3", "local32_leave2"], {"exchange": "host"}),
             nprocs=2, join=True)


def _rccl_library_worker(rank, world, port, names):
    import scenarios
    from swimhip import SwimCluster

    _init(rank, world, port, "nccl")
    try:
        for name in names:
            scenarios.run_pair(name, lambda *a, **k: ShardedSwimCluster(*a, **k), SwimCluster)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_library_rccl_one_rank_matches_unsharded():
    """The library-owned RCCL communicator (swim_rccl_unique_id, swim_shard_comm_init: collectives on the
    handle's stream, one status all-gather per exchange) on a one-rank group: the handle then runs every
    exchange of a period through RCCL to itself (gossip-id commits with the liveness maxima, the status
    rows). RCCL refuses two ranks on one GPU, so this is how far the library-owned path runs before a
    multi-GPU node. Bit-exact with the unsharded handle every period."""
    mp.spawn(_rccl_library_worker, args=(1, _free_port(), ["c1_local32_crash", "lan256_loss5_crash3", "local32_leave2"]),
             nprocs=1, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,names", [(2, ["test48_delay30_partition", "test64_long_partition_rejoin"]),
                                         (4, ["local128_partition_heal"])])
def test_hd4_shards_match_unsharded_hd8(world, names):
    """4-bit infection rounds on sharded handles, which C4's and C5's node shards pick
    by default: the escape table of rounds 15 or more after a slot's creation (members reached late
    across a partition cut, or by a delayed message), k_hx_sweep, and the slots' creation rounds (gc8)
    written by commits every shard makes from the exchanged batch. Sharded hd4 against the unsharded
    8-bit handle, bit-exact every period."""
    mp.spawn(_parity_worker, args=(world, _free_port(), names, {"infection_round_bits": 4}), nprocs=world,
             join=True)


def _nxk_worker(rank, world, port, names, k):
    import scenarios
    from swimhip import SwimCluster

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        for name in names:
            scenarios.run_pair(name, lambda *a, **kw: ShardedSwimCluster(*a, tracked_subjects=k, **kw),
                               lambda *a, **kw: SwimCluster(*a, tracked_subjects=k, **kw))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,names,k", [(2, ["c1_local32_crash"], 4),
                                           (2, ["local128_partition_heal"], 128),
                                           (2, ["lan256_loss5_crash3"], 256)])
def test_nxk_shards_match_unsharded(world, names, k):
    """N x K tracked-subject views sharded by observer rows: every shard's column requests are
    all-gathered and allocated in subject order, so all shards agree on the columns (a SYNC row
    between shards is a row of columns). Bit-exact with the unsharded N x K handle, which is
    itself bit-exact with the dense oracle (test_gpu_parity.py::test_nxk_scenario_parity)."""
    mp.spawn(_nxk_worker, args=(world, _free_port(), names, k), nprocs=world, join=True)


def _c4_worker(rank, world, port):
    import scenarios
    from swimhip import SwimCluster

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        scenarios.run_pair("lan4096_c4_shape", lambda *a, **k: ShardedSwimCluster(*a, **k), SwimCluster,
                           compare_every=4)
    finally:
        dist.destroy_process_group()


def _c5_worker(rank, world, port):
    import scenarios
    from swimhip import SwimCluster

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        scenarios.run_pair("nxk4096_c5_shape", lambda *a, **k: ShardedSwimCluster(*a, tracked_subjects=256, **k),
                           lambda *a, **k: SwimCluster(*a, tracked_subjects=256, **k), compare_every=5)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_c5_shape_world4_matches_unsharded():
    """C5's shape (BASELINE configs[4]: N x K views with K = 256, 256 concurrent crashes ... here 64
    of 4,096 members, LAN, gossip batches) over 4 observer-row shards (gloo, ranks sharing cuda:0):
    column requests all-gathered and allocated in subject order on every shard, SYNC rows of K
    columns, batch slots committed identically everywhere; bit-exact with the unsharded N x K
    handle, which the parity suite pins to the dense oracle."""
    mp.spawn(_c5_worker, args=(4, _free_port()), nprocs=4, join=True)


@pytest.mark.gpu
def test_c4_shape_world8_matches_unsharded():
    """C4's schedule shape (1 % loss, 0.1 % crash, LAN) at 4,096 members over 8 observer-row shards
    (8 ranks sharing cuda:0, gloo): the exchanges C4's 8-GPU run makes (gossip-id commits, sender
    windows to remote receivers, SYNC rows) at world 8, bit-exact with the unsharded handle."""
    mp.spawn(_c4_worker, args=(8, _free_port()), nprocs=8, join=True)


def _overflow_worker(rank, world, port):
    from swimhip import ClusterConfig

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        # rank 0 alone gets a 1-row SYNC staging area: only it detects the overflow
        c = ShardedSwimCluster(ClusterConfig.defaultLanConfig(), 256, seed=5, sync_capacity=1 if rank == 0 else 0)
        with pytest.raises(SwimError) as ei:
            c.step(40)
        assert ei.value.code == -75
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_overflow_on_one_rank_fails_every_rank():
    """An overflow only one shard detects raises SWIM_EOVERFLOW on both ranks (no hang)."""
    mp.spawn(_overflow_worker, args=(2, _free_port()), nprocs=2, join=True)


def _leave_mismatch_worker(rank, world, port):
    from swimhip import ClusterConfig, SwimCluster

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        c = ShardedSwimCluster(ClusterConfig.defaultLocalConfig(), 64, seed=3)
        c.step(2)
        if rank == 0:  # past the collective argument check: only rank 0's library counts the leave
            SwimCluster.leave(c, [5])
        with pytest.raises(SwimError) as ei:
            c.step(4)
        assert ei.value.code == -22
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_leave_on_one_rank_fails_every_rank():
    """swim_leave sets the layout of every later commit-exchange block (a {gossips, stopped} header),
    so the library's status all-gather carries each rank's leave count: a rank that left members the
    others did not fails every rank with SWIM_EINVAL at the next exchange, instead of one rank
    reading another's header as gossips."""
    mp.spawn(_leave_mismatch_worker, args=(2, _free_port()), nprocs=2, join=True)



@pytest.mark.gpu
def test_unattached_shard_fails_loudly():
    """A sharded handle (rank 0 of 2) with neither a transport nor exchange buffers: swim_step refuses it
    (no transport), and swim_shard_step refuses it (no buffers), each with SWIM_EINVAL and before any
    kernel of the period runs; stepping it again fails the same way (xready repeats the check at every
    exchange of a period that did start)."""
    import ctypes

    from swimhip import ClusterConfig, SwimCluster

    c = SwimCluster(ClusterConfig.defaultLocalConfig(), 64, 3, _shard=(0, 2))
    try:
        for _ in range(2):
            with pytest.raises(SwimError) as ei:
                c.step(1)
            assert ei.value.code == nat.SWIM_EINVAL and "attach a transport" in str(ei.value)
            x = nat.SwimXchg()
            with pytest.raises(SwimError) as ei:
                c._call("shard_step", c._h, ctypes.byref(x))
            assert ei.value.code == nat.SWIM_EINVAL and "swim_shard_attach first" in str(ei.value)
    finally:
        c.close()
