"""Parity proper: libswimhip.so (gfx950) vs the CPU oracle, bit-exact on every membership table,
suspicion-deadline table, MembershipEvent sequence and protocol counter, period by period."""
import ctypes

import numpy as np
import pytest

import oracle_py
import scenarios
from oracle_py import OracleCluster
from swimhip import ClusterConfig, SwimCluster

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(scenarios.SCENARIOS))
def test_scenario_parity(name):
    scenarios.run_pair(name, SwimCluster, OracleCluster)


# Gossip batches: lossless scenarios run batched by default; every scenario with one
# ring slot per gossip and the LDS-hash apply (gossip_batching off) must match the oracle too


@pytest.mark.parametrize("name,wraps", [("local100_loss20_ring3k", 4), ("lan1024_loss5_ring17k", 1)])
def test_non_power_of_two_ring_matches_oracle(name, wraps):
    """Rings of any multiple of 1,024 slots (C4's shards use 5,128 x 1,024): gossip ids map to
    slots and bitmap words mod GC (gmod / wmod) once the ring is not a power of two. Scenarios that issue
    several rings' worth of one-gossip slots (20 % loss over 120 periods into 3,072 slots), or keep the
    ring nearly full (C2-like loss at 1,024 members in 17,408 slots): bit-exact with the oracle every
    period, no overflow."""
    a, b = scenarios.run_pair(name, SwimCluster, OracleCluster)
    s = a.stats()
    gcap = scenarios.scenario(name)[4]["gossip_capacity"]
    assert gcap & (gcap - 1) and s["overflow"] == 0
    assert s["gossips_created"] > wraps * gcap, s["gossips_created"]


@pytest.mark.parametrize("name", list(scenarios.SCENARIOS))
def test_scenario_parity_unbatched(name):
    """Handles without the record dictionary (gossip_batching off): one gossip per ring slot and the
    LDS-hash apply (k_gossip_apply), lossless and lossy scenarios alike."""
    def make(cfg, n, seed, **kw):
        return SwimCluster(cfg, n, seed, gossip_batching=False, **kw)

    scenarios.run_pair(name, make, OracleCluster)


def test_batches_share_slots_and_refuse_probabilistic_loss():
    """Batching stores each (origin, phase) batch in one slot: the C3 storm at N = 1,024 then needs
    several times fewer live slots than gossips, with every counter equal to the unbatched run's.
    A probabilistic loss cannot start while a multi-gossip slot is live (loss draws are per
    gossip): SWIM_EINVAL, the handle unchanged; once every batch is swept it is accepted."""
    import bench
    from swimhip import SwimError

    cfg = bench.preset_config("lan")
    n = 1024
    a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 17)
    b = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 17, gossip_batching=False)
    for c in (a, b):
        c.step(3)
        bench.inject_faults(c, "c3", 3, 1, n=n)
        c.step(8)
    sa, sb = a.stats(), b.stats()
    assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
    assert a.digest() == b.digest()
    assert sb["live_gossip_slots"] == sb["live_gossip_records"]  # one gossip per slot
    assert 0 < sa["live_gossip_slots"] * 2 < sa["live_gossip_records"]
    assert sa["apply_records"] > 0 and sb["apply_records"] == 0
    with pytest.raises(SwimError) as ei:
        a.set_loss(5.0)
    assert ei.value.code == -22
    b.set_loss(5.0)  # one gossip per slot: always allowed
    a.set_loss(100.0)  # blockAllOutbound draws nothing: allowed
    a.set_loss(0.0)


# N x K tracked-subject mode vs the dense oracle: K columns cover every subject whose record ever
# leaves the converged baseline in the scenario (crashes, false suspicions under loss, leaves)
NXK = {
    "c1_local32_crash": 4,
    "local32_leave2": 4,
    "lan256_loss5_crash3": 256,
    "local128_partition_heal": 128,
    "local48_links": 48,
    "local24_inbound_blocks": 24,
    "local64_delay100_loss10": 64,
}


@pytest.mark.parametrize("name", sorted(NXK))
def test_nxk_scenario_parity(name):
    k = NXK[name]

    def make_nxk(cfg, n, seed, **kw):
        return SwimCluster(cfg, n, seed, tracked_subjects=k, **kw)

    scenarios.run_pair(name, make_nxk, OracleCluster)


def test_nxk_c2_shape_4096_parity():
    """C2's shape (4,096, 5 % loss, 1 % crash) with 1,024 tracked columns for 12 periods."""
    cfg = ClusterConfig.defaultLanConfig()
    n = 4096
    a = SwimCluster(cfg, n, seed=7, tracked_subjects=1024, event_capacity=1 << 22)
    b = OracleCluster(cfg, n, seed=7, event_capacity=1 << 22)
    crashed = scenarios.crash_ids(n, 41, 7)
    for c in (a, b):
        c.set_loss(5.0)
        c.step(2)
        c.crash(crashed)
    for _ in range(3):
        for c in (a, b):
            c.step(4)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
        assert [e.key() for e in a.events()] == [e.key() for e in b.events()]
    for i in range(0, n, 97):
        assert np.array_equal(a.view(i), b.view(i)) and np.array_equal(a.deadlines(i), b.deadlines(i))
    pa, pb = a.presence(), b.presence()
    assert np.array_equal(pa[0], pb[0]) and np.array_equal(pa[1], pb[1])


def test_nxk_column_overflow_is_loud():
    """More subjects leaving the baseline than columns -> SWIM_EOVERFLOW, never a silent merge."""
    from swimhip import SwimError

    c = SwimCluster(ClusterConfig.defaultLocalConfig(), 64, seed=3, tracked_subjects=2)
    c.step(2)
    c.crash([1, 2, 3, 4, 5])
    with pytest.raises(SwimError) as ei:
        c.step(10)
    assert ei.value.code == -75
    # the failed run stays inspectable and every entry point stays memory-safe: ncells() is
    # clamped to the K columns that exist (ctl->ncols counts the refused requests too), k_crash /
    # k_digest / k_leave never index a column past K (round-2 r02_k illegal memory access)
    c.crash([6, 7])
    c.leave([8])
    dg = c.digest()
    assert len(dg) == 2
    for obs in (0, 9, 63):
        assert c.view(obs).shape == (64,)
        assert c.deadlines(obs).shape == (64,)
    pres, last = c.presence()
    assert pres.shape == (64,) and last.shape == (64,)
    with pytest.raises(SwimError) as ei2:  # still failed, still loud, and no HIP error
        c.step(1)
    assert ei2.value.code == -75


def test_philox_device_matches_oracle():
    from swimhip import native

    lib = native.load_swimhip()
    rng = np.random.default_rng(0)
    abct = rng.integers(0, 2**32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    for kind in (1, 7, 19):
        out = np.zeros(len(abct), dtype=np.uint32)
        P = ctypes.POINTER(ctypes.c_uint32)
        seed = 0x1234_5678_9ABC_DEF0
        assert lib.swim_kat_philox(seed, kind, abct.ctypes.data_as(P), out.ctypes.data_as(P), len(abct)) == 0
        ref = [oracle_py.philox(seed, kind, *map(int, r)) for r in abct[:256]]
        assert out[:256].tolist() == ref


def test_c2_shape_4096_full_parity():
    """BASELINE config 2 shape (4,096 dense, 5 % loss, fanout 3, 1 % crash), 12 periods: every
    membership table, every suspicion deadline, the ordered MembershipEvent stream and the
    protocol counters equal the oracle's every 4 periods."""
    cfg = ClusterConfig.defaultLanConfig()
    n = 4096
    a = SwimCluster(cfg, n, seed=2024, event_capacity=1 << 22)
    b = OracleCluster(cfg, n, seed=2024, event_capacity=1 << 22)
    crashed = scenarios.crash_ids(n, 41, 2024)
    for c in (a, b):
        c.set_loss(5.0)
        c.step(2)
        c.crash(crashed)
    for _ in range(3):
        for c in (a, b):
            c.step(4)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
        assert [e.key() for e in a.events()] == [e.key() for e in b.events()]
        for i in range(n):
            assert np.array_equal(a.view(i), b.view(i)), f"view row {i}"
            assert np.array_equal(a.deadlines(i), b.deadlines(i)), f"deadline row {i}"


def test_crash_converges_and_gossip_capacity_reports_overflow():
    """A too-small gossip ring must fail loudly (SWIM_EOVERFLOW), never silently diverge."""
    from swimhip import SwimError

    cfg = ClusterConfig.defaultLanConfig()
    with pytest.raises(SwimError):
        SwimCluster(cfg, 2048, seed=3, gossip_capacity=16)  # below the 1024-slot minimum
    c = SwimCluster(cfg, 2048, seed=3, gossip_capacity=1024)
    c.crash(scenarios.crash_ids(2048, 400, 3))
    with pytest.raises(SwimError) as ei:
        c.step(12)
    assert ei.value.code == -75  # SWIM_EOVERFLOW


def test_c3_schedule_small_parity():
    """The bench's C3 fault schedule (10 % simultaneous crash + a 16-member partition for 40
    periods healed by SYNC, LAN defaults) at N = 1,024: the gossip storm it triggers (SYNC merges
    re-spreading accepted SUSPECT records) must match the oracle bit for bit."""
    import bench

    cfg = bench.preset_config("lan")
    n = 1024
    a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 17)
    b = OracleCluster(cfg, n, seed=1)
    for c in (a, b):
        c.step(3)
        bench.inject_faults(c, "c3", 3, 1, n=n)
    for _ in range(12):
        for c in (a, b):
            c.step(5)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
    assert a.stats()["gossips_created"] > 10 * n  # the storm really happened


_SPILL_SCRIPT = """
import sys
sys.path[:0] = {paths!r}
import scenarios
from oracle_py import OracleCluster
from swimhip import SwimCluster
# k_gossip_apply (the LDS-hash apply) runs on handles without the record dictionary (gossip_batching
# off); with it, one-gossip slots go through k_gossip_apply_b too
def unbatched(cfg, n, seed, **kw):
    return SwimCluster(cfg, n, seed, gossip_batching=False, **kw)
a, b = scenarios.run_pair("lan288_restart_join_loss5", unbatched, OracleCluster)
spills = a.stats()["apply_spills"]
# a lossy run (one gossip per slot) with more receivers than workgroups and few gossips in flight:
# small receipt sets, which k_gossip_apply pairs
a2, b2 = scenarios.run_pair("lan1024_loss5_crash10", unbatched, OracleCluster, full_tables=False)
spills += a2.stats()["apply_spills"]
import bench
from swimhip import ClusterConfig
n = 1024
x = SwimCluster(bench.preset_config("lan"), n, seed=1, gossip_capacity=1 << 17)
y = OracleCluster(bench.preset_config("lan"), n, seed=1)
for c in (x, y):
    c.step(3)
    bench.inject_faults(c, "c3", 3, 1, n=n)
for _ in range(6):
    for c in (x, y):
        c.step(5)
    assert x.digest() == y.digest()
    sx, sy = x.stats(), y.stats()
    assert {{k: sx[k] for k in scenarios.PARITY_KEYS}} == {{k: sy[k] for k in scenarios.PARITY_KEYS}}
spills += x.stats()["apply_spills"]
pairs = a.stats()["apply_pairs"] + a2.stats()["apply_pairs"] + x.stats()["apply_pairs"]
radix = a.stats()["commit_radix"] + x.stats()["commit_radix"]
print("SPILLS", spills, "PAIRS", pairs, "RADIX", radix, "RECORDS", x.stats()["apply_records"])
"""


def _run_variant(name, script):
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib = os.path.join(repo, "variants", name)
    assert os.path.exists(lib), "variant not built: run __graft_entry__.build()"
    paths = [here, repo, os.path.join(repo, "oracle"), os.path.join(repo, "scalecube-cluster_amd")]
    env = dict(os.environ, SWIMHIP_LIB=lib)
    out = subprocess.run([sys.executable, "-c", script.format(paths=paths)], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    return out.stdout


def test_commit_radix_path_parity():
    """Phases that stage more gossips than k_commit's LDS bitonic sort holds (4,096) go through the
    chip-wide radix sort (k_rs_hist, k_rs_pass with decoupled look-back, k_rs_commit). At the
    parity sizes only storm phases get there, so a variant built with a 32-gossip LDS sort
    (-DSWIM_CS_SMALL=32) runs the churn scenario and the C3 storm at N = 1,024 through it: bit-exact
    with the oracle (the radix order must equal the bitonic order up to ties, which are unobservable).
    The variant sorts every batch in the single-launch chain (k_rs_fused, -DSWIM_RS_FUSE_ALL=1: at most
    32 workgroups walking the tiles, grid barriers between the steps), which the product takes for
    gossip rounds; the product's parity runs cover the eleven-launch chain of bigger phases. The
    variant also pulls with one wave per receiver at every size (-DSWIM_PULL_SPLIT_N=0), the product's
    path above 16 rows per CU (4,096) per shard, which it splits over a workgroup's 4 waves below."""
    out = _run_variant("libswimhip_cs32.so", _SPILL_SCRIPT)
    radix = int(out.split("RADIX")[-1].split()[0])
    assert radix > 0, "the chip-wide radix sort never ran"


def test_apply_spill_path_parity():
    """k_gossip_apply's overflow paths (a subject that finds no LDS hash slot within HPROBE probes
    goes through the global inbox and the LDS spill list; the summary walk without compaction when
    the table is at its cap) only run in storm rounds of the full C3 bench with the product's
    16,384-slot hash. A variant built with a 128-slot hash (__graft_entry__.build, -DSWIM_APPLY_HLOG=7)
    takes them in almost every round, and still pairs small receivers (two 64-slot half tables, each
    with half the spill list): it must match the oracle bit for bit, and the spill and pair counters
    prove both paths ran. The same variant gives the batch-slot kernel (k_gossip_apply_b, lossless C3
    part) a 4-subject record dictionary (-DSWIM_DICT_SIDS=4) and a 4-entry spill list: most records
    find no entry, so the bitmap maxima go through the inbox with them (the exactly-once merge of
    DESIGN.md §3.15) and the inbox-row scan runs too."""
    out = _run_variant("libswimhip_hlog7.so", _SPILL_SCRIPT)
    spills = int(out.split("SPILLS")[-1].split()[0])
    pairs = int(out.split("PAIRS")[-1].split()[0])
    assert spills > 0, "the spill path never ran"
    assert pairs > 0, "no receivers were paired"


def test_c3long_schedule_small_parity():
    """SURVEY §8(d)'s C3 variant at N = 1,024: 10 % crash + a 16-member group cut for 120 periods,
    past the suspicion timeout, seeds 0..15 (MembershipProtocolTest.testLongNetworkPartition...
    Removed, :320-371, scaled up). Both sides remove each other, the group rejoins through the
    seeds after the heal, and the crashed members the group never probed stay in its views until
    its own FD reaches them. Digests and counters equal the oracle's every 25 periods for 250."""
    import bench

    n = 1024
    cfg = bench.preset_config("lan").membership(lambda o: o.seedMembers(list(range(16))))
    a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 18)
    b = OracleCluster(cfg, n, seed=1)
    for c in (a, b):
        c.step(3)
        bench.inject_faults(c, "c3long", 3, 1, n=n)
    for _ in range(10):
        for c in (a, b):
            c.step(25)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
    assert 0 < a.stats()["not_converged"] < 1322  # the cut group's unprobed crashed members, draining


def test_refused_set_delay_leaves_the_handle_unchanged():
    """A set_delay the device refuses (a mean whose longest delay, in gossip rounds, would outrun the
    256-round head history) must leave the handle as it was: the live threshold table, the ring
    window and delay_on of the accepted mean. Both sides run 1,000 ms mean delays under 2 % loss
    (LAN: 200 ms rounds; NetworkEmulator.java:189-201 allows any mean); the device then refuses
    3,000 ms with SWIM_EINVAL and must stay bit-exact with the oracle, which never saw the refused
    call. (1 s means need the delayed-message rings sized by memory, not 65,536 entries.)"""
    from swimhip import SwimError

    cfg = ClusterConfig.defaultLanConfig()
    n = 256
    a = SwimCluster(cfg, n, seed=21, event_capacity=1 << 20)
    b = OracleCluster(cfg, n, seed=21, event_capacity=1 << 20)
    for c in (a, b):
        c.set_loss(2.0)
        c.set_delay(1000)
        c.step(3)
    with pytest.raises(SwimError) as ei:
        a.set_delay(3000)
    assert ei.value.code == -22
    crashed = scenarios.crash_ids(n, 3, 21)
    for c in (a, b):
        c.crash(crashed)
    # 12 periods after the crash, compared every 3. The oracle's cost grows with the storm: measured on
    # the build container (one core), 12 periods take 67 s (3.2e8 GossipRequests) and 24 take 230 s
    # (1.0e9), more than a third of the whole -m gpu suite's time, so the comparison stops at 12
    for _ in range(4):
        for c in (a, b):
            c.step(3)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
        assert [e.key() for e in a.events()] == [e.key() for e in b.events()]


@pytest.mark.parametrize("dsub", [None, 16384], ids=["id16", "id32"])
def test_c3_half_partition_1024_matches_oracle(dsub):
    """SURVEY §8(d)'s C3 partition as written (10 % crash, half/half cut by id parity for 40 periods,
    healed by SYNC) at 1,024 members against the oracle: on heal every SYNC / SYNC_ACK re-spreads each
    accepted SUSPECT record (MembershipProtocolImpl.java:649-656), ~5e5 gossips in batch slots whose
    records merge through the record dictionary and the merge marks. Events, counters and digests
    every 5 periods through the heal and the first suspicion timeouts. The default 8,192-block
    dictionary names entries in 16 bits; a 16,384-block one (dict_subjects) in 32.
    The heal's long batch ranges reach their receivers as slot entry bitmaps."""
    def make(cfg, n, seed, **kw):
        return SwimCluster(cfg, n, seed, **({"dict_subjects": dsub} if dsub else {}), **kw)

    a, _ = scenarios.run_pair("c3half1024", make, OracleCluster, compare_every=5, full_tables=False,
                              event_capacity=1 << 22)
    # the heal's long batch ranges were ORed as their slots' entry bitmaps (k_slot_bm), not walked
    assert a.stats()["apply_bitmaps"] > 0


# The sharded rehearsals' shapes of BASELINE configs 3 and 4 (tests/test_sharded.py compares their
# shards with the unsharded handle), pinned to the oracle here: C4's schedule (1 % loss, 0.1 % crash,
# LAN; one gossip per slot) and C5's (64 concurrent crashes, no loss, gossip batches, past the first
# suspicion timeouts) at 4,096 members, dense, and C5's as N x K with K = 256 columns against the
# dense oracle: the many concurrent churn columns C5 is defined by (MembershipProtocolImpl.java:620-647)
@pytest.mark.parametrize("name", ["lan4096_c4_shape", "nxk4096_c5_shape"])
def test_sharded_shapes_match_oracle(name):
    scenarios.run_pair(name, SwimCluster, OracleCluster, compare_every=4)


def test_nxk_k256_64_concurrent_crashes_match_dense_oracle():
    def make_nxk(cfg, n, seed, **kw):
        return SwimCluster(cfg, n, seed, tracked_subjects=256, **kw)

    a, _ = scenarios.run_pair("nxk4096_c5_shape", make_nxk, OracleCluster, compare_every=5)
    st = a.stats()
    assert st["events_removed"] > 200_000  # the 64 columns' suspicion timeouts fired (oracle: 241,919)


# 4-bit infection rounds: the same scenarios with every (member, slot) round kept as
# a 4-bit offset from the slot's creation round and the far ones in the escape table: partitions,
# delays and rejoins put rounds far from creation (escapes), so both paths run
HD4 = ["c1_local32_crash", "lan256_loss5_crash3", "local128_partition_heal", "test64_long_partition_rejoin",
       "local32_asym_partition_loss20", "lan256_leave3_loss5", "local40_restart_join", "local64_delay100_loss10",
       "test48_delay30_partition", "local64_user_gossips_loss10"]


@pytest.mark.parametrize("name", HD4)
def test_scenario_parity_hd4(name):
    def make(cfg, n, seed, **kw):
        return SwimCluster(cfg, n, seed, infection_round_bits=4, **kw)

    scenarios.run_pair(name, make, OracleCluster)


def test_c3_schedule_small_parity_hd4():
    """The C3 storm at N = 1,024 (batched) with 4-bit rounds: the 16-member cut group receives the
    storm's gossips 40 periods after their creation, through the escape table."""
    import bench

    cfg = bench.preset_config("lan")
    n = 1024
    a = SwimCluster(cfg, n, seed=1, gossip_capacity=1 << 17, infection_round_bits=4)
    b = OracleCluster(cfg, n, seed=1)
    for c in (a, b):
        c.step(3)
        bench.inject_faults(c, "c3", 3, 1, n=n)
    for _ in range(12):
        for c in (a, b):
            c.step(5)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
    for i in (0, 64, 333, 1023):
        assert a.debug_holdings(i) == b.debug_holdings(i)
