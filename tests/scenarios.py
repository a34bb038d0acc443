"""Scenario scripts shared by the parity tests, the golden-fixture generator and smoke checks.

Each scenario drives a cluster object (SwimCluster on the GPU or OracleCluster on the CPU)
through the same calls. They restate the reference's test shapes on the discrete replay:
FailureDetectorTest, MembershipProtocolTest, GossipProtocolTest and the BASELINE configs.
"""
from __future__ import annotations

import numpy as np

from swimhip import ClusterConfig, FailureDetectorConfig, GossipConfig, MembershipConfig

PARITY_KEYS = [
    "period", "fd_probes", "fd_direct_ok", "fd_ping_req", "fd_suspect_events", "fd_alive_events",
    "gossips_created", "gossip_first_receipts", "gossip_sends", "syncs_sent", "syncs_delivered",
    "sync_acks_delivered", "records_accepted", "events_added", "events_removed", "suspicion_timeouts",
    "refutations", "not_converged", "infected_suppressed", "fd_dead_events", "events_updated",
]


def crash_ids(n, k, seed):
    rng = np.random.default_rng(seed)
    return sorted(int(x) for x in rng.choice(n, size=k, replace=False))


def test_membership_config():
    """MembershipProtocolTest.java:920-928 (sync 500 ms, ping 200/100 ms, suspicion local)."""
    return (
        ClusterConfig.defaultLocalConfig()
        .membership(lambda o: o.syncInterval(1000).syncTimeout(200))
        .failureDetector(lambda o: o.pingInterval(200).pingTimeout(100))
        .gossip(lambda o: o.gossipInterval(20))
    )


# name -> (config, n, seed, script) ; script(cluster) yields after each step so callers can compare
def _c1(c):
    c.step(10)
    yield
    c.crash(crash_ids(c.n, 1, 1))
    for _ in range(30):
        c.step(1)
        yield


def _lan_loss(c, n_crash, periods, loss, t0=5):
    c.set_loss(loss)
    c.step(t0)
    yield
    c.crash(crash_ids(c.n, n_crash, c.seed))
    for _ in range(periods):
        c.step(1)
        yield


def _c3_half(c, t0, length, after, crash_frac=0.10):
    """SURVEY §8(d)'s C3 partition as written: a simultaneous crash of `crash_frac` of the members
    and a half/half cut by id parity for `length` periods from t0, healed by SYNC (every accepted
    SUSPECT record re-spread, MembershipProtocolImpl.java:649-656), bench.py's c3half schedule."""
    import bench

    c.step(t0)
    yield
    c.crash(bench.crash_set(c.n, crash_frac, c.seed))
    c.partition((np.arange(c.n) % 2).astype(np.uint8), t0, t0 + length)
    for _ in range(length + after):
        c.step(1)
        yield


def _partition_heal(c, t_part, length, after):
    g = (np.arange(c.n) % 2).astype(np.uint8)
    c.partition(g, t_part, t_part + length)
    for _ in range(t_part + length + after):
        c.step(1)
        yield


def _links(c):
    # FailureDetectorTest.testTrustedDespiteBadNetwork (:116-146) + MembershipProtocolTest
    # testMemberLostNetworkDueNoOutboundThenRecover (:140-193) shapes, scaled up
    c.block_outbound(0, [1])
    c.block_outbound(2, range(3, 12))
    for _ in range(6):
        c.step(1)
        yield
    c.unblock_outbound(2, range(3, 12))
    for _ in range(8):
        c.step(1)
        yield


def _asym_partition(c, k, t0, length, after, loss):
    # A small group {0..k-1} cut off past the suspicion timeout, with message loss: the small
    # side's view sizes (and with them gossipPeriodsToSpread / ToSweep, ClusterMath.java:99-113)
    # drop below the large side's, so a sender can still spread a gossip that the peer it got it
    # from has already swept. GossipState.infectedFrom (GossipProtocolImpl.java:181,248) keeps it
    # from re-infecting that peer; the round-1 oracle, which ignored infectedFrom, diverged here
    # (first at period 22: 13,176 vs 13,174 first receipts).
    c.set_loss(loss)
    c.partition((np.arange(c.n) >= k).astype(np.uint8), t0, t0 + length)
    for _ in range(t0 + length + after):
        c.step(1)
        yield


def _inbound(c):
    # NetworkEmulator.blockInbound (NetworkEmulator.java:255-269): member 3 drops everything
    # (blockAllInbound) for 20 periods, member 5 drops member 6's messages, member 9 drops
    # member 0's; an inbound block lets the sender's send succeed, so ping-req subscriptions stay
    # pending instead of failing at once (FailureDetectorImpl.java:183-208).
    c.block_inbound(3, [x for x in range(c.n) if x != 3])
    c.block_inbound(5, [6])
    c.block_inbound(9, [0])
    c.block_outbound(11, [12])
    for _ in range(20):
        c.step(1)
        yield
    c.unblock_inbound(3, [x for x in range(c.n) if x != 3])
    for _ in range(12):
        c.step(1)
        yield


def _leave(c, ids, loss, before, after):
    # Cluster.shutdown() (ClusterImpl.java:370-408): leaveCluster gossips the member's DEAD record
    # (MembershipProtocolImpl.java:203-212); every receiver removes it (onDeadMemberDetected,
    # :571-587) without waiting for a suspicion timeout; the leaver stops once its own sweep
    # drops that gossip (GossipProtocolImpl.java:299-302).
    c.set_loss(loss)
    for _ in range(before):
        c.step(1)
        yield
    c.leave(ids)
    for _ in range(after):
        c.step(1)
        yield


def _churn(c, crash, restart_new, join_new, loss, before=3, mid=4, after=25):
    # Restarts and joins (MembershipProtocolTest.testRestartStoppedMembers / ...OnSameAddresses,
    # :374-520, scaled up): members crash; some restart on their old addresses as new member ids
    # (spare slots), whose replies to pings of the old ids are DEST_GONE (FailureDetectorImpl.java:
    # 231-235); fresh members join on new addresses through the initial SYNC to the seeds
    # (MembershipProtocolImpl.start0, :222-257).
    c.set_loss(loss)
    for _ in range(before):
        c.step(1)
        yield
    c.crash(crash)
    for _ in range(mid):
        c.step(1)
        yield
    c.restart(crash[:len(restart_new)], restart_new)
    c.join(join_new)
    for _ in range(after):
        c.step(1)
        yield


def _metadata(c, loss):
    # Cluster.updateMetadata (ClusterImpl.java:364-367) -> updateIncarnation (MembershipProtocolImpl.
    # java:184-196): the updated members' ALIVE records with incarnation + 1 spread; every member
    # that had them fetches the new metadata and emits UPDATED (:589-610). A second update of one
    # member, a crash in between, and (with loss) fetches that fail and are silently skipped (:540).
    c.set_loss(loss)
    c.step(3)
    yield
    c.update_metadata([3, 10, 20])
    for _ in range(3):
        c.step(1)
        yield
    c.update_metadata([10])
    c.crash([5])
    for _ in range(20):
        c.step(1)
        yield


def _delay(c, mean_ms, loss, n_crash, before, periods, part=0):
    # NetworkEmulator mean delays (NetworkEmulator.java:189-201,358-368):
    # GossipRequests arrive rounds late (and may find their gossip swept), pings / ping-req relays /
    # metadata fetches time out when the round trip is too slow; with loss, a crash and optionally
    # an even/odd partition that heals
    c.set_loss(loss)
    c.set_delay(mean_ms)
    c.step(before)
    yield
    c.crash(crash_ids(c.n, n_crash, c.seed))
    if part:
        c.partition((np.arange(c.n) % 2).astype(np.uint8), before + 2, before + 2 + part)
    for _ in range(periods):
        c.step(1)
        yield


def _user_gossips(c, loss):
    # GossipProtocol.spread (GossipProtocolImpl.java:124-128) of user payloads by several members,
    # two in the same period, one after a crash, under loss: every first receipt is a
    # GossipProtocol.listen() event (SWIM_EV_GOSSIP)
    c.set_loss(loss)
    c.step(2)
    yield
    c.spread(3, 0xA1)
    c.spread(40, 0xB2)
    for _ in range(3):
        c.step(1)
        yield
    c.crash([7])
    c.spread(63, 0xC3)
    for _ in range(12):
        c.step(1)
        yield


SCENARIOS = {
    "c1_local32_crash": (ClusterConfig.defaultLocalConfig(), 32, 1, _c1),
    "lan256_loss5_crash3": (ClusterConfig.defaultLanConfig(), 256, 2, lambda c: _lan_loss(c, 3, 40, 5.0)),
    "local100_loss20": (ClusterConfig.defaultLocalConfig(), 100, 3, lambda c: _lan_loss(c, 2, 30, 20.0)),
    "local128_partition_heal": (
        ClusterConfig.defaultLocalConfig().membership(lambda o: o.syncInterval(3000)),
        128, 4, lambda c: _partition_heal(c, 3, 8, 12)),
    "test64_long_partition_rejoin": (
        test_membership_config().membership(lambda o: o.seedMembers(0, 1, 2, 3)),
        64, 5, lambda c: _partition_heal(c, 2, 30, 25)),
    "local48_links": (ClusterConfig.defaultLocalConfig(), 48, 6, _links),
    "lan1024_loss5_crash10": (ClusterConfig.defaultLanConfig(), 1024, 7, lambda c: _lan_loss(c, 10, 30, 5.0)),
    "local32_asym_partition_loss20": (
        ClusterConfig.defaultLocalConfig().membership(lambda o: o.seedMembers(list(range(32))).syncInterval(2000)),
        32, 0, lambda c: _asym_partition(c, 6, 2, 25, 20, 20.0)),
    "local32_leave2": (ClusterConfig.defaultLocalConfig(), 32, 9, lambda c: _leave(c, [5, 17], 0.0, 3, 12)),
    "lan256_leave3_loss5": (ClusterConfig.defaultLanConfig(), 256, 10, lambda c: _leave(c, [1, 100, 200], 5.0, 4, 30)),
    "local24_inbound_blocks": (
        ClusterConfig.defaultLocalConfig().membership(lambda o: o.seedMembers([0, 1]).syncInterval(2000)),
        24, 8, _inbound),
    # (config, n, seed, script, create kwargs): n_initial < n leaves spare slots for joins/restarts
    "local40_restart_join": (
        ClusterConfig.defaultLocalConfig().membership(lambda o: o.seedMembers([0, 1, 2]).syncInterval(3000)),
        40, 11, lambda c: _churn(c, [3, 7, 20], [32, 33], [34, 35], 0.0), {"n_initial": 32}),
    "local64_update_metadata": (ClusterConfig.defaultLocalConfig(), 64, 14, lambda c: _metadata(c, 0.0)),
    "lan128_update_metadata_loss10": (ClusterConfig.defaultLanConfig(), 128, 15, lambda c: _metadata(c, 10.0)),
    "lan288_restart_join_loss5": (
        ClusterConfig.defaultLanConfig().membership(lambda o: o.seedMembers([0, 1, 2, 3])),
        288, 12, lambda c: _churn(c, [5, 40, 41, 100, 200, 255], [256, 257, 258, 259], [260, 261, 262], 5.0),
        {"n_initial": 256}),
    # message delays: local (gossip 100 ms: P(delay >= 1 round) = e^-1 at 100 ms mean), LAN (200 ms
    # rounds, 500 ms ping timeout), and the MembershipProtocolTest config (20 ms rounds, 100 ms ping
    # timeout: delays of up to ~30 rounds, most ping round trips time out) with a partition
    "local64_delay100_loss10": (ClusterConfig.defaultLocalConfig(), 64, 16, lambda c: _delay(c, 100, 10.0, 2, 3, 25)),
    "lan256_delay200_crash3": (ClusterConfig.defaultLanConfig(), 256, 17, lambda c: _delay(c, 200, 0.0, 3, 3, 30)),
    "local64_user_gossips_loss10": (ClusterConfig.defaultLocalConfig(), 64, 20, lambda c: _user_gossips(c, 10.0)),
    "test48_delay30_partition": (
        test_membership_config().membership(lambda o: o.seedMembers(0, 1)),
        48, 18, lambda c: _delay(c, 30, 5.0, 1, 4, 30, part=8)),
}


# Larger shapes, run only where their cost is the point (sharded rehearsals of BASELINE configs)
SCENARIOS_EXTRA = {
    # the C3 half/half heal at 1,024 members: ~4.96e5 gossips re-spread in the heal's first periods
    # (the oracle needs ~2 minutes)
    "c3half1024": (ClusterConfig.defaultLanConfig(), 1024, 3, lambda c: _c3_half(c, 3, 40, 20)),
    # C4's schedule shape (BASELINE configs[3]: LAN defaults, 1 % loss, 0.1 % simultaneous crash)
    # at 4,096 members
    "lan4096_c4_shape": (ClusterConfig.defaultLanConfig(), 4096, 13, lambda c: _lan_loss(c, 4, 16, 1.0, t0=3)),
    # C5's shape (BASELINE configs[4]: N x K views, concurrent crashes, LAN, no loss: gossip batches)
    # at 4,096 members with 64 crashes, past the first suspicion timeouts (65 periods at b = 13)
    "nxk4096_c5_shape": (ClusterConfig.defaultLanConfig(), 4096, 19, lambda c: _lan_loss(c, 64, 70, 0.0, t0=3)),
    # rings that are not powers of two (ids mod GC, C4's 5,128 x 1,024 slots; tools/probe_ring.py sized
    # them): 20 % loss over 120 periods issues ~14,000 one-gossip slots into 3,072 (the ring wraps ~4
    # times at ~560 live); C2-like loss at 1,024 members keeps ~15,100 of 17,408 slots live at its peak
    "local100_loss20_ring3k": (ClusterConfig.defaultLocalConfig(), 100, 3, lambda c: _lan_loss(c, 2, 120, 20.0),
                               {"gossip_capacity": 3 * 1024}),
    "lan1024_loss5_ring17k": (ClusterConfig.defaultLanConfig(), 1024, 7, lambda c: _lan_loss(c, 10, 30, 5.0),
                              {"gossip_capacity": 17 * 1024}),
}


def scenario(name):
    """(config, n, seed, script, create kwargs) of scenario `name`."""
    cfg, n, seed, script, *kw = SCENARIOS[name] if name in SCENARIOS else SCENARIOS_EXTRA[name]
    return cfg, n, seed, script, (kw[0] if kw else {})


def run_pair(name, make_a, make_b, compare_every=1, full_tables=True, event_capacity=1 << 20):
    """Drive two implementations through scenario `name`, asserting equality as it goes."""
    cfg, n, seed, script, kw = scenario(name)
    a = make_a(cfg, n, seed, event_capacity=event_capacity, **kw)
    b = make_b(cfg, n, seed, event_capacity=event_capacity, **kw)
    ga, gb = script(a), script(b)
    step = 0
    for _ in ga:
        next(gb)
        step += 1
        if step % compare_every:
            continue
        ea = [e.key() for e in a.events()]
        eb = [e.key() for e in b.events()]
        if ea != eb:
            first = next((i for i, (x, y) in enumerate(zip(ea, eb)) if x != y), min(len(ea), len(eb)))
            raise AssertionError(f"{name}: events differ at step {step}, index {first}: "
                                 f"{ea[first:first + 3]} vs {eb[first:first + 3]} (len {len(ea)} vs {len(eb)})")
        sa, sb = a.stats(), b.stats()
        bad = {k: (sa[k], sb[k]) for k in PARITY_KEYS if sa[k] != sb[k]}
        assert not bad, f"{name}: stats differ at step {step}: {bad}"
        assert a.digest() == b.digest(), f"{name}: digests differ at step {step}"
    if full_tables:
        for i in range(n):
            assert np.array_equal(a.view(i), b.view(i)), f"{name}: view row {i} differs"
            assert np.array_equal(a.deadlines(i), b.deadlines(i)), f"{name}: deadline row {i} differs"
        pa, pb = a.presence(), b.presence()
        assert np.array_equal(pa[0], pb[0]) and np.array_equal(pa[1], pb[1])
    return a, b
