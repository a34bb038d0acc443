"""Behavioural restatements of the reference's FD / membership tests on the discrete replay.

Each function takes a cluster factory `make(config, n, seed)` (OracleCluster on the CPU,
SwimCluster on the GPU) and asserts what the reference test asserts, with its wall-clock waits
converted to protocol periods (period = pingInterval). Member a, b, c, d = ids
0, 1, 2, 3. The reference tests wire every member with all addresses as seeds
(MembershipProtocolTest.java:920-928), so the configs here use seedMembers(0..n-1).
"""
from __future__ import annotations

from swimhip import ClusterConfig, FailureDetectorConfig
from swimhip import cluster_math

# MembershipProtocolTest.java:44-45
TEST_SYNC_INTERVAL = 500
PING_INTERVAL = 200


def membership_test_config(n):
    """MembershipProtocolTest.testConfig (:920-928): LAN defaults, sync 500 ms / timeout 100 ms,
    ping 200 / 100 ms, metadataTimeout 100 ms, every member a seed."""
    return (
        ClusterConfig()
        .membership(lambda o: o.seedMembers(list(range(n))).syncInterval(TEST_SYNC_INTERVAL).syncTimeout(100))
        .failureDetector(lambda o: o.pingInterval(PING_INTERVAL).pingTimeout(100))
        .metadataTimeout(100)
    )


def fd_test_config(n):
    """FailureDetectorTest.createFd (:400-407): local preset, timeout 100 / interval 200, pingReq 2."""
    return ClusterConfig.defaultLocalConfig().failureDetector(
        lambda o: FailureDetectorConfig.defaultLocalConfig().pingTimeout(100).pingInterval(200).pingReqMembers(2)
    ).membership(lambda o: o.seedMembers(list(range(n))))


def seconds(s):
    """awaitSeconds(s) (BaseTest.java:33-39) in periods of PING_INTERVAL."""
    return int(s * 1000 // PING_INTERVAL)


def await_suspicion(cluster_size):
    """BaseTest.awaitSuspicion (:41-47): suspicionTimeout(5, size, 200 ms) + 2 s, in periods."""
    ms = cluster_math.suspicionTimeout(5, cluster_size, PING_INTERVAL)
    return seconds(ms // 1000 + 2)


# -- assertion helpers (MembershipProtocolTest.java:1007-1078) ------------------------------
def assert_trusted(c, obs, *expected):
    """ALIVE records = expected + the local member (assertTrusted :1014-1032)."""
    got = sorted(r.member for r in c.membershipRecords(obs) if r.status == "ALIVE")
    assert got == sorted(set(expected) | {obs}), f"member {obs} trusts {got}, expected {sorted(expected)} + self"


def assert_suspected(c, obs, *expected):
    got = sorted(r.member for r in c.membershipRecords(obs) if r.status == "SUSPECT")
    assert got == sorted(expected), f"member {obs} suspects {got}, expected {sorted(expected)}"


def block_outbound(c, src, dsts):
    c.block_outbound(src, [d for d in dsts if d != src])


def unblock_all_outbound(c, src):
    c.unblock_outbound(src, [d for d in range(c.n) if d != src])


A, B, C, D = 0, 1, 2, 3


# -- FailureDetectorTest ------------------------------------------------------------------
def fd_trusted(make):
    """testTrusted (:50-77): clean network, every member keeps the others ALIVE."""
    c = make(fd_test_config(3), 3, 11)
    c.step(6)
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def fd_suspected(make):
    """testSuspected (:79-114): all outbound blocked, every member suspects the others."""
    c = make(fd_test_config(3), 3, 12)
    for m in (A, B, C):
        block_outbound(c, m, (A, B, C))
    c.step(4)
    for m in (A, B, C):
        assert_trusted(c, m)
        assert_suspected(c, m, *[x for x in (A, B, C) if x != m])


def fd_trusted_despite_bad_network(make):
    """testTrustedDespiteBadNetwork (:116-146): A -> B blocked; ping-req through C keeps B ALIVE."""
    c = make(fd_test_config(3), 3, 13)
    block_outbound(c, A, (B,))
    for _ in range(10):
        c.step(1)
        for m in (A, B, C):
            assert_suspected(c, m)


# -- FailureDetectorTest on the FailureDetectorEvent stream (swim_trace, EV_FD) ------------
# The reference asserts the next FailureDetectorEvent each detector publishes about each member
# (listenNextEventFor / assertStatus, FailureDetectorTest.java:444-494). FailureDetectorImpl runs
# alone there; here membership runs on top, with a suspicion timeout and a SYNC interval far past
# every test window, so no member is ever removed and every FD keeps probing every member, as in
# the FD-only test.
def fd_events_config(n, fd=None):
    cfg = fd_test_config(n) if fd is None else ClusterConfig.defaultLocalConfig().failureDetector(
        lambda o: fd).membership(lambda o: o.seedMembers(list(range(n))))
    return cfg.membership(lambda o: o.suspicionMult(1000).syncInterval(10 ** 7))


def next_fd_events(c, members, max_periods=50):
    """listenNextEventFor(fd, members) of every member: the first FailureDetectorEvent each one
    publishes about each other member from now on (awaitEvents waits up to 10 s: max_periods)."""
    c.events()
    want = {(o, s) for o in members for s in members if o != s}
    first = {}
    for _ in range(max_periods):
        c.step(1)
        for e in c.events():
            if e.isFailureDetector() and (e.observer, e.member) in want and (e.observer, e.member) not in first:
                first[(e.observer, e.member)] = e.record
        if len(first) == len(want):
            break
    assert len(first) == len(want), f"no FD event yet for {sorted(want - set(first))}"
    return first


def assert_fd_status(first, obs, status, *expected):
    """assertStatus (:465-487): the members obs's next events give `status` are exactly `expected`."""
    got = sorted(s for (o, s), st in first.items() if o == obs and st == status)
    assert got == sorted(expected), f"member {obs}: {status} events about {got}, expected {sorted(expected)}"


ALIVE_ST, SUSPECT_ST = 1, 2


def fd_events_trusted(make):
    """testTrusted (:50-77): clean network, every next event is ALIVE."""
    c = make(fd_events_config(3), 3, 61)
    c.trace(True)
    first = next_fd_events(c, (A, B, C))
    for m in (A, B, C):
        assert_fd_status(first, m, ALIVE_ST, *[x for x in (A, B, C) if x != m])


def fd_events_suspected(make):
    """testSuspected (:79-114): every member blocks all its outbound traffic: every event SUSPECT."""
    c = make(fd_events_config(3), 3, 62)
    c.trace(True)
    for m in (A, B, C):
        block_outbound(c, m, (A, B, C))
    first = next_fd_events(c, (A, B, C))
    for m in (A, B, C):
        assert_fd_status(first, m, SUSPECT_ST, *[x for x in (A, B, C) if x != m])


def fd_events_trusted_despite_bad_network(make):
    """testTrustedDespiteBadNetwork (:116-146): a -> b blocked; the ping-req through c keeps every
    event ALIVE."""
    c = make(fd_events_config(3), 3, 63)
    c.trace(True)
    block_outbound(c, A, (B,))
    first = next_fd_events(c, (A, B, C))
    for m in (A, B, C):
        assert_fd_status(first, m, ALIVE_ST, *[x for x in (A, B, C) if x != m])


def fd_events_trusted_despite_different_ping_timings(make):
    """testTrustedDespiteDifferentPingTimings (:148-176): b and c run FailureDetectorConfig
    defaults (ping 1,000 / timeout 500). The simulator steps every member with one config, so the
    whole cluster runs the defaults: clean network, every next event ALIVE."""
    c = make(fd_events_config(3, FailureDetectorConfig.defaultConfig()), 3, 64)
    c.trace(True)
    first = next_fd_events(c, (A, B, C))
    for m in (A, B, C):
        assert_fd_status(first, m, ALIVE_ST, *[x for x in (A, B, C) if x != m])


def fd_events_suspected_member_with_bad_network(make):
    """testSuspectedMemberWithBadNetworkGetsPartitioned (:178-236): a blocks its outbound traffic
    to everyone: a suspects b, c, d; each of them suspects a only. After unblocking and 4 s, every
    next event is ALIVE."""
    n = 4
    c = make(fd_events_config(n), n, 65)
    c.trace(True)
    block_outbound(c, A, (A, B, C, D))
    first = next_fd_events(c, (A, B, C, D))
    assert_fd_status(first, A, SUSPECT_ST, B, C, D)
    for m in (B, C, D):
        assert_fd_status(first, m, SUSPECT_ST, A)
    unblock_all_outbound(c, A)
    c.step(seconds(4))
    first = next_fd_events(c, (A, B, C, D))
    for m in (A, B, C, D):
        assert_fd_status(first, m, ALIVE_ST, *[x for x in (A, B, C, D) if x != m])


def fd_events_suspected_member_with_normal_network(make):
    """testSuspectedMemberWithNormalNetworkGetsPartitioned (:238-299): a, b, c block their traffic
    to d: they suspect d, d suspects all three (its acks come back through them). After
    unblocking and 4 s, every next event is ALIVE."""
    n = 4
    c = make(fd_events_config(n), n, 66)
    c.trace(True)
    for m in (A, B, C):
        block_outbound(c, m, (D,))
    first = next_fd_events(c, (A, B, C, D))
    for m in (A, B, C):
        assert_fd_status(first, m, SUSPECT_ST, D)
    assert_fd_status(first, D, SUSPECT_ST, A, B, C)
    for m in (A, B, C):
        unblock_all_outbound(c, m)
    c.step(seconds(4))
    first = next_fd_events(c, (A, B, C, D))
    for m in (A, B, C, D):
        assert_fd_status(first, m, ALIVE_ST, *[x for x in (A, B, C, D) if x != m])


def fd_events_status_change_after_network_recovery(make):
    """testMemberStatusChangeAfterNetworkRecovery (:301-341): a and b block each other: both
    suspect; unblocked, within 2 s both are ALIVE again."""
    c = make(fd_events_config(2), 2, 67)
    c.trace(True)
    block_outbound(c, A, (B,))
    block_outbound(c, B, (A,))
    first = next_fd_events(c, (A, B))
    assert_fd_status(first, A, SUSPECT_ST, B)
    assert_fd_status(first, B, SUSPECT_ST, A)
    unblock_all_outbound(c, A)
    unblock_all_outbound(c, B)
    c.step(seconds(2))
    first = next_fd_events(c, (A, B))
    assert_fd_status(first, A, ALIVE_ST, B)
    assert_fd_status(first, B, ALIVE_ST, A)


# -- MembershipProtocolTest ---------------------------------------------------------------
def mp_initial_phase_ok(make):
    """testInitialPhaseOk (:68-91)."""
    c = make(membership_test_config(3), 3, 21)
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def mp_partition_no_outbound_then_recover(make):
    """testNetworkPartitionDueNoOutboundThenRecover (:93-137): everyone isolated until removed,
    then unblocked: SYNC to the seeds brings everyone back."""
    c = make(membership_test_config(3), 3, 22)
    c.step(seconds(3))
    for m in (A, B, C):
        block_outbound(c, m, (A, B, C))
    c.step(await_suspicion(3))
    for m in (A, B, C):
        assert_trusted(c, m)  # assertSelfTrusted
        assert_suspected(c, m)
    removed = {(e.observer, e.member) for e in c.events() if e.isRemoved()}
    assert removed == {(o, s) for o in (A, B, C) for s in (A, B, C) if o != s}
    for m in (A, B, C):
        unblock_all_outbound(c, m)
    c.step(seconds(TEST_SYNC_INTERVAL * 2 / 1000))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def mp_member_lost_network_then_recover(make):
    """testMemberLostNetworkDueNoOutboundThenRecover (:139-193)."""
    c = make(membership_test_config(3), 3, 23)
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
    block_outbound(c, B, (A, C))
    block_outbound(c, A, (B,))
    block_outbound(c, C, (B,))
    c.step(seconds(1))
    assert_trusted(c, A, C)
    assert_suspected(c, A, B)
    assert_trusted(c, B)
    assert_suspected(c, B, A, C)
    assert_trusted(c, C, A)
    assert_suspected(c, C, B)
    for m in (A, B, C):
        unblock_all_outbound(c, m)
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def mp_partition_twice_then_recover(make):
    """testNetworkPartitionTwiceDueNoOutboundThenRecover (:195-263)."""
    c = make(membership_test_config(3), 3, 24)
    c.step(seconds(1))
    block_outbound(c, B, (A, C))
    block_outbound(c, A, (B,))
    block_outbound(c, C, (B,))
    c.step(seconds(1))
    assert_trusted(c, A, C)
    assert_suspected(c, A, B)
    assert_trusted(c, B)
    assert_suspected(c, B, A, C)
    block_outbound(c, A, (C,))
    block_outbound(c, C, (A,))
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m)
        assert_suspected(c, m, *[x for x in (A, B, C) if x != m])
    for m in (A, B, C):
        unblock_all_outbound(c, m)
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def mp_network_lost_on_all_nodes_then_recover(make):
    """testNetworkLostOnAllNodesDueNoOutboundThenRecover (:265-318)."""
    c = make(membership_test_config(3), 3, 25)
    c.step(seconds(1))
    for m in (A, B, C):
        block_outbound(c, m, (A, B, C))
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m)
        assert_suspected(c, m, *[x for x in (A, B, C) if x != m])
    for m in (A, B, C):
        unblock_all_outbound(c, m)
    c.step(seconds(1))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
        assert_suspected(c, m)


def mp_long_partition_then_removed(make):
    """testLongNetworkPartitionDueNoOutboundThenRemoved (:320-371): {a,b} | {c,d} until the
    suspicion timeout removes the other side."""
    c = make(membership_test_config(4), 4, 26)
    c.step(seconds(1))
    for m in (A, B, C, D):
        assert_trusted(c, m, *[x for x in (A, B, C, D) if x != m])
    block_outbound(c, A, (C, D))
    block_outbound(c, B, (C, D))
    block_outbound(c, C, (A, B))
    block_outbound(c, D, (A, B))
    c.step(seconds(2))
    assert_trusted(c, A, B)
    assert_suspected(c, A, C, D)
    assert_trusted(c, B, A)
    assert_suspected(c, B, C, D)
    assert_trusted(c, C, D)
    assert_suspected(c, C, A, B)
    assert_trusted(c, D, C)
    assert_suspected(c, D, A, B)
    c.step(await_suspicion(4))
    assert_trusted(c, A, B)
    assert_suspected(c, A)
    assert_trusted(c, B, A)
    assert_suspected(c, B)
    assert_trusted(c, C, D)
    assert_suspected(c, C)
    assert_trusted(c, D, C)
    assert_suspected(c, D)


# -- MembershipProtocolTest, inbound-only blocks (:681-918) --------------------------------
# (testNodeJoinClusterWithNoInbound / ...ThenInboundRecover, :597-679, start members that join
# through INITIAL_SYNC; the simulator's members start converged, so those two are not restated.)
def seeds_a_config(n):
    """The inbound tests wire b and c with seed a only (createMembership(x, [a.address()]))."""
    return membership_test_config(n).membership(lambda o: o.seedMembers([A]))


def block_all_inbound(c, dst):
    """NetworkEmulator.blockAllInbound (:237-242) of member dst."""
    c.block_inbound(dst, [x for x in range(c.n) if x != dst])


def unblock_all_inbound(c, dst):
    c.unblock_inbound(dst, [x for x in range(c.n) if x != dst])


def removed_by(c):
    out = {}
    for e in c.events():
        if e.isRemoved():
            out.setdefault(e.observer, set()).add(e.member)
    return out


def mp_partition_no_inbound_then_removed(make, recover=False):
    """testNetworkPartitionDueNoInboundThenRemoved (:681-720): c drops every inbound message; a
    and b remove c, c removes a and b, and nobody stays suspected. With recover=True,
    testNetworkPartitionDueNoInboundUntilRemovedThenInboundRecover (:722-775): after unblocking,
    SYNC to the seed brings all three back."""
    c = make(seeds_a_config(3), 3, 31 if not recover else 32)
    c.step(seconds(3))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
    c.events()
    block_all_inbound(c, C)
    c.step(await_suspicion(3))
    assert_trusted(c, A, B)
    assert_suspected(c, A)
    assert_trusted(c, B, A)
    assert_suspected(c, B)
    assert_trusted(c, C)
    assert_suspected(c, C)
    rem = removed_by(c)
    assert rem.get(A) == {C} and rem.get(B) == {C} and rem.get(C) == {A, B}, rem
    if recover:
        unblock_all_inbound(c, C)
        c.step(seconds(3))
        for m in (A, B, C):
            assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
            assert_suspected(c, m)


def mp_partition_no_inbound_then_recover(make):
    mp_partition_no_inbound_then_removed(make, recover=True)


def mp_between_two_members(make, mode):
    """testNetworkPartitionBetweenTwoMembersDueNoInbound / NoOutbound / NoTrafficAtAll
    (:777-851): c blocks b's inbound, outbound or both; ping-req through a keeps everyone
    trusted for a whole suspicion timeout."""
    c = make(seeds_a_config(3), 3, {"in": 33, "out": 34, "both": 35}[mode])
    c.step(seconds(3))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])
    if mode in ("in", "both"):
        c.block_inbound(C, [B])
    if mode in ("out", "both"):
        c.block_outbound(C, [B])
    c.step(await_suspicion(3))
    for m in (A, B, C):
        assert_trusted(c, m, *[x for x in (A, B, C) if x != m])


def mp_between_two_members_no_inbound(make):
    mp_between_two_members(make, "in")


def mp_between_two_members_no_outbound(make):
    mp_between_two_members(make, "out")


def mp_between_two_members_no_traffic(make):
    mp_between_two_members(make, "both")


def mp_partition_many_no_inbound_then_recover(make):
    """testNetworkPartitionManyDueNoInboundThenRemovedThenRecover (:853-918): all four drop all
    inbound, suspect then remove each other, then recover once unblocked."""
    c = make(membership_test_config(4), 4, 36)
    c.step(seconds(1))
    for m in (A, B, C, D):
        assert_trusted(c, m, *[x for x in (A, B, C, D) if x != m])
        assert_suspected(c, m)
    c.events()
    for m in (A, B, C, D):
        block_all_inbound(c, m)
    c.step(seconds(2))
    for m in (A, B, C, D):
        assert_trusted(c, m)
        assert_suspected(c, m, *[x for x in (A, B, C, D) if x != m])
    c.step(await_suspicion(4))
    rem = removed_by(c)
    for m in (A, B, C, D):
        assert rem.get(m) == {x for x in (A, B, C, D) if x != m}, rem
    for m in (A, B, C, D):
        unblock_all_inbound(c, m)
    c.step(seconds(3))
    for m in (A, B, C, D):
        assert_trusted(c, m, *[x for x in (A, B, C, D) if x != m])
        assert_suspected(c, m)


def cluster_shutdown_removed(make):
    """ClusterTest.testMembershipEventsOnShutdown shape (:357-470): after node.shutdown() every
    other member emits REMOVED for it, through the leave gossip, long before a suspicion timeout
    could have fired; the leaver stops (no longer trusted by anyone, nobody suspects it)."""
    n = 8
    cfg = ClusterConfig.defaultLocalConfig()
    c = make(cfg, n, 41)
    c.step(2)
    c.events()
    c.leave([B])
    c.step(2)  # the DEAD gossip reaches everyone within a couple of periods (10 rounds each)
    evs = c.events()
    rem = {}
    for e in evs:
        if e.isRemoved():
            rem.setdefault(e.observer, set()).add(e.member)
    assert all(rem.get(m) == {B} for m in range(n) if m != B), rem
    # removed through the leave's DEAD record (gossip, or a SYNC carrying it), never by a
    # suspicion timeout (MembershipProtocolImpl.java:203-212, :571-587)
    assert all(e.reason in (1, 2) for e in evs if e.isRemoved()), [e for e in evs if e.isRemoved()]
    susp = cluster_math.suspicionTimeout(cfg.membershipConfig().suspicionMult(), n, 1)
    c.step(susp + 5)
    for m in range(n):
        if m != B:
            assert B not in c.members(m)
            assert_suspected(c, m)


def gossip_dissemination_bound(make):
    """GossipProtocolTest (:48-64, :154-161) restated on membership gossip: the SUSPECT gossip
    about a crashed member reaches every alive member within gossipTimeoutToSweep rounds, with
    loss 0..50 %; every member then removes it within the suspicion timeout + sweep bound."""
    for n, loss in ((10, 0.0), (50, 10.0), (50, 25.0), (50, 50.0)):
        cfg = ClusterConfig.defaultLocalConfig()
        c = make(cfg, n, 100 + n + int(loss))
        c.set_loss(loss)
        c.step(2)
        c.crash([n - 1])
        g = cfg.gossipConfig()
        rounds_per_period = cfg.failureDetectorConfig().pingInterval() // g.gossipInterval()
        sweep_rounds = cluster_math.gossipPeriodsToSweep(g.gossipRepeatMult(), n)
        susp = cluster_math.suspicionTimeout(cfg.membershipConfig().suspicionMult(), n, 1)
        bound = susp + sweep_rounds // rounds_per_period + 10
        for _ in range(bound):
            c.step(1)
            if all(c.view(o)[n - 1] == 0 for o in range(n - 1)):
                break
        assert all(c.view(o)[n - 1] == 0 for o in range(n - 1)), (n, loss)


# -- GossipProtocolTest (:48-64 grid, asserts :154, :155-161, :173) ------------------------
# (N, loss %, mean delay ms) of the reference's experiments, delays included: a
# GossipRequest is handled delay // gossipInterval rounds after it was sent
GOSSIP_GRID = [(2, 0, 2), (2, 0, 2), (3, 0, 2), (5, 0, 2), (10, 0, 2), (10, 10, 2), (10, 25, 2), (10, 25, 100),
               (10, 50, 2), (50, 0, 2), (50, 10, 2), (50, 10, 100)]


def gossip_test_config(n):
    """GossipProtocolTest.initGossipProtocol (:258-263): GossipConfig defaults (fanout 3, interval
    200 ms, repeat mult 3). The test runs GossipProtocolImpl alone on a fixed member list; here
    membership runs too, with no removal and no SYNC inside the window (the member list stays
    fixed, as there)."""
    return ClusterConfig.defaultLanConfig().membership(lambda o: o.suspicionMult(1000).syncInterval(10 ** 7))


def gossip_protocol_grid(make):
    """testGossipProtocol (:110-208): member 0 spreads one gossip; every other member receives it
    (:154) within gossipTimeoutToSweep (:155-161), and no member has it delivered twice (:173),
    over the whole gossip lifetime plus three intervals (awaitFullCompletion, :163-169)."""
    for idx, (n, loss, delay) in enumerate(GOSSIP_GRID):
        cfg = gossip_test_config(n)
        g = cfg.gossipConfig()
        interval = g.gossipInterval()
        rounds_per_period = cfg.failureDetectorConfig().pingInterval() // interval
        c = make(cfg, n, 300 + idx)
        c.set_loss(loss)
        c.set_delay(delay)
        c.step(1)
        c.events()
        tag = 0x5EED0000 + idx
        p0 = c.stats()["period"]
        c.spread(0, tag)  # created for round p0 * G (the next period's first round)
        timeout_ms = cluster_math.gossipTimeoutToSweep(g.gossipRepeatMult(), n, interval)
        # the latch waits 2 x gossipTimeout (:152); then the rest of the lifetime + 3 intervals
        total_rounds = 2 * timeout_ms // interval + 3
        first, double = {}, []
        for _ in range((total_rounds + rounds_per_period - 1) // rounds_per_period):
            c.step(1)
            for e in c.events():
                if e.isGossip() and e.record == tag and e.member == 0:
                    r = e.period * rounds_per_period + e.phase - 1  # the round it arrived in
                    if e.observer in first:
                        double.append(e.observer)
                    else:
                        first[e.observer] = r
        assert set(first) == set(range(1, n)), (n, loss, "Not all members received gossip")
        # dissemination time: spread to the end of the round the last member got it in
        dissem_ms = (max(first.values()) + 1 - p0 * rounds_per_period) * interval if first else 0
        assert dissem_ms < timeout_ms, (n, loss, f"Too long dissemination time {dissem_ms}ms (timeout {timeout_ms}ms)")
        assert not double, (n, loss, "Delivered gossip twice to same member", double)


def mp_restart_stopped_members(make):
    """testRestartStoppedMembers (:374-451): c and d stop; a and b suspect, then remove them; new
    members start on new addresses (spare ids 4 and 5) with the four old addresses as seeds and
    join through the initial SYNC: everyone trusts everyone, nobody is suspected."""
    c = make(membership_test_config(4), 6, 51, n_initial=4)
    c.step(seconds(1))
    for m in (A, B, C, D):
        assert_trusted(c, m, *[x for x in (A, B, C, D) if x != m])
    c.events()
    c.crash([C, D])
    c.step(seconds(1))
    for m, o in ((A, B), (B, A)):
        assert_trusted(c, m, o)
        assert_suspected(c, m, C, D)
    c.step(await_suspicion(4))
    rem = removed_by(c)
    for m, o in ((A, B), (B, A)):
        assert_trusted(c, m, o)
        assert_suspected(c, m)
        assert rem.get(m) == {C, D}, rem
    c2, d2 = 4, 5
    c.join([c2, d2])
    c.step(seconds(2))
    for m in (A, B, c2, d2):
        assert_trusted(c, m, *[x for x in (A, B, c2, d2) if x != m])
        assert_suspected(c, m)


def mp_restart_on_same_addresses(make):
    """testRestartStoppedMembersOnSameAddresses (:453-520): c and d stop and are suspected; new
    members (new ids 4 and 5) start on c's and d's addresses. A ping to the old ids now reaches the
    new members, which answer DEST_GONE (FailureDetectorImpl.java:231-235): a and b remove the old
    ids without waiting for the suspicion timeout, and everyone trusts the new ones."""
    c = make(membership_test_config(4), 6, 52, n_initial=4)
    c.step(seconds(1))
    for m in (A, B, C, D):
        assert_trusted(c, m, *[x for x in (A, B, C, D) if x != m])
    c.events()
    c.crash([C, D])
    c.step(seconds(1))
    for m, o in ((A, B), (B, A)):
        assert_trusted(c, m, o)
        assert_suspected(c, m, C, D)
    c2, d2 = 4, 5
    c.restart([C, D], [c2, d2])
    c.step(seconds(2))
    assert seconds(3) < await_suspicion(4)  # the removals below cannot be suspicion timeouts
    rem = removed_by(c)
    for m in (A, B, c2, d2):
        assert_trusted(c, m, *[x for x in (A, B, c2, d2) if x != m])
        assert_suspected(c, m)
    for m in (A, B):
        assert rem.get(m) == {C, D}, rem
    assert c.stats()["fd_dead_events"] > 0


ALL = [
    fd_trusted, fd_suspected, fd_trusted_despite_bad_network,
    fd_events_trusted, fd_events_suspected, fd_events_trusted_despite_bad_network,
    fd_events_trusted_despite_different_ping_timings, fd_events_suspected_member_with_bad_network,
    fd_events_suspected_member_with_normal_network, fd_events_status_change_after_network_recovery,
    gossip_protocol_grid,
    mp_initial_phase_ok, mp_partition_no_outbound_then_recover, mp_member_lost_network_then_recover,
    mp_partition_twice_then_recover, mp_network_lost_on_all_nodes_then_recover, mp_long_partition_then_removed,
    mp_partition_no_inbound_then_removed, mp_partition_no_inbound_then_recover, mp_between_two_members_no_inbound,
    mp_between_two_members_no_outbound, mp_between_two_members_no_traffic, mp_partition_many_no_inbound_then_recover,
    cluster_shutdown_removed, gossip_dissemination_bound, mp_restart_stopped_members, mp_restart_on_same_addresses,
]
