"""The wire-format bridge (swimhip/wire.py): the reference's JSON messages and
framing, and real-node messages delivered into the simulation (swim_deliver_records).

Byte-level parity with Jackson is unpinned (no JVM in the image); these restate the reference's own
codec tests as round trips — GossipRequestTest.testSerializationAndDeserialization (:38-67) and
JacksonMessageCodecTest's ByteBuffer cases (:21-69) — plus the DefaultObjectMapper conventions
(DefaultObjectMapper.java:20-31) and the framing (TransportImpl.java:383-397)."""
import json
import os

import numpy as np
import pytest

import scenarios
from oracle_py import OracleCluster
from swimhip import ClusterConfig, SwimCluster, wire
from swimhip import _native as nat


def _member(i):
    return wire.Member(f"m{i}", wire.Address("localhost", 1234 + i))


def test_gossip_request_round_trip():
    """GossipRequestTest (:38-67): a GossipRequest of two gossips whose messages carry an application
    object (qualifier "scalecube/testData") keeps its class, its correlation id and the payload."""
    test_data = wire.Opaque("io.scalecube.cluster.gossip.GossipRequestTest$TestData",
                            {"@class": "io.scalecube.cluster.gossip.GossipRequestTest$TestData",
                             "properties": {"key": "123"}})
    gossips = [wire.Gossip(gid, wire.Message({wire.HEADER_QUALIFIER: "scalecube/testData"}, test_data))
               for gid in ("idGossip", "idGossip2")]
    msg = wire.Message({wire.HEADER_CORRELATION_ID: "CORR_ID"}, wire.GossipRequest(gossips, "0"))
    out = wire.encode(msg)
    assert len(out) > 0
    back = wire.decode(out)
    assert isinstance(back.data, wire.GossipRequest)
    assert back.correlationId == "CORR_ID"
    g0 = back.data.gossips[0]
    assert isinstance(g0.message.data, wire.Opaque)
    assert g0.message.data.cls.endswith("GossipRequestTest$TestData")
    assert g0.message.data.body["properties"] == {"key": "123"}
    assert back == msg


@pytest.mark.parametrize("n", [0, 5, 512])
def test_metadata_bytes_round_trip(n):
    """JacksonMessageCodecTest (:21-69): a ByteBuffer (here GetMetadataResponse.metadata) survives
    encode/decode, empty and 512 random bytes included; Jackson writes it as base64."""
    payload = os.urandom(n) if n != 5 else b"hello"
    msg = wire.Message({wire.HEADER_QUALIFIER: wire.GET_METADATA_RESP, wire.HEADER_CORRELATION_ID: "7"},
                       wire.GetMetadataResponse(_member(3), payload))
    back = wire.decode(wire.encode(msg))
    assert back.data.metadata == payload
    assert back == msg


def test_default_object_mapper_conventions():
    """DefaultObjectMapper (:20-31): "@class" on the Object-typed data, enums by toString, is-getters
    as properties, NON_NULL, HashMap header order ("q" before "cid"), unknown properties ignored."""
    rec = wire.MembershipRecord(_member(1), "SUSPECT", 4)
    msg = wire.Message({wire.HEADER_CORRELATION_ID: "c1", wire.HEADER_QUALIFIER: wire.SYNC},
                       wire.SyncData([rec], "default"))
    o = json.loads(wire.encode(msg))
    assert list(o["headers"]) == ["q", "cid"]
    assert "sender" not in o
    assert list(o["data"])[0] == "@class" and o["data"]["@class"] == wire.CLS_SYNC_DATA
    r = o["data"]["membership"][0]
    assert r["status"] == "SUSPECT" and r["incarnation"] == 4
    assert (r["alive"], r["suspect"], r["dead"]) == (False, True, False)
    # a newer node's extra property is ignored on read
    o["data"]["membership"][0]["future"] = 1
    assert wire.decode(json.dumps(o).encode()).data.membership[0] == rec
    ping = wire.Message({wire.HEADER_QUALIFIER: wire.PING, wire.HEADER_CORRELATION_ID: "5"},
                        wire.PingData(_member(0), _member(2)))
    po = json.loads(wire.encode(ping))["data"]
    assert "originalIssuer" not in po and "ackType" not in po
    ack = wire.decode(wire.encode(wire.Message({wire.HEADER_QUALIFIER: wire.PING_ACK},
                                               wire.PingData(_member(0), _member(2), _member(1), "DEST_GONE"))))
    assert ack.data.ackType == "DEST_GONE" and ack.data.originalIssuer == _member(1)


def test_framing_split_and_coalesced():
    msgs = [wire.encode(wire.Message({wire.HEADER_QUALIFIER: wire.PING}, wire.PingData(_member(i), _member(i + 1))))
            for i in range(5)]
    stream = b"".join(wire.frame(m) for m in msgs)
    dec = wire.FrameDecoder()
    got = []
    rng = np.random.default_rng(3)
    pos = 0
    while pos < len(stream):  # arbitrary TCP segmentation
        k = int(rng.integers(1, 40))
        got += dec.feed(stream[pos:pos + k])
        pos += k
    assert got == msgs
    with pytest.raises(wire.WireError):
        wire.FrameDecoder(max_frame=16).feed(wire.frame(b"x" * 17))


def test_packed_records_round_trip():
    d = wire.Directory(4)
    for cell in (nat.pack(0, nat.ALIVE), nat.pack(7, nat.SUSPECT), nat.DEAD, nat.pack((1 << 30) - 1, nat.ALIVE)):
        r = wire.MembershipRecord.from_packed(d[2], cell)
        assert r.packed() == cell
        assert wire.MembershipRecord.from_json(json.loads(json.dumps(r.to_json()))) == r
    with pytest.raises(wire.WireError):
        wire.MembershipRecord(d[1], "ALIVE", -1).packed()
    with pytest.raises(wire.WireError):
        wire.MembershipRecord.from_packed(d[1], nat.ABSENT)


def _external_sync(directory, n, inc_of, status_of, group="default"):
    recs = [wire.MembershipRecord(directory[j], status_of(j), inc_of(j)) for j in range(n)]
    return wire.Message({wire.HEADER_QUALIFIER: wire.SYNC}, wire.SyncData(recs, group))


def test_sync_from_a_real_node_into_the_oracle():
    """A real node's SYNC, framed and decoded, delivered to simulated member 0 of the oracle: every
    record goes through updateMembership with reason SYNC — a SUSPECT about member 5 overrides ALIVE
    inc 0 and is re-spread as a gossip, a SUSPECT about member 0 itself makes it refute (incarnation
    + 1, spread), a foreign sync group is ignored. The simulated member's own SYNC_ACK then carries
    the merged table back."""
    cfg = ClusterConfig.defaultLocalConfig()
    n = 16
    d = wire.Directory(n)
    c = OracleCluster(cfg, n, seed=4, event_capacity=1 << 12)
    c.step(2)
    msg = _external_sync(d, n, lambda j: 0, lambda j: "SUSPECT" if j in (0, 5) else "ALIVE")
    got = wire.FrameDecoder().feed(wire.frame(wire.encode(msg)))
    assert len(got) == 1
    foreign = _external_sync(d, n, lambda j: 0, lambda j: "SUSPECT", group="other")
    assert wire.deliver(c, 0, foreign, d) == 0
    before = c.stats()
    assert wire.deliver(c, 0, wire.decode(got[0]), d) == n
    after = c.stats()
    row = c.view(0)
    assert row[5] == nat.pack(0, nat.SUSPECT)
    assert row[0] == nat.pack(1, nat.ALIVE)  # refuted
    assert after["refutations"] == before["refutations"] + 1
    assert after["gossips_created"] == before["gossips_created"] + 2  # the SUSPECT and the refutation
    ack = wire.sync_message(c, 0, d, wire.SYNC_ACK, cid="9")
    back = wire.decode(wire.encode(ack))
    assert back.correlationId == "9" and back.qualifier == wire.SYNC_ACK
    assert [r.packed() for r in back.data.membership] == [int(x) for x in row if x]
    c.step(3)  # the spread SUSPECT reaches member 5, which refutes it: everyone ends at ALIVE inc 1
    assert c.view(5)[5] == nat.pack(1, nat.ALIVE)
    assert sum(1 for i in range(n) if c.view(i)[5] == nat.pack(1, nat.ALIVE)) == n


def test_gossip_request_is_forwarded_once_per_id():
    """GossipProtocolImpl.onGossipReq (:171-183) on the bridge: a real node's membership gossip with
    a new id is put into the simulated member's gossips (forwarded to simulated peers in the coming
    rounds, a gossip the observer created) and handed to membership once; the same id from a second
    real peer is dropped; once the observer's sweep drops the id (gossipPeriodsToSweep) a copy counts
    as new again."""
    cfg = ClusterConfig.defaultLocalConfig()
    n = 16
    d = wire.Directory(n)
    c = OracleCluster(cfg, n, seed=5, event_capacity=1 << 12)
    c.step(2)
    gossip = wire.membership_gossip_request(d, 9, 0, wire.MembershipRecord(d[7], "SUSPECT", 0))
    before = c.stats()["gossips_created"]
    seq0 = c.debug_member_state()["gossip_seq"].copy()
    assert wire.deliver(c, 3, gossip, d) == 1
    assert c.stats()["gossips_created"] == before + 1  # the forwarded copy
    # the forward keeps the real node's id namespace: member 3's gossipCounter (GPI:48) does not move, so
    # the ids of the gossips it creates itself later are the reference's
    assert np.array_equal(c.debug_member_state()["gossip_seq"], seq0)
    assert c.view(3)[7] == nat.pack(0, nat.SUSPECT)
    assert wire.deliver(c, 3, gossip, d) == 0  # a repeat of a held id
    assert c.stats()["gossips_created"] == before + 1
    c.step(1)  # the forward reaches the other simulated members (10 rounds per local period)
    assert sum(1 for i in range(n) if c.view(i)[7] in (nat.pack(0, nat.SUSPECT), nat.pack(1, nat.ALIVE))) == n
    c.step(wire._sweep_periods(c, 3))
    assert wire.deliver(c, 3, gossip, d) == 1  # swept: new again


def test_sync_ack_with_correlation_id_is_dropped():
    """MembershipProtocolImpl.onMessage (:331-334) ignores a SYNC_ACK carrying a correlation id (only
    start0's initial sync consumes one); a SYNC_ACK without one is onSyncAck (:343-349)."""
    cfg = ClusterConfig.defaultLocalConfig()
    n = 8
    d = wire.Directory(n)
    c = OracleCluster(cfg, n, seed=6, event_capacity=1 << 12)
    c.step(1)
    recs = [wire.MembershipRecord(d[j], "SUSPECT" if j == 4 else "ALIVE", 0) for j in range(n)]
    with_cid = wire.Message({wire.HEADER_QUALIFIER: wire.SYNC_ACK, wire.HEADER_CORRELATION_ID: "3"},
                            wire.SyncData(recs))
    assert wire.deliver(c, 1, with_cid, d) == 0
    assert c.view(1)[4] == nat.pack(0, nat.ALIVE)
    plain = wire.Message({wire.HEADER_QUALIFIER: wire.SYNC_ACK}, wire.SyncData(recs))
    assert wire.deliver(c, 1, plain, d) == n
    assert c.view(1)[4] == nat.pack(0, nat.SUSPECT)


def test_membership_gossip_request_round_trip():
    d = wire.Directory(8)
    rec = wire.MembershipRecord(d[3], "SUSPECT", 2)
    msg = wire.membership_gossip_request(d, 1, 17, rec)
    back = wire.decode(wire.encode(msg))
    g = back.data.gossips[0]
    assert g.gossipId == "sim-1-17" and back.data.from_ == "sim-1"
    assert g.message.qualifier == wire.MEMBERSHIP_GOSSIP and g.message.data == rec


@pytest.mark.gpu
@pytest.mark.parametrize("tracked", [0, 48])
def test_delivered_records_match_oracle(tracked):
    """swim_deliver_records on the GPU equals the oracle's: a real node's SYNC (SUSPECTs, a self
    SUSPECT that forces refutation, an ALIVE of higher incarnation, a DEAD) and a membership-gossip
    GossipRequest delivered between periods (forwarded by the receiving member, its repeat dropped),
    under 10 % loss (metadata fetches draw), then 12 periods
    stepped: tables, deadlines, events and counters bit-exact (dense, and N x K with 48 columns: 10 % loss over 14
    periods takes ~20 of the 64 subjects off the baseline)."""
    cfg = ClusterConfig.defaultLocalConfig()
    n = 64
    d = wire.Directory(n)
    kw = {"tracked_subjects": tracked} if tracked else {}
    a = SwimCluster(cfg, n, seed=11, event_capacity=1 << 16, **kw)
    b = OracleCluster(cfg, n, seed=11, event_capacity=1 << 16)
    st = {3: ("SUSPECT", 0), 9: ("SUSPECT", 0), 12: ("ALIVE", 2), 20: ("DEAD", 0)}
    sync = wire.Message({wire.HEADER_QUALIFIER: wire.SYNC},
                        wire.SyncData([wire.MembershipRecord(d[j], *st.get(j, ("ALIVE", 0))) for j in range(n)]))
    gossip = wire.membership_gossip_request(d, 40, 0, wire.MembershipRecord(d[7], "SUSPECT", 0))
    for c in (a, b):
        c.set_loss(10.0)
        c.step(2)
        assert wire.deliver(c, 12, sync, d) == n      # ALIVE inc 2 about 12 itself: refuted with inc 3
        assert wire.deliver(c, 3, sync, d) == n       # 3 refutes its SUSPECT
        seq30 = c.debug_member_state()["gossip_seq"][30]
        assert wire.deliver(c, 30, gossip, d) == 1    # MEMBERSHIP_GOSSIP: applied and forwarded
        assert wire.deliver(c, 30, gossip, d) == 0    # the same id again: dropped
        assert c.debug_member_state()["gossip_seq"][30] == seq30  # (a foreign id: the counter stays)
    for _ in range(4):
        for c in (a, b):
            c.step(3)
        assert a.digest() == b.digest()
        sa, sb = a.stats(), b.stats()
        assert {k: sa[k] for k in scenarios.PARITY_KEYS} == {k: sb[k] for k in scenarios.PARITY_KEYS}
        assert [e.key() for e in a.events()] == [e.key() for e in b.events()]
    for i in range(n):
        assert np.array_equal(a.view(i), b.view(i)) and np.array_equal(a.deadlines(i), b.deadlines(i))
