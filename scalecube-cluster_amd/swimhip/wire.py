"""Wire-format bridge: the reference's JSON messages, so real JVM members can talk
to simulated ones.

A scalecube node frames every message with a 4-byte big-endian length (Netty LengthFieldPrepender /
LengthFieldBasedFrameDecoder, transport-netty/.../TransportImpl.java:383-397; maxFrameLength 2 MiB,
TransportConfig.java:20) and encodes it with Jackson as configured in DefaultObjectMapper
(cluster-testlib/.../utils/DefaultObjectMapper.java:20-31, used by JacksonMessageCodec.java:18-32):
  * every field and every bean getter / is-getter is a property (visibility ANY), so
    MembershipRecord also carries "alive" / "suspect" / "dead" (its isAlive()/isSuspect()/isDead());
  * null properties are left out (NON_NULL): a Message without a sender has no "sender";
  * enums are written with toString() (MemberStatus, PingData.AckType);
  * a property declared as java.lang.Object (Message.data) carries its class name in an "@class"
    property first (DefaultTyping.JAVA_LANG_OBJECT, As.PROPERTY);
  * unknown properties are ignored when reading (FAIL_ON_UNKNOWN_PROPERTIES off);
  * a ByteBuffer is written as a base64 string (GetMetadataResponse.metadata).
Message headers are a java.util.HashMap, so "q" (the qualifier) precedes "cid" (the correlation id):
their HashMap buckets are 1 and 15 of 16 (tapi/Message.java:18-24,190-241).

The shapes (tapi/Message.java, api/Member.java, membership/MembershipRecord.java, membership/SyncData.java,
gossip/GossipRequest.java, gossip/Gossip.java, fdetector/PingData.java, metadata/GetMetadata*.java) are
restated field by field; Address comes from scalecube-commons 1.0.1 (pom.xml:22-33), which is not in
the reference tree: it is written as {"host", "port"} (its two fields). No JVM exists in this image,
so byte-level parity with Jackson is unpinned; tests/test_wire.py restates the reference's codec tests
(GossipRequestTest.java:38-67, JacksonMessageCodecTest.java:21-69) as round trips.

The bridge proper: `sync_message` turns a simulated member's membership table into the SYNC /
SYNC_ACK a real node would receive from it (prepareSyncDataMsg, MembershipProtocolImpl.java:457-461),
`membership_gossip_request` the GossipRequest of one membership gossip (GossipProtocolImpl.java:
211-213,276-279; MembershipProtocolImpl.java:658-673), and `deliver` hands a decoded SYNC / SYNC_ACK /
membership gossip from a real node to a simulated member (swim_deliver_records: updateMembership of
every record, reason SYNC or MEMBERSHIP_GOSSIP; a SYNC of another sync group is ignored, checkSyncGroup,
MembershipProtocolImpl.java:442-448).
"""
from __future__ import annotations

import base64
import json
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import _native as nat

# qualifiers (FailureDetectorImpl.java:35-37, GossipProtocolImpl.java:37, MembershipProtocolImpl.java:68-70,
# MetadataStoreImpl.java:28-29)
PING = "sc/fdetector/ping"
PING_REQ = "sc/fdetector/pingReq"
PING_ACK = "sc/fdetector/pingAck"
GOSSIP_REQ = "sc/gossip/req"
SYNC = "sc/membership/sync"
SYNC_ACK = "sc/membership/syncAck"
MEMBERSHIP_GOSSIP = "sc/membership/gossip"
GET_METADATA_REQ = "sc/metadata/req"
GET_METADATA_RESP = "sc/metadata/resp"
HEADER_QUALIFIER, HEADER_CORRELATION_ID = "q", "cid"  # tapi/Message.java:18,24

CLS_SYNC_DATA = "io.scalecube.cluster.membership.SyncData"
CLS_RECORD = "io.scalecube.cluster.membership.MembershipRecord"
CLS_GOSSIP_REQUEST = "io.scalecube.cluster.gossip.GossipRequest"
CLS_PING_DATA = "io.scalecube.cluster.fdetector.PingData"
CLS_METADATA_REQ = "io.scalecube.cluster.metadata.GetMetadataRequest"
CLS_METADATA_RESP = "io.scalecube.cluster.metadata.GetMetadataResponse"

MAX_FRAME = 2 * 1024 * 1024  # TransportConfig.maxFrameLength default
STATUSES = ("ALIVE", "SUSPECT", "DEAD")  # MemberStatus.java:3-16


class WireError(ValueError):
    pass


# ---- framing (TransportImpl.java:383-397) ------------------------------------------------------
def frame(payload: bytes) -> bytes:
    if len(payload) > MAX_FRAME:
        raise WireError(f"frame of {len(payload)} B exceeds maxFrameLength {MAX_FRAME}")
    return struct.pack(">I", len(payload)) + payload


class FrameDecoder:
    """Incremental LengthFieldBasedFrameDecoder(maxFrameLength, 0, 4, 0, 4): feed bytes as they
    arrive, get whole payloads back (the 4-byte length field stripped)."""

    def __init__(self, max_frame: int = MAX_FRAME):
        self.buf = bytearray()
        self.max_frame = max_frame

    def feed(self, data: bytes) -> List[bytes]:
        self.buf += data
        out = []
        while len(self.buf) >= 4:
            (n,) = struct.unpack(">I", self.buf[:4])
            if n > self.max_frame:
                raise WireError(f"frame of {n} B exceeds maxFrameLength {self.max_frame}")
            if len(self.buf) < 4 + n:
                break
            out.append(bytes(self.buf[4:4 + n]))
            del self.buf[:4 + n]
        return out


# ---- the reference's message types ----------------------------------------------------------------
@dataclass(frozen=True)
class Address:
    host: str
    port: int

    def to_json(self):
        return {"host": self.host, "port": int(self.port)}

    @staticmethod
    def from_json(o):
        return Address(str(o["host"]), int(o["port"]))


@dataclass(frozen=True)
class Member:  # api/Member.java:11-73
    id: str
    address: Address

    def to_json(self):
        return {"id": self.id, "address": self.address.to_json()}

    @staticmethod
    def from_json(o):
        return Member(str(o["id"]), Address.from_json(o["address"]))


@dataclass(frozen=True)
class MembershipRecord:  # membership/MembershipRecord.java:12-109
    member: Member
    status: str
    incarnation: int

    def to_json(self):
        return {"member": self.member.to_json(), "status": self.status, "incarnation": int(self.incarnation),
                "alive": self.status == "ALIVE", "suspect": self.status == "SUSPECT", "dead": self.status == "DEAD"}

    @staticmethod
    def from_json(o):
        st = o.get("status")
        if st not in STATUSES:  # READ_UNKNOWN_ENUM_VALUES_AS_NULL: an unknown status reads as null
            raise WireError(f"membership record without a known status: {st!r}")
        return MembershipRecord(Member.from_json(o["member"]), st, int(o.get("incarnation", 0)))

    def packed(self) -> int:
        """The simulator's cell (include/swimhip.h): inc << 2 | code, DEAD the tombstone (a DEAD
        record's incarnation never matters to isOverrides, MembershipRecord.java:66-84)."""
        if self.status == "DEAD":
            return nat.DEAD
        if not 0 <= self.incarnation < (1 << 30):
            raise WireError(f"incarnation {self.incarnation} outside the packed 30 bits")
        return nat.pack(self.incarnation, nat.ALIVE if self.status == "ALIVE" else nat.SUSPECT)

    @staticmethod
    def from_packed(member: Member, cell: int, dead_incarnation: int = 0):
        if cell == nat.DEAD:
            return MembershipRecord(member, "DEAD", dead_incarnation)
        code = cell & 3
        if cell == nat.ABSENT or code not in (nat.ALIVE, nat.SUSPECT):
            raise WireError(f"cell {cell:#x} is not a record")
        return MembershipRecord(member, "ALIVE" if code == nat.ALIVE else "SUSPECT", cell >> 2)


@dataclass(frozen=True)
class SyncData:  # membership/SyncData.java:11-41
    membership: List[MembershipRecord]
    syncGroup: str = "default"

    def to_json(self):
        return {"membership": [r.to_json() for r in self.membership], "syncGroup": self.syncGroup}

    @staticmethod
    def from_json(o):
        return SyncData([MembershipRecord.from_json(r) for r in o.get("membership") or []], o.get("syncGroup"))


@dataclass(frozen=True)
class Gossip:  # gossip/Gossip.java:7-49
    gossipId: str
    message: "Message"

    def to_json(self):
        return {"gossipId": self.gossipId, "message": self.message.to_json()}

    @staticmethod
    def from_json(o):
        return Gossip(str(o["gossipId"]), Message.from_json(o["message"]))


@dataclass(frozen=True)
class GossipRequest:  # gossip/GossipRequest.java:8-37
    gossips: List[Gossip]
    from_: str

    def to_json(self):
        return {"gossips": [g.to_json() for g in self.gossips], "from": self.from_}

    @staticmethod
    def from_json(o):
        return GossipRequest([Gossip.from_json(g) for g in o.get("gossips") or []], str(o.get("from")))


@dataclass(frozen=True)
class PingData:  # fdetector/PingData.java:6-93
    from_: Member
    to: Member
    originalIssuer: Optional[Member] = None
    ackType: Optional[str] = None  # "DEST_OK" / "DEST_GONE" (PingData.AckType, :8-23)

    def to_json(self):
        o = {"from": self.from_.to_json(), "to": self.to.to_json()}
        if self.originalIssuer is not None:
            o["originalIssuer"] = self.originalIssuer.to_json()
        if self.ackType is not None:
            o["ackType"] = self.ackType
        return o

    @staticmethod
    def from_json(o):
        oi = o.get("originalIssuer")
        return PingData(Member.from_json(o["from"]), Member.from_json(o["to"]),
                        Member.from_json(oi) if oi else None, o.get("ackType"))


@dataclass(frozen=True)
class GetMetadataRequest:  # metadata/GetMetadataRequest.java
    member: Member

    def to_json(self):
        return {"member": self.member.to_json()}

    @staticmethod
    def from_json(o):
        return GetMetadataRequest(Member.from_json(o["member"]))


@dataclass(frozen=True)
class GetMetadataResponse:  # metadata/GetMetadataResponse.java
    member: Member
    metadata: bytes

    def to_json(self):
        return {"member": self.member.to_json(), "metadata": base64.b64encode(self.metadata).decode("ascii")}

    @staticmethod
    def from_json(o):
        m = o.get("metadata")
        return GetMetadataResponse(Member.from_json(o["member"]), base64.b64decode(m) if m is not None else b"")


@dataclass(frozen=True)
class Opaque:
    """Message data of a class this bridge does not model (application payloads): kept as the
    JSON object it arrived as, "@class" included, and written back unchanged."""
    cls: str
    body: dict

    def to_json(self):
        return {k: v for k, v in self.body.items() if k != "@class"}


TYPES = {CLS_SYNC_DATA: SyncData, CLS_RECORD: MembershipRecord, CLS_GOSSIP_REQUEST: GossipRequest,
         CLS_PING_DATA: PingData, CLS_METADATA_REQ: GetMetadataRequest, CLS_METADATA_RESP: GetMetadataResponse}
CLASS_OF = {v: k for k, v in TYPES.items()}


@dataclass(frozen=True)
class Message:  # tapi/Message.java:12-242
    headers: Dict[str, str] = field(default_factory=dict)
    data: object = None
    sender: Optional[Address] = None

    @property
    def qualifier(self):
        return self.headers.get(HEADER_QUALIFIER)

    @property
    def correlationId(self):
        return self.headers.get(HEADER_CORRELATION_ID)

    def to_json(self):
        o = {"headers": _java_hashmap_order(self.headers)}
        if self.data is not None:
            o["data"] = _typed(self.data)
        if self.sender is not None:
            o["sender"] = self.sender.to_json()
        return o

    @staticmethod
    def from_json(o):
        data = o.get("data")
        if isinstance(data, dict):
            cls = data.get("@class")
            typ = TYPES.get(cls)
            data = typ.from_json(data) if typ else Opaque(str(cls), data)
        snd = o.get("sender")
        return Message(dict(o.get("headers") or {}), data, Address.from_json(snd) if snd else None)


def _typed(data):
    """A java.lang.Object property under DefaultTyping.JAVA_LANG_OBJECT / As.PROPERTY: "@class" first."""
    if isinstance(data, Opaque):
        return {"@class": data.cls, **data.to_json()}
    cls = CLASS_OF.get(type(data))
    if cls is None:
        if isinstance(data, (str, int, float, bool)):  # natural JSON types carry no type id
            return data
        raise WireError(f"no Java class for {type(data).__name__}")
    return {"@class": cls, **data.to_json()}


def _java_string_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def _java_hashmap_order(d: Dict[str, str]) -> Dict[str, str]:
    """Iteration order of a java.util.HashMap holding d (default capacity 16, load 0.75; resized by
    doubling): by bucket (hash ^ hash >>> 16) & (capacity - 1), then insertion order within a bucket."""
    cap = 16
    while len(d) > cap * 3 // 4:
        cap *= 2

    def bucket(k):
        h = _java_string_hash(k)
        return (h ^ (h >> 16)) & (cap - 1)

    return {k: d[k] for k in sorted(d, key=bucket)}  # sorted() is stable: insertion order within a bucket


def encode(msg: Message) -> bytes:
    return json.dumps(msg.to_json(), separators=(",", ":")).encode("utf-8")


def decode(payload: bytes) -> Message:
    try:
        return Message.from_json(json.loads(payload.decode("utf-8")))
    except (KeyError, TypeError, ValueError) as e:
        raise WireError(f"not a scalecube message: {e}") from e


# ---- the bridge: simulated members <-> the wire -------------------------------------------------
class Directory:
    """Simulated member index <-> the Member (id, address) real nodes know it by. By default member
    i is "sim-<i>" at sim:<base_port + i>; real nodes' ids are whatever they announce (Member.java:48-50)."""

    def __init__(self, n: int, host: str = "sim", base_port: int = 10000, ids=None):
        self.members = [Member(ids[i] if ids else f"sim-{i}", Address(host, base_port + i)) for i in range(n)]
        self.index = {m.id: i for i, m in enumerate(self.members)}

    def __getitem__(self, i) -> Member:
        return self.members[i]

    def of(self, member_id: str) -> Optional[int]:
        return self.index.get(member_id)


def records_of_row(row, directory: Directory) -> List[MembershipRecord]:
    """A membership table row (packed cells, swim_read_view) as the records of a SyncData, in
    member order (membershipTable.values(), MembershipProtocolImpl.java:457-461)."""
    return [MembershipRecord.from_packed(directory[j], int(c)) for j, c in enumerate(row) if int(c) != nat.ABSENT]


def sync_message(cluster, observer: int, directory: Directory, qualifier: str = SYNC, cid: Optional[str] = None,
                 sync_group: str = "default") -> Message:
    """The SYNC (or SYNC_ACK with the request's cid) simulated member `observer` sends: its whole
    table (prepareSyncDataMsg, MembershipProtocolImpl.java:457-461)."""
    h = {HEADER_QUALIFIER: qualifier}
    if cid is not None:
        h[HEADER_CORRELATION_ID] = cid
    return Message(h, SyncData(records_of_row(cluster.view(observer), directory), sync_group),
                   directory[observer].address)


def membership_gossip_request(directory: Directory, origin: int, seq: int, record: MembershipRecord) -> Message:
    """One membership gossip of member `origin` as the GossipRequest it sends per gossip and peer:
    id "<member id>-<counter>" (generateGossipId, GossipProtocolImpl.java:211-213), the record wrapped
    in a MEMBERSHIP_GOSSIP message (MembershipProtocolImpl.java:658-673), GossipRequest from the
    origin's id (GossipProtocolImpl.java:276-279)."""
    inner = Message({HEADER_QUALIFIER: MEMBERSHIP_GOSSIP}, record)
    gid = f"{directory[origin].id}-{seq}"
    return Message({HEADER_QUALIFIER: GOSSIP_REQ}, GossipRequest([Gossip(gid, inner)], directory[origin].id))


def decoded_records(records: List[MembershipRecord], directory: Directory):
    """(subjects, packed records) of the records about members the directory knows (a record about
    an unknown member has no row in the simulation and is skipped)."""
    subj, rec = [], []
    for r in records:
        j = directory.of(r.member.id)
        if j is not None:
            subj.append(j)
            rec.append(r.packed())
    return subj, rec


def _seen_ids(cluster, observer: int) -> dict:
    """The gossip ids a simulated member holds from real nodes: GossipProtocolImpl.gossips keyed by
    gossipId (:171-183), each until the period its sweep drops it (sweepGossips, :281-304)."""
    seen = cluster.__dict__.setdefault("_wire_seen", {})
    return seen.setdefault(int(observer), {})


def _sweep_periods(cluster, observer: int) -> int:
    """Periods a received gossip stays in the observer's `gossips`. sweepGossips (GossipProtocolImpl.java:
    280-303) drops a GossipState in the first gossip round r with r > infectionPeriod + periodsToSweep,
    periodsToSweep = gossipPeriodsToSweep(repeatMult, remoteMembers.size() + 1) (ClusterMath.java:99-102)
    at the observer's table size. A gossip delivered before period p has infectionPeriod p * G (G gossip
    rounds per period), so the round that drops it is p * G + sweep + 1, in period p + (sweep + 1) // G:
    it is held until that period has run (the table size taken at delivery)."""
    from .cluster_math import gossipPeriodsToSweep

    g = cluster.config.gossipConfig()
    rounds_per_period = max(1, cluster.config.failureDetectorConfig().pingInterval() // g.gossipInterval())
    sweep = gossipPeriodsToSweep(g.gossipRepeatMult(), len(cluster.members(observer)))
    return (sweep + 1) // rounds_per_period + 1


def deliver(cluster, observer: int, msg: Message, directory: Directory, sync_group: str = "default") -> int:
    """Hand a real node's message to simulated member `observer` (before the next period). Returns
    the number of records delivered.

    SYNC: syncMembership with reason SYNC (accepted records re-spread), a foreign sync group ignored
    (checkSyncGroup, MembershipProtocolImpl.java:442-448). SYNC_ACK: only one without a correlation id
    (a reply to a periodic SYNC, onSyncAck, :343-349); onMessage drops a SYNC_ACK that carries one
    (:331-334): it answers an initial sync the simulated member never sent to a real node.
    GossipRequest: each membership gossip whose id the observer does not hold yet (onGossipReq,
    GossipProtocolImpl.java:171-183; a repeat from another real peer is dropped): its GossipState is put,
    so the observer forwards it to simulated peers in the coming rounds (SWIM_DELIVER_FORWARD), and
    its record goes to onMembershipGossip with reason MEMBERSHIP_GOSSIP (:407-414). An id is held until
    the observer's sweep drops it (gossipPeriodsToSweep), then a copy counts as new again. Other
    messages (pings, metadata, application gossips) carry no membership records."""
    q, data = msg.qualifier, msg.data
    if q in (SYNC, SYNC_ACK) and isinstance(data, SyncData):
        if data.syncGroup != sync_group:
            return 0
        if q == SYNC_ACK and msg.correlationId is not None:
            return 0
        subj, rec = decoded_records(data.membership, directory)
        reason = nat.R_SYNC
    elif q == GOSSIP_REQ and isinstance(data, GossipRequest):
        seen = _seen_ids(cluster, observer)
        now = cluster.period
        for gid in [g for g, until in seen.items() if until <= now]:
            del seen[gid]
        recs = []
        for g in data.gossips:
            if g.gossipId in seen:
                continue
            seen[g.gossipId] = now + _sweep_periods(cluster, observer)
            if g.message.qualifier == MEMBERSHIP_GOSSIP and isinstance(g.message.data, MembershipRecord):
                recs.append(g.message.data)
        subj, rec = decoded_records(recs, directory)
        reason = nat.R_MEMBERSHIP_GOSSIP | nat.DELIVER_FORWARD
    else:
        return 0
    if subj:
        cluster.deliver_records(observer, subj, rec, reason)
    return len(subj)
