"""SwimCluster — N simulated scalecube members stepped in bulk through the C ABI.

The facade mirrors what a user of the reference sees per member:
  MembershipProtocol.members()/otherMembers()/listen()   (core/membership/MembershipProtocol.java:14-65)
  MembershipEvent{ADDED, REMOVED, UPDATED}               (api/membership/MembershipEvent.java:11-117)
  NetworkEmulator loss / block / partition               (cluster-testlib/.../utils/NetworkEmulator.java:58-297)
  transport.stop() as crash                               (MembershipProtocolTest.java:991-1000)

`SwimCluster(...)` always drives libswimhip.so (HIP, gfx950). The class is also used by the test
suite with the oracle's function table to compare both implementations call-for-call.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native as nat
from .config import ClusterConfig, to_swim_config


class SwimError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with status {code}")
        self.code = code


@dataclass(frozen=True)
class MembershipEvent:
    """api/membership/MembershipEvent.java:13-67, plus the simulated observer and period."""

    type: int
    member: int
    observer: int
    period: int
    record: int
    reason: int
    phase: int

    ADDED = nat.EV_ADDED
    REMOVED = nat.EV_REMOVED
    UPDATED = nat.EV_UPDATED

    def isAdded(self):
        return self.type == nat.EV_ADDED

    def isRemoved(self):
        return self.type == nat.EV_REMOVED

    def isUpdated(self):
        return self.type == nat.EV_UPDATED

    def isGossip(self):  # GossipProtocol.listen(): first receipt of a user gossip (member = origin)
        return self.type == nat.EV_GOSSIP

    def isFailureDetector(self):  # FailureDetectorEvent: member = probed member, record = status
        return self.type == nat.EV_FD

    def key(self):
        return (self.period, self.observer, self.phase, self.member, self.type, self.reason, self.record)


@dataclass(frozen=True)
class MembershipRecord:
    """core/membership/MembershipRecord.java:12-109 decoded from a packed cell."""

    member: int
    status: str
    incarnation: int

    @staticmethod
    def decode(member: int, cell: int):
        if cell == nat.ABSENT:
            return None
        if cell == nat.DEAD:
            return MembershipRecord(member, "DEAD", -1)
        return MembershipRecord(member, {1: "ALIVE", 2: "SUSPECT"}.get(cell & 3, "?"), cell >> 2)


class SwimCluster:
    def __init__(self, config: ClusterConfig, n_members: int, seed: int = 0, *, event_capacity: int = 0,
                 gossip_capacity: int = 0, sync_capacity: int = 0, tracked_subjects: int = 0, device: int = 0,
                 n_initial: int = 0, gossip_batching: bool = True, record_capacity: int = 0,
                 infection_round_bits: int = 0, dict_subjects: int = 0, _lib=None,
                 _prefix: str = "swim_", _shard=(0, 1)):
        self._lib = _lib if _lib is not None else nat.load_swimhip()
        self._p = _prefix
        self.config = config
        self.n = int(n_members)
        self.seed = int(seed)
        self._cfg = to_swim_config(config, self.n, seed, gossip_capacity=gossip_capacity,
                                   event_capacity=event_capacity, sync_capacity=sync_capacity,
                                   tracked_subjects=tracked_subjects, device=device, shard_rank=_shard[0],
                                   shard_world=_shard[1], n_initial=n_initial, gossip_batching=gossip_batching,
                                   record_capacity=record_capacity, infection_round_bits=infection_round_bits,
                                   dict_subjects=dict_subjects)
        h = ctypes.c_void_p()
        self._h = None
        self._call("create", ctypes.byref(self._cfg), ctypes.byref(h))
        self._h = h
        self._alive = np.arange(self.n) < (n_initial or self.n)
        self.period = 0  # periods stepped (host count; swim_stats.period on the device)

    # -- plumbing -------------------------------------------------------------------------
    def _fn(self, name):
        return getattr(self._lib, self._p + name)

    def _call(self, name, *args):
        rc = self._fn(name)(*args)
        if rc != nat.SWIM_OK:
            msg = name
            if self._p == "swim_" and self._h is not None:
                err = self._lib.swim_last_error(self._h)
                if err:
                    msg += ": " + err.decode(errors="replace")
            raise SwimError(rc, msg)
        return rc

    def close(self):
        if self._h is not None:
            self._fn("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- fault injection (NetworkEmulator) ------------------------------------------------
    def set_loss(self, percent: float):
        """setDefaultOutboundSettings(lossPercent, 0) on every member (NetworkEmulator.java:81-84)."""
        self._call("set_loss", self._h, int(round(percent * 100)))

    def set_delay(self, mean_ms: int):
        """setDefaultOutboundSettings(lossPercent, meanDelay) on every member, the delay part
        (NetworkEmulator.java:81-84,189-201,358-368): each message is delayed by an exponential draw
        of mean `mean_ms`. GossipRequests then arrive rounds later, ping / ping-req
        / metadata round trips must come back within their timeouts. Unsharded handles."""
        self._call("set_delay", self._h, int(mean_ms))

    def partition(self, groups, t0: int, t1: int):
        g = np.ascontiguousarray(np.asarray(groups, dtype=np.uint8))
        assert g.shape == (self.n,)
        self._call("set_partition", self._h, g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), self.n, t0, t1)

    def block_outbound(self, src: int, dsts, blocked: bool = True):
        """NetworkEmulator.blockOutbound(Address...) (NetworkEmulator.java:105-119): a send from
        src to a blocked destination fails immediately (tryFailOutbound, :166-180)."""
        for d in dsts:
            self._call("block_link", self._h, int(src), int(d), 1 if blocked else 0)

    def unblock_outbound(self, src: int, dsts):
        self.block_outbound(src, dsts, blocked=False)

    def block_inbound(self, dst: int, srcs, blocked: bool = True):
        """NetworkEmulator.blockInbound (NetworkEmulator.java:255-269): dst silently drops every
        message whose sender is in srcs (NetworkEmulatorTransport.java:66-68,73-77); the sender's
        send succeeds, unlike an outbound block."""
        for s in srcs:
            self._call("block_inbound", self._h, int(dst), int(s), 1 if blocked else 0)

    def unblock_inbound(self, dst: int, srcs):
        self.block_inbound(dst, srcs, blocked=False)

    def crash(self, ids):
        ids = np.ascontiguousarray(np.asarray(list(ids), dtype=np.uint32))
        self._call("crash", self._h, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(ids))
        self._alive[ids] = False

    def leave(self, ids):
        """Cluster.shutdown() of each member (ClusterImpl.java:370-408): leaveCluster spreads its
        DEAD record (MembershipProtocolImpl.java:203-212); the member stops once its own sweep
        drops that gossip."""
        ids = np.ascontiguousarray(np.asarray(list(ids), dtype=np.uint32))
        self._call("leave", self._h, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(ids))

    def update_metadata(self, ids):
        """Cluster.updateMetadata (ClusterImpl.java:364-367) of each member: a new metadata version
        and updateIncarnation (MembershipProtocolImpl.java:184-196): its own record ALIVE with
        incarnation + 1, spread; members that had it emit UPDATED once they fetch the new metadata."""
        ids = np.ascontiguousarray(np.asarray(list(ids), dtype=np.uint32))
        self._call("update_metadata", self._h, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(ids))

    def spread(self, origin: int, tag: int):
        """GossipProtocol.spread (GossipProtocolImpl.java:124-128) of a user gossip by member
        `origin`; every member's first receipt shows up as an EV_GOSSIP event (GossipProtocol.listen)."""
        self._call("spread", self._h, int(origin), int(tag) & 0xFFFFFFFF)

    def deliver_records(self, observer: int, subjects, records, reason: int = nat.R_SYNC):
        """A message of an external node (decoded by swimhip.wire) delivered to member `observer`
        before the next period: updateMembership of each (subject, packed record) in order with
        `reason` (SYNC / INITIAL_SYNC: syncMembership, MembershipProtocolImpl.java:463-473;
        MEMBERSHIP_GOSSIP: onMembershipGossip, :407-414)."""
        s = np.ascontiguousarray(np.asarray(list(subjects), dtype=np.uint32))
        r = np.ascontiguousarray(np.asarray(list(records), dtype=np.uint32))
        assert s.shape == r.shape
        P = ctypes.POINTER(ctypes.c_uint32)
        self._call("deliver_records", self._h, int(observer), s.ctypes.data_as(P), r.ctypes.data_as(P), len(s),
                   int(reason))

    def trace(self, fd: bool = True):
        """FailureDetector.listen() (FailureDetectorImpl.java:365-368) into the event ring as EV_FD."""
        self._call("trace", self._h, nat.TRACE_FD if fd else 0)

    def join(self, ids):
        """ClusterImpl.start() of new members in spare slots (ids >= n_initial), each at an address
        of its own: initial SYNC to the seeds (MembershipProtocolImpl.start0, :222-257)."""
        ids = np.ascontiguousarray(np.asarray(list(ids), dtype=np.uint32))
        self._call("join", self._h, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(ids))
        self._alive[ids] = True

    def restart(self, old_ids, new_ids):
        """Restart stopped members on their addresses as new member ids (spare slots new_ids):
        MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses (:453-520)."""
        o = np.ascontiguousarray(np.asarray(list(old_ids), dtype=np.uint32))
        w = np.ascontiguousarray(np.asarray(list(new_ids), dtype=np.uint32))
        assert len(o) == len(w)
        P = ctypes.POINTER(ctypes.c_uint32)
        self._call("restart", self._h, o.ctypes.data_as(P), w.ctypes.data_as(P), len(o))
        self._alive[w] = True

    # -- stepping -------------------------------------------------------------------------
    def step(self, periods: int = 1):
        self._call("step", self._h, int(periods))
        self.period += int(periods)

    # -- observation ----------------------------------------------------------------------
    def view(self, observer: int) -> np.ndarray:
        row = np.zeros(self.n, dtype=np.uint32)
        self._call("read_view", self._h, int(observer), row.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), self.n)
        return row

    def views(self) -> np.ndarray:
        return np.stack([self.view(i) for i in range(self.n)])

    def deadlines(self, observer: int) -> np.ndarray:
        row = np.zeros(self.n, dtype=np.uint32)
        self._call("read_deadlines", self._h, int(observer), row.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                   self.n)
        return row

    def digest(self):
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._call("digest", self._h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def presence(self):
        pres = np.zeros(self.n, dtype=np.uint32)
        last = np.zeros(self.n, dtype=np.uint32)
        self._call("read_presence", self._h, pres.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                   last.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), self.n)
        return pres, last

    def stats(self) -> dict:
        s = nat.SwimStats()
        self._call("stats_get", self._h, ctypes.byref(s))
        return {f: getattr(s, f) for f in nat.STAT_FIELDS}

    def events(self, cap: int = 1 << 20):
        buf = (nat.SwimEvent * cap)()
        n = ctypes.c_uint64()
        self._call("drain_events", self._h, buf, cap, ctypes.byref(n))
        return [
            MembershipEvent(e.type, e.subject, e.observer, e.period, e.record, e.reason, e.phase)
            for e in buf[: n.value]
        ]

    def discard_events(self) -> int:
        """Drop the pending events, returning how many there were (a listener that only counts)."""
        n = ctypes.c_uint64()
        self._call("drain_events", self._h, None, 0, ctypes.byref(n))
        return int(n.value)

    # -- MembershipProtocol-shaped accessors (MembershipProtocol.java:14-65) ----------------
    def members(self, observer: int):
        row = self.view(observer)
        return [int(j) for j in np.nonzero(row)[0]]

    def otherMembers(self, observer: int):
        return [j for j in self.members(observer) if j != observer]

    def membershipRecords(self, observer: int):
        """getMembershipRecords (MembershipProtocolImpl.java:716-718)."""
        row = self.view(observer)
        return [MembershipRecord.decode(int(j), int(row[j])) for j in np.nonzero(row)[0]]

    def alive(self, observer: int):
        row = self.view(observer)
        return [int(j) for j in np.nonzero((row & 3) == 1)[0] if j != observer]

    def suspected(self, observer: int):
        row = self.view(observer)
        return [int(j) for j in np.nonzero((row != 0) & ((row & 3) == 2))[0]]

    def debug_holdings(self, member: int, cap: int = 1 << 20):
        """(gossip hash, infection round) pairs the member's GossipProtocol holds (debug)."""
        hs = np.zeros(cap, dtype=np.uint32)
        inf = np.zeros(cap, dtype=np.uint32)
        n = ctypes.c_uint32()
        P = ctypes.POINTER(ctypes.c_uint32)
        self._call("debug_holdings", self._h, int(member), hs.ctypes.data_as(P), inf.ctypes.data_as(P), cap,
                   ctypes.byref(n))
        k = min(n.value, cap)
        return sorted(zip(hs[:k].tolist(), inf[:k].tolist()))

    def debug_member_state(self):
        """Per-member protocol cursors (debug): dict of arrays."""
        out = np.zeros(6 * self.n, dtype=np.uint32)
        self._call("debug_member_state", self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), self.n)
        names = ["fd_epoch", "fd_cursor", "g_epoch", "g_cursor", "gossip_seq", "others"]
        return {k: out[i * self.n:(i + 1) * self.n] for i, k in enumerate(names)}

    def debug_sends(self):
        """Per sender (debug): cumulative GossipRequests to alive peers before infectedFrom, and suppressed."""
        out = np.zeros(2 * self.n, dtype=np.uint64)
        self._call("debug_sends", self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), self.n)
        return out[0::2], out[1::2]

    # -- bench helpers (HIP library only) ---------------------------------------------------
    KERNEL_CLASSES = ["k_fd", "k_gossip_pull", "k_gossip_apply", "k_susp_sweep", "k_sync_merge", "k_sync_ack",
                      "k_sync_snapshot", "bookkeeping", "k_gossip_select", "k_gossip_inhist", "k_gossip_pairwin",
                      "k_gossip_record"]

    def step_async(self, periods: int = 1):
        self._call("step_async", self._h, int(periods))
        self.period += int(periods)

    def sync(self):
        self._call("sync", self._h)

    def kernel_timing(self, enable: bool, classes=None):
        """Reset the per-class device times; with `classes` (names of KERNEL_CLASSES) only those
        launches are bracketed by HIP events."""
        mask = 1 if enable else 0
        if enable and classes:
            mask = sum(1 << self.KERNEL_CLASSES.index(c) for c in classes)
            mask = mask if mask != 1 else 1 | (1 << 30)  # (class 0 alone: not the "every class" value)
        self._call("kernel_time_reset", self._h, mask)

    def kernel_times(self) -> dict:
        """{kernel class: (total device ms, launches)} since the last kernel_timing() reset."""
        out = {}
        for i, name in enumerate(self.KERNEL_CLASSES):
            ms, n = ctypes.c_double(), ctypes.c_uint64()
            self._call("kernel_time", self._h, i, ctypes.byref(ms), ctypes.byref(n))
            out[name] = (ms.value, n.value)
        return out
