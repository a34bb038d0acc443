"""Config surface of the reference, mirrored 1:1 (names, defaults, presets, clone-on-write).

  FailureDetectorConfig  cluster-api/src/main/java/io/scalecube/cluster/fdetector/FailureDetectorConfig.java:5-133
  GossipConfig           cluster-api/src/main/java/io/scalecube/cluster/gossip/GossipConfig.java:5-127
  MembershipConfig       cluster-api/src/main/java/io/scalecube/cluster/membership/MembershipConfig.java:10-184
  ClusterConfig          cluster-api/src/main/java/io/scalecube/cluster/ClusterConfig.java:21-296

Setters return a modified clone, exactly like the Java builders. `seedMembers` takes member
ids of the simulated cluster (the reference takes addresses; an address is a member slot here).
"""
from __future__ import annotations

import copy


class _Cfg:
    def _with(self, **kw):
        c = copy.copy(self)
        for k, v in kw.items():
            setattr(c, "_" + k, v)
        return c

    def __repr__(self):
        items = ", ".join(f"{k[1:]}={v}" for k, v in sorted(vars(self).items()))
        return f"{type(self).__name__}({items})"


class FailureDetectorConfig(_Cfg):
    DEFAULT_PING_INTERVAL = 1_000
    DEFAULT_PING_TIMEOUT = 500
    DEFAULT_PING_REQ_MEMBERS = 3
    DEFAULT_WAN_PING_TIMEOUT = 3_000
    DEFAULT_WAN_PING_INTERVAL = 5_000
    DEFAULT_LOCAL_PING_TIMEOUT = 200
    DEFAULT_LOCAL_PING_INTERVAL = 1_000
    DEFAULT_LOCAL_PING_REQ_MEMBERS = 1

    def __init__(self):
        self._pingInterval = self.DEFAULT_PING_INTERVAL
        self._pingTimeout = self.DEFAULT_PING_TIMEOUT
        self._pingReqMembers = self.DEFAULT_PING_REQ_MEMBERS

    @classmethod
    def defaultConfig(cls):
        return cls()

    @classmethod
    def defaultLanConfig(cls):
        return cls.defaultConfig()

    @classmethod
    def defaultWanConfig(cls):
        return cls.defaultConfig().pingTimeout(cls.DEFAULT_WAN_PING_TIMEOUT).pingInterval(cls.DEFAULT_WAN_PING_INTERVAL)

    @classmethod
    def defaultLocalConfig(cls):
        return (
            cls.defaultConfig()
            .pingTimeout(cls.DEFAULT_LOCAL_PING_TIMEOUT)
            .pingInterval(cls.DEFAULT_LOCAL_PING_INTERVAL)
            .pingReqMembers(cls.DEFAULT_LOCAL_PING_REQ_MEMBERS)
        )

    def pingInterval(self, v=None):
        return self._pingInterval if v is None else self._with(pingInterval=int(v))

    def pingTimeout(self, v=None):
        return self._pingTimeout if v is None else self._with(pingTimeout=int(v))

    def pingReqMembers(self, v=None):
        return self._pingReqMembers if v is None else self._with(pingReqMembers=int(v))


class GossipConfig(_Cfg):
    DEFAULT_GOSSIP_INTERVAL = 200
    DEFAULT_GOSSIP_FANOUT = 3
    DEFAULT_GOSSIP_REPEAT_MULT = 3
    DEFAULT_WAN_GOSSIP_FANOUT = 4
    DEFAULT_LOCAL_GOSSIP_REPEAT_MULT = 2
    DEFAULT_LOCAL_GOSSIP_INTERVAL = 100

    def __init__(self):
        self._gossipFanout = self.DEFAULT_GOSSIP_FANOUT
        self._gossipInterval = self.DEFAULT_GOSSIP_INTERVAL
        self._gossipRepeatMult = self.DEFAULT_GOSSIP_REPEAT_MULT

    @classmethod
    def defaultConfig(cls):
        return cls()

    @classmethod
    def defaultLanConfig(cls):
        return cls.defaultConfig()

    @classmethod
    def defaultWanConfig(cls):
        return cls.defaultConfig().gossipFanout(cls.DEFAULT_WAN_GOSSIP_FANOUT)

    @classmethod
    def defaultLocalConfig(cls):
        return (
            cls.defaultConfig()
            .gossipRepeatMult(cls.DEFAULT_LOCAL_GOSSIP_REPEAT_MULT)
            .gossipInterval(cls.DEFAULT_LOCAL_GOSSIP_INTERVAL)
        )

    def gossipFanout(self, v=None):
        return self._gossipFanout if v is None else self._with(gossipFanout=int(v))

    def gossipInterval(self, v=None):
        return self._gossipInterval if v is None else self._with(gossipInterval=int(v))

    def gossipRepeatMult(self, v=None):
        return self._gossipRepeatMult if v is None else self._with(gossipRepeatMult=int(v))


class MembershipConfig(_Cfg):
    DEFAULT_SYNC_INTERVAL = 30_000
    DEFAULT_SYNC_TIMEOUT = 3_000
    DEFAULT_SUSPICION_MULT = 5
    DEFAULT_WAN_SUSPICION_MULT = 6
    DEFAULT_WAN_SYNC_INTERVAL = 60_000
    DEFAULT_LOCAL_SUSPICION_MULT = 3
    DEFAULT_LOCAL_SYNC_INTERVAL = 15_000

    def __init__(self):
        self._seedMembers = []
        self._syncInterval = self.DEFAULT_SYNC_INTERVAL
        self._syncTimeout = self.DEFAULT_SYNC_TIMEOUT
        self._suspicionMult = self.DEFAULT_SUSPICION_MULT
        self._syncGroup = "default"

    @classmethod
    def defaultConfig(cls):
        return cls()

    @classmethod
    def defaultLanConfig(cls):
        return cls.defaultConfig()

    @classmethod
    def defaultWanConfig(cls):
        return cls.defaultConfig().suspicionMult(cls.DEFAULT_WAN_SUSPICION_MULT).syncInterval(cls.DEFAULT_WAN_SYNC_INTERVAL)

    @classmethod
    def defaultLocalConfig(cls):
        return (
            cls.defaultConfig()
            .suspicionMult(cls.DEFAULT_LOCAL_SUSPICION_MULT)
            .syncInterval(cls.DEFAULT_LOCAL_SYNC_INTERVAL)
        )

    def seedMembers(self, *ids):
        if not ids:
            return list(self._seedMembers)
        if len(ids) == 1 and isinstance(ids[0], (list, tuple, range)):
            ids = tuple(ids[0])
        return self._with(seedMembers=[int(i) for i in ids])

    def syncInterval(self, v=None):
        return self._syncInterval if v is None else self._with(syncInterval=int(v))

    def syncTimeout(self, v=None):
        return self._syncTimeout if v is None else self._with(syncTimeout=int(v))

    def suspicionMult(self, v=None):
        return self._suspicionMult if v is None else self._with(suspicionMult=int(v))

    def syncGroup(self, v=None):
        return self._syncGroup if v is None else self._with(syncGroup=str(v))


class ClusterConfig(_Cfg):
    DEFAULT_METADATA_TIMEOUT = 3_000
    DEFAULT_WAN_METADATA_TIMEOUT = 10_000
    DEFAULT_LOCAL_METADATA_TIMEOUT = 1_000

    def __init__(self):
        self._metadataTimeout = self.DEFAULT_METADATA_TIMEOUT
        self._failureDetectorConfig = FailureDetectorConfig.defaultConfig()
        self._gossipConfig = GossipConfig.defaultConfig()
        self._membershipConfig = MembershipConfig.defaultConfig()

    @classmethod
    def defaultConfig(cls):
        return cls()

    @classmethod
    def defaultLanConfig(cls):
        return cls.defaultConfig()

    @classmethod
    def defaultWanConfig(cls):
        return (
            cls.defaultConfig()
            .failureDetector(lambda o: FailureDetectorConfig.defaultWanConfig())
            .gossip(lambda o: GossipConfig.defaultWanConfig())
            .membership(lambda o: MembershipConfig.defaultWanConfig())
            .metadataTimeout(cls.DEFAULT_WAN_METADATA_TIMEOUT)
        )

    @classmethod
    def defaultLocalConfig(cls):
        return (
            cls.defaultConfig()
            .failureDetector(lambda o: FailureDetectorConfig.defaultLocalConfig())
            .gossip(lambda o: GossipConfig.defaultLocalConfig())
            .membership(lambda o: MembershipConfig.defaultLocalConfig())
            .metadataTimeout(cls.DEFAULT_LOCAL_METADATA_TIMEOUT)
        )

    def metadataTimeout(self, v=None):
        return self._metadataTimeout if v is None else self._with(metadataTimeout=int(v))

    def failureDetector(self, op):
        return self._with(failureDetectorConfig=op(self._failureDetectorConfig))

    def gossip(self, op):
        return self._with(gossipConfig=op(self._gossipConfig))

    def membership(self, op):
        return self._with(membershipConfig=op(self._membershipConfig))

    def failureDetectorConfig(self):
        return self._failureDetectorConfig

    def gossipConfig(self):
        return self._gossipConfig

    def membershipConfig(self):
        return self._membershipConfig


def to_swim_config(cfg: ClusterConfig, n_members: int, seed: int = 0, *, gossip_capacity: int = 0,
                   event_capacity: int = 0, sync_capacity: int = 0, tracked_subjects: int = 0, device: int = 0,
                   shard_rank: int = 0, shard_world: int = 1, n_initial: int = 0, gossip_batching: bool = True,
                   record_capacity: int = 0, infection_round_bits: int = 0, dict_subjects: int = 0):
    """Marshal a ClusterConfig into the C struct of include/swimhip.h. n_initial < n_members leaves
    ids [n_initial, n_members) as spare slots for joins and restarts."""
    from ._native import SwimConfig

    fd, g, m = cfg.failureDetectorConfig(), cfg.gossipConfig(), cfg.membershipConfig()
    seeds = sorted(set(m.seedMembers()))
    if seeds and seeds != list(range(len(seeds))):
        raise ValueError("simulated seedMembers must be the ids 0..k-1")
    c = SwimConfig()
    c.n_members = n_members
    c.mode = 1 if tracked_subjects else 0  # N x K tracked-subject views
    c.seed = seed & 0xFFFFFFFFFFFFFFFF
    c.ping_interval_ms = fd.pingInterval()
    c.ping_timeout_ms = fd.pingTimeout()
    c.ping_req_members = fd.pingReqMembers()
    c.gossip_fanout = g.gossipFanout()
    c.gossip_interval_ms = g.gossipInterval()
    c.gossip_repeat_mult = g.gossipRepeatMult()
    c.sync_interval_ms = m.syncInterval()
    c.sync_timeout_ms = m.syncTimeout()
    c.suspicion_mult = m.suspicionMult()
    c.metadata_timeout_ms = cfg.metadataTimeout()
    c.n_seeds = len(seeds)
    c.gossip_capacity = gossip_capacity
    c.event_capacity = event_capacity
    c.sync_capacity = sync_capacity
    c.tracked_subjects = tracked_subjects
    c.n_initial = n_initial
    c.device = device
    c.shard_rank = shard_rank
    c.shard_world = shard_world
    c.gossip_batching = 0 if gossip_batching else 1
    c.record_capacity = record_capacity
    c.infection_round_bits = infection_round_bits
    c.dict_subjects = dict_subjects
    return c
