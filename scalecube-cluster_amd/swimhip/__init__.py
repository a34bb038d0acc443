"""swimhip — MI355X-native SWIM membership simulator (scalecube-cluster hot path).

The compute path is libswimhip.so (hand-written HIP for gfx950, C ABI in include/swimhip.h);
this package is the host-side mirror of the reference's config/event surface.
"""
from .config import ClusterConfig, FailureDetectorConfig, GossipConfig, MembershipConfig, to_swim_config
from .cluster import MembershipEvent, MembershipRecord, SwimCluster, SwimError
from .sharded import ShardedSwimCluster
from . import _native as native
from . import cluster_math

__all__ = [
    "ClusterConfig",
    "FailureDetectorConfig",
    "GossipConfig",
    "MembershipConfig",
    "MembershipEvent",
    "MembershipRecord",
    "ShardedSwimCluster",
    "SwimCluster",
    "SwimError",
    "cluster_math",
    "native",
    "to_swim_config",
]
