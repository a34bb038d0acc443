"""ClusterMath (cluster/src/main/java/io/scalecube/cluster/ClusterMath.java:8-136), host side.

Integer formulas are exact; the two floating-point helpers are reporting-only in the reference
(used by GossipProtocolTest to log theory vs observation, GossipProtocolTest.java:176-203).
"""
from __future__ import annotations


def ceilLog2(num: int) -> int:
    """ClusterMath.java:133-135: 32 - numberOfLeadingZeros(num) == bit_length for num >= 0."""
    num &= 0xFFFFFFFF
    return num.bit_length()


def gossipConvergencePercent(fanout: int, repeatMult: int, clusterSize: int, lossPercent: float) -> float:
    return gossipConvergenceProbability(fanout, repeatMult, clusterSize, lossPercent / 100.0) * 100  # :23-27


def gossipConvergenceProbability(fanout: int, repeatMult: int, clusterSize: int, loss: float) -> float:
    fanoutWithLoss = (1.0 - loss) * fanout  # :38-43
    spreadSize = clusterSize - clusterSize ** (-(fanoutWithLoss * repeatMult - 2))
    return spreadSize / clusterSize


def maxMessagesPerGossipTotal(fanout: int, repeatMult: int, clusterSize: int) -> int:
    return clusterSize * maxMessagesPerGossipPerNode(fanout, repeatMult, clusterSize)  # :53-55


def maxMessagesPerGossipPerNode(fanout: int, repeatMult: int, clusterSize: int) -> int:
    return fanout * repeatMult * ceilLog2(clusterSize)  # :65-67


def gossipDisseminationTime(repeatMult: int, clusterSize: int, gossipInterval: int) -> int:
    return gossipPeriodsToSpread(repeatMult, clusterSize) * gossipInterval  # :77-79


def gossipTimeoutToSweep(repeatMult: int, clusterSize: int, gossipInterval: int) -> int:
    return gossipPeriodsToSweep(repeatMult, clusterSize) * gossipInterval  # :88-90


def gossipPeriodsToSweep(repeatMult: int, clusterSize: int) -> int:
    return 2 * (gossipPeriodsToSpread(repeatMult, clusterSize) + 1)  # :99-102


def gossipPeriodsToSpread(repeatMult: int, clusterSize: int) -> int:
    return repeatMult * ceilLog2(clusterSize)  # :111-113


def suspicionTimeout(suspicionMult: int, clusterSize: int, pingInterval: int) -> int:
    return suspicionMult * ceilLog2(clusterSize) * pingInterval  # :123-125
