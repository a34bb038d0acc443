"""ctypes mirror of include/swimhip.h and the loader for libswimhip.so.

The product path is the HIP library only: `load_swimhip()` raises if the in-tree
libswimhip.so is missing or cannot be loaded — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)  # scalecube-cluster_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
# SWIMHIP_LIB: an alternative build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("SWIMHIP_LIB") or os.path.join(HERE, "libswimhip.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "swimhip.h")

SWIM_OK = 0
SWIM_EINVAL = -22
SWIM_ENOMEM = -12
SWIM_EHIP = -5
SWIM_ERCCL = -6
SWIM_EOVERFLOW = -75

ABSENT, ALIVE, SUSPECT, DEAD = 0, 1, 2, 0xFFFFFFFF

EV_ADDED, EV_REMOVED, EV_UPDATED = 1, 2, 3
EV_GOSSIP, EV_FD = 8, 9  # GossipProtocol.listen() / FailureDetector.listen() streams (include/swimhip.h)
TRACE_FD = 1
R_FAILURE_DETECTOR_EVENT, R_MEMBERSHIP_GOSSIP, R_SYNC, R_INITIAL_SYNC, R_SUSPICION_TIMEOUT = 0, 1, 2, 3, 4
DELIVER_FORWARD = 0x100  # swim_deliver_records reason flag: the records are gossips new to the observer


def pack(inc: int, code: int) -> int:
    return ((inc << 2) | code) & 0xFFFFFFFF


class SwimConfig(ctypes.Structure):
    _fields_ = [
        ("n_members", ctypes.c_uint32),
        ("mode", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
        ("ping_interval_ms", ctypes.c_int32),
        ("ping_timeout_ms", ctypes.c_int32),
        ("ping_req_members", ctypes.c_int32),
        ("gossip_fanout", ctypes.c_int32),
        ("gossip_interval_ms", ctypes.c_int32),
        ("gossip_repeat_mult", ctypes.c_int32),
        ("sync_interval_ms", ctypes.c_int32),
        ("sync_timeout_ms", ctypes.c_int32),
        ("suspicion_mult", ctypes.c_int32),
        ("metadata_timeout_ms", ctypes.c_int32),
        ("n_seeds", ctypes.c_uint32),
        ("gossip_capacity", ctypes.c_uint32),
        ("event_capacity", ctypes.c_uint32),
        ("sync_capacity", ctypes.c_uint32),
        ("tracked_subjects", ctypes.c_uint32),
        ("n_initial", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("shard_rank", ctypes.c_uint32),
        ("shard_world", ctypes.c_uint32),
        ("gossip_batching", ctypes.c_uint32),
        ("record_capacity", ctypes.c_uint32),
        ("infection_round_bits", ctypes.c_uint32),
        ("dict_subjects", ctypes.c_uint32),
    ]


class SwimEvent(ctypes.Structure):
    _fields_ = [
        ("period", ctypes.c_uint64),
        ("observer", ctypes.c_uint32),
        ("subject", ctypes.c_uint32),
        ("record", ctypes.c_uint32),
        ("type", ctypes.c_uint8),
        ("reason", ctypes.c_uint8),
        ("phase", ctypes.c_uint8),
        ("pad", ctypes.c_uint8),
    ]


STAT_FIELDS = [
    "period",
    "fd_probes",
    "fd_direct_ok",
    "fd_ping_req",
    "fd_suspect_events",
    "fd_alive_events",
    "gossips_created",
    "gossip_first_receipts",
    "gossip_sends",
    "syncs_sent",
    "syncs_delivered",
    "sync_acks_delivered",
    "records_accepted",
    "events_added",
    "events_removed",
    "suspicion_timeouts",
    "refutations",
    "overflow",
    "live_gossip_slots",
    "not_converged",
    "gossip_scanned",
    "gossip_probes",
    "sweep_cells",
    "merge_cells",
    "ack_cells",
    "gossip_hd_words",
    "gossip_window_words",
    "gossip_pull_words",
    "infected_pruned_pairs",
    "infected_records",
    "infected_suppressed",
    "apply_words",
    "apply_runs",
    "apply_subjects",
    "fd_dead_events",
    "apply_spills",
    "apply_records",
    "live_gossip_records",
    "events_updated",
    "apply_pairs",
    "commit_radix",
    "escape_entries",
    "escape_capacity",
    "apply_skipped",
    "apply_bitmaps",
    "apply_bitmap_records",
    "quiet_periods",
]


class SwimStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in STAT_FIELDS]


MAX_WORLD = 64
X_DONE, X_ALLGATHER, X_ALLTOALLV, X_ALLREDUCE_MAX = 0, 1, 2, 3


class SwimXchg(ctypes.Structure):
    """swim_xchg (include/swimhip.h): one cross-shard exchange of a sharded period."""

    _fields_ = [
        ("op", ctypes.c_uint32),
        ("world", ctypes.c_uint32),
        ("send_words", ctypes.c_uint64),
        ("send_counts", ctypes.c_uint64 * MAX_WORLD),
        ("recv_counts", ctypes.c_uint64 * MAX_WORLD),
        ("recv_stride", ctypes.c_uint64),
    ]


# swim_transport (include/swimhip.h): the host's collectives, called back by the library
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                ctypes.c_void_p)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)


class SwimTransport(ctypes.Structure):
    _fields_ = [
        ("ctx", ctypes.c_void_p),
        ("host_staged", ctypes.c_uint32),
        ("allgather", ALLGATHER_FN),
        ("alltoallv", ALLTOALLV_FN),
    ]


# (name, restype, argtypes) for every entry point of include/swimhip.h
_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_pU32 = ctypes.POINTER(ctypes.c_uint32)
_pU64 = ctypes.POINTER(ctypes.c_uint64)
_pU8 = ctypes.POINTER(ctypes.c_uint8)


def api_table(prefix: str):
    """Signature table shared by libswimhip (prefix 'swim_') and the oracle ('oracle_')."""
    return [
        (prefix + "create", _I, [ctypes.POINTER(SwimConfig), ctypes.POINTER(_P)]),
        (prefix + "destroy", _I, [_P]),
        (prefix + "set_loss", _I, [_P, _U32]),
        (prefix + "set_delay", _I, [_P, _U32]),
        (prefix + "set_partition", _I, [_P, _pU8, _U32, _U64, _U64]),
        (prefix + "block_link", _I, [_P, _U32, _U32, _I]),
        (prefix + "block_inbound", _I, [_P, _U32, _U32, _I]),
        (prefix + "crash", _I, [_P, _pU32, _U32]),
        (prefix + "leave", _I, [_P, _pU32, _U32]),
        (prefix + "join", _I, [_P, _pU32, _U32]),
        (prefix + "restart", _I, [_P, _pU32, _pU32, _U32]),
        (prefix + "update_metadata", _I, [_P, _pU32, _U32]),
        (prefix + "spread", _I, [_P, _U32, _U32]),
        (prefix + "trace", _I, [_P, _U32]),
        (prefix + "deliver_records", _I, [_P, _U32, _pU32, _pU32, _U32, _U32]),
        (prefix + "step", _I, [_P, _U32]),
        (prefix + "drain_events", _I, [_P, ctypes.POINTER(SwimEvent), _U64, _pU64]),
        (prefix + "read_view", _I, [_P, _U32, _pU32, _U32]),
        (prefix + "read_deadlines", _I, [_P, _U32, _pU32, _U32]),
        (prefix + "digest", _I, [_P, _pU64, _pU64]),
        (prefix + "read_presence", _I, [_P, _pU32, _pU32, _U32]),
        (prefix + "stats_get", _I, [_P, ctypes.POINTER(SwimStats)]),
    ]


SWIM_ONLY = [
    ("swim_step_async", _I, [_P, _U32]),
    ("swim_sync", _I, [_P]),
    ("swim_last_error", ctypes.c_char_p, [_P]),
    ("swim_kat_is_overrides", _I, [_pU32, _pU32, _pU8, _U64]),
    ("swim_kat_philox", _I, [_U64, _U32, _pU32, _pU32, _U64]),
    ("swim_kat_philox4", _I, [_U64, _U32, _pU32, _pU32, _U64]),
    ("swim_kat_scan", _I, [_pU32, _U64, _pU32, _pU32, _pU32, _pU32]),
    ("swim_debug_holdings", _I, [_P, _U32, _pU32, _pU32, _U32, _pU32]),
    ("swim_debug_member_state", _I, [_P, _pU32, _U32]),
    ("swim_debug_sends", _I, [_P, _pU64, _U32]),
    ("swim_kernel_time", _I, [_P, _U32, ctypes.POINTER(ctypes.c_double), _pU64]),
    ("swim_kernel_time_reset", _I, [_P, _I]),
    ("swim_shard_buffer_words", _I, [_P, _pU64, _pU64]),
    ("swim_shard_attach", _I, [_P, _P, _P]),
    ("swim_shard_step", _I, [_P, ctypes.POINTER(SwimXchg)]),
    ("swim_shard_set_transport", _I, [_P, ctypes.POINTER(SwimTransport)]),
    ("swim_rccl_unique_id", _I, [_pU8]),
    ("swim_shard_comm_init", _I, [_P, _pU8, _U32, _U32]),
]


def bind(lib, table):
    for name, res, args in table:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/swimhip.h."""
    import re

    txt = open(path).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(swim_\w+)\s*\(", txt, re.M)))


_LIB = None


class NativeMissing(RuntimeError):
    pass


def load_swimhip():
    """Load the in-tree HIP library. Fails loudly: no CPU fallback exists."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeMissing(
            f"libswimhip.so not built at {LIB_PATH}; run __graft_entry__.build() (hipcc --offload-arch=gfx950)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    bind(lib, api_table("swim_") + SWIM_ONLY)
    _LIB = lib
    return lib
