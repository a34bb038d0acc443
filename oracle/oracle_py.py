"""Python binding of the CPU oracle. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It exposes the oracle through the same facade as the product (`OracleCluster` has the
SwimCluster surface) so parity tests drive both implementations call-for-call.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))

from swimhip import _native as nat  # noqa: E402
from swimhip.cluster import SwimCluster  # noqa: E402

LIB_PATH = os.path.join(HERE, "liboracle_swim.so")
_LIB = None


def build(force: bool = False):
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "liboracle_swim.so"], check=True, stdout=subprocess.DEVNULL)


def load_oracle():
    global _LIB
    if _LIB is None:
        build()
        lib = ctypes.CDLL(LIB_PATH)
        nat.bind(lib, nat.api_table("oracle_"))
        lib.oracle_debug_holdings.restype = ctypes.c_int
        P = ctypes.POINTER(ctypes.c_uint32)
        lib.oracle_debug_holdings.argtypes = [ctypes.c_void_p, ctypes.c_uint32, P, P, ctypes.c_uint32, P]
        lib.oracle_debug_member_state.restype = ctypes.c_int
        lib.oracle_debug_member_state.argtypes = [ctypes.c_void_p, P, ctypes.c_uint32]
        lib.oracle_debug_sends.restype = ctypes.c_int
        lib.oracle_debug_sends.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
        lib.oracle_is_overrides.restype = ctypes.c_int
        lib.oracle_is_overrides.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_philox.restype = ctypes.c_uint32
        lib.oracle_philox.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [ctypes.c_uint32] * 4
        lib.oracle_philox4.restype = None
        lib.oracle_philox4.argtypes = [ctypes.c_uint64, ctypes.c_uint32, P, P]
        lib.oracle_cluster_math.restype = ctypes.c_int64
        lib.oracle_cluster_math.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        lib.oracle_perm.restype = ctypes.c_uint32
        lib.oracle_perm.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        _LIB = lib
    return _LIB


class OracleCluster(SwimCluster):
    def __init__(self, config, n_members, seed=0, **kw):
        super().__init__(config, n_members, seed, _lib=load_oracle(), _prefix="oracle_", **kw)


def is_overrides(r1: int, r0: int) -> bool:
    return bool(load_oracle().oracle_is_overrides(r1 & 0xFFFFFFFF, r0 & 0xFFFFFFFF))


def philox(seed: int, kind: int, a: int, b: int, c: int, tick: int) -> int:
    return load_oracle().oracle_philox(seed, kind, a, b, c, tick)


def philox4(seed: int, kind: int, a: int, b: int, c: int, tick: int):
    ctr = (ctypes.c_uint32 * 4)(a, b, c, tick)
    out = (ctypes.c_uint32 * 4)()
    load_oracle().oracle_philox4(seed, kind, ctr, out)
    return list(out)


def cluster_math(which: int, mult: int, n: int, fanout: int = 0) -> int:
    return load_oracle().oracle_cluster_math(which, mult, n, fanout)
