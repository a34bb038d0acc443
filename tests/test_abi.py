"""The drop-in boundary: libswimhip.so loads here (no GPU needed) and exports exactly the entry
points include/swimhip.h declares; the oracle mirrors every stateful entry point."""
import ctypes
import os

from swimhip import _native as nat


def test_header_declares_expected_surface():
    syms = nat.header_symbols()
    for s in ("swim_create", "swim_destroy", "swim_step", "swim_drain_events", "swim_read_view", "swim_crash",
              "swim_set_loss", "swim_set_partition", "swim_stats_get", "swim_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    assert os.path.exists(nat.LIB_PATH), "build() must produce the in-tree libswimhip.so"
    lib = ctypes.CDLL(nat.LIB_PATH)
    missing = [s for s in nat.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_table_covers_header():
    bound = {name for name, _, _ in nat.api_table("swim_") + nat.SWIM_ONLY}
    assert set(nat.header_symbols()) == bound


def test_oracle_mirrors_stateful_api():
    import oracle_py

    lib = oracle_py.load_oracle()
    for name, _, _ in nat.api_table("oracle_"):
        assert hasattr(lib, name)


def test_struct_sizes_match_c_layout():
    assert ctypes.sizeof(nat.SwimEvent) == 24
    assert ctypes.sizeof(nat.SwimStats) == 8 * len(nat.STAT_FIELDS)
    assert ctypes.sizeof(nat.SwimConfig) == 112
    assert ctypes.sizeof(nat.SwimXchg) == 16 + 2 * 8 * nat.MAX_WORLD + 8


def test_struct_layout_matches_the_c_compiler(tmp_path):
    """Every field offset of the ctypes mirror equals the C compiler's for include/swimhip.h."""
    import shutil
    import subprocess

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        import pytest

        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{nat.HEADER_PATH}"', "int main(void) {"]
    for cname, cls in (("swim_config", nat.SwimConfig), ("swim_stats", nat.SwimStats),
                       ("swim_event", nat.SwimEvent), ("swim_xchg", nat.SwimXchg)):
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-o", str(exe), str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                               text=True).stdout.split("\n") if line)
    for cname, cls in (("swim_config", nat.SwimConfig), ("swim_stats", nat.SwimStats),
                       ("swim_event", nat.SwimEvent), ("swim_xchg", nat.SwimXchg)):
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_create_without_gpu_fails_cleanly():
    import torch

    if torch.cuda.is_available():
        return
    lib = nat.load_swimhip()
    from swimhip import ClusterConfig, to_swim_config

    cfg = to_swim_config(ClusterConfig.defaultLocalConfig(), 8)
    h = ctypes.c_void_p()
    assert lib.swim_create(ctypes.byref(cfg), ctypes.byref(h)) == nat.SWIM_EHIP


def _create_rc(**fields):
    """swim_create's status for the local preset with `fields` overridden (a handle made on a GPU box is
    destroyed again). Validation precedes every HIP call: EINVAL comes back the same with or without a GPU."""
    lib = nat.load_swimhip()
    from swimhip import ClusterConfig, to_swim_config

    cfg = to_swim_config(ClusterConfig.defaultLocalConfig(), fields.pop("n_members", 8))
    for k, v in fields.items():
        setattr(cfg, k, v)
    h = ctypes.c_void_p()
    rc = lib.swim_create(ctypes.byref(cfg), ctypes.byref(h))
    if rc == nat.SWIM_OK:
        lib.swim_destroy(h)
    return rc


def test_create_refuses_suspicion_beyond_u16_deadline_window():
    # deadlines are u16 cells decoded within +-2^14 periods (swim_device.h dl_dec): suspicionMult x
    # bit_length(N) + 64 must stay below 2^14 (ClusterMath.suspicionTimeout, ClusterMath.java:123-125)
    assert _create_rc(n_members=65536, suspicion_mult=1000) == nat.SWIM_EINVAL  # 17,000 periods
    assert _create_rc(n_members=8, suspicion_mult=4080) == nat.SWIM_EINVAL  # 4 x 4,080 + 64 = 16,384
    assert _create_rc(n_members=8, suspicion_mult=4079) != nat.SWIM_EINVAL


def test_create_refuses_dictionary_beyond_lds():
    # one receiver's entry bitmap (dict_subjects bytes) must fit a workgroup's 160 KiB of LDS
    assert _create_rc(n_members=8, dict_subjects=1 << 18) == nat.SWIM_EINVAL
    assert _create_rc(n_members=8, dict_subjects=1 << 20) == nat.SWIM_EINVAL
    assert _create_rc(n_members=8, dict_subjects=1 << 17) != nat.SWIM_EINVAL
    assert _create_rc(n_members=8, dict_subjects=3000) == nat.SWIM_EINVAL  # not a power of two


def test_create_accepts_non_power_of_two_rings_in_kib():
    assert _create_rc(n_members=8, gossip_capacity=5 * 1024) != nat.SWIM_EINVAL
    assert _create_rc(n_members=8, gossip_capacity=5 * 1024 + 512) == nat.SWIM_EINVAL
