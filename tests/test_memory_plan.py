"""The node configurations' memory plans on one MI355X: rank 0's shard of C4
(262,144 dense members over 8 GPUs: 32,768 observer rows, a 5,128 * 1,024-slot gossip ring, 1.25x the ~4.2e6
live one-gossip slots C4's storm law predicts) and of C5 (2^20 members, N x K with
K = 256, over 8 GPUs: 131,072 rows, a 2^20-slot ring against ~4e5 live batch slots) is created,
initialised and given its exchange buffers by tools/c4_alloc_probe.py in a child process; the shard
must fit with headroom left for RCCL and the HIP context. Stepping needs the other seven ranks."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _probe(workload):
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "c4_alloc_probe.py"), "8", workload],
                         capture_output=True, text=True, timeout=240, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_c4_shard_fits_with_ring_headroom():
    r = _probe("c4")
    print(r)
    assert r["rows_per_gpu"] == 32768 and r["gossip_ring_slots"] >= 1.25 * 4.2e6
    assert r["infection_round_bits"] == 4
    assert r["hbm_left_gib"] >= 24.0, r  # RCCL buffers, the HIP context and the allocator's slack


def test_c5_shard_fits_with_headroom():
    r = _probe("c5")
    print(r)
    assert r["rows_per_gpu"] == 131072 and r["gossip_ring_slots"] >= 1.25 * 4.0e5
    assert r["hbm_used_gib"] <= 0.75 * r["hbm_total_gib"], r
