"""Phase profile of the batched apply and of select on the bench's C3 window: run with a library
built with -DSWIM_APPLY_PROF -DSWIM_SEL_PROF (SWIMHIP_LIB=...); swim_destroy prints the per-phase
wall clock summed over waves (100 MHz clock) to stderr.
python tools/phase_profile.py [workload] [steps] [warmup]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scalecube-cluster_amd")]
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 5
c = bench.make_cluster(wl, 0, seed=1)
c.step(warmup)
bench.inject_faults(c, wl, warmup, 1)
c.step(steps)
print({k: c.stats()[k] for k in ("gossips_created", "gossip_first_receipts", "apply_records", "apply_subjects")}, flush=True)
c.close()
