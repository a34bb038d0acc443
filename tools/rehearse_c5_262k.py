"""C5's schedule (N x K views, K = 256, 256 simultaneous crashes, LAN) at 262,144 members - a quarter of
BASELINE configs[4]'s 2^20 - on 8 observer-row shards (8 gloo ranks sharing cuda:0) against the unsharded
handle, compared every 10 periods through 110 periods, past the suspicion timeouts (5 x bit_length(262,143)
= 90 periods): the one-off beyond tests/test_c4_rehearsal.py's 131,072. The ring has 80 x 1,024 slots
(not a power of two), 1.85x the ~44,300 live batch slots of this storm's peak: two
copies of the cluster with a 2^18-slot ring do not fit one GPU's HBM. Uses that test's worker."""
import os
import sys

import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "scalecube-cluster_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)
import test_c4_rehearsal as t  # noqa: E402

if __name__ == "__main__":
    mp.spawn(t._worker, args=(8, t._free_port(), 1 << 18, dict(gossip_capacity=80 * 1024, tracked_subjects=256), 0.0,
                              256, 3, 110, 10, 1), nprocs=8, join=True)
    print("C5 schedule at 262,144 on 8 shards: equal to the unsharded handle through 110 periods", flush=True)
