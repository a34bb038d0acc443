"""The cost of the library-driven exchanges on one GPU: bench.py's workload on a one-rank
RCCL group (ShardedSwimCluster: every exchange of a period goes through the library's communicator to
itself, with its status all-gather and host stops) against the unsharded handle, the same seed, faults
and periods; ms per period of each and the difference. Also checks that the two end bit-exact.

    python tools/exchange_overhead.py [workload] [periods] [warmup] [repeats]
"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scalecube-cluster_amd"))


def main(workload="c3", periods=20, warmup=5, reps=1, seed=1):
    import torch
    import torch.distributed as dist

    import bench

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        # interleaved repeats (unsharded, sharded, unsharded, sharded, ...): the unsharded period alone
        # moves by ~0.15 ms from box to box and run to run, about the size of the difference measured
        out = {False: [], True: []}
        digests = {}
        for rep in range(reps):
            for sharded in (False, True):
                c = bench.make_cluster(workload, 0, seed, sharded=sharded)
                c.step(warmup)
                bench.inject_faults(c, workload, warmup, seed)
                c.sync()
                t0 = time.perf_counter()
                for _ in range(periods // 5):
                    c.step_async(5)
                    c.sync()
                ms = (time.perf_counter() - t0) * 1e3 / periods
                out[sharded].append(ms)
                digests.setdefault(sharded, c.digest())
                print(f"rep {rep} {'one-rank RCCL' if sharded else 'unsharded'}: {ms:.3f} ms/period", flush=True)
                del c
                torch.cuda.empty_cache()
        assert digests[False] == digests[True], "digests differ"
        u, s_ = min(out[False]), min(out[True])
        print(f"exchange overhead: {s_ - u:.3f} ms/period (best of {reps}: {s_:.3f} against {u:.3f}; "
              f"{periods} periods of {workload} after {warmup}); digests equal", flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "c3", int(a[1]) if len(a) > 1 else 20, int(a[2]) if len(a) > 2 else 5,
         int(a[3]) if len(a) > 3 else 1)
