"""Probe: can two ranks share one GPU over the nccl (RCCL) backend? (all_gather + all_to_all_single)

Run as: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
        --master-port 29511 tools/nccl_probe.py
"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), rank, dtype=torch.int32, device="cuda")
out = torch.empty(4 * world, dtype=torch.int32, device="cuda")
dist.all_gather_into_tensor(out, x)
inp = torch.arange(2 * world, dtype=torch.int32, device="cuda") + 100 * rank
o2 = torch.empty_like(inp)
dist.all_to_all_single(o2, inp, [2] * world, [2] * world)
torch.cuda.synchronize()
print(f"rank {rank}: all_gather {out.tolist()} all_to_all {o2.tolist()}", flush=True)
dist.destroy_process_group()
