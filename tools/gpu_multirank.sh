#!/bin/bash
# Rehearsal of bench.py's multi-GPU (observer-row shard) path on ONE GPU: N ranks share cuda:0
# and exchange over gloo (the driver's 8-GPU run uses RCCL). Small workload so N shards fit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-multirank}
out=gpurun_out/$tag
mkdir -p $out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --workload c2 --steps 20 --no-cpu-baseline \
      > $out/bench_c2_x$n.json 2> $out/bench_c2_x$n.err || exit $?
done
timeout -k 10 300 python bench.py --workload c2 --steps 20 --no-cpu-baseline > $out/bench_c2_x1.json 2> $out/bench_c2_x1.err
