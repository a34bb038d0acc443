#!/bin/bash
# Round 5, session AC: rehearsal of bench.py's multi-GPU path (observer-row shards, the library driving
# its exchanges) on ONE GPU: N ranks share cuda:0 and exchange over gloo (the driver's node run uses the
# library's RCCL communicator). The work counters of C2 at 1 / 2 / 4 shards and of C3's storm at 1 / 4
# shards must be identical (sharding is bit-exact); the timings are not meaningful (host-staged gloo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ac
mkdir -p $out
run() {  # name, nproc, bench args...
  local name=$1 n=$2; shift 2
  if [ "$n" = 1 ]; then
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  else
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --backend gloo "$@" --no-cpu-baseline --converge 0 \
      > $out/bench_$name.json 2> $out/bench_$name.err
  fi
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
run c2_x1 1 --workload c2 --steps 20 --warmup 5 && \
run c2_x2 2 --workload c2 --steps 20 --warmup 5 && \
run c2_x4 4 --workload c2 --steps 20 --warmup 5 && \
run c3_x1 1 --steps 6 --warmup 5 && \
run c3_x4 4 --steps 6 --warmup 5 || exit 1
