#!/bin/bash
# Round 5, session AD: the other bench workloads on the final tree (documentation): the fault-free
# steady state at 65,536, the half/half partition at 8,192 and 32,768, C4's schedule at 131,072 N x K,
# C5's geometry at 262,144 N x K.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ad
mkdir -p $out
b() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b steady65k --workload steady65k --steps 60 --warmup 5 && \
b c3half8k --workload c3half8k --steps 60 --warmup 5 && \
b c3half32k --workload c3half32k --steps 20 --warmup 5 && \
b c4s --workload c4s --steps 20 --warmup 5 && \
b c5s --workload c5s --steps 20 --warmup 5 || exit 1
