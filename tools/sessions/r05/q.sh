#!/bin/bash
# Round 5, session Q: the infectedFrom kernels' positions per wave (SWIM_PCHUNK 1024, product; 256;
# 128) on C2, C4's schedule at 65,536 and C3, with events around every kernel class (--timing all).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_q
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 --timing all > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
for wl in c2 c4d65 c3; do
  b ${wl} "" --workload $wl --steps 20 --warmup 5 && \
  b ${wl}_pc256 variants_ab/libswimhip_pc256.so --workload $wl --steps 20 --warmup 5 && \
  b ${wl}_pc128 variants_ab/libswimhip_pc128.so --workload $wl --steps 20 --warmup 5 || exit 1
done
