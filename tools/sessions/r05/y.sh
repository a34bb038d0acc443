#!/bin/bash
# Round 5, session Y: the batched apply with a wave per possible receiver (ap0: the dispatcher hands
# out the receiver list) against the persistent grid walking it at a grid stride (product).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_y
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b c3 "" --steps 20 --warmup 5 && \
b c3_ap0 variants_ab/libswimhip_ap0.so --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_ap0 variants_ab/libswimhip_ap0.so --workload c4d65 --steps 20 --warmup 5 && \
b c2 "" --workload c2 --steps 20 --warmup 5 && \
b c2_ap0 variants_ab/libswimhip_ap0.so --workload c2 --steps 20 --warmup 5 && \
b c3half16k "" --workload c3half16k --steps 60 --warmup 5 && \
b c3half16k_ap0 variants_ab/libswimhip_ap0.so --workload c3half16k --steps 60 --warmup 5 && \
b c3_r2 "" --steps 20 --warmup 5 && \
b c3_ap0_r2 variants_ab/libswimhip_ap0.so --steps 20 --warmup 5 || exit 1
