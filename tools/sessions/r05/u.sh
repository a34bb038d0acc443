#!/bin/bash
# Round 5, session U: the batched apply's merge pass testing 2 / 4 groups of 512 bitmap words before
# flattening their blocks (mc2, mc4) against one group at a time (product): C3, C4's schedule, the
# half/half partition at 16,384.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_u
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b c3 "" --steps 20 --warmup 5 && \
b c3_mc2 variants_ab/libswimhip_mc2.so --steps 20 --warmup 5 && \
b c3_mc4 variants_ab/libswimhip_mc4.so --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_mc4 variants_ab/libswimhip_mc4.so --workload c4d65 --steps 20 --warmup 5 && \
b c3half16k "" --workload c3half16k --steps 60 --warmup 5 && \
b c3half16k_mc4 variants_ab/libswimhip_mc4.so --workload c3half16k --steps 60 --warmup 5 && \
b c3_r2 "" --steps 20 --warmup 5 && \
b c3_mc4_r2 variants_ab/libswimhip_mc4.so --steps 20 --warmup 5 || exit 1
