#!/bin/bash
# Round 5, session AE: k_gossip_record over 2,048 / 4,096 workgroups (rg2048, rg4096) instead of 1,024
# (product: 4 waves per SIMD of a kernel whose registers allow 7): C2 (records at 256 list positions
# per wave), C4's schedule, C3; rocprofv3 kernel stats of C2 through rg2048.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ae
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
for r in 1 2; do
  for v in "" rg2048 rg4096; do
    lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
    sfx=${v:+_$v}_r$r
    b c2$sfx "$lib" --workload c2 --steps 20 --warmup 5 || exit 1
  done
done
for v in "" rg2048; do
  lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
  b c4d65${v:+_$v} "$lib" --workload c4d65 --steps 20 --warmup 5 && \
  b c3${v:+_$v} "$lib" --steps 20 --warmup 5 || exit 1
done
