#!/bin/bash
# Round 5, session AB: the pull without the branch on the receiver's holdings before the senders'
# window loads (nsk: they issue beside the holdings load) against the product: C3, C4's schedule, C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ab
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
for r in 1 2; do
  for v in "" nsk; do
    lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
    sfx=${v:+_$v}_r$r
    b c3$sfx "$lib" --steps 20 --warmup 5 && \
    b c4d65$sfx "$lib" --workload c4d65 --steps 20 --warmup 5 && \
    b c2$sfx "$lib" --workload c2 --steps 20 --warmup 5 || exit 1
  done
done
