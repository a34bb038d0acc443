#!/bin/bash
# Round 5, session Z: the pull's list quad loaded beside its lack word (as1), and the next step's pair
# loaded before this step's work (as2: 133 VGPRs, 3 waves per SIMD; as2w4: held to 4) against the
# product (the list quad loaded after its lack word said the quad has work): C3, C4's schedule, C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_z
mkdir -p $out
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
for v in "" as1 as2 as2w4; do
  lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
  sfx=${v:+_$v}
  b c3$sfx "$lib" --steps 20 --warmup 5 && \
  b c4d65$sfx "$lib" --workload c4d65 --steps 20 --warmup 5 && \
  b c2$sfx "$lib" --workload c2 --steps 20 --warmup 5 || exit 1
done
