#!/bin/bash
# Round 5, session AG: k_gossip_pairprune with a wave per (pair, chunk) walking the pair's records
# (pw1) instead of a wave per (pair, record slot, chunk): the parity file + sharded through pw1, then
# C2 (twice), C3, C4's schedule against the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ag
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_pw1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity_pw1.log 2>&1
rc=$?; echo "pytest pw1 rc=$rc" >> $out/status.log
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
for r in 1 2; do
  for v in "" pw1; do
    lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
    b c2${v:+_$v}_r$r "$lib" --workload c2 --steps 20 --warmup 5 || exit 1
  done
done
for v in "" pw1; do
  lib=""; [ -n "$v" ] && lib=variants_ab/libswimhip_$v.so
  b c3${v:+_$v} "$lib" --steps 20 --warmup 5 && \
  b c4d65${v:+_$v} "$lib" --workload c4d65 --steps 20 --warmup 5 || exit 1
done
