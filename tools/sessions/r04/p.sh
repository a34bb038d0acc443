#!/bin/bash
# Round 4, session P: the batched apply's long-range threshold around session N's best (256), and 4
# instead of 2 quads in flight per lane in the flattened stream, on C3's 20/5 window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_p
mkdir -p $out
for v in long128 long256 long512 long1024 long256q4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
     --converge 0 > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
