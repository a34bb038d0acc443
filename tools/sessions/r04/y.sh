#!/bin/bash
# Round 4, session Y: the batched apply with 3 instead of 2 quads of entry ids in flight per lane in the
# flattened range stream (aq3), and 4 instead of 2 in the long-range walk (av4), C3 twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_y
mkdir -p $out
for rep in 1 2; do
  for v in abase aq3 av4; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
       --no-cpu-baseline --converge 0 > $out/bench_c3_${v}_$rep.json 2> $out/bench_c3_${v}_$rep.err
    rc=$?; echo "c3 $v $rep rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
