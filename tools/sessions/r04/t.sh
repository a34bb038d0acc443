#!/bin/bash
# Round 4, session T: the batched apply's receipt word loaded beside its list entry (not after it),
# C3 and C4's schedule with the tree before (wbase) and after (wpar), twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_t
mkdir -p $out
for rep in 1 2; do
  for v in wbase wpar; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
       --no-cpu-baseline --converge 0 > $out/bench_c3_${v}_$rep.json 2> $out/bench_c3_${v}_$rep.err
    rc=$?; echo "c3 $v $rep rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
