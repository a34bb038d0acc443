#!/bin/bash
# Round 6, session H: A/B on C3's driver window of the select list-quad prefetch (SWIM_SEL_PF=1) and the
# batched apply's merge pass loading 4 bitmap words' marks per step (SWIM_AW_MW=4) against the product
# (AW_DIRECT 2); C4's schedule and C2 for the select variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_h
mkdir -p $out
for v in direct2 selpf mw4 direct2 selpf mw4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 \
     --no-cpu-baseline --converge 0 > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
for w in c4d65 c2; do
  for v in direct2 selpf; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 \
       --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
