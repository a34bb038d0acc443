#!/bin/bash
# Round 4, session AC: the batched apply's merge with the next step's entry records and subjects
# loaded before the current step's table cells (mp1) against the product (mp0): the parity file
# through mp1, then C3 twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_ac
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_mp1.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_mp1.log 2>&1
rc=$?; echo "pytest mp1 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in mp0 mp1; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
       --no-cpu-baseline --converge 0 > $out/bench_c3_${v}_$rep.json 2> $out/bench_c3_${v}_$rep.err
    rc=$?; echo "c3 $v $rep rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
