#!/bin/bash
# Round 4, session Z: the batched apply with a 4,096-subject record dictionary (half the LDS per wave,
# so the LDS no longer caps a CU at 4 waves per SIMD) at its natural 4 waves and held to 5 and 6,
# against the product's 8,192, C3 and C4's schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_z
mkdir -p $out
for v in abase d4096 d4096w5 d4096w6; do
  for wl in c3 c4d65; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload $wl \
       --no-cpu-baseline --converge 0 > $out/bench_${wl}_$v.json 2> $out/bench_${wl}_$v.err
    rc=$?; echo "$wl $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
