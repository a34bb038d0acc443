#!/bin/bash
# Round 4, session W: k_gossip_select with one list quad per lane per step at 4, 5, 6 and 8 waves per
# SIMD (the register budget the compiler is held to), against the product (2 quads), C3 and C4's schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_w
mkdir -p $out
for v in sb2 sb1w4 sb1w5 sb1w6 sb1w8; do
  for wl in c3 c4d65; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload $wl \
       --no-cpu-baseline --converge 0 > $out/bench_${wl}_$v.json 2> $out/bench_${wl}_$v.err
    rc=$?; echo "$wl $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
