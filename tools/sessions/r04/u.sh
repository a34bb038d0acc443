#!/bin/bash
# Round 4, session U: k_gossip_select with 1, 2 (product) or 3 list quads per lane per step (with the
# flattened MIXED pass), C3 and C4's schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_u
mkdir -p $out
for v in sb2 sb1 sb3; do
  for wl in c3 c4d65; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload $wl \
       --no-cpu-baseline --converge 0 > $out/bench_${wl}_$v.json 2> $out/bench_${wl}_$v.err
    rc=$?; echo "$wl $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
