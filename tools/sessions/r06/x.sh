#!/bin/bash
# Round 6, session X: 8 inline entry ids per short slot (-DSWIM_SID8=1, ab/) against the product's 4
# on C3, C2 and C4's schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_x
mkdir -p $out
for w in c3 c2 c4d65; do
  for v in new sid8 new2; do
    lib=""
    [ $v = sid8 ] && lib=$PWD/ab/libswimhip_sid8.so
    SWIMHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline \
       --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
