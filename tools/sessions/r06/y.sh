#!/bin/bash
# Round 6, session Y: run starts per list position (act_rw) against the same tree built with -DSWIM_ACT_RW=0 (ab/)
# on C3, C2 and C4's schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_y
mkdir -p $out
for w in c3 c2 c4d65; do
  for v in new base new2; do
    lib=""
    [ $v = base ] && lib=$PWD/ab/libswimhip_noactrw.so
    SWIMHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline \
       --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
