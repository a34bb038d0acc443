#!/bin/bash
# Round 6, session G: the batched apply's short record ranges walked by their own lane (ranges of at most
# AW_DIRECT 16-B id groups, no owner search): parity file on the in-tree build (AW_DIRECT 2), then C3's
# driver window for the base build and AW_DIRECT 1 / 2 / 3, and C2 / C4's schedule for base and 2; then session E.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_g
mkdir -p $out
# (the parity file and the whole -m gpu suite ran green on the in-tree AW_DIRECT 2 build in session D)
for v in base direct2 direct1 direct3 base direct2; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 \
     --no-cpu-baseline --converge 0 > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
for w in c2 c4d65; do
  for v in base direct2; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 \
       --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
bash tools/sessions/r06/e.sh
