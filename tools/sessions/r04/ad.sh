#!/bin/bash
# Round 4, session AD: bench lines of the other configs on the final tree (after the select / pull
# occupancy changes): C2, C4's schedule (65,536 dense; 131,072 N x K), C5's shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_ad
mkdir -p $out
for wl in c4d65 c4s c5s c5g; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload $wl --no-cpu-baseline > $out/bench_$wl.json 2> $out/bench_$wl.err
  rc=$?; echo "$wl rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --workload c2 > $out/bench_c2.json 2> $out/bench_c2.err
rc=$?; echo "c2 rc=$rc" >> $out/status.log; exit $rc
