#!/bin/bash
# Round 4, session AE: k_sync_merge / k_sync_ack at their natural 5 waves per SIMD (sw1) or held to 6 /
# 8 (sw6 / sw8), on the fault-free steady state (SYNC-bound) and C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_ae
mkdir -p $out
for v in sw1 sw6 sw8; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --workload steady65k \
     --no-cpu-baseline > $out/bench_steady_$v.json 2> $out/bench_steady_$v.err
  rc=$?; echo "steady $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
     --no-cpu-baseline > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
