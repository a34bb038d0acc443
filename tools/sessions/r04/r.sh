#!/bin/bash
# Round 4, session R: k_gossip_select's MIXED entries (those whose 32 infection rounds must be read)
# flattened across the wave instead of walked per lane: the parity file through the product (the
# per-entry code moved into a lambda) and through the flattened build, then C3 and C4's schedule
# with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_r
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
   --timeout-method thread > $out/pytest_product.log 2>&1
rc=$?; echo "pytest product rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_self1.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_self1.log 2>&1
rc=$?; echo "pytest self1 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in self0 self1; do
  for wl in c3 c4d65; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload $wl \
       --no-cpu-baseline --converge 0 > $out/bench_${wl}_$v.json 2> $out/bench_${wl}_$v.err
    rc=$?; echo "$wl $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
