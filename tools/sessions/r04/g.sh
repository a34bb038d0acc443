#!/bin/bash
# Round 4, session G: the wire test at 48 N x K columns; C5 as stated — its storm per period (live
# slots, live records) with a 2^23 record ring, then the bench line; rank 0's C4 shard at 2^22 slots.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_g
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_wire.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
   > $out/pytest_wire.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c4_alloc_probe.py 8 > $out/c4_alloc.json 2> $out/c4_alloc.err
rc=$?; echo "alloc rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5 18 40 23 > $out/c5_storm.log 2>&1
rc=$?; echo "probe rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
grep -q ERROR $out/c5_storm.log && exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --workload c5 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
rc=$?; echo "c5 rc=$rc" >> $out/status.log; exit $rc
