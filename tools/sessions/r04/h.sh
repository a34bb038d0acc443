#!/bin/bash
# Round 4, session H: C4's schedule at 65,536 dense (full-size property test); the driver's bench
# command with the MembershipEvent ring; C5's storm (256 crashes) at 2^19 members on a 2^18 ring.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_h
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k c4_schedule -x -v -p no:cacheprovider --timeout 280 \
   --timeout-method thread > $out/pytest_c4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5 18 45 23 524288 > $out/c5_n2e19_storm.log 2>&1
rc=$?; echo "probe rc=$rc" >> $out/status.log; exit $rc
