#!/bin/bash
# Round 5, session L: SYNC merge / ack over 32-member blocks (no work lists). The whole -m gpu suite
# as the driver runs it, then C3 and steady65k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_l
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload steady65k --steps 60 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_steady65k.json 2> $out/bench_steady65k.err
rc=$?; echo "steady rc=$rc" >> $out/status.log; exit $rc
