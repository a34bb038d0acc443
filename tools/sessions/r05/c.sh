#!/bin/bash
# Round 5, session C: touched-column SYNC payloads, merge marks read with the bitmap words, the
# half/half parity test at 1,024; the parity file + wire tests, then the driver's C3 window with
# events on the major kernel classes only (the default) and on every class (A/B of the event cost).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_c
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 --timing all > $out/bench_c3_tall.json 2> $out/bench_c3_tall.err
rc=$?; echo "c3 all rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --workload steady65k --no-cpu-baseline --converge 0 > $out/bench_steady65k.json 2> $out/bench_steady65k.err
rc=$?; echo "steady rc=$rc" >> $out/status.log; exit $rc
