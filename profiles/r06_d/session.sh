#!/bin/bash
# Round 6, session D: quiet periods (the gossip rounds of a period where nobody holds a gossip are
# skipped): their A/B test, steady65k and the driver's C3 command on it, the ring probe, then the whole
# -m gpu suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_d
mkdir -p $out
timeout -k 10 200 python3 -u bench.py --workload steady65k --steps 60 --warmup 3 --no-cpu-baseline --converge 0 \
   > $out/bench_steady65k.json 2> $out/bench_steady65k.err
rc=$?; echo "steady rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --workload c3k --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_c3k.json 2> $out/bench_c3k.err
rc=$?; echo "c3k rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u -m pytest tests/test_quiet.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_quiet.log 2>&1
rc=$?; echo "quiet rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_ring.py > $out/probe_ring.log 2>&1
rc=$?; echo "probe rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   --ignore=tests/test_quiet.py --deselect tests/test_c4_rehearsal.py::test_c4_schedule_65536_world8_matches_unsharded \
   --deselect tests/test_c4_rehearsal.py::test_c5_schedule_131072_world8_matches_unsharded --durations 30 > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
