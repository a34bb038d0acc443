#!/bin/bash
# Round 6, session AB (certification of the final tree): smoke(), the whole -m gpu suite, the driver's bench
# command (CPU baseline and converge tail), steady65k and C2 on the driver's window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ab
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   --durations 15 > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --workload steady65k --steps 60 --warmup 3 --no-cpu-baseline --converge 0 \
   > $out/bench_steady65k.json 2> $out/bench_steady65k.err
rc=$?; echo "steady rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
   > $out/bench_c2.json 2> $out/bench_c2.err
rc=$?; echo "c2 rc=$rc" >> $out/status.log; exit $rc
