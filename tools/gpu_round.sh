#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench (default workload), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
echo "start $(date +%T)" > $out/status.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
  && echo "smoke ok $(date +%T)" >> $out/status.log \
  && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
       > $out/pytest_gpu.log 2>&1 \
  && echo "pytest ok $(date +%T)" >> $out/status.log \
  && timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $out/bench.json 2> $out/bench.err \
  && echo "bench ok $(date +%T)" >> $out/status.log \
  && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
       python3 bench.py --no-cpu-baseline --converge 0 ${BENCH_ARGS} > $out/prof_bench.json 2> $out/prof_bench.err \
  && echo "rocprof ok $(date +%T)" >> $out/status.log
rc=$?
echo "rc=$rc $(date +%T)" >> $out/status.log
exit $rc
