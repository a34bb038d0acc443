#!/bin/bash
# GPU session without the test suite: bench (default workload) + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
echo "start $(date +%T)" > $out/status.log
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $out/bench.json 2> $out/bench.err \
  && echo "bench ok $(date +%T)" >> $out/status.log \
  && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
       python3 bench.py --no-cpu-baseline --converge 0 ${BENCH_ARGS} > $out/prof_bench.json 2> $out/prof_bench.err \
  && echo "rocprof ok $(date +%T)" >> $out/status.log
rc=$?
echo "rc=$rc $(date +%T)" >> $out/status.log
exit $rc
