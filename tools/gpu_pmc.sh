#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters: one pass per counter group
# (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: never in one pass), kernel-trace only, no tracing
# domains. A shorter timed region than the default bench keeps the instrumented run short.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-pmc}
out=gpurun_out/$tag
mkdir -p $out
args="--steps ${PMC_STEPS:-100} --no-cpu-baseline --converge 0 ${BENCH_ARGS}"
echo "start $(date +%T)" > $out/status.log
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
    python3 bench.py $args > $out/fetch_bench.json 2> $out/fetch_bench.err \
  && echo "fetch ok $(date +%T)" >> $out/status.log \
  && timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
    python3 bench.py $args > $out/write_bench.json 2> $out/write_bench.err \
  && echo "write ok $(date +%T)" >> $out/status.log \
  && python3 tools/pmc_summary.py $out > $out/pmc_traffic.json \
  && echo "summary ok $(date +%T)" >> $out/status.log
rc=$?
echo "rc=$rc $(date +%T)" >> $out/status.log
exit $rc
