#!/bin/bash
# A/B of library builds on the default bench workload: parity tests on the in-tree build, then the
# bench (no CPU leg, no convergence tail) once per variants/*.so via SWIMHIP_LIB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-ab}
out=gpurun_out/$tag
mkdir -p $out
echo "start $(date +%T)" > $out/status.log
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?" >> $out/status.log; exit 1; }
  echo "pytest ok $(date +%T)" >> $out/status.log
fi
for lib in ${AB_DIR:-variants_ab}/*.so; do
  name=$(basename $lib .so)
  SWIMHIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --converge 0 ${BENCH_ARGS} \
    > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed rc=$?" >> $out/status.log; exit 1; }
  echo "$name ok $(date +%T)" >> $out/status.log
done
echo "rc=0 $(date +%T)" >> $out/status.log
