#!/bin/bash
# Round 6, session I: the product after session H (the lossy pull's draws flattened across the wave on
# shards of more than 4,096 rows; select / merge variants dropped): the parity file (its radix variant
# pulls without the split, so its lossy scenarios take the flattened draws), the sharded and full-size
# tests, C4's schedule and C2 on the driver's window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_i
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py tests/test_gpu_fullsize.py tests/test_quiet.py \
   -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations 10 > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for w in c4d65 c2; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
     > $out/bench_$w.json 2> $out/bench_$w.err
  rc=$?; echo "$w rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
