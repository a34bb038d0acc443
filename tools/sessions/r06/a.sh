#!/bin/bash
# Round 6, session A: smoke(), bench.py's own --gpus 4 launch (gloo ranks sharing cuda:0) against --gpus 1,
# the driver's bench command, and C2's PMC traffic over the driver-shaped window (--steps 20 --warmup 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_a
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_bench_ranks.py -m gpu -x -v -p no:cacheprovider --timeout 500 --timeout-method thread \
   > $out/pytest_ranks.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c2 bash tools/gpu_pmc.sh r06_a/pmc_c2
rc=$?; echo "pmc c2 rc=$rc" >> $out/status.log; exit $rc
