#!/bin/bash
# Round 6, session B: bench.py's own --gpus 4 launch against --gpus 1 (protocol counters), the ring probe
# (non-power-of-two ring sizing), the driver's bench command, C2's PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_bench_ranks.py -m gpu -x -v -p no:cacheprovider --timeout 500 --timeout-method thread \
   > $out/pytest_ranks.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_ring.py > $out/probe_ring.log 2>&1
rc=$?; echo "probe rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c2 bash tools/gpu_pmc.sh r06_b/pmc_c2
rc=$?; echo "pmc c2 rc=$rc" >> $out/status.log; exit $rc
