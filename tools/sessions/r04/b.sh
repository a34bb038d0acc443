#!/bin/bash
# Round 4, session B: -m gpu suite, then bench lines: C3 (driver window), C4's schedule at the sizes one
# GPU holds (65,536 dense, 131,072 N x K).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_b
mkdir -p $out
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $out/status.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > $out/bench_c3.json 2> $out/bench_c3.err
echo "c3 rc=$?" >> $out/status.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --workload c4d65 > $out/bench_c4d65.json 2> $out/bench_c4d65.err
echo "c4d65 rc=$?" >> $out/status.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --workload c4s --no-cpu-baseline > $out/bench_c4s.json 2> $out/bench_c4s.err
echo "c4s rc=$?" >> $out/status.log
