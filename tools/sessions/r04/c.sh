#!/bin/bash
# Round 4, session C: -m gpu suite (hd4 parity, sharded lifecycle, wire bridge, scan KAT), C3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_c
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $out/status.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > $out/bench_c3.json 2> $out/bench_c3.err
echo "c3 rc=$?" >> $out/status.log
