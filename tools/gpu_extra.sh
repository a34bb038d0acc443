#!/bin/bash
# Sharded parity tests, the multi-rank bench rehearsal, and context bench lines (steady state,
# 0.1 % crash) on one GPU. Every step has its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-extra}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_sharded.py -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $out/pytest_sharded.log 2>&1 \
  && bash tools/gpu_multirank.sh ${1:-extra}/mr \
  && timeout -k 10 300 python bench.py --workload steady65k --steps 100 --no-cpu-baseline > $out/steady65k.json 2> $out/steady65k.err \
  && timeout -k 10 300 python bench.py --workload c3s --steps 100 --no-cpu-baseline > $out/c3s.json 2> $out/c3s.err
