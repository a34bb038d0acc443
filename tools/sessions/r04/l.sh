#!/bin/bash
# Round 4, session L: the lossy pull's loss draws with their id-hash loads in flight (k_gossip_pull_loss):
# the parity file on this tree, then C4's schedule at 65,536 with the previous build and 2 / 4 draws per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_l
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
   --timeout-method thread > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in base ilp2 ilp4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload c4d65 \
     --no-cpu-baseline --converge 0 > $out/bench_c4d65_$v.json 2> $out/bench_c4d65_$v.err
  rc=$?; echo "c4d65 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
