#!/bin/bash
# Round 4, session O: k_gossip_record's loss draws (delivery records of GossipState.infectedFrom) with
# 1 (product), 2 or 4 id-hash loads in flight per lane: the parity file through the 4-wide build, then
# C4's schedule at 65,536 with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_o
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_rec4.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_rec4.log 2>&1
rc=$?; echo "pytest rec4 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in rec1 rec2 rec4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload c4d65 \
     --no-cpu-baseline --converge 0 > $out/bench_c4d65_$v.json 2> $out/bench_c4d65_$v.err
  rc=$?; echo "c4d65 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
