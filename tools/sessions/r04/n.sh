#!/bin/bash
# Round 4, session N: the batched apply's record ranges — walked one range at a time by the whole wave
# from 64 records up (the product), from 256 up, or never (every range flattened into the quad stream):
# the parity file through the all-flattened build, then C3's 20/5 window with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_n
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_longall.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_longall.log 2>&1
rc=$?; echo "pytest longall rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in long64 long256 longall; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
     --converge 0 > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
