#!/bin/bash
# Round 4, session I: the one-gossip-slot storm (C4's 1 % loss) through the dictionary apply — parity
# file on that build, then C4's schedule at 65,536 with each build; the product's parity file (the
# sweep's events now allocated per workgroup tile, age bounds as one u16 per word) and C3 (base build vs
# this tree; its converge window with the event ring); the fault-free steady state (SYNC-bound), base vs this
# tree (the chunked SYNC first pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_i
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_lossydict.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_lossydict.log 2>&1
rc=$?; echo "pytest lossydict rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in base lossydict; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload c4d65 \
     --no-cpu-baseline --converge 0 > $out/bench_c4d65_$v.json 2> $out/bench_c4d65_$v.err
  rc=$?; echo "c4d65 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
   --timeout-method thread > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest product rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_base.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
   --converge 0 > $out/bench_c3_base.json 2> $out/bench_c3_base.err
rc=$?; echo "c3 base rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in base product; do
  lib=$PWD/variants_ab/libswimhip_base.so; [ $v = product ] && lib=$PWD/scalecube-cluster_amd/swimhip/libswimhip.so
  SWIMHIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --workload steady65k --no-cpu-baseline \
     > $out/bench_steady_$v.json 2> $out/bench_steady_$v.err
  rc=$?; echo "steady $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
