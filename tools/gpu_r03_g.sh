#!/bin/bash
# Round-3: parity + full-size + sharded tests touched by the SYNC merge rewrite and the C5 / pair /
# RCCL test fixes, then the SYNC merge A/B (round-3 baseline, 2 and 4 quads per thread) on the
# fault-free steady state (SYNC-bound) and on C3 with its convergence window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03g}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_sharded.py tests/test_behaviour.py \
  -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
for v in base mu2 product; do
  lib=variants_ab/libswimhip_$v.so; [ $v = product ] && lib=scalecube-cluster_amd/swimhip/libswimhip.so
  SWIMHIP_LIB=$lib timeout -k 10 200 python -u bench.py --workload steady65k --steps 20 --warmup 5 --converge 0 \
    --no-cpu-baseline > $out/steady_$v.json 2> $out/steady_$v.err
  rc=$?; echo "steady $v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --converge 140 \
    --no-cpu-baseline > $out/c3_$v.json 2> $out/c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
done
