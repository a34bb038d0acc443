#!/bin/bash
# Round 6, session K: the FD commit sorted within its bound (two gossips per member plus the host's staged
# ones: one k_rs_fused launch or k_commit's LDS sort instead of the eleven-launch radix chain); the
# parity file and the sharded tests on it; steady65k / C3 / C2 / c4d65 / c3half65k against a variant that
# sorts every commit in one launch (SWIM_RS_FUSE_ALL=1, the end-of-period commit too).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_k
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py tests/test_quiet.py -m gpu -x -v \
   -p no:cacheprovider --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for w in steady65k c3 c2 c4d65; do
  for v in prod fuseall; do
    st=20; [ $w = steady65k ] && st=60
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload $w --steps $st \
       --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
