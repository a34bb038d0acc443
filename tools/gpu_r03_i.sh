#!/bin/bash
# Round-3: the whole -m gpu suite, then the suspicion-sweep A/B over the convergence windows of C3
# and C5's 2^20 geometry (sweep_roofline / converge_kernels_frac in the bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03i}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
for v in product sweepold; do
  lib=variants_ab/libswimhip_$v.so; [ $v = product ] && lib=scalecube-cluster_amd/swimhip/libswimhip.so
  for wl in c3 c5g; do
    SWIMHIP_LIB=$lib timeout -k 10 240 python -u bench.py --workload $wl --steps 20 --warmup 5 --converge 140 \
      --no-cpu-baseline > $out/${wl}_$v.json 2> $out/${wl}_$v.err
    rc=$?; echo "$wl $v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
  done
done
