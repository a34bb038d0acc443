#!/bin/bash
# Round-3: the whole -m gpu suite, then the C3 20/5 bench A/B (round-3 baseline, entry bitmaps
# off, product), the apply/select phase profiles, and the C5 storm probes. pytest rc 1 (a failed
# assertion) lets the rest run; anything else (fault, abort, time limit) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03f}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
for v in base nobm product prof; do
  lib=variants_ab/libswimhip_$v.so; [ $v = product ] && lib=scalecube-cluster_amd/swimhip/libswimhip.so
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --converge 0 \
    --no-cpu-baseline > $out/bench_$v.json 2> $out/bench_$v.err
  rc=$?; echo "$v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
done
[ -n "$NO_PROBE" ] && exit 0
timeout -k 10 240 python -u tools/probe_storm.py c5s 18 40 > $out/probe_c5s.log 2>&1
rc=$?; echo "c5s rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u tools/probe_storm.py c5 17 25 > $out/probe_c5.log 2>&1
rc=$?; echo "c5 rc=$rc" >> $out/status.log
exit $rc
