#!/bin/bash
# Round-3: the spill/pair, radix (+ entry bitmaps), sharded N x K / C5-shape and RCCL exchange tests,
# the batched-apply phase profile with and without entry bitmaps on the C3 20/5 window, and the C5
# storm probes. pytest rc 1 (a failed assertion) lets the rest run; anything else (fault, abort,
# time limit) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03e}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "spill or radix or nxk_shards or rccl or c5_shape or delay" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
for v in prof_nobm prof selprof; do
  SWIMHIP_LIB=variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --converge 0 \
    --no-cpu-baseline > $out/bench_$v.json 2> $out/bench_$v.err
  rc=$?; echo "$v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python -u tools/probe_storm.py c5s 18 40 > $out/probe_c5s.log 2>&1
rc=$?; echo "c5s rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5 17 25 > $out/probe_c5.log 2>&1
rc=$?; echo "c5 rc=$rc" >> $out/status.log
exit $rc
