#!/bin/bash
# Round-3: the spill/pair and sharded N x K tests, the C5 storm probes, and the batched-apply phase
# profile on the C3 20/5 window. pytest rc 1 (a failed assertion) lets the rest run; anything else
# (fault, abort, time limit) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03e}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "spill or nxk_shards" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
SWIMHIP_LIB=variants_ab/libswimhip_prof.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --converge 0 \
  --no-cpu-baseline > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "prof rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5s 18 40 > $out/probe_c5s.log 2>&1
rc=$?; echo "c5s rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5 17 25 > $out/probe_c5.log 2>&1
rc=$?; echo "c5 rc=$rc" >> $out/status.log
exit $rc
