#!/bin/bash
# Round-3 GPU check of the delay model and the sharded N x K fix, then the C5 storm probes. A test
# failure (pytest rc 1) still lets the probes run; any other status (a fault, an abort, a time
# limit) ends the call there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_behaviour.py tests/test_sharded.py -m gpu -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "${PYTEST_K:-delay or behaviour or nxk_shards or spill or radix}" \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log
[ $rc -le 1 ] || exit $rc
[ -n "$NO_PROBE" ] && exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5s 18 40 > $out/probe_c5s.log 2>&1
rc=$?; echo "c5s rc=$rc" >> $out/status.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/probe_storm.py c5 17 25 > $out/probe_c5.log 2>&1
rc=$?; echo "c5 rc=$rc" >> $out/status.log
exit $rc
