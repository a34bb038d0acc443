#!/bin/bash
# Round-3 GPU check of the delay model and the sharded N x K fix, then the C5 storm probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03d}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_behaviour.py tests/test_sharded.py -m gpu -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "delay or behaviour or nxk_shards or spill or radix" \
  > $out/pytest.log 2>&1; echo "pytest rc=$?" >> $out/status.log
timeout -k 10 300 python -u tools/probe_storm.py c5s 18 40 > $out/probe_c5s.log 2>&1; echo "c5s rc=$?" >> $out/status.log
timeout -k 10 300 python -u tools/probe_storm.py c5 17 25 > $out/probe_c5.log 2>&1; echo "c5 rc=$?" >> $out/status.log
