#!/bin/bash
# Round-3: parity + behaviour suites on the split pull kernel, then the occupancy A/B (C3 20/5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03j}
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py tests/test_behaviour.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_r03_occ.sh ${1:-r03j}/occ
