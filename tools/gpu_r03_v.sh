#!/bin/bash
# Round-3: wave scans over DPP row shifts / broadcasts instead of lane shuffles (SWIM_DPP_SCAN build):
# its parity file through that build, then the A/B against the product on C3 20/5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03v}
mkdir -p $out
SWIMHIP_LIB=variants_ab/libswimhip_dpp.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $out/parity_dpp.log 2>&1
rc=$?; echo "dpp parity rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
OCC_VARIANTS="product dpp" bash tools/gpu_r03_occ.sh ${1:-r03v}/ab
