#!/bin/bash
# Round-3: the whole -m gpu suite on the flattened dictionary merge of the batched apply, then its
# A/B on C3 20/5 against the per-lane merge (SWIM_AW_MERGE_OLD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03o}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
OCC_VARIANTS="product mold" bash tools/gpu_r03_occ.sh ${1:-r03o}/ab
