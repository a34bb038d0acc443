#!/bin/bash
# Round-3: the whole -m gpu suite with the short record ranges of the batched apply read as aligned
# 16-B quads (one owner search per quad), its A/B on C3 20/5 (per-record flattening: srec; one quad
# load in flight per lane: qilp1), and the apply phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03s}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
OCC_VARIANTS="product srec qilp1" bash tools/gpu_r03_occ.sh ${1:-r03s}/ab || exit $?
SWIMHIP_LIB=variants_ab/libswimhip_aprof.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
  --no-cpu-baseline > $out/aprof.json 2> $out/aprof.err
rc=$?; echo "aprof rc=$rc" >> $out/status.log; exit $rc
