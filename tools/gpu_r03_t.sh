#!/bin/bash
# Round-3: short-range quads (SWIM_AW_SHORT_QUAD build) with every lane shuffling (run s lost records
# whose owner lane was past the quad total): the quad build's scenario parity and the whole -m gpu
# suite through it, then the A/B against the product (per-record flattening) on C3 20/5, and the
# apply phase split of the quad build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03t}
mkdir -p $out
export SWIMHIP_LIB=variants_ab/libswimhip_quad.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "scenario_parity" \
  --timeout 200 --timeout-method thread > $out/parity_quick.log 2>&1
rc=$?; echo "quick parity rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
unset SWIMHIP_LIB
OCC_VARIANTS="product quad" bash tools/gpu_r03_occ.sh ${1:-r03t}/ab || exit $?
SWIMHIP_LIB=variants_ab/libswimhip_aprof.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
  --no-cpu-baseline > $out/aprof.json 2> $out/aprof.err
rc=$?; echo "aprof rc=$rc" >> $out/status.log; exit $rc
