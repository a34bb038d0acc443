#!/bin/bash
# Round-3: batched-apply phase split (words / long ranges / short ranges) on C3 20/5, and the A/B of
# short ranges walked per lane (slane) against the flattened walk, with slane's scenario parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03r}
mkdir -p $out
for v in aprof slaneprof; do
  SWIMHIP_LIB=variants_ab/libswimhip_$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
    --no-cpu-baseline > $out/$v.json 2> $out/$v.err
  rc=$?; echo "$v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
done
OCC_VARIANTS="product slane" bash tools/gpu_r03_occ.sh ${1:-r03r}/ab || exit $?
SWIMHIP_LIB=variants_ab/libswimhip_slane.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q \
  -p no:cacheprovider -k "scenario_parity" --timeout 300 --timeout-method thread > $out/slane_parity.log 2>&1
rc=$?; echo "slane parity rc=$rc" >> $out/status.log; exit $rc
