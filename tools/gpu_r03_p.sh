#!/bin/bash
# Round-3: the batched apply's phase profile on C3 20/5 (SWIM_APPLY_PROF build): phase wall clocks and
# the share of records that arrive in receipt words received whole.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03p}
mkdir -p $out
SWIMHIP_LIB=variants_ab/libswimhip_aprof.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
  --no-cpu-baseline > $out/aprof.json 2> $out/aprof.err
rc=$?; echo "aprof rc=$rc" >> $out/status.log; exit $rc
