#!/bin/bash
# Round 6, session V: inline entry ids of short slots (k_slot_ids, g_sid) - A/B against the same tree
# built with -DSWIM_SLOT_IDS=0 (ab/) on C3, C2 and C4's schedule, then the GPU parity file.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_v
mkdir -p $out
for w in c3 c2 c4d65; do
  for v in new old new2; do
    lib=""
    [ $v = old ] && lib=$PWD/ab/libswimhip_noslotids.so
    SWIMHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline \
       --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 400 \
   --timeout-method thread > $out/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $out/status.log; exit $rc
