#!/bin/bash
# Round 6, session Z: the commit's bookkeeping in fewer launches (batch-slot word counts in k_dict_claim,
# short slots' entry ids in k_dict_free) against the last commit's library (ab/), then the GPU parity and
# quiet-period files.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_z
mkdir -p $out
for w in c2 c3 steady65k; do
  for v in new base new2; do
    lib=""
    [ $v = base ] && lib=$PWD/ab/libswimhip_head.so
    st=20; [ $w = steady65k ] && st=60
    SWIMHIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload $w --steps $st --warmup 5 --no-cpu-baseline \
       --converge 0 > $out/bench_${w}_$v.json 2> $out/bench_${w}_$v.err
    rc=$?; echo "$w $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_quiet.py -m gpu -x -q -p no:cacheprovider \
   --timeout 400 --timeout-method thread > $out/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $out/status.log; exit $rc
