#!/bin/bash
# Round 6, session L: k_gossip_record's lossy / delayed draws flattened across the wave (SWIM_REC_FLAT=1)
# against the product: the lossy and delayed parity cases on the variant, then C2 and c4d65 twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_l
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_recflat.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread -k "loss or c2 or c4 or delay" > $out/pytest_recflat.log 2>&1
rc=$?; echo "parity recflat rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for w in c2 c4d65; do
    for v in prod recflat; do
      SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 \
         --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_${w}_${v}_r$r.json 2> $out/bench_${w}_${v}_r$r.err
      rc=$?; echo "$w $v r$r rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
    done
  done
done
