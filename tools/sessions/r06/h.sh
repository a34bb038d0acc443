#!/bin/bash
# Round 6, session H: A/B on C3's driver window of the select list-quad prefetch (SWIM_SEL_PF=1) and the
# batched apply's merge pass loading 4 bitmap words' marks per step (SWIM_AW_MW=4) against the product;
# C4's schedule for the select variant; the lossy pull's draws flattened across the wave (SWIM_PULL_FLAT, at 6
# and 4 waves per SIMD) on C4's schedule and C2, with the lossy parity cases; SQ stall counters of C4's schedule and C2 (the lossy pull).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_h
mkdir -p $out
for r in 1 2; do
  for v in base selpf mw4; do
    SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 \
       --no-cpu-baseline --converge 0 > $out/bench_c3_${v}_r$r.json 2> $out/bench_c3_${v}_r$r.err
    rc=$?; echo "c3 $v r$r rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  done
done
for v in base selpf pflat pflat4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload c4d65 --steps 20 \
     --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c4d65_$v.json 2> $out/bench_c4d65_$v.err
  rc=$?; echo "c4d65 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
for v in base pflat pflat4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python3 -u bench.py --workload c2 --steps 20 \
     --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c2_$v.json 2> $out/bench_c2_$v.err
  rc=$?; echo "c2 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_pflat4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
   -p no:cacheprovider --timeout 300 --timeout-method thread -k "loss or c2 or c4 or delay" > $out/pytest_parity_pflat4.log 2>&1
rc=$?; echo "parity pflat4 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for w in c4d65 c2; do
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM \
      --output-format csv -d $out/sq_$w -o run -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
      > $out/sq_bench_$w.json 2> $out/sq_bench_$w.err
  rc=$?; echo "sq $w rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
  python3 tools/sq_summary.py $out/sq_$w 20 5 > $out/sq_${w}_s20_w5.json
done
