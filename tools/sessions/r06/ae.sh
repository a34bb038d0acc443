#!/bin/bash
# Round 6, session AE: the split lossy pull (C2's k_gossip_pull_loss_s4) at 6 waves per SIMD (the product,
# spilling) against 4 and 1 (ab/, -DSWIM_PULL_LOSS_S4_WAVES), interleaved on C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ae
mkdir -p $out
for v in w6 w4 w1 w6b w4b w1b; do
  lib=""
  case $v in w4*) lib=$PWD/ab/libswimhip_s4w4.so;; w1*) lib=$PWD/ab/libswimhip_s4w1.so;; esac
  SWIMHIP_LIB=$lib timeout -k 10 200 python3 -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline \
     --converge 0 --timing all > $out/bench_c2_$v.json 2> $out/bench_c2_$v.err
  rc=$?; echo "c2 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
