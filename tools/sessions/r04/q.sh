#!/bin/bash
# Round 4, session Q: k_gossip_pull with 1, 2 (product), 3 or 4 senders' window loads in flight per lane
# (3 also forced to 4 waves per SIMD), on C3's 20/5 window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_q
mkdir -p $out
for v in silp2 silp1 silp3 silp3w4 silp4; do
  SWIMHIP_LIB=$PWD/variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
     --converge 0 > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
