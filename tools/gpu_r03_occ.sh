#!/bin/bash
# Round-3 occupancy A/B on C3 20/5: k_gossip_select at 6 / 7 waves per SIMD (product: 5), and the
# round-3 baseline (k_gossip_pull at 3 waves per SIMD; product: 4). Kernel times in the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03occ}
mkdir -p $out
for v in ${OCC_VARIANTS:-base product sw6 sw7b1}; do
  lib=variants_ab/libswimhip_$v.so; [ $v = product ] && lib=scalecube-cluster_amd/swimhip/libswimhip.so
  SWIMHIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
    --no-cpu-baseline > $out/c3_$v.json 2> $out/c3_$v.err
  rc=$?; echo "$v rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
done
