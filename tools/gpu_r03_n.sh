#!/bin/bash
# Round-3 refresh on the final tree: bench lines of C2, C5's one-GPU shapes and C3's 20/5 window,
# the rocprofv3 kernel stats of C3 20/5, and one cache pass (L2 hits / misses per kernel) over it.
# Each GPU step has its own limit; the chain stops at the first failure.
#   usage: tools/gpu_r03_n.sh <tag>   -> gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r03n}
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/c3.json 2> $out/c3.err \
  && echo "c3 ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 5 --converge 0 > $out/c2.json 2> $out/c2.err \
  && echo "c2 ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c5s --steps 20 --warmup 5 --converge 120 --no-cpu-baseline \
       > $out/c5s.json 2> $out/c5s.err \
  && echo "c5s ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c5g --steps 20 --warmup 5 --converge 130 --no-cpu-baseline \
       > $out/c5g.json 2> $out/c5g.err \
  && echo "c5g ok" >> $out/status.log \
  && bash tools/profile.sh ${1:-r03n}_c3 --steps 20 --warmup 5 \
  && echo "c3 prof ok" >> $out/status.log \
  && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/l2 -o run -- \
       python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/l2_bench.json 2> $out/l2_bench.err \
  && echo "l2 ok" >> $out/status.log \
  && SWIMHIP_LIB=variants_ab/libswimhip_aprof.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --converge 0 \
       --no-cpu-baseline > $out/aprof.json 2> $out/aprof.err \
  && echo "aprof ok" >> $out/status.log
rc=$?
echo "rc=$rc" >> $out/status.log
exit $rc
