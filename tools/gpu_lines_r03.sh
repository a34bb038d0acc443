#!/bin/bash
# Round-3 bench lines of the non-default BASELINE configs on one GPU plus the PMC traffic of the
# default C3 window. Each GPU step has its own time limit; the chain stops at the first failure.
#   C2 at the driver's 20/5 window with its same-size CPU baseline (the oracle at 4,096 members);
#   C5's shapes one GPU holds (2^18 members with its 256 crashes; 2^20 with 8), with the suspicion
#   sweep's roofline over their convergence windows, and a rocprofv3 kernel-stats pass of the 2^18 one;
#   C4's schedule on one GPU in N x K mode (262,144 members, 1 % loss, 0.1 % crash): its storm;
#   the FETCH_SIZE / WRITE_SIZE passes over C3 20/5 (tools/gpu_pmc.sh).
#   usage: tools/gpu_lines_r03.sh <tag>   -> gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-lines3}
mkdir -p $out
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 5 --converge 0 > $out/c2.json 2> $out/c2.err \
  && echo "c2 ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c5s --steps 20 --warmup 5 --converge 120 --no-cpu-baseline \
       > $out/c5s.json 2> $out/c5s.err \
  && echo "c5s ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c5g --steps 20 --warmup 5 --converge 130 --no-cpu-baseline \
       > $out/c5g.json 2> $out/c5g.err \
  && echo "c5g ok" >> $out/status.log \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c5s -o run -- \
       python3 bench.py --workload c5s --steps 20 --warmup 5 --converge 0 --no-cpu-baseline > $out/prof_c5s.json 2> $out/prof_c5s.err \
  && echo "c5s prof ok" >> $out/status.log \
  && timeout -k 10 300 python -u bench.py --workload c4nxk --steps 20 --warmup 5 --converge 0 --no-cpu-baseline \
       > $out/c4nxk.json 2> $out/c4nxk.err \
  && echo "c4nxk ok" >> $out/status.log \
  && PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh ${1:-lines3}/pmc \
  && echo "pmc ok" >> $out/status.log
rc=$?
echo "rc=$rc" >> $out/status.log
exit $rc
