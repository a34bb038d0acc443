#!/bin/bash
# Round-3 bench lines of the non-default BASELINE configs on one GPU, each under its own time limit,
# stopping at the first failure: C2 at the driver's 20/5 window with its same-size CPU baseline (the
# oracle at 4,096 members, like the GPU), C5 at its stated churn (2^20 members, N x K K = 256, 256
# crashes) with the sweep roofline over the convergence window and its kernel stats, then C4's
# schedule on one GPU in N x K mode (262,144 members, 1 % loss, 0.1 % crash) to measure its storm.
#   usage: tools/gpu_lines_r03.sh <tag>   -> gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-lines3}
mkdir -p $out
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 5 --converge 0 > $out/c2.json 2> $out/c2.err \
  && echo "c2 ok" >> $out/status.log \
  && timeout -k 10 400 python -u bench.py --workload c5 --steps 20 --warmup 5 --converge 130 --no-cpu-baseline \
       > $out/c5.json 2> $out/c5.err \
  && echo "c5 ok" >> $out/status.log \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c5 -o run -- \
       python3 bench.py --workload c5 --steps 20 --warmup 5 --converge 0 --no-cpu-baseline > $out/prof_c5.json 2> $out/prof_c5.err \
  && echo "c5 prof ok" >> $out/status.log \
  && timeout -k 10 400 python -u bench.py --workload c4nxk --steps 20 --warmup 5 --converge 0 --no-cpu-baseline \
       > $out/c4nxk.json 2> $out/c4nxk.err \
  && echo "c4nxk ok" >> $out/status.log
rc=$?
echo "rc=$rc" >> $out/status.log
exit $rc
