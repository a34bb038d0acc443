#!/bin/bash
# Bench lines of the non-default BASELINE configs on one GPU: C2 (4,096 dense, 5 % loss) with its
# rocprofv3 kernel stats, then the N x K C5 shapes. Every GPU step has its own time limit; the chain
# stops at the first failure (the full C5 storm, which may overflow the ring, runs last).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-lines}
mkdir -p $out
timeout -k 10 400 python -u bench.py --workload c2 --steps 200 --warmup 3 --converge 320 > $out/c2.json 2> $out/c2.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c2 -o run -- \
       python3 bench.py --workload c2 --steps 200 --warmup 3 --converge 0 --no-cpu-baseline > $out/prof_c2.json 2> $out/prof_c2.err \
  && timeout -k 10 400 python -u bench.py --workload c5s --steps 100 --warmup 3 --no-cpu-baseline > $out/c5s.json 2> $out/c5s.err \
  && timeout -k 10 400 python -u bench.py --workload c5g --steps 100 --warmup 3 --no-cpu-baseline > $out/c5g.json 2> $out/c5g.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c5g -o run -- \
       python3 bench.py --workload c5g --steps 100 --warmup 3 --converge 0 --no-cpu-baseline > $out/prof_c5g.json 2> $out/prof_c5g.err \
  && timeout -k 10 400 python -u bench.py --workload c5 --steps 100 --warmup 3 --no-cpu-baseline > $out/c5.json 2> $out/c5.err
rc=$?
echo "rc=$rc" > $out/status.log
exit $rc
