#!/bin/bash
# Round 6, session J: the quiet A/B test (exact counters only), C4's schedule and C2 on the driver's window
# with the flattened lossy draws, then the C4 / C5 rehearsals on 8 gloo shards (session F).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_j
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests/test_quiet.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 \
   --timeout-method thread > $out/pytest_quiet.log 2>&1
rc=$?; echo "quiet rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for w in c4d65 c2; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
     > $out/bench_$w.json 2> $out/bench_$w.err
  rc=$?; echo "$w rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/sessions/r06/f.sh
