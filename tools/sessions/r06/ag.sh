#!/bin/bash
# Round 6, session AG: AF again with every rank's sync_capacity in its SYNC status row (the SYNC batch check of
# every rank uses each rank's own capacity) - the one-rank RCCL period, the sharded suite, the bench's
# rank spawner and the C4/C5 rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ag
mkdir -p $out
timeout -k 10 500 python3 -u tools/exchange_overhead.py c3 20 5 2 > $out/overhead_new.log 2>&1
rc=$?; echo "overhead new rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_sharded.py tests/test_bench_ranks.py tests/test_c4_rehearsal.py \
   -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations 15 > $out/pytest_sharded.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
