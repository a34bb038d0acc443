#!/bin/bash
# Round 6, session S: library-driven exchanges without the ordering-only host stops (xorder in
# swim_api.hip) - the sharded suite, the one-rank RCCL tests, the bench's rank spawner and the C4/C5
# rehearsals against the unsharded handle.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_s
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_sharded.py tests/test_bench_ranks.py tests/test_c4_rehearsal.py \
   -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations 15 > $out/pytest_sharded.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
