#!/bin/bash
# Round 6, session AH: the final tree after the reverted AF/AG attempt (the certified source of session AB):
# smoke(), the sharded suite, the bench's rank spawner and the C4/C5 rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ah
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_sharded.py tests/test_bench_ranks.py tests/test_c4_rehearsal.py \
   -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations 15 > $out/pytest_sharded.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
