#!/bin/bash
# Round 6, session F: C4's schedule at 65,536 and C5's at 131,072 on 8 gloo shards sharing cuda:0 against
# the unsharded handle (tests/test_c4_rehearsal.py), with their wall times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_f
mkdir -p $out
timeout -k 10 560 python -u -m pytest tests/test_c4_rehearsal.py -m gpu -x -v -s -p no:cacheprovider --timeout 540 \
   --timeout-method thread -k "65536" --durations 5 > $out/pytest_c4_65536.log 2>&1
rc=$?; echo "c4 65536 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python -u -m pytest tests/test_c4_rehearsal.py -m gpu -x -v -s -p no:cacheprovider --timeout 540 \
   --timeout-method thread -k "262144" --durations 5 > $out/pytest_c5_262144.log 2>&1
rc=$?; echo "c5 262144 rc=$rc" >> $out/status.log; exit $rc
