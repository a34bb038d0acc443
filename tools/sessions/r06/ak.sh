#!/bin/bash
# Round 6, session AK: the NEED and SYNC_ACK exchanges without status all-gathers again (each rank's SYNC
# capacity in its row; the host-staged receive vector grown only after the stream is synchronized), with the
# multi-rank tests on one hardware queue per rank: the one-rank RCCL period, the sharded suite, the bench's
# rank spawner and the C4/C5 rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ak
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_c4_rehearsal.py tests/test_sharded.py tests/test_bench_ranks.py -m gpu -x -v -s \
   -p no:cacheprovider --timeout 400 --timeout-method thread --durations 12 > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/exchange_overhead.py c3 20 5 2 > $out/overhead_new.log 2>&1
rc=$?; echo "overhead new rc=$rc" >> $out/status.log; exit $rc
