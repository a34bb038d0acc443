#!/bin/bash
# Round 6, session AI: the multi-process GPU tests with one hardware queue per rank (GPU_MAX_HW_QUEUES=1 in
# the workers: 8 shards plus the unsharded handle on one GPU), progress lines written as they come (-s).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ai
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests/test_c4_rehearsal.py tests/test_sharded.py -m gpu -x -v -s -p no:cacheprovider \
   --timeout 400 --timeout-method thread --durations 20 > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
