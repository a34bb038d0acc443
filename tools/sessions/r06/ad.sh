#!/bin/bash
# Round 6, session AD: the unattached-shard refusals (tests/test_sharded.py::test_unattached_shard_fails_loudly)
# and the host-driven protocol.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ad
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_sharded.py -m gpu -k "unattached or host_driven" -x -v -p no:cacheprovider \
   --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; exit $rc
