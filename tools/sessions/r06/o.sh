#!/bin/bash
# Round 6, session O: C3's schedule at 8,192 members against the oracle (tools/parity_c3_8k.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_o
mkdir -p $out
timeout -k 10 900 python3 -u tools/parity_c3_8k.py > $out/parity_c3_8k.log 2>&1
rc=$?; echo "parity c3 8k rc=$rc" >> $out/status.log; exit $rc
