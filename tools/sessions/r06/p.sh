#!/bin/bash
# Round 6, session P: C3's schedule at 16,384 members against the oracle (one-off; ~90 GB of oracle state)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_p
mkdir -p $out
timeout -k 10 1000 python3 -u tools/parity_c3_8k.py 16384 > $out/parity_c3_16k.log 2>&1
rc=$?; echo "parity c3 16k rc=$rc" >> $out/status.log; exit $rc
