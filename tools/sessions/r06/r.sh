#!/bin/bash
# Round 6, session R: C5's schedule at 262,144 members on 8 gloo shards against the unsharded handle
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_r
mkdir -p $out
timeout -k 10 1000 python3 -u tools/rehearse_c5_262k.py > $out/rehearse_c5_262k.log 2>&1
rc=$?; echo "c5 262k rc=$rc" >> $out/status.log; exit $rc
