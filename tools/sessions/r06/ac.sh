#!/bin/bash
# Round 6, session AC: the library-driven exchanges' cost on the final tree - C3 on a one-rank RCCL
# communicator against the unsharded handle, three interleaved repeats each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_ac
mkdir -p $out
timeout -k 10 700 python3 -u tools/exchange_overhead.py c3 20 5 3 > $out/overhead.log 2>&1
rc=$?; echo "overhead rc=$rc" >> $out/status.log; exit $rc
