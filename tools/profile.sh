#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run (no PMC counters in this pass).
# usage: tools/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --no-cpu-baseline --converge 0 "$@" > gpurun_out/prof_$tag/bench.json 2> gpurun_out/prof_$tag/bench.err
rc=$?
find gpurun_out/prof_$tag -name "*stats*" | head
exit $rc
