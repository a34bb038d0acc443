#!/bin/bash
# Full GPU session: smoke + GPU tests + bench + kernel stats, then the PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}
bash tools/gpu_round.sh $tag && bash tools/gpu_pmc.sh $tag/pmc
