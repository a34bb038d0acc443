#!/bin/bash
# Round 5, session X: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the C3 bench window the
# driver times, and of C4's schedule at 65,536 (tools/gpu_pmc.sh), on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh r05_x_c3 && PMC_WORKLOAD=c4d65 bash tools/gpu_pmc.sh r05_x_c4d65
