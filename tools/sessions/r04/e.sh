#!/bin/bash
# Round 4, session E: -m gpu suite, then (tools/gpu_r04_d.sh) calibration, C5 as stated, C4 storm at 131k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_e
mkdir -p $out
timeout -k 10 660 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/status.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r04_d.sh
