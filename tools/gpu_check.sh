#!/bin/bash
# Run smoke + GPU tests on the gpurun box. Stops at the first fault-like exit status
# (anything other than 0 = pass or 1 = assertion failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log
ok $rc || exit $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log
exit $rc
