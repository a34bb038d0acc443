#!/bin/bash
# Round-3 GPU check: a pytest selection (default: the parity suite), then the C3 bench (20/5, no
# CPU baseline). Every GPU step runs under its own time limit; the script stops at the first
# failure. Usage: tools/gpu_r03.sh <tag> [pytest paths...]; OUT=gpurun_out/<tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03}
shift
TESTS=${*:-tests/test_gpu_parity.py}
mkdir -p "$OUT"
timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu ${PYTEST_X--x} -q -p no:cacheprovider --timeout 400 \
  --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo "pytest ok"
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.json" \
  2> "$OUT/bench.err" || { echo "bench rc=$?"; exit 1; }
echo "bench ok"
