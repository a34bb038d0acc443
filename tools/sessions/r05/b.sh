#!/bin/bash
# Round 5, session B: merge marks, u16 deadlines, the spill table (no dense inbox), per-subject spill
# fallback, runtime dictionary size, non-power-of-two rings, memory-sized delay rings, the bridge's
# forwarded gossips, library-driven shard exchanges (RCCL / host transports): the parity file + wire
# tests, the driver's C3 window (no CPU baseline), the sharded tests and the memory plans.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_b
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_sharded.py tests/test_memory_plan.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_c4_rehearsal.py -m gpu -x -v -s -p no:cacheprovider --timeout 540 --timeout-method thread \
   > $out/pytest_c4_rehearsal.log 2>&1
rc=$?; echo "c4 rehearsal rc=$rc" >> $out/status.log; exit $rc
