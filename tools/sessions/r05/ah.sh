#!/bin/bash
# Round 5, session AH (certification of the final tree: pruned pairs walked per (pair, chunk)): smoke(), the whole -m gpu suite, the driver's bench command
# (with its CPU baseline and converge tail), and the rocprofv3 kernel-trace summary of that command;
# C2's kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_ah
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "rocprof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
# C2's kernel stats (where its period goes beyond the three bracketed classes)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c2 -o run -- \
    python3 bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_bench_c2.json 2> $out/prof_bench_c2.err
rc=$?; echo "rocprof c2 rc=$rc" >> $out/status.log; exit $rc
