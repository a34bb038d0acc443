#!/bin/bash
# Round 5, session M: the commit's tail in one launch (counter weights + dictionary steps,
# k_commit_tail), SYNC merge / ack over 8-member blocks. Parity file + sharded tests; C3, steady65k
# (+ kernel profile), C4's schedule at 65,536, C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_m
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b c3 --steps 20 --warmup 5 && \
b steady65k --workload steady65k --steps 60 --warmup 5 && \
b c4d65 --workload c4d65 --steps 20 --warmup 5 && \
b c2 --workload c2 --steps 20 --warmup 5 && \
b c3_2 --steps 20 --warmup 5 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_steady -o run -- \
    python3 bench.py --workload steady65k --steps 30 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_steady.json 2> $out/prof_steady.err
rc=$?; echo "steady prof rc=$rc" >> $out/status.log; exit $rc
