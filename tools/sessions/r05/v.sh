#!/bin/bash
# Round 5, session V: small shards (at most 16,384 rows) select and apply with a workgroup's 4 waves per
# member (product; the pull already did) against one wave per member (ns); the batched apply's merge
# pass testing 2 / 4 groups of 512 bitmap words before flattening their blocks (mc2, mc4). Parity file
# + sharded through the product; C2, C3, C4's schedule, the half/half partition at 16,384.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_v
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b c2 "" --workload c2 --steps 20 --warmup 5 && \
b c2_ns variants_ab/libswimhip_ns.so --workload c2 --steps 20 --warmup 5 && \
b c3 "" --steps 20 --warmup 5 && \
b c3_mc2 variants_ab/libswimhip_mc2.so --steps 20 --warmup 5 && \
b c3_mc4 variants_ab/libswimhip_mc4.so --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_mc4 variants_ab/libswimhip_mc4.so --workload c4d65 --steps 20 --warmup 5 && \
b c3half16k "" --workload c3half16k --steps 60 --warmup 5 && \
b c3half16k_mc4 variants_ab/libswimhip_mc4.so --workload c3half16k --steps 60 --warmup 5 || exit 1
