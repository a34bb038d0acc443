#!/bin/bash
# Round 5, session R: the infectedFrom kernels at 256 positions per wave, the LDS bitonic commit sort
# with wave-level barriers. Parity file + sharded; C2, C3, C4's schedule at 65,536, the half/half
# partition at 16,384 (with four id loads in flight per lane as A/B: av4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_r
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
b c3 "" --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c3half16k "" --workload c3half16k --steps 60 --warmup 5 && \
b c3half16k_av4 variants_ab/libswimhip_av4.so --workload c3half16k --steps 60 --warmup 5 && \
b c3_av4 variants_ab/libswimhip_av4.so --steps 20 --warmup 5 || exit 1
