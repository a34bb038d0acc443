#!/bin/bash
# Round 5, session S: the pull split over a workgroup's 4 waves for shards of at most 16,384 rows
# (product), A/B against no split (ps0) and a split up to 65,536 rows (ps65k); 32-bit-id apply at 4
# loads in flight. Parity file + sharded; C2, C3, C4's schedule, the half/half partition at 16,384;
# the C3 phase profile of apply and select.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_s
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
b c2_ps0 variants_ab/libswimhip_ps0.so --workload c2 --steps 20 --warmup 5 && \
b c3 "" --steps 20 --warmup 5 && \
b c3_ps65k variants_ab/libswimhip_ps65k.so --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_ps65k variants_ab/libswimhip_ps65k.so --workload c4d65 --steps 20 --warmup 5 && \
b c3half16k "" --workload c3half16k --steps 60 --warmup 5 || exit 1
SWIMHIP_LIB=variants_ab/libswimhip_prof.so timeout -k 10 300 python -u tools/phase_profile.py c3 20 5 > $out/phase_profile_c3.txt 2>&1
echo "prof rc=$?" >> $out/status.log
