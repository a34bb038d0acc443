#!/bin/bash
# Round 5, session J: the radix chain in one launch for gossip-round commits (k_rs_fused; the test
# variant fuses every sort), cheaper requester listing. Parity file + sharded tests; C3, steady65k
# (+ the unfused chain as A/B, + a kernel profile), C4's schedule at 65,536, C2; batched-apply A/B
# variants on C3; the phase profile of the half/half partition at 16,384.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_j
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, lib ('' = product), bench args...
  local name=$1 lib=$2; shift 2
  SWIMHIP_LIB=$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --converge 0 > $out/bench_$name.json 2> $out/bench_$name.err
  local rc=$?; echo "$name rc=$rc" >> $out/status.log; return $rc
}
b c3 "" --steps 20 --warmup 5 && \
b steady65k "" --workload steady65k --steps 60 --warmup 5 && \
b steady65k_nofuse variants_ab/libswimhip_nofuse.so --workload steady65k --steps 60 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c2 "" --workload c2 --steps 20 --warmup 5 && \
b c2_nofuse variants_ab/libswimhip_nofuse.so --workload c2 --steps 20 --warmup 5 && \
b c3_along512 variants_ab/libswimhip_along512.so --steps 20 --warmup 5 && \
b c3_along128 variants_ab/libswimhip_along128.so --steps 20 --warmup 5 && \
b c3_aq3 variants_ab/libswimhip_aq3.so --steps 20 --warmup 5 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_steady -o run -- \
    python3 bench.py --workload steady65k --steps 30 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_steady.json 2> $out/prof_steady.err
rc=$?; echo "steady prof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=variants_ab/libswimhip_prof.so timeout -k 10 300 python -u tools/phase_profile.py c3half16k 60 5 > $out/phase_profile_c3half16k.txt 2>&1
rc=$?; echo "phase half16k rc=$rc" >> $out/status.log; exit $rc
