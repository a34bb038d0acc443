#!/bin/bash
# Round 5, session O: SYNC merge / ack over striped work lists, the commit-tail fusion reverted
# (session M: 38 us per fused launch), grid-barrier fences once per workgroup. Parity file + sharded;
# C3 twice, steady65k (+ profile), C2, C4's schedule at 65,536 with the lossy pull at 6 (product),
# 5 and 4 waves per SIMD (4: no spills; 4 with four draws in flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_o
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
b c2 "" --workload c2 --steps 20 --warmup 5 && \
b c4d65 "" --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_pl5 variants_ab/libswimhip_pl5.so --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_pl4 variants_ab/libswimhip_pl4.so --workload c4d65 --steps 20 --warmup 5 && \
b c4d65_pl4i4 variants_ab/libswimhip_pl4i4.so --workload c4d65 --steps 20 --warmup 5 && \
b c2_pl4 variants_ab/libswimhip_pl4.so --workload c2 --steps 20 --warmup 5 && \
b c3_2 "" --steps 20 --warmup 5 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_steady -o run -- \
    python3 bench.py --workload steady65k --steps 30 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_steady.json 2> $out/prof_steady.err
rc=$?; echo "steady prof rc=$rc" >> $out/status.log; exit $rc
