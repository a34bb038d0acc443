#!/bin/bash
# Round 5, session F: 16-bit dictionary entry ids (and the shuffle owner search again): the parity
# file + wire tests, C3 with 16-bit vs 32-bit ids (A/B), then session E's list: the apply / select
# phase profile on C3, the half/half partition at 16,384 and 32,768 members, C4's schedule at 65,536
# dense, and C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_f
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=variants_ab/libswimhip_cid32.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3_cid32.json 2> $out/bench_c3_cid32.err
rc=$?; echo "c3 cid32 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=variants_ab/libswimhip_prof.so timeout -k 10 300 python -u tools/phase_profile.py c3 20 5 > $out/phase_profile_c3.txt 2>&1
rc=$?; echo "phase rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3half16k --steps 60 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3half16k.json 2> $out/bench_c3half16k.err
rc=$?; echo "half16k rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c4d65 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c4d65.json 2> $out/bench_c4d65.err
rc=$?; echo "c4d65 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c2.json 2> $out/bench_c2.err
rc=$?; echo "c2 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python -u bench.py --workload c3half32k --steps 60 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3half32k.json 2> $out/bench_c3half32k.err
rc=$?; echo "half32k rc=$rc" >> $out/status.log; exit $rc
