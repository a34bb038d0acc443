#!/bin/bash
# Round 5, session D2 (after the sharded tests passed in D): the sharded tests through the library-driven exchanges (gloo transports, the
# one-rank library RCCL path, sharded 4-bit rounds), the memory plans of C4 / C5's node shards, C4's
# schedule at 32,768 members on 8 gloo shards, and the owner-search A/B on C3 plus a C2 kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_d2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_memory_plan.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
SWIMHIP_LIB=variants_ab/libswimhip_owner_shfl.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3_owner_shfl.json 2> $out/bench_c3_owner_shfl.err
rc=$?; echo "c3 shfl rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c2 -o run -- \
    python3 bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_c2.json 2> $out/prof_c2.err
rc=$?; echo "c2 prof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_steady -o run -- \
    python3 bench.py --workload steady65k --steps 30 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_steady.json 2> $out/prof_steady.err
rc=$?; echo "steady prof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_c4_rehearsal.py -m gpu -x -v -s -p no:cacheprovider --timeout 540 --timeout-method thread \
   > $out/pytest_c4_rehearsal.log 2>&1
rc=$?; echo "c4 rehearsal rc=$rc" >> $out/status.log; exit $rc
