#!/bin/bash
# Round 4, session V (final tree): rocprofv3 kernel stats of the driver's bench command, PMC FETCH /
# WRITE over its timed window, the driver's command itself (CPU baseline included), and the half/half
# partition heal at 16,384 members.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_v
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "prof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh r04_v/pmc
rc=$?; echo "pmc rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --workload c3half16k --no-cpu-baseline > $out/bench_c3half16k.json 2> $out/bench_c3half16k.err
rc=$?; echo "half16k rc=$rc" >> $out/status.log; exit $rc
