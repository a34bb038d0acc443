#!/bin/bash
# Round 6, session AA (final tree, part 1): rocprofv3 kernel-trace stats of the driver's command (C3) and of
# C2, the apply kernel's timed-window average from that trace, PMC traffic of C3's and C2's driver windows
# (two passes each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_aa
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "rocprof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
python3 tools/rocprof_window.py $out/prof k_gossip_apply_b16 20 5 $out/prof_bench.json > $out/rocprof_apply_timed_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c2 -o run -- \
    python3 bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_bench_c2.json 2> $out/prof_bench_c2.err
rc=$?; echo "rocprof c2 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh r06_aa/pmc_c3
rc=$?; echo "pmc c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c2 bash tools/gpu_pmc.sh r06_aa/pmc_c2
rc=$?; echo "pmc c2 rc=$rc" >> $out/status.log; exit $rc
