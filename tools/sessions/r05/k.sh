#!/bin/bash
# Round 5, session K: PMC HBM traffic of C3's and C4-schedule (c4d65) bench windows (tools/gpu_pmc.sh:
# one rocprofv3 pass per counter group, kernel-trace only), and the half/half partition at 32,768.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_k
mkdir -p $out
PMC_WORKLOAD=c3 tools/gpu_pmc.sh r05_k_pmc_c3
rc=$?; echo "pmc c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_WORKLOAD=c4d65 tools/gpu_pmc.sh r05_k_pmc_c4d65
rc=$?; echo "pmc c4d65 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python -u bench.py --workload c3half32k --steps 60 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3half32k.json 2> $out/bench_c3half32k.err
rc=$?; echo "half32k rc=$rc" >> $out/status.log; exit $rc
