#!/bin/bash
# Round 4, session F (run after J): the final tree's profiles — rocprofv3 kernel stats of the driver's bench command,
# PMC FETCH/WRITE over its timed window (tools/gpu_pmc.sh), PMC over the converge window (merge / sweep),
# and the half/half partition heal at 8,192 members.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_f
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "prof rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh r04_f/pmc
rc=$?; echo "pmc rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
args="--steps 20 --warmup 5 --no-cpu-baseline --converge 120"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/conv/fetch -o run -- \
    python3 bench.py $args > $out/conv_fetch.json 2> $out/conv_fetch.err \
 && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/conv/write -o run -- \
    python3 bench.py $args > $out/conv_write.json 2> $out/conv_write.err \
 && python3 tools/pmc_converge.py $out/conv 20 5 > $out/pmc_converge_c3.json
rc=$?; echo "conv rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c4_alloc_probe.py 8 c5 > $out/c5_alloc.json 2> $out/c5_alloc.err
rc=$?; echo "c5 alloc rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 60 --warmup 5 --workload c3half8k --no-cpu-baseline > $out/bench_c3half8k.json 2> $out/bench_c3half8k.err
rc=$?; echo "half rc=$rc" >> $out/status.log; exit $rc
