#!/bin/bash
# Round 6, session E: SQ stall counters of C3's driver window (which kernels wait on memory), C2 on the
# driver's command shape with its PMC traffic (two passes), the half/half partition at 65,536 (c3half65k).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_e
mkdir -p $out
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM \
    --output-format csv -d $out/sq -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
    > $out/sq_bench.json 2> $out/sq_bench.err
rc=$?; echo "sq rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
python3 tools/sq_summary.py $out/sq 20 5 > $out/sq_c3_s20_w5.json
timeout -k 10 300 python3 -u bench.py --workload c2 --steps 20 --warmup 5 > $out/bench_c2.json 2> $out/bench_c2.err
rc=$?; echo "c2 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c2 bash tools/gpu_pmc.sh r06_e/pmc_c2
rc=$?; echo "pmc c2 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c3half65k --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
   > $out/bench_c3half65k.json 2> $out/bench_c3half65k.err
rc=$?; echo "c3half65k rc=$rc" >> $out/status.log; exit $rc
