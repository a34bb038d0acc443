#!/bin/bash
# Round 4, session D: FETCH/WRITE calibration on known access patterns; C5 as stated (2^20 members,
# N x K K = 256, 256 crashes; 4-bit infection rounds); C4's storm at 131,072 members over 45 periods.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_d
mkdir -p $out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/calib/fetch -o run -- ./tools/pmc_calib \
   > $out/calib_fetch.log 2>&1 \
 && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/calib/write -o run -- ./tools/pmc_calib \
   > $out/calib_write.log 2>&1 \
 && python3 tools/pmc_calib_summary.py $out/calib > $out/pmc_calibration.json
echo "calib rc=$?" >> $out/status.log
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 --workload c5 > $out/bench_c5.json 2> $out/bench_c5.err
echo "c5 rc=$?" >> $out/status.log
timeout -k 10 300 python -u tools/probe_c4_storm.py 131072 20 45 5 24576 > $out/n131k_nxk.log 2>&1
echo "probe rc=$?" >> $out/status.log
