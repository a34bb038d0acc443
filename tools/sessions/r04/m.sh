#!/bin/bash
# Round 4, session M: C4's schedule on the final tree — 65,536 dense with 8-bit and with 4-bit
# infection rounds (what the 8-GPU shards use); the driver's own command (C3, CPU baseline included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_m
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload c4d65 --no-cpu-baseline > $out/bench_c4d65.json 2> $out/bench_c4d65.err
rc=$?; echo "c4d65 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workload c4d65 --no-cpu-baseline --infection-round-bits 4 \
   > $out/bench_c4d65_hd4.json 2> $out/bench_c4d65_hd4.err
rc=$?; echo "c4d65 hd4 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $out/status.log; exit $rc
