#!/bin/bash
# Round 5, session H: the apply / select phase profile on the half/half partition at 16,384
# (-DSWIM_APPLY_PROF -DSWIM_SEL_PROF build), PMC HBM traffic of C3's and C4-schedule (c4d65) bench windows (tools/gpu_pmc.sh: one
# rocprofv3 pass per counter group), batched-apply A/B variants on C3, and the half/half partition at
# 32,768 members.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r05_h
mkdir -p $out
SWIMHIP_LIB=variants_ab/libswimhip_prof.so timeout -k 10 300 python -u tools/phase_profile.py c3half16k 60 5 > $out/phase_profile_c3half16k.txt 2>&1
rc=$?; echo "phase half16k rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_WORKLOAD=c3 tools/gpu_pmc.sh r05_h_pmc_c3
rc=$?; echo "pmc c3 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_WORKLOAD=c4d65 tools/gpu_pmc.sh r05_h_pmc_c4d65
rc=$?; echo "pmc c4d65 rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
for v in along512 along128 aq3; do  # batched apply A/B: range length walked by the whole wave; id loads in flight
  SWIMHIP_LIB=variants_ab/libswimhip_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge 0 \
     > $out/bench_c3_$v.json 2> $out/bench_c3_$v.err
  rc=$?; echo "c3 $v rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 480 python -u bench.py --workload c3half32k --steps 60 --warmup 5 --no-cpu-baseline --converge 0 > $out/bench_c3half32k.json 2> $out/bench_c3half32k.err
rc=$?; echo "half32k rc=$rc" >> $out/status.log; exit $rc
