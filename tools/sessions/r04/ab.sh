#!/bin/bash
# Round 4, session AB: phase profiles of the batched apply and of select on C3's 20/5 window
# (a -DSWIM_APPLY_PROF -DSWIM_SEL_PROF build; tools/phase_profile.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_ab
mkdir -p $out
SWIMHIP_LIB=$PWD/variants_ab/libswimhip_prof.so timeout -k 10 300 python -u tools/phase_profile.py c3 20 5 > $out/phase_c3.txt 2>&1
rc=$?; echo "c3 rc=$rc" >> $out/status.log; exit $rc
