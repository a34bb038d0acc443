#!/bin/bash
# Round-3: C4's storm on one GPU (N x K, 262,144 members, 1 % loss) with a 2^19-slot ring, the final
# C3 20/5 kernel stats, the select slot-count A/B, and the C3 PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r03k}
mkdir -p $out
timeout -k 10 240 python -u tools/probe_storm.py c4nxk 19 12 > $out/probe_c4nxk.log 2>&1
rc=$?; echo "c4nxk rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
bash tools/profile.sh r03k_c3 --steps 20 --warmup 5
rc=$?; echo "prof rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
OCC_VARIANTS="nosg mp3 mp4 product" bash tools/gpu_r03_occ.sh ${1:-r03k}/ab
rc=$?; echo "ab rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh ${1:-r03k}/pmc
rc=$?; echo "pmc rc=$rc" >> $out/status.log
exit $rc
