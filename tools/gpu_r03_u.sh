#!/bin/bash
# Round-3 final tree (also after the DPP wave scans): the whole -m gpu suite, the C3 20/5 bench line with its CPU baseline, the
# rocprofv3 kernel stats of the same window, and the FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r03u}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/c3.json 2> $out/c3.err \
  && echo "c3 ok" >> $out/status.log \
  && bash tools/profile.sh ${1:-r03u}_c3 --steps 20 --warmup 5 \
  && echo "c3 prof ok" >> $out/status.log \
  && PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 bash tools/gpu_pmc.sh ${1:-r03u}/pmc \
  && echo "pmc ok" >> $out/status.log
rc=$?
echo "rc=$rc" >> $out/status.log
exit $rc
