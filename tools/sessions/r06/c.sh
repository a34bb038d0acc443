#!/bin/bash
# Round 6, session C: the ring probe (non-power-of-two ring sizing), the whole -m gpu suite on the tree
# without the rejected A/B variants (bench.py's own --gpus 4 launch included), the driver's bench
# command, C2's PMC traffic over the driver-shaped window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r06_c
mkdir -p $out
timeout -k 10 200 python -u tools/probe_ring.py > $out/probe_ring.log 2>&1
rc=$?; echo "probe rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc" >> $out/status.log; [ $rc -eq 0 ] || exit $rc
PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c2 bash tools/gpu_pmc.sh r06_c/pmc_c2
rc=$?; echo "pmc c2 rc=$rc" >> $out/status.log; exit $rc
