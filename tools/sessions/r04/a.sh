#!/bin/bash
# Round 4, session A: -m gpu suite on the tree, then the C4 storm at 131,072 (N x K, largest one GPU holds)
# and the C4 shard allocation at the 2^21-slot ring the storm measurements call for.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_a
mkdir -p $out
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
   > $out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $out/status.log
timeout -k 10 120 python -u tools/c4_alloc_probe.py 8 > $out/c4_alloc.json 2> $out/c4_alloc.err
echo "alloc rc=$?" >> $out/status.log
timeout -k 10 250 python -u tools/probe_c4_storm.py 131072 20 45 5 24576 > $out/n131k_nxk.log 2>&1
echo "probe rc=$?" >> $out/status.log
