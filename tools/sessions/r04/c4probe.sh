#!/bin/bash
# C4 storm probe at 16k / 32k / 65k members (1 % loss, 0.1 % crash), one GPU, dense.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
out=gpurun_out/r04_c4probe
mkdir -p $out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
 && timeout -k 10 240 python -u tools/probe_c4_storm.py 16384 19 45 > $out/n16k.log 2>&1 \
 && timeout -k 10 300 python -u tools/probe_c4_storm.py 32768 20 45 > $out/n32k.log 2>&1 \
 && timeout -k 10 400 python -u tools/probe_c4_storm.py 65536 20 45 > $out/n65k.log 2>&1
echo "rc=$?" > $out/status.log
