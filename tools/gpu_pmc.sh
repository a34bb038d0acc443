#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters over exactly the bench window the
# driver times (bench.py --steps S --warmup W): one pass per counter group (FETCH_SIZE uses 3 TCC
# slots, WRITE_SIZE 2: never in one pass), kernel-trace only, no tracing domains.
#   usage: PMC_STEPS=20 PMC_WARMUP=5 PMC_WORKLOAD=c3 tools/gpu_pmc.sh <tag>
# writes gpurun_out/<tag>/pmc_traffic_<workload>_s<S>_w<W>.json, the file bench.py reads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-pmc}
S=${PMC_STEPS:-20}; W=${PMC_WARMUP:-5}; WL=${PMC_WORKLOAD:-c3}
out=gpurun_out/$tag
mkdir -p $out
args="--steps $S --warmup $W --workload $WL --no-cpu-baseline --converge 0"
echo "start $(date +%T)" > $out/status.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
    python3 bench.py $args > $out/fetch_bench.json 2> $out/fetch_bench.err \
  && echo "fetch ok $(date +%T)" >> $out/status.log \
  && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
    python3 bench.py $args > $out/write_bench.json 2> $out/write_bench.err \
  && echo "write ok $(date +%T)" >> $out/status.log \
  && python3 tools/pmc_summary.py $out "$WL" "$S" "$W" > $out/pmc_traffic_${WL}_s${S}_w${W}.json \
  && echo "summary ok $(date +%T)" >> $out/status.log
rc=$?
echo "rc=$rc $(date +%T)" >> $out/status.log
exit $rc
