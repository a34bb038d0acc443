#!/bin/bash
# One SQ-counter pass (stall breakdown) over a short bench run; per-kernel sums in sq.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-sq}
mkdir -p $out
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM \
    --output-format csv -d $out/sq -o run -- python3 bench.py --steps 20 --no-cpu-baseline --converge 0 \
    > $out/bench.json 2> $out/bench.err \
  && python3 - $out <<'PY'
import collections, csv, glob, json, os, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(sys.argv[1], "sq", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("swim::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
json.dump({k: dict(v) for k, v in acc.items() if k.startswith("k_gossip")}, open(os.path.join(sys.argv[1], "sq.json"), "w"), indent=1)
PY
