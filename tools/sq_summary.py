"""Per-kernel SQ stall counters over the bench's timed window (the last S / (S + W) of each kernel's
dispatches, as tools/pmc_summary.py): wave cycles split into parked on a wait (SQ_WAIT_ANY: s_waitcnt on
memory or LDS, barriers), issue stalls (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), plus the
LDS and vector-memory instructions per dispatch. usage: sq_summary.py <dir> <steps> <warmup>"""
import collections
import csv
import glob
import json
import os
import sys


def main(path, steps, warmup):
    keep = int(steps) / (int(steps) + int(warmup))
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("swim::", "")
            rows[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in rows.items():
        d = {}
        for c, v in cs.items():
            v.sort()
            tail = v[len(v) - max(1, round(len(v) * keep)):]
            d[c] = sum(x for _, x in tail) / len(tail)
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c + "_frac"] = d[c] / wc
        out[k] = d
    top = sorted(out, key=lambda k: -out[k].get("SQ_WAVE_CYCLES", 0.0))[:16]
    print(json.dumps({k: out[k] for k in top}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
