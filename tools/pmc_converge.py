"""HBM traffic of the merge / sweep kernels over bench.py's CONVERGE window, from the FETCH_SIZE /
WRITE_SIZE passes of `bench.py --steps S --warmup W --converge C` (tools/gpu_pmc.sh with
PMC_CONVERGE=C). These kernels run once per period, so a kernel's i-th dispatch is period i:
k_sync_merge / k_sync_ack are averaged over the periods after the timed window (W + S onwards, the
window of bench.py's converge_kernels_frac); k_susp_sweep over the periods whose suspicion deadlines
fired (the window of bench.py's sweep_roofline: the dispatches that moved more than 1 MiB).
FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950 note for 16-B streaming reads (the merges);
the sweep's widths are reported both ways. usage:
pmc_converge.py <dir> S W"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("k_sync_merge", "k_sync_ack", "k_susp_sweep")


def load(path, counter):
    v = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("swim::", "")
            if name in KERNELS:
                v[name].append((int(row["Dispatch_Id"]), float(row["Counter_Value"]) * 1024.0))
    return {k: [x for _, x in sorted(xs)] for k, xs in v.items()}


def main(d, steps, warmup):
    s, w = int(steps), int(warmup)
    fe, wr = load(os.path.join(d, "fetch"), "FETCH_SIZE"), load(os.path.join(d, "write"), "WRITE_SIZE")
    out = {"window": {"converge_from_period": s + w, "sweep": "dispatches that moved > 1 MiB"}}
    for k in KERNELS:
        f, wv = fe.get(k, []), wr.get(k, [])
        n = min(len(f), len(wv))
        if k == "k_susp_sweep":
            idx = [i for i in range(n) if f[i] + wv[i] > (1 << 20)]
        else:
            idx = list(range(s + w, n))
        if not idx:
            continue
        fa = sum(f[i] for i in idx) / len(idx)
        wa = sum(wv[i] for i in idx) / len(idx)
        out[k] = {"dispatches": len(idx), "fetch_bytes": fa, "fetch_bytes_x2": 2 * fa, "write_bytes": wa,
                  "traffic_x2": 2 * fa + wa, "traffic_x1": fa + wa}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
