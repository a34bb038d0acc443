"""Calibration of FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths of the simulator's kernels
(tools/pmc_calib.hip): per kernel, the counter bytes per dispatch against the bytes it reads / writes
and against its distinct 128-B lines. Prints JSON.  usage: pmc_calib_summary.py <dir with fetch/ write/>"""
import collections
import csv
import glob
import json
import os
import sys

LINES = 1 << 22
USEFUL = {"k_stream16": (2 << 30, 0), "k_gather4": (4 * LINES, 0), "k_gather1": (LINES, 0),
          "k_gather32": (32 * LINES, 0), "k_scatter4": (0, 4 * LINES), "k_rmw4": (4 * LINES, 4 * LINES)}
TOUCHED = {"k_stream16": (2 << 30, 0), "k_gather4": (128 * LINES, 0), "k_gather1": (128 * LINES, 0),
           "k_gather32": (128 * LINES, 0), "k_scatter4": (0, 128 * LINES), "k_rmw4": (128 * LINES, 128 * LINES)}


def load(path, counter):
    v = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                v[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(x) / len(x) for k, x in v.items()}


def main(d):
    fe, wr = load(os.path.join(d, "fetch"), "FETCH_SIZE"), load(os.path.join(d, "write"), "WRITE_SIZE")
    out = {}
    for k in USEFUL:
        f, w = fe.get(k), wr.get(k)
        ur, uw = USEFUL[k]
        lr, lw = TOUCHED[k]
        out[k] = {"fetch_bytes": f, "write_bytes": w,
                  "fetch_per_line": f / (lr / 128) if f is not None and lr else None,
                  "fetch_over_lines_x128": f / lr if f is not None and lr else None,
                  "fetch_over_useful": f / ur if f is not None and ur else None,
                  "write_per_line": w / (lw / 128) if w is not None and lw else None,
                  "write_over_useful": w / uw if w is not None and uw else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
