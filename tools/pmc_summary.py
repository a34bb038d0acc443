"""Per-kernel average HBM traffic per dispatch from the FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_pmc.sh (rocprofv3 counter_collection CSVs, values in KiB). Prints JSON:
{kernel: {"fetch_bytes": ..., "write_bytes": ..., "fetch_bytes_x2": ..., "dispatches": n}}.
MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads
(hence the x2 column); other access widths are uncalibrated, so both are reported."""
import collections
import csv
import glob
import json
import os
import sys


def load(path, counter):
    acc = collections.defaultdict(lambda: [0.0, 0])
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("swim::", "")
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1] += 1
    return acc


def main(out):
    fe, wr = load(os.path.join(out, "fetch"), "FETCH_SIZE"), load(os.path.join(out, "write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f = fe[k][0] / max(1, fe[k][1]) * 1024.0
        w = wr[k][0] / max(1, wr[k][1]) * 1024.0
        res[k] = {"fetch_bytes": f, "write_bytes": w, "fetch_bytes_x2": 2 * f, "dispatches": fe[k][1]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
