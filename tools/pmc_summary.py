"""Per-kernel average HBM traffic per dispatch of the bench's TIMED window from the FETCH_SIZE /
WRITE_SIZE passes of tools/gpu_pmc.sh (rocprofv3 counter_collection CSVs, values in KiB).

The profiled command is `bench.py --steps S --warmup W --converge 0`: the timed periods are the run's
last. A per-period kernel is dispatched (W + S) x (launches per period) times, so its window is the last
S / (W + S) of its dispatches (by Dispatch_Id); a gossip-round kernel is dispatched G times per busy
period and not at all in the quiet fault-free warm-up, so its window is its last S x G
dispatches. Averages are over those only, which is what bench.py's HIP-event averages cover. Prints JSON:
{"window": {...}, kernel: {"fetch_bytes", "write_bytes", "fetch_bytes_x2", "dispatches"}}.
MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads
(hence the x2 column); other access widths are uncalibrated, so both are reported."""
import collections
import csv
import glob
import json
import os
import sys


def load(path, counter, steps, warmup, rounds):
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("swim::", "")
            rows[name].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    out = {}
    for name, v in rows.items():
        v.sort()
        # the timed periods are the run's last (--converge 0). A gossip-round kernel is dispatched G times
        # per busy period and not at all in a quiet one (the fault-free warm-up): its last
        # S x G dispatches; a per-period kernel its last S / (S + W) share
        if name.startswith("k_gossip_"):
            n = min(len(v), steps * rounds)
        else:
            n = max(1, round(len(v) * steps / (steps + warmup)))
        tail = v[len(v) - n:]
        out[name] = (sum(x for _, x in tail) / len(tail) * 1024.0, len(tail))
    return out


def main(out, workload=None, steps=None, warmup=None, rounds=None):
    s, w = int(steps or 1), int(warmup or 0)
    g = int(rounds or 5)
    fe = load(os.path.join(out, "fetch"), "FETCH_SIZE", s, w, g)
    wr = load(os.path.join(out, "write"), "WRITE_SIZE", s, w, g)
    res = {"window": {"workload": workload, "steps": s, "warmup": w,
                      "command": f"bench.py --steps {s} --warmup {w} --workload {workload}",
                      "dispatches": f"the timed periods: the last {s} x {g} dispatches of a gossip-round kernel, "
                                    f"the last {s}/{s + w} of a per-period kernel's (--converge 0)"}}
    for k in sorted(set(fe) | set(wr)):
        f = fe.get(k, (0.0, 0))[0]
        res[k] = {"fetch_bytes": f, "write_bytes": wr.get(k, (0.0, 0))[0], "fetch_bytes_x2": 2 * f,
                  "dispatches": fe.get(k, (0.0, 0))[1]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
