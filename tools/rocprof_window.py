"""Average duration of one kernel over the bench's timed window, from a rocprofv3 --kernel-trace CSV.

The bench's warmup periods are fault-free, so the library skips their gossip rounds as quiet (DESIGN.md
§5): a round kernel's first dispatches are the timed window's (the crash comes at its start). The window
is taken as the first `steps x rounds` dispatches of the kernel and checked against the bench's own
launch count (HIP events). usage: rocprof_window.py <trace dir> <kernel> <steps> <rounds per period>
<bench json of the same run>"""
import csv
import glob
import json
import os
import sys


def main(path, kernel, steps, rounds, bench_json):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].split("(")[0].replace("swim::", "") == kernel:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    n = int(steps) * int(rounds)
    win = rows[:n]
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    rl = bench["roofline"]
    out = {"kernel": kernel, "dispatches_total": len(rows), "timed_window_dispatches": f"first {len(win)}",
           "timed_window_avg_ms": sum(e - s for s, e in win) / max(1, len(win)) / 1e6,
           "bench_kernel": rl.get("kernel"), "bench_launches": rl.get("launches"),
           "bench_hip_event_avg_ms_same_run": rl.get("avg_launch_ms")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
