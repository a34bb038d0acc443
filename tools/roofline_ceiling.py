"""Roofline ceiling of a bench run: the HBM-time floor of its timed window.

Each bench line carries, per kernel class, the time over the timed window (`kernels_ms`) and the
fraction of the 8 TB/s peak its algorithmic bytes reach (`kernels_frac` = bytes / time / peak). So
the algorithmic bytes of the window are sum(frac x peak x time); moving them at peak takes
bytes / peak seconds, and N x K member-periods in that time is the ceiling every kernel at 100 % of
HBM peak would reach (60 %: the target's bar). Host-side bookkeeping kernels carry no byte model
and are left out (they are < 3 % of a period).

python tools/roofline_ceiling.py BENCH_JSON [BENCH_JSON ...]   (last JSON line of each file)"""
import json
import sys

PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(f"{path}: no JSON line")


def ceiling(d):
    wall_s = d["ms_per_step"] * d["steps"] / 1e3
    gbytes = sum(d["kernels_frac"][k] * PEAK * d["kernels_ms"][k] / 1e3 for k in d["kernels_frac"])
    floor_s = gbytes / PEAK
    units = d["value"] * wall_s  # member-periods of the window (all ranks)
    return {"workload": d["config"].get("workload", "")[:60], "member_periods": units,
            "algorithmic_GB": round(gbytes, 1), "wall_ms_per_period": round(d["ms_per_step"], 2),
            "floor_ms_per_period": round(1e3 * floor_s / d["steps"], 3),
            "measured": d["value"], "ceiling_100pct": units / floor_s, "ceiling_60pct": 0.6 * units / floor_s,
            "frac_of_ceiling": round(floor_s / wall_s, 4)}


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps({"file": p, **ceiling(last_json(p))}))
