#!/usr/bin/env python
"""bench.py — whole-node member-periods/s of the SWIM protocol-period step on MI355X.

Metric (BASELINE.json): member-periods/sec at 65k/262k members; periods to DEAD convergence.
A "step" is one protocol period for every simulated member: FD probe, G gossip
rounds, suspicion timeouts, SYNC/SYNC_ACK. Inputs are synthetic (a converged cluster, a
Philox-chosen crash set) and resident in HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3s]

N > 1 runs one rank per GPU under torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE from the env;
`--gpus N` from a plain `python bench.py` starts those N ranks itself as children and touches no GPU;
a WORLD_SIZE that differs from --gpus is refused): the workload's ONE cluster is split into observer-row shards, one per GPU, exchanging
gossip windows, gossip ids and SYNC tables over RCCL each round (strong scaling);
barrier + max-over-ranks timing, value = the cluster's member-periods / time.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# name -> workload spec. The default ("c3") is BASELINE.json configs[2], the 65,536-member config
# the metric is quoted on that fits one GPU: a 10 % simultaneous crash plus a 2-way partition from
# t0 to t0+40 periods (< the 85-period suspicion timeout, so it heals by refutation and SYNC), LAN
# defaults, no loss; t0 = the end of the warmup. The partition cuts a 16-member group (ids that are
# multiples of N/16) from the rest. SURVEY §8(d)'s half/half cut by id parity is the workload
# c3half65k: on heal every SYNC/SYNC_ACK re-spreads each accepted SUSPECT record as a new gossip
# (MembershipProtocolImpl.java:649-656), ~0.47 N^2 gossips over the heal (oracle: 25.7k / 112k / 491k at
# N = 256 / 512 / 1,024); it runs on one MI355X at 236 ms per period of the driver's window (180.6 GiB,
# 1.1e7 gossips live at its end), 17x the 16-member cut's period.
WORKLOADS = {
    "c3": dict(desc="C3: 65,536 members, dense N x N views, LAN defaults, 10% simultaneous crash + 2-way "
                    "partition (16-member group) for 40 periods healed via SYNC",
               n=65536, preset="lan", loss=0.0, crash=0.10, part=40, part_group=16, gcap=1 << 17, scap=8192),
    # SURVEY §8(d) C3 variant: the partition outlasts the 85-period suspicion timeout, so both
    # sides remove each other; the cut group rejoins through the seed addresses (ids 0..15) after
    # the heal (MembershipProtocolTest.testLongNetworkPartitionNoOutboundThenRemoved, :844-918)
    "c3long": dict(desc="C3 variant: 65,536 members, LAN defaults, seeds 0..15, 10% simultaneous crash + a "
                        "16-member group partitioned for 120 periods (past the suspicion timeout), rejoining "
                        "through the seeds",
                   n=65536, preset="lan", loss=0.0, crash=0.10, part=120, part_group=16, gcap=1 << 18,
                   scap=8192, seeds=16),
    # C3 on the column-allocated layout (N x K views with K = N: a subject gets a column when some row
    # first changes its record, so the touched columns are the first ones of every row and SYNC
    # payloads stream them)
    "c3k": dict(desc="C3 on column-allocated views (K = N): 65,536 members, LAN defaults, 10% simultaneous crash + "
                     "2-way partition (16-member group) for 40 periods healed via SYNC",
                n=65536, preset="lan", loss=0.0, crash=0.10, part=40, part_group=16, gcap=1 << 17, scap=8192,
                tracked=65536),
    "c3s": dict(desc="C3 geometry: 65,536 members, dense N x N views, LAN defaults, 0.1% simultaneous crash",
                n=65536, preset="lan", loss=0.0, crash=0.001, part=0, gcap=1 << 16),
    "c3crash": dict(desc="65,536 members, dense, LAN defaults, 10% simultaneous crash, no partition",
                    n=65536, preset="lan", loss=0.0, crash=0.10, part=0, gcap=1 << 17, scap=8192),
    "c2": dict(desc="C2: 4,096 members, dense N x N views, LAN defaults, 5% uniform loss, 1% crash",
               n=4096, preset="lan", loss=5.0, crash=0.01, part=0, gcap=1 << 18),
    # BASELINE configs[4] as stated: the 8-GPU node's (its SYNC re-spread storm
    # outgrows the 2^18-slot ring one GPU can hold for 2^20 members; ~4e5 live batch slots by the
    # storm's measured growth). Per GPU at 2^17 rows: 2^20 slots of 4-bit infection rounds (auto),
    # holdings, windows, receipts and age bounds = 120 GiB
    "c5": dict(desc="C5: 1,048,576 members, N x K tracked-subject views (K = 256), LAN defaults, 256 simultaneous "
                    "crashes (concurrent churn), suspicion-timeout sweep",
               n=1 << 20, preset="lan", loss=0.0, crash_n=256, part=0, gcap=1 << 20, tracked=256,
               rcap=1 << 24),
    # C5's full size with the churn one GPU holds at that size (tests/test_gpu_fullsize.py)
    "c5g": dict(desc="C5 geometry at 1,048,576 members: N x K tracked-subject views (K = 256), LAN defaults, 8 "
                     "simultaneous crashes, suspicion-timeout sweep",
                n=1 << 20, preset="lan", loss=0.0, crash_n=8, part=0, gcap=1 << 17, tracked=256),
    "c5s": dict(desc="C5 geometry at 262,144 members: N x K tracked-subject views (K = 256), LAN defaults, 256 "
                     "simultaneous crashes",
                n=1 << 18, preset="lan", loss=0.0, crash_n=256, part=0, gcap=1 << 18, tracked=256),
    # BASELINE configs[3]: needs >= 8 GPUs (dense 256 GiB of views); one rank's shard is 32,768 rows.
    # Ring: 5,128 * 1,024 = 5,251,072 slots (a non-power-of-two ring, ids mod GC), 1.25x the ~4.2e6 live one-gossip slots
    # C4's storm law predicts
    "c4": dict(desc="C4: 262,144 members, dense N x N views row-sharded over the GPUs, LAN defaults, 1% loss, "
                    "0.1% simultaneous crash",
               n=1 << 18, preset="lan", loss=1.0, crash=0.001, part=0, gcap=5128 * 1024, scap=4096),
    # C4's schedule on ONE GPU in N x K mode (the dense 262,144^2 view needs 8 GPUs): measures the
    # storm C4's 1 % loss and 0.1 % crash create, to size C4's ring (1 % loss: one gossip per slot)
    "c4nxk": dict(desc="C4 schedule on one GPU: 262,144 members, N x K views (K = 1,024), LAN defaults, 1% loss, "
                       "0.1% simultaneous crash",
                  n=1 << 18, preset="lan", loss=1.0, crash=0.001, part=0, gcap=1 << 18, tracked=1024),
    # C4's schedule on one GPU at the largest sizes one MI355X holds (the 1 % loss storm
    # keeps 1.04e6 one-gossip slots live at 131,072 members, ~4x per doubling: ~4.2e6 at 262,144, the
    # 2^22-slot ring of the 8-GPU node's shards, with 4-bit infection rounds)
    "c4d65": dict(desc="C4 schedule on one GPU at 65,536 members: dense N x N views, LAN defaults, 1% loss, "
                       "0.1% simultaneous crash",
                  n=65536, preset="lan", loss=1.0, crash=0.001, part=0, gcap=1 << 20),
    "c4s": dict(desc="C4 schedule on one GPU at 131,072 members: N x K views (K = 24,576), LAN defaults, 1% loss, "
                     "0.1% simultaneous crash",
                n=1 << 17, preset="lan", loss=1.0, crash=0.001, part=0, gcap=1 << 20, tracked=24576),
    # SURVEY §8(d)'s C3 partition as written (half/half by id parity, healed by SYNC) at the largest
    # sizes one GPU holds: on heal every SYNC re-spreads each accepted SUSPECT record (~0.47 N^2
    # gossips), held as batches of one origin's records per commit
    "c3half8k": dict(desc="C3 schedule with the half/half partition at 8,192 members: dense, LAN defaults, 10% "
                          "simultaneous crash + id-parity partition for 40 periods healed via SYNC",
                     n=8192, preset="lan", loss=0.0, crash=0.10, part=40, part_group=4096, gcap=1 << 17,
                     rcap=1 << 26),
    "c3half16k": dict(desc="C3 schedule with the half/half partition at 16,384 members: dense, LAN defaults, 10% "
                           "simultaneous crash + id-parity partition for 40 periods healed via SYNC",
                      n=16384, preset="lan", loss=0.0, crash=0.10, part=40, part_group=8192, gcap=1 << 18,
                      rcap=1 << 27, dsub=16384),
    "c3half32k": dict(desc="C3 schedule with the half/half partition at 32,768 members: dense, LAN defaults, 10% "
                           "simultaneous crash + id-parity partition for 40 periods healed via SYNC",
                      n=32768, preset="lan", loss=0.0, crash=0.10, part=40, part_group=16384, gcap=1 << 18,
                      rcap=1 << 29, dsub=32768),
    # ... and at the C3 size itself: 2^30 record slots (the storm's records, batched per origin commit),
    # a 65,536-block dictionary (64 KiB of entry bitmap per receiver: 2 receivers per workgroup)
    "c3half65k": dict(desc="C3 as SURVEY states it: 65,536 members, dense, LAN defaults, 10% simultaneous crash + "
                           "id-parity (half/half) partition for 40 periods healed via SYNC",
                      n=65536, preset="lan", loss=0.0, crash=0.10, part=40, part_group=32768, gcap=1 << 18,
                      rcap=1 << 30, dsub=65536),
    "steady65k": dict(desc="65,536 members, dense, LAN defaults, fault-free steady state",
                      n=65536, preset="lan", loss=0.0, crash=0.0, part=0, gcap=1 << 14),
}


def partition_groups(n, group_size):
    """Group 1 = `group_size` members spread evenly over the id space (ids k * n // group_size);
    group_size = n // 2: the 2-way half/half cut by id parity (SURVEY §8(d) C3 as written)."""
    if 2 * group_size == n:
        return (np.arange(n) % 2).astype(np.uint8)
    g = np.zeros(n, dtype=np.uint8)
    g[(np.arange(group_size, dtype=np.int64) * n) // group_size] = 1
    return g


def kernel_bytes(name, d, rounds_per_period=5):
    """Algorithmic HBM bytes of one kernel class over the timed region.
    d = stats deltas over the timed region; rounds_per_period = G (gossip rounds per period)."""
    if name == "k_sync_merge":  # read SYNC payload row + read table row + write SYNC_ACK payload
        return 12 * d["merge_cells"]
    if name == "k_sync_ack":  # read SYNC_ACK payload row + read table row
        return 8 * d["ack_cells"]
    if name == "k_sync_snapshot":  # copy the sender's row into the SYNC payload
        return 8 * d["merge_cells"]
    if name == "k_gossip_select":  # holds word per active word, 64 B of infection rounds per MIXED word,
        return 4 * d["gossip_scanned"] + 32 * d["gossip_hd_words"] + 4 * d["gossip_window_words"]  # + window
    if name == "k_gossip_pull":  # receiver holds word r/w + receipts word per active window word, one
        return 12 * d["gossip_pull_words"] + 4 * d["gossip_probes"]  # sender window word per probe
    if name == "k_gossip_apply":
        # per receipt word: receipts r/w (8 B: read, clear), holdings r/w (8), newest/oldest round (2),
        # run starts (4), infection rounds read-modify-write (32 + 32), liveness word (4), list entry (4).
        # One-gossip slots (k_gossip_apply): per subject run one ring record (8 B), per subject the
        # table cell and its deadline (8 B). Batch slots (k_gossip_apply_b):
        # per run top its record range (8 B), per record its dictionary entry id (2 B with at most
        # 8,192 dictionary blocks, else 4: entry_id_bytes), per block with
        # received entries its merge mark and the block's generation (8 B), and per block merged (not
        # skipped by its mark) the entry's record, the block's subject and the table cell (12 B)
        # (records of long ranges ORed as their slot's entry bitmap: the bitmap's bytes, dsids, instead)
        recs = d.get("apply_records", 0)
        if recs:
            blocks = d["apply_subjects"] + d.get("apply_skipped", 0)
            walked = recs - d.get("apply_bitmap_records", 0)
            return (93 * d["apply_words"] + 8 * d["apply_runs"] + d.get("id_bytes", 4) * walked
                    + d.get("dict_bytes", 8192) * d.get("apply_bitmaps", 0) + 8 * blocks + 12 * d["apply_subjects"])
        return 93 * d["apply_words"] + 8 * d["apply_runs"] + 8 * d["apply_subjects"]
    if name == "k_susp_sweep":  # stream a u16 deadline column; per fired cell the deadline write, the
        # view cell read + write, and (a handle with an event ring) its 24-B REMOVED event
        return 2 * d["sweep_cells"] + 10 * d["suspicion_timeouts"] + 24 * d.get("sweep_events", 0)
    if name == "k_fd":  # cursor + count + liveness + target/proxy cells + own cell r/w (~24 B/member)
        return 24 * d["fd_probes"]
    # infectedFrom bookkeeping: in-history ring entries (16 B per registration,
    # ~gossip_probes / words per registration is not tracked, so per probe), pruned windows and
    # dense delivery records (a window word read + a word written per active position)
    # active words per member-round: gossip_scanned counts (member, round) pairs x the round's list
    act = max(1, d["gossip_scanned"] // max(1, d["fd_probes"] * rounds_per_period))
    if name == "k_gossip_inhist":  # in_list entry + ring entry per registered sender
        return 20 * d["fd_probes"] * 3
    if name == "k_gossip_pairwin":  # per pruned pair: the window copied and pruned over the list
        return 12 * d["infected_pruned_pairs"] * act
    if name == "k_gossip_record":  # per record: list entry + sender window read + body word written
        return 12 * d["infected_records"] * act
    return 0


# the kernel classes that can dominate a period (the roofline line's candidates): only these carry HIP
# events in the timed region by default (--timing major)
MAJOR_CLASSES = ["k_gossip_select", "k_gossip_pull", "k_gossip_apply", "k_susp_sweep", "k_sync_merge", "k_sync_ack",
                 "k_sync_snapshot"]

# kernel class (swim_kernel_time index names) -> the kernels rocprof sees under it
KERNEL_NAMES = {"k_gossip_apply": ["k_gossip_apply", "k_gossip_apply_b", "k_gossip_apply_h4", "k_gossip_apply_b_h4",
                                   "k_gossip_apply_b16", "k_gossip_apply_b16_h4"],
                "k_gossip_select": ["k_gossip_select", "k_gossip_select_h4"],
                "k_gossip_pull": ["k_gossip_pull", "k_gossip_pull_loss", "k_gossip_pull_dq", "k_gossip_pull_s4",
                                  "k_gossip_pull_loss_s4"],
                "k_gossip_pairwin": ["k_gossip_pairfill", "k_gossip_pairprune", "k_gossip_pairdelay"]}


def pmc_traffic(kernel, workload="c3", world=1, steps=None, warmup=None):
    """HBM bytes per launch of `kernel` from the committed PMC summary of exactly this run: the same
    workload, --steps and --warmup on one GPU (tools/gpu_pmc.sh: separate FETCH_SIZE and WRITE_SIZE
    rocprofv3 passes over `bench.py --steps S --warmup W`; FETCH_SIZE doubled per the gfx950 note
    in MI355X_MICROARCH.md): profiles/pmc_traffic_<workload>_s<S>_w<W>.json. None when no summary
    covers that window or kernel, or for a sharded run (per-launch traffic changes with the shard)."""
    if world != 1 or steps is None or warmup is None:
        return None
    path = os.path.join(REPO, "profiles", f"pmc_traffic_{workload}_s{steps}_w{warmup}.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    # a kernel class may be one of several kernels (k_gossip_apply is k_gossip_apply_b while the
    # ring holds batch slots): the one of the class this window dispatched most
    cands = [d[n] for n in KERNEL_NAMES.get(kernel, [kernel]) if n in d]
    if not cands:
        return None
    k = max(cands, key=lambda v: v.get("dispatches", 0))
    return k["fetch_bytes_x2"] + k["write_bytes"]


def entry_id_bytes(w):
    """Bytes of a record's dictionary entry id: 16 bits while the dictionary has at most 8,192 blocks
    (the library's c_id16), else 32."""
    return 2 if (w.get("dsub") or 8192) <= 8192 else 4


def roofline_of(name, ktimes, d, world, rounds_per_period=5):
    """achieved GB/s = algorithmic bytes per launch (kernel_bytes) / average launch time (HIP events
    on the handle's stream), for one kernel class over a measured window."""
    ms, launches = ktimes.get(name, (0.0, 0))
    byts = kernel_bytes(name, d, rounds_per_period)
    if not launches or not ms or not byts:
        return None
    avg_s = ms / 1e3 / launches
    per_launch = byts / world / launches  # work counters are cluster-wide, launches per shard
    achieved = per_launch / avg_s / 1e9
    return {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS, "bytes_per_launch": per_launch,
            "avg_launch_ms": avg_s * 1e3, "launches": launches}


def hbm_used_gib(device):
    """Device memory in use (hipMemGetInfo), GiB: the handle's arrays plus the HIP context."""
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        if hip.hipSetDevice(int(device)) or hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)):
            return None
        return round((total.value - free.value) / 2**30, 1)
    except OSError:
        return None


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def preset_config(preset):
    from swimhip import ClusterConfig

    return {"lan": ClusterConfig.defaultLanConfig, "local": ClusterConfig.defaultLocalConfig}[preset]()


def make_cluster(workload, device, seed, event_capacity=0, sharded=False, batching=True, **extra):
    """One cluster of the workload: on this GPU alone, or (sharded) this rank's observer rows of
    a cluster spread over the torch.distributed world."""
    from swimhip import ShardedSwimCluster, SwimCluster

    w = WORKLOADS[workload]
    cls = ShardedSwimCluster if sharded else SwimCluster
    kw = {"tracked_subjects": w["tracked"]} if w.get("tracked") else {}
    cfg = preset_config(w["preset"])
    if w.get("seeds"):  # the first `seeds` member ids are the seed addresses
        cfg = cfg.membership(lambda o: o.seedMembers(list(range(w["seeds"]))))
    # one slot per gossip without batches: the ring of round 2's C3 runs
    gcap = w["gcap"] if batching else max(w["gcap"], w.get("gcap_unbatched", 1 << 20))
    if w.get("rcap"):
        kw["record_capacity"] = w["rcap"]
    if w.get("dsub"):
        kw["dict_subjects"] = w["dsub"]
    kw.update(extra)
    c = cls(cfg, w["n"], seed=seed, gossip_capacity=gcap, device=device, gossip_batching=batching,
            event_capacity=event_capacity, sync_capacity=w.get("scap", 0), **kw)
    if w["loss"]:
        c.set_loss(w["loss"])
    return c


def inject_faults(c, workload, t0, seed, n=None):
    """The workload's fault schedule at period t0: crash set, then the partition window."""
    w = WORKLOADS[workload]
    n = n or w["n"]
    crashed = crash_set(n, w["crash_n"] / w["n"] if "crash_n" in w else w["crash"], seed)
    if crashed:
        c.crash(crashed)
    if w["part"]:
        c.partition(partition_groups(n, w["part_group"]), t0, t0 + w["part"])
    return crashed


def crash_set(n, frac, seed):
    k = int(round(n * frac))
    if k == 0:
        return []
    rng = np.random.default_rng(seed)
    return sorted(int(x) for x in rng.choice(n, size=k, replace=False))


# The oracle keeps per-member gossip maps and every delivery's infectedFrom record; the full-size
# C3 storm (~1e6 live gossips x 65,536 members) does not fit host RAM, so its CPU sample runs the
# same schedule at this many members (~3 GB of oracle state).
CPU_SAMPLE_N = 4096


def _oracle_run(args):
    """One oracle replica: warmup, the faults, then `periods` timed periods (or until `budget_s`)."""
    workload, warmup, seed, periods, budget_s = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle_py import OracleCluster

    w = WORKLOADS[workload]
    n = min(w["n"], CPU_SAMPLE_N)
    c = OracleCluster(preset_config(w["preset"]), n, seed=seed)
    if w["loss"]:
        c.set_loss(w["loss"])
    c.step(warmup)
    inject_faults(c, workload, warmup, seed, n=n)
    r0 = c.stats()["gossip_first_receipts"]
    done, t0 = 0, time.perf_counter()
    while done < periods and (budget_s is None or time.perf_counter() - t0 < budget_s):
        c.step(1)
        done += 1
    dt = time.perf_counter() - t0
    receipts = c.stats()["gossip_first_receipts"] - r0
    c.close()
    import resource

    return n, done, dt, receipts, resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024


# host memory the CPU replicas may hold together (the box caps one command at 270 GiB; the bench's own
# process holds the GPU handle beside them)
CPU_MEM_BUDGET = 128 << 30


def cpu_baseline(workload, warmup, budget_s=15.0, seed=1, max_periods=20):
    """The oracle (oracle/, C++ restatement, `kind: port`) on the same schedule at
    min(N, CPU_SAMPLE_N) members: first single-threaded for up to `max_periods` timed periods or
    ~budget_s, then that many periods on every host core at once (one independent replica per core,
    seeds seed .. seed + P - 1: the oracle is a sequential restatement, so the cores are used as
    replicas, which bounds what a thread-per-observer port could reach). `value` is the all-core
    aggregate; the single-thread rate is reported beside it."""
    import multiprocessing as mp

    # the single-thread sample in a child of its own, so that its peak resident set is the oracle's
    with mp.get_context("spawn").Pool(1) as pool:
        n, done, dt, rcpt, rss = pool.apply(_oracle_run, ((workload, warmup, seed, max_periods, budget_s),))
    single = n * done / dt
    # the box's CPU share for one GPU is 16; a lossy storm's oracle state grows by GBs per period
    # (C2: ~36 GB per replica after 20 periods), so the replicas are also bounded by host memory
    cores = max(1, min(16, os.cpu_count() or 1, CPU_MEM_BUDGET // max(1, int(rss * 1.25))))
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_oracle_run, [(workload, warmup, seed + k, done, None) for k in range(cores)])
    wall = time.perf_counter() - t0
    # each replica's own timed region; the pool's wall time (incl. its warmup) for the aggregate
    agg = sum(r[0] * r[1] for r in res) / max(r[2] for r in res)
    w = WORKLOADS[workload]
    return {"value": agg, "unit": "member-periods/s", "cores": cores, "kind": "port",
            "single_thread": {"value": single, "cores": 1, "periods": done, "seconds": round(dt, 2),
                              "peak_rss_gb": round(rss / 2**30, 2),
                              "gossip_first_receipts_per_s": rcpt / dt},
            "gossip_first_receipts_per_s": sum(r[3] for r in res) / max(r[2] for r in res),
            "sample": f"oracle (C++ restatement of the reference's per-member logic) on the same schedule at {n} of "
                      f"{w['n']} members: {warmup} untimed periods, the faults, then the first {done} timed periods; "
                      f"single thread {dt:.1f} s, then {cores} replicas (seeds {seed}..{seed + cores - 1}) on "
                      f"{cores} host cores at once ({wall:.1f} s wall incl. their warmup)"}


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch(gpus, argv, env=None):
    """How this invocation gets its `gpus` ranks (one process per GPU).

    Returns None when this process is already the one to run: `--gpus 1` without a launcher, or a
    rank started by torch.distributed.run whose WORLD_SIZE equals `--gpus`. A WORLD_SIZE that
    differs from `--gpus` is refused (ValueError): the line would name a GPU count it did not run on.
    Otherwise (`--gpus N > 1` with no WORLD_SIZE) returns the torch.distributed.run command that
    starts N ranks of this same script with the same arguments; the caller runs it as a child and
    relays its exit code, touching no GPU itself (the ranks inherit stdout, so rank 0's JSON line is
    this process's output)."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws}: launch {gpus} ranks, or pass --gpus {ws}")
        return None
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--converge", type=int, default=120,
                    help="untimed periods after the timed region to measure periods-to-DEAD (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="no MembershipEvent ring (the round-3 bench handle)")
    ap.add_argument("--infection-round-bits", type=int, default=0, choices=[0, 4, 8],
                    help="per (member, slot) infection rounds: 0 = the library's choice (DESIGN.md §4.4)")
    ap.add_argument("--unbatched", action="store_true", help="one ring slot per gossip (A/B of DESIGN.md §3.12)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--timing", default="major", choices=["major", "all"],
                    help="kernel classes bracketed by HIP events in the timed region: the ones that can dominate "
                         "a period (gossip select / pull / apply, suspicion sweep, SYNC merges), or every class "
                         "(each event pair adds a few microseconds of stream time to every small launch)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for --gpus > 1 (nccl = RCCL over xGMI; gloo = host-staged rehearsal)")
    args = ap.parse_args()

    try:
        launch = rank_launch(args.gpus, sys.argv[1:])
    except ValueError as e:
        ap.error(str(e))
    if launch is not None:  # --gpus N > 1 from a plain `python bench.py`: N ranks as children, no GPU here
        import subprocess

        log(f"--gpus {args.gpus}: starting {args.gpus} ranks under torch.distributed.run")
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(launch, env=env))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share a GPU
        torch.cuda.set_device(local)
        tdist.init_process_group(args.backend)
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    w = WORKLOADS[args.workload]
    n = w["n"]
    pc = preset_config(w["preset"])
    G = pc.failureDetectorConfig().pingInterval() // pc.gossipConfig().gossipInterval()  # rounds per period
    # the product path emits MembershipEvents (REMOVED from the suspicion sweep): an event ring that
    # holds one period's worst case (every crashed member removed by every local row), drained (count
    # and discard, like a listener that only counts) after every period of the converge window
    n_crash = w["crash_n"] if "crash_n" in w else int(round(n * w["crash"]))
    ecap = 0 if args.no_events else 1 << max(16, min(29, (max(1, n_crash) * (n // world) - 1).bit_length()))
    ecap = min(ecap, w.get("ecap", ecap))
    extra = {"infection_round_bits": args.infection_round_bits} if args.infection_round_bits else {}
    c = make_cluster(args.workload, local, args.seed, event_capacity=ecap, sharded=world > 1,
                     batching=not args.unbatched, **extra)
    hbm_used = hbm_used_gib(local)
    log(f"created {args.workload}: N={n}, event ring {ecap}, HBM used {hbm_used} GiB")
    c.step(args.warmup)
    log(f"warmup {args.warmup} periods done")
    crashed = inject_faults(c, args.workload, args.warmup, args.seed)
    crash_period = args.warmup
    s0 = c.stats()
    c.kernel_timing(True, classes=None if args.timing == "all" else MAJOR_CLASSES)
    barrier()
    c.sync()
    t0 = time.perf_counter()
    done, last_print = 0, t0
    while done < args.steps:  # chunks of 5 periods: a host sync per chunk, progress on stderr
        k = min(5, args.steps - done)
        c.step_async(k)
        c.sync()
        done += k
        now = time.perf_counter()
        if now - last_print > 20.0:
            log(f"timed: {done}/{args.steps} periods, {now - t0:.1f} s")
            last_print = now
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch

        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    s1 = c.stats()
    ktimes = c.kernel_times()
    c.kernel_timing(False)
    d = {k: s1[k] - s0[k] for k in s1}
    d["id_bytes"] = entry_id_bytes(w)
    d["dict_bytes"] = w.get("dsub") or 8192  # a slot entry bitmap: one bit per entry, 8 per block
    n_events = c.discard_events() if ecap else 0  # (none expected: no timeout falls due in the window)

    # dominant kernel + roofline over the timed region
    dom = max((k for k in ktimes if k != "bookkeeping"), key=lambda k: ktimes[k][0])
    rl = roofline_of(dom, ktimes, d, world, G) or {"achieved": 0.0, "frac": 0.0, "bytes_per_launch": 0.0,
                                                 "avg_launch_ms": 0.0, "launches": 0}
    fracs = {k: round(v["frac"], 4) for k in ktimes if k != "bookkeeping"
             for v in [roofline_of(k, ktimes, d, world, G)] if v}

    # periods to DEAD convergence (untimed): every alive observer removed every crashed member;
    # the kernels are timed here too, for the suspicion sweep (no timeout fires in the timed region)
    periods_to_dead = None
    conv = None
    sweep_rl = None
    if crashed and args.converge:
        sc0 = c.stats()
        c.kernel_timing(True)
        extra = 0
        # the suspicion sweep only has work in the periods whose deadlines fall due: its roofline is
        # taken over those launches (one period at a time, kernel-time and sweep_cells deltas)
        fire_ms, fire_n, fire_cells, fire_dead, fire_ev = 0.0, 0, 0, 0, 0
        st = c.stats()
        while extra < args.converge and st["not_converged"]:
            k0 = c.kernel_times().get("k_susp_sweep", (0.0, 0))
            c.step(1)
            extra += 1
            ev = c.discard_events() if ecap else 0
            n_events += ev
            st1 = c.stats()
            k1 = c.kernel_times().get("k_susp_sweep", (0.0, 0))
            if st1["sweep_cells"] > st["sweep_cells"]:
                fire_ms += k1[0] - k0[0]
                fire_n += k1[1] - k0[1]
                fire_cells += st1["sweep_cells"] - st["sweep_cells"]
                fire_dead += st1["suspicion_timeouts"] - st["suspicion_timeouts"]
                fire_ev += ev
            st = st1
            if extra % 5 == 0:
                log(f"converge: +{extra} periods, not_converged={st['not_converged']}")
        pres, last = c.presence()
        if c.stats()["not_converged"] == 0:
            periods_to_dead = int(max(last[crashed])) - 1 - crash_period
        kt2 = c.kernel_times()
        dc = {k: v - sc0[k] for k, v in c.stats().items()}
        conv = {k: round(v["frac"], 4) for k in ("k_sync_merge", "k_sync_ack")
                for v in [roofline_of(k, kt2, dc, world, G)] if v}
        if fire_n:
            sweep_rl = roofline_of("k_susp_sweep", {"k_susp_sweep": (fire_ms, fire_n)},
                                   {"sweep_cells": fire_cells, "suspicion_timeouts": fire_dead,
                                    "sweep_events": fire_ev * world}, world)
            conv["k_susp_sweep"] = round(sweep_rl["frac"], 4)
        c.kernel_timing(False)

    value = n * args.steps / elapsed  # the one cluster's member-periods (all shards together)
    out = {
        "metric": "member-periods/sec (whole node)",
        "value": value,
        "unit": "member-periods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",  # the one cluster of the workload, its observers split over the GPUs
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (converged start, Philox-chosen crash set, seeded)",
        "config": {"workload": w["desc"], "members": n, "members_per_gpu": n // world,
                   "parallelism": f"observer-row shards x{world}" if world > 1 else "1 GPU",
                   "crashed": len(crashed), "loss_pct": w["loss"], "partition_periods": w["part"],
                   "gossip_ring_slots": w["gcap"] if not args.unbatched else max(w["gcap"], w.get("gcap_unbatched", 1 << 20)),
                   "gossip_batching": not args.unbatched, "tracked_subjects": w.get("tracked")},
        "periods_to_dead": periods_to_dead,
        # work-normalised rates: the storm's work per member-period grows with N, so member-periods/s
        # alone does not compare runs of different sizes
        "rates": {"gossip_first_receipts_per_s": d["gossip_first_receipts"] / elapsed,
                  "gossips_created_per_s": d["gossips_created"] / elapsed,
                  "gossip_requests_per_s": d["gossip_sends"] / elapsed},
        "roofline": {"bound": "hbm", "kernel": dom, "timed_classes": args.timing, "achieved": rl["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": rl["frac"], "traffic": pmc_traffic(dom, args.workload, world, args.steps, args.warmup),
                     "bytes_per_launch": rl["bytes_per_launch"], "avg_launch_ms": rl["avg_launch_ms"],
                     "launches": rl["launches"]},
        "kernels_ms": {k: round(v[0], 3) for k, v in ktimes.items()},
        "kernels_frac": fracs,
        "converge_kernels_frac": conv,
        "sweep_roofline": None if sweep_rl is None else {
            "achieved": sweep_rl["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sweep_rl["frac"],
            "bytes_per_launch": sweep_rl["bytes_per_launch"], "avg_launch_ms": sweep_rl["avg_launch_ms"],
            "launches": sweep_rl["launches"], "window": "the periods whose suspicion deadlines fell due",
            "events": "REMOVED events emitted" if ecap else "no event ring (--no-events)"},
        "events": {"capacity": ecap, "emitted": n_events} if ecap else None,
        "hbm_used_gib": hbm_used,
        "work": {k: d[k] for k in ("fd_probes", "gossips_created", "gossip_first_receipts", "syncs_delivered",
                                   "merge_cells", "gossip_scanned", "gossip_hd_words", "gossip_window_words",
                                   "gossip_pull_words", "gossip_probes", "events_removed", "gossip_sends",
                                   "infected_suppressed", "infected_pruned_pairs", "infected_records",
                                   "apply_words", "apply_runs", "apply_subjects", "apply_records", "apply_spills",
                                   "apply_skipped", "apply_bitmaps", "apply_bitmap_records")},
        "gossip_slots": {"live_at_end": s1["live_gossip_slots"], "gossips_live_at_end": s1["live_gossip_records"]},
    }
    c.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU baseline is an N = 1 figure
        cb = out["cpu_baseline"] = cpu_baseline(args.workload, args.warmup, args.cpu_budget, args.seed, args.steps)
        # The comparison: the CPU sample runs a smaller cluster of the same schedule (the full-size storm
        # does not fit the oracle's host tables), and a storm's work per member-period grows with N, so
        # member-periods/s of the two are not the same unit of work; first gossip receipts (one
        # onGossipReq of a new gossip id each, GossipProtocolImpl.java:171-183) are
        if cb and cb.get("value") and cb.get("gossip_first_receipts_per_s"):
            out["vs_cpu"] = {"basis": "gossip first receipts per second (work-normalised: the CPU sample's cluster "
                                      "is smaller, and per-member-period work grows with N)",
                             "ratio": out["rates"]["gossip_first_receipts_per_s"] / cb["gossip_first_receipts_per_s"],
                             "member_periods_ratio_not_comparable": out["value"] / cb["value"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
