"""ShardedSwimCluster — one simulated cluster row-sharded over several GPUs / processes.

Rank r of a torch.distributed group owns observers [r*N/W, (r+1)*N/W): their membership tables,
suspicion deadlines, gossip holdings and protocol cursors. Each rank drives its
libswimhip.so handle with swim_shard_step and performs the exchanges the library describes on
the group: all-gather of each phase's new gossips (ids stay identical on every shard; each block
also carries the rank's per-word gossip liveness), all-to-all-v of sender windows bound for remote
receivers and of SYNC / SYNC_ACK tables of cross-shard pairs. Every collective, and every period
end, is preceded by a small status all-gather, so an error on one rank is raised on all. On ROCm the "nccl" backend is RCCL over xGMI and
the buffers stay in HBM; with "gloo" (tests on one GPU, or CPU rehearsal of the protocol) they are
staged through host memory. Results equal the unsharded SwimCluster's bit for bit.

Every rank must make the same calls in the same order (fault injection, stepping and the
observation accessors, which are collective).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat
from .cluster import MembershipEvent, SwimCluster, SwimError


class ShardedSwimCluster(SwimCluster):
    """exchange = "library" (default): the library drives every exchange of a period itself
    (swim_step): over its own RCCL communicator on the "nccl" backend (swim_shard_comm_init; rank 0's
    unique id broadcast once), or through host-staged gloo callbacks (swim_shard_set_transport);
    one status all-gather and one host stop per exchange. exchange = "host": this class runs each
    exchange the library describes (swim_shard_step), with torch.distributed."""

    def __init__(self, config, n_members: int, seed: int = 0, *, group=None, device: int = 0,
                 exchange: str = "library", **kw):
        import torch
        import torch.distributed as dist

        self._dist = dist
        self._torch = torch
        self._group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._gloo = dist.get_backend(group) == "gloo"
        super().__init__(config, n_members, seed, device=device, _shard=(self.rank, self.world), **kw)
        self.nloc = self.n // self.world
        self.row0 = self.rank * self.nloc
        sw, rw = ctypes.c_uint64(), ctypes.c_uint64()
        self._call("shard_buffer_words", self._h, ctypes.byref(sw), ctypes.byref(rw))
        dev = torch.device("cuda", device)
        self._send = torch.empty(max(1, sw.value), dtype=torch.int32, device=dev)
        self._recv = torch.empty(max(1, rw.value), dtype=torch.int32, device=dev)
        self._call("shard_attach", self._h, ctypes.c_void_p(self._send.data_ptr()),
                   ctypes.c_void_p(self._recv.data_ptr()))
        self._x = nat.SwimXchg()
        if exchange not in ("library", "host"):
            raise ValueError("exchange: 'library' or 'host'")
        self._lib_x = exchange == "library"
        if self._lib_x:
            self._attach_transport()

    # -- library-driven exchanges ------------------------------------------------------------
    def _attach_transport(self):
        if not self._gloo:  # the library's own RCCL communicator over xGMI
            uid = (ctypes.c_uint8 * 128)()
            if self.rank == 0:
                self._call_raw("rccl_unique_id", uid)
            obj = [bytes(uid)]
            self._dist.broadcast_object_list(obj, src=0, group=self._group)
            ctypes.memmove(uid, obj[0], 128)
            self._call("shard_comm_init", self._h, uid, self.rank, self.world)
            return
        torch, dist, grp, W = self._torch, self._dist, self._group, self.world
        errors = self._cb_errors = []

        def words(ptr, nbytes):  # a host buffer of the library as int32 words (sizes are multiples of 4)
            return np.ctypeslib.as_array((ctypes.c_int32 * (nbytes // 4)).from_address(ptr)) if nbytes else \
                np.zeros(0, dtype=np.int32)

        def allgather(ctx, send, recv, nbytes, stream):
            try:
                src = torch.from_numpy(words(send, nbytes).copy())
                parts = [torch.empty_like(src) for _ in range(W)]
                dist.all_gather(parts, src, group=grp)
                words(recv, W * nbytes)[:] = torch.cat(parts).numpy()
                return 0
            except Exception as e:  # noqa: BLE001 (reported after the library returns)
                errors.append(e)
                return -1

        def alltoallv(ctx, send, sb, recv, rb, stream):
            try:
                sc = [int(sb[q]) // 4 for q in range(W)]
                rc = [int(rb[q]) // 4 for q in range(W)]
                src = torch.from_numpy(words(send, 4 * sum(sc)).copy())
                out = torch.empty(sum(rc), dtype=torch.int32)
                dist.all_to_all_single(out, src, rc, sc, group=grp)
                words(recv, 4 * sum(rc))[:] = out.numpy()
                return 0
            except Exception as e:  # noqa: BLE001
                errors.append(e)
                return -1

        self._cbs = (nat.ALLGATHER_FN(allgather), nat.ALLTOALLV_FN(alltoallv))  # kept alive with the handle
        t = nat.SwimTransport(None, 1, self._cbs[0], self._cbs[1])
        self._call("shard_set_transport", self._h, ctypes.byref(t))

    def _call_raw(self, name, *args):
        rc = getattr(self._lib, "swim_" + name)(*args)
        if rc != nat.SWIM_OK:
            raise SwimError(rc, name)

    # -- collectives ---------------------------------------------------------------------
    def _all_gather_ints(self, vals):
        """Every rank's row of ints, in rank order: one collective into one tensor and (RCCL) one
        device-to-host copy, not one per rank."""
        torch = self._torch
        t = torch.tensor(vals, dtype=torch.int64)
        if self._gloo:
            out = [torch.empty_like(t) for _ in range(self.world)]
            self._dist.all_gather(out, t, group=self._group)
            return [o.tolist() for o in out]
        t = t.to(self._send.device)
        out = torch.empty(self.world * t.numel(), dtype=torch.int64, device=t.device)
        self._dist.all_gather_into_tensor(out, t, group=self._group)
        return out.view(self.world, -1).cpu().tolist()

    def _exchange(self, status):
        """The collective the library described; `status` = every rank's [code, op, counts...]
        (one row per rank, from the status all-gather that precedes it)."""
        torch, dist, x, W = self._torch, self._dist, self._x, self.world
        if x.op == nat.X_ALLGATHER:
            counts = [row[2] for row in status]
            m = max(counts)
            if m:
                src = self._send[:m]
                dst = self._recv[:W * m]
                if self._gloo:
                    parts = [torch.empty(m, dtype=torch.int32) for _ in range(W)]
                    dist.all_gather(parts, src.cpu(), group=self._group)
                    dst.copy_(torch.cat(parts))
                else:
                    dist.all_gather_into_tensor(dst, src, group=self._group)
            for q in range(W):
                x.recv_counts[q] = counts[q]
            x.recv_stride = m
        elif x.op == nat.X_ALLTOALLV:
            allc = [row[2:] for row in status]  # allc[q][r] = words rank q sends to rank r
            sc = allc[self.rank]
            rc = [allc[q][self.rank] for q in range(W)]
            si, ri = sum(sc), sum(rc)
            # every rank checks every rank's volumes (same buffer sizes everywhere): all raise together
            over = [r for r in range(W) if sum(allc[r]) > self._send.numel()
                    or sum(allc[q][r] for q in range(W)) > self._recv.numel()]
            if over:
                raise SwimError(-75, f"shard exchange over the buffer capacity on rank(s) {over}")
            if max(max(row) for row in allc):
                src, dst = self._send[:si], self._recv[:ri]
                if self._gloo:
                    hd = torch.empty(ri, dtype=torch.int32)
                    dist.all_to_all_single(hd, src.cpu(), rc, sc, group=self._group)
                    dst.copy_(hd)
                else:
                    dist.all_to_all_single(dst, src, rc, sc, group=self._group)
            for q in range(W):
                x.recv_counts[q] = rc[q]
            x.recv_stride = sum(sum(row) for row in allc)  # global volume: 0 lets the library skip ahead
        else:
            raise RuntimeError(f"unknown exchange op {x.op}")
        if self._send.is_cuda:  # the library resumes on its own stream
            torch.cuda.synchronize(self._send.device)

    def _status(self, err):
        """Status all-gather before every collective and at the end of every period: a failure on
        one rank (an overflow only it detected, a bad size) becomes the same SwimError on every
        rank instead of leaving the others blocked in the next collective."""
        x, W = self._x, self.world
        if err is not None:
            row = [int(err.code), -1] + [0] * W
        elif x.op == nat.X_ALLGATHER:
            row = [0, int(x.op), int(x.send_words)] + [0] * (W - 1)
        elif x.op == nat.X_ALLTOALLV:
            row = [0, int(x.op)] + [int(x.send_counts[q]) for q in range(W)]
        else:
            row = [0, int(x.op)] + [0] * W
        status = self._all_gather_ints(row)
        bad = [(q, r[0]) for q, r in enumerate(status) if r[0]]
        if err is not None:
            raise err
        if bad:
            q, code = bad[0]
            raise SwimError(code, f"shard_step failed on rank {q} (status {code})")
        if len({r[1] for r in status}) != 1:
            raise SwimError(-22, f"shards out of step: exchange ops {[r[1] for r in status]}")
        return status

    def step(self, periods: int = 1):
        if self._lib_x:
            if getattr(self, "_cb_errors", None):  # a failure of an earlier step is not this step's cause
                self._cb_errors.clear()
            try:
                self._call("step", self._h, int(periods))
            except SwimError:
                if getattr(self, "_cb_errors", None):
                    raise SwimError(-6, f"host collective failed: {self._cb_errors[0]!r}")
                raise
            self.period += int(periods)
            return
        for _ in range(int(periods)):
            while True:
                err = None
                try:
                    self._call("shard_step", self._h, ctypes.byref(self._x))
                except SwimError as e:
                    err = e
                status = self._status(err)
                if self._x.op == nat.X_DONE:
                    break
                self._exchange(status)
            self.period += 1

    def step_async(self, periods: int = 1):
        self.step(periods)

    # -- collective fault injection: every rank must pass the same arguments ----------------
    def _same_args(self, name, ids):
        """All-gather a digest of the call's arguments and fail on every rank when they differ. A
        leave changes the layout of every later commit exchange block (a {gossips, stopped} header,
        include/swimhip.h); ranks that disagree would read each other's blocks wrongly."""
        ids = np.asarray(list(ids), dtype=np.uint64)
        dig = int((ids * np.uint64(0x9E3779B97F4A7C15) + np.arange(len(ids), dtype=np.uint64)).sum()
                  & np.uint64(0x7FFFFFFFFFFFFFFF)) if len(ids) else 0
        rows = self._all_gather_ints([len(ids), dig])
        if any(r != rows[0] for r in rows):
            raise SwimError(-22, f"{name}: ranks passed different arguments {rows}")

    def leave(self, ids):
        ids = list(ids)
        self._same_args("leave", ids)
        super().leave(ids)

    def crash(self, ids):
        ids = list(ids)
        self._same_args("crash", ids)
        super().crash(ids)

    def join(self, ids):
        """Joins on a sharded handle: every rank makes the same call; the joiner's row
        lives on its shard, its initial SYNCs to seeds on other shards travel in the SYNC exchange."""
        ids = list(ids)
        self._same_args("join", ids)
        super().join(ids)

    def restart(self, old_ids, new_ids):
        old_ids, new_ids = list(old_ids), list(new_ids)
        self._same_args("restart", old_ids + new_ids)
        super().restart(old_ids, new_ids)

    def update_metadata(self, ids):
        ids = list(ids)
        self._same_args("update_metadata", ids)
        super().update_metadata(ids)

    def sync(self):
        self._call("sync", self._h)

    # -- collective observation ------------------------------------------------------------
    def _owner(self, i):
        return int(i) // self.nloc

    def _bcast_row(self, i, reader):
        obj = [reader(i) if self._owner(i) == self.rank else None]
        self._dist.broadcast_object_list(obj, src=self._owner(i), group=self._group)
        return obj[0]

    def view(self, observer: int) -> np.ndarray:
        return self._bcast_row(observer, lambda i: SwimCluster.view(self, i))

    def deadlines(self, observer: int) -> np.ndarray:
        return self._bcast_row(observer, lambda i: SwimCluster.deadlines(self, i))

    def _gather_objects(self, obj):
        out = [None] * self.world
        self._dist.all_gather_object(out, obj, group=self._group)
        return out

    def digest(self):
        parts = self._gather_objects(SwimCluster.digest(self))
        m = (1 << 64) - 1
        return sum(p[0] for p in parts) & m, sum(p[1] for p in parts) & m

    def presence(self):
        parts = self._gather_objects(SwimCluster.presence(self))
        pres = np.sum([p[0] for p in parts], axis=0).astype(np.uint32)
        last = np.max([p[1] for p in parts], axis=0).astype(np.uint32)
        return pres, last

    _SAME = ("period", "live_gossip_slots", "live_gossip_records", "quiet_periods")

    def stats(self) -> dict:
        parts = self._gather_objects(SwimCluster.stats(self))
        out = {}
        for k in parts[0]:
            if k in self._SAME:
                out[k] = parts[0][k]
            elif k == "overflow":
                out[k] = int(np.bitwise_or.reduce([p[k] for p in parts]))
            else:
                out[k] = sum(p[k] for p in parts)
        return out

    def events(self, cap: int = 1 << 20):
        mine = [tuple(e.__dict__.values()) for e in SwimCluster.events(self, cap)]
        allev = [MembershipEvent(*t) for part in self._gather_objects(mine) for t in part]
        allev.sort(key=lambda e: (e.period, e.observer, e.phase, e.member, e.type))
        return allev
