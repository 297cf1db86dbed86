"""Slot sharding across GPUs and the global-commit exchange.

Slots are independent consensus instances (each PhaseId has its own PhaseData,
rabia-engine/src/state.rs:21), so a window splits into contiguous shards, one per
rank (one process per GPU), with no data-path collective. The one real exchange
is the total-order commit: every shard publishes its step result (contiguous
watermark, last_committed, counts) and, optionally, its decided bitmap; ranks
all_gather them (RCCL over xGMI when the backend is "nccl") and fold them into
the global commit view here.

Results are shard-invariant in both modes. WMVC: the coin is keyed by the
GLOBAL slot id. REF: every rank holds the SAME engine seed and the window's one
StdRng stream (engine.rs:59-62) is consumed in ascending slot order across the
shards: shard r's k-th VQ slot takes the draw at  rng_next + (VQ slots of shards
< r) + k  (engine.rs:567-611). The device does it without a cross-GPU wait in the
step (include/rabia_gpu.h, "Sharded REF"): step with provisional draw positions
+ draw records -> all_gather of the rows -> fix-up at the global positions ->
all_gather of the final rows -> commit fold. `draw_bases` / `combine` below are the
same algebra on the host.
"""
from __future__ import annotations

from dataclasses import dataclass

RESULT_FIELDS = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws",
                 "last_committed_max", "first_undecided", "rng_next", "commit_watermark", "flags"]


def shard_range(total_slots: int, world: int, rank: int, align: int = 128):
    """Contiguous shard [start, start+count) of a window, boundaries on `align`
    slots so each shard's planes start on a 16-B word boundary."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    units = (total_slots + align - 1) // align
    lo = units * rank // world
    hi = units * (rank + 1) // world
    start = min(lo * align, total_slots)
    end = min(hi * align, total_slots)
    return start, end - start


@dataclass
class GlobalCommit:
    n_slots: int
    n_decided: int
    n_v1: int
    n_pending_r1: int
    n_draws: int
    last_committed: int
    first_undecided: int
    commit_watermark: int
    flags: int


def combine(results, starts, counts, slot_base: int, watermark_in: int, last_committed_in: int = 0):
    """Fold per-shard step results of ONE window (shards in rank order) into the
    global commit: counts add, last_committed is the max (commit_phase's CAS max,
    state.rs:77-99), first_undecided is the min over shards, and the contiguous
    watermark advances exactly as a single evaluator over the whole window would
    (first undecided slot, if the window starts at or before the watermark)."""
    tot = {k: 0 for k in ("n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "flags")}
    lc = last_committed_in
    end = slot_base + sum(counts)
    fu = end
    for r, start, count in zip(results, starts, counts):
        for k in tot:
            tot[k] = tot[k] | int(r.get(k, 0)) if k == "flags" else tot[k] + int(r[k])
        lc = max(lc, int(r["last_committed_max"]))
        if count:
            fu = min(fu, int(r["first_undecided"]))
    wm = fu if slot_base <= watermark_in < fu else watermark_in
    return GlobalCommit(tot["n_slots"], tot["n_decided"], tot["n_v1"], tot["n_pending_r1"],
                        tot["n_draws"], lc, fu, wm, tot["flags"])


def draw_bases(n_draws, rng_base: int):
    """Global StdRng position of each shard's first draw: rng_base + the VQ slots of
    the shards before it (exclusive prefix in rank order)."""
    out, acc = [], int(rng_base)
    for c in n_draws:
        out.append(acc)
        acc += int(c)
    return out, acc


def window_draw_bases(n_draws, rank: int, rng_base: int):
    """The fix-up's stream positions for K consecutive windows of one step (the device's
    fix_first_draw / finish algebra, rg_kernels.h): n_draws[r][w] = shard r's VQ slots in
    window w (the step rows, rank-major as the all-gather lays them out). Window w of
    shard `rank` draws from g0[w] = rng_base + every shard's draws of windows < w + the
    lower shards' draws of window w (ascending slot order over the windows,
    engine.rs:567-611); after[w] = the engine position after window w."""
    world, K = len(n_draws), len(n_draws[0]) if n_draws else 0
    g0, after, pos = [], [], int(rng_base)
    for w in range(K):
        col = [int(n_draws[r][w]) for r in range(world)]
        g0.append(pos + sum(col[:rank]))
        pos += sum(col)
        after.append(pos)
    return g0, after


def commit_windows(rows_all, window_base: int, window_slots: int, watermark_in: int, last_committed_in: int):
    """The commit fold of K consecutive windows (rg_shard_commit_windows_async): rows_all
    [world][K] final rows (dicts); each window folds like `combine`, the watermark and
    last_committed chaining from window to window. Returns the K GlobalCommits."""
    world, K = len(rows_all), len(rows_all[0]) if rows_all else 0
    out, wm, lc = [], int(watermark_in), int(last_committed_in)
    for w in range(K):
        base = window_base + w * window_slots
        fu = base + window_slots
        tot = {k: 0 for k in ("n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "flags")}
        for r in range(world):
            x = rows_all[r][w]
            for k in tot:
                tot[k] = tot[k] | int(x.get(k, 0)) if k == "flags" else tot[k] + int(x[k])
            lc = max(lc, int(x["last_committed_max"]))
            if int(x["n_slots"]):
                fu = min(fu, int(x["first_undecided"]))
        if tot["n_slots"] != window_slots:
            tot["flags"] |= 16
        if base <= wm < fu:
            wm = fu
        out.append(GlobalCommit(tot["n_slots"], tot["n_decided"], tot["n_v1"], tot["n_pending_r1"], tot["n_draws"],
                                lc, fu, wm, tot["flags"]))
    return out


CLUSTER_FIELDS = ["all_decided", "decided_v1", "sum_phases", "max_phases", "sum_coin_phases",
                  "sum_first_decision_phase", "slots", "reserved"]


def combine_cluster(rows):
    """Fold per-shard Weak-MVC cluster statistics (rg_wmvc_cluster_async stats_dev,
    shards in rank order): counts and sums add, the phase maximum is the max. The
    coin is keyed by the GLOBAL slot id, so the fold equals one run over the window."""
    out = [0] * 8
    for r in rows:
        r = [int(x) for x in r]
        for k in range(8):
            out[k] = max(out[k], r[k]) if k == 3 else out[k] + r[k]
    return dict(zip(CLUSTER_FIELDS, out))


def result_row(d: dict):
    return [int(d.get(k, 0)) for k in RESULT_FIELDS]


def row_result(row) -> dict:
    return {k: int(v) for k, v in zip(RESULT_FIELDS, row)}


def exchange_results(row_tensor, group=None):
    """all_gather one rank's 10-u64 step result (int64 tensor on the rank's
    device for "nccl", CPU for "gloo"); returns [world, 10]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    src = row_tensor.contiguous().view(-1)
    out = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.view((world,) + tuple(row_tensor.shape))


def exchange_bitmap(plane_tensor, group=None):
    """all_gather of each shard's decided (committed) bit plane, equal-sized
    shards; the concatenation is the window's global decided bitmap."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    src = plane_tensor.contiguous().view(-1)
    out = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.view((world,) + tuple(plane_tensor.shape))


def rendezvous_store(rank: int, world: int, timeout_s: float = 300.0):
    """The host channel that carries rank 0's RCCL id to every rank: the TCP store of the
    launcher (torch.distributed.run's agent store, TORCHELASTIC_USE_AGENT_STORE) or,
    without one, a store rank 0 serves at MASTER_ADDR:MASTER_PORT. A key-value store,
    not a collective: the data path runs through the C ABI's communicator."""
    import datetime
    import os
    from torch.distributed import PrefixStore, TCPStore
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    store = TCPStore(host, port, world, is_master=(rank == 0 and not agent),
                     timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
    return PrefixStore("rabia_rg_comm/", store)


class RcclComm:
    """Rank `rank` of `world`: the RCCL id (rank 0 makes it, the rendezvous store carries
    it) to attach to this rank's evaluator contexts (rg_comm_create, a collective). World
    1 needs no store."""

    _made = 0  # communicators made by this process (every rank makes them in the same order)

    def __init__(self, rank: int, world: int, store=None, key: str = None, make_uid=None):
        if make_uid is None:  # rank 0's id maker (rg_comm_unique_id); tests pass their own
            from .engine import PhaseEvaluator
            make_uid = PhaseEvaluator.comm_unique_id
        self.rank, self.world = rank, world
        if world == 1:
            self.uid = make_uid()
            return
        store = store if store is not None else rendezvous_store(rank, world)
        self.key = key if key is not None else self.default_key()
        if rank == 0:
            self.uid = bytes(make_uid())
            store.set(self.key, self.uid)
        else:
            self.uid = bytes(store.get(self.key))
            if len(self.uid) != 128:
                raise RuntimeError(f"rendezvous key {self.key}: {len(self.uid)}-byte value, not a 128-byte RCCL id")

    @classmethod
    def default_key(cls) -> str:
        """A key no earlier communicator of the job used: the launcher's agent store outlives
        worker restarts (TORCHELASTIC_RESTART_COUNT changes on each) and one process may make
        several communicators (a per-process counter, advanced alike on every rank)."""
        import os
        RcclComm._made += 1
        return f"uid/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/{RcclComm._made}"

    def attach(self, ev):
        ev.comm_create(self.uid, self.rank, self.world)
        return ev

    @staticmethod
    def reserve(ev, max_windows: int, max_slots: int, undecided_cap: int = 0):
        """Size the attached context's exchange scratch (rg_comm_reserve, synchronous): the
        exchange calls themselves never allocate."""
        ev.comm_reserve(max_windows, max_slots, undecided_cap)


class ShardedRefStep:
    """One rank's driver of the sharded REF window (include/rabia_gpu.h): the four
    stages of one window on this rank's evaluator. With an RCCL communicator attached
    to the evaluator (RcclComm.attach, rccl=True) stages 2-4 are ONE C-ABI call
    (rg_shard_exchange_windows_async: the all-gathers run on the device stream);
    otherwise the two row exchanges go through torch.distributed (host copies for
    "gloo": the CPU rehearsal). Synchronous per window; bench.py pipelines the same
    calls across windows.

    shared_gpu=True: the ranks share one GPU (a rehearsal: one process per rank on one
    device). Their step launches then take turns: a tiled-kernel look-back launch
    (small shards) relies on dispatch order, and two such launches running at once on
    one GPU can wait on each other across kernels (include/rabia_gpu.h).
    The in-process chain of the C ABI cannot order launches of other processes."""

    def __init__(self, ev, rank: int, world: int, n_slots_cap: int, group=None, shared_gpu: bool = False,
                 rccl: bool = False):
        import torch
        self.ev, self.rank, self.world, self.group = ev, rank, world, group
        self.shared_gpu = shared_gpu
        self.rccl = rccl
        self.cap = int(n_slots_cap)
        from .engine import record_window_words
        # the shard's draw-record region (chunk table + 4-B records) for shards of up to cap slots
        self.records = torch.empty(record_window_words(max(self.cap, 1), max(self.cap, 1)), dtype=torch.int32,
                                   device="cuda")
        self.row = torch.zeros(10, dtype=torch.int64, device="cuda")
        self.fixed = torch.zeros(10, dtype=torch.int64, device="cuda")
        self.result = torch.zeros(10, dtype=torch.int64, device="cuda")

    def _gather(self, row):
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return row.view(1, 10).clone()
        if dist.get_backend(self.group) == "nccl":
            return exchange_results(row, self.group)
        got = exchange_results(row.cpu(), self.group)
        return got.to(row.device)

    def step(self, votes_ptr, out_ptr, n_slots, stride, shard_base, window_base, window_slots,
             max_phase=0, stream=0):
        """Evaluate this rank's shard [shard_base, shard_base + n_slots) of the window
        [window_base, window_base + window_slots); returns the global step result."""
        import torch
        ev = self.ev
        if self.rccl:
            ev.phase_step_shard_async(votes_ptr, out_ptr, n_slots, stride, shard_base, self.records.data_ptr(),
                                      self.cap, self.row.data_ptr(), max_phase, stream)
            ev.shard_exchange_windows_async(1, out_ptr, 0, n_slots, stride, shard_base, window_base, window_slots,
                                            self.records.data_ptr(), self.cap, self.row.data_ptr(),
                                            self.result.data_ptr(), max_phase=max_phase, stream=stream)
            ev.sync(stream)
            return row_result(self.result.cpu().numpy().view("uint64").tolist())
        for r in (range(self.world) if self.shared_gpu and self.world > 1 else [self.rank]):
            if r == self.rank:
                ev.phase_step_shard_async(votes_ptr, out_ptr, n_slots, stride, shard_base, self.records.data_ptr(),
                                          self.cap, self.row.data_ptr(), max_phase, stream)
                torch.cuda.synchronize()
            if self.shared_gpu and self.world > 1:
                import torch.distributed as dist
                dist.barrier(self.group)
        rows = self._gather(self.row).contiguous()
        ev.shard_fixup_async(out_ptr, n_slots, stride, shard_base, self.records.data_ptr(), self.cap,
                             rows.data_ptr(), self.rank, self.world, self.fixed.data_ptr(), max_phase, stream)
        torch.cuda.synchronize()
        fixed = self._gather(self.fixed).contiguous()
        ev.shard_commit_async(fixed.data_ptr(), self.world, window_base, window_slots, self.result.data_ptr(),
                              stream)
        torch.cuda.synchronize()
        return row_result(self.result.cpu().numpy().view("uint64").tolist())
