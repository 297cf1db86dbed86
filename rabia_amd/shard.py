"""Slot sharding across GPUs and the global-commit exchange.

Slots are independent consensus instances (each PhaseId has its own PhaseData,
rabia-engine/src/state.rs:21), so a window splits into contiguous shards, one per
rank (one process per GPU), with no data-path collective. The one real exchange
is the total-order commit: every shard publishes its step result (contiguous
watermark, last_committed, counts) and, optionally, its decided bitmap; ranks
all_gather them (RCCL over xGMI when the backend is "nccl") and fold them into
the global commit view here.

Results are shard-invariant in WMVC mode (the coin is keyed by the GLOBAL slot
id). In REF mode each shard is its own engine with its own StdRng stream
(sharded-KV instances); a single REF stream spanning shards would need the
cross-shard VQ prefix.
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
