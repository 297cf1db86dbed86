#!/usr/bin/env python3
"""Benchmark: consensus slots decided/sec on the batched Rabia phase evaluator.

Workload (BASELINE.json configs[1], "C2"): 5 replicas, windows of 2^20 slots,
90%-agreement synthetic vote trace, REF single phase sweep. One bench "step" is
one launch over `--windows` consecutive 2^20-slot windows (default 256: the
steady-state streaming batch; --windows 1 is the single-sweep latency case and is
also reported as `sweep_1m_us`). Inputs are generated on the device before the
timed region and rotate over 3 buffer sets (> 2x the 256 MiB Infinity Cache) so
every step reads from HBM.

Multi-GPU (torchrun, one rank per GPU): every rank is one slot shard with its own
engine context (weak scaling); after each step the per-shard step results
(commit watermark, last_committed, counts) are exchanged with an RCCL all_gather
that overlaps the next step.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the native library: shared HIP runtime)

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
WINDOW = 1 << 20


def bytes_per_slot_ref(n: int) -> float:
    """Algorithmic bytes per slot per REF phase evaluation:
    read R1 + R2 codes (4n bits), write 8 output bits."""
    return (4 * n + 8) / 8.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--windows", type=int, default=256)
    ap.add_argument("--replicas", type=int, default=5)
    ap.add_argument("--sets", type=int, default=3)
    ap.add_argument("--tile-words", type=int, default=1024,
                    help="slot-tiled plane layout (include/rabia_gpu.h); 0 = planar")
    ap.add_argument("--cpu-sample-windows", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_c2.json"))
    ap.add_argument("--config", choices=["c2", "c5"], default="c2",
                    help="c2: the headline (weak scaling, per-shard results exchanged); c5: 9 replicas x "
                         "2^26 slots per step split over the ranks (strong scaling) with the decision "
                         "bitmaps all-gathered every step")
    ap.add_argument("--c5-windows", type=int, default=64, help="C5: 2^20-slot windows per step, all ranks")
    return ap.parse_args()


def cpu_baseline(n: int, windows: int):
    """Structure-faithful REF path (oracle/rabia_oracle.c:or_ref_structured: per-slot
    NodeId->StateValue maps, one handler call per vote, PhaseData clone per read),
    single thread, on `windows` x 2^20 slots of the same trace kind."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    S = windows * WINDOW
    r1, r2, _ = O.trace(1, n, 42, 1, S)
    t0 = time.perf_counter()
    _, res = O.ref_structured(n, n // 2 + 1, n - 1, 42, 0, 1, r1, r2)
    dt = time.perf_counter() - t0
    return {"value": res["n_decided"] / dt, "unit": "slots decided/s", "cores": 1, "kind": "port",
            "sample": f"{S} slots ({windows} x 2^20 windows, agree90 trace, n={n}) through the "
                      f"structure-faithful REF restatement (oracle/rabia_oracle.c:or_ref_structured), "
                      f"1 thread, {dt:.2f} s"}


def load_pmc(path: str, n: int, slots: int):
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("replicas") == n and d.get("slots_per_launch") == slots:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def run_c5(a, world, rank, local, dist):
    """C5 (BASELINE.json configs[4]): 9 replicas, a 2^26-slot window per step split into
    equal contiguous shards (one per rank), REF sweep, then the streaming exchange: every
    rank extracts its committed + V1 bitmaps and all-gathers them and its step result
    (RCCL over xGMI) on the collective stream while the next step computes. After the
    timed loop the gathered rows are folded into the global commit watermark
    (rabia_amd/shard.py:combine) and checked against the per-shard counts."""
    from rabia_amd import shard
    n, T = 9, a.tile_words
    total = a.c5_windows * WINDOW
    start, S = shard.shard_range(total, world, rank, align=32 * (T or 4))
    assert S * world == total, "C5 needs equal shards"
    nw = S // 32
    stride = T if T else ((S + 127) // 128) * 4
    in_words = ((nw + T - 1) // T) * (4 * n + 1) * T if T else (4 * n + 1) * stride
    out_words = ((nw + T - 1) // T) * 8 * T if T else 8 * stride
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    ev = PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=42 + rank, device=local, tile_words=T)
    sets = []
    for i in range(a.sets):
        votes = torch.empty(in_words, dtype=torch.int32, device="cuda")
        out = torch.empty(out_words, dtype=torch.int32, device="cuda")
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 1000 * rank + i, 1 + start, S, stride, votes.data_ptr(), sp)
        sets.append((votes, out))
    n_total = a.warmup + a.steps
    res_dev = torch.zeros((n_total, 10), dtype=torch.int64, device="cuda")
    gathered = torch.zeros((n_total, world, 10), dtype=torch.int64, device="cuda")
    bm = torch.zeros((n_total, 2, nw), dtype=torch.int32, device="cuda")
    bm_all = torch.zeros((n_total, world, 2, nw), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    works = []

    def step(t):
        votes, out = sets[t % a.sets]
        base = 1 + t * total
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=base + start,
                            result_ptr=res_dev[t].data_ptr(), stream=sp)
        ev.decision_bitmap_async(out.data_ptr(), S, stride, bm[t, 0].data_ptr(), bm[t, 1].data_ptr(), sp)
        if dist is not None:
            works.append(dist.all_gather_into_tensor(gathered[t], res_dev[t], async_op=True))
            works.append(dist.all_gather_into_tensor(bm_all[t], bm[t], async_op=True))

    for t in range(a.warmup):
        step(t)
    for w in works:
        w.wait()
    works.clear()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_begin, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_begin.record(stream)
    for k in range(a.steps):
        step(a.warmup + k)
    for w in works:
        w.wait()
    t_end.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    total_ms = t_begin.elapsed_time(t_end)
    res = res_dev.cpu().numpy().view(np.uint64)
    if int(res[:, 9].max()) != 0:
        raise RuntimeError("device-side protocol fault flagged in a step result")
    g = gathered.cpu().numpy().view(np.uint64) if dist is not None else res[:, None, :]
    b_all = bm_all.cpu().numpy().view(np.uint32) if dist is not None else bm.cpu().numpy().view(np.uint32)[:, None]
    decided = 0
    for t in range(a.warmup, n_total):  # global commit per step, checked against the bitmaps
        rows = [shard.row_result(g[t, r]) for r in range(world)]
        starts = [shard.shard_range(total, world, r, align=32 * (T or 4))[0] for r in range(world)]
        gc = shard.combine(rows, [1 + t * total + s_ for s_ in starts], [S] * world, 1 + t * total, 1 + t * total)
        pop = int(np.unpackbits(b_all[t, :, 0].view(np.uint8)).sum())
        assert pop == gc.n_decided, (pop, gc.n_decided)
        decided += gc.n_decided
    tm = torch.tensor([total_ms], dtype=torch.float64, device="cuda")
    if dist is not None:
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    total_ms = float(tm[0])
    if rank == 0:
        bitmap_bytes = 2 * nw * 4 * world
        line = {
            "metric": "consensus slots decided/sec (9 replicas, 2^26 slots per step, bitmap all-gather)",
            "value": decided / (total_ms / 1000.0),
            "unit": "slots decided/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": total_ms / a.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u32 bit-sliced 2-bit vote codes (integer only)",
            "data": "synthetic (seeded agree90 vote trace generated on device)",
            "config": {"workload": f"C5: {n} replicas x {total} slots per step, REF sweep, committed + V1 "
                                   f"bitmaps ({bitmap_bytes} B per step in all) and step results all-gathered "
                                   f"every step, overlapped with the next step",
                       "replicas": n, "slots_per_step": total, "slots_per_gpu": S,
                       "layout": f"slot-tiled {T}" if T else "planar", "parallelism": f"slot-shard x{world}"},
        }
        print(json.dumps(line), flush=True)
    ev.close()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if a.config == "c5":
        run_c5(a, world, rank, local, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    n, G = a.replicas, a.windows
    S = G * WINDOW
    T = a.tile_words
    nw = S // 32
    if T:  # slot-tiled: the planes of each T-word slot tile are contiguous
        stride = T
        in_words = ((nw + T - 1) // T) * (4 * n + 1) * T
        out_words = ((nw + T - 1) // T) * 8 * T
    else:
        stride = ((S + 127) // 128) * 4
        in_words, out_words = (4 * n + 1) * stride, 8 * stride
    # A dedicated stream: the legacy default stream has handle 0, which the C ABI
    # reads as "the context's own stream"; events must sit on the launch stream.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0

    ev = PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=42 + rank, device=local, tile_words=T)
    sets = []
    for i in range(a.sets):
        votes = torch.empty(in_words, dtype=torch.int32, device="cuda")
        out = torch.empty(out_words, dtype=torch.int32, device="cuda")
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 1000 * rank + i, 1 + i * S, S, stride,
                                votes.data_ptr(), sp)
        sets.append((votes, out))
    n_total = a.warmup + a.steps
    res_dev = torch.zeros((n_total, 10), dtype=torch.int64, device="cuda")
    gathered = torch.zeros((n_total, world, 10), dtype=torch.int64, device="cuda") if world > 1 else None
    torch.cuda.synchronize()

    rank_base = 1 + rank * (1 << 40)  # disjoint slot-id range per shard
    works = []

    def step(t, evs=None):
        votes, out = sets[t % a.sets]
        if evs is not None:
            evs[0].record(stream)
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride,
                            slot_base=rank_base + t * S, result_ptr=res_dev[t].data_ptr(), stream=sp)
        if evs is not None:
            evs[1].record(stream)
        if dist is not None:  # global commit exchange, overlapped with the next step
            works.append(dist.all_gather_into_tensor(gathered[t], res_dev[t], async_op=True))

    for t in range(a.warmup):
        step(t)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]
    t_begin = torch.cuda.Event(enable_timing=True)
    t_end = torch.cuda.Event(enable_timing=True)
    t_begin.record(stream)
    for k in range(a.steps):
        step(a.warmup + k, evs[k])
    for w in works:
        w.wait()
    t_end.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    total_ms = t_begin.elapsed_time(t_end)
    kern_ms = [b.elapsed_time(e) for b, e in evs]
    res = res_dev.cpu().numpy().view(np.uint64)
    if int(res[:, 9].max()) != 0:
        raise RuntimeError("device-side protocol fault flagged in a step result")
    timed = res[a.warmup:]
    assert (timed[:, 0] == S).all(), "a timed step did not complete"
    decided_total = int(timed[:, 1].sum())
    if dist is not None:  # every shard's step results arrived through the exchange
        g = gathered.cpu().numpy().view(np.uint64)
        assert (g[a.warmup:, :, 0] == S).all()

    tmax = torch.tensor([total_ms, float(np.mean(kern_ms)), float(decided_total)], dtype=torch.float64,
                        device="cuda")
    if dist is not None:
        t_all = tmax.clone()
        dist.all_reduce(t_all[:2], op=dist.ReduceOp.MAX)
        dec_all = tmax[2:].clone()
        dist.all_reduce(dec_all, op=dist.ReduceOp.SUM)
        total_ms, kavg_ms, decided_all = float(t_all[0]), float(t_all[1]), float(dec_all[0])
    else:
        kavg_ms, decided_all = float(np.mean(kern_ms)), float(decided_total)

    # single-window (C2 one sweep) latency, untimed w.r.t. the headline
    sweep_us = None
    if rank == 0:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(stream)
        for i in range(reps):
            ev.phase_step_async(sets[i % a.sets][0].data_ptr(), sets[i % a.sets][1].data_ptr(), WINDOW,
                                stride, slot_base=1, stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        sweep_us = e0.elapsed_time(e1) * 1000.0 / reps

    if rank == 0:
        value = decided_all / (total_ms / 1000.0)
        alg_bytes = S * bytes_per_slot_ref(n)
        achieved = alg_bytes / (kavg_ms / 1000.0) / 1e9
        cpu = None if a.no_cpu_baseline else cpu_baseline(n, a.cpu_sample_windows)
        line = {
            "metric": "consensus slots decided/sec (5 replicas, 1M slots) + HBM GB/s as % of peak",
            "value": value,
            "unit": "slots decided/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": total_ms / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 bit-sliced 2-bit vote codes (integer only)",
            "data": "synthetic (seeded agree90 vote trace generated on device)",
            "config": {"workload": f"C2: {n} replicas x 2^20-slot windows, agree90 trace, REF single phase "
                                   f"sweep; {G} windows per step per GPU",
                       "replicas": n, "slots_per_window": WINDOW, "windows_per_step": G,
                       "slots_per_step_per_gpu": S, "mode": "ref", "layout": f"slot-tiled {T}" if T else "planar",
                       "parallelism": f"slot-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": load_pmc(a.pmc_file, n, S),
                         "alg_bytes_per_launch": alg_bytes, "kernel_avg_us": kavg_ms * 1000.0},
            "cpu_baseline": cpu,
            "sweep_1m_us": sweep_us,
        }
        print(json.dumps(line), flush=True)
    ev.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
