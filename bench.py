#!/usr/bin/env python3
"""Benchmark: consensus slots decided/sec on the batched Rabia phase evaluator.

Workload (BASELINE.json configs[1], "C2"): 5 replicas, windows of 2^20 slots,
90%-agreement synthetic vote trace, REF single phase sweep. One bench "step" is
one launch over `--windows` consecutive 2^20-slot windows per GPU (default 1024:
the steady-state streaming batch, 2^30 slots, 3.76 GB of planes per launch; a
launch carries ≈20 us of fixed ramp/drain/fold cost, so 256 windows run at 59 %,
512 at 62.5 %, 1024 at 64 %, 2048 at 65 % of the HBM peak; the
single-window latency is reported as `sweep_1m_us`). Inputs are generated on the device before the timed region and
rotate over 3 buffer sets (> 2x the 256 MiB Infinity Cache) so every step reads
from HBM.

Multi-GPU (torchrun, one rank per GPU): ONE engine — every rank holds the same
StdRng seed — over a global window of world x (windows x 2^20) slots per step,
rank r owning the r-th contiguous shard (weak scaling). The shard's REF step runs
with provisional draw positions and leaves draw records; the shard rows are
all-gathered over RCCL, each rank re-draws its VQ slots at their global stream
positions (rg_shard_fixup_async), the final rows are all-gathered again and folded
into every rank's engine state (rg_shard_commit_async). The exchange and fix-up
run on a second stream, so the step kernels of later windows never wait for them.
`--config c5`: 9 replicas x 2^26 slots per step split over the ranks (strong
scaling), decided/V1 bitmaps all-gathered every step as well.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the native library: shared HIP runtime)

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator, record_window_words  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
WINDOW = 1 << 20
SEED = 42  # RabiaConfig.randomization_seed of the one engine (integration_consensus.rs:404-408)


def bytes_per_slot_ref(n: int) -> float:
    """Algorithmic bytes per slot per REF phase evaluation:
    read R1 + R2 codes (4n bits), write 8 output bits."""
    return (4 * n + 8) / 8.0


C3_COIN_TABLE_PHASES = 8  # rabia_gpu.hip cluster_run: kCoinTablePhases (RG_COIN_TABLE_PHASES), held in LDS per workgroup


def c3_bytes_per_slot(n: int, mean_phases: float) -> float:
    """Bytes per slot of the call the C3 step makes, rg_wmvc_cluster_bitmaps_async (the
    decided / V1 bitmaps built inside the cluster kernel, no second pass over the info
    words): n initial-state bits read, the u32 info word written, 2 bitmap bits written.
    The common-coin bits of the first C3_COIN_TABLE_PHASES phases are computed into LDS by
    each workgroup (round 6; before, a coin-table launch wrote them to HBM and the kernel
    read them back), so they move no HBM bytes."""
    return n / 8 + 4 + 2 / 8


# SQ_INSTS_VALU / (512 x GRBM_GUI_ACTIVE / 8) that independent v_xor_b32 / v_add_u32 chains reach
# at 8 waves per SIMD (tools/valu_peak.hip under rocprofv3 --pmc, profiles/r06/valu_peak_counters.csv):
# the issue ceiling of 32-bit integer VALU work, below the 512-per-cycle issue figure
C3_INT_ISSUE_CEILING = 0.79


def c3_roofline(r, bytes_slot):
    """C3 is VALU-issue bound (per phase 2n keyed scheduler picks per slot + the coin),
    not HBM bound. achieved = VALU wave-instructions per launch (per-slot count from the
    SQ_INSTS_VALU pass of THIS round's kernel, profiles/pmc_c3.json, tools/pmc_c3.sh)
    / the live kernel time; peak = 256 CUs x 4 SIMDs x 1/2 wave64 instruction per cycle
    (a SIMD-32 issues a wave64 VALU instruction over 2 cycles, MI355X_MICROARCH.md "Wave
    scheduling") = 512 per cycle at the 2.4 GHz peak engine clock. The HBM fraction is
    kept beside it."""
    kern_s = r["kern_ms"] / 1000.0
    hbm = r["S"] * bytes_slot / kern_s / 1e9
    out = {"bound": "valu", "achieved": None, "peak": 512 * 2.4, "unit": "G VALU wave-instr/s", "frac": None,
           "traffic": None, "kernel_avg_us": r["kern_ms"] * 1000.0, "hbm_gbs": hbm, "hbm_frac": hbm / HBM_PEAK_GBS}
    path = os.path.join(ROOT, "profiles", "pmc_c3.json")
    if os.path.exists(path):
        pmc = json.load(open(path))
        achieved = pmc["valu_wave_instr_per_slot"] * r["S"] / kern_s / 1e9
        out.update(achieved=achieved, frac=achieved / out["peak"], counter_issue_util=pmc["valu_issue_util"],
                   counter_file="profiles/pmc_c3.json", measured_int_issue_ceiling=C3_INT_ISSUE_CEILING,
                   frac_of_measured_ceiling=pmc["valu_issue_util"] / C3_INT_ISSUE_CEILING,
                   note="achieved = the cluster kernel's VALU wave-instructions over the rg_wmvc_cluster_bitmaps_async call's "
                        "time (cluster kernel with its LDS coin table and the bitmaps + statistics fold: a lower bound for the kernel); "
                        "counter_issue_util = SQ_INSTS_VALU / (512 x GRBM_GUI_ACTIVE/8 cycles) of the cluster kernel "
                        "alone, at the clock the chip actually ran (DVFS); mix_per_slot in the counter file; "
                        "measured_int_issue_ceiling = the same ratio for independent 32-bit integer ALU chains at 8 waves "
                        "per SIMD (tools/valu_peak.hip, profiles/r06/valu_peak_counters.csv: v_xor / v_add 0.79, "
                        "v_mul_lo_u32 / v_bcnt 0.48)")
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run; without an external launcher (no WORLD_SIZE) N > 1 starts N "
                         "rank processes itself; under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=25)  # clocks settle over ~20 launches (tools/warm_probe.py)
    ap.add_argument("--windows", type=int, default=1024)
    ap.add_argument("--replicas", type=int, default=5)
    ap.add_argument("--sets", type=int, default=3)
    ap.add_argument("--launch-events", action="store_true",
                    help="an event pair around every timed launch (costs the stream 6-10 us per step)")
    ap.add_argument("--launch-sample", type=int, default=16,
                    help="sharded pipeline: an event pair around every n-th timed step kernel (its kernel "
                         "time; each pair costs the stream 6-10 us)")
    ap.add_argument("--tile-words", type=int, default=1024,
                    help="slot-tiled plane layout (include/rabia_gpu.h); 0 = planar")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-core CPU baseline (0: OMP_NUM_THREADS, else min(cpus, 16))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=None,
                    help="HBM traffic record (tools/pmc_traffic.py); default profiles/pmc_<config>[_sharded].json, "
                         "used when its replicas and slots per launch match the run's step launch")
    ap.add_argument("--c3-slots", type=int, default=1 << 24, help="C3: slots per step, all ranks")
    ap.add_argument("--config", choices=["c2", "c3", "c5"], default="c2",
                    help="c2: the headline (weak scaling); c5: 9 replicas x 2^26 slots per step split over the "
                         "ranks (strong scaling) with the decision bitmaps all-gathered every step")
    ap.add_argument("--c5-windows", type=int, default=64, help="C5: 2^20-slot windows per C5 window, all ranks")
    ap.add_argument("--c5-batch", type=int, default=32,
                    help="C5: consecutive C5 windows per step: one shard-step launch of K windows per rank (the "
                         "multi-window lag kernel from 2^28 slots per launch at n = 9), one K-window launch at N = 1")
    ap.add_argument("--c5-payload", choices=["lists", "lists-v1", "bitmaps"], default="lists",
                    help="C5 decided-slot payload per step: every rank's undecided-slot lists (the decided-slot "
                         "bitmaps' complement, ~0.04 %% of the slots at agree90; default: the state machine is sharded "
                         "with the slots, so a rank applies its own shard's V1 batches and needs only the global "
                         "decided set and watermark), the lists + every rank's V1 bitmap (every rank applies every "
                         "batch), or the round-5 committed + V1 bitmaps")
    ap.add_argument("--sharded", "--c5-sharded", dest="sharded", action="store_true",
                    help="N = 1: run the multi-GPU pipeline (shard step + fix-up + commit, exchanges with one "
                         "rank) instead of the single evaluator: the per-GPU cost of the N > 1 path")
    ap.add_argument("--fixup-stream", choices=["fix", "comp"], default="fix",
                    help="N > 1 / --sharded: the fix-up of step t on the second stream (overlapping step t + 1; "
                         "0.80 vs 0.81, 0.84 vs 0.86, 0.86 vs 0.88 ms per one-shard step in three round-4 "
                         "runs, profiles/r04_c2_sharded_n1*.json) or on the compute stream right behind step "
                         "t + 1's launch")
    ap.add_argument("--comp-priority", type=int, default=0, choices=[0, 1],
                    help="N > 1 / --sharded: the step kernels' stream at high priority (1) or default (0)")
    ap.add_argument("--fixup-eager", action="store_true",
                    help="N > 1 / --sharded: enqueue step t's exchange right after step t's launch (default: after "
                         "step t + 1's launch)")
    ap.add_argument("--diag", type=lambda x: int(x, 0), default=0,
                    help="rg_debug_set switches for experiments (include/rabia_gpu_debug.h); 0 = the product path")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI; gloo = several ranks on one GPU (rehearsal only)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1 only): the reference's Rust/Tokio path cannot run
# here (no toolchain), so three C restatements of it are timed on this host:
#   structure-faithful (per-slot NodeId->StateValue maps, one handler call per
#   vote, PhaseData clone per read: oracle/rabia_oracle.c:or_ref_structured),
#   1 thread and one independent engine instance per core; and the fast SoA
#   path (oracle/rabia_cpu_soa.c: bit-sliced, 64 slots per op, OpenMP) on all
#   cores over the same planes the GPU reads.
# ---------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def granted_cpus() -> dict:
    """The CPUs this process may actually run on: the affinity mask, capped by the
    cgroup CPU quota (cgroup v2 cpu.max, v1 cfs_quota/period) when one is set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    granted = aff if quota is None else max(1, min(aff, int(quota)))
    return {"granted": granted, "affinity": aff, "cgroup_quota": quota, "host_cpus": os.cpu_count()}


def cpu_threads(a) -> int:
    if a.cpu_threads > 0:
        return a.cpu_threads
    return granted_cpus()["granted"]


def cpu_baseline_c3(a, gpu_info) -> dict:
    """C3 CPU baseline: the C cluster restatement (oracle/rabia_oracle.c:or_wmvc_cluster,
    one replica set per slot, phases to termination) on all granted cores, one
    contiguous slot range per thread (ctypes drops the GIL), on the first slots of the
    GPU's own trace; checked against the GPU's per-slot info words."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    th = cpu_threads(a)
    n, S = 5, min(1 << 22, a.c3_slots)
    q, fp1 = n // 2 + 1, (n - 1) // 2 + 1
    states = O.cluster_trace(n, SEED, 1, S)
    chunks = np.array_split(np.arange(S), th)
    outs = [None] * th

    def run(i):
        lo, hi = int(chunks[i][0]), int(chunks[i][-1]) + 1
        outs[i] = O.wmvc_cluster(n, q, fp1, SEED, 1, 99, 32, 1 + lo, states[lo:hi])

    ts = [threading.Thread(target=run, args=(i,)) for i in range(th) if len(chunks[i])]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    info = np.concatenate([o for o in outs if o is not None])
    decided = int(((info & 0xFF) != 3).sum())  # dec code 3 (none) = not all replicas decided
    agree = bool(np.array_equal(info, gpu_info[:S]))
    g = granted_cpus()
    return {"value": decided / dt, "unit": "slots decided/s", "cores": th, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": g["host_cpus"], "granted_cpus": g["granted"],
            "affinity_cpus": g["affinity"], "cgroup_quota_cpus": g["cgroup_quota"],
            "sample": f"C cluster restatement (oracle/rabia_oracle.c:or_wmvc_cluster), {th} threads over the "
                      f"first {S} slots of the GPU's adversarial trace (n=5, <= 32 phases): {dt:.3f} s; "
                      f"per-slot info words equal the GPU's: {agree}"}


def cpu_baseline(a, n: int, r: dict) -> dict:
    """CPU legs on the GPU box's host cores, rank 0, N = 1. The reported value is the
    SoA all-core path (oracle/rabia_cpu_soa.c) over the input planes of the bench's own
    set 0, and its outputs are checked bit for bit against the GPU's output of the last
    TIMED step that read set 0 (the kernel the headline times: the persistent lag
    kernel at the C2 shape), from that step's engine position (StdRng draw index,
    last_committed, watermark: the previous step's result)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    th = cpu_threads(a)
    q, lane = n // 2 + 1, n - 1
    # (1) structure-faithful, one thread
    S1 = 4 * WINDOW
    r1, r2, _ = O.trace(1, n, SEED, 1, S1)
    t0 = time.perf_counter()
    _, res = O.ref_structured(n, q, lane, SEED, 0, 1, r1, r2)
    dt1 = time.perf_counter() - t0
    sf1 = res["n_decided"] / dt1
    # (2) structure-faithful, one engine instance per core (ctypes drops the GIL)
    out = [0.0] * th

    def inst(i):
        t = time.perf_counter()
        _, rr = O.ref_structured(n, q, lane, SEED + i, 0, 1, r1, r2)
        out[i] = (rr["n_decided"], time.perf_counter() - t)

    ts = [threading.Thread(target=inst, args=(i,)) for i in range(th)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dtp = time.perf_counter() - t0
    sfp = sum(x[0] for x in out) / dtp
    # (3) SoA all cores over set 0's planes (planar copy of the slot-tiled buffer)
    S, T, P = r["S"], r["T"], 4 * n + 1
    nw = (S + 31) // 32
    votes, gout = r["sets"][0]
    res_all = r["res"]
    t_last = ((a.warmup + a.steps - 1) // a.sets) * a.sets  # the last step that read set 0
    prev = res_all[t_last - 1] if t_last else None
    rng0 = int(prev[7]) if prev is not None else 0
    lc0 = int(prev[5]) if prev is not None else 0
    wm0 = int(prev[8]) if prev is not None else 1
    base = 1 + t_last * S
    torch.cuda.synchronize()
    if T:
        tiles = (nw + T - 1) // T
        host = votes.view(tiles, P, T).permute(1, 0, 2).reshape(P, tiles * T).cpu().numpy().view(np.uint32)
        g_out = gout.view(tiles, 8, T).permute(1, 0, 2).reshape(8, tiles * T).cpu().numpy().view(np.uint32)
        stride = tiles * T
    else:
        stride = r["stride"]
        host = votes.view(P, stride).cpu().numpy().view(np.uint32)
        g_out = gout.view(8, stride).cpu().numpy().view(np.uint32)
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        s_out, sres = O.ref_step_soa(n, q, lane, SEED, rng0, base, host, stride, S, 0, lc0, wm0, threads=th)
        times.append(time.perf_counter() - t0)
    dt3 = float(np.median(times))
    soa = sres["n_decided"] / dt3
    gres = dict(zip(N.RESULT_FIELDS, [int(x) for x in res_all[t_last]]))
    keys = ("n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max", "first_undecided",
            "rng_next", "commit_watermark")
    agree_res = all(sres[k] == gres[k] for k in keys)
    agree_out = bool(np.array_equal(s_out[:, :nw], g_out[:, :nw]))
    g = granted_cpus()
    return {"value": soa, "unit": "slots decided/s", "cores": th, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": g["host_cpus"], "granted_cpus": g["granted"],
            "affinity_cpus": g["affinity"], "cgroup_quota_cpus": g["cgroup_quota"],
            "sample": f"SoA all-core path (oracle/rabia_cpu_soa.c, {th} OpenMP threads) over the bench's set-0 "
                      f"input ({S} slots, n={n}, agree90), median of 5 = {dt3:.3f} s, from the engine position of "
                      f"timed step {t_last}; its 8 output planes equal that GPU step's bit for bit: {agree_out}; "
                      f"step results equal: {agree_res}",
            "gpu_agrees": agree_out and agree_res,
            "structure_faithful_1t": {"value": sf1, "slots": S1, "seconds": dt1},
            "structure_faithful_per_core": {"value": sfp, "instances": th, "slots_each": S1, "seconds": dtp},
            "soa_all_cores": {"value": soa, "threads": th, "slots": S, "seconds": dt3, "gpu_step": t_last,
                              "outputs_equal": agree_out, "results_equal": agree_res}}


def load_pmc(path: str, n: int, slots: int):
    """HBM bytes per launch from a committed PMC record of this launch size: the file holds
    one record, or {"records": [...]} for several launch sizes."""
    try:
        with open(path) as f:
            d = json.load(f)
        for rec in d.get("records", [d]):
            if rec.get("replicas") == n and rec.get("slots_per_launch") == slots:
                return rec.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def launch_events(a, every=0):
    """Per-launch timing events inside the timed region. An event recorded between two step
    kernels puts a barrier packet in the stream: 6-10 us per step between back-to-back
    2^30-slot steps (tools/gap_probe.py, profiles/r05/gap_probe.json). --launch-events: a
    pair around every launch. Otherwise, every > 0 (the sharded pipeline, whose step time
    also holds the exchange): a pair around every every-th launch only; every = 0 (the
    single evaluator, steps back to back): none, and the average launch duration is the
    span / K (it includes the launch gaps: an upper bound on the kernel time, which the
    committed rocprofv3 summaries sit just below)."""
    def pair():
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.launch_events:
        return [pair() for _ in range(a.steps)]
    if every:
        return [pair() if k % every == 0 else None for k in range(a.steps)]
    return None


def launch_ms(evs, total_ms, steps):
    timed = [p for p in (evs or []) if p is not None]
    if timed:
        return float(np.mean([b.elapsed_time(e) for b, e in timed]))
    return total_ms / steps


def layout(n, S, T):
    nw = (S + 31) // 32
    if T:  # slot-tiled: the planes of each T-word slot tile are contiguous
        return T, ((nw + T - 1) // T) * (4 * n + 1) * T, ((nw + T - 1) // T) * 8 * T
    stride = ((S + 127) // 128) * 4
    return stride, (4 * n + 1) * stride, 8 * stride


# ---------------------------------------------------------------------------
# one GPU: the single evaluator
# ---------------------------------------------------------------------------
def run_single(a, n, S, label):
    T = a.tile_words
    stride, in_words, out_words = layout(n, S, T)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    ev = PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=SEED, tile_words=T, device=torch.cuda.current_device())
    if a.diag:
        N.check(ev.lib.rg_debug_set(ev.ctx, a.diag), ev.ctx)
    sets = []
    for i in range(a.sets):
        votes = torch.empty(in_words, dtype=torch.int32, device="cuda")
        out = torch.empty(out_words, dtype=torch.int32, device="cuda")
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 1000 + i, 1 + i * S, S, stride, votes.data_ptr(), sp)
        sets.append((votes, out))
    n_total = a.warmup + a.steps
    res_dev = torch.zeros((n_total, 10), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step(t, evs=None):
        votes, out = sets[t % a.sets]
        if evs is not None:
            evs[0].record(stream)
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=1 + t * S,
                            result_ptr=res_dev[t].data_ptr(), stream=sp)
        if evs is not None:
            evs[1].record(stream)

    for t in range(a.warmup):
        step(t)
    torch.cuda.synchronize()
    evs = launch_events(a)
    t_begin, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_begin.record(stream)
    for k in range(a.steps):
        step(a.warmup + k, evs[k] if evs else None)
    t_end.record(stream)
    torch.cuda.synchronize()
    total_ms = t_begin.elapsed_time(t_end)
    kern_ms = launch_ms(evs, total_ms, a.steps)
    res = res_dev.cpu().numpy().view(np.uint64)
    if int(res[:, 9].max()) != 0:
        raise RuntimeError("device-side protocol fault flagged in a step result")
    timed = res[a.warmup:]
    assert (timed[:, 0] == S).all(), "a timed step did not complete"
    decided = int(timed[:, 1].sum())
    launch = ev.last_launch()  # the timed steps' kernel shape
    sweep_us = None
    if label == "c2":  # single-window (C2 one sweep) latency, outside the headline
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        w_out = torch.empty(layout(n, WINDOW, T)[2], dtype=torch.int32, device="cuda")  # the sets' outputs stay
        e0.record(stream)
        for i in range(reps):
            ev.phase_step_async(sets[i % a.sets][0].data_ptr(), w_out.data_ptr(), WINDOW, stride, slot_base=1,
                                stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        sweep_us = e0.elapsed_time(e1) * 1000.0 / reps
    return {"total_ms": total_ms, "kern_ms": kern_ms, "decided": decided, "sweep_us": sweep_us, "ev": ev,
            "stream": stream, "sets": sets, "res": res, "S": S, "T": T, "stride": stride, "launch": launch}


# ---------------------------------------------------------------------------
# N GPUs: one engine over a window split into contiguous shards
# ---------------------------------------------------------------------------
def make_gather(dist, backend):
    """all_gather of one row/bitmap per rank into out[world, ...], enqueued on the
    current stream (RCCL); "gloo" is a one-GPU rehearsal through host copies."""
    if backend == "nccl":
        return lambda out, inp: dist.all_gather_into_tensor(out, inp, async_op=True).wait()

    def gather(out, inp):
        torch.cuda.current_stream().synchronize()
        parts = [torch.empty_like(inp, device="cpu") for _ in range(out.shape[0])]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.stack(parts))
    return gather


def run_sharded(a, n, S, window_slots, world, rank, dist, comm, bitmaps):
    """One engine over windows split into `world` contiguous shards. A step is K =
    a.c5_batch consecutive windows: every rank's shard step runs the K windows' shards
    in ONE launch (rg_phase_step_shard_windows_async; K = 1: rg_phase_step_shard_async),
    then per window: rows all-gathered, fix-up, final rows all-gathered, commit, and
    (C5) the committed/V1 bitmaps all-gathered, on a second stream. world = 1 runs the
    same pipeline with one shard (the 1-GPU measurement of a shard-size step).
    comm (RCCL, the product path): stages 2-4 and the bitmaps are one C-ABI call per step,
    rg_shard_exchange_windows_async, whose all-gathers run on the device stream through
    the context's communicator; no torch.distributed collective. dist (gloo): the
    one-GPU rehearsal through host copies."""
    T = a.tile_words
    K = max(1, a.c5_batch) if a.config == "c5" else 1  # C2: one 2^30-slot shard per rank, as at N = 1
    gather = (None if comm is not None else
              make_gather(dist, a.backend) if world > 1 else (lambda out, inp: out.copy_(inp.unsqueeze(0))))
    stride, in_words, out_words = layout(n, S, T)
    # the step kernels' stream at high priority: when a step kernel ends, the exchange
    # kernels it releases and the next step kernel race for the freed CUs
    comp = torch.cuda.Stream(priority=-1) if a.comp_priority else torch.cuda.Stream()
    fix = torch.cuda.Stream()
    torch.cuda.set_stream(comp)
    # one seed on every rank; the context on this rank's GPU (main: torch.cuda.set_device(LOCAL_RANK))
    ev = PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=SEED, tile_words=T, device=torch.cuda.current_device())
    if comm is not None:
        comm.attach(ev)
    if a.diag:
        N.check(ev.lib.rg_debug_set(ev.ctx, a.diag), ev.ctx)
    cap = max(S // 8, 1 << 16)  # draw records per shard window (agree90: ~1 % of slots are VQ); overflow -> flags
    sets = []
    start = rank * S
    for i in range(a.sets):
        votes = torch.empty(K * in_words, dtype=torch.int32, device="cuda")
        out = torch.empty(K * out_words, dtype=torch.int32, device="cuda")
        rec = torch.empty(K * record_window_words(S, cap), dtype=torch.int32, device="cuda")  # draw-record regions
        for k in range(K):
            ev.trace_generate_async(N.RG_TRACE_AGREE90, 1000 + i * K + k, 1 + (i * K + k) * window_slots + start, S,
                                    stride, votes.data_ptr() + 4 * k * in_words, comp.cuda_stream)
        sets.append((votes, out, rec))
    n_total = a.warmup + a.steps
    i64 = dict(dtype=torch.int64, device="cuda")
    rows = torch.zeros((n_total, K, 10), **i64)
    g_rows = torch.zeros((n_total, world, K, 10), **i64)  # rank-major: one all-gather of every rank's K rows
    fixed = torch.zeros((n_total, K, 10), **i64)
    g_fixed = torch.zeros((n_total, world, K, 10), **i64)
    result = torch.zeros((n_total, K, 10), **i64)
    nw = (S + 31) // 32
    # C5 payload: undecided lists (cap per window; count > cap flags the window, 32) + V1 bitmaps
    lists = bitmaps and a.c5_payload != "bitmaps"
    und_cap = max(S // 512, 1024)  # agree90: ~0.04 % of a shard's slots are undecided
    P = K * (1 + und_cap) + (K * nw if a.c5_payload == "lists-v1" else 0)
    if comm is not None:  # the exchange scratch (rows; C5: the decided-slot payload) sized before the pipeline
        comm.reserve(ev, K, S if bitmaps else 1, und_cap)
    if bitmaps and not lists:
        bm = torch.zeros((n_total, K, 2, nw), dtype=torch.int32, device="cuda")
        bm_all = torch.zeros((n_total, world, K, 2, nw), dtype=torch.int32, device="cuda")
    elif lists:
        if comm is None:
            raise SystemExit("bench.py: --c5-payload lists runs through the C ABI's communicator (--backend nccl)")
        dec_all = torch.zeros((n_total, world, P), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e_main = [torch.cuda.Event() for _ in range(n_total)]
    e_rows = [torch.cuda.Event() for _ in range(n_total)]
    e_fixed = [torch.cuda.Event() for _ in range(n_total)]
    e_done = [torch.cuda.Event() for _ in range(n_total)]
    # the fix-up of step t: on the second stream, overlapping step t + 1's launch, or on the
    # compute stream right behind step t + 1's launch (no competition for the CUs)
    fix_on_comp = a.fixup_stream == "comp"
    # submission order: the exchange of step t is enqueued after step t + 1's launch (the
    # default), so step t + 1's kernel never sits behind step t's exchange in a hardware
    # queue the two streams may share (GPU_MAX_HW_QUEUES = 4 for every stream of the process)
    defer = fix_on_comp or not a.fixup_eager
    fs_main = comp if fix_on_comp else fix

    def shard_step(votes, out, rec, base, t):
        if K == 1:
            ev.phase_step_shard_async(votes.data_ptr(), out.data_ptr(), S, stride, base + start, rec.data_ptr(), cap,
                                      rows[t, 0].data_ptr(), stream=comp.cuda_stream)
        else:
            ev.phase_step_shard_windows_async(K, votes.data_ptr(), in_words, out.data_ptr(), out_words, S, stride,
                                              base + start, window_slots, rec.data_ptr(), cap, rows[t].data_ptr(),
                                              stream=comp.cuda_stream)

    # comm (the product path): the compute stream carries the step kernels and one event per
    # step (the exchange's dependency); the host waits for step t - sets' exchange before it
    # reuses that step's buffers (the host runs ahead of the device by less than `sets` steps),
    # so the compute queue holds no cross-stream wait. Every packet between two step kernels
    # costs the stream 6-10 us (an event record 7, a one-thread kernel 6, a wait 5-6:
    # tools/gap_probe.py, profiles/r05/gap_probe.json); back-to-back step kernels cost 0.

    host_wait = [0.0]  # host time blocked on e_done (the rest of the loop is enqueue work)

    def step(t, evs=None, chain=True):
        votes, out, rec = sets[t % a.sets]
        base = 1 + t * K * window_slots
        if t >= a.sets:  # the output buffers and records of step t - sets must be fixed up first
            if comm is not None:
                w0 = time.perf_counter()
                e_done[t - a.sets].synchronize()
                host_wait[0] += time.perf_counter() - w0
            else:
                comp.wait_event(e_done[t - a.sets])
        if evs is not None:
            evs[0].record(comp)
        if a.backend == "gloo" and world > 1:
            # Rehearsal: the ranks share one GPU, and two tiled-kernel look-back launches
            # of different processes running at once on one GPU can wait on each other
            # across kernels (include/rabia_gpu.h). Real runs have one GPU per rank. So
            # the ranks' step kernels take turns here.
            for r in range(world):
                if r == rank:
                    shard_step(votes, out, rec, base, t)
                    comp.synchronize()
                dist.barrier()
        else:
            shard_step(votes, out, rec, base, t)
        if evs is not None:
            evs[1].record(comp)
        e_main[t].record(comp)
        if comm is None:
            with torch.cuda.stream(fix):  # the rows' all-gather
                fix.wait_event(e_main[t])
                gather(g_rows[t], rows[t])
                e_rows[t].record(fix)
        if not defer:
            later(t, fix)
        elif chain and t >= 1:  # the previous step's exchange behind this step's launch
            later(t - 1, fs_main)

    def later(t, fs_stream):
        """Stages 3-4 of step t (+ C5 bitmaps): the fix-up on fs_stream, the final rows'
        all-gather, the commit and the bitmaps on the second stream."""
        votes, out, rec = sets[t % a.sets]
        base = 1 + t * K * window_slots
        if comm is not None:  # stages 2-4 + bitmaps: one C-ABI call, RCCL on the device stream
            fs_stream.wait_event(e_main[t])
            if lists:
                ev.shard_exchange_decisions_async(K, out.data_ptr(), out_words, S, stride, base + start, base,
                                                  window_slots, rec.data_ptr(), cap, rows[t].data_ptr(),
                                                  result[t].data_ptr(), und_cap, dec_all[t].data_ptr(),
                                                  with_v1=a.c5_payload == "lists-v1", stream=fs_stream.cuda_stream)
            else:
                ev.shard_exchange_windows_async(K, out.data_ptr(), out_words, S, stride, base + start, base,
                                                window_slots, rec.data_ptr(), cap, rows[t].data_ptr(),
                                                result[t].data_ptr(), bm_all[t].data_ptr() if bitmaps else 0,
                                                stream=fs_stream.cuda_stream)
            e_done[t].record(fs_stream)
            return
        fs_stream.wait_event(e_rows[t])
        ev.shard_fixup_windows_async(K, out.data_ptr(), out_words, S, stride, base + start, window_slots,
                                     rec.data_ptr(), cap, g_rows[t].data_ptr(), rank, world,
                                     fixed[t].data_ptr(), stream=fs_stream.cuda_stream)
        e_fixed[t].record(fs_stream)
        with torch.cuda.stream(fix):
            fix.wait_event(e_fixed[t])
            fs = fix.cuda_stream
            gather(g_fixed[t], fixed[t])
            ev.shard_commit_windows_async(K, g_fixed[t].data_ptr(), world, base, window_slots, result[t].data_ptr(),
                                          stream=fs)
            if bitmaps:
                ev.decision_bitmap_windows_async(K, out.data_ptr(), out_words, S, stride, bm[t, 0, 0].data_ptr(),
                                                 bm[t, 0, 1].data_ptr(), 2 * nw, stream=fs)
                gather(bm_all[t], bm[t])
            e_done[t].record(fix)

    def barrier():
        if comm is not None:
            ev.comm_barrier()
        elif dist is not None:
            dist.barrier()

    for t in range(a.warmup):
        step(t)
    if defer and a.warmup:
        later(a.warmup - 1, fs_main)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    evs = launch_events(a, every=max(1, a.launch_sample))  # the step kernel alone, sampled (the step time holds the exchange too)
    t_begin, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_begin.record(comp)
    host_wait[0] = 0.0
    h0 = time.perf_counter()
    for k in range(a.steps):  # (the warm-up's last fix-up is done: the timed chain starts afresh)
        step(a.warmup + k, evs[k] if evs else None, chain=k > 0)
    if defer:
        later(n_total - 1, fs_main)
    comp.wait_event(e_done[n_total - 1])
    t_end.record(comp)
    host_ms = (time.perf_counter() - h0) * 1000.0  # the host's enqueue time (it may block on e_done waits)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    total_ms = t_begin.elapsed_time(t_end)
    kern_ms = launch_ms(evs, total_ms, a.steps)
    res = result.reshape(-1, 10).cpu().numpy().view(np.uint64)
    fx = fixed.reshape(-1, 10).cpu().numpy().view(np.uint64)
    if int(res[:, 9].max()) != 0 or int(fx[:, 9].max()) != 0:
        raise RuntimeError("device-side fault flagged in a step result (1/2 look-back/fold timeout, 4 stale record "
                           f"ring, 8 draw-record overflow): result flags {sorted(set(res[:, 9].tolist()))}, shard "
                           f"flags {sorted(set(fx[:, 9].tolist()))}, rows flags "
                           f"{sorted(set(rows.reshape(-1, 10).cpu().numpy().view(np.uint64)[:, 9].tolist()))}")
    timed = res[a.warmup * K:]
    assert (timed[:, 0] == window_slots).all(), "a timed window did not complete"
    decided = int(timed[:, 1].sum())  # global (every shard), identical on every rank
    if bitmaps and not lists:  # the gathered committed bitmaps carry exactly the folded decided count
        b_all = bm_all[a.warmup:].cpu().numpy().view(np.uint32)
        pop = int(np.unpackbits(b_all[:, :, :, 0].view(np.uint8)).sum())
        assert pop == decided, (pop, decided)
    elif lists:  # the gathered undecided lists count exactly the slots the folded rows left undecided
        heads = dec_all[a.warmup:, :, :K * (1 + und_cap)].reshape(a.steps, world, K, 1 + und_cap)[..., 0]
        und = int(heads.cpu().numpy().view(np.uint32).astype(np.int64).sum())
        assert und == a.steps * K * window_slots - decided, (und, decided)
    if comm is not None and world > 1:
        total_ms, kern_ms = ev.comm_max([total_ms, kern_ms])
    elif dist is not None:
        tm = torch.tensor([total_ms, kern_ms], dtype=torch.float64, device="cuda" if a.backend == "nccl" else "cpu")
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        total_ms, kern_ms = float(tm[0]), float(tm[1])
    payload = None
    if bitmaps:  # decided-slot payload bytes all-gathered per step (every rank's share)
        payload = {"kind": a.c5_payload, "bytes_per_step": world * (P if lists else K * 2 * nw) * 4,
                   "undecided_cap": und_cap if lists else None}
    return {"total_ms": total_ms, "kern_ms": kern_ms, "decided": decided, "sweep_us": None, "ev": ev,
            "stream": comp, "windows_per_launch": K, "launch": ev.last_launch(), "sharded": True,
            "payload": payload, "host_ms_per_step": host_ms / a.steps,
            "host_enqueue_ms_per_step": (host_ms - host_wait[0] * 1000.0) / a.steps}


# ---------------------------------------------------------------------------
# C3 (BASELINE.json configs[2]): 5 replicas x 2^24 slots, adversarial split,
# Weak-MVC to termination with the common coin, sharded over the GPUs. The coin is
# keyed by the GLOBAL slot id, so the shards need no data-path exchange; the
# per-shard statistics and decided/V1 bitmaps are all-gathered every step.
# ---------------------------------------------------------------------------
def run_c3(a, world, rank, dist, comm):
    from rabia_amd import shard
    n, total = 5, a.c3_slots
    start, S = shard.shard_range(total, world, rank, align=128)
    stride = ((S + 127) // 128) * 4
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    ev = PhaseEvaluator(n, mode="wmvc", coin_seed=SEED, epoch=1, device=torch.cuda.current_device())
    if comm is not None:
        comm.attach(ev)
    states = torch.empty(n * stride, dtype=torch.int32, device="cuda")
    info = torch.empty(max(S, 1), dtype=torch.int32, device="cuda")
    nw = (S + 31) // 32
    n_total = a.warmup + a.steps
    stats = torch.zeros((n_total, 8), dtype=torch.int64, device="cuda")
    bm = torch.zeros((n_total, 2, nw), dtype=torch.int32, device="cuda")
    g_stats = torch.zeros((n_total, world, 8), dtype=torch.int64, device="cuda")
    g_bm = torch.zeros((n_total, world, 2, nw), dtype=torch.int32, device="cuda")
    ev.cluster_trace_async(SEED, 1 + start, S, stride, states.data_ptr(), sp)
    torch.cuda.synchronize()
    if world == 1:
        gather = None
    elif comm is not None:  # RCCL through the C ABI, on the step's stream
        def gather(out, inp):
            ev.comm_allgather_async(inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size(), sp)
    else:
        gather = make_gather(dist, a.backend)
    kern = []

    def step(t, evs=None):
        if evs is not None:
            evs[0].record(stream)
        # the cluster run with its decided / V1 bitmaps built in the cluster kernel
        ev.wmvc_cluster_bitmaps_async(states.data_ptr(), stride, S, 1 + start, 99, 32, info.data_ptr(),
                                      bm[t, 0].data_ptr(), bm[t, 1].data_ptr(), stats[t].data_ptr(), sp)
        if evs is not None:
            evs[1].record(stream)
        if gather is not None:
            gather(g_stats[t], stats[t])
            gather(g_bm[t], bm[t])

    def barrier():
        if comm is not None:
            ev.comm_barrier()
        elif dist is not None:
            dist.barrier()

    for t in range(a.warmup):
        step(t)
    torch.cuda.synchronize()
    barrier()
    # the cluster call (cluster kernel with the bitmaps, statistics fold): at world 1
    # it is the whole step (span / K); with the all-gathers in the step, every 2nd call bracketed
    evs = launch_events(a, every=2 if world > 1 else 0)
    t_begin, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_begin.record(stream)
    for k in range(a.steps):
        step(a.warmup + k, evs[k] if evs else None)
    t_end.record(stream)
    torch.cuda.synchronize()
    barrier()
    total_ms = t_begin.elapsed_time(t_end)
    kern_ms = launch_ms(evs, total_ms, a.steps)
    rows = (g_stats if world > 1 else stats[:, None, :]).cpu().numpy().view(np.uint64)
    decided = 0
    for t in range(a.warmup, n_total):
        g = shard.combine_cluster(rows[t].tolist())
        assert g["slots"] == total
        decided += g["all_decided"]
        if world > 1:  # the gathered decided bitmaps carry the folded count
            pop = int(np.unpackbits(g_bm[t, :, 0].cpu().numpy().view(np.uint8)).sum())
            assert pop == g["all_decided"], (pop, g["all_decided"])
    if comm is not None and world > 1:
        total_ms, kern_ms = ev.comm_max([total_ms, kern_ms])
    elif dist is not None:
        tm = torch.tensor([total_ms, kern_ms], dtype=torch.float64, device="cuda" if a.backend == "nccl" else "cpu")
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        total_ms, kern_ms = float(tm[0]), float(tm[1])
    last = shard.combine_cluster(rows[n_total - 1].tolist())
    return {"total_ms": total_ms, "kern_ms": kern_ms, "decided": decided, "ev": ev, "S": S, "total": total,
            "mean_phases": last["sum_phases"] / max(last["all_decided"], 1), "max_phases": last["max_phases"],
            "info": info}


def spawn_ranks(a) -> int:
    """--gpus N > 1 without an external launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them,
    rendezvous on 127.0.0.1) before this process touches the GPU; returns the worst
    exit code. A rank that fails ends the others (they would wait in a collective)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 128 - code)
                for o in live:
                    o.kill()
        time.sleep(0.2)
    return rc


def json_stdout():
    """The one JSON line goes to the process's original stdout; everything written to fd 1
    after this (native libraries: RCCL prints a version banner when a communicator is
    created) goes to stderr, so stdout carries exactly the line."""
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(spawn_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    out = json_stdout()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.backend == "gloo":  # rehearsal: ranks may share the box's one GPU
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist = comm = None
    if world > 1 and a.backend == "gloo":  # one-GPU rehearsal: host copies over gloo
        import torch.distributed as dist
        dist.init_process_group("gloo")
    elif world > 1 or a.sharded:  # RCCL through the C ABI (rg_comm_*); the id travels by the launcher's store
        from rabia_amd.shard import RcclComm
        comm = RcclComm(rank, world)
    if a.config == "c3":
        r = run_c3(a, world, rank, dist, comm)
        if rank == 0:
            # bytes the cluster call moves per slot (c3_bytes_per_slot); the kernel is VALU-bound
            # (per phase: 2n keyed scheduler hashes per slot), so this is not a roofline claim
            bytes_slot = c3_bytes_per_slot(5, r["mean_phases"])
            line = {
                "metric": "consensus slots decided/sec (5 replicas, 2^24 slots, adversarial split, "
                          "Weak-MVC to termination)",
                "value": r["decided"] / (r["total_ms"] / 1000.0), "unit": "slots decided/s", "n_gpus": world,
                "steps": a.steps, "warmup": a.warmup, "ms_per_step": r["total_ms"] / a.steps,
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "u32 replica bit masks (integer only)",
                "data": "synthetic (adversarial split initial states generated on device)",
                "config": {"workload": f"C3: 5 replicas x {r['total']} slots, every replica of every slot runs "
                                       f"Weak-MVC phases (f+1 decide, common coin) until all decided (<= 32)",
                           "replicas": 5, "slots_per_step": r["total"], "slots_per_gpu": r["S"],
                           "mean_phases": r["mean_phases"], "max_phases": r["max_phases"],
                           "parallelism": f"slot-shard x{world}, stats + decided bitmaps all-gathered"},
                "roofline": c3_roofline(r, bytes_slot),
                "cpu_baseline": (None if (a.no_cpu_baseline or world > 1)
                                 else cpu_baseline_c3(a, r["info"].cpu().numpy().view(np.uint32))),
                "sweep_1m_us": None,
            }
            print(json.dumps(line), file=out, flush=True)
        r["ev"].close()
        if dist is not None:
            dist.destroy_process_group()
        return
    if a.config == "c5":
        n, window_slots = 9, a.c5_windows * WINDOW
        assert window_slots % (world * 32 * (a.tile_words or 4)) == 0, "C5 needs equal tile-aligned shards"
        S = window_slots // world
    else:
        n, S = a.replicas, a.windows * WINDOW
        window_slots = S * world
    if world == 1 and not a.sharded:
        if a.config == "c5":  # the N = 1 stream: K consecutive C5 windows per launch (one engine, ascending
            # slot order: the same outputs and engine state as K one-window launches)
            r = run_single(a, n, max(1, a.c5_batch) * S, a.config)
            r["windows_per_launch"] = max(1, a.c5_batch)
        else:
            r = run_single(a, n, S, a.config)
    else:
        r = run_sharded(a, n, S, window_slots, world, rank, dist, comm, bitmaps=a.config == "c5")
    K = r.get("windows_per_launch", 1)
    if rank == 0:
        value = r["decided"] / (r["total_ms"] / 1000.0)
        alg_bytes = K * S * bytes_per_slot_ref(n)
        achieved = alg_bytes / (r["kern_ms"] / 1000.0) / 1e9
        cpu = (None if (a.no_cpu_baseline or world > 1 or "sets" not in r or a.config != "c2")
               else cpu_baseline(a, n, r))
        sharded = r.get("sharded", False)
        par = f"slot-shard x{world}" + (
            (f", one engine: sharded draws + fix-up, {K} C5 windows per shard launch" if a.config == "c5" else
             ", one engine: each rank's 2^30-slot shard at provisional draws, shard rows all-gathered, VQ slots "
             "re-drawn at their global positions, final rows all-gathered and folded") if sharded else "")
        if a.config == "c5":
            metric = "consensus slots decided/sec (9 replicas, 2^26 slots per step, decided-slot all-gather)"
            carried = {"lists": "undecided-slot lists", "lists-v1": "undecided-slot lists + V1 bitmaps",
                       "bitmaps": "committed + V1 bitmaps"}[a.c5_payload]
            workload = (f"C5: {n} replicas x {window_slots}-slot windows, {K} per step (one engine), REF sweep "
                        f"split over {world} GPU(s)" + (f", shard rows and {carried} all-gathered every step"
                                                        if sharded else ""))
            scaling = "strong"
        else:
            metric = "consensus slots decided/sec (5 replicas, 1M slots) + HBM GB/s as % of peak"
            workload = (f"C2: {n} replicas x 2^20-slot windows, agree90 trace, REF single phase sweep; "
                        f"{a.windows} windows per step per GPU, one engine over all GPUs' windows")
            scaling = "weak"
        line = {
            "metric": metric,
            "value": value,
            "unit": "slots decided/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": r["total_ms"] / a.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32 bit-sliced 2-bit vote codes (integer only)",
            "data": "synthetic (seeded agree90 vote trace generated on device)",
            "config": {"workload": workload, "replicas": n, "slots_per_window": WINDOW,
                       "slots_per_step_per_gpu": K * S, "slots_per_step": K * window_slots, "mode": "ref",
                       "layout": f"slot-tiled {a.tile_words}" if a.tile_words else "planar", "parallelism": par},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": load_pmc(a.pmc_file or os.path.join(
                             ROOT, "profiles", f"pmc_{a.config}{'_sharded' if sharded else ''}.json"), n, K * S),
                         "alg_bytes_per_launch": alg_bytes, "kernel_avg_us": r["kern_ms"] * 1000.0,
                         "kernel": r["launch"]},
            "cpu_baseline": cpu,
            "sweep_1m_us": r["sweep_us"],
        }
        if r.get("payload"):
            line["config"]["payload"] = r["payload"]
        if r.get("host_ms_per_step") is not None:  # the pipeline's host time per step (rank 0): all,
            line["host_ms_per_step"] = r["host_ms_per_step"]  # and without the waits for buffer reuse
            line["host_enqueue_ms_per_step"] = r["host_enqueue_ms_per_step"]
        print(json.dumps(line), file=out, flush=True)
    r["ev"].close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
