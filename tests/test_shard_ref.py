"""Sharded REF on the GPU: ONE engine (one StdRng stream, engine.rs:59-62) over a
window split into contiguous shards, each shard on its own context (= its own
rank), must equal one evaluator over the whole window — outputs bit for bit, the
step result, and the engine state (rng_next, last_committed, contiguous
watermark) on every rank. The single evaluator is itself checked against the
oracle (test_gpu_parity.py); here both are also compared with the oracle directly
where it finishes in seconds.

Stages per window (include/rabia_gpu.h "Sharded REF"): step with provisional draw
positions + draw records -> rows exchanged -> fix-up at the global positions ->
final rows exchanged -> commit fold. In one process the exchange is a stack of the
ranks' device rows; test_two_process_gloo runs it across processes."""
import os
import socket

import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd import shard
from rabia_amd.engine import PhaseEvaluator, decode_outputs, plane_stride, record_window_words

pytestmark = pytest.mark.gpu

RES_CMP = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max",
           "first_undecided", "rng_next", "commit_watermark", "flags"]


def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def rows_of(t):
    return [shard.row_result(r) for r in t.cpu().numpy().view(np.uint64).tolist()]


def run_sharded(n, world, window_sizes, votes, out, stride, seed=42, self_lane=None, state=None, max_phase=0,
                cap=None, aligned=128, keep=None, diag=0, launches=None):
    """Every window's stage 1 on every shard first (provisional positions pile up,
    as in the pipelined bench), then fix-ups and commits window by window.
    diag: rg_debug_set switches of every context (e.g. the lag kernel forced);
    launches: gets each stage-1 launch's shape (rg_debug_last_launch)."""
    torch = torch_cuda()
    self_lane = n // 2 if self_lane is None else self_lane
    ctxs = [PhaseEvaluator(n, self_lane=self_lane, seed=seed) for _ in range(world)]
    try:
        for ev in ctxs:
            if state:
                ev.set_state(**state)
            if diag:
                ev.debug_set(diag)
        W = len(window_sizes)
        rows = torch.zeros((W, world, 10), dtype=torch.int64, device="cuda")
        fixed = torch.zeros((W, world, 10), dtype=torch.int64, device="cuda")
        result = torch.zeros((W, world, 10), dtype=torch.int64, device="cuda")
        recs, plan = [], []
        for S in window_sizes:
            for r in range(world):
                cnt_r = max(shard.shard_range(S, world, r, align=aligned)[1], 1)
                c = cap if cap is not None else cnt_r
                recs.append(torch.zeros(record_window_words(cnt_r, max(c, 1)), dtype=torch.int32, device="cuda"))
        # torch fills on its own stream; the contexts' streams do not wait for it
        torch.cuda.synchronize()
        base, off = 1, 0
        for w, S in enumerate(window_sizes):
            parts = []
            for r in range(world):
                start, cnt = shard.shard_range(S, world, r, align=aligned)
                c = cap if cap is not None else max(cnt, 1)
                rec = recs[w * world + r]
                parts.append((start, cnt, rec, c))
                if cnt:
                    w0 = (off + start) // 32
                    ctxs[r].phase_step_shard_async(votes.data_ptr() + 4 * w0, out.data_ptr() + 4 * w0, cnt, stride,
                                                   base + start, rec.data_ptr(), c, rows[w, r].data_ptr(),
                                                   max_phase=max_phase)
                    if launches is not None:
                        launches.append(ctxs[r].last_launch())
                else:  # an empty shard still reports a row
                    rows[w, r, 6] = base + S
                    torch.cuda.synchronize()
            plan.append((base, off, S, parts))
            base += S
            off += ((S + 127) // 128) * 128
        torch.cuda.synchronize()
        for w, (base, off, S, parts) in enumerate(plan):
            g = rows[w].contiguous()
            for r, (start, cnt, rec, c) in enumerate(parts):
                if cnt:
                    w0 = (off + start) // 32
                    ctxs[r].shard_fixup_async(out.data_ptr() + 4 * w0, cnt, stride, base + start, rec.data_ptr(), c,
                                              g.data_ptr(), r, world, fixed[w, r].data_ptr(), max_phase=max_phase)
                else:
                    fixed[w, r] = rows[w, r]
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            fg = fixed[w].contiguous()
            for r in range(world):
                ctxs[r].shard_commit_async(fg.data_ptr(), world, base, S, result[w, r].data_ptr())
            torch.cuda.synchronize()
        # rg_last_stage_result: each context keeps its latest fix-up row and commit result
        last = len(window_sizes) - 1
        for r, ev in enumerate(ctxs):
            if plan[last][3][r][1]:
                assert shard.result_row(ev.last_stage_result(0)) == fixed[last, r].cpu().numpy().view(np.uint64).tolist()
            assert shard.result_row(ev.last_stage_result(1)) == result[last, r].cpu().numpy().view(np.uint64).tolist()
        states = [ev.get_state() for ev in ctxs]
        if keep is not None:
            keep.extend(r.cpu().numpy().view(np.uint64) for r in recs)
    finally:
        for ev in ctxs:
            ev.close()
    return [rows_of(result[w]) for w in range(len(window_sizes))], states, rows_of(rows[0]), rows_of(fixed[0])


def run_sharded_windows(n, world, K, S, votes, out, stride, seed=42, self_lane=None, state=None, max_phase=0,
                        batched_stages=False, diag=0, launches=None):
    """As run_sharded over K equal windows, but stage 1 of each shard runs as ONE
    multi-window launch (rg_phase_step_shard_windows_async) over its K windows;
    batched_stages: the fix-ups and commits too (one call each for the K windows)."""
    torch = torch_cuda()
    self_lane = n // 2 if self_lane is None else self_lane
    Sp = ((S + 127) // 128) * 128
    ctxs = [PhaseEvaluator(n, self_lane=self_lane, seed=seed) for _ in range(world)]
    try:
        for ev in ctxs:
            if state:
                ev.set_state(**state)
            if diag:
                ev.debug_set(diag)
        rows = torch.zeros((K, world, 10), dtype=torch.int64, device="cuda")
        fixed = torch.zeros((K, world, 10), dtype=torch.int64, device="cuda")
        result = torch.zeros((K, world, 10), dtype=torch.int64, device="cuda")
        parts = [shard.shard_range(S, world, r, align=128) for r in range(world)]
        recs = [torch.zeros(K * record_window_words(max(cnt, 1), max(cnt, 1)), dtype=torch.int32, device="cuda")
                for _, cnt in parts]
        rows_r = [torch.zeros((K, 10), dtype=torch.int64, device="cuda") for _ in range(world)]
        torch.cuda.synchronize()
        for r, (start, cnt) in enumerate(parts):
            w0 = start // 32
            ctxs[r].phase_step_shard_windows_async(K, votes.data_ptr() + 4 * w0, Sp // 32, out.data_ptr() + 4 * w0,
                                                   Sp // 32, cnt, stride, 1 + start, S, recs[r].data_ptr(), cnt,
                                                   rows_r[r].data_ptr(), max_phase=max_phase)
            if launches is not None:
                launches.append(ctxs[r].last_launch())
        torch.cuda.synchronize()
        for r in range(world):
            rows[:, r] = rows_r[r]
        if batched_stages:  # rank-major rows [world][K], as an all-gather of each rank's K rows
            g = torch.stack(rows_r).contiguous()
            fixed_r = [torch.zeros((K, 10), dtype=torch.int64, device="cuda") for _ in range(world)]
            for r, (start, cnt) in enumerate(parts):
                w0 = start // 32
                ctxs[r].shard_fixup_windows_async(K, out.data_ptr() + 4 * w0, Sp // 32, cnt, stride, 1 + start, S,
                                                  recs[r].data_ptr(), cnt, g.data_ptr(), r, world,
                                                  fixed_r[r].data_ptr(), max_phase=max_phase)
            torch.cuda.synchronize()
            fg = torch.stack(fixed_r).contiguous()
            res_r = [torch.zeros((K, 10), dtype=torch.int64, device="cuda") for _ in range(world)]
            for r in range(world):
                ctxs[r].shard_commit_windows_async(K, fg.data_ptr(), world, 1, S, res_r[r].data_ptr())
            torch.cuda.synchronize()
            for r in range(world):
                result[:, r] = res_r[r]
        for w in range(K if not batched_stages else 0):
            base, off = 1 + w * S, w * Sp
            g = rows[w].contiguous()
            for r, (start, cnt) in enumerate(parts):
                w0 = (off + start) // 32
                ctxs[r].shard_fixup_async(out.data_ptr() + 4 * w0, cnt, stride, base + start,
                                          recs[r].data_ptr() + 4 * w * record_window_words(cnt, cnt), cnt,
                                          g.data_ptr(), r, world,
                                          fixed[w, r].data_ptr(), max_phase=max_phase)
            torch.cuda.synchronize()
            fg = fixed[w].contiguous()
            for r in range(world):
                ctxs[r].shard_commit_async(fg.data_ptr(), world, base, S, result[w, r].data_ptr())
            torch.cuda.synchronize()
        states = [ev.get_state() for ev in ctxs]
    finally:
        for ev in ctxs:
            ev.close()
    return [rows_of(result[w]) for w in range(K)], states, [rows_of(rows[w]) for w in range(K)]


def run_single(n, window_sizes, votes, out, stride, seed=42, self_lane=None, state=None, max_phase=0):
    torch = torch_cuda()
    self_lane = n // 2 if self_lane is None else self_lane
    res = torch.zeros((len(window_sizes), 10), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=self_lane, seed=seed) as ev:
        if state:
            ev.set_state(**state)
        base, off = 1, 0
        for w, S in enumerate(window_sizes):
            w0 = off // 32
            ev.phase_step_async(votes.data_ptr() + 4 * w0, out.data_ptr() + 4 * w0, S, stride, slot_base=base,
                                max_phase=max_phase, result_ptr=res[w].data_ptr())
            base += S
            off += ((S + 127) // 128) * 128
        ev.sync()
        st = ev.get_state()
    return rows_of(res), st


def make_votes(n, window_sizes, kind=1, seed=7):
    """Windows laid out back to back (each padded to 128 slots) in one planar buffer."""
    torch = torch_cuda()
    total = sum(((S + 127) // 128) * 128 for S in window_sizes)
    stride = plane_stride(total)
    votes = torch.zeros((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n) as ev:
        base, off = 1, 0
        for S in window_sizes:
            ev.trace_generate_async(kind, seed, base, S, stride, votes.data_ptr() + 4 * (off // 32))
            base += S
            off += ((S + 127) // 128) * 128
        ev.sync()
    return votes, stride, total


@pytest.mark.parametrize("n,world,sizes,kind", [
    (5, 2, [300_007], 1),
    (3, 4, [100_003, 777, 50_000], 0),
    (9, 3, [1 << 20], 1),
    (7, 5, [262_144, 131_071], 2),
    (16, 2, [70_001], 0),
])
def test_sharded_equals_one_engine(oracle, n, world, sizes, kind):
    torch = torch_cuda()
    votes, stride, total = make_votes(n, sizes, kind)
    out_s = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    state = {"rng_next": 1234, "last_committed": 3, "commit_watermark": 1, "steps": 0}
    mp = sum(sizes) * 2 // 3  # commit_phase refuses V1 slots above current_phase
    res_s, st_s, _, _ = run_sharded(n, world, sizes, votes, out_s, stride, state=state, max_phase=mp)
    res_1, st_1 = run_single(n, sizes, votes, out_1, stride, state=state, max_phase=mp)
    assert torch.equal(out_s, out_1)
    for w in range(len(sizes)):
        for r in range(world):
            assert {k: res_s[w][r][k] for k in RES_CMP} == {k: res_1[w][k] for k in RES_CMP}, (w, r)
    for st in st_s:
        assert st == st_1
    # and the oracle over the whole concatenation of windows (one stream across them)
    planes = out_s.view(8, stride).cpu().numpy().view(np.uint32)
    got = decode_outputs(planes, total)
    base, off, rng = 1, 0, 1234
    lc = 3
    for w, S in enumerate(sizes):
        r1, r2, _ = oracle.trace(kind, n, 7, base, S)
        exp, eres = oracle.ref_step(n, n // 2 + 1, n // 2, 42, rng, base, r1, r2, max_phase=mp, lc_in=lc,
                                    wm_in=res_1[w - 1]["commit_watermark"] if w else 1)
        for k in exp:
            np.testing.assert_array_equal(got[k][off:off + S], exp[k], err_msg=f"window {w} {k}")
        assert eres["rng_next"] == res_s[w][0]["rng_next"]
        assert eres["commit_watermark"] == res_s[w][0]["commit_watermark"]
        rng, lc = eres["rng_next"], eres["last_committed_max"]
        base += S
        off += ((S + 127) // 128) * 128


@pytest.mark.parametrize("n,world,K,S,kind", [
    (5, 2, 4, 300_032, 1),
    (9, 3, 3, 1 << 20, 1),
    (7, 1, 5, 262_144, 2),
    (3, 4, 2, 100_096, 0),
])
@pytest.mark.parametrize("batched", [False, True])
def test_shard_windows_launch_equals_per_window(n, world, K, S, kind, batched):
    """K windows of one shard in ONE launch (rg_phase_step_shard_windows_async) ==
    K per-window shard launches: identical fixed outputs, per-window shard rows
    (counts, extremes, n_draws), global results (rng_next, watermarks) and engine state;
    batched: the fix-ups and commits of the K windows as one call each as well."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S] * K, kind)
    out_m = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    out_w = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    state = {"rng_next": 99, "last_committed": 5, "commit_watermark": 1, "steps": 0}
    mp = K * S * 3 // 4
    res_m, st_m, rows_m = run_sharded_windows(n, world, K, S, votes, out_m, stride, state=state, max_phase=mp,
                                              batched_stages=batched)
    res_w, st_w, _, _ = run_sharded(n, world, [S] * K, votes, out_w, stride, state=state, max_phase=mp)
    assert torch.equal(out_m, out_w)
    for w in range(K):
        for r in range(world):
            assert {k: res_m[w][r][k] for k in RES_CMP} == {k: res_w[w][r][k] for k in RES_CMP}, (w, r)
        assert all(x["flags"] == 0 for x in rows_m[w])
    assert st_m == st_w
    # and against one evaluator over the K windows
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * K, votes, out_1, stride, state=state, max_phase=mp)
    assert torch.equal(out_m, out_1) and all(st == st_1 for st in st_m)


def test_sharded_full_size_c5_shape():
    """C5 shape (9 replicas x 2^26 slots) over 8 shards == one evaluator (device
    results compared bit for bit; the single evaluator is oracle-checked elsewhere)."""
    torch = torch_cuda()
    n, S, world = 9, 1 << 26, 8
    votes, stride, total = make_votes(n, [S], 1, seed=11)
    out_s = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_s, st_s, rows, fixed = run_sharded(n, world, [S], votes, out_s, stride)
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S], votes, out_1, stride)
    assert torch.equal(out_s, out_1)
    for r in range(world):
        assert {k: res_s[0][r][k] for k in RES_CMP} == {k: res_1[0][k] for k in RES_CMP}
    assert all(st == st_1 for st in st_s)
    assert sum(x["n_draws"] for x in rows) == res_1[0]["n_draws"] > 0
    del votes


def test_records_capacity_overflow_is_flagged():
    torch = torch_cuda()
    n, S = 5, 200_000
    votes, stride, total = make_votes(n, [S], 0)
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res, _, _, _ = run_sharded(n, 2, [S], votes, out, stride, cap=16)
    assert res[0][0]["flags"] & 8


def test_shard_argument_errors():
    torch = torch_cuda()
    buf = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(5, mode="wmvc") as ev:
        with pytest.raises(N.RabiaGpuError):
            ev.phase_step_shard_async(buf.data_ptr(), buf.data_ptr(), 100, 4, 1, buf.data_ptr(), 100)
    with PhaseEvaluator(5) as ev:
        with pytest.raises(N.RabiaGpuError):
            ev.phase_step_shard_async(buf.data_ptr(), buf.data_ptr(), 100, 4, 1, 0, 100)
        with pytest.raises(N.RabiaGpuError):
            ev.shard_fixup_async(buf.data_ptr(), 100, 4, 1, buf.data_ptr(), 100, buf.data_ptr(), 2, 2)
        # planar multi-window layouts whose windows alias (stride == pitch: window 1's plane p
        # is window 0's plane p + 1) are refused by the step and the fix-up alike
        S, nw = 4096, 128
        rows = torch.zeros((2, 10), dtype=torch.int64, device="cuda")
        with pytest.raises(N.RabiaGpuError, match="overlap"):
            ev.phase_step_shard_windows_async(2, buf.data_ptr(), nw, buf.data_ptr(), nw, S, nw, 1, S,
                                              buf.data_ptr(), S, rows.data_ptr())
        with pytest.raises(N.RabiaGpuError, match="overlap"):
            ev.shard_fixup_windows_async(2, buf.data_ptr(), nw, S, nw, 1, S, buf.data_ptr(), S, rows.data_ptr(), 0,
                                         1, rows.data_ptr())
        # plane-major (stride >= K x pitch) and window-major (pitch >= 20 planes x stride + n_words) pass the check
        big = torch.zeros(21 * 2 * nw, dtype=torch.int32, device="cuda")
        big_out = torch.zeros(8 * 2 * nw, dtype=torch.int32, device="cuda")
        rec = torch.zeros(2 * S, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ev.phase_step_shard_windows_async(2, big.data_ptr(), nw, big_out.data_ptr(), nw, S, 2 * nw, 1, S,
                                          rec.data_ptr(), S, rows.data_ptr())
        ev.phase_step_shard_windows_async(2, big.data_ptr(), 21 * nw, big_out.data_ptr(), 8 * nw, S, nw, 1, S,
                                          rec.data_ptr(), S, rows.data_ptr())
        ev.sync()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import torch
    import torch.distributed as dist
    from rabia_amd import shard as SH
    from rabia_amd.engine import PhaseEvaluator as PE, plane_stride as ps
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, S = 5, 500_000
        start, cnt = SH.shard_range(S, world, rank)
        stride = ps(cnt)
        votes = torch.zeros((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
        out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        with PE(n, self_lane=2, seed=42) as ev:  # the same engine seed on every rank
            ev.trace_generate_async(1, 9, 1 + start, cnt, stride, votes.data_ptr())
            drv = SH.ShardedRefStep(ev, rank, world, cnt, shared_gpu=True)  # both ranks on the one GPU
            g = drv.step(votes.data_ptr(), out.data_ptr(), cnt, stride, 1 + start, 1, S)
            st = ev.get_state()
        planes = out.view(8, stride).cpu().numpy().view(np.uint32)
        q.put((rank, g, st, planes.tobytes(), stride, start, cnt))
    finally:
        dist.destroy_process_group()


def test_two_process_gloo(oracle):
    """Two ranks (processes) on the one GPU, rows exchanged over gloo: the folded
    global result and every rank's state == the oracle's single engine. The ranks'
    step launches take turns (ShardedRefStep shared_gpu: the rule of include/rabia_gpu.h
    for tiled-kernel look-back launches of different processes on one device)."""
    torch_cuda()
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    while len(got) < world:
        try:
            got.append(q.get(timeout=1))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), "a rank died"
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n, S = 5, 500_000
    r1, r2, _ = oracle.trace(1, n, 9, 1, S)
    exp, eres = oracle.ref_step(n, 3, 2, 42, 0, 1, r1, r2)
    for rank, g, st, raw, stride, start, cnt in sorted(got, key=lambda x: x[0]):
        for k in ("n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max",
                  "first_undecided", "rng_next", "commit_watermark"):
            assert g[k] == eres[k], (rank, k)
        assert st["rng_next"] == eres["rng_next"] and st["commit_watermark"] == eres["commit_watermark"]
        assert st["last_committed"] == eres["last_committed_max"]
        dec = decode_outputs(np.frombuffer(raw, np.uint32).reshape(8, stride), cnt)
        for k in exp:
            np.testing.assert_array_equal(dec[k], exp[k][start:start + cnt], err_msg=f"rank {rank} {k}")


def test_pipelined_two_streams_equals_one_engine():
    """The C5 schedule on two shards (two contexts): each step's K-window shard launch
    runs on a compute stream while the previous step's fix-ups and commits run on a
    second stream per context (events only, no host synchronisation between steps),
    as bench.py pipelines it. Final outputs, per-window results and engine states ==
    one evaluator over all windows."""
    torch = torch_cuda()
    n, world, K, steps, S = 5, 2, 3, 4, 262_144
    W = K * steps
    votes, stride, total = make_votes(n, [S] * W, 1, seed=21)
    Sp = ((S + 127) // 128) * 128
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    parts = [shard.shard_range(S, world, r, align=128) for r in range(world)]
    i64 = dict(dtype=torch.int64, device="cuda")
    rows = torch.zeros((steps, world, K, 10), **i64)
    g_rows = torch.zeros((steps, world, world, K, 10), **i64)
    fixed = torch.zeros((steps, world, K, 10), **i64)
    g_fixed = torch.zeros((steps, world, world, K, 10), **i64)
    result = torch.zeros((steps, world, K, 10), **i64)
    recs = [[torch.zeros(K * record_window_words(cnt, cnt), dtype=torch.int32, device="cuda") for _, cnt in parts]
            for _ in range(steps)]
    ctxs = [PhaseEvaluator(n, self_lane=2, seed=42) for _ in range(world)]
    comp = [torch.cuda.Stream() for _ in range(world)]
    fix = [torch.cuda.Stream() for _ in range(world)]
    torch.cuda.synchronize()
    try:
        for t in range(steps):
            e_main = []
            for r, (start, cnt) in enumerate(parts):
                w0 = (t * K * Sp + start) // 32
                ctxs[r].phase_step_shard_windows_async(K, votes.data_ptr() + 4 * w0, Sp // 32, out.data_ptr() + 4 * w0,
                                                       Sp // 32, cnt, stride, 1 + t * K * S + start, S,
                                                       recs[t][r].data_ptr(), cnt, rows[t, r].data_ptr(),
                                                       stream=comp[r].cuda_stream)
                e = torch.cuda.Event()
                e.record(comp[r])
                e_main.append(e)
            e_fix = []
            for r, (start, cnt) in enumerate(parts):  # the row all-gather, then the fix-up
                with torch.cuda.stream(fix[r]):
                    for e in e_main:
                        fix[r].wait_event(e)
                    g_rows[t, r].copy_(rows[t])
                    w0 = (t * K * Sp + start) // 32
                    ctxs[r].shard_fixup_windows_async(K, out.data_ptr() + 4 * w0, Sp // 32, cnt, stride,
                                                      1 + t * K * S + start, S, recs[t][r].data_ptr(), cnt,
                                                      g_rows[t, r].data_ptr(), r, world, fixed[t, r].data_ptr(),
                                                      stream=fix[r].cuda_stream)
                    e = torch.cuda.Event()
                    e.record(fix[r])
                    e_fix.append(e)
            for r in range(world):  # the final-row all-gather, then the commit
                with torch.cuda.stream(fix[r]):
                    for e in e_fix:
                        fix[r].wait_event(e)
                    g_fixed[t, r].copy_(fixed[t])
                    ctxs[r].shard_commit_windows_async(K, g_fixed[t, r].data_ptr(), world, 1 + t * K * S, S,
                                                       result[t, r].data_ptr(), stream=fix[r].cuda_stream)
        torch.cuda.synchronize()
        states = [ev.get_state() for ev in ctxs]
    finally:
        for ev in ctxs:
            ev.close()
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * W, votes, out_1, stride, self_lane=2)
    assert torch.equal(out, out_1)
    got = result.cpu().numpy().view(np.uint64)
    for t in range(steps):
        for r in range(world):
            for k in range(K):
                g = shard.row_result(got[t, r, k].tolist())
                assert {f: g[f] for f in RES_CMP} == {f: res_1[t * K + k][f] for f in RES_CMP}, (t, r, k)
    assert all(st == st_1 for st in states)


@pytest.mark.parametrize("n,K,S,kind", [(5, 3, 300_032, 1), (9, 4, 1 << 20, 2)])
def test_rccl_exchange_world1_equals_one_evaluator(n, K, S, kind):
    """The multi-GPU pipeline through the C ABI's RCCL communicator (rg_comm_create at
    world 1, rg_shard_exchange_windows_async: rows all-gathered, fix-up, final rows
    all-gathered, commit, bitmaps all-gathered, all on one device stream) equals one
    evaluator window by window: outputs, results, engine state; the gathered bitmaps
    equal rg_decision_bitmap_windows_async of the fixed outputs. Also the single-window
    driver (ShardedRefStep(rccl=True)), the generic all-gather, max and barrier."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S] * K, kind, seed=41)
    Sp = ((S + 127) // 128) * 128
    nw = (S + 31) // 32
    i64 = dict(dtype=torch.int64, device="cuda")
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    rows = torch.zeros((K, 10), **i64)
    res = torch.zeros((K, 10), **i64)
    rec = torch.zeros(K * S, **i64)
    bm_all = torch.zeros((1, K, 2, nw), dtype=torch.int32, device="cuda")
    state = {"rng_next": 55, "last_committed": 2, "commit_watermark": 1, "steps": 0}
    mp = K * S * 2 // 3
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n // 2, seed=42) as ev:
        with pytest.raises(N.RabiaGpuError, match="no communicator"):
            ev.comm_barrier()
        shard.RcclComm(0, 1).attach(ev)
        assert ev.comm_rank() == (0, 1)
        ev.set_state(**state)
        ev.phase_step_shard_windows_async(K, votes.data_ptr(), Sp // 32, out.data_ptr(), Sp // 32, S, stride, 1, S,
                                          rec.data_ptr(), S, rows.data_ptr(), max_phase=mp)
        with pytest.raises(N.RabiaGpuError, match="rg_comm_reserve"):  # no payload reserved: nothing enqueued
            ev.shard_exchange_windows_async(K, out.data_ptr(), Sp // 32, S, stride, 1, 1, S, rec.data_ptr(), S,
                                            rows.data_ptr(), res.data_ptr(), bm_all.data_ptr(), max_phase=mp)
        ev.comm_reserve(K, S)
        ev.shard_exchange_windows_async(K, out.data_ptr(), Sp // 32, S, stride, 1, 1, S, rec.data_ptr(), S,
                                        rows.data_ptr(), res.data_ptr(), bm_all.data_ptr(), max_phase=mp)
        ev.sync()
        st = ev.get_state()
        # generic all-gather (world 1: a copy), max over ranks, barrier
        src = torch.arange(37, dtype=torch.int32, device="cuda")
        dst = torch.zeros(37, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        ev.comm_allgather_async(src.data_ptr(), dst.data_ptr(), 37 * 4)
        ev.sync()
        assert torch.equal(src, dst)
        assert ev.comm_max([1.5, -2.0, 7.0]) == [1.5, -2.0, 7.0]
        ev.comm_barrier()
        ev.comm_destroy()
        with pytest.raises(N.RabiaGpuError):
            ev.comm_rank()
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * K, votes, out_1, stride, self_lane=n // 2, state=state, max_phase=mp)
    assert torch.equal(out, out_1) and st == st_1
    got = rows_of(res)
    for w in range(K):
        assert {k: got[w][k] for k in RES_CMP} == {k: res_1[w][k] for k in RES_CMP}, w
    bm = torch.zeros((K, 2, nw), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n) as ev:
        ev.decision_bitmap_windows_async(K, out.data_ptr(), Sp // 32, S, stride, bm[0, 0].data_ptr(),
                                         bm[0, 1].data_ptr(), 2 * nw)
        ev.sync()
    assert torch.equal(bm_all[0], bm)
    # the single-window driver over the first window through the communicator
    out_d = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n // 2, seed=42) as ev:
        shard.RcclComm(0, 1).attach(ev)
        ev.set_state(**state)
        drv = shard.ShardedRefStep(ev, 0, 1, S, rccl=True)
        g = drv.step(votes.data_ptr(), out_d.data_ptr(), S, stride, 1, 1, S, max_phase=mp)
    assert {k: g[k] for k in RES_CMP} == {k: res_1[0][k] for k in RES_CMP}
    assert torch.equal(out_d[: Sp // 32], out_1[: Sp // 32])



def _committed_from_lists(lists, K, cap, nw, S):
    """Committed bitmaps rebuilt from undecided lists: every valid slot set, listed slots
    cleared (the consumer side of rg_shard_exchange_decisions_async)."""
    bits = np.ones((K, nw * 32), np.uint8)
    bits[:, S:] = 0
    for w in range(K):
        cnt = int(lists[w, 0])
        assert cnt <= cap
        offs = lists[w, 1:1 + cnt].astype(np.int64)
        assert np.all(np.diff(offs) > 0) and (cnt == 0 or offs[-1] < S)  # ascending, inside the shard
        bits[w, offs] = 0
    return np.packbits(bits, axis=1, bitorder="little").view(np.uint32)


@pytest.mark.parametrize("n,K,S,kind", [(5, 3, 300_032, 1), (9, 4, 1 << 20, 2), (7, 2, 65_601, 0)])
def test_rccl_exchange_decisions_world1(n, K, S, kind):
    """rg_shard_exchange_decisions_async at world 1: the rows, results and engine state
    equal one evaluator's; the gathered undecided lists hold exactly the slots whose
    committed bit is clear (ascending, count = n_slots - n_decided of the final row), so
    the committed bitmap rebuilt from them equals rg_decision_bitmap_windows_async's; the
    V1 bitmaps equal its V1 bitmaps (bits past n_slots cleared). A list capacity below a
    window's undecided count flags the window (32) and keeps the first `cap` offsets."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S] * K, kind, seed=43)
    Sp = ((S + 127) // 128) * 128
    nw = (S + 31) // 32
    i64 = dict(dtype=torch.int64, device="cuda")
    state = {"rng_next": 7, "last_committed": 0, "commit_watermark": 1, "steps": 0}
    bm = torch.zeros((K, 2, nw), dtype=torch.int32, device="cuda")
    runs = {}
    for cap, with_v1 in ((S, True), (S // 3, False), (3, True)):
        out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
        rows = torch.zeros((K, 10), **i64)
        res = torch.zeros((K, 10), **i64)
        rec = torch.zeros(K * S, **i64)
        P = K * (1 + cap) + (K * nw if with_v1 else 0)
        dec = torch.full((P,), -1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        with PhaseEvaluator(n, self_lane=n // 2, seed=42) as ev:
            shard.RcclComm(0, 1).attach(ev)
            ev.comm_reserve(K, S, cap)
            ev.set_state(**state)
            ev.phase_step_shard_windows_async(K, votes.data_ptr(), Sp // 32, out.data_ptr(), Sp // 32, S, stride, 1,
                                              S, rec.data_ptr(), S, rows.data_ptr())
            ev.shard_exchange_decisions_async(K, out.data_ptr(), Sp // 32, S, stride, 1, 1, S, rec.data_ptr(), S,
                                              rows.data_ptr(), res.data_ptr(), cap, dec.data_ptr(), with_v1=with_v1)
            ev.sync()
            st = ev.get_state()
            if not runs:
                ev.decision_bitmap_windows_async(K, out.data_ptr(), Sp // 32, S, stride, bm[0, 0].data_ptr(),
                                                 bm[0, 1].data_ptr(), 2 * nw)
                ev.sync()
        runs[(cap, with_v1)] = (out, rows_of(res), st, dec.cpu().numpy().view(np.uint32))
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * K, votes, out_1, stride, self_lane=n // 2, state=state)
    b = bm.cpu().numpy().view(np.uint32)
    tail = np.uint32((1 << (S % 32)) - 1) if S % 32 else np.uint32(0xFFFFFFFF)
    full = None
    for (cap, with_v1), (out, got, st, dec) in runs.items():
        assert torch.equal(out, out_1) and st == st_1
        lists = dec[:K * (1 + cap)].reshape(K, 1 + cap)
        for w in range(K):
            und = res_1[w]["n_slots"] - res_1[w]["n_decided"]
            assert int(lists[w, 0]) == und, (cap, w)
            exp_flags = 32 if und > cap else 0
            assert got[w]["flags"] == exp_flags, (cap, w)
            assert {k: got[w][k] for k in RES_CMP if k != "flags"} == {k: res_1[w][k] for k in RES_CMP if k != "flags"}
        if cap == S:  # complete lists: the committed bitmap rebuilt equals the step's
            committed = _committed_from_lists(lists, K, cap, nw, S)
            exp = b[:, 0].copy()
            exp[:, -1] &= tail
            np.testing.assert_array_equal(committed, exp)
            full = lists
        else:  # truncated: the first min(count, cap) offsets of the complete list
            for w in range(K):
                m = min(int(lists[w, 0]), cap)
                np.testing.assert_array_equal(lists[w, 1:1 + m], full[w, 1:1 + m])
        if with_v1:
            v1 = dec[K * (1 + cap):].reshape(K, nw)
            exp = b[:, 1].copy()
            exp[:, -1] &= tail
            np.testing.assert_array_equal(v1, exp)
        else:
            assert dec.size == K * (1 + cap)


def test_async_calls_refuse_past_reservation():
    """The _async entry points never allocate or synchronise: past the context's
    reservation (rg_reserve; rg_create's default is 128 windows per call) they return
    RG_EINVAL and enqueue nothing; after rg_reserve the same calls run and equal one
    evaluator."""
    torch = torch_cuda()
    n, K, S = 5, 130, 1024
    votes, stride, total = make_votes(n, [S] * K, 1, seed=5)
    i64 = dict(dtype=torch.int64, device="cuda")
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    rows = torch.zeros((K, 10), **i64)
    fixed = torch.zeros((K, 10), **i64)
    res = torch.zeros((K, 10), **i64)
    rec = torch.zeros(K * S, **i64)
    lists = torch.zeros(K * (1 + S), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=2, seed=42) as ev:
        step = lambda: ev.phase_step_shard_windows_async(K, votes.data_ptr(), S // 32, out.data_ptr(), S // 32, S,  # noqa
                                                         stride, 1, S, rec.data_ptr(), S, rows.data_ptr())
        fix = lambda: ev.shard_fixup_windows_async(K, out.data_ptr(), S // 32, S, stride, 1, S, rec.data_ptr(), S,  # noqa
                                                   rows.data_ptr(), 0, 1, fixed.data_ptr())
        lst = lambda: ev.decision_lists_windows_async(K, out.data_ptr(), S // 32, S, stride, lists.data_ptr(), S)  # noqa
        for call in (step, fix, lst):
            with pytest.raises(N.RabiaGpuError, match="rg_reserve") as e:
                call()
            assert e.value.code == N.RG_EINVAL
        ev.reserve(K * S, K)
        step()
        fix()
        ev.shard_commit_windows_async(K, fixed.data_ptr(), 1, 1, S, res.data_ptr())
        lst()
        ev.sync()
        st = ev.get_state()
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * K, votes, out_1, stride, self_lane=2)
    assert torch.equal(out, out_1) and st == st_1
    got = rows_of(res)
    for w in range(K):
        assert {k: got[w][k] for k in RES_CMP} == {k: res_1[w][k] for k in RES_CMP}, w
    ls = lists.cpu().numpy().view(np.uint32).reshape(K, 1 + S)
    assert [int(x) for x in ls[:, 0]] == [r["n_slots"] - r["n_decided"] for r in res_1]


@pytest.mark.parametrize("n,K,S,kind,force_lag", [(5, 3, 300_032, 1, True), (9, 2, 262_144, 0, True),
                                                   (7, 1, 100_000, 2, False), (3, 2, 65_536, 1, False)])
def test_shard_step_records_equal_oracle(oracle, n, K, S, kind, force_lag):
    """Stage 1 itself against the oracle's restatement (or_shard_step): the device's record
    region (the segment table; per VQ slot the offset in its segment, c1-vs-c0 class, the
    decision under each own vote, the provisional vote) and its row of the non-VQ slots,
    bit for bit. The lag kernel's provisional vote is the likelier outcome, as the oracle's;
    the tiled kernel draws at the provisional position instead (bit 30 then differs: the
    fix-up re-draws either)."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S] * K, kind, seed=61)
    Sp = ((S + 127) // 128) * 128
    i64 = dict(dtype=torch.int64, device="cuda")
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    rows = torch.zeros((K, 10), **i64)
    rww = record_window_words(S, S)
    rec = torch.zeros(K * rww, dtype=torch.int32, device="cuda")
    mp = K * S // 2
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n // 2, seed=42) as ev:
        if force_lag:
            ev.debug_set(0x200000)
        ev.phase_step_shard_windows_async(K, votes.data_ptr(), Sp // 32, out.data_ptr(), Sp // 32, S, stride, 1, S,
                                          rec.data_ptr(), S, rows.data_ptr(), max_phase=mp)
        ev.sync()
        la = ev.last_launch()
    assert la["kernel"] == ("lag" if force_lag else "tiled"), la
    got_rows = rows_of(rows)
    regs = rec.cpu().numpy().view(np.uint32).reshape(K, rww)
    planes = out.view(8, stride).cpu().numpy().view(np.uint32)
    n_chunks = (S + 0xFFFFFF) >> 24
    tw = rww - S
    for w in range(K):
        base = 1 + w * S
        r1, r2, _ = oracle.trace(kind, n, 61, base, S)
        exp, ereg, erow = oracle.shard_step(n, n // 2 + 1, n // 2, base, r1, r2, max_phase=mp)
        for k in ("n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max", "first_undecided"):
            assert got_rows[w][k] == erow[k], (w, k)
        np.testing.assert_array_equal(regs[w, :n_chunks], ereg[:n_chunks], err_msg=f"window {w} segment table")
        nd = erow["n_draws"]
        mask = np.uint32(0xFFFFFFFF if force_lag else ~(1 << 30) & 0xFFFFFFFF)
        np.testing.assert_array_equal(regs[w, tw:tw + nd] & mask, ereg[tw:tw + nd] & mask, err_msg=f"window {w} records")
        if force_lag:  # the provisional outputs too
            w0 = (w * Sp) // 32
            dec = decode_outputs(planes[:, w0:w0 + (S + 31) // 32], S)
            for k in exp:
                np.testing.assert_array_equal(dec[k], exp[k], err_msg=f"window {w} {k}")
