"""The persistent lag REF kernel (ref_lag_kernel, rg_kernels.h) in every shape the
C ABI's dispatch (step_impl, rabia_gpu.hip) can pick, compared with the oracle
directly — not only with the tiled kernel:

- the bench shape: n = 5, 2^30 slots, slot-tiled 1024, default dispatch
  (ref_lag_kernel<5, 4, 512, false>): size-independent properties over all 2^30
  slots, oracle slices at both ends, across workgroup-tile boundaries and in the
  middle (each slice's StdRng offset = the VQ slots before it), the tiled kernel's
  output over the same slots, and one call == two calls;
- the one-workgroup-per-CU shape forced at 2^25 (+ ragged) slots for n = 3, 5, 7, 9 against
  the full oracle, on the default grid and on a 5-workgroup grid (many tickets each);
- the shape chosen without any switch for n = 3, 7, 9 at the first size that selects it;
- the SHARD = true instantiation (draw records, VQ slots left to the fix-up) in 2-4
  shards, forced on small launches and chosen without a switch at 2^29 slots per
  shard, against one evaluator and the oracle; its draw-record overflow.

Every test asserts which kernel shape ran (rg_debug_last_launch).
Reference: engine.rs:483-682 (round-1/round-2 handlers, the StdRng draw),
messages.rs:185-222 (count_votes, set_decision), state.rs:65-103 (commit_phase).

Run on an MI355X: python -m pytest tests/test_lag_shapes.py -m gpu -x -q
"""
import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator, decode_outputs, plane_stride
from test_gpu_parity import RES_CMP, torch_cuda
from test_shard_ref import make_votes, run_sharded, run_sharded_windows, run_single

pytestmark = pytest.mark.gpu

LAG = 0x200000     # rg_debug_set: the lag kernel at any launch size
TILED = 0x100000   # rg_debug_set: large launches keep the tiled kernel
KEYS = ("r1", "r2own", "dec", "committed", "value")


def n_cu(torch):
    return torch.cuda.get_device_properties(0).multi_processor_count


def lag_words(n):
    """Words per thread of the two-workgroups-per-CU (512-thread) lag shape; its tile
    (512 x lag_words) is half the one-workgroup-per-CU tile (1024 x lag_words words)."""
    return 2 if n <= 5 else 1


def one_shape(n):
    """(threads, words per thread) of the one-workgroup-per-CU lag shape: 2048-word tiles as
    512 x 4 (16-byte plane loads) at every n <= 10 (round 5; n > 5 ran 1024 x 1 before)."""
    return (512, 4)


def popc(torch, x):
    """Per-word population count of an int32 tensor (int64 result)."""
    x = x.to(torch.int64) & 0xFFFFFFFF
    x = x - ((x >> 1) & 0x55555555)
    x = (x & 0x33333333) + ((x >> 2) & 0x33333333)
    x = (x + (x >> 4)) & 0x0F0F0F0F
    return ((x * 0x01010101) & 0xFFFFFFFF) >> 24


def word_planes(out, nw, T, stride):
    """The 8 output planes as int32 tensors of nw words in slot order (planar or
    slot-tiled T-word layout)."""
    if T:
        o = out.view(-1, 8, T)
        return [o[:, i, :].reshape(-1)[:nw] for i in range(8)]
    o = out.view(8, stride)
    return [o[i, :nw] for i in range(8)]


def check_properties(torch, p, S, slot_base, max_phase, res, rng0, rng1, lc_in=0):
    """What must hold over every slot whatever the draws were (engine.rs:495-505,
    523-542, 613-628; messages.rs:217-222; state.rs:65-103). Returns the per-word VQ
    counts (the draw offset of any slice is their prefix)."""
    nw = p[0].numel()
    valid = torch.full((nw,), -1, dtype=torch.int32, device=p[0].device)
    if S % 32:
        valid[-1] = (1 << (S % 32)) - 1
    vq = ~p[0] & p[1]                     # round-1 result VQuestion
    pend = p[0] & p[1] & valid            # round 1 without quorum
    cvq = popc(torch, vq)
    assert res["n_draws"] == int(cvq.sum()) == rng1 - rng0 > 0
    assert res["n_pending_r1"] == int(popc(torch, pend).sum())
    assert res["n_decided"] == int(popc(torch, p[6]).sum())
    assert res["n_v1"] == int(popc(torch, p[7]).sum())
    assert torch.equal(p[6], ~p[5] & valid), "committed <=> decision in {V0, V1}"
    assert torch.equal(p[7], p[4] & ~p[5]), "apply <=> decision V1"
    assert torch.equal(p[3], pend), "own round-2 vote: none exactly when round 1 is pending"
    r1v1 = p[0] & ~p[1]
    assert torch.equal(p[2] & ~vq, (r1v1 | pend) & ~vq), "own round-2 vote = round-1 result off the VQ slots"
    # contiguous watermark / first undecided
    und = (~p[6] & valid).to(torch.int64) & 0xFFFFFFFF
    nz = torch.nonzero(und)
    if nz.numel():
        w = int(nz[0])
        x = int(und[w])
        fu = slot_base + 32 * w + ((x & -x).bit_length() - 1)
    else:
        fu = slot_base + S
    assert res["first_undecided"] == fu
    # commit_phase's max over V1 ids <= max_phase (state.rs:77-99)
    lim = S - 1 if not max_phase else min(S - 1, max_phase - slot_base)
    exp_lc = lc_in
    if lim >= 0:
        v1 = p[7][: lim // 32 + 1].to(torch.int64) & 0xFFFFFFFF
        v1[-1] &= (2 << (lim % 32)) - 1
        nz = torch.nonzero(v1)
        if nz.numel():
            w = int(nz[-1])
            exp_lc = max(exp_lc, slot_base + 32 * w + int(v1[w]).bit_length() - 1)
    assert res["last_committed_max"] == exp_lc
    return cvq


def check_slices(oracle, torch, p, cvq, n, kind, seed, slot_base, rng0, self_lane, slices, cnt=8192):
    q = n // 2 + 1
    pref = torch.cumsum(cvq, 0)
    for lo in slices:
        assert lo % 32 == 0
        w0 = lo // 32
        k0 = rng0 + (int(pref[w0 - 1]) if w0 else 0)
        planes = np.stack([x[w0:w0 + cnt // 32].cpu().numpy().view(np.uint32) for x in p])
        got = decode_outputs(planes, cnt)
        r1, r2, _ = oracle.trace(kind, n, seed, slot_base + lo, cnt)
        exp, _ = oracle.ref_step(n, q, self_lane, 42, k0, slot_base + lo, r1, r2)
        for k in KEYS:
            np.testing.assert_array_equal(got[k], exp[k], err_msg=f"{k}: slice at slot {lo}")


@pytest.mark.parametrize("kind", [N.RG_TRACE_AGREE90, N.RG_TRACE_UNIFORM])
def test_bench_shape_vs_oracle(oracle, kind):
    """The launch bench.py times (n = 5, 2^30 slots = 1024 windows, slot-tiled 1024,
    default dispatch): ref_lag_kernel<5, 4, 512, false> on one workgroup per CU."""
    torch = torch_cuda()
    n, S, T = 5, 1 << 30, 1024
    nw = S // 32
    tiles = nw // T
    mp = S - 1000
    votes = torch.empty(tiles * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    out = torch.empty(tiles * 8 * T, dtype=torch.int32, device="cuda")
    res_d = torch.zeros(10, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T) as ev:
        ev.trace_generate_async(kind, 11, 1, S, T, votes.data_ptr())
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, T, slot_base=1, max_phase=mp,
                            result_ptr=res_d.data_ptr())
        launch = ev.last_launch()
        res = ev.last_result()
        st = ev.get_state()
    assert launch == {"kernel": "lag", "shard": False, "block": 512, "words": 4, "grid": n_cu(torch),
                      "windows": 1}, launch
    assert res["flags"] == 0 and res["n_slots"] == S
    assert res == N.RgStepResult(*res_d.cpu().numpy().view(np.uint64).tolist()).as_dict()
    p = word_planes(out, nw, T, 0)
    cvq = check_properties(torch, p, S, 1, mp, res, 0, st["rng_next"])
    assert res["commit_watermark"] == res["first_undecided"] == st["commit_watermark"]
    assert res["last_committed_max"] == st["last_committed"]
    tw = 1024 * 2  # one workgroup tile of the lag kernel, in words
    slices = [0, S - 8192, 32 * (tw - 128), 32 * (37 * tw - 64), 32 * (S // 96), 32 * (nw // 2 - 100),
              32 * (nw - 3 * tw - 17)]
    check_slices(oracle, torch, p, cvq, n, kind, 11, 1, 0, n - 1, slices)
    del p, cvq
    # the tiled kernel over the same slots, and the same slots as two calls
    for diag, calls in ((TILED, 1), (0, 2)):
        out2 = torch.empty_like(out)
        torch.cuda.synchronize()
        with PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T) as ev:
            ev.debug_set(diag)
            part = S // calls
            for c in range(calls):
                t0 = c * (part // 32) // T
                ev.phase_step_async(votes.data_ptr() + 4 * t0 * (4 * n + 1) * T, out2.data_ptr() + 4 * t0 * 8 * T,
                                    part, T, slot_base=1 + c * part, max_phase=mp)
                assert ev.last_launch()["kernel"] == ("tiled" if diag else "lag")
            st2 = ev.get_state()
            r2 = ev.last_result()
        assert torch.equal(out, out2), (diag, calls)
        assert st2["rng_next"] == st["rng_next"] and st2["last_committed"] == st["last_committed"]
        assert st2["commit_watermark"] == st["commit_watermark"]
        if calls == 1:
            assert r2 == res
        del out2


def _planar_step(torch, n, S, kind, seed, slot_base, diag, rng0=99, lc_in=3, wm_in=7, max_phase=0, self_lane=None):
    stride = plane_stride(S)
    votes = torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    out = torch.empty(8 * stride, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n - 1 if self_lane is None else self_lane, seed=42) as ev:
        ev.debug_set(diag)
        ev.set_state(rng_next=rng0, last_committed=lc_in, commit_watermark=wm_in)
        ev.trace_generate_async(kind, seed, slot_base, S, stride, votes.data_ptr())
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=slot_base, max_phase=max_phase)
        launch = ev.last_launch()
        res = ev.last_result()
        st = ev.get_state()
    assert res["flags"] == 0
    assert st["rng_next"] == res["rng_next"] and st["last_committed"] == res["last_committed_max"]
    return out, stride, res, launch


@pytest.mark.parametrize("n,kind", [(3, 1), (5, 1), (5, 2), (7, 1), (9, 1), (9, 0)])
def test_forced_lag1024_vs_full_oracle(oracle, n, kind):
    """The one-workgroup-per-CU shape (forced, ragged 2^25 + 4099 slots) on the default grid
    and on 5 workgroups (~100 tickets each): every slot and the step result equal the
    oracle's."""
    torch = torch_cuda()
    S, base = (1 << 25) + 4099, 7
    mp = base + S // 3
    q = n // 2 + 1
    r1, r2, _ = oracle.trace(kind, n, 300 + n, base, S)
    exp, eres = oracle.ref_step(n, q, n - 1, 42, 99, base, r1, r2, max_phase=mp, lc_in=3, wm_in=7)
    del r1, r2
    for grid in (0, 5):
        out, stride, res, launch = _planar_step(torch, n, S, kind, 300 + n, base, LAG | (grid << 24), max_phase=mp)
        assert launch["kernel"] == "lag" and (launch["block"], launch["words"]) == one_shape(n)
        assert launch["grid"] == (grid or n_cu(torch))
        got = decode_outputs(out.view(8, stride).cpu().numpy().view(np.uint32), S)
        for k in KEYS:
            np.testing.assert_array_equal(got[k], exp[k], err_msg=f"{k} (grid {grid})")
        assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}, grid
        del out, got


@pytest.mark.parametrize("n", [3, 7, 9])
def test_default_dispatch_lag1024(oracle, n):
    """No switch: at the first size where every CU runs >= 32 lag tiles step_impl
    picks the one-workgroup-per-CU lag shape, 512 x 4 (n = 3: 2^29 slots; n = 7, 9: 2^28).
    Properties over every slot, oracle slices, the tiled kernel's output."""
    torch = torch_cuda()
    S = 32 * 32 * n_cu(torch) * 1024 * lag_words(n)
    base, kind, seed = 1, N.RG_TRACE_AGREE90, 50 + n
    out, stride, res, launch = _planar_step(torch, n, S, kind, seed, base, 0, rng0=5, lc_in=0, wm_in=1)
    assert launch == {"kernel": "lag", "shard": False, "block": one_shape(n)[0], "words": one_shape(n)[1],
                      "grid": n_cu(torch), "windows": 1}, launch
    nw = S // 32
    p = word_planes(out, nw, 0, stride)
    cvq = check_properties(torch, p, S, base, 0, res, 5, res["rng_next"], lc_in=0)
    tw = 2048  # one workgroup tile of the lag kernel, in words
    check_slices(oracle, torch, p, cvq, n, kind, seed, base, 5, n - 1,
                 [0, S - 8192, 32 * (tw - 64), 32 * (nw // 3), 32 * (nw - 2 * tw - 32)])
    del p, cvq
    out2, _, res2, launch2 = _planar_step(torch, n, S, kind, seed, base, TILED, rng0=5, lc_in=0, wm_in=1)
    assert launch2["kernel"] == "tiled"
    assert torch.equal(out, out2)
    assert {k: res[k] for k in RES_CMP} == {k: res2[k] for k in RES_CMP}


SHARD_CASES = [
    # n, world, window sizes, trace kind, lag grid (0 = one WG per CU)
    (5, 2, [300_007], 1, 3),
    (3, 4, [1_000_003, 777], 0, 2),
    (9, 3, [1 << 21], 2, 5),
    (7, 2, [524_288, 131_071], 1, 0),
    (9, 2, [1 << 25], 1, 7),   # 2^24-slot shards: the one-workgroup-per-CU shape
    (5, 2, [1 << 26], 2, 0),   # 2^25-slot shards: the one-workgroup-per-CU shape, all VQ
]


@pytest.mark.parametrize("n,world,sizes,kind,grid", SHARD_CASES)
def test_shard_lag_forced_vs_one_engine_and_oracle(oracle, n, world, sizes, kind, grid):
    """ref_lag_kernel<.., SHARD = true> (forced) in 2-4 shards: after the fix-up and
    the commit fold, outputs, per-rank results and engine states equal one evaluator
    (the tiled kernel at these sizes) and the oracle over the concatenated windows."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, sizes, kind)
    out_s = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    state = {"rng_next": 1234, "last_committed": 3, "commit_watermark": 1, "steps": 0}
    mp = sum(sizes) * 2 // 3
    launches = []
    res_s, st_s, rows, fixed = run_sharded(n, world, sizes, votes, out_s, stride, state=state, max_phase=mp,
                                           diag=LAG | (grid << 24), launches=launches)
    for la in launches:
        assert la["kernel"] == "lag" and la["shard"], la
    assert all(1 <= la["grid"] <= (grid or 2 * n_cu(torch)) for la in launches)
    if sizes[0] >= 1 << 25:
        assert (launches[0]["block"], launches[0]["words"]) == one_shape(n)
    res_1, st_1 = run_single(n, sizes, votes, out_1, stride, state=state, max_phase=mp)
    assert torch.equal(out_s, out_1)
    for w in range(len(sizes)):
        for r in range(world):
            assert {k: res_s[w][r][k] for k in RES_CMP} == {k: res_1[w][k] for k in RES_CMP}, (w, r)
    assert all(st == st_1 for st in st_s)
    assert all(x["flags"] == 0 for x in rows) and all(x["flags"] == 0 for x in fixed)
    planes = out_s.view(8, stride).cpu().numpy().view(np.uint32)
    got = decode_outputs(planes, total)
    base, off, rng, lc = 1, 0, 1234, 3
    for w, S in enumerate(sizes):
        r1, r2, _ = oracle.trace(kind, n, 7, base, S)
        exp, eres = oracle.ref_step(n, n // 2 + 1, n // 2, 42, rng, base, r1, r2, max_phase=mp, lc_in=lc,
                                    wm_in=res_1[w - 1]["commit_watermark"] if w else 1)
        for k in KEYS:
            np.testing.assert_array_equal(got[k][off:off + S], exp[k], err_msg=f"window {w} {k}")
        assert eres["rng_next"] == res_s[w][0]["rng_next"]
        rng, lc = eres["rng_next"], eres["last_committed_max"]
        base += S
        off += ((S + 127) // 128) * 128


@pytest.mark.parametrize("n,world,S,grid", [(5, 3, 600_064, 4), (9, 2, 1 << 22, 0)])
def test_shard_lag_windows_entry_k1(n, world, S, grid):
    """rg_phase_step_shard_windows_async with one window takes the lag kernel as well
    (forced): == the single-window shard entry point == one evaluator."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S], 1, seed=13)
    out_k = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    out_w = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    launches = []
    res_k, st_k, rows_k = run_sharded_windows(n, world, 1, S, votes, out_k, stride, batched_stages=True,
                                              diag=LAG | (grid << 24), launches=launches)
    assert all(la["kernel"] == "lag" and la["shard"] for la in launches), launches
    res_w, st_w, _, _ = run_sharded(n, world, [S], votes, out_w, stride, diag=LAG | (grid << 24))
    assert torch.equal(out_k, out_w)
    for r in range(world):
        assert {k: res_k[0][r][k] for k in RES_CMP} == {k: res_w[0][r][k] for k in RES_CMP}
    assert st_k == st_w
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S], votes, out_1, stride)
    assert torch.equal(out_k, out_1) and all(st == st_1 for st in st_k)


def test_shard_lag_default_dispatch_2e29():
    """No switch: 2^30 slots (n = 5, slot-tiled 1024, as the bench lays them out) over
    2 shards of 2^29 — each shard launch picks ref_lag_kernel<5, 4, 512, true> —
    equals one evaluator over the 2^30 slots (ref_lag_kernel<5, 4, 512, false>):
    outputs, per-rank results, engine states. (Planar planes of 2^30 slots exceed the
    lag kernel's 31-bit buffer offsets, so this shape needs the tiled layout.)"""
    torch = torch_cuda()
    n, S, world, T = 5, 1 << 30, 2, 1024
    P, nw = 4 * n + 1, S // 32
    tiles = nw // T
    i64 = dict(dtype=torch.int64, device="cuda")
    votes = torch.empty(tiles * P * T, dtype=torch.int32, device="cuda")
    out_s = torch.zeros(tiles * 8 * T, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, tile_words=T) as ev:
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 17, 1, S, T, votes.data_ptr())
        ev.sync()
    cnt, cap = S // world, 1 << 24
    rows, fixed, result = (torch.zeros((world, 10), **i64) for _ in range(3))
    recs = [torch.zeros(cap, **i64) for _ in range(world)]
    torch.cuda.synchronize()
    ctxs = [PhaseEvaluator(n, self_lane=2, seed=42, tile_words=T) for _ in range(world)]
    try:
        launches = []
        t0 = [r * cnt // 32 // T for r in range(world)]
        for r in range(world):
            ctxs[r].phase_step_shard_async(votes.data_ptr() + 4 * t0[r] * P * T, out_s.data_ptr() + 4 * t0[r] * 8 * T,
                                           cnt, T, 1 + r * cnt, recs[r].data_ptr(), cap, rows[r].data_ptr())
            launches.append(ctxs[r].last_launch())
        torch.cuda.synchronize()
        g = rows.clone()
        for r in range(world):
            ctxs[r].shard_fixup_async(out_s.data_ptr() + 4 * t0[r] * 8 * T, cnt, T, 1 + r * cnt, recs[r].data_ptr(),
                                      cap, g.data_ptr(), r, world, fixed[r].data_ptr())
        torch.cuda.synchronize()
        fg = fixed.clone()
        for r in range(world):
            ctxs[r].shard_commit_async(fg.data_ptr(), world, 1, S, result[r].data_ptr())
        torch.cuda.synchronize()
        st_s = [ev.get_state() for ev in ctxs]
    finally:
        for ev in ctxs:
            ev.close()
    assert all(la == {"kernel": "lag", "shard": True, "block": 512, "words": 4, "grid": n_cu(torch),
                      "windows": 1} for la in launches), launches
    out_1 = torch.zeros_like(out_s)
    res_1 = torch.zeros(10, **i64)
    with PhaseEvaluator(n, self_lane=2, seed=42, tile_words=T) as ev:
        ev.phase_step_async(votes.data_ptr(), out_1.data_ptr(), S, T, slot_base=1, result_ptr=res_1.data_ptr())
        assert ev.last_launch()["kernel"] == "lag"
        st_1 = ev.get_state()
    assert torch.equal(out_s, out_1)
    r1 = res_1.cpu().numpy().view(np.uint64).tolist()
    rows_h = rows.cpu().numpy().view(np.uint64)
    for r, x in enumerate(result.cpu().numpy().view(np.uint64).tolist()):
        assert x[:9] == r1[:9] and x[9] == 0, r
    assert all(st == st_1 for st in st_s)
    assert int(rows_h[:, 4].sum()) == r1[4] > 0
    assert int(rows_h[:, 9].max()) == 0 and int(fixed.cpu().numpy().view(np.uint64)[:, 9].max()) == 0


def test_shard_lag_records_overflow_flagged():
    torch = torch_cuda()
    n, S = 5, 200_000
    votes, stride, total = make_votes(n, [S], 0)
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    launches = []
    res, _, rows, fixed = run_sharded(n, 2, [S], votes, out, stride, cap=16, diag=LAG | (3 << 24),
                                      launches=launches)
    assert all(la["kernel"] == "lag" for la in launches)
    assert rows[0]["n_draws"] > 16  # the step wrote the first 16 records and counted the rest
    assert fixed[0]["flags"] & 8 and res[0][0]["flags"] & 8  # the fix-up flags the incomplete patch


MW_CASES = [
    # n, world, K windows, window slots, trace kind, lag grid (0 = one WG per CU)
    (5, 2, 4, 300_032, 1, 3),
    (9, 3, 3, 1 << 20, 2, 5),
    (3, 4, 5, 100_096, 0, 2),
    (9, 2, 6, 1 << 22, 1, 0),
    (7, 1, 3, 266_240, 1, 1),   # one workgroup takes every ticket of every window in turn
    (5, 3, 2, (1 << 24) + 384, 1, 0),  # ragged shards, the 512 x 4 shape over two windows
]


@pytest.mark.parametrize("n,world,K,S,kind,grid", MW_CASES)
def test_shard_lag_windows_forced_vs_oracle(oracle, n, world, K, S, kind, grid):
    """The multi-window lag launch (ref_lag_kernel<.., SHARD, .., MW = true>: tickets
    window-major over the K windows, one look-back chain, draw-record base and row per
    window), forced, in 1-4 shards: the K windows' pre-fix-up rows equal the tiled
    K-window launch's; after the batched fix-up and commit, outputs, per-window results
    and engine states equal the tiled K-window pipeline, one evaluator window by window,
    and the oracle over the concatenated windows (one StdRng stream across them)."""
    torch = torch_cuda()
    votes, stride, total = make_votes(n, [S] * K, kind, seed=31 + n)
    state = {"rng_next": 777, "last_committed": 4, "commit_watermark": 1, "steps": 0}
    mp = K * S * 3 // 4
    launches = []
    out_m = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_m, st_m, rows_m = run_sharded_windows(n, world, K, S, votes, out_m, stride, state=state, max_phase=mp,
                                              batched_stages=True, diag=LAG | (grid << 24), launches=launches)
    for la in launches:
        assert la["kernel"] == "lag" and la["shard"] and la["windows"] == K, la
        assert (la["block"], la["words"]) == one_shape(n), la
        assert 1 <= la["grid"] <= (grid or n_cu(torch)), la
    tl = []
    out_t = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_t, st_t, rows_t = run_sharded_windows(n, world, K, S, votes, out_t, stride, state=state, max_phase=mp,
                                              batched_stages=True, diag=TILED, launches=tl)
    assert all(la["kernel"] == "tiled" for la in tl), tl
    for w in range(K):
        for r in range(world):
            assert rows_m[w][r] == rows_t[w][r], (w, r)
            assert {k: res_m[w][r][k] for k in RES_CMP} == {k: res_t[w][r][k] for k in RES_CMP}, (w, r)
            assert res_m[w][r]["flags"] == 0
    assert torch.equal(out_m, out_t)
    assert st_m == st_t
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S] * K, votes, out_1, stride, state=state, max_phase=mp)
    assert torch.equal(out_m, out_1) and all(st == st_1 for st in st_m)
    for w in range(K):
        assert {k: res_m[w][0][k] for k in RES_CMP} == {k: res_1[w][k] for k in RES_CMP}, w
    got = decode_outputs(out_m.view(8, stride).cpu().numpy().view(np.uint32), total)
    base, off, rng, lc = 1, 0, 777, 4
    Sp = ((S + 127) // 128) * 128
    for w in range(K):
        r1, r2, _ = oracle.trace(kind, n, 31 + n, base, S)
        exp, eres = oracle.ref_step(n, n // 2 + 1, n // 2, 42, rng, base, r1, r2, max_phase=mp, lc_in=lc,
                                    wm_in=res_1[w - 1]["commit_watermark"] if w else 1)
        for k in KEYS:
            np.testing.assert_array_equal(got[k][off:off + S], exp[k], err_msg=f"window {w} {k}")
        assert {k: eres[k] for k in RES_CMP if k != "flags"} == {k: res_m[w][0][k] for k in RES_CMP if k != "flags"}
        rng, lc = eres["rng_next"], eres["last_committed_max"]
        base += S
        off += Sp


def test_shard_lag_windows_default_dispatch_c5_shape(oracle):
    """No switch, the 8-GPU C5 per-rank launch shape: n = 9, 32 windows of 2^24 slots
    split over 2 shards (2^23-slot shards, as 2^26-slot C5 windows over 8 GPUs), slot-tiled
    1024 as the bench lays them out. Each shard's 32-window launch (2^28 slots) picks the
    multi-window lag kernel; after the batched fix-up and commit the outputs, the 32
    per-window results and the engine states equal one evaluator window by window, and
    oracle slices at window and shard boundaries hold."""
    torch = torch_cuda()
    n, world, K, T = 9, 2, 32, 1024
    S_win = 1 << 24
    S, P = S_win // world, 4 * n + 1
    tiles_win, tiles_sh = S_win // 32 // T, S // 32 // T
    total = K * S_win
    i64 = dict(dtype=torch.int64, device="cuda")
    votes = torch.empty(total // 32 // T * P * T, dtype=torch.int32, device="cuda")
    out_s = torch.zeros(total // 32 // T * 8 * T, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, tile_words=T) as ev:
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 23, 1, total, T, votes.data_ptr())
        ev.sync()
    cap = S // 8
    rows = [torch.zeros((K, 10), **i64) for _ in range(world)]
    fixed = [torch.zeros((K, 10), **i64) for _ in range(world)]
    result = [torch.zeros((K, 10), **i64) for _ in range(world)]
    recs = [torch.zeros(K * cap, **i64) for _ in range(world)]
    torch.cuda.synchronize()
    ctxs = [PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T) for _ in range(world)]
    try:
        launches = []
        for r in range(world):
            t0 = r * tiles_sh
            ctxs[r].phase_step_shard_windows_async(K, votes.data_ptr() + 4 * t0 * P * T, tiles_win * P * T,
                                                   out_s.data_ptr() + 4 * t0 * 8 * T, tiles_win * 8 * T, S, T,
                                                   1 + r * S, S_win, recs[r].data_ptr(), cap, rows[r].data_ptr())
            launches.append(ctxs[r].last_launch())
        torch.cuda.synchronize()
        g = torch.stack(rows).contiguous()
        for r in range(world):
            t0 = r * tiles_sh
            ctxs[r].shard_fixup_windows_async(K, out_s.data_ptr() + 4 * t0 * 8 * T, tiles_win * 8 * T, S, T, 1 + r * S,
                                              S_win, recs[r].data_ptr(), cap, g.data_ptr(), r, world,
                                              fixed[r].data_ptr())
        torch.cuda.synchronize()
        fg = torch.stack(fixed).contiguous()
        for r in range(world):
            ctxs[r].shard_commit_windows_async(K, fg.data_ptr(), world, 1, S_win, result[r].data_ptr())
        torch.cuda.synchronize()
        st_s = [ev.get_state() for ev in ctxs]
    finally:
        for ev in ctxs:
            ev.close()
    assert all(la == {"kernel": "lag", "shard": True, "block": 512, "words": 4, "grid": n_cu(torch),
                      "windows": K} for la in launches), launches
    rows_h = [x.cpu().numpy().view(np.uint64) for x in rows]
    assert all(int(x[:, 9].max()) == 0 for x in rows_h)
    out_1 = torch.zeros_like(out_s)
    res_1 = torch.zeros((K, 10), **i64)
    with PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T) as ev:
        for w in range(K):
            t0 = w * tiles_win
            ev.phase_step_async(votes.data_ptr() + 4 * t0 * P * T, out_1.data_ptr() + 4 * t0 * 8 * T, S_win, T,
                                slot_base=1 + w * S_win, result_ptr=res_1[w].data_ptr())
        st_1 = ev.get_state()
    assert torch.equal(out_s, out_1)
    r1 = res_1.cpu().numpy().view(np.uint64)
    for r in range(world):
        assert result[r].cpu().numpy().view(np.uint64)[:, :9].tolist() == r1[:, :9].tolist(), r
        assert int(result[r].cpu().numpy().view(np.uint64)[:, 9].max()) == 0
    assert all(st == st_1 for st in st_s)
    assert int(sum(x[:, 4].sum() for x in rows_h)) == int(r1[:, 4].sum()) > 0
    del votes, out_1
    p = word_planes(out_s, total // 32, T, 0)
    cvq = popc(torch, ~p[0] & p[1])
    assert int(cvq.sum()) == int(r1[:, 4].sum())
    slices = [0, S - 4096, S_win - 4096, 5 * S_win + S - 2048, 17 * S_win + 32 * 1000, total - 8192]
    check_slices(oracle, torch, p, cvq, n, N.RG_TRACE_AGREE90, 23, 1, 0, 4, slices)
