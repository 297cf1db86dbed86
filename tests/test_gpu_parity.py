"""GPU parity tests: the HIP path through the C ABI vs the oracle, bit-exact.

Run on an MI355X: python -m pytest tests -m gpu -x -q
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs

pytestmark = pytest.mark.gpu

RES_CMP = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max",
           "first_undecided", "rng_next", "commit_watermark"]


def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def run_ref(n, q, self_lane, seed, rng_base, slot_base, r1, r2, max_phase=0, lc_in=0, wm_in=1):
    with PhaseEvaluator(n, quorum=q, self_lane=self_lane, mode="ref", seed=seed) as ev:
        ev.set_state(rng_next=rng_base, last_committed=lc_in, commit_watermark=wm_in)
        w = PhaseWindow.from_codes(r1, r2, slot_base=slot_base)
        out, res = ev.phase_step_host(w, max_phase=max_phase)
        st = ev.get_state()
    assert res["flags"] == 0
    assert st["rng_next"] == res["rng_next"] and st["last_committed"] == res["last_committed_max"]
    assert st["commit_watermark"] == res["commit_watermark"]
    return decode_outputs(out, r1.shape[0]), res, out


def run_wmvc(n, q, fp1, self_lane, coin_seed, epoch, phase, slot_base, r1, r2, state, lc_in=0, wm_in=1):
    with PhaseEvaluator(n, quorum=q, decide_threshold=fp1, self_lane=self_lane, mode="wmvc",
                        coin_seed=coin_seed, epoch=epoch) as ev:
        ev.set_state(last_committed=lc_in, commit_watermark=wm_in)
        w = PhaseWindow.from_codes(r1, r2, state, slot_base=slot_base)
        out, res = ev.phase_step_host(w, phase=phase)
    assert res["flags"] == 0
    return decode_outputs(out, r1.shape[0]), res, out


def assert_same(got, exp, res, eres):
    for k in ("r1", "r2own", "dec", "committed", "value"):
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(GOLDEN) if f.startswith("trace_")))
def test_golden_traces(golden, name):
    g = golden(name)
    p = json.loads(str(g["params"]))
    if str(g["mode"]) == "ref":
        got, res, _ = run_ref(p["n"], p["q"], p["self_lane"], p["seed"], p["rng_base"], p["slot_base"],
                              g["r1"], g["r2"], p["max_phase"], p["lc_in"], p["wm_in"])
    else:
        got, res, _ = run_wmvc(p["n"], p["q"], p["fp1"], p["self_lane"], p["coin_seed"], p["epoch"],
                               p["phase"], p["slot_base"], g["r1"], g["r2"], g["state"], p["lc_in"], p["wm_in"])
    exp = {k: g[f"out_{k}"] for k in ("r1", "r2own", "dec", "committed", "value")}
    eres = dict(zip(RES_CMP, [int(x) for x in g["result"]]))
    assert_same(got, exp, res, eres)


@pytest.mark.parametrize("n,q", [(3, 2), (4, 3), (4, 2), (5, 3), (7, 4), (9, 5)])
def test_truth_tables_exhaustive(golden, n, q):
    """Every one of the 4^n received-vote vectors as one slot each."""
    g = golden(f"truth_n{n}_q{q}.npz")
    idx = np.arange(4 ** n)
    vecs = np.stack([(idx >> (2 * j)) & 3 for j in range(n)], axis=1).astype(np.uint8)
    zeros = np.zeros_like(vecs)
    # R1 = every vector: round-1 result (REF rule) ; no self lane so R2 is untouched
    got, _, _ = run_ref(n, q, -1, 1, 0, 1, vecs, zeros)
    np.testing.assert_array_equal(got["r1"], g["ref_round1"])
    # R2 = every vector: decision = count_votes
    got, _, _ = run_ref(n, q, -1, 1, 0, 1, zeros, vecs)
    np.testing.assert_array_equal(got["dec"], g["count_votes"])
    # WMVC round 1 classification
    fp1 = (n - 1) // 2 + 1
    st = (idx & 1).astype(np.uint8)
    got, _, _ = run_wmvc(n, q, fp1, -1, 9, 0, 1, 1, vecs, zeros, st)
    np.testing.assert_array_equal(got["r1"], g["wmvc_round1"])
    # WMVC round 2 classes (R1 = all V0 so round 1 is live)
    got, _, _ = run_wmvc(n, q, fp1, -1, 9, 0, 4, 1, zeros, vecs, st)
    cls = g["wmvc_round2_class"]
    import oracle_lib
    coins = oracle_lib.coin_range(9, 0, 4, 1, 4 ** n)
    exp_dec = np.where(cls == 0, 0, np.where(cls == 1, 1, 3))
    exp_val = np.select([cls == 0, cls == 1, cls == 2, cls == 3, cls == 4, cls == 5],
                        [np.zeros_like(st), np.ones_like(st), np.zeros_like(st), np.ones_like(st),
                         coins.astype(np.uint8), st])
    np.testing.assert_array_equal(got["dec"], exp_dec)
    np.testing.assert_array_equal(got["value"], exp_val)


SIZES = [1, 31, 32, 33, 127, 128, 129, 4097, 100003, (1 << 20) + 17]


@pytest.mark.parametrize("S", SIZES)
@pytest.mark.parametrize("n", [3, 5, 9])
def test_random_ref_vs_oracle(oracle, n, S):
    for kind in (0, 1, 2):
        r1, r2, _ = oracle.trace(kind, n, 1000 + S, 7, S)
        q = n // 2 + 1
        exp, eres = oracle.ref_step(n, q, n // 2, 42, 123, 7, r1, r2, max_phase=7 + S // 2, lc_in=2, wm_in=7)
        got, res, _ = run_ref(n, q, n // 2, 42, 123, 7, r1, r2, max_phase=7 + S // 2, lc_in=2, wm_in=7)
        assert_same(got, exp, res, eres)


@pytest.mark.parametrize("n", list(range(1, 17)))
def test_every_replica_count(oracle, n):
    S = 70001
    r1, r2, st = oracle.trace(0, n, n, 1, S)
    q = n // 2 + 1
    exp, eres = oracle.ref_step(n, q, n - 1, 5, 0, 1, r1, r2)
    got, res, _ = run_ref(n, q, n - 1, 5, 0, 1, r1, r2)
    assert_same(got, exp, res, eres)
    fp1 = (n - 1) // 2 + 1
    exp, eres = oracle.wmvc_step(n, q, fp1, 0, 3, 1, 2, 1, r1, r2, st)
    got, res, _ = run_wmvc(n, q, fp1, 0, 3, 1, 2, 1, r1, r2, st)
    assert_same(got, exp, res, eres)


@pytest.mark.parametrize("slot_base", [1, 32, 33, 511, 512, 1000003])
def test_wmvc_unaligned_coins(oracle, slot_base):
    n, S = 5, 20000
    r1, r2, st = oracle.trace(2, n, 3, slot_base, S)  # split: all-'?' round 2 -> coins
    r1 = np.where(r1 == 2, 1, r1).astype(np.uint8)     # WMVC states are binary
    exp, eres = oracle.wmvc_step(n, 3, 3, 0, 77, 5, 3, slot_base, r1, r2, st)
    got, res, _ = run_wmvc(n, 3, 3, 0, 77, 5, 3, slot_base, r1, r2, st)
    assert_same(got, exp, res, eres)


def test_multi_window_continuity(oracle):
    """Three consecutive windows (ragged sizes) == one window: same outputs, same
    StdRng position, watermark and last_committed (device state carried)."""
    n, q = 5, 3
    sizes = [1000, 70001, 333]
    S = sum(sizes)
    r1, r2, _ = oracle.trace(0, n, 77, 1, S)
    exp, eres = oracle.ref_step(n, q, 4, 42, 0, 1, r1, r2)
    with PhaseEvaluator(n, self_lane=4, seed=42) as ev:
        outs, base = [], 1
        for sz in sizes:
            sl = slice(base - 1, base - 1 + sz)
            w = PhaseWindow.from_codes(r1[sl], r2[sl], slot_base=base)
            out, res = ev.phase_step_host(w)
            outs.append(decode_outputs(out, sz))
            base += sz
        st = ev.get_state()
    for k in exp:
        np.testing.assert_array_equal(np.concatenate([o[k] for o in outs]), exp[k], err_msg=k)
    assert st["rng_next"] == eres["rng_next"]
    assert st["last_committed"] == eres["last_committed_max"]
    assert st["steps"] == 3


def test_device_path_large_properties(oracle):
    """Full-size (C2 shape x 16 windows = 16M slots) device-resident step:
    size-independent properties + window-split equivalence + sampled oracle slices."""
    torch = torch_cuda()
    n, S = 5, 1 << 24
    stride = ((S + 127) // 128) * 4
    votes = torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    out1 = torch.empty(8 * stride, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, self_lane=4, seed=42) as ev:
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 42, 1, S, stride, votes.data_ptr())
        ev.phase_step_async(votes.data_ptr(), out1.data_ptr(), S, stride, slot_base=1)
        res1 = ev.last_result()
        st1 = ev.get_state()
    planes = out1.view(8, stride).cpu().numpy().view(np.uint32)
    dec = decode_outputs(planes, S)
    assert res1["n_decided"] == int(dec["committed"].sum())
    assert res1["n_v1"] == int(dec["value"].sum())
    assert res1["n_draws"] == int((dec["r1"] == 2).sum()) == st1["rng_next"]
    assert ((dec["dec"] <= 1) == (dec["committed"] == 1)).all()
    # oracle on slices at both ends (draw offsets need the prefix count)
    r1, r2, _ = oracle.trace(1, n, 42, 1, 4096)
    exp, _ = oracle.ref_step(n, 3, 4, 42, 0, 1, r1, r2)
    for k in exp:
        np.testing.assert_array_equal(dec[k][:4096], exp[k], err_msg=k)
    tail0 = S - 4096
    r1, r2, _ = oracle.trace(1, n, 42, 1 + tail0, 4096)
    k0 = int((dec["r1"][:tail0] == 2).sum())
    exp, _ = oracle.ref_step(n, 3, 4, 42, k0, 1 + tail0, r1, r2)
    for k in exp:
        np.testing.assert_array_equal(dec[k][tail0:], exp[k], err_msg=k)
    # the same slots as 4 windows on a fresh context
    out2 = torch.empty_like(out1)
    with PhaseEvaluator(n, self_lane=4, seed=42) as ev:
        q4 = S // 4
        for i in range(4):
            off = i * q4 // 32
            ev.phase_step_async(votes.data_ptr() + 4 * off, out2.data_ptr() + 4 * off, q4, stride,
                                slot_base=1 + i * q4)
        st2 = ev.get_state()
    assert torch.equal(out1, out2)
    assert st1["rng_next"] == st2["rng_next"] and st1["last_committed"] == st2["last_committed"]
    assert st1["commit_watermark"] == st2["commit_watermark"]


def test_trace_generator_matches_oracle(oracle):
    torch = torch_cuda()
    for n, S, kind in ((5, 10001, 1), (9, 4096, 0), (16, 777, 2)):
        stride = ((S + 127) // 128) * 4
        votes = torch.zeros((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
        with PhaseEvaluator(n) as ev:
            ev.trace_generate_async(kind, 99, 5, S, stride, votes.data_ptr())
            ev.sync()
        planes = votes.view(4 * n + 1, stride).cpu().numpy().view(np.uint32)
        r1, r2, st = oracle.trace(kind, n, 99, 5, S)
        np.testing.assert_array_equal(planes[: 2 * n], oracle.pack_planes(r1, stride))
        np.testing.assert_array_equal(planes[2 * n: 4 * n], oracle.pack_planes(r2, stride))
        bits = np.unpackbits(planes[4 * n].view(np.uint8), bitorder="little")[:S]
        np.testing.assert_array_equal(bits, st)


@pytest.mark.parametrize("n", [5, 7, 16])
def test_digest_majority(oracle, golden, n):
    torch = torch_cuda()
    cases = []
    if n in (5, 7):
        g = golden(f"digest_n{n}.npz")
        cases.append((g["digests"], g["state"]))
    for S_ in (131074, 100003):  # even stride: 16-B vector path; odd: 8-B path
        d = oracle.digest_trace(n, 4, 1, S_)
        cases.append((d, oracle.digest_majority(d, n // 2 + 1)))
    S = 100003
    for dg, exp in cases:
        S = dg.shape[1]
        stride = ((S + 127) // 128) * 4
        dgt = torch.from_numpy(np.ascontiguousarray(dg).view(np.int64)).cuda()
        st = torch.zeros(stride, dtype=torch.int32, device="cuda")
        with PhaseEvaluator(n) as ev:
            ev.digest_majority_async(dgt.data_ptr(), S, st.data_ptr(), S)
            ev.sync()
        bits = np.unpackbits(st.cpu().numpy().view(np.uint8), bitorder="little")[:S]
        np.testing.assert_array_equal(bits, exp)
    # device trace generator for digests
    stride = S
    dgt = torch.zeros(n * S, dtype=torch.int64, device="cuda")
    with PhaseEvaluator(n) as ev:
        ev.digest_trace_async(4, 1, S, S, dgt.data_ptr())
        ev.sync()
    np.testing.assert_array_equal(dgt.view(n, S).cpu().numpy().view(np.uint64), d)


def test_coins_and_draws(oracle, golden):
    torch = torch_cuda()
    g = golden("rng_fixtures.npz")
    with PhaseEvaluator(5, seed=42, coin_seed=7, epoch=3) as ev:
        d = torch.zeros(64, dtype=torch.int64, device="cuda")
        ev.ref_draws_async(0, 64, d.data_ptr())
        c = torch.zeros(32 * 4, dtype=torch.int32, device="cuda")
        ev.sync()
        np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), g["stdrng42_next_u64"])
        for pi, phase in enumerate(g["coin_phases"]):
            ev.coin_async(int(g["coin_slot_base"]), 1024, int(phase), c.data_ptr())
            ev.sync()
            bits = np.unpackbits(c.cpu().numpy().view(np.uint8), bitorder="little")[:1024]
            np.testing.assert_array_equal(bits, g["coins_seed7_epoch3"][pi])
        d2 = torch.zeros(1000, dtype=torch.int64, device="cuda")
        ev.ref_draws_async(10 ** 9, 1000, d2.data_ptr())
        ev.sync()
        np.testing.assert_array_equal(d2.cpu().numpy().view(np.uint64), oracle.ref_draws(42, 10 ** 9, 1000))


def test_argument_errors():
    torch = torch_cuda()
    with PhaseEvaluator(5) as ev:
        buf = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
        with pytest.raises(N.RabiaGpuError) as e:
            ev.phase_step_async(buf.data_ptr(), buf.data_ptr(), 0, 4)
        assert e.value.code == N.RG_EINVAL
        with pytest.raises(N.RabiaGpuError):
            ev.phase_step_async(buf.data_ptr(), buf.data_ptr(), 1000, 30)      # stride too small
        with pytest.raises(N.RabiaGpuError):
            ev.phase_step_async(buf.data_ptr() + 4, buf.data_ptr(), 100, 4)    # misaligned
    with pytest.raises(N.RabiaGpuError):
        PhaseEvaluator(17)
    with pytest.raises(N.RabiaGpuError):
        PhaseEvaluator(5, quorum=6)
    with pytest.raises(N.RabiaGpuError):
        with PhaseEvaluator(5, mode="wmvc") as ev:
            w = PhaseWindow(5, 10)
            ev.phase_step_host(w, phase=0)


def test_state_resume_roundtrip(oracle):
    """Persist the device engine state and resume on a new context (checkpoint
    of current/last_committed_phase, rabia-core/src/persistence.rs:9-42)."""
    n = 5
    r1, r2, _ = oracle.trace(0, n, 5, 1, 5000)
    with PhaseEvaluator(n, self_lane=0, seed=3) as ev:
        w = PhaseWindow.from_codes(r1[:2500], r2[:2500], slot_base=1)
        ev.phase_step_host(w)
        saved = ev.get_state()
    with PhaseEvaluator(n, self_lane=0, seed=3) as ev:
        ev.set_state(**saved)
        w = PhaseWindow.from_codes(r1[2500:], r2[2500:], slot_base=2501)
        out, res = ev.phase_step_host(w)
    exp, eres = oracle.ref_step(n, 3, 0, 3, 0, 1, r1, r2)
    got = decode_outputs(out, 2500)
    for k in exp:
        np.testing.assert_array_equal(got[k], exp[k][2500:], err_msg=k)
    assert res["rng_next"] == eres["rng_next"]
    assert res["last_committed_max"] == eres["last_committed_max"]


@pytest.mark.parametrize("T", [64, 1024, 4096])
@pytest.mark.parametrize("mode", ["ref", "wmvc"])
def test_slot_tiled_layout(oracle, T, mode):
    """The slot-tiled plane arrangement gives bit-identical results."""
    n, S = 5, 300_007
    r1, r2, st = oracle.trace(0, n, T, 1, S)
    if mode == "ref":
        exp, eres = oracle.ref_step(n, 3, 4, 42, 7, 1, r1, r2)
    else:
        exp, eres = oracle.wmvc_step(n, 3, 3, 4, 42, 2, 3, 1, r1, r2, st)
    with PhaseEvaluator(n, self_lane=4, seed=42, mode=mode, coin_seed=42, epoch=2, tile_words=T) as ev:
        ev.set_state(rng_next=7 if mode == "ref" else 0)
        out, res = ev.phase_step_host(PhaseWindow.from_codes(r1, r2, st, slot_base=1), phase=3)
    assert_same(decode_outputs(out, S), exp, res, eres)


def test_device_tiled_generator_matches_planar(oracle):
    """Device trace generator writing the tiled arrangement == planar arrangement."""
    torch = torch_cuda()
    from rabia_amd.engine import from_tiled
    n, S, T = 5, 1 << 20, 1024
    nw = S // 32
    vt = torch.zeros(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, tile_words=T) as ev:
        ev.trace_generate_async(1, 5, 1, S, T, vt.data_ptr())
        ev.sync()
    planar = from_tiled(vt.cpu().numpy().view(np.uint32), 4 * n + 1, nw, T, nw)
    r1, r2, st = oracle.trace(1, n, 5, 1, S)
    np.testing.assert_array_equal(planar[: 2 * n], oracle.pack_planes(r1, nw))
    np.testing.assert_array_equal(planar[2 * n: 4 * n], oracle.pack_planes(r2, nw))


@pytest.mark.parametrize("n", [3, 5, 7, 9, 16])
def test_wmvc_cluster_vs_oracle(oracle, golden, n):
    """Weak-MVC to termination over all replicas of each slot (config 3)."""
    torch = torch_cuda()
    q, fp1 = n // 2 + 1, (n - 1) // 2 + 1
    S = 50_001
    stride = ((S + 127) // 128) * 4
    states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
    info = torch.zeros(S, dtype=torch.int32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
        ev.cluster_trace_async(42, 1, S, stride, states.data_ptr())
        ev.wmvc_cluster_async(states.data_ptr(), stride, S, 1, 99, 32, info.data_ptr(), stats.data_ptr())
        ev.sync()
    st = oracle.cluster_trace(n, 42, 1, S)
    planes = states.view(n, stride).cpu().numpy().view(np.uint32)
    for r in range(n):
        bits = np.unpackbits(planes[r].view(np.uint8), bitorder="little")[:S]
        np.testing.assert_array_equal(bits, st[:, r])
    exp = oracle.wmvc_cluster(n, q, fp1, 7, 3, 99, 32, 1, st)
    got = info.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, exp)
    sv = stats.cpu().numpy().view(np.uint64)
    dec = exp & 255
    assert sv[0] == (dec != 3).sum() and sv[1] == (dec == 1).sum()
    assert sv[2] == ((exp >> 8) & 255).sum() and sv[3] == ((exp >> 8) & 255).max() and sv[6] == S
    if n in (3, 5, 7):
        g = golden(f"cluster_n{n}.npz")
        np.testing.assert_array_equal(got[: g["info"].shape[0]], g["info"])


@pytest.mark.parametrize("S", [1, 33, 50_001, 1_000_003, (1 << 24) + 77])
def test_wmvc_cluster_fused_bitmaps(S):
    """rg_wmvc_cluster_bitmaps_async: the cluster run's decided / V1 bitmaps built in the
    cluster kernel equal rg_cluster_bitmap_async's over the same info words, every word
    written (buffers start as garbage), info and statistics unchanged. Sizes cover one
    partial word, a chunk rounded up to whole words with empty trailing workgroups
    (1,000,003) and the grid grown past 2,048 workgroups (2^24 + 77)."""
    torch = torch_cuda()
    n = 5
    stride = ((S + 127) // 128) * 4
    nw = (S + 31) // 32
    states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
    info_a = torch.zeros(S, dtype=torch.int32, device="cuda")
    info_b = torch.full((S,), -1, dtype=torch.int32, device="cuda")
    stats_a = torch.zeros(8, dtype=torch.int64, device="cuda")
    stats_b = torch.zeros(8, dtype=torch.int64, device="cuda")
    bm_a = torch.zeros((2, nw), dtype=torch.int32, device="cuda")
    bm_b = torch.full((2, nw), -1, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
        ev.cluster_trace_async(42, 1, S, stride, states.data_ptr())
        ev.wmvc_cluster_async(states.data_ptr(), stride, S, 1, 99, 32, info_a.data_ptr(), stats_a.data_ptr())
        ev.cluster_bitmap_async(info_a.data_ptr(), S, bm_a[0].data_ptr(), bm_a[1].data_ptr())
        ev.wmvc_cluster_bitmaps_async(states.data_ptr(), stride, S, 1, 99, 32, info_b.data_ptr(),
                                      bm_b[0].data_ptr(), bm_b[1].data_ptr(), stats_b.data_ptr())
        ev.sync()
    torch.testing.assert_close(info_b, info_a, rtol=0, atol=0)
    torch.testing.assert_close(stats_b, stats_a, rtol=0, atol=0)
    torch.testing.assert_close(bm_b, bm_a, rtol=0, atol=0)
    if S <= 50_001:  # the bitmaps against the info words directly
        dec = info_a.cpu().numpy() & 255
        bits = np.unpackbits(bm_b.cpu().numpy().view(np.uint8), axis=1, bitorder="little")
        np.testing.assert_array_equal(bits[0, :S], dec <= 1)
        np.testing.assert_array_equal(bits[1, :S], dec == 1)
        assert not bits[:, S:].any()


@pytest.mark.parametrize("slot_base", [512, 1 + 32 * 7, 1000, (1 << 40) + 300, 479])
def test_wmvc_cluster_slot_base_offsets(oracle, slot_base):
    """The coin table's block alignment (slot_base mod 512: a chunk's slots start inside
    an LDS coin block at a whole-word and a bit offset, both, or none) against the CPU
    restatement, n = 5, and past the 8 tabled phases (inline coins) for a few slots."""
    torch = torch_cuda()
    n, S = 5, 300_001
    q, fp1 = n // 2 + 1, (n - 1) // 2 + 1
    stride = ((S + 127) // 128) * 4
    states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
    info = torch.zeros(S, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
        ev.cluster_trace_async(42, slot_base, S, stride, states.data_ptr())
        ev.wmvc_cluster_async(states.data_ptr(), stride, S, slot_base, 99, 32, info.data_ptr())
        ev.sync()
    exp = oracle.wmvc_cluster(n, q, fp1, 7, 3, 99, 32, slot_base, oracle.cluster_trace(n, 42, slot_base, S))
    got = info.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, exp)
    assert ((exp >> 8) & 255).max() > 8  # some slots ran past the coin table
