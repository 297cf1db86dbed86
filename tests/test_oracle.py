"""CPU tests: pin the oracle (C restatement) against the golden fixtures, the
RFC 7539 / openssl ChaCha20 keystreams and the independent Python restatement.
No GPU needed."""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import rabia_ref as R
from conftest import GOLDEN, ROOT

TRUTH = [(3, 2), (4, 3), (4, 2), (5, 3), (7, 4), (9, 5)]


@pytest.mark.parametrize("n,q", TRUTH)
def test_truth_tables_c_oracle(oracle, golden, n, q):
    """count_votes (messages.rs:185-211) and the round-1 rule (engine.rs:495-505)
    over every received-vote vector, C oracle vs the Python-generated fixture."""
    g = golden(f"truth_n{n}_q{q}.npz")
    if n == 9:  # 262k ctypes calls: check a strided sample on CPU (full table runs on GPU)
        idx = np.arange(0, 4 ** n, 7)
    else:
        idx = np.arange(4 ** n)
    lib = oracle.load()
    codes = np.stack([(idx >> (2 * j)) & 3 for j in range(n)], axis=1).astype(np.uint8)
    p = oracle.u8p
    cv = np.array([lib.or_count_votes(c.ctypes.data_as(p), n, q) for c in codes], np.uint8)
    r1 = np.array([lib.or_ref_round1(c.ctypes.data_as(p), n, q) for c in codes], np.uint8)
    np.testing.assert_array_equal(cv, g["count_votes"][idx])
    np.testing.assert_array_equal(r1, g["ref_round1"][idx])


def test_truth_table_spot_semantics(golden):
    """Hand-checked rows: priority V0 > V1 > VQ when q is not a strict majority."""
    g = golden("truth_n4_q2.npz")
    def idx(v):
        return sum(c << (2 * j) for j, c in enumerate(v))
    assert g["count_votes"][idx([1, 1, 0, 0])] == R.V0      # c0 = c1 = 2 >= q: V0 wins
    assert g["count_votes"][idx([2, 2, 1, 3])] == R.VQ
    assert g["ref_round1"][idx([0, 1, 2, 3])] == R.VQ       # |votes| = 3 >= q, no majority
    g5 = golden("truth_n5_q3.npz")
    assert g5["ref_round1"][idx([0, 1, 3, 3, 3])] == R.NONE  # pending: 2 votes < q
    assert g5["count_votes"][idx([2, 2, 2, 0, 1])] == R.VQ
    assert g5["wmvc_round2_class"][idx([2, 2, 2, 2, 2])] == 4  # all '?': coin


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(GOLDEN) if f.startswith("trace_")))
def test_trace_fixtures_c_oracle(oracle, golden, name):
    g = golden(name)
    params = json.loads(str(g["params"]))
    n = params["n"]
    # inputs: the committed vectors equal the C restatement of the generator
    r1, r2, st = oracle.trace(int(g["kind"]), n, int(g["trace_seed"]), params["slot_base"], g["r1"].shape[0])
    np.testing.assert_array_equal(r1, g["r1"])
    np.testing.assert_array_equal(r2, g["r2"])
    np.testing.assert_array_equal(st, g["state"])
    if str(g["mode"]) == "ref":
        out, res = oracle.ref_step(n, params["q"], params["self_lane"], params["seed"], params["rng_base"],
                                   params["slot_base"], g["r1"], g["r2"], params["max_phase"],
                                   params["lc_in"], params["wm_in"])
    else:
        out, res = oracle.wmvc_step(n, params["q"], params["fp1"], params["self_lane"], params["coin_seed"],
                                    params["epoch"], params["phase"], params["slot_base"], g["r1"], g["r2"],
                                    g["state"], params["lc_in"], params["wm_in"])
    for k in out:
        np.testing.assert_array_equal(out[k], g[f"out_{k}"], err_msg=k)
    assert [res[k] for k in oracle.RES_KEYS] == [int(x) for x in g["result"]]


def test_chacha20_kat(oracle):
    """ChaCha core at 20 rounds vs RFC 7539 A.1 and openssl keystreams (committed)."""
    with open(os.path.join(GOLDEN, "chacha20_kat.json")) as f:
        kat = json.load(f)
    assert kat["cases"][0]["keystream_hex"].startswith("76b8e0ada0f13d90405d6ae55386bd28")  # RFC 7539 A.1 #1
    for c in kat["cases"]:
        got = oracle.chacha_block(c["key_words"], c["counter"], 0, 20)
        assert struct.pack("<16I", *[int(x) for x in got]).hex() == c["keystream_hex"]
        py = R.chacha_block(c["key_words"], c["counter"], 0, 20)
        assert struct.pack("<16I", *py).hex() == c["keystream_hex"]


def test_seed_from_u64_c_vs_python(oracle):
    for seed in (0, 1, 42, 2 ** 63, 2 ** 64 - 1):
        assert [int(x) for x in oracle.seed_from_u64(seed)] == R.seed_from_u64(seed)


def test_stdrng_stream_fixture(oracle, golden):
    """StdRng(42).next_u64() sequence: sequential BlockRng model == random access."""
    g = golden("rng_fixtures.npz")
    np.testing.assert_array_equal(oracle.ref_draws(42, 0, 64), g["stdrng42_next_u64"])
    assert list(g["gen_bool08"]) == [int(d < R.P_INT[0.8]) for d in g["stdrng42_next_u64"]]
    for p, expect in ((0.5, 0x8000000000000000), (0.7, 0xB333333333333000),
                      (0.8, 0xCCCCCCCCCCCCD000), (0.9, 0xE666666666666800)):
        assert R.P_INT[p] == expect


def test_coin_fixture(oracle, golden):
    g = golden("rng_fixtures.npz")
    for pi, phase in enumerate(g["coin_phases"]):
        got = oracle.coin_range(7, 3, int(phase), int(g["coin_slot_base"]), 1024)
        np.testing.assert_array_equal(got, g["coins_seed7_epoch3"][pi])


@pytest.mark.parametrize("n", [5, 7])
def test_digest_fixture(oracle, golden, n):
    g = golden(f"digest_n{n}.npz")
    np.testing.assert_array_equal(oracle.digest_majority(g["digests"], int(g["q"])), g["state"])


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("n", [3, 5, 8])
def test_structured_equals_batch(oracle, n, kind):
    """The structure-faithful REF path (CPU baseline) decides exactly as the batch oracle."""
    q = n // 2 + 1
    r1, r2, _ = oracle.trace(kind, n, 11, 1, 3000)
    out, res = oracle.ref_step(n, q, n - 1, 42, 5, 1, r1, r2)
    dec, res2 = oracle.ref_structured(n, q, n - 1, 42, 5, 1, r1, r2)
    np.testing.assert_array_equal(out["dec"], dec)
    for k in ("n_decided", "n_v1", "n_draws", "rng_next", "last_committed_max"):
        assert res[k] == res2[k], k


def test_python_restatement_matches_c_random(oracle):
    """Fresh random vectors (not the fixture seeds): both restatements agree."""
    rng = np.random.default_rng(3)
    for n in (1, 2, 6, 11, 16):
        q = n // 2 + 1
        r1 = rng.integers(0, 4, (400, n), dtype=np.uint8)
        r2 = rng.integers(0, 4, (400, n), dtype=np.uint8)
        st = rng.integers(0, 2, 400, dtype=np.uint8)
        out, res = oracle.ref_step(n, q, n // 2, 99, 17, 1000, r1, r2, max_phase=1200, lc_in=3, wm_in=1000)
        pout, pres = R.ref_step(n, q, n // 2, 99, 17, 1000, r1.tolist(), r2.tolist(), max_phase=1200,
                                lc_in=3, wm_in=1000)
        for k in out:
            np.testing.assert_array_equal(out[k], np.array(pout[k], np.uint8), err_msg=k)
        assert res == {k: pres[k] for k in res}
        fp1 = (n - 1) // 2 + 1
        out, res = oracle.wmvc_step(n, q, fp1, 0, 5, 2, 3, 77, r1, r2, st, lc_in=0, wm_in=77)
        pout, pres = R.wmvc_step(n, q, fp1, 0, 5, 2, 3, 77, r1.tolist(), r2.tolist(), st.tolist(), 0, 77)
        for k in out:
            np.testing.assert_array_equal(out[k], np.array(pout[k], np.uint8), err_msg=k)
        assert res == {k: pres[k] for k in res}


def test_oracle_sanitized():
    """Host-code sanitizers (ASan + UBSan) over every oracle entry point."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "build/oracle_san"], check=True,
                   capture_output=True)
    p = subprocess.run([os.path.join(ROOT, "oracle", "build", "oracle_san")], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "selftest ok" in p.stdout


@pytest.mark.parametrize("n", [3, 5, 7])
def test_cluster_fixture(oracle, golden, n):
    """Weak-MVC to termination (cluster view): C restatement == Python fixture."""
    g = golden(f"cluster_n{n}.npz")
    p = json.loads(str(g["params"]))
    st = oracle.cluster_trace(n, 42, p["slot_base"], g["states"].shape[0])
    np.testing.assert_array_equal(st, g["states"])
    info = oracle.wmvc_cluster(n, p["q"], p["fp1"], p["coin_seed"], p["epoch"], p["delivery_seed"],
                               p["max_phases"], p["slot_base"], g["states"])
    np.testing.assert_array_equal(info, g["info"])
    phases = (info >> 8) & 255
    assert (info & 255 != 3).all() and phases.max() >= 3  # multi-round coin phases occur


def test_cluster_safety_and_validity():
    """Agreement (asserted inside the restatement) and validity over random and
    unanimous initial states (weak_mvc.ivy invariants decision_bc_same_round_agree,
    vl_decision_bc_agree)."""
    rng = np.random.default_rng(11)
    for n in (3, 4, 5, 6, 9):
        q, fp1 = n // 2 + 1, (n - 1) // 2 + 1
        st = rng.integers(0, 2, (300, n)).tolist()
        R.wmvc_cluster(n, q, fp1, 1, 0, 5, 64, 1, st)
        for v in (0, 1):
            outs = R.wmvc_cluster(n, q, fp1, 1, 0, 5, 64, 1, [[v] * n] * 50)
            assert all(o[0] == v and o[1] == 1 for o in outs)


@pytest.mark.parametrize("n", [1, 3, 5, 9, 16])
@pytest.mark.parametrize("S", [1, 63, 64, 65, 100_003, 300_001])
def test_soa_cpu_path_equals_oracle(oracle, n, S):
    """The all-core CPU baseline (rabia_cpu_soa.c) computes exactly or_ref_step:
    outputs, counts, StdRng position, watermarks — with the VQ prefix split over
    OpenMP chunks and a max_phase cut."""
    from rabia_amd.engine import decode_outputs, plane_stride
    for kind in (0, 1, 2):
        r1, r2, _ = oracle.trace(kind, n, 31 + S, 9, S)
        q, lane = n // 2 + 1, n // 2
        exp, eres = oracle.ref_step(n, q, lane, 42, 55, 9, r1, r2, max_phase=9 + S // 2, lc_in=4, wm_in=9)
        stride = plane_stride(S)
        planes = np.zeros((4 * n + 1, stride), np.uint32)
        planes[: 2 * n] = oracle.pack_planes(r1, stride)
        planes[2 * n: 4 * n] = oracle.pack_planes(r2, stride)
        out, res = oracle.ref_step_soa(n, q, lane, 42, 55, 9, planes, stride, S, max_phase=9 + S // 2, lc_in=4,
                                       wm_in=9, threads=4)
        got = decode_outputs(out, S)
        for k in exp:
            np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
        assert res == eres


@pytest.mark.parametrize("n,world,K,W,kind", [(5, 1, 2, 3000, 1), (3, 4, 3, 1001, 0), (9, 3, 2, 2048, 2),
                                              (7, 5, 1, 777, 0)])
def test_shard_protocol_equals_one_engine(oracle, n, world, K, W, kind):
    """The sharded pipeline's algebra on the oracle alone (or_shard_step -> rows ->
    window_draw_bases -> or_shard_fixup -> commit_windows) over `world` shards of K
    consecutive windows == or_ref_step over the windows in order: every output, every
    window's result, the engine position. Shards are ragged (world does not divide W)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rabia_amd import shard
    q, lane, seed, rng0, wm0, lc0 = n // 2 + 1, n // 2, 42, 1000, 1, 3
    max_phase = K * W * 2 // 3
    traces = [oracle.trace(kind, n, 11 + w, 1 + w * W, W) for w in range(K)]
    parts = [shard.shard_range(W, world, r, align=32) for r in range(world)]
    outs = [[None] * K for _ in range(world)]
    recs = [[None] * K for _ in range(world)]
    rows = [[None] * K for _ in range(world)]
    for r, (start, cnt) in enumerate(parts):
        for w in range(K):
            r1, r2, _ = traces[w]
            sl = slice(start, start + cnt)
            outs[r][w], recs[r][w], rows[r][w] = oracle.shard_step(n, q, lane, 1 + w * W + start, r1[sl], r2[sl],
                                                                   max_phase=max_phase)
            assert len(recs[r][w]) == oracle.record_window_words(cnt, cnt)  # segment table + records
    n_draws = [[rows[r][w]["n_draws"] for w in range(K)] for r in range(world)]
    fixed = [[None] * K for _ in range(world)]
    for r, (start, cnt) in enumerate(parts):
        g0, after = shard.window_draw_bases(n_draws, r, rng0)
        for w in range(K):
            fixed[r][w], flags = oracle.shard_fixup(seed, g0[w], 1 + w * W + start, outs[r][w], recs[r][w],
                                                    rows[r][w], after[w], max_phase=max_phase)
            assert flags == 0
    res = shard.commit_windows(fixed, 1, W, wm0, lc0)
    rng, wm, lc = rng0, wm0, lc0
    for w in range(K):
        r1, r2, _ = traces[w]
        exp, e = oracle.ref_step(n, q, lane, seed, rng, 1 + w * W, r1, r2, max_phase=max_phase, lc_in=lc, wm_in=wm)
        rng, wm, lc = e["rng_next"], e["commit_watermark"], e["last_committed_max"]
        g = res[w]
        assert (g.n_slots, g.n_decided, g.n_v1, g.n_pending_r1, g.n_draws) == \
            (e["n_slots"], e["n_decided"], e["n_v1"], e["n_pending_r1"], e["n_draws"]), w
        assert (g.last_committed, g.first_undecided, g.commit_watermark, g.flags) == \
            (e["last_committed_max"], e["first_undecided"], e["commit_watermark"], 0), w
        assert fixed[world - 1][w]["rng_next"] == e["rng_next"]
        for k in exp:
            got = np.concatenate([outs[r][w][k] for r in range(world)])
            np.testing.assert_array_equal(got, exp[k], err_msg=f"window {w} {k}")


def test_shard_fixup_flags_record_overflow(oracle):
    """Records past the capacity are not written: the fix-up flags it (8) and leaves those
    slots provisional, as the device does (include/rabia_gpu.h, flags value 8)."""
    n, W = 5, 4000
    r1, r2, _ = oracle.trace(0, n, 3, 1, W)
    out, rec, row = oracle.shard_step(n, 3, 2, 1, r1, r2, records_cap=10)
    assert row["n_draws"] > 10 and len(rec) == oracle.record_window_words(W, 10)
    fixed, flags = oracle.shard_fixup(42, 0, 1, out, rec, row, row["n_draws"], records_cap=10)
    assert flags == 8
