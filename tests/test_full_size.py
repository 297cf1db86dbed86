"""The BASELINE.json configs at their full sizes on the GPU (C2's 2^20 window is in
test_gpu_parity.py, C5 over 8 shards in test_shard_ref.py):

  C3  5 replicas x 2^24 slots, adversarial split, Weak-MVC to termination (cluster view)
  C4  7 replicas x 2^22 slots: digest exchange -> REF sweep -> kvstore apply of the V1 batches
  C5  9 replicas x 2^26 slots, one REF sweep (the bench's slot-tiled layout)

Checked through size-independent properties (counts = plane popcounts, agreement,
termination bounds, stats = info sums), the oracle on slices (every slot of C3 is
independent; REF slices take the prefix-derived draw offset), full-size oracle runs
where the C oracle finishes in seconds (C4's 2^22 REF sweep and digests, and the
C restatement of the kvstore apply), and window-split equivalence."""
import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator, decode_outputs, from_tiled, plane_stride

pytestmark = pytest.mark.gpu


def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_c3_full_size_cluster(oracle):
    torch = torch_cuda()
    n, S, q, fp1, maxp = 5, 1 << 24, 3, 3, 32
    stride = plane_stride(S)
    states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
    info = torch.zeros(S, dtype=torch.int32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
        ev.cluster_trace_async(42, 1, S, stride, states.data_ptr())
        ev.wmvc_cluster_async(states.data_ptr(), stride, S, 1, 99, maxp, info.data_ptr(), stats.data_ptr())
        ev.sync()
    got = info.cpu().numpy().view(np.uint32)
    dec, phases = got & 255, (got >> 8) & 255
    first, coins = (got >> 16) & 255, got >> 24
    assert not (dec == 2).any(), "agreement violated"
    assert ((dec == 3) == (phases == 0)).all()
    assert phases.max() <= maxp and (first <= phases).all() | (phases == 0).all()
    assert ((first >= 1) | (dec == 3)).all()
    assert (dec != 3).mean() > 0.999  # the coin terminates the adversarial split fast
    sv = stats.cpu().numpy().view(np.uint64)
    assert sv[0] == (dec != 3).sum() and sv[1] == (dec == 1).sum()
    assert sv[2] == phases.sum() and sv[3] == phases.max() and sv[4] == coins.sum()
    assert sv[5] == first.sum() and sv[6] == S
    # the coin makes both values reachable; several phases are needed on average
    assert 0.3 < (dec == 1).mean() < 0.7 and phases.mean() > 1.5
    for lo in (0, S // 2 + 12345, S - 30000):
        cnt = 30000
        st = oracle.cluster_trace(n, 42, 1 + lo, cnt)
        exp = oracle.wmvc_cluster(n, q, fp1, 7, 3, 99, maxp, 1 + lo, st)
        np.testing.assert_array_equal(got[lo:lo + cnt], exp, err_msg=f"slice at {lo}")


def test_c4_full_size_pipeline(oracle):
    torch = torch_cuda()
    from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig
    n, S, ks = 7, 1 << 22, 1 << 20
    q = n // 2 + 1
    stride = plane_stride(S)
    votes = torch.zeros((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    out = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    digests = torch.zeros(n * S, dtype=torch.int64, device="cuda")
    slot_off = torch.arange(S + 1, dtype=torch.int64, device="cuda")  # one command per slot
    cmd_data = torch.zeros(68 * S, dtype=torch.uint8, device="cuda")
    cmd_off = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    mask = torch.zeros(S, dtype=torch.uint8, device="cuda")
    res = torch.zeros(S, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n - 1, seed=42) as ev, DeviceKVStore(KVStoreConfig(max_keys=4 * ks)) as kv:
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 5, 1, S, stride, votes.data_ptr())
        ev.digest_trace_async(5, 1, S, S, digests.data_ptr())
        kv.trace_async(1, S, ks, cmd_data.data_ptr(), cmd_data.numel(), cmd_off.data_ptr())
        ev.sync()
        kv.sync()
        ev.digest_majority_async(digests.data_ptr(), S, votes.data_ptr() + 4 * 4 * n * stride, S)
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=1)
        ev.sync()
        kv.mark_applied_async(out.data_ptr(), stride, 0, S, slot_off.data_ptr(), mask.data_ptr())
        kv.apply_async(cmd_data.data_ptr(), cmd_off.data_ptr(), S, mask.data_ptr(), res.data_ptr())
        kv.sync()
        stats = kv.stats()
        # exchange stage vs the oracle over all 2^22 slots
        dg = oracle.digest_trace(n, 5, 1, S)
        np.testing.assert_array_equal(digests.view(n, S).cpu().numpy().view(np.uint64), dg)
        st_bits = np.unpackbits(votes.view(4 * n + 1, stride)[4 * n].cpu().numpy().view(np.uint8),
                                bitorder="little")[:S]
        np.testing.assert_array_equal(st_bits, oracle.digest_majority(dg, q))
        del dg
        # REF sweep vs the oracle over all 2^22 slots
        r1, r2, _ = oracle.trace(1, n, 5, 1, S)
        exp, eres = oracle.ref_step(n, q, n - 1, 42, 0, 1, r1, r2)
        del r1, r2
        got = decode_outputs(out.view(8, stride).cpu().numpy().view(np.uint32), S)
        for k in exp:
            np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
        # the apply: every command's result and the final store vs the C restatement
        m = mask.cpu().numpy()
        np.testing.assert_array_equal(m, exp["value"])
        data = cmd_data.cpu().numpy()
        offs = cmd_off.cpu().numpy().view(np.uint64)
        ref = oracle.KVStoreC(max_keys=4 * ks)
        exp_res = ref.apply(data[: int(offs[-1])], offs, m)
        np.testing.assert_array_equal(res.cpu().numpy(), exp_res)
        rs = ref.stats()
        assert stats["live_keys"] == rs["live_keys"] and stats["version"] == rs["version"]
        assert stats["total_operations"] == rs["total_operations"] and stats["flags"] == 0
        got_state, exp_state = kv.get_state(), ref.state()
        assert got_state["version"] == exp_state["version"]
        assert got_state["data"] == exp_state["data"]


def test_c4_full_size_store_full(oracle):
    """StoreFull at full size (2^22 commands over 2^20 keys, max_keys 500,000, the
    device trace with its DELETEs made GETs): the capacity-ranked keyed path (mode 3)
    against the sequential C restatement, every result and the final store; then a
    second batch on the full store (every create refused, updates in place)."""
    torch = torch_cuda()
    from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig
    S, ks, mk = 1 << 22, 1 << 20, 500_000
    cmd_data = torch.zeros(68 * S, dtype=torch.uint8, device="cuda")
    cmd_off = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    res = torch.zeros(S, dtype=torch.uint8, device="cuda")
    ref = oracle.KVStoreC(max_keys=mk)
    torch.cuda.synchronize()
    with DeviceKVStore(KVStoreConfig(max_keys=mk)) as kv:
        for seed in (3, 4):
            kv.trace_async(seed, S, ks, cmd_data.data_ptr(), cmd_data.numel(), cmd_off.data_ptr())
            kv.sync()
            first = cmd_off[:-1]
            kind = cmd_data[first]
            cmd_data[first[kind == 2]] = 1  # DELETE -> GET (first byte of the u32 variant)
            torch.cuda.synchronize()
            kv.apply_async(cmd_data.data_ptr(), cmd_off.data_ptr(), S, 0, res.data_ptr())
            kv.sync()
            stats = kv.stats()
            assert stats["last_path"] == 3 and stats["ordered_batches"] == 0, stats
            data = cmd_data.cpu().numpy()
            offs = cmd_off.cpu().numpy().view(np.uint64)
            exp_res = ref.apply(data[: int(offs[-1])], offs, np.ones(S, dtype=np.uint8))
            got = res.cpu().numpy()
            np.testing.assert_array_equal(got, exp_res)
            assert (got == 5).any()  # RG_KV_E_FULL
            rs = ref.stats()
            assert stats["live_keys"] == rs["live_keys"] == mk and stats["version"] == rs["version"]
            assert stats["total_operations"] == rs["total_operations"] and stats["flags"] == 0
        got_state, exp_state = kv.get_state(), ref.state()
        assert got_state["version"] == exp_state["version"]
        assert got_state["data"] == exp_state["data"]


def kv_blobs(kinds, ids, vals):
    """bincode KVOperation blobs (u32 variant, u64 key length, key, [u64 value length,
    value]) for keys "k%011d" % id and 8-digit values, built with numpy: (data, offsets)."""
    n = len(kinds)
    rows = np.zeros((n, 40), dtype=np.uint8)
    rows[:, 0] = kinds
    rows[:, 4] = 12
    rows[:, 12] = ord("k")
    pw = 10 ** np.arange(10, -1, -1, dtype=np.int64)
    rows[:, 13:24] = (ids[:, None] // pw) % 10 + ord("0")
    rows[:, 24] = 8
    rows[:, 32:40] = (vals[:, None] // pw[3:]) % 10 + ord("0")
    lens = np.where(kinds == 0, 40, 24)
    data = rows[np.arange(40)[None, :] < lens[:, None]]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return data, offs


def test_c4_full_size_store_full_live_deletes(oracle):
    """StoreFull with live-key DELETEs at full size (2^22 commands per batch, max_keys
    3,000,000): batch 1 creates 2^22 distinct keys (the last 1,194,304 refused: the cut);
    batch 2 interleaves DELETEs (1/4 of the commands, over half of the live keys), creates
    of fresh keys (each SET once), updates and GETs of the other half: decide's clamped scan over 2^22 events picks the refused
    creates (path 3, no ordered replay), against the sequential C restatement: every
    result, the counters and the final store."""
    torch = torch_cuda()
    from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig
    S, mk = 1 << 22, 3_000_000
    rng = np.random.default_rng(11)
    res = torch.zeros(S, dtype=torch.uint8, device="cuda")
    ref = oracle.KVStoreC(max_keys=mk)
    with DeviceKVStore(KVStoreConfig(max_keys=mk)) as kv:
        b1 = (np.zeros(S, dtype=np.uint8), np.arange(S, dtype=np.int64), rng.integers(0, 10**8, S))
        r = rng.random(S)
        kinds = np.select([r < 0.25, r < 0.55, r < 0.65], [2, 0, 0], 1).astype(np.uint8)
        # DELETEs hit keys [0, mk / 2), updates / GETs keys [mk / 2, mk) (never deleted: an
        # update is never a create), fresh keys are SET once: every refused create is its
        # key's last mutation, so the batch stays on the keyed path
        ids = np.where(r < 0.25, rng.integers(0, mk // 2, S),
              np.where(r < 0.55, S + np.arange(S), rng.integers(mk // 2, mk, S)))
        b2 = (kinds, ids, rng.integers(0, 10**8, S))
        for want_path, (k, i, v) in ((3, b1), (3, b2)):
            data, offs = kv_blobs(k, i, v)
            d_data = torch.from_numpy(data).to("cuda")
            d_off = torch.from_numpy(offs.view(np.int64)).to("cuda")
            kv.apply_async(d_data.data_ptr(), d_off.data_ptr(), S, 0, res.data_ptr())
            kv.sync()
            stats = kv.stats()
            assert stats["last_path"] == want_path and stats["ordered_batches"] == 0, stats
            exp_res = ref.apply(data, offs, np.ones(S, dtype=np.uint8))
            got = res.cpu().numpy()
            np.testing.assert_array_equal(got, exp_res)
            assert (got == 5).any() and (got == 0).any()  # RG_KV_E_FULL and Success
            rs = ref.stats()
            assert stats["live_keys"] == rs["live_keys"] and stats["version"] == rs["version"]
            assert stats["total_operations"] == rs["total_operations"] and stats["flags"] == 0
            del d_data, d_off
        got_state, exp_state = kv.get_state(), ref.state()
        assert got_state["version"] == exp_state["version"]
        assert got_state["data"] == exp_state["data"]


def test_c5_full_size_step(oracle):
    torch = torch_cuda()
    n, S, T = 9, 1 << 26, 1024
    q = n // 2 + 1
    nw = S // 32
    P = 4 * n + 1
    votes = torch.zeros((nw // T) * P * T, dtype=torch.int32, device="cuda")
    out1 = torch.zeros((nw // T) * 8 * T, dtype=torch.int32, device="cuda")
    out2 = torch.zeros_like(out1)
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T) as ev:
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 11, 1, S, T, votes.data_ptr())
        ev.phase_step_async(votes.data_ptr(), out1.data_ptr(), S, T, slot_base=1, max_phase=S - 1000)
        res = ev.last_result()
        st1 = ev.get_state()
    planes = from_tiled(out1.cpu().numpy().view(np.uint32), 8, nw, T, nw)
    dec = decode_outputs(planes, S)
    del planes
    assert res["n_decided"] == int(dec["committed"].sum()) and res["n_v1"] == int(dec["value"].sum())
    assert res["n_draws"] == int((dec["r1"] == 2).sum()) == st1["rng_next"] > 0
    assert res["n_pending_r1"] == int((dec["r1"] == 3).sum())
    assert ((dec["dec"] <= 1) == (dec["committed"] == 1)).all()
    assert ((dec["dec"] == 1) == (dec["value"] == 1)).all()
    ids_v1 = np.nonzero(dec["value"][: S - 1000])[0]
    assert res["last_committed_max"] == int(ids_v1[-1]) + 1   # commit_phase refuses ids above max_phase
    und = np.nonzero(dec["committed"] == 0)[0]
    assert res["first_undecided"] == int(und[0]) + 1 == res["commit_watermark"]
    for lo in (0, S // 3, S - 8192):
        k0 = int((dec["r1"][:lo] == 2).sum())
        r1, r2, _ = oracle.trace(1, n, 11, 1 + lo, 8192)
        exp, _ = oracle.ref_step(n, q, n - 1, 42, k0, 1 + lo, r1, r2)
        for k in exp:
            np.testing.assert_array_equal(dec[k][lo:lo + 8192], exp[k], err_msg=f"{k} at {lo}")
    del dec
    # the same 2^26 slots as 4 windows of 2^24 on a fresh context (tiled offsets)
    with PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T) as ev:
        qw = nw // 4
        for i in range(4):
            t0 = i * qw // T
            ev.phase_step_async(votes.data_ptr() + 4 * t0 * P * T, out2.data_ptr() + 4 * t0 * 8 * T, S // 4, T,
                                slot_base=1 + i * (S // 4), max_phase=S - 1000)
        st2 = ev.get_state()
    assert torch.equal(out1, out2)
    assert st1["rng_next"] == st2["rng_next"] and st1["last_committed"] == st2["last_committed"]
    assert st1["commit_watermark"] == st2["commit_watermark"]


def test_c3_two_shards_equal_one_run():
    """A C3 window split into 2 contiguous shards (two contexts, as two ranks would
    run it; shard states generated at the shards' global slot ids) == one run over
    the window: identical per-slot info words and folded statistics
    (shard.combine_cluster)."""
    torch = torch_cuda()
    from rabia_amd import shard as SH
    n, S, maxp = 5, (1 << 22) + 1000, 32
    stride = plane_stride(S)
    states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
    info = torch.zeros(S, dtype=torch.int32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
        ev.cluster_trace_async(42, 1, S, stride, states.data_ptr())
        ev.wmvc_cluster_async(states.data_ptr(), stride, S, 1, 99, maxp, info.data_ptr(), stats.data_ptr())
        ev.sync()
    rows, parts = [], []
    for rank in range(2):
        start, cnt = SH.shard_range(S, 2, rank)
        st = plane_stride(cnt)
        s_states = torch.zeros(n * st, dtype=torch.int32, device="cuda")
        s_info = torch.zeros(cnt, dtype=torch.int32, device="cuda")
        s_stats = torch.zeros(8, dtype=torch.int64, device="cuda")
        with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
            ev.cluster_trace_async(42, 1 + start, cnt, st, s_states.data_ptr())
            ev.wmvc_cluster_async(s_states.data_ptr(), st, cnt, 1 + start, 99, maxp, s_info.data_ptr(),
                                  s_stats.data_ptr())
            ev.sync()
        parts.append(s_info)
        rows.append(s_stats.cpu().numpy().view(np.uint64).tolist())
    assert torch.equal(torch.cat(parts), info)
    one = SH.combine_cluster([stats.cpu().numpy().view(np.uint64).tolist()])
    assert SH.combine_cluster(rows) == one
    assert one["slots"] == S
