"""kvstore apply: the CPU restatement
(oracle/kvstore_ref.py) against the reference's own kvstore test outcomes, and the
device apply (include/rabia_kv.h) against the restatement."""
import json
import os
import random

import numpy as np
import pytest

import kvstore_ref as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kv_reference_cases.json")
KIND = {"Set": R.SET, "Get": R.GET, "Delete": R.DELETE, "Exists": R.EXISTS}
CODE = {"Success": R.OK, "NotFound": R.NOT_FOUND}


def golden_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def blob(cmd):
    kind = KIND[cmd[0]]
    return R.encode_op(kind, cmd[1].encode(), cmd[2].encode() if len(cmd) > 2 else b"")


def random_blobs(rng: random.Random, n: int, key_space: int, edge: bool = True):
    """Mixed commands over a small key space (many same-key conflicts), with the
    edge cases the reference validates: empty / 256 / 257-byte keys, values over
    max_value_size, non-UTF-8 strings, truncated and unknown-variant data."""
    out = []
    for _ in range(n):
        r = rng.random()
        key = f"key{rng.randrange(key_space)}".encode()
        if edge and r < 0.02:
            out.append(R.encode_op(R.SET, b"", b"v"))
        elif edge and r < 0.03:
            out.append(R.encode_op(rng.choice([R.SET, R.GET]), b"a" * 256, b"x"))
        elif edge and r < 0.04:
            out.append(R.encode_op(R.GET, b"b" * 257))
        elif edge and r < 0.05:
            out.append(R.encode_op(R.SET, key, b"y" * 70))       # > max_value_size=64 below
        elif edge and r < 0.06:
            out.append(R.encode_op(R.SET, key + b"\xff", b"v"))  # key not UTF-8
        elif edge and r < 0.07:
            out.append(R.encode_op(R.SET, key, b"\xed\xa0\x80"))  # surrogate: not UTF-8
        elif edge and r < 0.08:
            out.append(R.encode_op(R.SET, key, b"v")[:-3])        # truncated
        elif edge and r < 0.09:
            out.append(b"\x07\x00\x00\x00" + R.encode_op(R.GET, key)[4:])  # unknown variant
        elif edge and r < 0.10:
            out.append(R.encode_op(R.GET, key) + b"trailing")     # trailing bytes are allowed
        elif edge and r < 0.11:
            out.append(R.encode_op(R.SET, "ключ".encode() + key, "значение€".encode()))
        elif r < 0.55:
            out.append(R.encode_op(R.SET, key, f"v{rng.randrange(1 << 20)}".encode()))
        elif r < 0.75:
            out.append(R.encode_op(R.GET, key))
        elif r < 0.90:
            out.append(R.encode_op(R.DELETE, key))
        else:
            out.append(R.encode_op(R.EXISTS, key))
    return out


# ---------------------------------------------------------------- CPU -------
def test_oracle_matches_reference_tests():
    for case in golden_cases():
        st = R.KVStoreRef()
        res = st.apply_commands([blob(c) for c in case["commands"]])
        for got, exp in zip(res, case["expect"]):
            if exp is not None:
                assert got == CODE[exp], case["name"]
        if case["state"] is not None:
            data = st.state()["data"]
            assert {k.decode(): v[0].decode() for k, v in data.items()} == case["state"], case["name"]


def test_bincode_roundtrip_and_rejects():
    for kind in (R.SET, R.GET, R.DELETE, R.EXISTS):
        b = R.encode_op(kind, b"k1", b"v1")
        assert R.decode_op(b) == (kind, b"k1", b"v1" if kind == R.SET else b"")
    # layout: u32 variant, u64 length, bytes (bincode 1.3 fixint little-endian)
    assert R.encode_op(R.GET, b"ab") == b"\x01\x00\x00\x00\x02\x00\x00\x00\x00\x00\x00\x00ab"
    assert R.decode_op(b"\x04" + b"\x00" * 11) is None
    assert R.decode_op(R.encode_op(R.SET, b"k", b"v")[:-1]) is None
    assert R.decode_op(R.encode_op(R.GET, b"k\xc0\xaf")) is None          # overlong
    assert R.decode_op(R.encode_op(R.GET, b"k") + b"xx") == (R.GET, b"k", b"")


def test_oracle_semantics_versions_and_full():
    st = R.KVStoreRef(max_keys=2)
    seq = [(R.SET, b"a", b"1"), (R.SET, b"a", b"2"), (R.SET, b"b", b"1"), (R.SET, b"c", b"1"),
           (R.DELETE, b"a", b""), (R.SET, b"c", b"2"), (R.SET, b"a", b"3"), (R.DELETE, b"zz", b"")]
    res = [st.apply(*op) for op in seq]
    assert res == [R.OK, R.OK, R.OK, R.E_FULL, R.OK, R.OK, R.E_FULL, R.NOT_FOUND]
    assert st.state() == {"data": {b"b": (b"1", 1), b"c": (b"2", 1)}, "version": 5}
    assert st.total_operations == 6


def test_apply_decided_order():
    st = R.KVStoreRef()
    blobs = [R.encode_op(R.SET, b"k", b"s0"), R.encode_op(R.SET, b"k", b"s1"), R.encode_op(R.GET, b"k")]
    res = R.apply_decided(st, blobs, [0, 1, 2, 3], applied_slots=[1, 2])
    assert res == [R.NOT_APPLIED, R.OK, R.OK]
    assert st.state()["data"] == {b"k": (b"s1", 1)}


# ---------------------------------------------------------------- GPU -------
def _store(**kw):
    from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig
    return DeviceKVStore(KVStoreConfig(**kw))


def _check_state(dev, ref):
    got = dev.get_state()
    exp = ref.state()
    assert got["version"] == exp["version"]
    assert got["data"] == exp["data"]
    st = dev.stats()
    assert st["live_keys"] == len(exp["data"])
    assert st["total_operations"] == ref.total_operations
    assert st["flags"] == 0


@pytest.mark.gpu
def test_gpu_reference_cases():
    for case in golden_cases():
        with _store() as dev:
            ref = R.KVStoreRef()
            blobs = [blob(c) for c in case["commands"]]
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs), case["name"]
            for g, exp in zip(got, case["expect"]):
                if exp is not None:
                    assert g == CODE[exp]
            _check_state(dev, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,key_space,batches", [(1, 1, 3), (37, 5, 4), (1000, 50, 3), (20000, 3000, 3),
                                                 (20000, 20, 2)])
def test_gpu_random_batches_vs_oracle(n, key_space, batches):
    rng = random.Random(n * 131 + key_space)
    with _store(max_value_size=64) as dev:
        ref = R.KVStoreRef(max_value_size=64)
        for _ in range(batches):
            blobs = random_blobs(rng, n, key_space)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        assert dev.stats()["ordered_batches"] == 0


@pytest.mark.gpu
def test_gpu_store_full_takes_ordered_path():
    rng = random.Random(5)
    with _store(max_keys=40, max_value_size=64) as dev:
        ref = R.KVStoreRef(max_keys=40, max_value_size=64)
        for _ in range(4):
            blobs = random_blobs(rng, 300, 80)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        assert R.E_FULL in got or dev.stats()["ordered_batches"] > 0
        assert dev.stats()["ordered_batches"] >= 1


def no_delete(blobs):
    """The same commands with every DELETE turned into a GET (a batch whose live count
    only grows: the capacity-ranked path)."""
    out = []
    for b in blobs:
        if len(b) >= 4 and b[:4] == b"\x02\x00\x00\x00":
            b = b"\x01\x00\x00\x00" + b[4:]
        out.append(b)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n,key_space,max_keys,bucket_bits,batches",
                         [(3000, 2000, 500, 0, 2), (3000, 400, 100, 8, 3), (500, 100, 1, 0, 2), (4000, 900, 600, 0, 3)])
def test_gpu_store_full_capacity_ranked(n, key_space, max_keys, bucket_bits, batches):
    """StoreFull reachable in a batch with no DELETE of a live key: the live count only
    grows, so a create succeeds iff fewer than max_keys - live creates precede it in
    command order. The keyed path with the creates ranked (mode 3, the cut from the
    plan's create bitmap) equals the in-order restatement: results (StoreFull for the
    refused keys' SETs, NotFound for their GETs), the store and the counters, also in
    runs of several keys (8-bit buckets) and once the store is full (free = 0)."""
    rng = random.Random(n + max_keys)
    with _store(max_keys=max_keys, max_value_size=64, bucket_bits=bucket_bits) as dev:
        ref = R.KVStoreRef(max_keys=max_keys, max_value_size=64)
        paths = []
        for _ in range(batches):
            blobs = no_delete(random_blobs(rng, n, key_space))
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
            paths.append(dev.stats()["last_path"])
            _check_state(dev, ref)
        assert R.E_FULL in got
        assert 3 in paths and dev.stats()["ordered_batches"] == 0, paths
        # a DELETE of a live key in a batch that meets StoreFull: the clamped scan (3) when
        # every refused create is its key's last mutation, else the ordered replay (1)
        victim = next(iter(ref.data))
        blobs = [R.encode_op(R.DELETE, victim)] + no_delete(random_blobs(rng, n, key_space))
        got = [int(x) for x in dev.apply_commands(blobs)]
        assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        st = dev.stats()
        assert st["last_path"] in (1, 3) and st["ordered_batches"] == (st["last_path"] == 1)


def live_delete_batch(rng, live, n, fresh):
    """Creates of fresh keys (each SET once: a refused create is its key's last mutation),
    DELETEs of keys live before the batch, updates of live keys, GETs / EXISTS of both."""
    out, made = [], []
    for _ in range(n):
        r = rng.random()
        if r < 0.40:
            k = f"new{next(fresh)}".encode()
            made.append(k)
            out.append(R.encode_op(R.SET, k, f"v{rng.randrange(1 << 20)}".encode()))
        elif r < 0.60 and live:
            out.append(R.encode_op(R.DELETE, rng.choice(live)))
        elif r < 0.75 and made:
            out.append(R.encode_op(rng.choice([R.GET, R.EXISTS]), rng.choice(made)))
        elif r < 0.85 and live:
            out.append(R.encode_op(R.SET, rng.choice(live), b"u" + bytes(str(rng.randrange(99)), "ascii")))
        else:
            out.append(R.encode_op(R.EXISTS, rng.choice(live) if live else b"none"))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n,max_keys,bucket_bits,batches", [(3000, 800, 0, 3), (4000, 1500, 12, 3), (600, 50, 0, 4)])
def test_gpu_store_full_with_live_deletes(n, max_keys, bucket_bits, batches):
    """StoreFull reachable in batches that also DELETE live keys: the live count is a
    clamped walk over the creates and deletes in command order (decide's scan); a create is
    refused iff it finds the store full. Equal to the in-order restatement (results, store,
    counters) on the keyed path (3), also with multi-key runs (12-bit buckets) and a live key
    deleted and re-updated (its update a create, refused or not)."""
    import itertools
    rng = random.Random(n + max_keys)
    fresh = itertools.count()
    # (deleted keys keep their table slots: a table well above max_keys for the fresh keys)
    with _store(max_keys=max_keys, max_value_size=64, bucket_bits=bucket_bits, table_slots=1 << 15) as dev:
        ref = R.KVStoreRef(max_keys=max_keys, max_value_size=64)
        paths = []
        for _ in range(batches):
            blobs = live_delete_batch(rng, list(ref.data), n, fresh)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
            _check_state(dev, ref)
            paths.append(dev.stats()["last_path"])
        assert R.E_FULL in got and R.OK in got
        assert 3 in paths, paths


@pytest.mark.gpu
def test_gpu_store_full_live_delete_cases():
    """Hand-made StoreFull batches with live-key DELETEs: a refused create that is its key's
    last mutation stays on the keyed path (3), including a key live before the batch,
    deleted, then re-created and refused (its entry goes to version 0); a refused key SET
    again after a DELETE freed a slot takes the ordered replay (1)."""
    def run(dev, ref, cmds):
        blobs = [R.encode_op(k, key, val) for k, key, val in cmds]
        got = [int(x) for x in dev.apply_commands(blobs)]
        assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        return got, dev.stats()["last_path"]

    S, G, D = R.SET, R.GET, R.DELETE
    with _store(max_keys=3, max_value_size=64) as dev:
        ref = R.KVStoreRef(max_keys=3, max_value_size=64)
        run(dev, ref, [(S, b"a", b"1"), (S, b"b", b"1"), (S, b"c", b"1")])  # full
        got, path = run(dev, ref, [(S, b"k1", b"x"), (D, b"a", b""), (S, b"k2", b"y"), (G, b"k1", b""),
                                   (G, b"k2", b""), (S, b"k3", b"z")])
        assert path == 3 and got == [R.E_FULL, R.OK, R.OK, R.NOT_FOUND, R.OK, R.E_FULL]
        # b: live, deleted, k4 takes its place, b re-created and refused (its last mutation)
        got, path = run(dev, ref, [(D, b"b", b""), (S, b"k4", b"w"), (S, b"b", b"2"), (G, b"b", b"")])
        assert path == 3 and got == [R.OK, R.OK, R.E_FULL, R.NOT_FOUND]
        # k5 refused, then a DELETE frees a key and k5's second SET succeeds: ordered replay
        got, path = run(dev, ref, [(S, b"k5", b"1"), (D, b"c", b""), (S, b"k5", b"2"), (G, b"k5", b"")])
        assert path == 1 and got == [R.E_FULL, R.OK, R.OK, R.OK]


@pytest.mark.gpu
@pytest.mark.parametrize("hash_bits", [2, 5, 12])
def test_gpu_hash_collision_runs(hash_bits):
    """Truncated key hashes: every hash run holds several distinct keys (split by
    byte comparison); runs with more than 8 keys take the ordered path."""
    rng = random.Random(hash_bits)
    with _store(max_value_size=64, hash_bits=hash_bits, table_slots=1 << 16) as dev:
        ref = R.KVStoreRef(max_value_size=64)
        for _ in range(3):
            blobs = random_blobs(rng, 3000, 400)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        # 2 / 5 bits: runs of ~100 / ~12 distinct keys exceed the 8-key walker -> ordered
        # replay; 12 bits: runs of 1-3 keys stay on the keyed path
        assert (dev.stats()["ordered_batches"] > 0) == (hash_bits <= 5)


@pytest.mark.gpu
@pytest.mark.parametrize("n,hot_frac,warm,key_space", [(60000, 0.4, 10, 5000), (30000, 1.0, 0, 1),
                                                       (50000, 0.2, 200, 20000), (140000, 0.5, 50, 50000)])
def test_gpu_hot_keys_sort_bins(n, hot_frac, warm, key_space):
    """Skewed batches: a hot key (and warm keys) put far more commands into one
    top-digit bin of the sort than an LDS chunk holds, so the bin is sorted streamed
    through global memory (rg_kv.hip kv_l2_sort_kernel); every result and the final
    store equal the sequential restatement. The 140,000-command case puts ~49,000
    applied commands into the hot key's bin (3 x the 16,384-command LDS chunk) in a
    batch of more than 65,536 commands, whose buckets need 3 digit passes: the streamed
    path with an odd pass count (final pair a)."""
    rng = random.Random(n + warm)
    blobs = []
    for _ in range(n):
        r = rng.random()
        if r < hot_frac:
            key = b"hot"
        elif r < hot_frac + 0.3 and warm:
            key = f"warm{rng.randrange(warm)}".encode()
        else:
            key = f"key{rng.randrange(key_space)}".encode()
        x = rng.random()
        if x < 0.6:
            blobs.append(R.encode_op(R.SET, key, f"v{rng.randrange(1 << 20)}".encode()))
        elif x < 0.8:
            blobs.append(R.encode_op(R.GET, key))
        elif x < 0.9:
            blobs.append(R.encode_op(R.DELETE, key))
        else:
            blobs.append(R.encode_op(R.EXISTS, key))
    mask = [1 if rng.random() < 0.7 else 0 for _ in range(n)]
    with _store(max_value_size=64) as dev:
        ref = R.KVStoreRef(max_value_size=64)
        for _ in range(2):
            got = [int(x) for x in dev.apply_commands(blobs, mask=mask)]
            exp = [R.NOT_APPLIED if not m else ref.apply_data(b) for b, m in zip(blobs, mask)]
            assert got == exp
        _check_state(dev, ref)


@pytest.mark.gpu
def test_gpu_mask_not_applied():
    blobs = [R.encode_op(R.SET, b"a", b"1"), R.encode_op(R.SET, b"a", b"2"), R.encode_op(R.GET, b"b")]
    with _store() as dev:
        got = [int(x) for x in dev.apply_commands(blobs, mask=[1, 0, 1])]
        assert got == [R.OK, R.NOT_APPLIED, R.NOT_FOUND]
        assert dev.get_state()["data"] == {b"a": (b"1", 1)}


@pytest.mark.gpu
def test_gpu_device_trace_and_large_batch():
    """Device-generated C4 commands (2^20): decode on the host with the oracle,
    replay sequentially, compare every result and the final store."""
    import torch
    n, ks = 1 << 20, 1 << 18
    with _store(max_keys=1 << 20) as dev:
        data = torch.empty(68 * n, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        res = torch.empty(n, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()  # a real stream handle (0 would mean the store's own stream)
        torch.cuda.synchronize()
        dev.trace_async(7, n, ks, data.data_ptr(), data.numel(), off.data_ptr(), s.cuda_stream)
        dev.apply_async(data.data_ptr(), off.data_ptr(), n, None, res.data_ptr(), s.cuda_stream)
        s.synchronize()
        d = data.cpu().numpy().tobytes()
        o = off.cpu().numpy()
        blobs = [d[o[i]:o[i + 1]] for i in range(n)]
        assert all(R.decode_op(b) is not None for b in blobs[:1000])
        ref = R.KVStoreRef(max_keys=1 << 20)
        exp = np.array(ref.apply_commands(blobs), np.uint8)
        assert np.array_equal(res.cpu().numpy(), exp)
        _check_state(dev, ref)


@pytest.mark.gpu
def test_gpu_c4_pipeline_phase_step_then_apply(oracle):
    """C4: 7 replicas, REF phase step -> V1 decisions (output plane 7), then the
    V1 slots' batches (CSR by slot) applied in ascending slot order."""
    import torch
    from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs
    n, S = 7, 4096
    r1, r2, _ = oracle.trace(1, n, 11, 1, S)
    rng = random.Random(3)
    counts = [rng.randrange(0, 4) for _ in range(S)]
    slot_off = np.zeros(S + 1, np.uint64)
    slot_off[1:] = np.cumsum(counts)
    blobs = random_blobs(rng, int(slot_off[-1]), 300, edge=False)
    with PhaseEvaluator(n, self_lane=6, mode="ref", seed=9) as ev, _store() as dev:
        win = PhaseWindow.from_codes(r1, r2, slot_base=1)
        out, _ = ev.phase_step_host(win)
        dec = decode_outputs(out, S)
        out_d = torch.from_numpy(out.view(np.int32).copy()).cuda()
        stride = out.shape[1] if out.ndim == 2 else out.size // 8
        from rabia_amd.kvstore import pack_commands
        data, offs = pack_commands(blobs)
        d = torch.from_numpy(data.copy()).cuda()
        o = torch.from_numpy(offs.view(np.int64)).cuda()
        so = torch.from_numpy(slot_off.view(np.int64)).cuda()
        mask = torch.empty(len(blobs), dtype=torch.uint8, device="cuda")
        res = torch.empty(len(blobs), dtype=torch.uint8, device="cuda")
        stream = torch.cuda.Stream()
        torch.cuda.synchronize()
        s = stream.cuda_stream
        dev.mark_applied_async(out_d.data_ptr(), stride, 0, S, so.data_ptr(), mask.data_ptr(), s)
        dev.apply_async(d.data_ptr(), o.data_ptr(), len(blobs), mask.data_ptr(), res.data_ptr(), s)
        torch.cuda.synchronize()
        applied = [s_ for s_ in range(S) if dec["value"][s_]]
        ref = R.KVStoreRef()
        exp = R.apply_decided(ref, blobs, slot_off, applied)
        assert res.cpu().numpy().tolist() == exp
        _check_state(dev, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("lc_in_frac,max_frac", [(0.0, 0.0), (0.5, 0.0), (0.3, 0.7), (1.2, 0.0)])
def test_gpu_follower_gate_then_apply(oracle, lc_in_frac, max_frac):
    """a11: a follower applies a decided window's V1 batches only above its
    last_committed (handle_decision, engine.rs:723-728) — including a window
    evaluated after a later commit (last_committed inside or past the window) —
    and advances last_committed like commit_phase; vs the message-at-a-time
    restatement (oracle/rabia_ref.py:handle_decisions) and kvstore_ref."""
    import torch
    import rabia_ref as P
    from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs
    n, S, base = 7, 20_011, 101
    r1, r2, _ = oracle.trace(1, n, 5, base, S)
    lc_in = int(base + lc_in_frac * S) if lc_in_frac else 0
    mp = int(base + max_frac * S) if max_frac else 0
    rng = random.Random(7)
    counts = [rng.randrange(0, 3) for _ in range(S)]
    slot_off = np.zeros(S + 1, np.uint64)
    slot_off[1:] = np.cumsum(counts)
    blobs = random_blobs(rng, int(slot_off[-1]), 500, edge=False)
    with PhaseEvaluator(n, self_lane=6, seed=9) as prop:   # the proposer decided the window
        out, _ = prop.phase_step_host(PhaseWindow.from_codes(r1, r2, slot_base=base))
    dec = decode_outputs(out, S)
    exp_app, exp_lc = P.handle_decisions(dec["value"].tolist(), dec["committed"].tolist(), base, lc_in, mp)
    stride = out.shape[1]
    out_d = torch.from_numpy(out.view(np.int32).copy()).cuda()
    applied = torch.zeros(stride, dtype=torch.int32, device="cuda")
    gate = torch.zeros(1, dtype=torch.int64, device="cuda")
    res = torch.zeros(10, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with PhaseEvaluator(n, self_lane=2, seed=9) as fol, _store() as dev:
        fol.set_state(last_committed=lc_in, commit_watermark=base)
        fol.follower_commit_async(out_d.data_ptr(), S, stride, base, applied.data_ptr(), gate.data_ptr(),
                                  res.data_ptr(), max_phase=mp)
        fol.sync()
        st = fol.get_state()
        bits = np.unpackbits(applied.cpu().numpy().view(np.uint8), bitorder="little")[:S]
        np.testing.assert_array_equal(bits, np.array(exp_app, np.uint8))
        assert st["last_committed"] == exp_lc and int(gate.cpu()[0]) == lc_in
        r = res.cpu().numpy().view(np.uint64)
        assert int(r[2]) == sum(exp_app) and int(r[1]) == int(dec["committed"].sum())
        assert int(r[5]) == exp_lc
        # the follower's kv apply: only the applied slots' batches
        from rabia_amd.kvstore import pack_commands
        data, offs = pack_commands(blobs)
        d = torch.from_numpy(data.copy()).cuda()
        o = torch.from_numpy(offs.view(np.int64)).cuda()
        so = torch.from_numpy(slot_off.view(np.int64)).cuda()
        mask = torch.empty(len(blobs), dtype=torch.uint8, device="cuda")
        kres = torch.empty(len(blobs), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        dev.mark_applied_async(out_d.data_ptr(), stride, 0, S, so.data_ptr(), mask.data_ptr(), 0, slot_base=base,
                               gate_ptr=gate.data_ptr())
        dev.apply_async(d.data_ptr(), o.data_ptr(), len(blobs), mask.data_ptr(), kres.data_ptr(), 0)
        dev.sync()
        ref = R.KVStoreRef()
        exp = R.apply_decided(ref, blobs, slot_off, [s_ for s_ in range(S) if exp_app[s_]])
        assert kres.cpu().numpy().tolist() == exp
        _check_state(dev, ref)


def test_follower_restatement_skips_late_lower_phases():
    """The literal handler in arrival order skips a lower phase decided after a
    higher one (engine.rs:727); in ascending order only phases <= the starting
    last_committed are skipped — the closed form the device uses."""
    import rabia_ref as P
    vals, com = [1, 1, 1, 0, 1], [1, 1, 1, 1, 1]
    app, lc = P.handle_decisions(vals, com, 10, 0, order=[2, 0, 1, 3, 4])
    assert app == [0, 0, 1, 0, 1] and lc == 14
    app, lc = P.handle_decisions(vals, com, 10, 11)
    assert app == [0, 0, 1, 0, 1] and lc == 14
    app, lc = P.handle_decisions(vals, com, 10, 0, max_phase=12)
    assert app == [1, 1, 1, 0, 1] and lc == 12   # 14 applied, its commit_phase refused (state.rs:70-75)


def _packed(blobs):
    offs = np.zeros(len(blobs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    return np.frombuffer(b"".join(blobs), np.uint8), offs


def test_c_restatement_equals_python_restatement(oracle):
    """oracle/kvstore_ref.c (the full-size checker and C4 CPU baseline) == the
    Python restatement pinned by the reference's own test outcomes: the golden
    cases, random mixed batches with every edge case, StoreFull, masks."""
    for case in golden_cases():
        blobs = [blob(c) for c in case["commands"]]
        data, offs = _packed(blobs)
        c = oracle.KVStoreC(max_keys=case.get("max_keys", 0), max_value_size=case.get("max_value_size", 0))
        got = c.apply(data, offs).tolist()
        ref = R.KVStoreRef(max_keys=case.get("max_keys", R.DEFAULT_MAX_KEYS),
                           max_value_size=case.get("max_value_size", R.DEFAULT_MAX_VALUE))
        assert got == ref.apply_commands(blobs), case.get("name")
        assert c.state() == ref.state()
    rng = random.Random(5)
    for trial in range(6):
        blobs = random_blobs(rng, 5000, 50 + 400 * trial)
        data, offs = _packed(blobs)
        mask = np.array([rng.random() < 0.8 for _ in blobs], np.uint8) if trial % 2 else None
        mk = 40 if trial == 3 else 0
        c = oracle.KVStoreC(max_keys=mk, max_value_size=64)
        ref = R.KVStoreRef(max_keys=mk or R.DEFAULT_MAX_KEYS, max_value_size=64)
        got = c.apply(data, offs, mask).tolist()
        exp = [ref.apply_data(b) if mask is None or mask[i] else R.NOT_APPLIED for i, b in enumerate(blobs)]
        assert got == exp
        assert c.state() == ref.state()
        st = c.stats()
        assert st["total_operations"] == ref.total_operations and st["live_keys"] == len(ref.data)


@pytest.mark.gpu
def test_gpu_sustained_batches_heap_stays_bounded(oracle):
    """30 device-generated C4 batches on ONE store whose heap holds only a few
    batches' worth of bytes: value updates overwrite in place (size classes), so
    the heap stops growing once every key exists; no batch is refused, and every
    result and the final store equal the sequential C restatement."""
    import torch
    n, ks, batches = 1 << 16, 1 << 12, 30
    heap = 3 * ks * (16 + 32) + (1 << 16)   # keys + one value class each, plus slack
    with _store(max_keys=1 << 16, heap_bytes=heap) as dev:
        ref = oracle.KVStoreC(max_keys=1 << 16)
        data = torch.empty(68 * n, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        res = torch.empty(n, dtype=torch.uint8, device="cuda")
        used = []
        for b in range(batches):
            torch.cuda.synchronize()
            dev.trace_async(100 + b, n, ks, data.data_ptr(), data.numel(), off.data_ptr())
            dev.apply_async(data.data_ptr(), off.data_ptr(), n, None, res.data_ptr())
            dev.sync()
            st = dev.stats()
            assert st["flags"] == 0 and st["last_path"] == 0, (b, st)
            offs = off.cpu().numpy().view(np.uint64)
            exp = ref.apply(data.cpu().numpy()[: int(offs[-1])], offs)
            np.testing.assert_array_equal(res.cpu().numpy(), exp, err_msg=f"batch {b}")
            used.append(st["heap_used"])
        assert used[-1] == used[5], used   # no growth once the key space is populated
        got, exp = dev.get_state(), ref.state()
        assert got["data"] == exp["data"] and got["version"] == exp["version"]


@pytest.mark.gpu
@pytest.mark.parametrize("max_keys", [0, 30])  # 0: keyed path; 30: StoreFull reachable -> ordered path
def test_gpu_refused_batch_changes_nothing(max_keys):
    """A batch the heap cannot hold is refused whole: every pending command reports
    RG_KV_E_CAPACITY, the store (entries, counters, heap) is exactly as before, the
    flags say why, and the host apply raises. A later batch that fits applies."""
    from rabia_amd import _native as N
    rng = random.Random(9)
    mk = max_keys or R.DEFAULT_MAX_KEYS
    with _store(max_keys=max_keys, max_value_size=64, heap_bytes=2048, table_slots=1 << 10) as dev:
        ref = R.KVStoreRef(max_keys=mk, max_value_size=64)
        small = [R.encode_op(R.SET, f"k{i}".encode(), b"v" * 8) for i in range(8)]
        assert [int(x) for x in dev.apply_commands(small)] == ref.apply_commands(small)
        before, st0 = dev.get_state(), dev.stats()
        big = random_blobs(rng, 400, 300, edge=False)
        with pytest.raises(N.RabiaGpuError):
            dev.apply_commands(big)
        st1 = dev.stats()
        assert st1["last_path"] == 2 and st1["flags"] != 0
        for k in ("live_keys", "version", "total_operations", "occupied_slots", "heap_used"):
            assert st1[k] == st0[k], k
        assert dev.get_state() == before
        # results of the refused batch: every pending command says "refused"
        import torch
        from rabia_amd.kvstore import pack_commands
        data, offs = pack_commands(big)
        d = torch.from_numpy(data.copy()).cuda()
        o = torch.from_numpy(offs.view(np.int64)).cuda()
        r = torch.zeros(len(big), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        dev.apply_async(d.data_ptr(), o.data_ptr(), len(big), None, r.data_ptr())
        dev.sync()
        assert set(r.cpu().numpy().tolist()) <= {8, R.E_KEY_EMPTY, R.E_KEY_LONG, R.E_VALUE_LARGE, R.E_DECODE}
        assert 8 in r.cpu().numpy().tolist()
        more = [R.encode_op(R.SET, b"k1", b"w" * 8), R.encode_op(R.GET, b"k3")]
        assert [int(x) for x in dev.apply_commands(more)] == ref.apply_commands(more)
        got = dev.get_state()
        assert got["data"] == ref.state()["data"] and got["version"] == ref.state()["version"]


@pytest.mark.gpu
@pytest.mark.parametrize("bucket_bits", [3, 6, 10])
def test_gpu_narrow_buckets_mix_hashes(bucket_bits):
    """Sort buckets narrower than the hash (ADVICE: the 31-bit bucket path): one
    walker run holds keys with distinct full hashes, each looked up with its own
    hash; inserts, deletes and the more-than-8-keys ordered fallback vs the
    restatement."""
    rng = random.Random(bucket_bits)
    with _store(max_value_size=64, bucket_bits=bucket_bits, table_slots=1 << 14) as dev:
        ref = R.KVStoreRef(max_value_size=64)
        for _ in range(3):
            blobs = random_blobs(rng, 3000, 500)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)
        # 3 / 6 bits: ~60 / ~8 keys per run -> ordered replay; 10 bits: ~1 key per run
        assert (dev.stats()["ordered_batches"] > 0) == (bucket_bits <= 6)


def decode_edge_blobs(rng: random.Random):
    """Commands at the edges of the decode fast path (key <= 16 B, SET value region
    <= 64 B, ASCII, all loads in one round trip) and just outside it: every key
    length 1..17, every value length 0..66, trailing bytes after a value (non-ASCII
    and invalid UTF-8 ones included: not part of the value), value lengths that
    claim more bytes than the command holds, non-ASCII valid UTF-8 and invalid
    UTF-8 at the first and last byte of short keys and values."""
    out = []
    for kl in range(1, 18):
        key = (f"k{kl:02d}" + "abcdefghijklmnop")[:kl].encode()
        out.append(R.encode_op(R.SET, key, b"v" * (kl % 5)))
        out.append(R.encode_op(R.GET, key))
        out.append(R.encode_op(R.EXISTS, key) + b"\xff\xfe")
    for vl in range(0, 67):
        key = f"val{vl % 7}".encode()
        out.append(R.encode_op(R.SET, key, bytes(rng.choice(b"0123456789abcdef") for _ in range(vl))))
    for tail in (b"x", b"\xff", b"\xc3", b"trailing bytes!!", b"\x80" * 30):
        out.append(R.encode_op(R.SET, b"tail", b"abc") + tail)
        out.append(R.encode_op(R.SET, b"t" * 16, b"q" * 40) + tail)
    good = R.encode_op(R.SET, b"claim", b"12345678")
    for extra in (1, 8, 100):   # value length field larger than the bytes that follow
        out.append(good[:12 + 5] + (8 + extra).to_bytes(8, "little") + good[12 + 5 + 8:])
    out.append(good[:12 + 5] + (2).to_bytes(8, "little") + good[12 + 5 + 8:])  # shorter: rest trails
    for bad in (b"\xff", b"\xc3\x28", b"\xed\xa0\x80"):
        out.append(R.encode_op(R.SET, bad + b"key", b"v"))
        out.append(R.encode_op(R.SET, b"key" + bad, b"v"))
        out.append(R.encode_op(R.SET, b"key", bad + b"value"))
        out.append(R.encode_op(R.SET, b"key", b"value" + bad))
    for s in ("é", "ключ", "€uro", "a€", "日本語のキー"):
        out.append(R.encode_op(R.SET, s.encode(), s.encode() * 3))
        out.append(R.encode_op(R.GET, s.encode()))
    out.append(R.encode_op(R.GET, b""))
    out.append(b"\x00\x00\x00\x00" + (3).to_bytes(8, "little") + b"ab")  # key cut short
    rng.shuffle(out)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_decode_fast_path_edges(seed):
    rng = random.Random(seed)
    with _store(max_value_size=60) as dev:
        ref = R.KVStoreRef(max_value_size=60)
        for _ in range(2):
            blobs = decode_edge_blobs(rng)
            got = [int(x) for x in dev.apply_commands(blobs)]
            assert got == ref.apply_commands(blobs)
        _check_state(dev, ref)


def test_partitioned_cpu_baseline_equals_sequential():
    """The all-core C baseline of the apply (key-hash partitions, oracle/kvstore_ref.c:
    or_kv_apply_partitioned) gives the sequential restatement's results and counters
    when StoreFull cannot fire (CPU only)."""
    import oracle_lib as O
    rng = np.random.default_rng(5)
    cmds = []
    for _ in range(20000):
        k = f"key{int(rng.integers(0, 700))}".encode()
        op = int(rng.choice([0, 0, 0, 1, 2, 3]))
        body = op.to_bytes(4, "little") + len(k).to_bytes(8, "little") + k
        if op == 0:
            v = bytes(rng.integers(97, 123, int(rng.integers(0, 40))).astype(np.uint8))
            body += len(v).to_bytes(8, "little") + v
        cmds.append(body)
    cmds.append(b"\x05\x00")  # undecodable
    data = np.frombuffer(b"".join(cmds), np.uint8)
    offs = np.zeros(len(cmds) + 1, np.uint64)
    offs[1:] = np.cumsum([len(c) for c in cmds])
    mask = (rng.random(len(cmds)) < 0.8).astype(np.uint8)
    seq = O.KVStoreC(max_keys=10_000)
    exp = seq.apply(data, offs, mask)
    st = seq.stats()
    for parts in (1, 3, 16):
        got, tot = O.kv_apply_partitioned(data, offs, mask, parts=parts, max_keys=10_000)
        np.testing.assert_array_equal(got, exp)
        assert tot == {k: st[k] for k in ("live_keys", "version", "total_operations")}
