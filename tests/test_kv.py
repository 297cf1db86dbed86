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
