"""Per-step checkpoint: the reference's EngineState JSON
(rabia-core/src/persistence.rs:9-42) and the batched engine's resume record."""
import json
import zlib

import numpy as np
import pytest

from rabia_amd.checkpoint import Checkpoint, engine_state_json, parse_engine_state_json


def test_engine_state_json_matches_serde_layout():
    # serde_json::to_vec of EngineState { current_phase: PhaseId(7), last_committed_phase:
    # PhaseId(5), snapshot: None }: newtypes as bare numbers, fields in declaration order
    assert engine_state_json(7, 5) == b'{"current_phase":7,"last_committed_phase":5,"snapshot":null}'
    b = engine_state_json(9, 9, (3, b"hi"))
    assert b == (b'{"current_phase":9,"last_committed_phase":9,"snapshot":{"version":3,"data":[104,105],'
                 b'"checksum":' + str(zlib.crc32(b"hi")).encode() + b'}}')
    assert parse_engine_state_json(b)["snapshot"]["data"] == [104, 105]
    bad = json.loads(b)
    bad["snapshot"]["checksum"] ^= 1
    with pytest.raises(ValueError):
        parse_engine_state_json(json.dumps(bad).encode())


def test_checkpoint_roundtrip_and_corruption(tmp_path):
    rng = np.random.default_rng(1)
    n = 1000
    nw = (n + 31) // 32
    ck = Checkpoint(11, n, 1010, 900, 950, 77, 4, rng.integers(0, 2**32, nw, dtype=np.uint32),
                    rng.integers(0, 2**32, nw, dtype=np.uint32))
    b = ck.to_bytes()
    back = Checkpoint.from_bytes(b)
    assert (back.slot_base, back.n_slots, back.current_phase, back.last_committed, back.commit_watermark,
            back.rng_next, back.steps) == (11, n, 1010, 900, 950, 77, 4)
    assert np.array_equal(back.committed, ck.committed) and np.array_equal(back.v1, ck.v1)
    for pos in (0, 20, len(b) // 2, len(b) - 1):
        flipped = bytearray(b)
        flipped[pos] ^= 0x10
        with pytest.raises(ValueError):
            Checkpoint.from_bytes(bytes(flipped))
    path = str(tmp_path / "state.bin")
    assert Checkpoint.load(path) is None          # first start: load_state -> Ok(None)
    ck.save(path)
    assert Checkpoint.load(path).to_bytes() == b


@pytest.mark.gpu
def test_gpu_checkpoint_resume_equals_uninterrupted(oracle, tmp_path):
    """Three windows on one engine vs. two windows, checkpoint to disk, a fresh
    engine restored from it, third window: identical outputs and state; the
    checkpoint's bitmaps equal the step's committed / V1 planes."""
    import torch
    from rabia_amd import checkpoint as C
    from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs, unpack_bits
    n, S = 5, 50_000
    wins = []
    for w in range(3):
        r1, r2, _ = oracle.trace(w % 3, n, 100 + w, 1 + w * S, S)
        wins.append(PhaseWindow.from_codes(r1, r2, slot_base=1 + w * S))
    with PhaseEvaluator(n, self_lane=4, mode="ref", seed=5) as a:
        outs = [a.phase_step_host(win)[0] for win in wins]
        final_a = a.get_state()
    with PhaseEvaluator(n, self_lane=4, mode="ref", seed=5) as b:
        for win in wins[:2]:
            out, _ = b.phase_step_host(win)
        stride = out.shape[1]
        out_d = torch.from_numpy(out.view(np.int32).copy()).cuda()
        torch.cuda.synchronize()
        ck = C.capture(b, out_d.data_ptr(), S, stride, wins[1].slot_base, current_phase=wins[1].slot_base + S - 1)
        dec = decode_outputs(out, S)
        assert np.array_equal(unpack_bits(ck.committed, S), dec["committed"])
        assert np.array_equal(unpack_bits(ck.v1, S), dec["value"])
        ck.save(str(tmp_path / "ck.bin"))
    loaded = Checkpoint.load(str(tmp_path / "ck.bin"))
    with PhaseEvaluator(n, self_lane=4, mode="ref", seed=5) as c:
        C.restore(c, loaded)
        out3, _ = c.phase_step_host(wins[2])
        assert np.array_equal(out3, outs[2])
        assert c.get_state() == final_a
