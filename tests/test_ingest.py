"""Vote ingestion: wire messages -> packed vote planes.
CPU: the restatement (oracle/ingest_ref.py) on hand-built cases. GPU: the device
ingest (include/rabia_ingest.h) against the restatement on mixed streams, then the
phase step over the ingested window against the oracle's step on the same codes."""
import random
import struct

import numpy as np
import pytest

import ingest_ref as I

NOW = 1_700_000_000_000


def members_for(n, rng):
    return sorted(bytes(rng.randrange(256) for _ in range(16)) for _ in range(n))


def random_stream(rng, members, n_msgs, slot_base, n_slots, senders_known=True):
    """Valid votes (with duplicates that supersede), plus every rejection class."""
    n = len(members)
    msgs, senders = [], []
    outsider = bytes(rng.randrange(256) for _ in range(16))
    for _ in range(n_msgs):
        lane = rng.randrange(n)
        sender = members[lane]
        slot = slot_base + rng.randrange(n_slots)
        vote = rng.randrange(3)
        variant = rng.choice([I.VOTE_R1, I.VOTE_R2])
        ts = NOW - rng.randrange(5000)
        to = None if rng.random() < 0.7 else members[rng.randrange(n)]
        r1 = [(members[rng.randrange(n)], rng.randrange(3)) for _ in range(rng.randrange(1, 4))]
        kind = rng.random()
        slane = lane
        if kind < 0.03:
            slot = slot_base + n_slots + rng.randrange(100)           # outside the window
        elif kind < 0.05:
            slot = slot_base - 1 - rng.randrange(min(slot_base, 50) or 1) if slot_base > 0 else slot
        elif kind < 0.07:
            ts = NOW + 60_001 + rng.randrange(1000)                     # too far in the future
        elif kind < 0.09:
            ts = NOW - 600_001 - rng.randrange(1000)                    # too old
        elif kind < 0.11 and variant == I.VOTE_R2:
            r1 = []                                                      # empty round1_votes
        elif kind < 0.13:
            slane = (lane + 1) % n if n > 1 else lane                    # sender mismatch
        elif kind < 0.14:
            sender = outsider                                            # not a member
        body = I.vote_body(slot, bytes(16), vote, members[rng.randrange(n)],
                           r1 if variant == I.VOTE_R2 else None)
        m = I.encode_message(bytes(rng.randrange(256) for _ in range(16)), sender, to, ts, variant, body)
        if 0.14 <= kind < 0.16:
            m = m[:rng.randrange(len(m))]                                # truncated
        elif 0.16 <= kind < 0.17:
            m = m[:8 + 16 + 8 + 16] + b"\x02" + m[8 + 16 + 8 + 16 + 1:]  # Option tag 2
        elif 0.17 <= kind < 0.18:
            m = struct.pack("<Q", 15) + m[8:]                            # uuid length 15
        elif 0.18 <= kind < 0.19 and variant == I.VOTE_R1:
            m = m[:-28] + struct.pack("<I", 3) + m[-24:]                 # StateValue 3
        elif 0.19 <= kind < 0.22:
            m = I.encode_message(bytes(16), sender, None, ts, rng.choice([0, 3, 4, 5, 6, 7, 8]),
                                 bytes(rng.randrange(256) for _ in range(rng.randrange(40))))
        elif 0.22 <= kind < 0.23:
            m = I.encode_message(bytes(16), sender, None, ts, 9, b"")   # unknown variant
        msgs.append(m)
        senders.append(slane if senders_known else None)
    return msgs, senders


# ---------------------------------------------------------------- CPU -------
def test_parse_roundtrip_and_categories():
    rng = random.Random(1)
    mem = members_for(3, rng)
    body = I.vote_body(7, bytes(16), 1, mem[0], [(mem[1], 2)])
    m = I.encode_message(bytes(16), mem[2], None, NOW, I.VOTE_R2, body)
    assert I.parse(m) == ("vote", 2, mem[2], NOW, 7, 1, 1)
    r1 = np.full((3, 10), 3, np.uint8)
    r2 = np.full((3, 10), 3, np.uint8)
    st = I.ingest([m, m[:-1], I.encode_message(bytes(16), mem[2], None, NOW, 3, b"")], [2, 2, 2],
                  mem, NOW, 5, r1, r2)
    assert r2[2, 2] == 1 and (r1 == 3).all()
    assert st["r2"] == 1 and st["malformed"] == 1 and st["other"] == 1


def test_last_write_wins_by_sender_not_voter():
    rng = random.Random(2)
    mem = members_for(4, rng)
    msgs = [I.encode_message(bytes(16), mem[1], None, NOW, I.VOTE_R1, I.vote_body(3, bytes(16), v, mem[0]))
            for v in (0, 2, 1)]
    r1 = np.full((4, 8), 3, np.uint8)
    r2 = r1.copy()
    st = I.ingest(msgs, None, mem, NOW, 0, r1, r2)
    assert r1[1, 3] == 1 and r1[0, 3] == 3          # stored under the sender (lane 1)
    assert st["r1"] == 1 and st["superseded"] == 2


# ---------------------------------------------------------------- GPU -------
def _decode_codes(planes, n, S):
    from rabia_amd.engine import unpack_bits
    r1 = np.stack([unpack_bits(planes[2 * j], S) | (unpack_bits(planes[2 * j + 1], S) << 1) for j in range(n)])
    r2 = np.stack([unpack_bits(planes[2 * n + 2 * j], S) | (unpack_bits(planes[2 * n + 2 * j + 1], S) << 1)
                   for j in range(n)])
    return r1.astype(np.uint8), r2.astype(np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("n,S,T,calls,msgs", [(3, 100, 0, 2, 400), (5, 4096 + 7, 0, 3, 20000),
                                              (5, 1 << 16, 64, 2, 50000), (9, 3000, 128, 3, 9000),
                                              (16, 777, 0, 2, 5000)])
def test_gpu_ingest_vs_oracle(n, S, T, calls, msgs):
    import torch
    from rabia_amd.engine import from_tiled, plane_stride
    from rabia_amd.ingest import VoteIngestor
    rng = random.Random(n * 1000 + S)
    mem = members_for(n, rng)
    slot_base = 50
    P = 4 * n + 1
    nw = (S + 31) // 32
    if T:
        words = ((nw + T - 1) // T) * P * T
        stride = T
    else:
        stride = plane_stride(S)
        words = P * stride
    votes = torch.full((words,), -1, dtype=torch.int32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    r1 = np.full((n, S), 3, np.uint8)
    r2 = np.full((n, S), 3, np.uint8)
    exp = {c: 0 for c in I.CATS}
    with VoteIngestor(mem, tile_words=T) as ing:
        for c in range(calls):
            ms, snd = random_stream(rng, mem, msgs, slot_base, S, senders_known=(c % 2 == 0))
            I.ingest(ms, snd if c % 2 == 0 else None, mem, NOW, slot_base, r1, r2, exp)
            ing.ingest(ms, snd if c % 2 == 0 else None, NOW, votes, S, stride, slot_base, stats)
    host = votes.cpu().numpy().view(np.uint32)
    planes = from_tiled(host, P, nw, T, plane_stride(S)) if T else host.reshape(P, stride)
    g1, g2 = _decode_codes(planes, n, S)
    assert np.array_equal(g1, r1)
    assert np.array_equal(g2, r2)
    assert dict(zip(I.CATS, stats.cpu().numpy().tolist())) == exp


@pytest.mark.gpu
def test_gpu_ingest_then_phase_step(oracle):
    """End to end: wire messages -> ingest -> REF phase step == oracle step on the
    restated codes."""
    import torch
    from rabia_amd.engine import PhaseEvaluator, decode_outputs, plane_stride
    from rabia_amd.ingest import VoteIngestor
    n, S, slot_base = 5, 5000, 1
    rng = random.Random(77)
    mem = members_for(n, rng)
    ms, snd = random_stream(rng, mem, 40000, slot_base, S)
    r1 = np.full((n, S), 3, np.uint8)
    r2 = np.full((n, S), 3, np.uint8)
    I.ingest(ms, snd, mem, NOW, slot_base, r1, r2)
    stride = plane_stride(S)
    votes = torch.full(((4 * n + 1) * stride,), -1, dtype=torch.int32, device="cuda")
    stats = torch.zeros(8, dtype=torch.int64, device="cuda")
    with VoteIngestor(mem) as ing:
        ing.ingest(ms, snd, NOW, votes, S, stride, slot_base, stats)
    out = torch.empty(8 * stride, dtype=torch.int32, device="cuda")
    with PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=42) as ev:
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=slot_base)
        ev.sync()
    got = decode_outputs(out.cpu().numpy().view(np.uint32).reshape(8, stride), S)
    # oracle codes are [S][n] slot-major
    exp, _ = oracle.ref_step(n, n // 2 + 1, n - 1, 42, 0, slot_base, r1.T.copy(), r2.T.copy())
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
