"""Own round-1 votes for received proposals: determine_round1_vote
/ randomized_vote (rabia-engine/src/engine.rs:424-481) batched on the device
(rg_round1_votes_async) against the Python restatement (oracle/rabia_ref.py)."""
import random

import numpy as np
import pytest

import rabia_ref as R


def test_restatement_branches():
    # existing proposal: equal -> same value, conflicting -> VQ, no draws
    votes, draws = R.round1_votes(42, 0, [(5, 1), (5, 0), (6, 2)], [R.NONE, 1, R.NONE], 4)
    assert votes == [1, 2, 2] and draws == 0
    # first proposals draw (V0: P70, V1: P80); VQuestion proposals never draw
    key = R.seed_from_u64(42)
    u0, u1 = R.ref_draw(key, 0), R.ref_draw(key, 1)
    votes, draws = R.round1_votes(42, 0, [(1, 0), (2, 1), (3, 2)], [R.NONE] * 4, 0)
    assert draws == 2
    assert votes == [0 if u0 < R.P_INT[0.7] else 2, 1 if u1 < R.P_INT[0.8] else 2, 2]
    # the reference as it runs: phases never exist, every proposal draws
    votes, draws = R.round1_votes(42, 0, [(1, 1), (1, 1)], [], 0, track=False)
    assert draws == 2


@pytest.mark.gpu
@pytest.mark.parametrize("n_props,S,track", [(1, 10, True), (5000, 3000, True), (100_000, 40_000, True),
                                             (50_000, 0, False)])
def test_gpu_round1_votes_vs_restatement(n_props, S, track):
    import torch
    from rabia_amd.engine import PhaseEvaluator, plane_stride, unpack_bits
    rng = random.Random(n_props + S)
    slot_base = 100
    span = max(S, 1)
    props = [(slot_base - 3 + rng.randrange(span + 6), rng.choice([0, 1, 1, 1, 2])) for _ in range(n_props)]
    proposed = [rng.choice([R.NONE, R.NONE, R.NONE, 0, 1, 2]) for _ in range(S)]
    exp_prop = list(proposed)
    rng_base = 17
    exp, draws = R.round1_votes(7, rng_base, props, exp_prop, slot_base, track)
    stride = plane_stride(max(S, 1))
    planes = np.zeros((2, stride), np.uint32)
    for s_, c in enumerate(proposed):
        if c & 1:
            planes[0, s_ >> 5] |= 1 << (s_ & 31)
        if c & 2:
            planes[1, s_ >> 5] |= 1 << (s_ & 31)
    with PhaseEvaluator(5, self_lane=4, mode="ref", seed=7) as ev:
        ev.set_state(rng_next=rng_base)
        ph = torch.tensor([p for p, _ in props], dtype=torch.int64, device="cuda")
        vals = torch.tensor([v for _, v in props], dtype=torch.uint8, device="cuda")
        prop_d = torch.from_numpy(planes.view(np.int32).copy()).cuda()
        votes = torch.empty(n_props, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ev.round1_votes_async(ph.data_ptr(), vals.data_ptr(), n_props, prop_d.data_ptr(), stride, S, slot_base,
                              track, votes.data_ptr())
        ev.sync()
        assert votes.cpu().numpy().tolist() == exp
        assert ev.get_state()["rng_next"] == rng_base + draws
        if track:
            got = prop_d.cpu().numpy().view(np.uint32)
            codes = unpack_bits(got[0], S) | (unpack_bits(got[1], S) << 1)
            assert codes.tolist() == exp_prop
