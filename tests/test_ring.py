"""The persistent software-pipelined REF kernel (ref_pipe_kernel, rg_kernels.h) vs the
oracle and vs the default tiled kernel. It is a diagnostic path (rg_debug_set bits
8-10 = 6 force it at any size; measured slower than the tiled kernel),
kept bit-exact: small and ragged cases, more than 1024 draws in a tile (several
ChaCha12 staging passes), 1 or 2 workgroups per CU, and a bench-shaped 2^26-slot
launch compared with the tiled kernel bit for bit (outputs, step result, device state
over consecutive steps)."""
import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs

pytestmark = pytest.mark.gpu

RING = 6 << 8
PAIR = 7 << 8
TILED = 0x8000
RES_CMP = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws", "last_committed_max",
           "first_undecided", "rng_next", "commit_watermark"]


def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def run_ref(diag, n, q, self_lane, seed, rng_base, slot_base, r1, r2, max_phase=0, lc_in=0, wm_in=1):
    with PhaseEvaluator(n, quorum=q, self_lane=self_lane, mode="ref", seed=seed) as ev:
        N.check(ev.lib.rg_debug_set(ev.ctx, diag), ev.ctx)
        ev.set_state(rng_next=rng_base, last_committed=lc_in, commit_watermark=wm_in)
        w = PhaseWindow.from_codes(r1, r2, slot_base=slot_base)
        out, res = ev.phase_step_host(w, max_phase=max_phase)
        st = ev.get_state()
    assert res["flags"] == 0
    assert st["rng_next"] == res["rng_next"] and st["last_committed"] == res["last_committed_max"]
    return decode_outputs(out, r1.shape[0]), res


@pytest.mark.parametrize("S", [1, 33, 4097, 100003, (1 << 20) + 17, 3 << 20])
@pytest.mark.parametrize("n", [3, 5, 9, 16])
def test_pair_vs_oracle(oracle, n, S):
    """The paired-tile kernel (two consecutive look-back tiles per workgroup, the
    second without a look-back of its own), forced at every size."""
    q = n // 2 + 1
    for kind in (0, 1, 2):
        r1, r2, _ = oracle.trace(kind, n, 3000 + S + n, 7, S)
        exp, eres = oracle.ref_step(n, q, n // 2, 42, 123, 7, r1, r2, max_phase=7 + S // 2, lc_in=2, wm_in=7)
        got, res = run_ref(PAIR, n, q, n // 2, 42, 123, 7, r1, r2, max_phase=7 + S // 2, lc_in=2, wm_in=7)
        for k in exp:
            np.testing.assert_array_equal(got[k], exp[k], err_msg=f"{k} kind {kind}")
        assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}


@pytest.mark.parametrize("S", [1, 33, 4097, 100003, (1 << 20) + 17, 3 << 20])
@pytest.mark.parametrize("n", [3, 5, 9, 16])
def test_ring_vs_oracle(oracle, n, S):
    q = n // 2 + 1
    for kind in (0, 1, 2):
        r1, r2, _ = oracle.trace(kind, n, 2000 + S + n, 7, S)
        exp, eres = oracle.ref_step(n, q, n // 2, 42, 123, 7, r1, r2, max_phase=7 + S // 2, lc_in=2, wm_in=7)
        for per_cu in (1, 2):
            got, res = run_ref(RING | (per_cu << 12), n, q, n // 2, 42, 123, 7, r1, r2,
                               max_phase=7 + S // 2, lc_in=2, wm_in=7)
            for k in exp:
                np.testing.assert_array_equal(got[k], exp[k], err_msg=f"{k} kind {kind} per_cu {per_cu}")
            assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}


def test_ring_many_draws_per_tile(oracle):
    """Every slot VQ at round 1 (all lanes '?'): 65536 draws per tile, 64 ChaCha12
    staging passes of 1024 draws each."""
    n, q, S = 5, 3, (1 << 20) + 5
    rng = np.random.default_rng(5)
    r1 = np.full((S, n), 2, np.uint8)
    r1[rng.random(S) < 0.01, 0] = 0       # a few slots differ (c1 vs c0 classes)
    r1[rng.random(S) < 0.01, 1] = 1
    r2 = rng.integers(0, 4, (S, n)).astype(np.uint8)
    exp, eres = oracle.ref_step(n, q, 4, 9, 10 ** 9 + 3, 1, r1, r2)
    got, res = run_ref(RING, n, q, 4, 9, 10 ** 9 + 3, 1, r1, r2)
    for k in exp:
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}


def test_pair_many_draws_per_tile(oracle):
    """All-'?' round 1 with the paired kernel: both tiles of every workgroup draw
    65536 times (several ChaCha12 staging passes each)."""
    n, q, S = 5, 3, (3 << 20) + 5
    rng = np.random.default_rng(6)
    r1 = np.full((S, n), 2, np.uint8)
    r1[rng.random(S) < 0.01, 0] = 0
    r1[rng.random(S) < 0.01, 1] = 1
    r2 = rng.integers(0, 4, (S, n)).astype(np.uint8)
    exp, eres = oracle.ref_step(n, q, 4, 9, 10 ** 9 + 3, 1, r1, r2)
    got, res = run_ref(PAIR, n, q, 4, 9, 10 ** 9 + 3, 1, r1, r2)
    for k in exp:
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    assert {k: res[k] for k in RES_CMP} == {k: eres[k] for k in RES_CMP}


def test_ring_equals_tiled_bench_shape():
    """The bench's layout (slot-tiled 1024, n=5, agree90) at 2^26 slots, three
    consecutive steps on each kernel: identical output planes, step results and state."""
    torch = torch_cuda()
    n, T, S = 5, 1024, 1 << 26
    nw = S // 32
    votes = [torch.empty((nw // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda") for _ in range(3)]
    outs = {d: [torch.empty((nw // T) * 8 * T, dtype=torch.int32, device="cuda") for _ in range(3)]
            for d in (RING, PAIR, TILED)}
    res, st = {}, {}
    for d in (RING, PAIR, TILED):
        with PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T) as ev:
            N.check(ev.lib.rg_debug_set(ev.ctx, d), ev.ctx)
            if d == RING:
                for i in range(3):
                    ev.trace_generate_async(N.RG_TRACE_AGREE90, 30 + i, 1 + i * S, S, T, votes[i].data_ptr())
            torch.cuda.synchronize()
            res[d] = []
            for i in range(3):
                ev.phase_step_async(votes[i].data_ptr(), outs[d][i].data_ptr(), S, T, slot_base=1 + i * S,
                                    max_phase=3 * S - 999)
                res[d].append(ev.last_result())
            st[d] = ev.get_state()
    for d in (RING, PAIR):
        for i in range(3):
            assert torch.equal(outs[d][i], outs[TILED][i]), f"{d:#x} step {i}"
            assert res[d][i] == res[TILED][i], f"{d:#x} step {i}"
            assert res[d][i]["flags"] == 0 and res[d][i]["n_draws"] > 0
        assert st[d] == st[TILED]
