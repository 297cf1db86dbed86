"""Persistent lag REF kernel (ref_lag_kernel, rg_kernels.h): parity with the oracle
and with the tiled kernel, forced onto small launches with small grids so every
workgroup runs many tickets (parking, look-back bounded by its own previous tile,
the early and the continued look-back), and the concurrent-launch case that the
tiled kernel's dispatch-order look-back cannot take.

Run on an MI355X: python -m pytest tests/test_lag_kernel.py -m gpu -x -q
"""
import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs
from test_gpu_parity import RES_CMP, assert_same, torch_cuda

pytestmark = pytest.mark.gpu

LAG = 0x200000       # rg_debug_set: the lag kernel at any launch size
TILED = 0x100000     # rg_debug_set: large launches keep the tiled kernel


def lag_diag(grid=0):
    return LAG | ((grid & 0xFF) << 24)


def run_ref_diag(diag, n, q, self_lane, seed, rng_base, slot_base, r1, r2, max_phase=0, lc_in=0, wm_in=1):
    with PhaseEvaluator(n, quorum=q, self_lane=self_lane, mode="ref", seed=seed) as ev:
        N.check(ev.lib.rg_debug_set(ev.ctx, diag), ev.ctx)
        ev.set_state(rng_next=rng_base, last_committed=lc_in, commit_watermark=wm_in)
        out, res = ev.phase_step_host(PhaseWindow.from_codes(r1, r2, slot_base=slot_base), max_phase=max_phase)
        st = ev.get_state()
    assert res["flags"] == 0
    assert st["rng_next"] == res["rng_next"] and st["last_committed"] == res["last_committed_max"]
    return decode_outputs(out, r1.shape[0]), res


@pytest.mark.parametrize("grid", [1, 3, 7, 0])
@pytest.mark.parametrize("S", [1, 33, 16385, 100003, (1 << 20) + 17])
@pytest.mark.parametrize("n", [1, 3, 5, 9, 16])
def test_lag_vs_oracle(oracle, n, S, grid):
    for kind in (0, 1, 2):
        r1, r2, _ = oracle.trace(kind, n, 2000 + S + n, 11, S)
        q = n // 2 + 1
        exp, eres = oracle.ref_step(n, q, n // 2, 42, 99, 11, r1, r2, max_phase=11 + S // 3, lc_in=3, wm_in=11)
        got, res = run_ref_diag(lag_diag(grid), n, q, n // 2, 42, 99, 11, r1, r2, max_phase=11 + S // 3,
                                lc_in=3, wm_in=11)
        assert_same(got, exp, res, eres)


def test_lag_no_self_lane_and_low_quorum(oracle):
    S = 70001
    for n, q, self_lane in ((5, 2, -1), (4, 2, 0), (7, 3, 6)):
        r1, r2, _ = oracle.trace(0, n, 5 + n, 1, S)
        exp, eres = oracle.ref_step(n, q, self_lane, 9, 0, 1, r1, r2)
        got, res = run_ref_diag(lag_diag(2), n, q, self_lane, 9, 0, 1, r1, r2)
        assert_same(got, exp, res, eres)


def _device_step(torch, diag, n, S, kind, seed, windows=1):
    """Device-resident REF step(s) over `windows` consecutive S-slot windows; returns
    the output planes, per-window results and the final engine state."""
    stride = ((S + 127) // 128) * 4
    votes = torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    out = torch.empty(8 * stride * windows, dtype=torch.int32, device="cuda")
    res = torch.zeros((windows, 10), dtype=torch.int64, device="cuda")
    with PhaseEvaluator(n, self_lane=n - 1, seed=42) as ev:
        N.check(ev.lib.rg_debug_set(ev.ctx, diag), ev.ctx)
        for w in range(windows):
            ev.trace_generate_async(kind, seed + w, 1 + w * S, S, stride, votes.data_ptr())
            ev.phase_step_async(votes.data_ptr(), out.data_ptr() + 4 * 8 * stride * w, S, stride,
                                slot_base=1 + w * S, result_ptr=res[w].data_ptr())
        st = ev.get_state()
    return out, res.cpu().numpy().view(np.uint64), st


@pytest.mark.parametrize("shape", [0, 0x400000])  # one 1024-thread WG per CU (default); 2 x 512-thread WGs per CU
@pytest.mark.parametrize("kind", [N.RG_TRACE_AGREE90, N.RG_TRACE_SPLIT, N.RG_TRACE_UNIFORM])
def test_lag_equals_tiled_large(kind, shape):
    """2^25 slots (512 lag tiles over 256 workgroups, or 1024 over 512), three windows back to back:
    the lag kernel's outputs, step results and engine state equal the tiled kernel's."""
    torch = torch_cuda()
    n, S = 5, 1 << 25
    o1, r1, s1 = _device_step(torch, TILED, n, S, kind, 7, windows=3)
    o2, r2, s2 = _device_step(torch, shape, n, S, kind, 7, windows=3)
    assert (r1[:, 9] == 0).all() and (r2[:, 9] == 0).all()
    assert torch.equal(o1, o2)
    assert (r1 == r2).all()
    assert s1 == s2


def test_lag_small_grid_large_launch():
    """A 7-workgroup grid over 2^24 slots (73 tickets per workgroup, the look-back
    scan often ending at the workgroup's own previous tile) == the tiled kernel."""
    torch = torch_cuda()
    n, S = 5, 1 << 24
    o1, r1, s1 = _device_step(torch, TILED, n, S, N.RG_TRACE_AGREE90, 3)
    o2, r2, s2 = _device_step(torch, lag_diag(7), n, S, N.RG_TRACE_AGREE90, 3)
    assert r2[0, 9] == 0
    assert torch.equal(o1, o2) and (r1 == r2).all() and s1 == s2


@pytest.mark.parametrize("S", [1 << 29, 1 << 26, 1 << 23])
def test_lag_concurrent_contexts_two_streams(S):
    """Two contexts on one GPU launch REF steps on two streams at once. At 2^29 slots
    the lag kernel runs (>= 32 tiles per CU) and takes tiles by ticket, so neither
    launch can wait on a workgroup that the other holds off the GPU (the tiled
    kernel's cross-kernel look-back cycle); at 2^26 and 2^23 slots the tiled kernel
    runs and the C ABI chains the two contexts' launches through its per-device event.
    Both finish with flags 0 and outputs equal to serial runs."""
    torch = torch_cuda()
    n = 5
    stride = ((S + 127) // 128) * 4
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    votes = [torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda") for _ in range(2)]
    outs = [torch.empty(8 * stride, dtype=torch.int32, device="cuda") for _ in range(2)]
    res = torch.zeros((2, 4, 10), dtype=torch.int64, device="cuda")
    evs = [PhaseEvaluator(n, self_lane=4, seed=42 + i) for i in range(2)]
    try:
        for i in range(2):
            evs[i].trace_generate_async(N.RG_TRACE_AGREE90, 100 + i, 1, S, stride, votes[i].data_ptr())
        torch.cuda.synchronize()
        for rep in range(4):  # both streams busy at once, several launches deep
            for i in range(2):
                evs[i].phase_step_async(votes[i].data_ptr(), outs[i].data_ptr(), S, stride, slot_base=1 + rep * S,
                                        result_ptr=res[i, rep].data_ptr(), stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        st = [ev.get_state() for ev in evs]
    finally:
        for ev in evs:
            ev.close()
    r = res.cpu().numpy().view(np.uint64)
    assert (r[:, :, 9] == 0).all(), "look-back fault flags"
    # serial reference: the same four launches per context, one context at a time
    for i in range(2):
        o_ser = torch.empty_like(outs[i])
        with PhaseEvaluator(n, self_lane=4, seed=42 + i) as ev:
            rr = torch.zeros((4, 10), dtype=torch.int64, device="cuda")
            for rep in range(4):
                ev.phase_step_async(votes[i].data_ptr(), o_ser.data_ptr(), S, stride, slot_base=1 + rep * S,
                                    result_ptr=rr[rep].data_ptr())
            st_ser = ev.get_state()
        assert torch.equal(o_ser, outs[i])
        assert (rr.cpu().numpy().view(np.uint64) == r[i]).all()
        assert st_ser == st[i]
