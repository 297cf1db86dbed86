"""Decision bitmaps (the multi-GPU exchange payload, include/rabia_gpu.h
rg_decision_bitmap_async) equal output planes 6 and 7 of the step."""
import numpy as np
import pytest


@pytest.mark.gpu
@pytest.mark.parametrize("T,S", [(0, 100_003), (1024, 1 << 20), (64, 70_001)])
def test_decision_bitmap_matches_step_outputs(oracle, T, S):
    import torch
    from rabia_amd.engine import PhaseEvaluator, PhaseWindow, decode_outputs, plane_stride, to_tiled
    from rabia_amd.engine import unpack_bits
    n = 9
    r1, r2, _ = oracle.trace(1, n, 3, 1, S)
    win = PhaseWindow.from_codes(r1, r2, slot_base=1)
    nw = (S + 31) // 32
    with PhaseEvaluator(n, self_lane=8, mode="ref", seed=1, tile_words=T) as ev:
        planes = np.ascontiguousarray(win.planes)
        host_in = to_tiled(planes, nw, T) if T else planes.reshape(-1)
        votes = torch.from_numpy(host_in.view(np.int32).copy()).cuda()
        stride = T if T else plane_stride(S)
        out_words = ((nw + T - 1) // T) * 8 * T if T else 8 * stride
        out = torch.empty(out_words, dtype=torch.int32, device="cuda")
        cm = torch.empty(nw, dtype=torch.int32, device="cuda")
        v1 = torch.empty(nw, dtype=torch.int32, device="cuda")
        ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=1)
        ev.decision_bitmap_async(out.data_ptr(), S, stride, cm.data_ptr(), v1.data_ptr())
        ev.sync()
    exp, _ = oracle.ref_step(n, n // 2 + 1, 8, 1, 0, 1, r1, r2)
    assert np.array_equal(unpack_bits(cm.cpu().numpy().view(np.uint32), S), exp["committed"])
    assert np.array_equal(unpack_bits(v1.cpu().numpy().view(np.uint32), S), exp["value"])
