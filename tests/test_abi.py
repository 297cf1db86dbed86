"""CPU tests of the C-ABI library: it loads, exports every symbol the header
declares, and its host-side helpers agree with the oracle. No device calls."""
import ctypes

import numpy as np
import pytest

from rabia_amd import _native as N
from rabia_amd.engine import PhaseWindow, StateValue, node_id_from_u32, ClusterConfig, decode_outputs


def test_header_symbols_exported():
    lib = N.load()
    syms = N.header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"librabia_gpu.so does not export {s}"
        assert s in N._SIGS, f"binding lacks a signature for {s}"
    assert lib.rg_abi_version() == 6


def test_reservation_entry_points_error_path():
    """The reservation calls (rg_reserve, rg_comm_reserve) and the compact-payload entry
    points validate their arguments on the host before any device work: a null context is
    RG_EINVAL with a message, no device touched (no GPU needed)."""
    lib = N.load()
    assert lib.rg_reserve(None, 1 << 20, 4) == N.RG_EINVAL
    assert b"null context" in lib.rg_last_error(None)
    assert lib.rg_comm_reserve(None, 4, 1 << 20, 16) == N.RG_EINVAL
    assert lib.rg_decision_lists_windows_async(None, 1, None, 0, 1024, 0, None, 16, None, 0, None) == N.RG_EINVAL
    assert lib.rg_shard_exchange_decisions_async(None, 1, None, 0, 1024, 0, 1, 1, 1024, 0, None, 0, None, None, 16, 1,
                                                 None, None) == N.RG_EINVAL


def test_plane_stride():
    lib = N.load()
    for n, want in ((1, 4), (32, 4), (128, 4), (129, 8), (1 << 20, 1 << 15)):
        assert lib.rg_plane_stride(n) == want


@pytest.mark.parametrize("n,S", [(1, 1), (5, 33), (9, 1000), (16, 257)])
def test_pack_matches_oracle(oracle, n, S):
    rng = np.random.default_rng(n * 1000 + S)
    codes = rng.integers(0, 4, (S, n), dtype=np.uint8)
    stride = ((S + 127) // 128) * 4
    lib = N.load()
    planes = np.zeros((2 * n, stride), np.uint32)
    N.check(lib.rg_pack_codes(codes.ctypes.data, n, S, stride, planes.ctypes.data))
    np.testing.assert_array_equal(planes, oracle.pack_planes(codes, stride))
    back = np.zeros_like(codes)
    N.check(lib.rg_unpack_planes(planes.ctypes.data, n, S, stride, back.ctypes.data))
    np.testing.assert_array_equal(back, codes)


def test_pack_rejects_bad_args():
    lib = N.load()
    codes = np.zeros((4, 3), np.uint8)
    planes = np.zeros((6, 4), np.uint32)
    assert lib.rg_pack_codes(codes.ctypes.data, 17, 4, 4, planes.ctypes.data) == N.RG_EINVAL
    assert lib.rg_pack_codes(None, 3, 4, 4, planes.ctypes.data) == N.RG_EINVAL
    with pytest.raises(N.RabiaGpuError):
        N.check(lib.rg_pack_codes(codes.ctypes.data, 3, 1000, 4, planes.ctypes.data))


def test_phase_window_mirror():
    """PhaseWindow.add_round{1,2}_vote mirrors PhaseData (messages.rs:169-175):
    last write wins, absent by default."""
    w = PhaseWindow(5, 40, slot_base=100)
    w.add_round1_vote(101, 2, StateValue.V1)
    w.add_round1_vote(101, 2, StateValue.V0)   # overwrite
    w.add_round2_vote(139, 4, StateValue.VQuestion)
    codes = np.zeros((40, 5), np.uint8)
    lib = N.load()
    N.check(lib.rg_unpack_planes(w.planes[:10].ctypes.data, 5, 40, w.stride, codes.ctypes.data))
    assert codes[1, 2] == 0 and codes[0, 0] == 3 and (codes[2:] == 3).all()
    N.check(lib.rg_unpack_planes(w.planes[10:20].ctypes.data, 5, 40, w.stride, codes.ctypes.data))
    assert codes[39, 4] == 2 and codes[38, 4] == 3
    with pytest.raises(IndexError):
        w.add_round1_vote(140, 0, StateValue.V0)


def test_node_ids_and_quorum():
    """NodeId::from(u32) bytes (types.rs:49-75) and quorum n/2+1 (network.rs:15)."""
    assert node_id_from_u32(0x01020304) == bytes([1, 2, 3, 4] * 4)
    nodes = [node_id_from_u32(i) for i in (5, 1, 3)]
    cc = ClusterConfig(node_id=nodes[0], all_nodes=nodes)
    assert cc.quorum_size == 2 and cc.lane_of(nodes[0]) == 2
    assert ClusterConfig(nodes[0], [node_id_from_u32(i) for i in range(9)]).quorum_size == 5


def test_decode_outputs_layout():
    out = np.zeros((8, 4), np.uint32)
    out[0, 0] = 0b01
    out[1, 0] = 0b10
    out[6, 0] = 0b11
    d = decode_outputs(out, 3)
    assert list(d["r1"]) == [1, 2, 0] and list(d["committed"]) == [1, 1, 0]


def test_create_without_device_fails_loudly():
    """No CPU fallback: with no gfx950 device, rg_create must fail (RG_ENODEV)."""
    lib = N.load()
    cnt = ctypes.c_int(0)
    rc = lib.rg_device_count(ctypes.byref(cnt))
    if rc == 0 and cnt.value > 0:
        pytest.skip("a device is present")
    cfg = N.RgConfig(n_replicas=5)
    ctx = ctypes.c_void_p()
    rc = lib.rg_create(ctypes.byref(ctx), ctypes.byref(cfg))
    assert rc in (N.RG_ENODEV, N.RG_EHIP)
    assert not ctx.value
    assert lib.rg_last_error(None)


@pytest.mark.parametrize("P,nw,T", [(21, 1, 64), (21, 1000, 64), (8, 4096, 1024), (3, 5000, 2048)])
def test_tiled_layout_roundtrip(P, nw, T):
    """Slot-tiled arrangement: word w of plane p at (w//T)*P*T + p*T + w%T."""
    from rabia_amd.engine import to_tiled, from_tiled
    stride = ((nw + 3) // 4) * 4
    rng = np.random.default_rng(P * nw)
    planar = rng.integers(0, 2 ** 32, (P, stride), dtype=np.uint64).astype(np.uint32)
    planar[:, nw:] = 0
    tiled = to_tiled(planar, nw, T)
    assert tiled.size == ((nw + T - 1) // T) * P * T
    for w in (0, nw // 2, nw - 1):
        for p_ in (0, P - 1):
            assert tiled[(w // T) * P * T + p_ * T + w % T] == planar[p_, w]
    np.testing.assert_array_equal(from_tiled(tiled, P, nw, T, stride), planar)


def test_record_window_words_matches_host_helpers():
    """The record-region size the library computes (rg_record_window_words, a pure function:
    no device call) equals the Python mirror and the oracle's table size + capacity."""
    from rabia_amd import _native as N
    from rabia_amd.engine import record_window_words
    import oracle_lib
    lib = N.load()
    for S, cap in [(1, 1), ((1 << 24) - 1, 5), (1 << 24, 0), ((1 << 24) + 1, 100), (1 << 30, 1 << 27), ((1 << 32) - 1, 7)]:
        assert lib.rg_record_window_words(S, cap) == record_window_words(S, cap) == oracle_lib.record_window_words(S, cap)
        assert (record_window_words(S, cap) - cap) % 4 == 0  # records start 16-B aligned
