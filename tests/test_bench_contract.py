"""bench.py pieces that need no GPU: the defaults the driver's plain `python bench.py`
relies on (N = 1, the C2 headline at 2^30 slots per step, a warm-up past the clock
ramp), and the HBM traffic records the line attaches: one per step-kernel launch shape,
picked only when its replica count and slots per launch match the run's launch."""
import json
import os
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defaults(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus is None and a.config == "c2" and not a.sharded and a.backend == "nccl"
    assert a.windows * bench.WINDOW == 1 << 30 and a.replicas == 5 and a.tile_words == 1024
    assert a.steps == 50 and a.warmup >= 20  # tools/warm_probe.py: clocks settle over ~20 launches
    assert a.fixup_stream == "fix" and a.diag == 0 and a.pmc_file is None


def test_bytes_per_slot():
    assert bench.bytes_per_slot_ref(5) == 3.5  # 4n bits read + 8 bits written
    assert bench.bytes_per_slot_ref(9) == 5.5


@pytest.mark.parametrize("name,n,sizes", [("pmc_c2.json", 5, [1 << 30]), ("pmc_c2_sharded.json", 5, [1 << 30]),
                                          ("pmc_c5.json", 9, [1 << 31]), ("pmc_c5_sharded.json", 9, [1 << 31, 1 << 28])])
def test_pmc_records(name, n, sizes):
    path = os.path.join(ROOT, "profiles", name)
    with open(path) as f:
        recs = json.load(f)
    recs = recs.get("records", [recs])
    assert sorted(d["slots_per_launch"] for d in recs) == sorted(sizes)
    for d in recs:
        slots = d["slots_per_launch"]
        assert d["replicas"] == n
        assert d["alg_bytes_per_launch"] == slots * bench.bytes_per_slot_ref(n)
        # FETCH_SIZE doubled (the gfx950 correction) + WRITE_SIZE, both in KB
        assert d["hbm_bytes_per_launch"] == 2 * d["fetch_size_kb_median"] * 1024 + d["write_size_kb_median"] * 1024
        assert d["traffic_over_alg"] == pytest.approx(d["hbm_bytes_per_launch"] / d["alg_bytes_per_launch"])
        assert 1.0 <= d["traffic_over_alg"] < 1.05
        assert min(d["dispatches"]) >= 5
        assert bench.load_pmc(path, n, slots) == d["hbm_bytes_per_launch"]
        assert bench.load_pmc(path, n + 2, slots) is None
        assert bench.load_pmc(path, n, slots // 2) is None
        assert bench.load_pmc(path + ".missing", n, slots) is None


def test_c3_bytes_per_slot_matches_the_call():
    """The C3 roofline's bytes follow the call the step makes (the fused-bitmap cluster
    call: no bitmap-kernel re-read of the info words; the coin table lives in LDS, so it
    moves no HBM bytes) and the coin table's phase count in rabia_gpu.hip."""
    import re
    src = open(os.path.join(ROOT, "rabia_amd", "csrc", "rabia_gpu.hip")).read()
    assert int(re.search(r"#define RG_COIN_TABLE_PHASES (\d+)", src).group(1)) == bench.C3_COIN_TABLE_PHASES
    bsrc = open(os.path.join(ROOT, "bench.py")).read()
    assert "ev.wmvc_cluster_bitmaps_async(" in bsrc and "ev.wmvc_cluster_async(" not in bsrc
    assert bench.c3_bytes_per_slot(5, 2.0) == pytest.approx(5 / 8 + 4 + 2 / 8)


def test_layout():
    stride, in_w, out_w = bench.layout(5, 1 << 30, 1024)
    tiles = (1 << 25) // 1024
    assert stride == 1024 and in_w == tiles * 21 * 1024 and out_w == tiles * 8 * 1024
    stride, in_w, out_w = bench.layout(9, 1000, 0)  # planar: 16-byte aligned plane stride in words
    assert stride == 32 and in_w == 37 * 32 and out_w == 8 * 32


class _Ev:  # stands in for a recorded torch.cuda.Event pair (elapsed_time in ms)
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_launch_timing_policy(monkeypatch):
    """Per-launch events: none for the single evaluator (span / K), every `every`-th launch
    for the pipelines (the kernel alone), every launch with --launch-events."""
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    a.steps = 8
    assert bench.launch_events(a) is None
    assert bench.launch_ms(None, 10.0, 8) == pytest.approx(1.25)
    if bench.torch.cuda.is_available():
        evs = bench.launch_events(a, every=4)
        assert [e is not None for e in evs] == [True, False, False, False, True, False, False, False]
    timed = [(_Ev(0.0), _Ev(0.6)), None, None, None, (_Ev(1.0), _Ev(1.8)), None, None, None]
    assert bench.launch_ms(timed, 10.0, 8) == pytest.approx(0.7)  # the sampled launches only
