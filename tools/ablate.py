"""Where does a REF step's time go? Interleaved A/B timing of ablation variants
(diagnostic switches in rg_kernels.h) plus per-tile s_memrealtime stamps.
Run on the GPU box: python tools/ablate.py > gpurun_out/ablate.json"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

lib = N.load()
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sp = stream.cuda_stream
n = 5
S = int(os.environ.get("ABL_SLOTS", 1 << 26))
stride_min = ((S + 127) // 128) * 4
stride_pad = stride_min + 256
ev = PhaseEvaluator(n, self_lane=4, seed=42)
T = 1024
ev_t = PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T)
S_T = max(S, 1 << 28)  # slot-tiled sets also serve the 2^28-slot variants
nw = S_T // 32
tiled_sets = []
for i in range(3):
    v = torch.empty(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    o = torch.empty(((nw + T - 1) // T) * 8 * T, dtype=torch.int32, device="cuda")
    ev_t.trace_generate_async(N.RG_TRACE_AGREE90, i, 1, S_T, T, v.data_ptr(), sp)
    tiled_sets.append((v, o))
bufs = {}
for name, stride in (("min", stride_min), ("pad", stride_pad)):
    sets = []
    for i in range(3):
        v = torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
        o = torch.empty(8 * stride, dtype=torch.int32, device="cuda")
        ev.trace_generate_async(N.RG_TRACE_AGREE90, i, 1, S, stride, v.data_ptr(), sp)
        sets.append((v, o))
    bufs[name] = (stride, sets)
torch.cuda.synchronize()


def run(variant, k):
    if variant.get("tiled") and variant.get("probe"):
        v, o = tiled_sets[k % 3]
        N.check(lib.rg_debug_stream_probe(v.data_ptr(), o.data_ptr(), variant.get("slots", S) // 32, 0, T, 1, sp))
        return
    if variant.get("tiled"):
        v, o = tiled_sets[k % 3]
        lib.rg_debug_set(ev_t.ctx, variant.get("diag", 0))
        ev_t.phase_step_async(v.data_ptr(), o.data_ptr(), variant.get("slots", S), T, slot_base=1, stream=sp)
        return
    stride, sets = bufs[variant.get("stride", "min")]
    v, o = sets[k % 3]
    slots = variant.get("slots", S)
    if variant.get("probe"):
        N.check(lib.rg_debug_stream_probe(v.data_ptr(), o.data_ptr(), (slots + 31) // 32, stride, 0, 0, sp))
    else:
        lib.rg_debug_set(ev.ctx, variant.get("diag", 0))
        ev.phase_step_async(v.data_ptr(), o.data_ptr(), slots, stride, slot_base=1, stream=sp)


variants = {
    "big": {"tiled": True, "diag": 1 << 8},
    "big_no_lookback": {"tiled": True, "diag": 1 | (1 << 8)},
    "t_probe": {"tiled": True, "probe": True},
    "big_s28": {"tiled": True, "diag": 1 << 8, "slots": 1 << 28},
    "big_no_lookback_s28": {"tiled": True, "diag": 1 | (1 << 8), "slots": 1 << 28},
    "t_probe_s28": {"tiled": True, "probe": True, "slots": 1 << 28},
    "auto_1M": {"tiled": True, "slots": 1 << 20},
}
times = {k: [] for k in variants}
for r in range(8):
    for name, var in variants.items():
        for k in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run(var, k)
            e1.record(stream)
            e1.synchronize()
            if r > 0:
                times[name].append(e0.elapsed_time(e1) * 1000.0)
summary = {}
for name, ts in times.items():
    slots = variants[name].get("slots", S)
    med = float(np.median(ts))
    summary[name] = {"median_us": med, "min_us": float(np.min(ts)),
                     "GBps_at_3.5B": slots * 3.5 / (med * 1e-6) / 1e9}

print(json.dumps({"slots": S, "timing": summary}), flush=True)
stamps = {}
for slots in (S, 1 << 20):
    lib.rg_debug_set(ev_t.ctx, 4)
    v, o = tiled_sets[0]
    ev_t.phase_step_async(v.data_ptr(), o.data_ptr(), slots, T, slot_base=1, stream=sp)
    torch.cuda.synchronize()
    buf = np.zeros(1 << 20, np.uint64)
    N.check(lib.rg_debug_stamps(ev_t.ctx, buf.ctypes.data, buf.size), ev_t.ctx)
    ntl = int(np.count_nonzero(buf.reshape(-1, 8)[:, 0]))
    st = buf.reshape(-1, 8)
    st = st[st[:, 0] != 0].astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
    if st.shape[0] == 0:  # the persistent kernel writes no per-tile stamps
        stamps[str(slots)] = None
        continue
    t0 = st[:, 0].min()
    d = {"tiles": int(st.shape[0]),
         "start_span_us": float(st[:, 0].max() - t0),
         "end_us": float(st[:, 4][st[:, 4] > 0].max() - t0),
         "phase_median_us": {"compute_waves": float(np.median(st[:, 1] - st[:, 0])),
                             "lookback": float(np.median(st[:, 2] - st[:, 1])),
                             "draws+final_planes": float(np.median(st[:, 3] - st[:, 2])),
                             "finish": float(np.median(st[:, 4] - st[:, 3]))},
         "phase_p90_us": {"compute_waves": float(np.percentile(st[:, 1] - st[:, 0], 90)),
                          "lookback": float(np.percentile(st[:, 2] - st[:, 1], 90)),
                          "draws+final_planes": float(np.percentile(st[:, 3] - st[:, 2], 90)),
                          "finish": float(np.percentile(st[:, 4] - st[:, 3], 90))},
         "tile_life_median_us": float(np.median(st[:, 4] - st[:, 0]))}
    last = st[np.argmax(st[:, 0])]
    d["last_tile_reduce_us"] = float(last[5] - last[3]) if last[5] > 0 else None
    stamps[str(slots)] = d
lib.rg_debug_set(ev.ctx, 0)
lib.rg_debug_set(ev_t.ctx, 0)
print(json.dumps({"stamps": stamps}, indent=1))
