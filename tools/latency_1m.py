"""Single-window (2^20 slots, n=5) REF step latency by tile shape and with the
look-back (diag 1) or the statistics/finalisation (diag 2) switched off
(diagnostics only; a switched-off variant is not a valid result).
Run on the GPU box: python tools/latency_1m.py > gpurun_out/latency_1m.json"""
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
n, T, S = 5, 1024, 1 << 20
ev = PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T)
nw = S // 32
sets = []
for i in range(8):
    v = torch.empty(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    o = torch.empty(((nw + T - 1) // T) * 8 * T, dtype=torch.int32, device="cuda")
    ev.trace_generate_async(N.RG_TRACE_AGREE90, i, 1, S, T, v.data_ptr(), sp)
    sets.append((v, o))
torch.cuda.synchronize()

variants = {}
for shape, force in (("auto", 0), ("512x4", 1), ("256x4", 2), ("128x1", 3)):
    for tag, d in (("", 0), ("_no_lookback", 1), ("_no_stats", 2), ("_neither", 3)):
        variants[shape + tag] = (force << 8) | d
times = {k: [] for k in variants}
for r in range(6):
    for name, diag in variants.items():
        lib.rg_debug_set(ev.ctx, diag)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(20):
            v, o = sets[k % len(sets)]
            ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1, stream=sp)
        e1.record(stream)
        e1.synchronize()
        if r > 0:
            times[name].append(e0.elapsed_time(e1) * 1000.0 / 20)
lib.rg_debug_set(ev.ctx, 0)
print(json.dumps({"slots": S, "us_per_launch_median": {k: round(float(np.median(t)), 2) for k, t in times.items()}},
                 indent=1), flush=True)
