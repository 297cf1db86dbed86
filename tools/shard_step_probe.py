#!/usr/bin/env python3
"""The REF step vs the sharded step (draw records) at the bench shape (n = 5, 2^30
slots, slot-tiled 1024, lag kernel), alone on the GPU: median us per launch over
back-to-back launches on rotating inputs. RABIA_GPU_LIB selects an experiment build.
Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

n, T = 5, 1024
S = int(os.environ.get("PROBE_SLOTS", 1 << 30))
P, nw = 4 * n + 1, S // 32
tiles = nw // T
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sp = stream.cuda_stream
sets = []
gen = PhaseEvaluator(n, tile_words=T)
for i in range(2):
    v = torch.empty(tiles * P * T, dtype=torch.int32, device="cuda")
    o = torch.empty(tiles * 8 * T, dtype=torch.int32, device="cuda")
    gen.trace_generate_async(N.RG_TRACE_AGREE90, 70 + i, 1, S, T, v.data_ptr(), sp)
    sets.append((v, o))
gen.close()
rec = torch.empty(S // 8, dtype=torch.int64, device="cuda")
row = torch.zeros(10, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
out = {"lib": os.environ.get("RABIA_GPU_LIB", "default"), "slots": S}
for mode in ("step", "shard", "step", "shard"):
    ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
    ts = []
    for r in range(24):
        v, o = sets[r % 2]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if mode == "step":
            ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1 + r * S, stream=sp)
        else:
            ev.phase_step_shard_async(v.data_ptr(), o.data_ptr(), S, T, 1 + r * S, rec.data_ptr(), S // 8,
                                      row.data_ptr(), stream=sp)
        e1.record(stream)
        if r >= 4:
            ts.append((e0, e1))
    torch.cuda.synchronize()
    la = ev.last_launch()
    ev.close()
    us = [a.elapsed_time(b) * 1000 for a, b in ts]
    out.setdefault(mode, []).append({"median_us": float(np.median(us)), "kernel": la["kernel"], "block": la["block"]})
print(json.dumps(out))
