#!/usr/bin/env python3
"""How the REF step's time evolves over back-to-back launches (n = 5, 2^30 slots, the
bench shape, 3 rotating input sets as in bench.py): 300 launches, then 1 s idle, then 60
more. Prints one JSON object: the median us of each group of 10 launches, in order, and
the first 30 launches one by one. PROBE_ZERO=1: the output buffers are zeroed first (every
page touched before the first step)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402


def run(ev, sets, stream, count, base, raw=None):
    evs = []
    for r in range(count):
        v, o = sets[r % len(sets)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=base + r * S, stream=stream.cuda_stream)
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    us = [a.elapsed_time(b) * 1000 for a, b in evs]
    if raw is not None:
        raw.extend(round(x, 1) for x in us[:30])
    return [round(float(np.median(us[i:i + 10])), 1) for i in range(0, len(us), 10)]


n, T = 5, 1024
S = int(os.environ.get("PROBE_SLOTS", 1 << 30))
P, nw = 4 * n + 1, S // 32
tiles = nw // T
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
gen = PhaseEvaluator(n, tile_words=T)
sets = []
for i in range(3):
    v = torch.empty(tiles * P * T, dtype=torch.int32, device="cuda")
    o = (torch.zeros if os.environ.get("PROBE_ZERO") else torch.empty)(tiles * 8 * T, dtype=torch.int32, device="cuda")
    gen.trace_generate_async(N.RG_TRACE_AGREE90, 90 + i, 1, S, T, v.data_ptr(), stream.cuda_stream)
    sets.append((v, o))
gen.close()
torch.cuda.synchronize()
ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
first = []
out = {"slots": S, "zeroed_outputs": bool(os.environ.get("PROBE_ZERO")), "first_300": run(ev, sets, stream, 300, 1, first)}
out["first_30_each"] = first
time.sleep(1.0)
out["after_1s_idle_60"] = run(ev, sets, stream, 60, 1 + 300 * S)
ev.close()
print(json.dumps(out))
