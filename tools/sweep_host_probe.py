"""Single-window (2^20 slots, n=5) sweep: host enqueue time per rg_phase_step_async call
against the GPU time per sweep over back-to-back launches (is `sweep_1m_us` host-bound?).
Run on the GPU box: python tools/sweep_host_probe.py > gpurun_out/sweep_host.json"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

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
lib = N.load()
out = {"slots": S}
for reps in (20, 200):
    host, gpu = [], []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        t0 = time.perf_counter()
        for k in range(reps):
            v, o = sets[k % len(sets)]
            ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1, stream=sp)
        t1 = time.perf_counter()
        e1.record(stream)
        e1.synchronize()
        if r:
            host.append((t1 - t0) * 1e6 / reps)
            gpu.append(e0.elapsed_time(e1) * 1000.0 / reps)
    out[f"reps{reps}"] = {"host_enqueue_us_per_call": round(float(np.median(host)), 2),
                          "gpu_us_per_sweep": round(float(np.median(gpu)), 2)}
# the raw ctypes entry point (no Python wrapper): the C++ host path alone
fn = lib.rg_phase_step_async
v, o = sets[0]
host = []
for r in range(6):
    t0 = time.perf_counter()
    for k in range(200):
        fn(ev.ctx, v.data_ptr(), o.data_ptr(), S, T, 1, 1, 0, None, sp)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    if r:
        host.append((t1 - t0) * 1e6 / 200)
out["raw_ctypes_host_us_per_call"] = round(float(np.median(host)), 2)
print(json.dumps(out, indent=1), flush=True)
