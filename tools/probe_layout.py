"""Which plane layout streams best? Times the protocol-free stream probe
(20 in-planes + 8 out-planes per 32-slot word, 16 B/lane) under planar and
slot-tiled layouts, default and non-temporal. Interleaved rounds in one process.
Run on the GPU box: python tools/probe_layout.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rabia_amd import _native as N  # noqa: E402

lib = N.load()
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sp = stream.cuda_stream
S = 1 << 26
nw = S // 32
stride = nw
sets = [(torch.randint(0, 2 ** 31, (21 * stride,), dtype=torch.int32, device="cuda"),
         torch.empty(8 * stride, dtype=torch.int32, device="cuda")) for _ in range(3)]
padded = [(torch.randint(0, 2 ** 31, (21 * (stride + 256),), dtype=torch.int32, device="cuda"),
           torch.empty(8 * (stride + 256), dtype=torch.int32, device="cuda")) for _ in range(3)]
torch.cuda.synchronize()
variants = {"planar": (0, 0, False), "planar_nt": (0, 1, False), "planar_pad": (0, 0, True)}
for T in (256, 1024, 2048, 8192):
    variants[f"tiled{T}"] = (T, 0, False)
    variants[f"tiled{T}_nt"] = (T, 1, False)
times = {k: [] for k in variants}
for r in range(10):
    for name, (T, nt, pad) in variants.items():
        for k in range(3):
            v, o = (padded if pad else sets)[k]
            st = stride + 256 if pad else stride
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            N.check(lib.rg_debug_stream_probe(v.data_ptr(), o.data_ptr(), nw, st, T, nt, sp))
            e1.record(stream)
            e1.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) * 1000)
out = {k: {"median_us": float(np.median(t)), "min_us": float(np.min(t)),
           "TBps": S * 3.5 / (np.median(t) * 1e-6) / 1e12} for k, t in times.items()}
print(json.dumps(out, indent=1))
