#!/usr/bin/env python3
"""C5 step shapes in isolation (no fix-up, no collectives beside them): the per-GPU
launch of the 8-GPU C5 pipeline (n = 9, K windows of 2^23 slots per shard launch) and
its single-window counterparts, each variant timed with HIP events over back-to-back
launches on rotating input sets (> MALL), median per launch. Variants:
  shard_windows   rg_phase_step_shard_windows_async, K windows (the bench's launch)
  shard_single    rg_phase_step_shard_async over one window of K x 2^23 slots
  step_single     rg_phase_step_async over the same slots (no draw records)
each under the default dispatch and under rg_debug_set switches (AB: "name:diag").
Prints one JSON object. usage: python tools/c5_probe.py [--n 9] [--window-log2 23] [--k 8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=9)
    ap.add_argument("--window-log2", type=int, default=23)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--diags", default="default:0,lag:0x200000,lag512:0x600000")
    a = ap.parse_args()
    n, T, K = a.n, 1024, a.k
    S = 1 << a.window_log2
    P = 4 * n + 1
    tiles = S // 32 // T
    in_w, out_w = tiles * P * T, tiles * 8 * T
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    sets = []
    gen = PhaseEvaluator(n, tile_words=T)
    for i in range(3):
        v = torch.empty(K * in_w, dtype=torch.int32, device="cuda")
        o = torch.empty(K * out_w, dtype=torch.int32, device="cuda")
        rec = torch.empty(K * S, dtype=torch.int64, device="cuda")
        for k in range(K):  # one K x S-slot region of contiguous tiles: also one window of K x S slots
            gen.trace_generate_async(N.RG_TRACE_AGREE90, 100 + i * K + k, 1 + k * S, S, T,
                                     v.data_ptr() + 4 * k * in_w, sp)
        sets.append((v, o, rec))
    gen.close()
    rows = torch.zeros((K, 10), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    alg = K * S * (4 * n + 8) / 8.0
    out = {"n": n, "window_slots": S, "k": K, "alg_bytes": alg, "variants": {}}
    for item in a.diags.split(","):
        name, diag = item.split(":")
        for mode in ("shard_windows", "shard_single", "step_single"):
            ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
            ev.debug_set(int(diag, 0))
            ts = []
            for r in range(a.reps + 5):
                v, o, rec = sets[r % 3]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if mode == "shard_windows":
                    ev.phase_step_shard_windows_async(K, v.data_ptr(), in_w, o.data_ptr(), out_w, S, T, 1, S,
                                                      rec.data_ptr(), S, rows.data_ptr(), stream=sp)
                elif mode == "shard_single":
                    ev.phase_step_shard_async(v.data_ptr(), o.data_ptr(), K * S, T, 1, rec.data_ptr(), K * S,
                                              rows.data_ptr(), stream=sp)
                else:
                    ev.phase_step_async(v.data_ptr(), o.data_ptr(), K * S, T, slot_base=1 + r * K * S, stream=sp)
                e1.record(stream)
                if r >= 5:
                    ts.append((e0, e1))
            torch.cuda.synchronize()
            us = [x.elapsed_time(y) * 1000.0 for x, y in ts]
            la = ev.last_launch()
            flags = int(rows.cpu().numpy().view(np.uint64)[:, 9].max())
            ev.close()
            med = float(np.median(us))
            out["variants"][f"{name}/{mode}"] = {"median_us": med, "min_us": float(np.min(us)),
                                                 "hbm_frac": alg / (med * 1e-6) / 8e12, "launch": la, "flags": flags}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
