#!/usr/bin/env python3
"""The sharded-REF fix-up in isolation (rg_shard_fixup_async after a one-shard step,
synchronised around it): n = 5, 2^30 slots (the C2 per-rank shard), slot-tiled 1024.
delta = 0: the provisional draw positions are the global ones (nothing to patch);
delta = 1000: the engine position is moved before the fix-up, so every VQ slot is
re-drawn at a different position (as on a rank > 0): the patch traffic of N > 1.
Prints one JSON object (median us per fix-up; step and commit for scale)."""
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
    n, T = 5, 1024
    S = int(os.environ.get("FIX_SLOTS", 1 << 30))
    P, nw = 4 * n + 1, S // 32
    tiles = nw // T
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    votes = torch.empty(tiles * P * T, dtype=torch.int32, device="cuda")
    out = torch.empty(tiles * 8 * T, dtype=torch.int32, device="cuda")
    cap = S // 8
    rec = torch.empty(cap, dtype=torch.int64, device="cuda")
    row, fixed, res = (torch.zeros(10, dtype=torch.int64, device="cuda") for _ in range(3))
    res_out = {"slots": S}
    for delta in (0, 1000):
        ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
        ev.trace_generate_async(N.RG_TRACE_AGREE90, 5, 1, S, T, votes.data_ptr(), sp)
        times = {"step": [], "fixup": [], "commit": []}
        for k in range(6):
            ev.set_state(rng_next=0, last_committed=0, commit_watermark=1)  # shard_draws stays: provisional 0..
            ev.sync()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            e[0].record(stream)
            ev.phase_step_shard_async(votes.data_ptr(), out.data_ptr(), S, T, 1, rec.data_ptr(), cap, row.data_ptr(),
                                      stream=sp)
            e[1].record(stream)
            if delta:
                ev.sync()
                st = ev.get_state()
                ev.set_state(rng_next=st["rng_next"] + delta, last_committed=0, commit_watermark=1)
            e[2].record(stream)
            ev.shard_fixup_async(out.data_ptr(), S, T, 1, rec.data_ptr(), cap, row.data_ptr(), 0, 1,
                                 fixed.data_ptr(), stream=sp)
            e[3].record(stream)
            ev.shard_commit_async(fixed.data_ptr(), 1, 1, S, res.data_ptr(), stream=sp)
            e[4].record(stream)
            torch.cuda.synchronize()
            if k:
                times["step"].append(e[0].elapsed_time(e[1]) * 1000)
                times["fixup"].append(e[2].elapsed_time(e[3]) * 1000)
                times["commit"].append(e[3].elapsed_time(e[4]) * 1000)
        r = fixed.cpu().numpy().view(np.uint64)
        res_out[f"delta_{delta}"] = {k: float(np.median(v)) for k, v in times.items()}
        res_out[f"delta_{delta}"]["n_draws"] = int(r[4])
        res_out[f"delta_{delta}"]["flags"] = int(r[9])
        ev.close()
    print(json.dumps(res_out))


if __name__ == "__main__":
    main()
