"""Per-phase timing of the persistent lag REF kernel (rg_debug_set bit 4 stamps):
per workgroup, the time in each phase of its iterations and its start/end times.
Run on the GPU box: python tools/lag_stamps.py [extra_diag] > gpurun_out/lag_stamps.json
STAMP_SHARD=1: the sharded step (rg_phase_step_shard_async, draw records) instead."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

PHASES = ["start_to_loop", "tally", "scan_barrier", "decisions", "draws", "stores", "loop_end_to_record"]


def main():
    extra = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0
    S = int(os.environ.get("STAMP_SLOTS", 1 << 30))
    n, T = int(os.environ.get("STAMP_N", 5)), 1024
    nw = S // 32
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
    v = torch.empty(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    o = torch.empty(((nw + T - 1) // T) * 8 * T, dtype=torch.int32, device="cuda")
    ev.trace_generate_async(N.RG_TRACE_AGREE90, 1, 1, S, T, v.data_ptr(), sp)
    shard = os.environ.get("STAMP_SHARD", "0") == "1"
    cap = S // 8
    rec = torch.empty(cap if shard else 1, dtype=torch.int64, device="cuda")
    row = torch.zeros(10, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    out = {"shard": shard}
    for diag, name in ((extra, "plain"), (extra | 4, "stamped")):
        N.check(ev.lib.rg_debug_set(ev.ctx, diag), ev.ctx)
        ts = []
        for k in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if shard:
                ev.phase_step_shard_async(v.data_ptr(), o.data_ptr(), S, T, 1 + k * S, rec.data_ptr(), cap,
                                          row.data_ptr(), stream=sp)
            else:
                ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1 + k * S, stream=sp)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0)
        out[name + "_us"] = float(np.median(ts[2:]))
    grid = 512 if extra & 0x400000 else 256  # 2 x 512 (diag bit 22) or 1 x 1024 per CU
    buf = np.zeros(grid * 16, dtype=np.uint64)
    N.check(ev.lib.rg_debug_stamps(ev.ctx, buf.ctypes.data, buf.size), ev.ctx)
    d = buf.reshape(grid, 16).astype(np.float64)
    it = d[:, 7]
    ph = {PHASES[k]: float(np.sum(d[:, k]) / max(np.sum(it), 1) * 0.01) for k in range(1, 6)}  # us per iteration
    ph["draws.lookback_part"] = float(np.sum(d[:, 8]) / max(np.sum(it), 1) * 0.01)
    for k, nm in ((12, "draws.chacha"), (13, "draws.chacha_barrier"), (14, "draws.select")):
        ph[nm] = float(np.sum(d[:, k]) / max(np.sum(it), 1) * 0.01)
    out["continued_lookbacks_frac"] = float(np.sum(d[:, 9]) / max(np.sum(it), 1))
    out["per_iteration_us"] = ph
    out["per_iteration_total_us"] = sum(ph.values())  # "draws" is what the "draws.*" parts leave
    out["iterations_per_wg"] = {"min": int(it.min()), "max": int(it.max()), "mean": float(it.mean())}
    t0 = d[:, 10].min()
    out["start_spread_us"] = float((d[:, 10].max() - t0) * 0.01)
    out["start_to_loop_us_mean"] = float(d[:, 0].mean() * 0.01)
    out["loop_end_to_record_us_mean"] = float(d[:, 6].mean() * 0.01)
    ends = (d[:, 11] - t0) * 0.01
    out["end_us"] = {"min": float(ends.min()), "median": float(np.median(ends)), "max": float(ends.max())}
    print(json.dumps(out, indent=1))
    ev.close()


if __name__ == "__main__":
    main()
