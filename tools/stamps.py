"""Where does the REF step's look-back wait come from? Per-tile s_memrealtime
stamps (diag bit 4) of one 2^28-slot step (bench layout), analysed per tile and
per XCD. Run on the GPU box: python tools/stamps.py > gpurun_out/stamps.json

stamp slots per tile: 0 start, 1 after R1 tally + block scan (aggregate known),
2 after the look-back, 3 after the stores, 4 after the statistics, 6 XCC id,
7 HW_ID (CU / SIMD / SE)."""
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
n, T = int(os.environ.get("STAMP_N", 5)), 1024
S = int(os.environ.get("STAMP_SLOTS", 1 << 28))
nw = S // 32
ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
sets = []
for i in range(3):
    v = torch.empty(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    o = torch.empty(((nw + T - 1) // T) * 8 * T, dtype=torch.int32, device="cuda")
    ev.trace_generate_async(N.RG_TRACE_AGREE90, i, 1, S, T, v.data_ptr(), sp)
    sets.append((v, o))
torch.cuda.synchronize()
out = {}
for rep in range(4):
    lib.rg_debug_set(ev.ctx, 4 if rep == 3 else 0)
    v, o = sets[rep % 3]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1, stream=sp)
    e1.record(stream)
    torch.cuda.synchronize()
    out[f"launch_us_{rep}"] = e0.elapsed_time(e1) * 1000.0
buf = np.zeros(8 * (S // 65536 + 64), np.uint64)
N.check(lib.rg_debug_stamps(ev.ctx, buf.ctypes.data, buf.size), ev.ctx)
st = buf.reshape(-1, 8)
st = st[st[:, 0] != 0]
xcc = st[:, 6].astype(np.int64) & 0xF
hwid = st[:, 7].astype(np.int64)
t = st[:, :6].astype(np.float64) * 0.01  # 100 MHz ticks -> us
t0 = t[:, 0].min()
t = t - t0
tiles = t.shape[0]
wait = t[:, 2] - t[:, 1]
tally = t[:, 1] - t[:, 0]
tail = t[:, 3] - t[:, 2]
# the latest aggregate among the 64 predecessors vs this tile's own aggregate time
pred_late = np.zeros(tiles)
for i in range(1, tiles):
    lo = max(0, i - 64)
    pred_late[i] = max(0.0, t[lo:i, 1].max() - t[i, 1])
rounds = np.arange(tiles) // 512
per_xcd = {}
for x in range(8):
    m = xcc == x
    if not m.any():
        continue
    per_xcd[str(x)] = {"tiles": int(m.sum()), "start_med_us": float(np.median(t[m, 0])),
                       "wait_med_us": float(np.median(wait[m])), "tally_med_us": float(np.median(tally[m])),
                       "end_max_us": float(t[m, 4].max())}
# drift: per round, the spread over XCDs of the median start time
drift = []
for r in range(int(rounds.max()) + 1):
    m = rounds == r
    meds = [float(np.median(t[m & (xcc == x), 0])) for x in range(8) if (m & (xcc == x)).any()]
    if meds:
        drift.append(max(meds) - min(meds))
pct = lambda a: {p: float(np.percentile(a, p)) for p in (10, 50, 90, 99)}  # noqa: E731
# back-to-back launches of a trivial kernel: the per-launch cost outside any tile
tiny = torch.zeros(1, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    tiny.add_(1)
e0.record(stream)
for _ in range(50):
    tiny.add_(1)
e1.record(stream)
torch.cuda.synchronize()
out["trivial_launch_us"] = e0.elapsed_time(e1) * 1000.0 / 50
out.update({
    "slots": S, "n": n, "tiles": tiles,
    "kernel_span_us": float(t[:, 4].max()),
    "last_tile_fold_us": float(t[:, 5].max() - t[:, 4].max()),
    "tile_start_us": pct(t[:, 0]),
    "tally_us": pct(tally), "wait_us": pct(wait), "after_wait_us": pct(tail),
    "pred_aggregate_later_than_own_us": pct(pred_late),
    "wait_minus_pred_late_us": pct(wait - pred_late),
    "corr_wait_pred_late": float(np.corrcoef(wait[1:], pred_late[1:])[0, 1]),
    "xcc_of_tile_mod8_consistent": bool(all(len(set(xcc[i::8].tolist())) == 1 for i in range(8))),
    "per_xcd": per_xcd,
    "round_start_spread_over_xcds_us": pct(np.array(drift)) if drift else None,
    "distinct_cus": int(len(set(hwid.tolist()))),
})
lib.rg_debug_set(ev.ctx, 0)
print(json.dumps(out, indent=1))
