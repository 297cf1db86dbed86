#!/usr/bin/env python3
"""Where the sharded pipeline's gaps between consecutive step kernels come from: the
plain REF step at the bench shape (n = 5, 2^30 slots, slot-tiled 1024) back to back,
ms per step over K steps (events around the whole chain), in modes that add one piece
of the sharded pipeline's stream traffic at a time:
  plain   nothing else on the device
  xrec    + an event recorded after every step and waited on by a second stream that
            copies 80 bytes (the exchange's first dependency)
  xboth   + the compute stream waiting, before every step, on the second stream's event
            of the step before (the output-buffer reuse dependency)
  shard   the sharded step kernel alone (draw records), no exchange
  evt     plain + a timing event pair around every step (torch events)
  xrec_host  xrec + the host waiting, before every step, for the second stream's event of
            the step before last (the buffer-reuse dependency kept off the device queue:
            bench.py's sharded pipeline)
Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rabia_amd import _native as N  # noqa: E402
from rabia_amd.engine import PhaseEvaluator  # noqa: E402

n, T = 5, 1024
S = int(os.environ.get("PROBE_SLOTS", 1 << 30))
K = int(os.environ.get("PROBE_STEPS", 20))
P, nw = 4 * n + 1, S // 32
tiles = nw // T
comp = torch.cuda.Stream()
fix = torch.cuda.Stream()
torch.cuda.set_stream(comp)
sp = comp.cuda_stream
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
src = torch.zeros(10, dtype=torch.int64, device="cuda")
dst = torch.zeros(10, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
out = {"lib": os.environ.get("RABIA_GPU_LIB", "default"), "slots": S, "steps": K}
MODES = ("plain", "xrec", "xboth", "xrec_host", "evt", "shard")


class TorchEvent:
    def __init__(self, timing=False):
        self.e = torch.cuda.Event(enable_timing=timing)

    def record(self, s):
        self.e.record(s)

    def wait(self, s):
        s.wait_event(self.e)


for mode in MODES * 2:
    ev = PhaseEvaluator(n, self_lane=n - 1, seed=42, tile_words=T)
    mk, base_mode = TorchEvent, mode
    e_main = [mk() for _ in range(K + 4)]
    e_fix = [mk() for _ in range(K + 4)]
    e_t = [(mk(True), mk(True)) for _ in range(K + 4)]
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(K + 4):
        if r == 4:
            torch.cuda.synchronize()
            t0.record(comp)
        v, o = sets[r % 2]
        if base_mode == "xboth" and r >= 2 and r != 4:
            e_fix[r - 2].wait(comp)
        if base_mode == "xrec_host" and r >= 2:
            e_fix[r - 2].e.synchronize()
        if base_mode == "evt":
            e_t[r][0].record(comp)
        if mode == "shard":
            ev.phase_step_shard_async(v.data_ptr(), o.data_ptr(), S, T, 1 + r * S, rec.data_ptr(), S // 8,
                                      row.data_ptr(), stream=sp)
        else:
            ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1 + r * S, stream=sp)
        if base_mode == "evt":
            e_t[r][1].record(comp)
        if base_mode in ("xrec", "xboth", "xrec_host"):
            e_main[r].record(comp)
            with torch.cuda.stream(fix):
                e_main[r].wait(fix)
                dst.copy_(src)
                e_fix[r].record(fix)
    t1.record(comp)
    torch.cuda.synchronize()
    ev.close()
    out.setdefault(mode, []).append(round(t0.elapsed_time(t1) / K, 5))
print(json.dumps(out))
