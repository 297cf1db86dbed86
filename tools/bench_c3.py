#!/usr/bin/env python3
"""C3 timing (BASELINE.json configs[2]): 5 replicas x 2^24 slots, adversarial initial
states ((n-1)/2 replicas at V1 per slot) forcing multi-round common-coin Weak-MVC, run
to termination (max 32 phases) for every replica of every slot on one GPU
(rg_wmvc_cluster_bitmaps_async: each phase = round 1 + round 2 of all n replicas under the
seeded quorum-delivery scheduler + the common coin). At 8 GPUs each rank takes a
2^21-slot shard (coin keyed by the global slot id: shard-invariant); this tool runs
the per-GPU shard sizes 2^21 and 2^24 on one GPU.
Prints one JSON object (not the driver's bench line; bench.py is).
usage: python tools/bench_c3.py [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rabia_amd.engine import PhaseEvaluator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = 5
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    out = {"workload": "C3: n=5, adversarial split initial states, WMVC cluster view to termination "
                       "(<= 32 phases), coin seed 7, epoch 3, delivery seed 99", "sizes": {}}
    for log2 in (21, 24):
        S = 1 << log2
        stride = ((S + 127) // 128) * 4
        states = torch.zeros(n * stride, dtype=torch.int32, device="cuda")
        info = torch.zeros(S, dtype=torch.int32, device="cuda")
        stats = torch.zeros(8, dtype=torch.int64, device="cuda")
        bm = torch.zeros((2, (S + 31) // 32), dtype=torch.int32, device="cuda")
        with PhaseEvaluator(n, mode="wmvc", coin_seed=7, epoch=3) as ev:
            ev.cluster_trace_async(42, 1, S, stride, states.data_ptr(), sp)
            times = []
            for r in range(a.reps + 1):
                stats.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                ev.wmvc_cluster_bitmaps_async(states.data_ptr(), stride, S, 1, 99, 32, info.data_ptr(),
                                              bm[0].data_ptr(), bm[1].data_ptr(), stats.data_ptr(), sp)
                e1.record(stream)
                e1.synchronize()
                if r:
                    times.append(e0.elapsed_time(e1) * 1000.0)
        sv = stats.cpu().numpy().view(np.uint64)
        med = float(np.median(times))
        out["sizes"][f"2^{log2}"] = {
            "kernel_us_median": med, "slots_decided": int(sv[0]), "decided_v1": int(sv[1]),
            "mean_phases": float(sv[2]) / S, "max_phases": int(sv[3]), "mean_coin_phases": float(sv[4]) / S,
            "slots_decided_per_s": int(sv[0]) / (med * 1e-6),
            "replica_phase_evaluations_per_s": float(sv[2]) * n / (med * 1e-6),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
