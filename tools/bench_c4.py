#!/usr/bin/env python3
"""C4 pipeline timing (BASELINE.json configs[3]): 7 replicas x 2^22 slots with per-replica
proposal digests, one REF phase sweep, then the kvstore apply of the V1-decided slots'
batches (one bincode KVOperation per slot, device-generated).

Stages, all device-resident on one stream, timed with HIP events per stage:
  digest  rg_digest_majority_async (exchange: state = some digest held by >= q replicas)
  phase   rg_phase_step_async (REF, planar layout)
  mark    rg_kv_mark_applied_async (commands of V1 slots)
  apply   rg_kv_apply_async (decode, sort, keyed replay / commit)
Prints one JSON object. Not the driver's bench line (bench.py is): C4 is a parity
config; this records where its time goes. cpu_baseline = oracle/kvstore_ref.c (the
sequential C restatement, 1 thread) on the same commands and mask.
usage: python tools/bench_c4.py [--slots-log2 22] [--reps 5]
"""
import argparse
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
from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots-log2", type=int, default=22)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--key-space-log2", type=int, default=20)
    ap.add_argument("--bucket-bits", type=int, default=0, help="sort bucket width (0: the library's choice)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the C restatement baseline")
    a = ap.parse_args()
    n, S = 7, 1 << a.slots_log2
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    stride = ((S + 127) // 128) * 4
    ev = PhaseEvaluator(n, self_lane=n - 1, mode="ref", seed=42)
    votes = torch.empty((4 * n + 1) * stride, dtype=torch.int32, device="cuda")
    out = torch.empty(8 * stride, dtype=torch.int32, device="cuda")
    digests = torch.empty(n * S, dtype=torch.int64, device="cuda")
    ev.trace_generate_async(N.RG_TRACE_AGREE90, 5, 1, S, stride, votes.data_ptr(), sp)
    ev.digest_trace_async(5, 1, S, S, digests.data_ptr(), sp)
    slot_off = torch.arange(S + 1, dtype=torch.int64, device="cuda")  # one command per slot
    cmd_data = torch.empty(68 * S, dtype=torch.uint8, device="cuda")
    cmd_off = torch.empty(S + 1, dtype=torch.int64, device="cuda")
    mask = torch.empty(S, dtype=torch.uint8, device="cuda")
    res = torch.empty(S, dtype=torch.uint8, device="cuda")
    ks = 1 << a.key_space_log2
    times = {k: [] for k in ("digest", "phase", "mark", "apply")}
    applied, warm = [], []
    cmd_data2 = torch.empty(68 * S, dtype=torch.uint8, device="cuda")
    cmd_off2 = torch.empty(S + 1, dtype=torch.int64, device="cuda")
    res2 = torch.empty(S, dtype=torch.uint8, device="cuda")
    for rep in range(a.reps + 1):
        with DeviceKVStore(KVStoreConfig(max_keys=4 * ks, bucket_bits=a.bucket_bits)) as kv:
            kv.trace_async(rep, S, ks, cmd_data.data_ptr(), cmd_data.numel(), cmd_off.data_ptr(), sp)
            stream.synchronize()
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            evs[0].record(stream)
            ev.digest_majority_async(digests.data_ptr(), S, votes.data_ptr() + 4 * 4 * n * stride, S, sp)
            evs[1].record(stream)
            ev.phase_step_async(votes.data_ptr(), out.data_ptr(), S, stride, slot_base=1, stream=sp)
            evs[2].record(stream)
            kv.mark_applied_async(out.data_ptr(), stride, 0, S, slot_off.data_ptr(), mask.data_ptr(), sp)
            evs[3].record(stream)
            kv.apply_async(cmd_data.data_ptr(), cmd_off.data_ptr(), S, mask.data_ptr(), res.data_ptr(), sp)
            evs[4].record(stream)
            stream.synchronize()
            if rep:
                for k, i in zip(times, range(4)):
                    times[k].append(evs[i].elapsed_time(evs[i + 1]) * 1000.0)
                st = kv.stats()
                applied.append(int((mask.cpu().numpy() != 0).sum()))
                # a second batch on the same (now populated) store: most keys exist, so the
                # commit overwrites values in place instead of claiming slots and copying keys
                kv.trace_async(1000 + rep, S, ks, cmd_data2.data_ptr(), cmd_data2.numel(), cmd_off2.data_ptr(), sp)
                stream.synchronize()
                w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                w0.record(stream)
                kv.apply_async(cmd_data2.data_ptr(), cmd_off2.data_ptr(), S, mask.data_ptr(), res2.data_ptr(), sp)
                w1.record(stream)
                stream.synchronize()
                warm.append(w0.elapsed_time(w1) * 1000.0)
                st_warm = kv.stats()
    med = {k: float(np.median(v)) for k, v in times.items()}
    total_us = sum(med.values())
    n_applied = int(np.median(applied))
    # CPU baseline: the sequential C restatement (oracle/kvstore_ref.c, one thread; the
    # KVStore is one HashMap behind one lock, store.rs) applying the same commands with
    # the same mask, median of 3; its results must equal the device's
    if a.no_cpu:
        print(json.dumps({"bucket_bits": a.bucket_bits, "stage_us_median": med,
                          "apply_warm_us_median": float(np.median(warm)), "store": st}))
        return
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    data = cmd_data.cpu().numpy()
    offs = cmd_off.cpu().numpy().view(np.uint64)
    m_host = mask.cpu().numpy()
    cpu_times = []
    for _ in range(3):
        ref = O.KVStoreC(max_keys=4 * ks)
        t0 = time.perf_counter()
        exp = ref.apply(data[: int(offs[-1])], offs, m_host)
        cpu_times.append(time.perf_counter() - t0)
    cpu_s = float(np.median(cpu_times))
    agree = bool(np.array_equal(exp, res.cpu().numpy()))
    m = int((m_host != 0).sum())
    # all-core baseline: key-hash partitions, one store and one thread each (exact here:
    # max_keys is never reached), on the cores this process may use
    th = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            th = max(1, min(th, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    par_times = []
    for _ in range(3):
        t0 = time.perf_counter()
        exp_p, _tot = O.kv_apply_partitioned(data[: int(offs[-1])], offs, m_host, parts=4 * th, max_keys=4 * ks,
                                             threads=th)
        par_times.append(time.perf_counter() - t0)
    par_s = float(np.median(par_times))
    agree_p = bool(np.array_equal(exp_p, res.cpu().numpy()))
    print(json.dumps({
        "workload": f"C4: n={n}, 2^{a.slots_log2} slots, agree90 votes + per-replica digests, REF sweep, "
                    f"1 KVOperation per slot over 2^{a.key_space_log2} keys (85% Set)",
        "stage_us_median": med,  # apply = the first batch on a fresh store "total_us": total_us,
        "applied_commands": n_applied, "apply_commands_per_s": n_applied / (med["apply"] * 1e-6),
        "slots_per_s_end_to_end": S / (total_us * 1e-6),
        "store": st,
        "apply_warm_us_median": float(np.median(warm)),
        "apply_warm_note": "a second batch (another seed, same mask) on the store the first batch populated: "
                           "keys mostly exist, values overwritten in place",
        "store_after_warm": st_warm,
        "cpu_baseline": {"value": m / par_s, "unit": "applied commands/s", "cores": th, "kind": "port",
                         "sample": f"the last batch's {S} commands ({m} applied) through oracle/kvstore_ref.c:"
                                   f"or_kv_apply_partitioned ({4 * th} key-hash partitions, {th} OpenMP threads = the "
                                   f"granted CPUs), median of 3: {par_s:.3f} s; results equal the device's: {agree_p}",
                         "sequential_1t": {"value": m / cpu_s, "seconds": cpu_s, "results_equal": agree,
                                           "note": "oracle/kvstore_ref.c sequential replay (the reference's apply "
                                                   "is sequential per engine, smr_impl.rs:120-126)"}},
    }, indent=1))


if __name__ == "__main__":
    main()
