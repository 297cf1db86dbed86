"""Interleaved A/B of experiment builds of librabia_gpu.so (tools/build_variants.sh)
and of rg_debug_set diagnostic switches (AB_DIAGS="name:0x600,...") on the bench's REF step (n=5, 2^28 slots, slot-tiled 1024). Each variant runs in
its own process (RABIA_GPU_LIB), rounds interleave the variants, and every
variant's output buffer and step result must equal the default build's
(checksums). Run on the GPU box: python tools/ab_variants.py > gpurun_out/ab.json"""
import glob
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, os, json, hashlib
sys.path.insert(0, os.environ["ROOT"])
import numpy as np, torch
from rabia_amd import _native as N
from rabia_amd.engine import PhaseEvaluator
n, T, S = 5, 1024, int(os.environ.get("AB_SLOTS", 1 << 28))
nw = S // 32
stream = torch.cuda.Stream(); torch.cuda.set_stream(stream); sp = stream.cuda_stream
ev = PhaseEvaluator(n, self_lane=4, seed=42, tile_words=T)
N.check(ev.lib.rg_debug_set(ev.ctx, int(os.environ.get("AB_DIAG", "0"), 0)), ev.ctx)
sets = []
for i in range(3):
    v = torch.empty(((nw + T - 1) // T) * (4 * n + 1) * T, dtype=torch.int32, device="cuda")
    o = torch.empty(((nw + T - 1) // T) * 8 * T, dtype=torch.int32, device="cuda")
    ev.trace_generate_async(N.RG_TRACE_AGREE90, i, 1, S, T, v.data_ptr(), sp)
    sets.append((v, o))
res = torch.zeros((64, 10), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
ts = []
for k in range(60):
    v, o = sets[k % 3]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    ev.phase_step_async(v.data_ptr(), o.data_ptr(), S, T, slot_base=1 + k * S, result_ptr=res[k].data_ptr(), stream=sp)
    e1.record(stream)
    e1.synchronize()
    if k >= 20:  # clocks settle over ~20 launches (tools/warm_probe.py)
        ts.append(e0.elapsed_time(e1) * 1000.0)
r = res[:60].cpu().numpy().view(np.uint64)
h = hashlib.sha1(sets[59 % 3][1].cpu().numpy().tobytes()).hexdigest()
print(json.dumps({"median_us": float(np.median(ts)), "min_us": float(np.min(ts)), "flags": int(r[:, 9].max()),
                  "decided": int(r[:, 1].sum()), "rng_next": int(r[59, 7]), "out_sha1": h}))
'''


def main():
    lib0 = os.path.join(ROOT, "rabia_amd", "lib", "librabia_gpu.so")
    libs = {"default": (lib0, "0")}
    for p in sorted(glob.glob(os.path.join(ROOT, "rabia_amd", "lib", "variants", "*.so"))):
        libs[os.path.basename(p)[len("librabia_gpu_"):-3]] = (p, "0")
    # AB_DIAGS="name:diag,name:diag": the default library under rg_debug_set(diag)
    for item in filter(None, os.environ.get("AB_DIAGS", "").split(",")):
        name, diag = item.split(":")
        libs[name] = (lib0, diag)
    rounds = int(os.environ.get("AB_ROUNDS", 3))
    got = {k: [] for k in libs}
    for r in range(rounds):
        for name, (path, diag) in libs.items():
            env = dict(os.environ, ROOT=ROOT, RABIA_GPU_LIB=path, AB_DIAG=diag)
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                print(json.dumps({"variant": name, "error": out.stderr[-2000:]}), flush=True)
                return 1
            got[name].append(json.loads(out.stdout.strip().splitlines()[-1]))
            print(json.dumps({"round": r, "variant": name, **got[name][-1]}), file=sys.stderr, flush=True)
    ref = got["default"][0]
    summary = {}
    for name, runs in got.items():
        summary[name] = {"median_us": float(np.median([x["median_us"] for x in runs])),
                         "per_round": [x["median_us"] for x in runs],
                         "same_as_default": all(x["out_sha1"] == ref["out_sha1"] and x["decided"] == ref["decided"]
                                                and x["rng_next"] == ref["rng_next"] and x["flags"] == 0
                                                for x in runs)}
    print(json.dumps(summary, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
