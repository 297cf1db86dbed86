import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import numpy as np
import torch
from test_shard_ref import make_votes, run_sharded, run_single

def dec(r):
    info = int(r) >> 32
    return (int(r) & 0xffffffff, info & 3, (info >> 2) & 3, (info >> 4) & 3, (info >> 6) & 1)

for n, logS, world in [(9, 26, 8), (9, 23, 8), (9, 26, 4), (5, 26, 8), (9, 24, 2)]:
    S = 1 << logS
    votes, stride, total = make_votes(n, [S], 1, seed=11)
    out_s = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    keep = []
    res_s, st_s, rows, fixed = run_sharded(n, world, [S], votes, out_s, stride, keep=keep)
    out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
    res_1, st_1 = run_single(n, [S], votes, out_1, stride)
    a = out_s.view(8, stride); b = out_1.view(8, stride)
    bad = []
    for r in range(world):
        lo, hi = (S // world) * r // 32, (S // world) * (r + 1) // 32
        if not torch.equal(a[:, lo:hi], b[:, lo:hi]):
            bad.append(r)
    dv1 = [f["n_v1"] - x["n_v1"] for f, x in zip(fixed, rows)]
    print(n, logS, world, "bad shards", bad, "vq v1 per shard", dv1, flush=True)
    for r in bad[:1] + [0]:
        nd = rows[r]["n_draws"]
        print("  shard", r, "n_draws", nd, [dec(x) for x in keep[r][:6]], "nonzero recs", int((keep[r][:nd] != 0).sum()))
    del votes, out_s, out_1
    torch.cuda.empty_cache()
