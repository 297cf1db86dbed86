"""Diagnostic: sharded vs single REF at a given size; report the first differing
words and which side agrees with the oracle on a slice around them."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import numpy as np
import torch
import oracle_lib as O
from test_shard_ref import make_votes, run_sharded, run_single
from rabia_amd.engine import decode_outputs

n, logS, world = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
S = 1 << logS
votes, stride, total = make_votes(n, [S], 1, seed=11)
out_s = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
res_s, st_s, rows, fixed = run_sharded(n, world, [S], votes, out_s, stride)
out_1 = torch.zeros(8 * stride, dtype=torch.int32, device="cuda")
res_1, st_1 = run_single(n, [S], votes, out_1, stride)
a = out_s.view(8, stride).cpu().numpy().view(np.uint32)
b = out_1.view(8, stride).cpu().numpy().view(np.uint32)
print("rows", rows)
print("fixed", fixed)
print("res_s", res_s[0][0])
print("res_1", res_1[0])
diff = np.nonzero((a != b).any(axis=0))[0]
print("differing words:", len(diff), diff[:20], diff[-5:] if len(diff) else None)
for pl in range(8):
    print("plane", pl, int((a[pl] != b[pl]).sum()))
if len(diff):
    w = int(diff[0])
    lo = max(0, w * 32 - 2048)
    da = decode_outputs(a, S)
    db = decode_outputs(b, S)
    k0a = int((da["r1"][:lo] == 2).sum())
    r1, r2, _ = O.trace(1, n, 11, 1 + lo, 4096)
    exp, _ = O.ref_step(n, n // 2 + 1, n // 2, 42, k0a, 1 + lo, r1, r2)
    for k in exp:
        print(k, "shard==oracle", bool((da[k][lo:lo + 4096] == exp[k]).all()),
              "single==oracle", bool((db[k][lo:lo + 4096] == exp[k]).all()))
    print("shard boundaries (words):", [((S // world) * r) // 32 for r in range(world)])
