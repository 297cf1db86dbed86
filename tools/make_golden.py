"""Generate the committed golden fixtures under tests/golden/ from the pure-Python
restatement (oracle/rabia_ref.py). The C oracle and the HIP path are both
checked against these files; see DESIGN.md §Oracle for what they pin.

  truth_n{n}_q{q}.npz : exhaustive tables over all 4^n received-vote vectors
  trace_{mode}_k{kind}_n{n}.npz : seeded traces (inputs + expected outputs)

Run: python tools/make_golden.py
"""
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rabia_ref as R  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

# WMVC round-2 classes
CLS_DEC0, CLS_DEC1, CLS_ADOPT0, CLS_ADOPT1, CLS_COIN, CLS_PENDING = range(6)


def r2_class(v, q, fp1):
    c0 = sum(1 for c in v if c == R.V0)
    c1 = sum(1 for c in v if c == R.V1)
    present = sum(1 for c in v if c != R.NONE)
    if present < q:
        return CLS_PENDING
    if c0 >= fp1:
        return CLS_DEC0
    if c1 >= fp1:
        return CLS_DEC1
    if c0 > 0:
        return CLS_ADOPT0
    if c1 > 0:
        return CLS_ADOPT1
    return CLS_COIN


def wmvc_r1(v, q):
    c0 = sum(1 for c in v if c == R.V0)
    c1 = sum(1 for c in v if c == R.V1)
    present = sum(1 for c in v if c != R.NONE)
    if present < q:
        return R.NONE
    return R.V0 if c0 >= q else (R.V1 if c1 >= q else R.VQ)


def truth_tables():
    for n, q in ((3, 2), (4, 3), (4, 2), (5, 3), (7, 4), (9, 5)):
        fp1 = (n - 1) // 2 + 1
        N = 4 ** n
        cv = np.empty(N, np.uint8)
        r1 = np.empty(N, np.uint8)
        w1 = np.empty(N, np.uint8)
        w2 = np.empty(N, np.uint8)
        for idx, v in enumerate(itertools.product(range(4), repeat=n)):
            v = v[::-1]  # lane j = base-4 digit j of idx (lane 0 least significant)
            cv[idx] = R.count_votes(v, q)
            r1[idx] = R.ref_round1(v, q)
            w1[idx] = wmvc_r1(v, q)
            w2[idx] = r2_class(v, q, fp1)
        path = os.path.join(GOLD, f"truth_n{n}_q{q}.npz")
        np.savez_compressed(path, n=n, q=q, fp1=fp1, count_votes=cv, ref_round1=r1,
                            wmvc_round1=w1, wmvc_round2_class=w2)
        print("wrote", path)


RES_KEYS = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws",
            "last_committed_max", "first_undecided", "rng_next", "commit_watermark"]


def traces():
    S = 4096
    specs = [("ref", 1, 5), ("ref", 0, 5), ("ref", 2, 5), ("ref", 1, 3), ("ref", 1, 7),
             ("ref", 1, 9), ("ref", 0, 16), ("wmvc", 1, 5), ("wmvc", 0, 5), ("wmvc", 0, 7)]
    for mode, kind, n in specs:
        seed = 42
        slot_base = 1
        q = n // 2 + 1
        r1, r2, st = R.trace(kind, n, seed, slot_base, S)
        if mode == "ref":
            params = dict(n=n, q=q, self_lane=n - 1, seed=seed, rng_base=1000,
                          slot_base=slot_base, max_phase=0, lc_in=0, wm_in=1)
            out, res = R.ref_step(n, q, n - 1, seed, 1000, slot_base, r1, r2,
                                  max_phase=0, lc_in=0, wm_in=1)
        else:
            fp1 = (n - 1) // 2 + 1
            params = dict(n=n, q=q, fp1=fp1, self_lane=0, coin_seed=7, epoch=3, phase=2,
                          slot_base=slot_base, lc_in=0, wm_in=1)
            out, res = R.wmvc_step(n, q, fp1, 0, 7, 3, 2, slot_base, r1, r2, st,
                                   lc_in=0, wm_in=1)
        path = os.path.join(GOLD, f"trace_{mode}_k{kind}_n{n}.npz")
        np.savez_compressed(
            path, r1=np.array(r1, np.uint8), r2=np.array(r2, np.uint8),
            state=np.array(st, np.uint8),
            **{f"out_{k}": np.array(v, np.uint8) for k, v in out.items()},
            result=np.array([res[k] for k in RES_KEYS], np.uint64),
            params=json.dumps(params), kind=kind, mode=mode, trace_seed=seed)
        print("wrote", path, {k: res[k] for k in ("n_decided", "n_draws")})


def coins_and_draws():
    key = R.seed_from_u64(42)
    draws = [R.ref_draw(key, k) for k in range(64)]
    rng = R.StdRng(42)
    seq = [rng.next_u64() for _ in range(64)]
    assert seq == draws
    ckey = R.seed_from_u64(7)
    coins = [[R.coin(ckey, 3, s, p) for s in range(1000, 2024)] for p in (1, 2, 3, 32)]
    np.savez_compressed(os.path.join(GOLD, "rng_fixtures.npz"),
                        stdrng42_next_u64=np.array(draws, np.uint64),
                        gen_bool08=np.array([d < R.P_INT[0.8] for d in draws], np.uint8),
                        coins_seed7_epoch3=np.array(coins, np.uint8),
                        coin_phases=np.array([1, 2, 3, 32]), coin_slot_base=1000)
    print("wrote rng_fixtures.npz")


def digests():
    S = 2048
    for n in (5, 7):
        q = n // 2 + 1
        import random
        rnd = random.Random(5)
        rows = []
        for s in range(S):
            pool = [rnd.getrandbits(64) | 1 for _ in range(3)]
            rows.append([0 if rnd.random() < 0.1 else rnd.choice(pool) for _ in range(n)])
        st = R.digest_majority(rows, q)
        np.savez_compressed(os.path.join(GOLD, f"digest_n{n}.npz"),
                            digests=np.array(rows, np.uint64).T.copy(), q=q,
                            state=np.array(st, np.uint8))
        print("wrote digest", n, sum(st))


def clusters():
    """WMVC cluster view to termination (config 3 shape), Python restatement."""
    for n, S in ((5, 2048), (7, 1024), (3, 1024)):
        q, fp1 = n // 2 + 1, (n - 1) // 2 + 1
        st = R.cluster_trace(n, 42, 1, S)
        outs = R.wmvc_cluster(n, q, fp1, 7, 3, 99, 32, 1, st)
        info = np.array([o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24) for o in outs], np.uint32)
        np.savez_compressed(os.path.join(GOLD, f"cluster_n{n}.npz"), states=np.array(st, np.uint8),
                            info=info, params=json.dumps(dict(n=n, q=q, fp1=fp1, coin_seed=7, epoch=3,
                                                              delivery_seed=99, max_phases=32, slot_base=1)))
        print("wrote cluster", n, "mean phases", float(np.mean([o[1] for o in outs])))


if __name__ == "__main__":
    os.makedirs(GOLD, exist_ok=True)
    if sys.argv[1:] == ["clusters"]:
        clusters()
        sys.exit(0)
    truth_tables()
    traces()
    coins_and_draws()
    digests()
    clusters()
