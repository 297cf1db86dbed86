"""The clamped live-count scan kv_decide_kernel runs for StoreFull batches with live-key
DELETEs (rg_kv.hip, DESIGN.md §4b "Round 6"), restated with the kernel's own arithmetic:
bitmaps of create / delete events over command indices, 32 per word; each of T threads
folds a contiguous range of words into a map x -> min(C, x + D) (whole words by popcount
when they hold only creates or only deletes), an in-order scan composes the ranges, and
each thread replays its range from its starting live count to mark the refused creates.
Checked against the sequential walk (a create is refused iff the store is full) over
random event streams, including starting full, deletes below the cap and empty words."""
import random

import pytest

INF = 1 << 62


def fold_word(C, D, cw, dw, M):
    if not dw:
        k = bin(cw).count("1")
        return min(C + k, M), D + k
    if not cw:
        k = bin(dw).count("1")
        return C - k, D - k
    x = cw | dw
    while x:
        bit = x & -x
        if cw & bit:
            C, D = min(C + 1, M), D + 1
        else:
            C, D = C - 1, D - 1
        x &= x - 1
    return C, D


def replay_word(L, cw, dw, M):
    """(refused bits, L after) as the kernel's replay pass computes them."""
    if not dw and L + bin(cw).count("1") <= M:
        return 0, L + bin(cw).count("1")
    if not dw and L >= M:
        return cw, L
    if not cw:
        return 0, L - bin(dw).count("1")
    rw, x = 0, cw | dw
    while x:
        bit = x & -x
        if cw & bit:
            if L >= M:
                rw |= bit
            else:
                L += 1
        else:
            L -= 1
        x &= x - 1
    return rw, L


def scan_refused(creates, deletes, L0, M, T):
    W = len(creates)
    per = (W + T - 1) // T
    rng_ = [(t * per, min(t * per + per, W)) for t in range(T)]
    maps = []
    for w0, w1 in rng_:
        C, D = INF, 0
        for w in range(w0, w1):
            C, D = fold_word(C, D, creates[w], deletes[w], M)
        maps.append((C, D))
    incl = list(maps)  # Hillis-Steele, composing earlier ranges first
    o = 1
    while o < T:
        prev = list(incl)
        for t in range(o, T):
            pc, pd = prev[t - o]
            cc, dd = prev[t]
            incl[t] = (min(cc, pc + dd), pd + dd)
        o <<= 1
    refused = [0] * W
    for t, (w0, w1) in enumerate(rng_):
        L = L0 if t == 0 else min(incl[t - 1][0], L0 + incl[t - 1][1])
        for w in range(w0, w1):
            refused[w], L = replay_word(L, creates[w], deletes[w], M)
    return refused


def walk_refused(creates, deletes, L0, M):
    refused = [0] * len(creates)
    L = L0
    for w in range(len(creates)):
        for b in range(32):
            if creates[w] >> b & 1:
                if L >= M:
                    refused[w] |= 1 << b
                else:
                    L += 1
            elif deletes[w] >> b & 1:
                L -= 1
    return refused


@pytest.mark.parametrize("seed", range(12))
def test_clamped_scan_equals_sequential_walk(seed):
    rng = random.Random(seed)
    W = rng.choice([1, 7, 64, 300])
    T = rng.choice([1, 4, 256])
    M = rng.randrange(1, 200)
    L0 = rng.randrange(0, M + 1)  # decide takes the scan only when live <= max_keys
    p_c, p_d = rng.random() * 0.6, rng.random() * 0.3
    creates, deletes = [], []
    L = L0  # the true walk while generating: a live-key DELETE needs a live key
    for w in range(W):
        cw = dw = 0
        empty = rng.random() < 0.15
        for b in range(32):
            r = rng.random()
            if empty:
                continue
            if r < p_c:
                cw |= 1 << b
                L = L + 1 if L < M else L
            elif r < p_c + p_d and L > 0:
                dw |= 1 << b
                L -= 1
        creates.append(cw)
        deletes.append(dw)
    assert scan_refused(creates, deletes, L0, M, T) == walk_refused(creates, deletes, L0, M)
