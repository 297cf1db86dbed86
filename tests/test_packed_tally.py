"""The C3 cluster kernel's packed tallies (rg_kernels.h, wmvc_cluster_lc_kernel<N, Q, true>)
restated bit for bit in Python and checked against the popcount rules of the unpacked body
(the rules of oracle/rabia_oracle.c:or_wmvc_cluster) over every case: each receiver's heard
set of q members (itself + q - 1 others), every state / V1 / VQ vector. The field-wise
nonzero test (packed_nz) and the multiply that gathers the field flags (packed_compress)
are the kernel's own arithmetic, 32-bit wrapped; the raw-bits heard table (ClusterRaw) is
checked against the picks of heard_mask_k for every hash value's relevant bits."""
import itertools

import pytest

M32 = 0xFFFFFFFF


def rep(n):
    return sum(1 << (n * i) for i in range(n))


def packed_nz(n, x):
    lo = rep(n) * ((1 << (n - 1)) - 1)
    hi = rep(n) << (n - 1)
    return ((((x & lo) + lo) & M32) | x) & hi


def gather_mul(n):
    return sum(1 << ((n - 1) * (n - 1) - (n - 1) * r) for r in range(n))


def packed_compress(n, f):
    prod = ((f >> (n - 1)) & 0xFFFFFF) * gather_mul(n) & M32  # v_mul_u32_u24: low 32 bits
    return (prod >> ((n - 1) * (n - 1))) & ((1 << n) - 1)


def popcount(x):
    return bin(x).count("1")


def unpacked(n, q, fp1, hm0, hm1, st):
    """The unpacked body's rules (one receiver at a time, popcounts)."""
    v1 = vq = 0
    for r in range(n):
        c1, c0 = popcount(hm0[r] & st), popcount(hm0[r] & ~st & ((1 << n) - 1))
        v1 |= (c1 >= q) << r
        vq |= (c1 < q and c0 < q) << r
    nv1 = need = newly = newv = 0
    for r in range(n):
        c1, cq = popcount(hm1[r] & v1), popcount(hm1[r] & vq)
        c0 = q - c1 - cq
        d0 = c0 >= fp1
        d1 = not d0 and c1 >= fp1
        newly |= (d0 or d1) << r
        newv |= d1 << r
        nv1 |= (d1 or (not d0 and c0 == 0 and c1 > 0)) << r
        need |= (not d0 and not d1 and c0 == 0 and c1 == 0) << r
    return v1, vq, nv1, need, newly, newv


def packed(n, hm0, hm1, st):
    """The packed body (fp1 = q): receiver r's heard set in bits [n r, n r + n)."""
    R, H = rep(n), rep(n) << (n - 1)
    ph0 = sum(hm0[r] << (n * r) for r in range(n))
    ph1 = sum(hm1[r] << (n * r) for r in range(n))
    rs = st * R
    some1, some0 = packed_nz(n, ph0 & rs), packed_nz(n, ph0 & ~rs & M32)
    v1, vq = packed_compress(n, H & ~some0 & M32), packed_compress(n, some1 & some0)
    rv1, rvq = v1 * R, vq * R
    rnz = rv1 | rvq
    s1, snz = packed_nz(n, ph1 & rv1), packed_nz(n, ph1 & rnz)
    sn1, s0 = packed_nz(n, ph1 & ~rv1 & M32), packed_nz(n, ph1 & ~rnz & M32)
    snq = packed_nz(n, ph1 & ~rvq & M32)
    d1f, d0f = H & ~sn1 & M32, H & ~snz & M32
    return (v1, vq, packed_compress(n, d1f | (s1 & ~s0 & M32)), packed_compress(n, H & ~snq & M32),
            packed_compress(n, d0f | d1f), packed_compress(n, d1f))


def heard_sets(n, q, r):
    others = [x for x in range(n) if x != r]
    return [(1 << r) | sum(1 << x for x in c) for c in itertools.combinations(others, q - 1)]


@pytest.mark.parametrize("n", [1, 3, 5])
def test_compress_gathers_every_flag_pattern(n):
    for m in range(1 << n):
        f = sum(1 << (n * r + n - 1) for r in range(n) if m >> r & 1)
        assert packed_compress(n, f) == m


@pytest.mark.parametrize("n", [1, 3, 5])
def test_packed_nz_is_fieldwise_nonzero(n):
    for vals in itertools.product(range(1 << n), repeat=min(n, 3)):
        x = sum(v << (n * i) for i, v in enumerate(vals))
        want = sum(1 << (n * i + n - 1) for i, v in enumerate(vals) if v)
        assert packed_nz(n, x) == want


@pytest.mark.parametrize("n", [1, 3, 5])
def test_packed_rules_equal_popcount_rules(n):
    q = n // 2 + 1
    fp1 = (n - 1) // 2 + 1
    assert fp1 == q
    sets = [heard_sets(n, q, r) for r in range(n)]
    import random
    rng = random.Random(n)
    cases = 0
    for st in range(1 << n):
        # heard-set combinations: every one at n <= 3, a seeded sample at n = 5 (6^10 in all)
        combos = itertools.product(*(sets * 2)) if n <= 3 else (
            tuple(rng.choice(sets[r % n]) for r in range(2 * n)) for _ in range(3000))
        for hs in combos:
            hm0, hm1 = list(hs[:n]), list(hs[n:])
            assert packed(n, hm0, hm1, st) == unpacked(n, q, fp1, hm0, hm1, st), (n, st, hm0, hm1)
            cases += 1
    assert cases > 0


def raw_entry(n, q, e):
    """ClusterRaw's table entry e: receiver e >> nb, the picks from bits (e & mask) << lo."""
    picks, span0 = q - 1, n - 1
    log0 = {4: 2, 2: 1, 1: 0}.get(span0, -1)
    lo = 6 - log0 if picks >= 1 and log0 >= 0 else 0
    nb = 6 * picks - lo if picks >= 1 else 0
    r = e >> nb
    h = (e & ((1 << nb) - 1)) << lo
    avail, mask = ((1 << n) - 1) & ~(1 << r), 1 << r
    for i in range(picks):
        span = n - 1 - i
        k = (((h >> (6 * i)) & 63) * span) >> 6
        a = avail
        for _ in range(k):
            a &= a - 1
        pick = a & -a
        mask |= pick
        avail &= ~pick
    return mask << (n * r), lo, nb


def heard_k(n, q, h, r):
    """heard_mask_k's picks from a hash value (rg_kernels.h)."""
    avail, mask = ((1 << n) - 1) & ~(1 << r), 1 << r
    for i in range(q - 1):
        span = n - 1 - i
        k = (((h >> (6 * i)) & 63) * span) >> 6
        a, sel = avail, avail
        for t in range(1, span):
            a &= a - 1
            sel = a if t == k else sel
        pick = sel & -sel
        mask |= pick
        avail &= ~pick
    return mask


@pytest.mark.parametrize("n", [1, 3, 5])
def test_raw_bits_table_equals_picks(n):
    q = n // 2 + 1
    _, lo, nb = raw_entry(n, q, 0)
    for h in range(1 << 12):  # every value of the bits the picks read (q - 1 <= 2 picks: 12 bits)
        for r in range(n):
            e = (r << nb) + ((h >> lo) & ((1 << nb) - 1))
            assert raw_entry(n, q, e)[0] == heard_k(n, q, h, r) << (n * r)
