"""Pure-Python restatement of the rabia-rs phase-evaluation path.

TEST INFRASTRUCTURE ONLY: imported by tests/ and tools/make_golden.py, never by
the product (rabia_amd/). It is written independently of oracle/rabia_oracle.c
so the two restatements cross-check each other; the committed golden fixtures
under tests/golden/ are produced from THIS module.

Parity status: unpinned against the reference itself (Rust, unbuildable here;
no golden vectors for this path in the reference's tests — SURVEY.md §4/§8c).
The ChaCha core is pinned at 20 rounds by RFC 7539 A.1 / openssl keystreams.

Vote codes: StateValue variant order (rabia-core/src/types.rs:286-294):
V0=0, V1=1, VQuestion=2; 3 = absent voter / None.
"""
from __future__ import annotations

V0, V1, VQ, NONE = 0, 1, 2, 3
MASK64 = (1 << 64) - 1
MASK32 = (1 << 32) - 1

# rand 0.8.5 Bernoulli::new: p_int = (p * 2^64) as u64 (engine.rs:461,470,587,595,604)
P_INT = {p: int(p * 2.0 ** 64) for p in (0.5, 0.7, 0.8, 0.9)}


def count_votes(codes, q):
    """PhaseData::count_votes — rabia-core/src/messages.rs:185-211."""
    c0 = sum(1 for c in codes if c == V0)
    c1 = sum(1 for c in codes if c == V1)
    cq = sum(1 for c in codes if c == VQ)
    if c0 >= q:
        return V0
    if c1 >= q:
        return V1
    if cq >= q:
        return VQ
    return NONE


def ref_round1(codes, q):
    """handle_vote_round1 rule — rabia-engine/src/engine.rs:495-505."""
    r = count_votes(codes, q)
    if r != NONE:
        return r
    present = sum(1 for c in codes if c != NONE)
    return VQ if present >= q else NONE


def seed_from_u64(state):
    """rand_core 0.6.4 SeedableRng::seed_from_u64 (PCG32 key fill)."""
    key = []
    for _ in range(8):
        state = (state * 6364136223846793005 + 11634580027462260723) & MASK64
        xorshifted = (((state >> 18) ^ state) >> 27) & MASK32
        rot = state >> 59
        key.append(((xorshifted >> rot) | (xorshifted << ((32 - rot) % 32))) & MASK32)
    return key


def _rotl(v, c):
    return ((v << c) | (v >> (32 - c))) & MASK32


def chacha_block(key, counter, stream, rounds):
    """ChaCha block: 64-bit counter in words 12-13, 64-bit stream in 14-15."""
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, *key,
         counter & MASK32, (counter >> 32) & MASK32, stream & MASK32, (stream >> 32) & MASK32]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + s[i]) & MASK32 for i in range(16)]


class StdRng:
    """rand 0.8.5 StdRng = rand_chacha 0.3.1 ChaCha12Rng behind rand_core's
    BlockRng; only next_u64 is modelled (all the engine draws)."""

    def __init__(self, seed):
        self.key = seed_from_u64(seed)
        self.words = []
        self.block = 0

    def next_u64(self):
        if len(self.words) < 2:
            self.words += chacha_block(self.key, self.block, 0, 12)
            self.block += 1
        lo, hi = self.words[0], self.words[1]
        del self.words[:2]
        return lo | (hi << 32)

    def gen_bool(self, p):
        return self.next_u64() < P_INT[p]


def ref_draw(key, k):
    """Random access to draw k of the StdRng stream."""
    b = chacha_block(key, k >> 3, 0, 12)
    w = (k & 7) * 2
    return b[w] | (b[w + 1] << 32)


def round2_vote_for_question(c0, c1, u):
    """determine_round2_vote_for_question — engine.rs:567-611."""
    if c1 > c0:
        return V1 if u < P_INT[0.9] else V0
    if c1 < c0:
        return V0 if u < P_INT[0.9] else V1
    return V1 if u < P_INT[0.8] else V0


def round1_votes(seed, rng_base, props, proposed, slot_base, track=True):
    """Own round-1 votes for received proposals, in message order —
    RabiaEngine::handle_propose (engine.rs:380-422) -> determine_round1_vote
    (engine.rs:424-452) -> randomized_vote (engine.rs:454-481).
    props: list of (phase_id, proposed value code); proposed: mutable list of the
    window's PhaseData.proposed_value codes (NONE = unset), updated in place as
    handle_propose does (engine.rs:400-404). track=False restates the reference as
    it runs (phases never created, update_phase a no-op: state.rs:166-185): every
    proposal takes randomized_vote. Returns (votes, draws consumed); vote NONE =
    phase outside the window."""
    key = seed_from_u64(seed)
    k = rng_base
    votes = []
    for phase, value in props:
        existing = NONE
        if track:
            off = phase - slot_base
            if not 0 <= off < len(proposed):
                votes.append(NONE)
                continue
            existing = proposed[off]
        if existing != NONE:
            votes.append(value if existing == value else VQ)
            continue
        if value == VQ:
            vote = VQ
        else:
            u = ref_draw(key, k)
            k += 1
            vote = value if u < P_INT[0.7 if value == V0 else 0.8] else VQ
        votes.append(vote)
        if track:
            proposed[phase - slot_base] = value
    return votes, k - rng_base


def handle_decisions(values, committed, slot_base, last_committed, max_phase=0, order=None):
    """Follower (RabiaEngine::handle_decision, engine.rs:708-746), one Decision
    message at a time, in `order` (default ascending PhaseId): set_decision; if the
    decision is V1 and phase_id > last_committed (engine.rs:723-728): apply_batch,
    then commit_phase, which raises last_committed to phase_id (monotonic max) or
    refuses it when phase_id > current_phase (state.rs:65-75) AFTER the batch was
    applied (engine.rs:728-735). Returns (applied flags, last_committed)."""
    S = len(values)
    applied = [0] * S
    lc = last_committed
    for s in (order if order is not None else range(S)):
        pid = slot_base + s
        if committed[s] and values[s] and pid > lc:
            applied[s] = 1
            if max_phase == 0 or pid <= max_phase:
                lc = max(lc, pid)
    return applied, lc


def coin(coin_key, epoch, slot, phase):
    """Common coin (build-defined)."""
    b = chacha_block(coin_key, ((phase - 1) << 40) | (slot >> 9), epoch | (1 << 63), 12)
    return (b[(slot >> 5) & 15] >> (slot & 31)) & 1


def _finish(slot_base, S, lc_in, wm_in, max_v1, first_und):
    lc = lc_in if max_v1 is None or max_v1 <= lc_in else max_v1
    wm = first_und if slot_base <= wm_in < first_und else wm_in
    return lc, wm


def ref_step(n, q, self_lane, seed, rng_base, slot_base, r1, r2, max_phase=0,
             lc_in=0, wm_in=1):
    """REF phase step over per-slot code lists (final-vote-set semantics)."""
    key = seed_from_u64(seed)
    k = rng_base
    out = {"r1": [], "r2own": [], "dec": [], "committed": [], "value": []}
    n_dec = n_v1 = n_pend = 0
    max_v1 = None
    first_und = slot_base + len(r1)
    for s, (x1, x2) in enumerate(zip(r1, r2)):
        res1 = ref_round1(x1, q)
        if res1 in (V0, V1):
            own = res1
        elif res1 == VQ:
            c0 = sum(1 for c in x1 if c == V0)
            c1 = sum(1 for c in x1 if c == V1)
            own = round2_vote_for_question(c0, c1, ref_draw(key, k))
            k += 1
        else:
            own = NONE
            n_pend += 1
        v2 = list(x2)
        if own != NONE and 0 <= self_lane < n:
            v2[self_lane] = own
        d = count_votes(v2, q)
        committed = d in (V0, V1)
        sid = slot_base + s
        out["r1"].append(res1); out["r2own"].append(own); out["dec"].append(d)
        out["committed"].append(int(committed)); out["value"].append(int(d == V1))
        n_dec += committed
        if d == V1:
            n_v1 += 1
            if max_phase == 0 or sid <= max_phase:
                max_v1 = sid
        if not committed and sid < first_und:
            first_und = sid
    lc, wm = _finish(slot_base, len(r1), lc_in, wm_in, max_v1, first_und)
    res = dict(n_slots=len(r1), n_decided=n_dec, n_v1=n_v1, n_pending_r1=n_pend,
               n_draws=k - rng_base, last_committed_max=lc, first_undecided=first_und,
               rng_next=k, commit_watermark=wm)
    return out, res


def wmvc_round(codes_r1, codes_r2, state, n, q, fp1, self_lane, coin_bit):
    """One WMVC phase for one slot (docs/weak_mvc.ivy:129-191).
    Returns (r1_result, decision, next_state, used_coin)."""
    c0 = sum(1 for c in codes_r1 if c == V0)
    c1 = sum(1 for c in codes_r1 if c == V1)
    present = sum(1 for c in codes_r1 if c != NONE)
    if present < q:
        return NONE, NONE, state, False
    res1 = V0 if c0 >= q else (V1 if c1 >= q else VQ)
    v2 = list(codes_r2)
    if 0 <= self_lane < n:
        v2[self_lane] = res1
    c0 = sum(1 for c in v2 if c == V0)
    c1 = sum(1 for c in v2 if c == V1)
    present = sum(1 for c in v2 if c != NONE)
    if present < q:
        return res1, NONE, state, False
    if c0 >= fp1:
        return res1, V0, 0, False
    if c1 >= fp1:
        return res1, V1, 1, False
    if c0 > 0:
        return res1, NONE, 0, False
    if c1 > 0:
        return res1, NONE, 1, False
    return res1, NONE, coin_bit, True


def wmvc_step(n, q, fp1, self_lane, coin_seed, epoch, phase, slot_base, r1, r2,
              state, lc_in=0, wm_in=1):
    ckey = seed_from_u64(coin_seed)
    out = {"r1": [], "r2own": [], "dec": [], "committed": [], "value": []}
    n_dec = n_v1 = n_pend = n_coin = 0
    max_v1 = None
    first_und = slot_base + len(r1)
    for s in range(len(r1)):
        sid = slot_base + s
        cb = coin(ckey, epoch, sid, phase)
        res1, d, st, used = wmvc_round(r1[s], r2[s], state[s] & 1, n, q, fp1, self_lane, cb)
        n_pend += res1 == NONE
        n_coin += used
        committed = d != NONE
        out["r1"].append(res1); out["r2own"].append(res1); out["dec"].append(d)
        out["committed"].append(int(committed)); out["value"].append(st)
        n_dec += committed
        if d == V1:
            n_v1 += 1
            max_v1 = sid
        if not committed and sid < first_und:
            first_und = sid
    lc, wm = _finish(slot_base, len(r1), lc_in, wm_in, max_v1, first_und)
    res = dict(n_slots=len(r1), n_decided=n_dec, n_v1=n_v1, n_pending_r1=n_pend,
               n_draws=n_coin, last_committed_max=lc, first_undecided=first_und,
               rng_next=0, commit_watermark=wm)
    return out, res


def digest_majority(digests_per_slot, q):
    """weak_mvc.ivy:109-128: state 1 iff some (nonzero) digest is held by >= q."""
    out = []
    for ds in digests_per_slot:
        st = 0
        for d in ds:
            if d and sum(1 for e in ds if e == d) >= q:
                st = 1
                break
        out.append(st)
    return out


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def _trace_key(seed, key):
    return _mix64(seed ^ (((key + 1) * 0xD1B54A32D192ED03) & MASK64))


def trace(kind, n, seed, slot_base, S):
    """Synthetic traces. Returns (r1, r2, state)."""
    kmaj, kst, krot = _trace_key(seed, 0), _trace_key(seed, 1), _trace_key(seed, 2)
    keys = [[_trace_key(seed, 16 + r * 16 + j) for j in range(n)] for r in range(2)]
    nv0 = (n - 1) // 2
    split = [V0 if j < nv0 else (V1 if j < n - 1 else VQ) for j in range(n)]
    r1, r2, st = [], [], []
    for s in range(S):
        sid = slot_base + s
        m = _mix64((kmaj + sid) & MASK64) & 1
        st.append(_mix64((kst + sid) & MASK64) & 1)
        rot = _mix64((krot + sid) & MASK64) % n
        rows = []
        for r in range(2):
            row = []
            for j in range(n):
                u = _mix64((keys[r][j] + sid) & MASK64)
                if kind == 0:
                    c = u & 3
                elif kind == 1:
                    if u < P_INT[0.9]:
                        c = m
                    else:
                        pick = (u & MASK32) % 3
                        c = (1 - m) if pick == 0 else (VQ if pick == 1 else NONE)
                else:
                    c = VQ if r else split[(j + rot) % n]
                row.append(c)
            rows.append(row)
        r1.append(rows[0]); r2.append(rows[1])
    return r1, r2, st


def _cluster_key(seed, phase, rnd, r):
    return _mix64(seed ^ ((((phase << 32) | (rnd << 16) | r) * 0x9E6C63D0676A9A99) & MASK64))


def _fmix32(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & MASK32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & MASK32
    return h ^ (h >> 16)


def heard(delivery_seed, slot, phase, rnd, r, n, q):
    """Receiver r hears itself and q-1 others (scheduler hash version 2):
    h = fmix32(low word of the receiver key ^ the slot folded to 32 bits); pick i takes
    the k-th remaining sender, k = (6-bit chunk i % 5 of word i // 5) * span >> 6."""
    s32 = (slot & MASK32) ^ (((slot >> 32) * 0x9E3779B9) & MASK32)
    h = _fmix32((_cluster_key(delivery_seed, phase, rnd, r) & MASK32) ^ s32)
    avail = [j for j in range(n) if j != r]
    mask = 1 << r
    for i in range(q - 1):
        if i and i % 5 == 0:
            h = _fmix32((h + 0x9E3779B9) & MASK32)
        span = n - 1 - i
        k = (((h >> (6 * (i % 5))) & 63) * span) >> 6
        pick = avail.pop(k)
        mask |= 1 << pick
    return mask


def wmvc_cluster(n, q, fp1, coin_seed, epoch, delivery_seed, max_phases, slot_base, states):
    """Every replica of each slot runs weak_mvc.ivy phase_rnd1/phase_rnd2 until
    all decided. Returns per slot (dec, phases, first, coins)."""
    ckey = seed_from_u64(coin_seed)
    outs = []
    for s, row in enumerate(states):
        sid = slot_base + s
        st = list(row)
        decided = [None] * n
        o = [NONE, 0, 0, 0]
        for p in range(1, max_phases + 1):
            if all(d is not None for d in decided):
                break
            vote = []
            for r in range(n):
                h = heard(delivery_seed, sid, p, 1, r, n, q)
                got = [st[j] for j in range(n) if (h >> j) & 1]
                vote.append(1 if got.count(1) >= q else (0 if got.count(0) >= q else None))
            coin_v = None
            nst = []
            for r in range(n):
                h = heard(delivery_seed, sid, p, 2, r, n, q)
                got = [vote[j] for j in range(n) if (h >> j) & 1]
                c0, c1 = got.count(0), got.count(1)
                nv = 0 if c0 >= fp1 else (1 if c1 >= fp1 else None)
                if nv is not None and decided[r] is None:
                    decided[r] = nv
                    if not o[2]:
                        o[2] = p
                if nv is None:
                    if c0 > 0:
                        nv = 0
                    elif c1 > 0:
                        nv = 1
                    else:
                        if coin_v is None:
                            coin_v = coin(ckey, epoch, sid, p)
                            o[3] += 1
                        nv = coin_v
                if decided[r] is not None:
                    nv = decided[r]
                nst.append(nv)
            st = nst
            if all(d is not None for d in decided):
                o[1] = p
        if all(d is not None for d in decided):
            assert len(set(decided)) == 1, "agreement violated"
            o[0] = decided[0]
        outs.append(tuple(o))
    return outs


def cluster_trace(n, seed, slot_base, S):
    krot = _trace_key(seed, 4)
    out = []
    for s in range(S):
        rot = _mix64((krot + slot_base + s) & MASK64) % n
        out.append([1 if (r + rot) % n < (n - 1) // 2 else 0 for r in range(n)])
    return out
