"""ctypes loader for the CPU oracle (oracle/rabia_oracle.c). Test infrastructure:
used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "librabia_oracle.so")

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
i, u64 = ctypes.c_int, ctypes.c_uint64

RES_KEYS = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws",
            "last_committed_max", "first_undecided", "rng_next", "commit_watermark"]


class OrResult(ctypes.Structure):
    _fields_ = [(k, u64) for k in RES_KEYS]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k in RES_KEYS}


_lib = None


def build():
    src = [os.path.join(ORACLE_DIR, f) for f in ("rabia_oracle.c", "rabia_cpu_soa.c", "kvstore_ref.c", "rabia_oracle.h", "Makefile")]
    if not os.path.exists(ORACLE_SO) or any(os.path.getmtime(s) > os.path.getmtime(ORACLE_SO) for s in src):
        subprocess.run(["make", "-C", ORACLE_DIR, "build/librabia_oracle.so"], check=True,
                       capture_output=True)
    return ORACLE_SO


def load():
    global _lib
    if _lib is not None:
        return _lib
    build()
    lib = ctypes.CDLL(ORACLE_SO)
    lib.or_count_votes.argtypes = [u8p, i, i]
    lib.or_ref_round1.argtypes = [u8p, i, i]
    lib.or_seed_from_u64.argtypes = [u64, u32p]
    lib.or_chacha_block.argtypes = [u32p, u64, u64, i, u32p]
    lib.or_ref_draw.argtypes = [u32p, u64]
    lib.or_ref_draw.restype = u64
    lib.or_coin.argtypes = [u32p, u64, u64, u64]
    lib.or_ref_step.argtypes = [i, i, i, u64, u64, u64, u64, u64, u64, u8p, u8p, u64,
                                u8p, u8p, u8p, u8p, u8p, ctypes.POINTER(OrResult)]
    lib.or_wmvc_step.argtypes = [i, i, i, i, u64, u64, u64, u64, u64, u64, u8p, u8p, u8p, u64,
                                 u8p, u8p, u8p, u8p, u8p, ctypes.POINTER(OrResult)]
    lib.or_digest_majority.argtypes = [i, i, u64p, u64, u8p]
    lib.or_coin_range.argtypes = [u64, u64, u64, u64, u64, u8p]
    lib.or_ref_structured.argtypes = [i, i, i, u64, u64, u64, u8p, u8p, u64, u8p,
                                      ctypes.POINTER(OrResult)]
    lib.or_trace.argtypes = [i, i, u64, u64, u64, u8p, u8p, u8p]
    lib.or_digest_trace.argtypes = [i, u64, u64, u64, u64p]
    lib.or_pack_planes.argtypes = [u8p, i, u64, u64, u32p]
    lib.or_ref_step_soa.argtypes = [i, i, i, u64, u64, u64, u64, u64, u64, u32p, u64, u64, u32p,
                                    ctypes.POINTER(OrResult), i]
    lib.or_omp_max_threads.restype = i
    lib.or_kv_create.restype = ctypes.c_void_p
    lib.or_kv_create.argtypes = [u64, u64, i]
    lib.or_kv_destroy.argtypes = [ctypes.c_void_p]
    lib.or_kv_apply.argtypes = [ctypes.c_void_p, u8p, u64p, u64, u8p, u8p]
    lib.or_kv_stats.argtypes = [ctypes.c_void_p, u64p]
    lib.or_kv_apply_partitioned.argtypes = [ctypes.c_uint32, i, u64, u64, i, u8p, u64p, u64, u8p, u8p, u64p]
    lib.or_kv_dump.argtypes = [ctypes.c_void_p, u64p, u8p, u64p, u8p, u32p]
    lib.or_unpack_planes.argtypes = [u32p, i, u64, u64, u8p]
    lib.or_shard_step.argtypes = [i, i, i, u64, u64, u8p, u8p, u64, u8p, u8p, u8p, u8p, u8p, u32p, u64,
                                  ctypes.POINTER(OrResult)]
    lib.or_shard_fixup.argtypes = [u64, u64, u64, u64, u64, u32p, u64, u8p, u8p, u8p, u8p, ctypes.POINTER(OrResult),
                                   u64, ctypes.POINTER(OrResult), u64p]
    _lib = lib
    return lib


def _p(a, t):
    return a.ctypes.data_as(t)


def trace(kind, n, seed, slot_base, S):
    lib = load()
    r1 = np.zeros((S, n), np.uint8)
    r2 = np.zeros((S, n), np.uint8)
    st = np.zeros(S, np.uint8)
    lib.or_trace(kind, n, seed, slot_base, S, _p(r1, u8p), _p(r2, u8p), _p(st, u8p))
    return r1, r2, st


def ref_step(n, q, self_lane, seed, rng_base, slot_base, r1, r2, max_phase=0, lc_in=0, wm_in=1):
    lib = load()
    S = r1.shape[0]
    outs = [np.zeros(S, np.uint8) for _ in range(5)]
    res = OrResult()
    rc = lib.or_ref_step(n, q, self_lane, seed, rng_base, slot_base, max_phase, lc_in, wm_in,
                         _p(np.ascontiguousarray(r1), u8p), _p(np.ascontiguousarray(r2), u8p), S,
                         *[_p(o, u8p) for o in outs], ctypes.byref(res))
    assert rc == 0
    return dict(zip(["r1", "r2own", "dec", "committed", "value"], outs)), res.as_dict()


def record_window_words(S, cap):
    """u32 words of one window's record region (include/rabia_gpu.h rg_record_window_words)."""
    return ((((S + 0xFFFFFF) >> 24) + 1 + 3) & ~3) + cap


def shard_step(n, q, self_lane, slot_base, r1, r2, max_phase=0, records_cap=None):
    """Stage 1 of the sharded pipeline (or_shard_step): provisional outputs, the record
    region (segment table + 4-B draw records, np.uint32), the row of the shard's non-VQ slots."""
    lib = load()
    S = r1.shape[0]
    outs = [np.zeros(S, np.uint8) for _ in range(5)]
    cap = S if records_cap is None else records_cap
    region = np.zeros(record_window_words(S, cap), np.uint32)
    row = OrResult()
    rc = lib.or_shard_step(n, q, self_lane, slot_base, max_phase, _p(np.ascontiguousarray(r1), u8p),
                           _p(np.ascontiguousarray(r2), u8p), S, *[_p(o, u8p) for o in outs], _p(region, u32p), cap,
                           ctypes.byref(row))
    assert rc == 0
    return dict(zip(["r1", "r2own", "dec", "committed", "value"], outs)), region, row.as_dict()


def shard_fixup(seed, g0, slot_base, outs, region, row, rng_after, max_phase=0, records_cap=None):
    """Stage 3 (or_shard_fixup): re-draw the shard's VQ slots at global positions g0 + k
    from its record region; patches `outs` in place; returns (final row, flags)."""
    lib = load()
    S = len(outs["r2own"])
    rin = OrResult(**{k: int(row[k]) for k in RES_KEYS})
    rout = OrResult()
    flags = np.zeros(1, np.uint64)
    reg = np.ascontiguousarray(region, np.uint32)
    cap = len(reg) - (record_window_words(S, 0)) if records_cap is None else records_cap
    lib.or_shard_fixup(seed, g0, slot_base, max_phase, S, _p(reg, u32p), cap,
                       *[_p(outs[k], u8p) for k in ("r2own", "dec", "committed", "value")], ctypes.byref(rin),
                       rng_after, ctypes.byref(rout), _p(flags, u64p))
    return rout.as_dict(), int(flags[0])


def wmvc_step(n, q, fp1, self_lane, coin_seed, epoch, phase, slot_base, r1, r2, state,
              lc_in=0, wm_in=1):
    lib = load()
    S = r1.shape[0]
    outs = [np.zeros(S, np.uint8) for _ in range(5)]
    res = OrResult()
    rc = lib.or_wmvc_step(n, q, fp1, self_lane, coin_seed, epoch, phase, slot_base, lc_in, wm_in,
                          _p(np.ascontiguousarray(r1), u8p), _p(np.ascontiguousarray(r2), u8p),
                          _p(np.ascontiguousarray(state, np.uint8), u8p), S,
                          *[_p(o, u8p) for o in outs], ctypes.byref(res))
    assert rc == 0
    return dict(zip(["r1", "r2own", "dec", "committed", "value"], outs)), res.as_dict()


def ref_structured(n, q, self_lane, seed, rng_base, slot_base, r1, r2):
    lib = load()
    S = r1.shape[0]
    dec = np.zeros(S, np.uint8)
    res = OrResult()
    rc = lib.or_ref_structured(n, q, self_lane, seed, rng_base, slot_base,
                               _p(np.ascontiguousarray(r1), u8p), _p(np.ascontiguousarray(r2), u8p),
                               S, _p(dec, u8p), ctypes.byref(res))
    assert rc == 0
    return dec, res.as_dict()


def ref_step_soa(n, q, self_lane, seed, rng_base, slot_base, planes, stride, S, max_phase=0, lc_in=0, wm_in=1,
                 threads=0, want_out=True):
    """The fast all-core CPU path on planar planes [(4n+1) x stride] (rabia_cpu_soa.c)."""
    lib = load()
    planes = np.ascontiguousarray(planes, np.uint32)
    out = np.zeros((8, stride), np.uint32) if want_out else None
    res = OrResult()
    rc = lib.or_ref_step_soa(n, q, self_lane, seed, rng_base, slot_base, max_phase, lc_in, wm_in,
                             _p(planes, u32p), stride, S, _p(out, u32p) if want_out else None,
                             ctypes.byref(res), threads)
    assert rc == 0
    return out, res.as_dict()


def digest_majority(digests, q):
    lib = load()
    n, S = digests.shape
    out = np.zeros(S, np.uint8)
    lib.or_digest_majority(n, q, _p(np.ascontiguousarray(digests, np.uint64), u64p), S, _p(out, u8p))
    return out


def digest_trace(n, seed, slot_base, S):
    lib = load()
    d = np.zeros((n, S), np.uint64)
    lib.or_digest_trace(n, seed, slot_base, S, _p(d, u64p))
    return d


def coin_range(coin_seed, epoch, phase, slot_base, S):
    lib = load()
    out = np.zeros(S, np.uint8)
    lib.or_coin_range(coin_seed, epoch, phase, slot_base, S, _p(out, u8p))
    return out


def ref_draws(seed, first, count):
    lib = load()
    key = np.zeros(8, np.uint32)
    lib.or_seed_from_u64(seed, _p(key, u32p))
    return np.array([lib.or_ref_draw(_p(key, u32p), first + k) for k in range(count)], np.uint64)


def chacha_block(key_words, counter, stream, rounds):
    lib = load()
    key = np.array(key_words, np.uint32)
    out = np.zeros(16, np.uint32)
    lib.or_chacha_block(_p(key, u32p), counter, stream, rounds, _p(out, u32p))
    return out


def seed_from_u64(seed):
    lib = load()
    key = np.zeros(8, np.uint32)
    lib.or_seed_from_u64(seed, _p(key, u32p))
    return key


def pack_planes(codes, stride):
    lib = load()
    S, n = codes.shape
    planes = np.zeros((2 * n, stride), np.uint32)
    lib.or_pack_planes(_p(np.ascontiguousarray(codes), u8p), n, S, stride, _p(planes, u32p))
    return planes


def count_votes_table(n, q):
    """All 4^n vectors (lane j = base-4 digit j) through or_count_votes / or_ref_round1."""
    lib = load()
    N = 4 ** n
    idx = np.arange(N, dtype=np.int64)
    codes = np.stack([(idx >> (2 * j)) & 3 for j in range(n)], axis=1).astype(np.uint8)
    cv = np.array([lib.or_count_votes(_p(codes[k], u8p), n, q) for k in range(N)], np.uint8)
    r1 = np.array([lib.or_ref_round1(_p(codes[k], u8p), n, q) for k in range(N)], np.uint8)
    return codes, cv, r1


class ClusterOut(ctypes.Structure):
    _fields_ = [("dec", ctypes.c_uint8), ("phases", ctypes.c_uint8), ("first", ctypes.c_uint8),
                ("coins", ctypes.c_uint8)]


def wmvc_cluster(n, q, fp1, coin_seed, epoch, delivery_seed, max_phases, slot_base, states):
    """Returns uint32 info per slot packed like the device (dec | phases<<8 | first<<16 | coins<<24)."""
    lib = load()
    lib.or_wmvc_cluster.argtypes = [i, i, i, u64, u64, u64, ctypes.c_uint32, u64, u8p, u64,
                                    ctypes.POINTER(ClusterOut)]
    S = states.shape[0]
    out = (ClusterOut * S)()
    rc = lib.or_wmvc_cluster(n, q, fp1, coin_seed, epoch, delivery_seed, max_phases, slot_base,
                             _p(np.ascontiguousarray(states, np.uint8), u8p), S, out)
    assert rc == 0
    raw = np.frombuffer(out, dtype=np.uint8).reshape(S, 4).astype(np.uint32)
    return raw[:, 0] | (raw[:, 1] << 8) | (raw[:, 2] << 16) | (raw[:, 3] << 24)


def cluster_trace(n, seed, slot_base, S):
    lib = load()
    lib.or_cluster_trace.argtypes = [i, u64, u64, u64, u8p]
    st = np.zeros((S, n), np.uint8)
    lib.or_cluster_trace(n, seed, slot_base, S, _p(st, u8p))
    return st


def kv_apply_partitioned(data, offs, mask=None, parts=16, max_keys=0, max_value_size=0, notify=True, threads=0):
    """oracle/kvstore_ref.c:or_kv_apply_partitioned — the all-core CPU baseline of the
    apply (key-hash partitions, one store and one thread each; exact while StoreFull
    cannot fire). -> (results[n], {live_keys, version, total_operations})."""
    lib = load()
    data = np.ascontiguousarray(data, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    n = offs.size - 1
    res = np.zeros(max(n, 1), np.uint8)
    out = np.zeros(3, np.uint64)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    rc = lib.or_kv_apply_partitioned(parts, threads, max_keys, max_value_size, 1 if notify else 0,
                                     _p(data if data.size else np.zeros(1, np.uint8), u8p), _p(offs, u64p), n,
                                     _p(m, u8p) if m is not None else None, _p(res, u8p), _p(out, u64p))
    assert rc == 0
    return res[:n], {"live_keys": int(out[0]), "version": int(out[1]), "total_operations": int(out[2])}


class KVStoreC:
    """oracle/kvstore_ref.c: the sequential C restatement of the kvstore apply
    (same semantics as oracle/kvstore_ref.py, pinned by the reference's kvstore
    test outcomes). Used as the full-size checker and the C4 CPU baseline."""

    def __init__(self, max_keys=0, max_value_size=0, enable_notifications=True):
        self.lib = load()
        self.h = self.lib.or_kv_create(max_keys, max_value_size, 1 if enable_notifications else 0)
        assert self.h

    def close(self):
        if self.h:
            self.lib.or_kv_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def apply(self, data, offs, mask=None):
        """data: uint8 bytes of all commands, offs: uint64[n+1]; -> uint8 results[n]."""
        data = np.ascontiguousarray(data, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        n = offs.size - 1
        res = np.zeros(max(n, 1), np.uint8)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        rc = self.lib.or_kv_apply(self.h, _p(data if data.size else np.zeros(1, np.uint8), u8p), _p(offs, u64p), n,
                                  _p(m, u8p) if m is not None else None, _p(res, u8p))
        assert rc == 0
        return res[:n]

    def stats(self):
        out = np.zeros(5, np.uint64)
        self.lib.or_kv_stats(self.h, _p(out, u64p))
        return {"live_keys": int(out[0]), "version": int(out[1]), "total_operations": int(out[2]),
                "key_bytes": int(out[3]), "value_bytes": int(out[4])}

    def state(self):
        """{"data": {key: (value, entry version)}, "version"} like kvstore_ref.KVStoreRef.state()."""
        st = self.stats()
        n = st["live_keys"]
        ko = np.zeros(n + 1, np.uint64)
        vo = np.zeros(n + 1, np.uint64)
        kb = np.zeros(max(st["key_bytes"], 1), np.uint8)
        vb = np.zeros(max(st["value_bytes"], 1), np.uint8)
        ver = np.zeros(max(n, 1), np.uint32)
        self.lib.or_kv_dump(self.h, _p(ko, u64p), _p(kb, u8p), _p(vo, u64p), _p(vb, u8p), _p(ver, u32p))
        kbytes, vbytes = kb.tobytes(), vb.tobytes()
        data = {kbytes[ko[i]:ko[i + 1]]: (vbytes[vo[i]:vo[i + 1]], int(ver[i])) for i in range(n)}
        return {"data": data, "version": st["version"]}
