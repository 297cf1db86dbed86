"""N>1 path on CPU: world_size-2 gloo ranks each evaluate their slot shard (with the
oracle standing in for the device step on this GPU-less host), exchange results
and decided bitmaps with all_gather, and the folded global commit must equal one
evaluator over the whole window."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from rabia_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_range_partitions():
    for total in (1, 127, 128, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            parts = [shard.shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in parts) == total
            pos = 0
            for s, c in parts:
                assert s == pos and (s % 128 == 0 or c == 0)
                pos += c


def test_combine_single_shard_identity(oracle):
    r1, r2, st = oracle.trace(0, 5, 3, 10, 999)
    _, res = oracle.wmvc_step(5, 3, 3, 0, 7, 1, 2, 10, r1, r2, st, lc_in=4, wm_in=10)
    g = shard.combine([res], [0], [999], 10, 10, 4)
    assert g.commit_watermark == res["commit_watermark"]
    assert g.last_committed == res["last_committed_max"]
    assert g.first_undecided == res["first_undecided"]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import oracle_lib as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, S, base = 5, 10_000, 1
        r1, r2, st = O.trace(1, n, 5, base, S)
        start, count = shard.shard_range(S, world, rank)
        sl = slice(start, start + count)
        out, res = O.wmvc_step(n, 3, 3, 0, 11, 2, 1, base + start, r1[sl], r2[sl], st[sl],
                               lc_in=0, wm_in=1)
        rows = shard.exchange_results(torch.tensor(shard.result_row(res), dtype=torch.int64))
        starts = [shard.shard_range(S, world, r)[0] for r in range(world)]
        counts = [shard.shard_range(S, world, r)[1] for r in range(world)]
        g = shard.combine([shard.row_result(rw.tolist()) for rw in rows], starts, counts, base, 1, 0)
        width = max(counts)  # shards differ by <= one alignment unit: pad to equal size
        bm = np.zeros(width, np.uint8)
        bm[:count] = out["committed"]
        bms = shard.exchange_bitmap(torch.from_numpy(bm)).numpy()
        full = np.concatenate([bms[r][:counts[r]] for r in range(world)])
        q.put((rank, g, full.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_global_commit(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    while len(got) < world:
        try:
            got.append(q.get(timeout=1))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), "a rank died"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, S = 5, 10_000
    r1, r2, st = oracle.trace(1, n, 5, 1, S)
    out, res = oracle.wmvc_step(n, 3, 3, 0, 11, 2, 1, 1, r1, r2, st, lc_in=0, wm_in=1)
    for rank, g, bits in got:
        assert g.n_decided == res["n_decided"] and g.n_v1 == res["n_v1"]
        assert g.last_committed == res["last_committed_max"]
        assert g.first_undecided == res["first_undecided"]
        assert g.commit_watermark == res["commit_watermark"]
        assert g.n_draws == res["n_draws"]
        np.testing.assert_array_equal(np.array(bits, np.uint8), out["committed"])


def _ref_worker(rank, world, port, q):
    """REF mode through the product's sharded protocol (include/rabia_gpu.h "Sharded
    REF"), the oracle's restatement of each device stage standing in for the GPU: every
    rank holds the SAME engine seed; per step of K windows each rank evaluates its shard
    of every window at provisional draws and leaves draw records (or_shard_step), the K
    rows are all-gathered (rank-major [world][K]), each VQ slot is re-drawn at its global
    stream position (window_draw_bases: the fix-up's algebra; or_shard_fixup), the final
    rows are all-gathered and folded window by window (commit_windows). Two steps, so the
    second starts from the first one's engine position."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import oracle_lib as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, quorum, lane, seed, K, steps, W = 5, 3, 2, 42, 3, 2, 20_000
        kinds = (0, 1, 2)
        rng, wm, lc = 777, 1, 5
        max_phase = K * steps * W // 2
        start, count = shard.shard_range(W, world, rank)
        results, outs_all = [], []
        for t in range(steps):
            outs, recs, rows = [], [], []
            for w in range(K):
                base = 1 + (t * K + w) * W
                r1, r2, _ = O.trace(kinds[w % 3], n, 5 + w, base, W)
                sl = slice(start, start + count)
                out, rec, row = O.shard_step(n, quorum, lane, base + start, r1[sl], r2[sl], max_phase=max_phase)
                outs.append(out)
                recs.append(rec)
                rows.append(row)
            g = shard.exchange_results(torch.tensor([shard.result_row(r) for r in rows], dtype=torch.int64))
            n_draws = [[int(g[r, w, 4]) for w in range(K)] for r in range(world)]
            g0, after = shard.window_draw_bases(n_draws, rank, rng)
            fixed = []
            for w in range(K):
                base = 1 + (t * K + w) * W
                row, flags = O.shard_fixup(seed, g0[w], base + start, outs[w], recs[w], rows[w], after[w],
                                           max_phase=max_phase)
                assert flags == 0
                fixed.append(row)
            gf = shard.exchange_results(torch.tensor([shard.result_row(r) for r in fixed], dtype=torch.int64))
            rows_all = [[shard.row_result(gf[r, w].tolist()) for w in range(K)] for r in range(world)]
            res = shard.commit_windows(rows_all, 1 + t * K * W, W, wm, lc)
            wm, lc, rng = res[-1].commit_watermark, res[-1].last_committed, after[-1]
            results.extend(res)
            outs_all.extend(outs)
        width = max(shard.shard_range(W, world, r)[1] for r in range(world))
        keys = ("r1", "r2own", "dec", "committed", "value")
        full = []
        for out in outs_all:  # every window's fixed outputs, gathered
            packed = np.zeros((5, width), np.uint8)
            for i, k in enumerate(keys):
                packed[i, :count] = out[k]
            allp = shard.exchange_bitmap(torch.from_numpy(packed)).numpy()
            full.append({k: np.concatenate([allp[r][i][:shard.shard_range(W, world, r)[1]] for r in range(world)])
                         .tolist() for i, k in enumerate(keys)})
        q.put((rank, results, rng, full))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ref_shards_one_stream_gloo(oracle, world):
    """gloo world 2 and 3, the product's shard protocol (provisional likely-outcome votes,
    4-B draw records with a segment table, re-draw at global positions, K-window commit) == one engine
    (oracle.ref_step) over every window of both steps: outputs, results, engine position."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ref_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    while len(got) < world:
        try:
            got.append(q.get(timeout=1))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), "a rank died"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, K, steps, W = 5, 3, 2, 20_000
    kinds = (0, 1, 2)
    rng, wm, lc = 777, 1, 5
    max_phase = K * steps * W // 2
    exp_res, exp_out = [], []
    for t in range(steps):
        for w in range(K):
            base = 1 + (t * K + w) * W
            r1, r2, _ = oracle.trace(kinds[w % 3], n, 5 + w, base, W)
            out, res = oracle.ref_step(n, 3, 2, 42, rng, base, r1, r2, max_phase=max_phase, lc_in=lc, wm_in=wm)
            rng, wm, lc = res["rng_next"], res["commit_watermark"], res["last_committed_max"]
            exp_res.append(res)
            exp_out.append(out)
    assert sum(r["n_draws"] for r in exp_res) > 0
    for rank, results, rng_end, full in got:
        assert rng_end == rng
        for w, (g, e) in enumerate(zip(results, exp_res)):
            assert g.n_draws == e["n_draws"] and g.n_decided == e["n_decided"] and g.n_v1 == e["n_v1"], w
            assert g.n_pending_r1 == e["n_pending_r1"] and g.flags == 0
            assert g.last_committed == e["last_committed_max"], w
            assert g.first_undecided == e["first_undecided"], w
            assert g.commit_watermark == e["commit_watermark"], w
        for w, (f, e) in enumerate(zip(full, exp_out)):
            for k in e:
                np.testing.assert_array_equal(np.array(f[k], np.uint8), e[k], err_msg=f"rank {rank} window {w} {k}")


def _rendezvous_worker(rank, world, port, q):
    """Two RcclComm rendezvous through shard.rendezvous_store (the TCP store rank 0 serves
    at MASTER_ADDR:MASTER_PORT): rank 0 makes the 128-byte ids, every rank reads them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_RESTART_COUNT="3")
    import hashlib
    store = shard.rendezvous_store(rank, world, timeout_s=60)
    ids = []
    for i in range(2):  # two communicators of one job: distinct keys, distinct ids
        uid = lambda i=i: hashlib.sha512(b"rg-%d" % i).digest() * 2  # noqa: E731  (128 bytes)
        c = shard.RcclComm(rank, world, store=store, make_uid=uid)
        ids.append((c.key, c.uid))
    store.add("read", 1)  # rank 0 serves the store: it stays until every rank has read
    while int(store.add("read", 0)) < world:
        import time
        time.sleep(0.05)
    q.put((rank, ids))


def test_rendezvous_store_carries_128_byte_id():
    """The RCCL id's host channel on CPU: world 2, rank 0 serves the store and publishes
    two 128-byte ids; both ranks end with the same ids under restart-scoped, per-communicator
    keys (a restarted job or a second communicator never reads a stale id)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rendezvous_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]
    (k0, u0), (k1, u1) = got[0]
    assert len(u0) == len(u1) == 128 and u0 != u1
    assert k0 != k1 and k0.startswith("uid/3/") and k1.startswith("uid/3/")


def _cluster_stats(info):
    info = np.asarray(info, np.uint32)
    dec, ph = info & 255, (info >> 8) & 255
    first, coins = (info >> 16) & 255, info >> 24
    return [int((dec != 3).sum()), int((dec == 1).sum()), int(ph.sum()), int(ph.max(initial=0)),
            int(coins.sum()), int(first.sum()), int(info.size), 0]


def _cluster_worker(rank, world, port, q):
    """C3 across ranks: each rank runs Weak-MVC to termination on its contiguous
    slot shard (the coin is keyed by the global slot id), then the per-shard
    statistics and decided bitmaps are all-gathered and folded."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import oracle_lib as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, S = 5, 30_000
        start, count = shard.shard_range(S, world, rank)
        st = O.cluster_trace(n, 42, 1 + start, count)
        info = O.wmvc_cluster(n, 3, 3, 7, 3, 99, 32, 1 + start, st)
        rows = shard.exchange_results(torch.tensor(_cluster_stats(info), dtype=torch.int64))
        g = shard.combine_cluster(rows.tolist())
        width = max(shard.shard_range(S, world, r)[1] for r in range(world))
        bits = np.zeros(width, np.uint8)
        bits[:count] = (info & 255) <= 1
        allb = shard.exchange_bitmap(torch.from_numpy(bits)).numpy()
        full = np.concatenate([allb[r][:shard.shard_range(S, world, r)[1]] for r in range(world)])
        q.put((rank, g, full.tolist()))
    finally:
        dist.destroy_process_group()


def test_cluster_shards_gloo(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cluster_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    while len(got) < world:
        try:
            got.append(q.get(timeout=1))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), "a rank died"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, S = 5, 30_000
    info = oracle.wmvc_cluster(n, 3, 3, 7, 3, 99, 32, 1, oracle.cluster_trace(n, 42, 1, S))
    exp = shard.combine_cluster([_cluster_stats(info)])
    for rank, g, bits in got:
        assert g == exp
        np.testing.assert_array_equal(np.array(bits, np.uint8), ((info & 255) <= 1).astype(np.uint8))
