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
    """REF mode: every rank holds the SAME engine seed; the shard's draws start at
    the global exclusive prefix of the shards' VQ counts (shard.draw_bases over an
    all_gather), so the window consumes ONE StdRng stream in ascending slot order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import oracle_lib as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, S, base, rng0, seed = 5, 20_000, 1, 777, 42
        r1, r2, _ = O.trace(0, n, 5, base, S)
        start, count = shard.shard_range(S, world, rank)
        sl = slice(start, start + count)
        # the shard's VQ count does not depend on where its draws start
        _, probe = O.ref_step(n, 3, 2, seed, 0, base + start, r1[sl], r2[sl], max_phase=S // 2, lc_in=5, wm_in=1)
        counts = shard.exchange_results(torch.tensor([probe["n_draws"]], dtype=torch.int64)).view(-1).tolist()
        bases, total = shard.draw_bases(counts, rng0)
        out, res = O.ref_step(n, 3, 2, seed, bases[rank], base + start, r1[sl], r2[sl], max_phase=S // 2,
                              lc_in=5, wm_in=1)
        assert res["rng_next"] == bases[rank] + counts[rank]
        rows = shard.exchange_results(torch.tensor(shard.result_row(res), dtype=torch.int64))
        starts = [shard.shard_range(S, world, r)[0] for r in range(world)]
        cnts = [shard.shard_range(S, world, r)[1] for r in range(world)]
        g = shard.combine([shard.row_result(rw.tolist()) for rw in rows], starts, cnts, base, 1, 5)
        width = max(cnts)
        packed = np.zeros((5, width), np.uint8)
        for i, k in enumerate(("r1", "r2own", "dec", "committed", "value")):
            packed[i, :count] = out[k]
        allp = shard.exchange_bitmap(torch.from_numpy(packed)).numpy()
        full = {k: np.concatenate([allp[r][i][:cnts[r]] for r in range(world)])
                for i, k in enumerate(("r1", "r2own", "dec", "committed", "value"))}
        q.put((rank, g, total, {k: v.tolist() for k, v in full.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ref_shards_one_stream_gloo(oracle, world):
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
    n, S = 5, 20_000
    r1, r2, _ = oracle.trace(0, n, 5, 1, S)
    exp, eres = oracle.ref_step(n, 3, 2, 42, 777, 1, r1, r2, max_phase=S // 2, lc_in=5, wm_in=1)
    assert eres["n_draws"] > 0
    for rank, g, total, full in got:
        assert total == eres["rng_next"]
        assert g.n_draws == eres["n_draws"] and g.n_decided == eres["n_decided"] and g.n_v1 == eres["n_v1"]
        assert g.last_committed == eres["last_committed_max"]
        assert g.first_undecided == eres["first_undecided"]
        assert g.commit_watermark == eres["commit_watermark"]
        for k in exp:
            np.testing.assert_array_equal(np.array(full[k], np.uint8), exp[k], err_msg=k)


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
